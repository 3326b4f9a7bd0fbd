"""Utilities (subset of src/utilities.py on the sampling path) and the
process-group adapter used for sample sharding.

Distribution model: one process per GPU, samples sharded by
``shareRange`` (src/utilities.py:268-292), a single collective for the KL
value/gradient mean.  ``TorchComm`` exposes the slice of the mpi4py
communicator API the reference calls (Get_rank/Get_size/allgather/bcast/
Barrier) on top of ``torch.distributed`` (backend "nccl" = RCCL over xGMI on
the GPU box, "gloo" on CPU).
"""
import numpy as np
import torch


def myassert(val):
    if not val:
        raise AssertionError


def shareRange(nwork, nshares, myshare):
    """Fair contiguous split of `nwork` items (src/utilities.py:268-292)."""
    nbase = nwork // nshares
    additional = nwork % nshares
    lo = myshare * nbase + min(myshare, additional)
    hi = lo + nbase + int(myshare < additional)
    return lo, hi


def get_MPI_params_from_comm(comm):
    if comm is None:
        return 1, 0, True
    size = comm.Get_size()
    rank = comm.Get_rank()
    return size, rank, rank == 0


class TorchComm:
    """mpi4py-like communicator over an initialised torch.distributed group."""

    def __init__(self, group=None):
        import torch.distributed as dist
        if not dist.is_initialized():
            raise RuntimeError("torch.distributed is not initialised")
        self._dist = dist
        self._group = group

    def Get_rank(self):
        return self._dist.get_rank(self._group)

    def Get_size(self):
        return self._dist.get_world_size(self._group)

    def allgather(self, obj):
        out = [None] * self.Get_size()
        self._dist.all_gather_object(out, obj, group=self._group)
        return out

    def bcast(self, obj, root=0):
        lst = [obj]
        self._dist.broadcast_object_list(lst, src=root, group=self._group)
        return lst[0]

    def Barrier(self):
        self._dist.barrier(group=self._group)

    @property
    def backend(self):
        return self._dist.get_backend(self._group)

    def _staged(self, t):
        """gloo moves host memory only: a device tensor goes through a host
        copy (RCCL takes it in place)"""
        return t.is_cuda and self.backend == "gloo"

    def allreduce_tensor_(self, t):
        """In-place SUM all-reduce of a tensor (one RCCL call on GPU)."""
        if self._staged(t):
            h = t.cpu()
            self._dist.all_reduce(h, group=self._group)
            t.copy_(h)
        else:
            self._dist.all_reduce(t, group=self._group)
        return t

    def _global(self, r):
        return r if self._group is None else self._dist.get_global_rank(self._group, r)

    def send_tensor(self, t, dest):
        t = t.cpu() if self._staged(t) else t.contiguous()
        self._dist.send(t, self._global(dest), group=self._group)

    def recv_tensor_(self, t, source):
        if self._staged(t):
            h = torch_empty_like_host(t)
            self._dist.recv(h, self._global(source), group=self._group)
            t.copy_(h)
        else:
            self._dist.recv(t, self._global(source), group=self._group)
        return t

    def broadcast_tensor_(self, t, root):
        if self._staged(t):
            h = t.cpu()
            self._dist.broadcast(h, self._global(root), group=self._group)
            t.copy_(h)
        else:
            self._dist.broadcast(t, self._global(root), group=self._group)
        return t


def torch_empty_like_host(t):
    import torch
    return torch.empty(t.shape, dtype=t.dtype)


def pairwise_sum(vals):
    """The fixed pairwise summation order of allreduce_sum
    (src/utilities.py:374-387) for a local list.  Tuples are summed
    element by element."""
    vals = list(vals)
    if vals and isinstance(vals[0], tuple):
        return tuple(pairwise_sum(col) for col in zip(*vals))
    n = len(vals)
    step = 1
    while step < n:
        for j in range(0, n, 2 * step):
            if j + step < n:
                vals[j] = vals[j] + vals[j + step]
                vals[j + step] = None
        step *= 2
    return vals[0]


DETERMINISTIC_ALLREDUCE = False


def _flatten(obj):
    """object -> (list of tensors, rebuild function) for Field / MultiField /
    scalars / torch tensors and tuples of them"""
    from .field import Field
    from .multi_field import MultiField
    if isinstance(obj, tuple):
        parts = [_flatten(o) for o in obj]
        sizes = [len(ts) for ts, _ in parts]

        def rebuild(ts):
            out, off = [], 0
            for (_, rb), n in zip(parts, sizes):
                out.append(rb(ts[off:off + n]))
                off += n
            return tuple(out)
        return [t for ts, _ in parts for t in ts], rebuild
    if isinstance(obj, MultiField):
        return [f.val for f in obj.values()], lambda ts: MultiField(
            obj.domain, tuple(Field(d, t) for d, t in zip(obj.domain.values(), ts)))
    if isinstance(obj, Field):
        return [obj.val], lambda ts: Field(obj.domain, ts[0])
    if isinstance(obj, (float, int, np.floating)):
        return [torch.tensor(float(obj), dtype=torch.float64)], lambda ts: float(ts[0].item())
    if isinstance(obj, torch.Tensor):
        return [obj], lambda ts: ts[0]
    raise TypeError(f"cannot all-reduce {type(obj)}")


class _Packed:
    """one object (Field / MultiField / scalar / tuple of them) as flat
    buffers on the collective's device, ONE per element dtype (usually just
    fp64): every element is summed in its own dtype, as the serial pairwise
    sum does, and complex tensors travel as (re, im) pairs of their real
    dtype"""

    def __init__(self, obj, comm):
        self.ts, self.rebuild = _flatten(obj)
        self.dev = _comm_device(comm, self.ts[0].device)
        groups = {}
        for i, t in enumerate(self.ts):
            r = torch.view_as_real(t) if t.is_complex() else t
            if not r.is_floating_point():
                r = r.to(torch.float64)
            groups.setdefault(r.dtype, []).append((i, r))
        self.dtypes = sorted(groups, key=str)
        self.layout = [groups[d] for d in self.dtypes]
        self.bufs = [torch.cat([r.reshape(-1).to(self.dev) for _, r in grp]) for grp in self.layout]

    def zeros(self):
        return [torch.zeros_like(b) for b in self.bufs]

    def unpack(self, bufs):
        out = [None] * len(self.ts)
        for grp, buf in zip(self.layout, bufs):
            off = 0
            for i, r in grp:
                n = r.numel()
                v = buf[off:off + n].reshape(r.shape).to(self.ts[i].device)
                t = self.ts[i]
                # a complex run after an odd count of real elements starts at
                # an odd storage offset, which view_as_complex rejects: clone
                out[i] = torch.view_as_complex(v.clone()) if t.is_complex() else v.to(t.dtype)
                off += n
        return self.rebuild(out)


def _comm_device(comm, dev):
    """gloo runs its collectives on host tensors, RCCL ("nccl") on the GPU"""
    backend = getattr(comm, "backend", "gloo")
    if backend == "nccl":
        if dev.type != "cuda":
            from . import config
            return config.device()
        return dev
    return torch.device("cpu")


def allreduce_sum(obj, comm, deterministic=None, counts=None, template=None):
    """Sum of a list of per-sample objects held by the ranks
    (src/utilities.py:331-390).  Items may be Fields, MultiFields, scalars or
    tuples of them (summed element by element).

    Serial: the reference's pairwise tree.  Distributed, default: each rank
    sums its samples in pairwise order, then ONE all-reduce of a packed fp64
    buffer (RCCL over xGMI on the GPU box).  ``deterministic=True`` (or
    DETERMINISTIC_ALLREDUCE): the reference's global pairwise tree over the
    ranks with point-to-point send/recv of packed buffers and a final
    broadcast -- bit-identical to the serial sum for any number of ranks
    (test_mpi/test_kl.py semantics).

    ``counts``: the per-rank item counts if known (else one allgather).
    A rank holding no items needs ``template()``, a zero object of the
    result's layout (the reference instead splits off an active
    communicator, sample_list.py:62-70)."""
    vals = list(obj)
    if comm is None:
        return pairwise_sum(vals)
    if deterministic is None:
        deterministic = DETERMINISTIC_ALLREDUCE
    if counts is None:
        counts = comm.allgather(len(vals))
    counts = [int(c) for c in counts]
    if sum(counts) == 0:
        raise ValueError("allreduce_sum over no items at all")
    if min(counts) == 0:
        # every rank must issue the same per-dtype collectives: a rank without
        # items casts its template to the element dtypes of the ranks' items
        mine = tuple(str(t.dtype) for t in _flatten(vals[0])[0]) if vals else None
        lays = [x for x in comm.allgather(mine) if x is not None]
        if any(x != lays[0] for x in lays):
            raise RuntimeError("allreduce_sum: ranks hold items of different dtype layouts")
        if not vals and template is not None:
            template = _typed_template(template, lays[0])
    if deterministic:
        return _tree_sum(vals, comm, counts, template)
    if vals:
        pk = _Packed(pairwise_sum(vals), comm)
        bufs = pk.bufs
    else:
        if template is None:
            raise RuntimeError("a rank without items needs a template of the result layout")
        pk = _Packed(template(), comm)
        bufs = pk.zeros()
    for b in bufs:
        comm.allreduce_tensor_(b)
    return pk.unpack(bufs)


def _typed_template(template, dtypes):
    """template() with its tensors cast to `dtypes` (names as str(dtype))"""
    def typed():
        ts, rebuild = _flatten(template())
        if len(ts) != len(dtypes):
            raise RuntimeError("allreduce_sum: the template does not match the items' layout")
        return rebuild([t.to(getattr(torch, d.split(".")[-1])) for t, d in zip(ts, dtypes)])
    return typed


def _tree_sum(vals, comm, counts, template):
    """allreduce_sum's pairwise tree (src/utilities.py:358-390) with the items
    as packed fp64 buffers: who[j] holds item j; at distance `step` the
    holder of j + step sends its partial sum to the holder of j (a local add
    when both are on one rank); the total ends on who[0] and is broadcast."""
    rank = comm.Get_rank()
    hi = list(np.cumsum(counts))
    lo = [0] + hi[:-1]
    nobj = hi[-1]
    who = [t for t, (a, b) in enumerate(zip(lo, hi)) for _ in range(b - a)]
    mine = [_Packed(v, comm) for v in vals]
    like = mine[0] if mine else _Packed(template(), comm)
    bufs = [None] * nobj   # per item: its list of per-dtype buffers
    for i, p in enumerate(mine):
        bufs[lo[rank] + i] = p.bufs
    step = 1
    while step < nobj:
        for j in range(0, nobj, 2 * step):
            if j + step < nobj:
                if rank == who[j]:
                    if who[j] == who[j + step]:
                        bufs[j] = [a + b for a, b in zip(bufs[j], bufs[j + step])]
                    else:
                        other = like.zeros()
                        for o in other:
                            comm.recv_tensor_(o, who[j + step])
                        bufs[j] = [a + b for a, b in zip(bufs[j], other)]
                    bufs[j + step] = None
                elif rank == who[j + step]:
                    for b in bufs[j + step]:
                        comm.send_tensor(b, who[j])
                    bufs[j + step] = None
        step *= 2
    out = bufs[0] if rank == who[0] else like.zeros()
    for o in out:
        comm.broadcast_tensor_(o, who[0])
    return like.unpack(out)


def device_checksum(t):
    """An order- and bit-sensitive 64-bit checksum of a tensor's values,
    computed where the tensor lives (one int64 back to the host): each word's
    bits are mixed and weighted by an odd multiplier of its position, summed
    with wraparound.  Equal tensors give equal checksums on every rank; any
    bit flip or permutation changes it with overwhelming probability.  (The
    reference pickles the whole field and hashes the bytes,
    src/utilities.py:453-458.)"""
    import torch
    t = t.detach().contiguous()
    if t.is_complex():
        t = torch.view_as_real(t).contiguous()
    flat = t.reshape(-1)
    if flat.numel() == 0:
        return 0
    ints = {8: torch.int64, 4: torch.int32, 2: torch.int16, 1: torch.uint8}[flat.element_size()]
    w = (flat.view(ints) if flat.dtype != ints else flat).to(torch.int64)
    w = w ^ (w >> 29)
    idx = torch.arange(1, w.numel() + 1, dtype=torch.int64, device=w.device)
    mult = (idx * -7046029254386353131) | 1       # 0x9E3779B97F4A7C15 (golden ratio), odd
    return int(((w * mult) ^ (w >> 17)).sum())


def _sync_token(obj, hash_):
    """what check_MPI_equality gathers for obj: fields by (domain, dtype,
    device checksum) per key, domains by value (compared with ==; their
    pickles carry per-process cached hashes), anything else by its pickle
    (bytes as they are, e.g. getState()'s), blake2b-hashed on request"""
    import pickle
    from hashlib import blake2b
    from .domain_tuple import DomainTuple
    from .domains import Domain
    from .field import Field
    from .multi_domain import MultiDomain
    from .multi_field import MultiField
    if isinstance(obj, Field):
        return ("field", obj.domain, str(obj.dtype), device_checksum(obj.val))
    if isinstance(obj, MultiField):
        return ("multifield", obj.domain,
                tuple((k, str(obj[k].dtype), device_checksum(obj[k].val)) for k in obj.domain.keys()))
    if isinstance(obj, (DomainTuple, MultiDomain, Domain)):
        return ("domain", obj)
    b = obj if isinstance(obj, bytes) else pickle.dumps(obj)
    return ("bytes", blake2b(b).hexdigest() if hash_ else b)


def check_MPI_equality(obj, comm, hash_=False):
    """RuntimeError unless obj is the same on every task of comm
    (src/utilities.py:434-458)"""
    if comm is None:
        return
    lst = comm.allgather(_sync_token(obj, hash_))
    if not all(x == lst[0] for x in lst):
        raise RuntimeError("MPI tasks are not in sync")


def check_MPI_synced_random_state(comm):
    from .random import getState
    if comm is None:
        return
    check_MPI_equality(getState(), comm)


def lognormal_moments(mean, sigma, N=0):
    """(src/utilities.py:405-418)"""
    mean, sigma = (value_reshaper(p, N) for p in (mean, sigma))
    if not np.all(mean > 0):
        raise ValueError(f"mean must be greater 0; got {mean!r}")
    if not np.all(sigma > 0):
        raise ValueError(f"sig must be greater 0; got {sigma!r}")
    logsigma = np.sqrt(np.log1p((sigma / mean) ** 2))
    logmean = np.log(mean) - logsigma ** 2 / 2
    return logmean, logsigma


def value_reshaper(x, N):
    x = np.asarray(x, dtype=np.float64)
    if x.shape in [(), (1,)]:
        return np.full(N, x) if N != 0 else x.reshape(())
    if x.shape == (N,):
        return x
    raise TypeError("x and N are incompatible")


def infer_space(domain, space):
    if space is None:
        if len(domain) != 1:
            raise ValueError("'space' index must be given for objects based on DomainTuples "
                             "containing more than one domain")
        space = 0
    space = int(space)
    if space < 0 or space >= len(domain):
        raise ValueError("space index out of range")
    return space


def parse_spaces(spaces, nspc):
    nspc = int(nspc)
    if spaces is None:
        return tuple(range(nspc))
    if np.isscalar(spaces):
        spaces = (spaces,)
    spaces = tuple(int(i) for i in spaces)
    res = tuple(i if i >= 0 else i + nspc for i in spaces)
    if any(i < 0 or i >= nspc for i in res):
        raise ValueError("space index out of range")
    return res


def check_object_identity(obj1, obj2):
    if obj1 is not obj2:
        raise ValueError(f"Mismatch:\n{obj1}\n{obj2}")


def check_dtype_or_none(obj, domain=None):
    pass


def iscomplextype(dtype):
    if isinstance(dtype, torch.dtype):
        return dtype.is_complex
    return np.issubdtype(np.dtype(dtype), np.complexfloating)


def torch_dtype(dtype):
    """numpy-ish dtype -> torch dtype."""
    if isinstance(dtype, torch.dtype):
        return dtype
    if dtype is float or dtype is None:
        return torch.float64
    if dtype is complex:
        return torch.complex128
    dt = np.dtype(dtype)
    return {np.dtype(np.float64): torch.float64, np.dtype(np.float32): torch.float32,
            np.dtype(np.complex128): torch.complex128, np.dtype(np.complex64): torch.complex64,
            np.dtype(np.int64): torch.int64, np.dtype(np.int32): torch.int32,
            np.dtype(np.bool_): torch.bool}[dt]


def numpy_dtype(tdtype):
    return {torch.float64: np.float64, torch.float32: np.float32, torch.complex128: np.complex128,
            torch.complex64: np.complex64, torch.int64: np.int64, torch.int32: np.int32,
            torch.bool: np.bool_}[tdtype]


def indent(inp):
    return "\n".join((("  " + s).rstrip() for s in inp.splitlines()))


class frozendict(dict):
    def __setitem__(self, *a):
        raise TypeError("frozendict is immutable")

    def __hash__(self):
        return hash(tuple(sorted(self.items())))
