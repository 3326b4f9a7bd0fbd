"""Lock-step geoVI refinement of the local samples (batched NewtonCG).

The reference refines every sample of draw_samples on its own
(src/minimization/kl_energies.py:147-155):

    en = EnergyAdapter(pos_i, GaussianEnergy(m_i) @ transformation,
                       nanisinf=True, want_metric=True)
    en, _ = minimizer(en)                 # NewtonCG + LineSearch

with transformation = 1 + J0^T f_lh, J0 the Jacobian of the likelihood's
whitening map f_lh at the expansion point.  Here the k local samples run the
SAME minimizer code -- one DescentMinimizer.minimize_gen generator per sample
(descent_minimizers.py / line_search.py: its own controllers, every decision
on its own host floats) -- and their requests are served in batches:

  ("at", e, alpha, pk)  value, gradient, |gradient| at e.x + alpha * pk
  ("dd", e, pk)         directional derivative  e.gradient . pk
  ("dir", e, f_prev, s) NewtonCG direction: CG on the sample's metric

Energy of a batch X (k, latent) of positions, everything on the device:

  F  = f_lh(X)                 batched pipeline: CF model, pointwise maps,
                               LOSResponse / GeometryRemover, scalings
  T  = X + J0^T F              J0 shared by the batch (expansion point)
  R  = T - M;  value_i = R_i . R_i / 2
  G  = R + J_f(X)^T (J0 R)     per-sample Jacobians: the batched kernels with
                               per-item constants (nft_amp_*_batched
                               item_consts, nft_hartley_fuse a/b strides)

Newton metric of sample i (GaussianEnergy's metric is 1, so J_T^T J_T):

  M_i v = u + J_i^T J0 u,   u = v + J0^T J_i v

and the descent directions of all requesting samples come from one
FusedCGBatch loop whose matvec applies every sample's own M_i.

Supported f_lh: chains (outermost first) of ScalingOperator, DiagonalOperator,
GeometryRemover, LOSResponse and pointwise functions (ptw_dict) ending in a
SimpleCorrelatedField model; anything else returns None from ``plan`` and
draw_samples keeps the per-sample path."""
import copy
import math

import os

import numpy as np
import torch

from .. import _native
from ..logger import logger
from .energy import Energy

NS = _native.CG_NSCALARS
ENABLED = True   # tests compare against the per-sample path with ENABLED = False
# NFT_GEOVI_DEFER_DIR=0: serve Newton-direction requests as soon as they come
DEFER_DIR = os.environ.get("NFT_GEOVI_DEFER_DIR", "1") != "0"


def _rowdots(pairs):
    """[(A, B), ...] of (k, n) row batches -> host array (len(pairs), k) of
    the fp64 row dot products (nft_dot_batched: deterministic two-level
    reductions, one launch pair per operand pair, one D2H copy)."""
    lib = _native.load()
    k = pairs[0][0].shape[0]
    nmax = max(A.shape[1] for A, _ in pairs)
    out = torch.empty((len(pairs), k), dtype=torch.float64, device=pairs[0][0].device)
    ws = _native.workspace(k * lib.nft_reduce_workspace(nmax), out.device, "rowdot")
    P = _native.ptr
    for i, (A, B) in enumerate(pairs):
        A, B = A.contiguous(), B.contiguous()
        n = A.shape[1]
        assert A.shape == B.shape and A.shape[0] == k
        _native._check(lib.nft_dot_batched(P(A), P(B), n, n, k, _native.dtype_code(A.dtype), P(out[i]), 1,
                                           P(ws), _native.stream_ptr()))
    return out.cpu().numpy()


def _pairdots(pairs):
    """[(a, b), ...] of 1-D device vectors -> host array of their fp64 dot
    products (nft_dot per pair, one D2H copy; each equals the row of a
    batched nft_dot_batched bit for bit)"""
    lib = _native.load()
    nmax = max(a.numel() for a, _ in pairs)
    out = torch.empty(len(pairs), dtype=torch.float64, device=pairs[0][0].device)
    ws = _native.workspace(lib.nft_reduce_workspace(nmax), out.device, "pairdot")
    P = _native.ptr
    for i, (a, b) in enumerate(pairs):
        a, b = a.contiguous(), b.contiguous()
        assert a.shape == b.shape
        _native._check(lib.nft_dot(P(a), P(b), a.numel(), _native.dtype_code(a.dtype), P(out[i:]), P(ws),
                                   _native.stream_ptr()))
    return out.cpu().numpy()


# ------------------------------------------------------------------ stages
from ..library.correlated_fields_simple import _O2_PAIRS, _PRO_FOLD  # noqa: E402


def _items(st, k):
    """device nft_amp_const array for k right-hand sides: the state's own rows,
    or its single linearisation point shared by all k"""
    if st["k"] != 1 or k == 1:
        return st["dconst"].data_ptr()
    rep = st.setdefault("rep", {})
    if k not in rep:
        rep[k] = st["dconst"].repeat(k)
    return rep[k].data_ptr()


class _CFStage:
    """The fused correlated-field model (library/correlated_fields_simple.py)
    evaluated on a batch of packed latent rows."""

    def __init__(self, model):
        self.m = model
        self.lay = model.layout
        self.off = dict(zip(self.lay.keys, self.lay.offsets))
        self.grid = tuple(model.harmonic_partner.shape)
        self.N = int(np.prod(self.grid))
        self.axes = tuple(range(1, 1 + len(self.grid)))
        self.xo = self.off[model.k_xi]

    def fwd(self, X):
        m = self.m
        k = X.shape[0]
        amp = m.amp
        X = X.contiguous()
        # all rows' amplitudes and linearisation constants in one native pass
        # (nft_amp_forward_batched; device structs, no host round trip)
        lin = amp.forward_rows(amp._ptrs(X, self.off), k, X.shape[1], X.device)
        A = lin.a
        afull = torch.empty((k,) + self.grid, dtype=A.dtype, device=A.device)
        b = m.bins
        _native.bin_gather(A, b.pindex, afull, k, b.npix, b.nbin, 1)
        # A * xi inside the transform's first pass (the prologue's product is
        # the separate multiply's: bitwise), not a (k, N) pass of its own
        s = torch.empty_like(afull)
        from ..ducc_dispatch import hartley_convention_code
        _native.hartley_fused(s, self.axes, m.c_h, pro=dict(a=afull, x=X[0, self.xo:]),
                              convention=hartley_convention_code(), shape=s.shape,
                              batch=dict(period=self.N, x=X.shape[1], a=self.N))
        if m.offset_mean is not None:
            s.add_(m.offset_mean)
        return s, dict(afull=afull, X=X, lin=lin, lins=[lin], dconst=lin.dconst, k=k)

    @staticmethod
    def stack(states):
        """one batch state from per-sample (state, row) pairs"""
        if len(states) == 1 and states[0][0]["k"] == 1:
            return states[0][0]
        if all(st is states[0][0] for st, _ in states) and [r for _, r in states] == list(range(states[0][0]["k"])):
            return states[0][0]
        afull = torch.stack([st["afull"][r] for st, r in states])
        X = torch.stack([st["X"][r] for st, r in states])
        dconst = torch.cat([st["lin"].row_bytes(r) for st, r in states])
        lins = [ln for st, _ in states for ln in st["lins"]]
        return dict(afull=afull, X=X, lin=states[0][0]["lin"], lins=lins, dconst=dconst, k=len(states))

    def jvp(self, st, V):
        """(k, grid) = J_cf(x_b) V[b]; st shared (k = 1) or per item"""
        from ..ducc_dispatch import hartley_convention_code
        m = self.m
        k, size = V.shape
        B = m.amp.B
        N = self.N
        shared = st["k"] == 1
        out = torch.empty((k,) + self.grid, dtype=V.dtype, device=V.device)
        Xs = st["X"]
        if shared:
            da = torch.empty((B, k), dtype=torch.float64, device=V.device)
            m.amp.native_jvp_batched(st["lin"], V, self.off, da, interleave=True, item_consts=_items(st, k))
            batch = dict(period=N, x=size, c=1, c_elem=k)
        else:
            da = torch.empty((k, B), dtype=torch.float64, device=V.device)
            m.amp.native_jvp_batched(st["lin"], V, self.off, da, item_consts=_items(st, k))
            batch = dict(period=N, x=size, c=B, a=N, b=Xs.shape[1])
        pro = dict(a=st["afull"], x=V[0, self.xo:], b=Xs[0, self.xo:], c=da, index=m.bins.pindex)
        jb = m.jbins
        if _PRO_FOLD and jb.fold is not None:
            # dA once per mirror class (correlated_fields_simple._pro_bins)
            pro.update(index=jb.fold["pindex"], fold=True)
        _native.hartley_fused(out, self.axes, m.c_h, pro=pro, convention=hartley_convention_code(),
                              shape=out.shape, batch=batch)
        return out

    def vjp(self, st, G, Q, d=None, shift=0.0):
        """Q[b] (packed rows, padding zero) = J_cf(x_b)^T G[b] (+ shift * d[b],
        added as the transform stores and inside the amplitude VJP)"""
        from ..ducc_dispatch import hartley_convention_code
        m = self.m
        k = G.shape[0]
        size = Q.shape[1]
        N = self.N
        shared = st["k"] == 1
        Xs = st["X"]
        # xi0 * v as point-mirror pair sums on the half grid where the CF
        # Jacobian's own adjoint uses them (CFJacobian._pairs)
        jac_pairs = _O2_PAIRS and m.jbins.fold is not None and len(self.grid) >= 2 and \
            _native.hartley_cg_blocks((k,) + self.grid, self.axes, G.dtype) > 0
        wshape = self.grid[:-1] + (self.grid[-1] // 2 + 1,) if jac_pairs else self.grid
        w = torch.empty((k,) + wshape, dtype=G.dtype, device=G.device)
        epi = dict(a=st["afull"], b=Xs[0, self.xo:], out2=w, pairs=jac_pairs)
        batch = dict(period=N, out=size, out2=w[0].numel())
        if not shared:
            batch.update(ea=N, eb=Xs.shape[1])
        if d is not None and shift != 0.0:
            epi.update(d=d[0, self.xo:], shift=shift)
            batch["d"] = d.shape[1]
        _native.hartley_fused(Q[0, self.xo:], self.axes, m.c_h, x=G.contiguous(), epi=epi,
                              convention=hartley_convention_code(), shape=(k,) + self.grid, batch=batch)
        ga = torch.empty((k, m.amp.B), dtype=G.dtype, device=G.device)
        if jac_pairs:
            wf = torch.empty((k, m.jbins.fold["nf"]), dtype=G.dtype, device=G.device)
            m.jbins.scatter_from(m.jbins.fold_into(w, wf, k, half=True), ga, k)
        else:
            m.jbins.scatter(w, ga, k)
        m.amp.native_vjp_batched(st["lin"], ga, Q, self.off, D=d, shift=shift if d is not None else 0.0,
                                 item_consts=_items(st, k))
        return Q


# a pointwise stage in front of the LOS response rides in the LOS kernels
# (NFT_FUSE_PTW=0: separate multiplies, for measurement)
_FUSE_PTW = os.environ.get("NFT_FUSE_PTW", "1") != "0"


class _PtwStage:
    def __init__(self, name, args, kwargs):
        from ..pointwise import ptw_dict
        self.name = name
        self.f = ptw_dict[name][1]
        self.args, self.kwargs = args, kwargs

    def fwd(self, U):
        if self.name == "sigmoid" and not self.args and not self.kwargs and U.is_cuda and \
                U.dtype in (torch.float64, torch.float32):
            # value and derivative in one native pass (bitwise pointwise._sigmoid)
            U = U.contiguous()
            return _native.sigmoid_pair(U, torch.empty_like(U), torch.empty_like(U))
        v, d = self.f(U, *self.args, **self.kwargs)
        return v, d

    @staticmethod
    def stack(states):
        if len(states) == 1 and states[0][0].shape[0] == 1:
            return states[0][0]
        return torch.stack([st[r] for st, r in states])

    def jvp(self, d, V):
        return V * d

    def vjp(self, d, G):
        return G * d


class _LinStage:
    """linear stage without state: ('scale', s) | ('diag', t) | ('reshape',) | ('los', R)"""

    def __init__(self, kind, v, dom_shape, tgt_shape):
        self.kind, self.v = kind, v
        self.dshape, self.tshape = tuple(dom_shape), tuple(tgt_shape)

    def fwd(self, U):
        return self.jvp(None, U), None

    @staticmethod
    def stack(states):
        return None

    def jvp(self, _, V):
        k = V.shape[0]
        if self.kind == "scale":
            return (V * self.v).reshape((k,) + self.tshape)
        if self.kind == "diag":
            return (V.reshape((k,) + self.dshape) * self.v).reshape((k,) + self.tshape)
        if self.kind == "reshape":
            return V.reshape((k,) + self.tshape)
        return _los_fwd(self.v, V.reshape(k, -1))

    def vjp(self, _, G):
        k = G.shape[0]
        if self.kind == "scale":
            return (G * self.v).reshape((k,) + self.dshape)
        if self.kind == "diag":
            return (G.reshape((k,) + self.tshape) * self.v).reshape((k,) + self.dshape)
        if self.kind == "reshape":
            return G.reshape((k,) + self.dshape)
        return _los_adj(self.v, G.reshape(k, -1)).reshape((k,) + self.dshape)


def _pixel_rows(d, k, a, b):
    """rows a:b of a pointwise derivative shared (1 row) or one per vector"""
    if d is None:
        return None
    return d.reshape(1, -1) if d.shape[0] == 1 else d.reshape(k, -1)[a:b]


def _los_fwd(R, V, d=None, scale=1.0):
    """scale * R (d * V) row by row; d (the derivative of a pointwise stage in
    front of R) is applied as the kernel loads the pixels, the scalar of a
    scaling stage behind R as it stores each line (nft_los_forward_ex: the
    same product as the separate multiply)."""
    from ..library.los_response import LOS_KMAX
    plan = R._box_plan()
    k = V.shape[0]
    V = V.contiguous()
    y = torch.empty((k, R.target.shape[0]), dtype=V.dtype, device=V.device)
    for a in range(0, k, LOS_KMAX):
        b = min(k, a + LOS_KMAX)
        if d is None:
            _native.los_forward_batched(plan, V[a:b], y[a:b], scale=scale)
        else:
            _native.los_forward_ex(plan, V[a:b], y[a:b], colscale=_pixel_rows(d, k, a, b), scale=scale)
    return y


def _los_adj(R, Y, d=None, ys=None):
    """d * R^T (ys * Y) row by row (d applied as the pixels are stored,
    nft_los_adjoint_ex; ys, a per-line vector, as the line values are read --
    the same product as the separate multiply)."""
    from ..library.los_response import LOS_KMAX
    plan = R._box_plan()
    k = Y.shape[0]
    Y = Y.contiguous()
    npix = int(np.prod(R.domain.shape))
    out = torch.empty((k, npix), dtype=Y.dtype, device=Y.device)
    for a in range(0, k, LOS_KMAX):
        b = min(k, a + LOS_KMAX)
        if d is None and ys is None:
            _native.los_adjoint_batched(plan, Y[a:b], out[a:b])
        else:
            _native.los_adjoint_ex(plan, Y[a:b], out[a:b], colscale=ys, rowscale=_pixel_rows(d, k, a, b))
    return out


class Pipeline:
    """f_lh on batches of packed latent rows; stages innermost first."""

    def __init__(self, stages, layout):
        self.stages = stages
        self.layout = layout

    @classmethod
    def parse(cls, f_lh):
        from ..library.correlated_fields_simple import _CorrelatedFieldModel
        from ..library.los_response import LOSResponse
        from ..operators.diagonal_operator import DiagonalOperator
        from ..operators.operator import _FunctionApplier, _OpChain
        from ..operators.scaling_operator import ScalingOperator
        from ..operators.simple_linear_operators import GeometryRemover
        from ..pointwise import ptw_dict
        if isinstance(f_lh, (list, tuple)):
            ops = [o for op in f_lh for o in (op._ops if isinstance(op, _OpChain) else (op,))]
        else:
            ops = list(f_lh._ops) if isinstance(f_lh, _OpChain) else [f_lh]
        if not ops or not isinstance(ops[-1], _CorrelatedFieldModel):
            return None
        stages = [_CFStage(ops[-1])]
        for op in reversed(ops[:-1]):
            if isinstance(op, ScalingOperator) and np.isreal(op._factor):
                f = float(np.real(op._factor))
                stages.append(_LinStage("scale", f, op.domain.shape, op.target.shape))
            elif isinstance(op, DiagonalOperator) and not op._complex:
                stages.append(_LinStage("diag", op.diagonal_tensor, op.domain.shape, op.target.shape))
            elif isinstance(op, GeometryRemover):
                stages.append(_LinStage("reshape", None, op.domain.shape, op.target.shape))
            elif isinstance(op, LOSResponse):
                stages.append(_LinStage("los", op, op.domain.shape, op.target.shape))
            elif isinstance(op, _FunctionApplier) and op._funcname in ptw_dict:
                stages.append(_PtwStage(op._funcname, op._args, op._kwargs))
            else:
                return None
        return cls(stages, ops[-1].layout)

    def fwd(self, X):
        states = []
        U = X
        for s in self.stages:
            U, st = s.fwd(U)
            states.append(st)
        return U, states

    def stack(self, rows):
        """batch state from [(states, row), ...]"""
        return [type(s).stack([(st[j], r) for st, r in rows]) for j, s in enumerate(self.stages)]

    def _fused_ptw_los(self, i, d, U):
        """stage i pointwise and stage i + 1 the LOS response: the derivative
        d is folded into the LOS kernel's pixel loads / stores"""
        if i + 1 >= len(self.stages) or not isinstance(self.stages[i], _PtwStage):
            return False
        nx = self.stages[i + 1]
        if not (isinstance(nx, _LinStage) and nx.kind == "los" and _FUSE_PTW):
            return False
        return d.dtype == U.dtype and d.is_contiguous() and d.shape[0] in (1, U.shape[0])

    def _scalar_after(self, j, dtype):
        """the factor of a scalar scaling stage at index j (it rides in the LOS
        kernel next to it), else None.  fp64 only: the kernels apply the factor
        in double, which is the separate multiply's rounding only when the
        vectors are double (fp32 vectors round after every multiply)"""
        if dtype == torch.float64 and j < len(self.stages) and isinstance(self.stages[j], _LinStage) \
                and self.stages[j].kind == "scale" and _FUSE_PTW:
            return float(self.stages[j].v)
        return None

    def jvp(self, states, V):
        U = self.stages[0].jvp(states[0], V)
        i = 1
        while i < len(self.stages):
            s, st = self.stages[i], states[i]
            if self._fused_ptw_los(i, st, U):
                f = self._scalar_after(i + 2, U.dtype)
                U = _los_fwd(self.stages[i + 1].v, U.reshape(U.shape[0], -1), st, 1.0 if f is None else f)
                i += 2 if f is None else 3
                continue
            U = s.jvp(st, U)
            i += 1
        return U

    def vjp(self, states, G, Q, d=None, shift=0.0):
        """Q (k, size) zero-padded packed rows = J^T G (+ shift * d, fused into
        the correlated field's adjoint)"""
        U = G
        i = len(self.stages) - 1
        while i >= 1:
            s, st = self.stages[i], states[i]
            f = self._scalar_after(i, U.dtype)
            if f is not None and i >= 3 and isinstance(self.stages[i - 1], _LinStage) and \
                    self.stages[i - 1].kind == "los" and self._fused_ptw_los(i - 2, states[i - 2], U):
                # scale stage, LOS, pointwise stage: one adjoint launch with the
                # scale as a per-line factor of the line values
                R = self.stages[i - 1].v
                ys = self.__dict__.setdefault("_lsc", {}).get((i, str(U.device)))
                if ys is None:
                    ys = torch.full((R.target.shape[0],), f, dtype=torch.float64, device=U.device)
                    self._lsc[(i, str(U.device))] = ys
                U = _los_adj(R, U.reshape(U.shape[0], -1), states[i - 2], ys=ys.to(U.dtype)).reshape(
                    (U.shape[0],) + self.stages[i - 1].dshape)
                i -= 3
                continue
            if i >= 2 and self._fused_ptw_los(i - 1, states[i - 1], U):
                U = _los_adj(s.v, U.reshape(U.shape[0], -1), states[i - 1]).reshape((U.shape[0],) + s.dshape)
                i -= 2
                continue
            U = s.vjp(st, U)
            i -= 1
        return self.stages[0].vjp(states[0], U, Q, d, shift)


# ------------------------------------------------------------------ energies
class _BEnergy(Energy):
    """Energy of one sample at a packed position (value / gradient on the
    device, value and |gradient| already on the host)."""

    def __init__(self, ctx, x, g, value, gnorm, states, row):
        super().__init__(None)
        self.ctx, self.x, self.g = ctx, x, g
        self._val, self._gradnorm = value, gnorm
        self.states, self.row = states, row

    @property
    def position(self):
        return self.ctx.layout.unpack(self.x)

    @property
    def value(self):
        return self._val

    @property
    def gradient(self):
        return self.ctx.layout.unpack(self.g)

    @property
    def gradient_norm(self):
        return self._gradnorm

    def at(self, position):
        raise NotImplementedError("batched geoVI energies are evaluated by their driver")


class _Dir:
    """packed descent direction (what the line search's pk is here)"""

    def __init__(self, v):
        self.v = v

    def norm(self):
        return float(torch.linalg.vector_norm(self.v))


class GeoVIBatch:
    """Batched refinement of k samples around one expansion point."""

    def __init__(self, pipe, x0, minimizer):
        self.pipe = pipe
        self.layout = pipe.layout
        self.minimizer = minimizer
        X0 = x0.reshape(1, -1)
        F0, st0 = pipe.fwd(X0)
        self.st0 = st0                   # J0: shared by every sample
        self.x0 = X0
        # transformation_mean = x0 + J0^T f(x0)  (kl_energies.py:118)
        self.tmean = (X0 + self._J0T(F0))[0]

    # J0 / J0^T (shared) and J / J^T (per item) on packed rows
    def _J0(self, V):
        return self.pipe.jvp(self.st0, V)

    def _latent(self, k, device):
        """(k, size) buffer for a J^T output: every key segment is overwritten
        by the adjoint, so only the alignment padding is zeroed"""
        lay = self.layout
        Q = torch.empty((k, lay.size), dtype=torch.float64, device=device)
        ends = [o + n for o, n in zip(lay.offsets, lay.sizes)]
        starts = list(lay.offsets[1:]) + [lay.size]
        for a, b in zip(ends, starts):
            if b > a:
                Q[:, a:b] = 0.0
        return Q

    def _scratch(self, k, device):
        """a _latent buffer kept for intermediates that die inside one call
        (the metric's u, evaluate's residual): its padding is zeroed once, not
        by several fill launches per call.  Not created during a graph
        capture (the capture takes a fresh buffer from its own pool).
        One buffer per device, as many rows as the largest batch asked for;
        a batch of k rows gets its first k rows (the batches only shrink as
        samples finish: one buffer instead of one per batch size).  A buffer
        outgrown by a larger batch is retired, not freed: a captured graph may
        still write into it."""
        cache = self.__dict__.setdefault("_scr", {})
        key = str(device)
        Q = cache.get(key)
        if Q is None or Q.shape[0] < k:
            if torch.cuda.is_current_stream_capturing():
                return self._latent(k, device)
            if Q is not None:
                self.__dict__.setdefault("_scr_retired", []).append(Q)
            Q = cache[key] = self._latent(k, device)
        return Q[:k]

    def _J0T(self, F, plus=None, out=None):
        """J0^T F (+ plus, added inside the adjoint: bitwise the separate add)"""
        Q = self._latent(F.shape[0], F.device) if out is None else out
        return self.pipe.vjp(self.st0, F, Q, plus, 1.0)

    def _JT(self, states, G, plus=None):
        return self.pipe.vjp(states, G, self._latent(G.shape[0], G.device), plus, 1.0)

    def evaluate(self, X, M):
        """values, |gradient|, gradients and per-sample states at the rows of X"""
        F, states = self.pipe.fwd(X)
        # + X inside the adjoint (bitwise the separate add, _J0T)
        Rr = self._J0T(F, plus=X, out=self._scratch(X.shape[0], X.device))
        Rr.sub_(M)
        G = self._JT(states, self._J0(Rr), plus=Rr)
        k = X.shape[0]
        h = _rowdots([(Rr, Rr), (G, G)])
        vals = [0.5 * float(h[0, i]) for i in range(k)]
        gn = [math.sqrt(float(h[1, i])) for i in range(k)]
        return vals, gn, G, states

    def metric_batch(self, states):
        """callable (D, Q) -> Q = M_b D for the stacked per-sample states"""
        def mv(D, Q):
            U = self._J0T(self.pipe.jvp(states, D), plus=D, out=self._scratch(D.shape[0], D.device))
            self.pipe.vjp(states, self._J0(U), Q, U, 1.0)   # overwrites every key segment
            return Q
        return mv

    def refine(self, starts, means):
        """starts, means: lists of packed latent vectors.  Returns the final
        packed positions (one per sample)."""
        k = len(starts)
        X = torch.stack(starts)
        M = torch.stack(means)
        self._M = {i: M[i] for i in range(k)}
        self._Mall = M
        vals, gn, G, states = self.evaluate(X, M)
        gens, pending, results = [], {}, [None] * k
        for i in range(k):
            v = vals[i]
            if np.isnan(v):   # EnergyAdapter(nanisinf=True)
                v = np.inf
            e = _BEnergy(self, X[i], G[i], v, gn[i], states, i)
            e.sample = i
            # one minimizer per sample: controllers are stateful (the reference
            # reuses one minimizer sample after sample, start() resetting it)
            mz = copy.copy(self.minimizer)
            mz._controller = copy.deepcopy(self.minimizer._controller)
            gen = mz.minimize_gen(e)
            gens.append(gen)
            self._advance(i, gen, None, pending, results, first=True)
        while pending:
            kinds = {}
            for i, req in pending.items():
                kinds.setdefault(req[0], []).append(i)
            answers = {}
            # Newton directions wait while other samples still evaluate
            # energies (their next requests are mostly directions too): larger
            # direction batches, and the batched CG compacts as they stop
            if "dir" in kinds and not (DEFER_DIR and "at" in kinds):
                answers.update(self._serve_dir([(i, pending[i]) for i in kinds["dir"]]))
            if "at" in kinds:
                answers.update(self._serve_at([(i, pending[i]) for i in kinds["at"]]))
            if "dd" in kinds:
                answers.update(self._serve_dd([(i, pending[i]) for i in kinds["dd"]]))
            for i, ans in answers.items():
                self._advance(i, gens[i], ans, pending, results)
        return [r[0].x for r in results]

    @staticmethod
    def _advance(i, gen, ans, pending, results, first=False):
        try:
            pending[i] = next(gen) if first else gen.send(ans)
        except StopIteration as e:
            pending.pop(i, None)
            results[i] = e.value

    def _serve_at(self, reqs):
        # rows x + alpha p formed in place (alpha p, then + x: the reference's
        # two roundings), no stacking copy
        X = torch.empty((len(reqs), self.layout.size), dtype=reqs[0][1][1].x.dtype, device=self.x0.device)
        for j, (_, r) in enumerate(reqs):
            torch.mul(r[3].v, r[2], out=X[j])
            X[j].add_(r[1].x)
        idx = [r[1].sample for _, r in reqs]
        M = self._Mall if idx == list(range(self._Mall.shape[0])) else self._Mall[idx]
        vals, gn, G, states = self.evaluate(X, M)
        out = {}
        for j, (i, r) in enumerate(reqs):
            v = vals[j]
            if np.isnan(v):
                v = np.inf
            e = _BEnergy(self, X[j], G[j], v, gn[j], states, j)
            e.sample = r[1].sample
            out[i] = e
        return out

    def _serve_dd(self, reqs):
        # one dot per request on the rows where they live (bitwise the
        # batched dot of the stacked rows, without the stacking copies)
        h = _pairdots([(r[1].g, r[2].v) for _, r in reqs])
        return {i: float(h[j]) for j, (i, _) in enumerate(reqs)}

    def _serve_dir(self, reqs):
        from .conjugate_gradient import ConjugateGradient  # noqa: F401
        from .fused_cg import FusedCGBatch, _State
        from .iteration_controllers import AbsDeltaEnergyController, GradientNormController
        from . import trace
        mz = self.minimizer
        ctls = []
        for _, (_, e, old, stag) in reqs:
            if old is None:
                ctls.append(GradientNormController(iteration_limit=5))
            else:
                ediff = mz._alpha * (old - e.value)
                ctls.append(AbsDeltaEnergyController(ediff, iteration_limit=mz._max_cg_iterations, name=mz._name))
            trace.tag(ctls[-1], ("dir", stag))
        pairs = [(r[1].states, r[1].row) for _, r in reqs]
        G = torch.stack([r[1].g for _, r in reqs])

        def make(rows):
            """the stacked Newton metrics of the requests `rows`; restricts
            itself to any subset of them (FusedCGBatch compaction)"""
            c = _MetricCore(self.metric_batch(self.pipe.stack([pairs[i] for i in rows])), self.layout)
            c.subset = make
            return c
        core = make(list(range(len(pairs))))
        cg = FusedCGBatch(core, None, 0.0, ctls, mz._nreset)
        # QuadraticEnergy(0 * x, metric, g, _grad=-g) of NewtonCG.get_descent_direction:
        # value 0, |gradient| = |g|
        starts = [_State(0.0, r[1].gradient_norm, lambda: None) for _, r in reqs]
        X, status = cg.run_packed(torch.zeros_like(G), -G, G, starts)
        out = {}
        for j, (i, _) in enumerate(reqs):
            if status[j][0] == ctls[j].ERROR:
                raise ValueError("Cannot find descent direction")
            out[i] = _Dir(-X[j])
        return out


class _MetricCore:
    """metric_flat_batch adapter of per-sample Newton metrics for FusedCGBatch"""

    def __init__(self, mv, layout):
        self.mv = mv
        self.layout = layout
        self.device = layout.device
        # restriction to a subset of the rows (original indices), or None
        self.subset = None

    def metric_flat_batch(self, D, Q, W, shift):
        self.mv(D, Q)
        if shift != 0.0:
            Q.add_(D, alpha=shift)
        return Q


def plan(minimizer, f_lh, _unused, position):
    """GeoVIBatch for this draw_samples call (expansion point `position`, a
    latent MultiField), or None if the refinement has to run per sample
    (unsupported model chain or minimizer)."""
    from .descent_minimizers import NewtonCG
    from .line_search import LineSearch
    if not ENABLED:
        return None
    if type(minimizer) is not NewtonCG or type(minimizer.line_searcher) is not LineSearch:
        return None
    if minimizer._napprox != 0 or minimizer._history is not None:
        return None
    pipe = Pipeline.parse(f_lh)
    if pipe is None or pipe.layout.device.type != "cuda" or pipe.layout.domain != position.domain:
        return None
    try:
        return GeoVIBatch(pipe, pipe.layout.pack(position), minimizer)
    except NotImplementedError as e:
        logger.info(f"batched geoVI refinement unavailable: {e}")
        return None


# ------------------------------------------------------------------ KL terms
def _likelihood(hamiltonian, positions):
    """(kind, E, icov value, scale, pipeline) of a StandardHamiltonian whose
    likelihood is GaussianEnergy(data, scaling / diagonal inverse covariance)
    or PoissonianEnergy (optionally scaled) on a supported model chain, else
    None."""
    from ..operators.diagonal_operator import DiagonalOperator
    from ..operators.energy_operators import GaussianEnergy, PoissonianEnergy, _LikelihoodChain
    from ..operators.scaling_operator import ScalingOperator
    lh = hamiltonian.likelihood_energy
    if not isinstance(lh, _LikelihoodChain):
        return None
    ops = list(lh._op._ops)
    scale = 1.0
    if isinstance(ops[0], ScalingOperator):      # scaled likelihood (lh.scale(f))
        scale = float(np.real(ops[0]._factor))
        ops = ops[1:]
    E = ops[0]
    icv = None
    if isinstance(E, GaussianEnergy):
        if E._data is None:
            return None
        ic = E._icov
        if isinstance(ic, ScalingOperator) and np.isreal(ic._factor):
            icv = float(np.real(ic._factor))
        elif isinstance(ic, DiagonalOperator) and not ic._complex:
            icv = ic.diagonal_tensor.reshape(-1)
        else:
            return None
        kind = "gauss"
    elif isinstance(E, PoissonianEnergy):
        kind = "poisson"
    else:
        return None
    pipe = Pipeline.parse(ops[1:])
    if pipe is None or pipe.layout.device.type != "cuda" or pipe.layout.domain != positions[0].domain:
        return None
    return kind, E, icv, scale, pipe


def kl_batch(hamiltonian, positions):
    """Hamiltonian values and gradients at a list of latent MultiFields in one
    batched pass (SampledKLEnergyClass, kl_energies.py:295-356: its per
    sample H(Linearization.make_var(s)) evaluations), or None if the
    likelihood is not a GaussianEnergy(data, scaling / diagonal inverse
    covariance) or PoissonianEnergy applied to a supported model chain.

    Returns ([value_i], [gradient_i MultiField])."""
    # one position too: per row the batched pass does not depend on the
    # batch, so a rank holding one sample computes the 1-rank run's terms
    if not ENABLED or len(positions) < 1:
        return None
    parsed = _likelihood(hamiltonian, positions)
    if parsed is None:
        return None
    kind, E, icv, scale, pipe = parsed
    lay = pipe.layout
    X = torch.stack([lay.pack(p) for p in positions])
    k = X.shape[0]
    Sf, states = pipe.fwd(X)
    S = Sf.reshape(k, -1)
    if kind == "gauss":
        d = E._data.val.reshape(1, -1).to(S.dtype)
        R = S - d
        W = R * icv
        h = _rowdots([(R, W), (X, X)])
        lval = 0.5 * h[0]
        gs = W
    else:
        d = E._dfloat.val.reshape(1, -1)
        D = d.expand_as(S).contiguous()
        ones = torch.ones_like(S)
        h = _rowdots([(S, ones), (torch.log(S), D), (X, X)])
        lval = h[0] - h[1]
        h = h[[0, 2]]
        gs = 1. - D / S
    if scale != 1.0:
        lval = scale * lval
        gs = gs * scale
    Q = torch.empty((k, lay.size), dtype=torch.float64, device=X.device)
    ends = [o + n for o, n in zip(lay.offsets, lay.sizes)]
    starts = list(lay.offsets[1:]) + [lay.size]
    for a, b in zip(ends, starts):
        if b > a:
            Q[:, a:b] = 0.0
    G = pipe.vjp(states, gs.reshape(Sf.shape).contiguous(), Q)
    G.add_(X)                                      # prior: 0.5 x.x
    vals = [float(lval[i]) + 0.5 * float(h[1, i]) for i in range(k)]
    return vals, [lay.unpack(G[i]) for i in range(k)]


def kl_metric_batch(hamiltonian, positions):
    """The per-sample Hamiltonian metrics of SampledKLEnergyClass.apply_metric
    (kl_energies.py:340-350: per sample and per application a full
    H(Linearization.make_var(s, want_metric=True)) rebuild) linearised ONCE
    at the k local sample positions and applied to all of them in one batched
    pass: M_s x = J_s^T W_s J_s x + x with W_s the likelihood's Fisher metric
    at s (Gaussian: the inverse covariance; Poissonian: 1 / lambda_s; times
    the likelihood scale) and the identity of the standard prior.

    Returns a callable x -> [M_s x for every local sample] (MultiFields, in
    sample order, for the caller's sample average), or None when the
    Hamiltonian is not covered (then the caller keeps the reference's
    per-sample path)."""
    if not ENABLED or not positions:
        return None
    parsed = _likelihood(hamiltonian, positions)
    if parsed is None:
        return None
    kind, E, icv, scale, pipe = parsed
    lay = pipe.layout
    X = torch.stack([lay.pack(p) for p in positions])
    k = X.shape[0]
    Sf, states = pipe.fwd(X)
    if kind == "gauss":
        W = icv if isinstance(icv, float) else icv.reshape((1,) + tuple(Sf.shape[1:]))
    else:
        W = 1. / Sf
    if scale != 1.0:
        W = W * scale
    del X

    def apply(x):
        v = lay.pack(x)
        V = v.reshape(1, -1).expand(k, -1).contiguous()
        U = pipe.jvp(states, V)
        U = (U * W).contiguous()
        Q = torch.empty((k, lay.size), dtype=torch.float64, device=V.device)
        ends = [o + n for o, n in zip(lay.offsets, lay.sizes)]
        starts = list(lay.offsets[1:]) + [lay.size]
        for a, b in zip(ends, starts):
            if b > a:
                Q[:, a:b] = 0.0
        pipe.vjp(states, U, Q)
        Q.add_(V)
        return [lay.unpack(Q[i]) for i in range(k)]
    return apply
