"""On-disk state of optimize_kl: sample lists, random state, energy history.

Same directory layout, file-name stems and resume protocol as the reference
(src/minimization/optimize_kl.py:297-317,384-393,430-458,
src/minimization/sample_list.py:510-531,626-653):

    <out>/last_finished_iteration                      text, the last index
    <out>/pickle/<stem>.mean.npz                        mean (MPI master)
    <out>/pickle/<stem>.<global sample index>.npz       residual + neg flag
    <out>/pickle/nifty_random_state_<stem>.json         seed-sequence stack
    <out>/pickle/energy_history_<stem>.json             (iteration, KL value)

with <stem> = "last" or "iteration_<i>" (save_strategy).  The reference
pickles its Python objects; here every object is data only: fields as numpy
.npz (one array per key plus a JSON domain descriptor), states and histories
as JSON, so a checkpoint loads without executing anything from the file.
Domains are rebuilt from the descriptor (RGSpace, UnstructuredDomain) or
taken from the caller's domain for the keys it names."""
import json
import os

import numpy as np
import torch

from ..domain_tuple import DomainTuple
from ..domains import RGSpace, UnstructuredDomain
from ..field import Field
from ..multi_domain import MultiDomain
from ..multi_field import MultiField


def _dom_desc(dom):
    out = []
    for sp in dom:
        if isinstance(sp, RGSpace):
            out.append({"type": "RGSpace", "shape": list(sp.shape), "distances": list(sp.distances),
                        "harmonic": bool(sp.harmonic)})
        elif isinstance(sp, UnstructuredDomain):
            out.append({"type": "UnstructuredDomain", "shape": list(sp.shape)})
        else:
            out.append({"type": type(sp).__name__, "shape": list(sp.shape)})
    return out


def _dom_from_desc(desc):
    sps = []
    for d in desc:
        if d["type"] == "RGSpace":
            sps.append(RGSpace(tuple(d["shape"]), tuple(d["distances"]), d["harmonic"]))
        elif d["type"] == "UnstructuredDomain":
            sps.append(UnstructuredDomain(tuple(d["shape"])))
        else:
            raise ValueError(f"checkpoint: domain type {d['type']} needs the caller's domain")
    return DomainTuple.make(tuple(sps))


def save_field(fname, fld, extra=None, overwrite=False):
    """Field / MultiField (+ JSON-able extras) -> <fname> (.npz)"""
    if os.path.isfile(fname):
        if not overwrite:
            raise FileExistsError(fname)
        os.remove(fname)
    arrays, meta = {}, {"extra": extra or {}}
    if isinstance(fld, MultiField):
        meta["kind"] = "MultiField"
        meta["keys"] = list(fld.keys())
        meta["domains"] = {k: _dom_desc(fld.domain[k]) for k in fld.keys()}
        for k in fld.keys():
            arrays["k_" + k] = np.asarray(fld[k].val.cpu().numpy() if torch.is_tensor(fld[k].val) else fld[k].val)
    else:
        meta["kind"] = "Field"
        meta["domains"] = {"": _dom_desc(fld.domain)}
        arrays["k_"] = np.asarray(fld.val.cpu().numpy() if torch.is_tensor(fld.val) else fld.val)
    arrays["__meta__"] = np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8)
    tmp = fname + ".tmp.npz"
    np.savez(tmp, **arrays)
    os.replace(tmp, fname)


def load_field(fname, domain=None):
    """(Field / MultiField, extras); keys of `domain` (a MultiDomain or, for a
    Field, a DomainTuple) take that domain, the others their descriptor's"""
    with np.load(fname, allow_pickle=False) as z:
        meta = json.loads(bytes(z["__meta__"]).decode())
        arrs = {k[2:]: np.array(z[k]) for k in z.files if k.startswith("k_")}
    if meta["kind"] == "Field":
        dom = domain if domain is not None else _dom_from_desc(meta["domains"][""])
        return Field.from_raw(DomainTuple.make(dom), arrs[""]), meta["extra"]
    doms = {}
    for k in meta["keys"]:
        if isinstance(domain, MultiDomain) and k in domain.keys():
            doms[k] = domain[k]
        else:
            doms[k] = _dom_from_desc(meta["domains"][k])
    md = MultiDomain.make(doms)
    return MultiField.from_dict({k: Field.from_raw(md[k], arrs[k]) for k in meta["keys"]}, md), meta["extra"]


def load_domain(fname, domain=None):
    """the domain of the field stored in `fname` from its descriptor alone
    (no array is read); keys of `domain` take that domain, as in load_field"""
    with np.load(fname, allow_pickle=False) as z:
        meta = json.loads(bytes(z["__meta__"]).decode())
    if meta["kind"] == "Field":
        return DomainTuple.make(domain if domain is not None else _dom_from_desc(meta["domains"][""]))
    doms = {}
    for k in meta["keys"]:
        if isinstance(domain, MultiDomain) and k in domain.keys():
            doms[k] = domain[k]
        else:
            doms[k] = _dom_from_desc(meta["domains"][k])
    return MultiDomain.make(doms)


def save_json(fname, obj):
    tmp = fname + ".tmp"
    with open(tmp, "w") as f:
        json.dump(obj, f)
    os.replace(tmp, fname)


def load_json(fname):
    with open(fname) as f:
        return json.load(f)


# ------------------------------------------------------------ random state
def _sseq_state(ss):
    return {"entropy": ss.entropy if isinstance(ss.entropy, int) else [int(e) for e in ss.entropy],
            "spawn_key": [int(k) for k in ss.spawn_key], "pool_size": int(ss.pool_size),
            "n_children_spawned": int(ss.n_children_spawned)}


def random_state():
    """JSON-able state of nifty_amd.random (the reference: pickle of its
    (sseq stack, generator stack), src/random.py:89-111)"""
    from .. import random
    return {"sseq": [_sseq_state(s) for s in random._sseq],
            "rng": [r.bit_generator.state for r in random._rng]}


def set_random_state(st):
    from .. import random
    ss, rr = [], []
    for s, g in zip(st["sseq"], st["rng"]):
        seq = np.random.SeedSequence(s["entropy"], spawn_key=tuple(s["spawn_key"]), pool_size=s["pool_size"],
                                     n_children_spawned=s["n_children_spawned"])
        gen = np.random.Generator(np.random.PCG64(seq))
        gen.bit_generator.state = g
        ss.append(seq)
        rr.append(gen)
    random._sseq[:] = ss
    random._rng[:] = rr
