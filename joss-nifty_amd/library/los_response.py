"""Line-of-sight response (src/library/los_response.py:34-233).

Construction (host, setup only): every line of sight is traversed through the
pixel grid (Amanatides-Woo style cell crossing distances), giving per-pixel
path lengths (optionally tapered by the parallax error function); entries are
ordered by 16x16 pixel boxes exactly as the reference orders its COO matrix.
The triplets are then regrouped into the box-blocked layout of
csrc/nft_los.hip (box_plan): per 256-pixel box, the runs of each line (for
R x) and the runs of each pixel (for R^T y), float32 weights as in the
reference, fp64 accumulation in fixed order."""
import ctypes
import os

import numpy as np
import torch
from scipy.special import erfc

from .. import _native, config
from ..domain_tuple import DomainTuple
from ..domains import RGSpace, UnstructuredDomain
from ..field import Field
from ..operators.linear_operator import LinearOperator


def _gaussian_sf(x):
    return 0.5 * erfc(x / np.sqrt(2.))


def _apply_erf(wgt, dist, lo, mid, hi, sig, erf):
    wgt = wgt.copy()
    mask = dist > hi
    wgt[mask] = 0.
    mask = (dist > lo) & (dist <= hi)
    wgt[mask] *= erf((-1 / dist[mask] + 1 / mid) / sig)
    return wgt


def _traverse(start, end, shp, dist, lo, mid, hi, sig, erf):
    """Per-LOS (flat pixel indices, weights) (los_response.py:34-91)."""
    ndim = start.shape[0]
    nlos = start.shape[1]
    inc = np.full(len(shp), 1, dtype=np.int64)
    for i in range(-2, -len(shp) - 1, -1):
        inc[i] = inc[i + 1] * shp[i + 1]
    pmax = np.array(shp)
    out = [None] * nlos
    for i in range(nlos):
        direction = end[:, i] - start[:, i]
        dirx = np.where(direction == 0., 1e-12, direction)
        d0 = np.where(direction == 0., ((start[:, i] > 0) - 0.5) * 1e12, -start[:, i] / dirx)
        d1 = np.where(direction == 0., ((start[:, i] < pmax) - 0.5) * -1e12, (pmax - start[:, i]) / dirx)
        dmin = np.minimum(d0, d1).max()
        dmax = np.maximum(d0, d1).min()
        dmin = np.maximum(0., dmin)
        dmax = np.minimum(1., dmax)
        dmax = np.maximum(dmin, dmax)
        dmin += 1e-7
        dmax -= 1e-7
        if dmin >= dmax:
            out[i] = (np.full(0, 0, dtype=np.int64), np.full(0, 0.))
            continue
        c_first = np.ceil(start[:, i] + direction * dmin)
        c_first = np.where(direction > 0., c_first, c_first - 1.)
        c_first = (c_first - start[:, i]) / dirx
        pos1 = np.asarray((start[:, i] + dmin * direction), dtype=np.int64)
        pos1 = np.sum(pos1 * inc)
        cdist = np.empty(0, dtype=np.float64)
        add = np.empty(0, dtype=np.int64)
        for j in range(ndim):
            if direction[j] != 0:
                step = inc[j] if direction[j] > 0 else -inc[j]
                tmp = np.arange(start=c_first[j], stop=dmax, step=abs(1. / direction[j]))
                cdist = np.append(cdist, tmp)
                add = np.append(add, np.full(len(tmp), step, dtype=np.int64))
        idx = np.argsort(cdist)
        cdist = cdist[idx]
        add = add[idx]
        cdist = np.append(np.full(1, dmin), cdist)
        cdist = np.append(cdist, np.full(1, dmax))
        cdist *= np.linalg.norm(direction * dist)
        wgt = np.diff(cdist)
        mdist = 0.5 * (cdist[:-1] + cdist[1:])
        wgt = _apply_erf(wgt, mdist, lo[i], mid[i], hi[i], sig[i], erf)
        add = np.cumsum(np.append(pos1, add))
        out[i] = (add, wgt)
    return out


def los_coo(shape, distances, starts, ends, sigmas=None, truncation=3.):
    """(row=los, col=pixel, float32 weight) in the reference's storage order."""
    ndim = len(shape)
    starts = np.array(starts, dtype=np.float64)
    ends = np.array(ends, dtype=np.float64)
    nlos = starts.shape[1]
    if sigmas is None:
        sigmas = np.zeros(nlos, dtype=np.float32)
    sigmas = np.array(sigmas)
    if starts.shape[0] != ndim or nlos != sigmas.shape[0] or starts.shape != ends.shape:
        raise TypeError("dimension mismatch")
    diffs = ends - starts
    difflen = np.linalg.norm(diffs, axis=0)
    diffs /= difflen
    real_distances = 1. / (1. / difflen - truncation * sigmas)
    if np.any(real_distances < 0):
        raise ValueError("parallax error truncation to high: getting negative distances")
    real_ends = starts + diffs * real_distances
    dist = np.array(distances).reshape((-1, 1))
    w_i = _traverse(starts / dist + 0.5, real_ends / dist + 0.5, shape, np.array(distances),
                    1. / (1. / difflen + truncation * sigmas), difflen,
                    1. / (1. / difflen - truncation * sigmas), sigmas, _gaussian_sf)
    boxsz = 16
    npix = int(np.prod(shape))
    ntot = sum(len(i[1]) for i in w_i)
    pri = np.empty(ntot, dtype=np.float64)
    ilos = np.empty(ntot, dtype=np.int32)
    iarr = np.empty(ntot, dtype=np.int32)
    xwgt = np.empty(ntot, dtype=np.float32)
    ofs = 0
    for cnt, i in enumerate(w_i):
        nval = len(i[1])
        ilos[ofs:ofs + nval] = cnt
        iarr[ofs:ofs + nval] = i[0]
        xwgt[ofs:ofs + nval] = i[1]
        fullidx = np.unravel_index(i[0], shape)
        tmp = np.zeros(nval, dtype=np.float64)
        fct = 1.
        for j in range(ndim):
            tmp += (fullidx[j] // boxsz) * fct
            fct *= shape[j]
        tmp += cnt / float(nlos)
        tmp += iarr[ofs:ofs + nval] / (float(nlos) * float(npix))
        pri[ofs:ofs + nval] = tmp
        ofs += nval
    order = np.argsort(pri)
    return ilos[order], iarr[order], xwgt[order], nlos


LOS_CAP_F = 2048   # entries per forward work item (csrc/nft_los.hip)
LOS_KMAX = 8       # vectors per batched LOS launch (csrc/nft_los.hip)
# the carried CG's curvature fold inside the LOS adjoint launch
# (nft_los_adjoint_fold); NFT_LOS_FOLD=0: its own launch (A/B, tests)
_FOLD_IN_ADJ = os.environ.get("NFT_LOS_FOLD", "1") != "0"
BOX = 256


def box_plan(rows, cols, w, shape, nlos):
    """Regroup COO triplets (storage order) into the box-blocked layout of
    nft_los_plan (include/nifty_amd.h).  Returns a dict of numpy arrays and
    geometry ints.  Within every (box, line) segment and every (box, pixel)
    run the entries keep their COO order."""
    shape = tuple(int(v) for v in shape)
    ndim = len(shape)
    W = shape[-1]
    H = shape[-2] if ndim >= 2 else 1
    bh, bw = (16, 16) if ndim >= 2 else (1, BOX)
    nby, nbx = -(-H // bh), -(-W // bw)
    L = int(np.prod(shape[:-2])) if ndim > 2 else 1
    nbox = L * nby * nbx
    n = len(rows)
    if n >= 2 ** 31 - 1:
        raise ValueError("LOS response too large for int32 entry offsets")
    rows = np.asarray(rows, dtype=np.int64)
    c = np.asarray(cols, dtype=np.int64)
    x = c % W
    t = c // W
    y = t % H
    lyr = t // H
    box = (lyr * nby + y // bh) * nbx + x // bw
    loc = (y % bh) * bw + x % bw
    # ---- forward: segments = runs of one line inside one box
    key = box * nlos + rows
    of = np.argsort(key, kind="stable")
    kb = key[of]
    segstart = np.flatnonzero(np.r_[True, kb[1:] != kb[:-1]]) if n else np.zeros(0, np.int64)
    nseg = len(segstart)
    seg_ent = np.r_[segstart, n].astype(np.int32)
    seg_box = box[of][segstart]
    seg_los = rows[of][segstart]
    # work items: all segments of a box, split where a box exceeds 256
    # segments or LOS_CAP_F entries
    segcnt = np.bincount(seg_box, minlength=nbox)
    entcnt = np.bincount(box, minlength=nbox)
    first_seg = np.r_[0, np.cumsum(segcnt)][:-1]
    big = (segcnt > BOX) | (entcnt > LOS_CAP_F)
    item_box, item_seg = [], []
    for b in np.flatnonzero(segcnt):
        s0 = int(first_seg[b])
        s1 = s0 + int(segcnt[b])
        if not big[b]:
            item_box.append(b)
            item_seg.append(s0)
            continue
        s = s0
        while s < s1:
            e = s + 1
            while e < s1 and e - s < BOX and seg_ent[e + 1] - seg_ent[s] <= LOS_CAP_F:
                e += 1
            if seg_ent[e] - seg_ent[s] > LOS_CAP_F:
                raise ValueError("a single line crosses a box with more than LOS_CAP_F entries")
            item_box.append(b)
            item_seg.append(s)
            s = e
    item_seg.append(nseg)
    # the work items of every box (items are appended in box order)
    box_item = np.r_[0, np.cumsum(np.bincount(np.asarray(item_box, dtype=np.int64), minlength=nbox))].astype(np.int32)
    # partial slots in line-major order (boxes ascending within a line)
    olm = np.lexsort((seg_box, seg_los))
    seg_slot = np.empty(nseg, dtype=np.int32)
    seg_slot[olm] = np.arange(nseg, dtype=np.int32)
    los_ptr = np.r_[0, np.cumsum(np.bincount(seg_los, minlength=nlos))].astype(np.int32)
    # ---- adjoint: entries sorted by (box, local pixel)
    key2 = box * BOX + loc
    oa = np.argsort(key2, kind="stable")
    if entcnt.max(initial=0) >= 65536:
        raise ValueError("more than 65535 LOS entries in one 256-pixel box")
    pc = np.bincount(key2, minlength=nbox * BOX).reshape(nbox, BOX)
    pix_off = np.zeros((nbox, BOX + 1), dtype=np.uint16)
    pix_off[:, 1:] = np.cumsum(pc, axis=1)
    # lines crossing each box (= the forward segments, in (box, line) order)
    # and each adjoint entry's index into its box's list
    box_lptr = np.r_[0, np.cumsum(segcnt)].astype(np.int32)
    seg_id = np.searchsorted(kb[segstart], key[oa])
    lidx = seg_id - box_lptr[box[oa]]
    if segcnt.max(initial=0) > 65535:
        raise ValueError("more than 65535 lines of sight cross one 256-pixel box")
    lidx8 = segcnt.max(initial=0) <= 256
    wf = np.asarray(w, dtype=np.float32)
    item_seg = np.asarray(item_seg, dtype=np.int64)
    fwd = dict(seg_ent=seg_ent, seg_slot=seg_slot, ent_loc=loc[of].astype(np.uint8), ent_wf=wf[of])
    # 16 entries of padding: the per-box forward stages aligned 16-entry
    # chunks, the last one may reach past an item's (and the array's) end
    fwd["ent_loc"] = np.r_[fwd["ent_loc"], np.zeros(16, np.uint8)]
    fwd["ent_wf"] = np.r_[fwd["ent_wf"], np.zeros(16, np.float32)]
    return dict(H=H, W=W, bh=bh, bw=bw, nby=nby, nbx=nbx, nbox=nbox, nlos=int(nlos),
                nitems=len(item_box), nseg=nseg, L=L,
                item_box=np.asarray(item_box, dtype=np.int32), item_seg=item_seg.astype(np.int32),
                item_ent=seg_ent[item_seg].astype(np.int32), **fwd,
                box_item=box_item, los_ptr=los_ptr, box_ent=np.r_[0, np.cumsum(entcnt)].astype(np.int32), pix_off=pix_off,
                box_lptr=box_lptr, box_lines=seg_los.astype(np.int32),
                **_adj_entries(lidx.astype(np.uint8 if lidx8 else np.uint16), wf[oa], entcnt, lidx8))


def _adj_entries(lidx, wa, entcnt, lidx8):
    """The adjoint's entry arrays; with 8-bit line indices every box's run
    padded to a multiple of 16 entries (index 0, weight 0: never summed, the
    pixel runs end before them) and its start in box_ent_adj, so the batched
    adjoint stages them with 16-byte loads (4 x 2048^2: 96.4 -> 92.9 us)."""
    out = dict(ent_lidx=lidx, lidx8=int(lidx8), ent_wa=wa)
    if not lidx8 or len(entcnt) == 0:
        return out
    padded = -(-entcnt // 16) * 16
    start = np.r_[0, np.cumsum(padded)]
    n = int(start[-1])
    src0 = np.r_[0, np.cumsum(entcnt)][:-1]
    pos = np.repeat(start[:-1] - src0, entcnt) + np.arange(int(entcnt.sum()))
    li = np.zeros(n, dtype=lidx.dtype)
    w = np.zeros(n, dtype=np.float32)
    li[pos] = lidx
    w[pos] = wa
    out.update(ent_lidx=li, ent_wa=w, box_ent_adj=start.astype(np.int32))
    return out


def box_plan_apply(P, x, mode):
    """numpy restatement of the nft_los kernels' arithmetic on a box plan
    (host-side check of the layout; tests only)."""
    nlos = P["nlos"]
    H, W, bh, bw, nby, nbx = P["H"], P["W"], P["bh"], P["bw"], P["nby"], P["nbx"]
    t = np.arange(BOX)
    ly, lx = t // bw, t % bw

    def pix(b):
        lyr, r = divmod(b, nby * nbx)
        by, bx = divmod(r, nbx)
        yy, xx = by * bh + ly, bx * bw + lx
        ok = (yy < H) & (xx < W)
        return (lyr * H + yy) * W + xx, ok
    if mode == "times":
        x = x.reshape(-1)
        part = np.zeros(P["nseg"])
        for i in range(P["nitems"]):
            p, ok = pix(int(P["item_box"][i]))
            u = np.where(ok, x[np.where(ok, p, 0)], 0.)
            for s in range(P["item_seg"][i], P["item_seg"][i + 1]):
                acc = 0.
                for k in range(P["seg_ent"][s], P["seg_ent"][s + 1]):
                    acc += float(P["ent_wf"][k]) * u[P["ent_loc"][k]]
                part[P["seg_slot"][s]] = acc
        lp = P["los_ptr"]
        return np.array([part[lp[i]:lp[i + 1]].sum() for i in range(nlos)])
    out = np.zeros(P["L"] * H * W)
    for b in range(P["nbox"]):
        p, ok = pix(b)
        e0 = P["box_ent_adj"][b] if "box_ent_adj" in P else P["box_ent"][b]
        for tt in range(BOX):
            if not ok[tt]:
                continue
            acc = 0.
            lines = P["box_lines"][P["box_lptr"][b]:P["box_lptr"][b + 1]]
            for k in range(e0 + P["pix_off"][b, tt], e0 + P["pix_off"][b, tt + 1]):
                acc += float(P["ent_wa"][k]) * x[lines[P["ent_lidx"][k]]]
            out[p[tt]] = acc
    return out


class LOSResponse(LinearOperator):
    def __init__(self, domain, starts, ends, sigmas=None, truncation=3.):
        self._domain = DomainTuple.make(domain)
        self._capability = self.TIMES | self.ADJOINT_TIMES
        if (not isinstance(self.domain[0], RGSpace)) or (len(self._domain) != 1):
            raise TypeError("The domain must be exactly one RGSpace instance.")
        sp = self.domain[0]
        rows, cols, w, nlos = los_coo(sp.shape, sp.distances, starts, ends, sigmas, truncation)
        self._coo = (rows, cols, w)
        self._target = DomainTuple.make(UnstructuredDomain(nlos))
        self._plan_np = box_plan(rows, cols, w, sp.shape, nlos)
        self._plan = None

    def _box_plan(self):
        """Device copy of the box-blocked layout + its ctypes descriptor."""
        if self._plan is None:
            P = self._plan_np
            dev = config.device()
            keep = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev)
                    for k, v in P.items() if isinstance(v, np.ndarray)}
            d = _native.LosPlan()
            for k in ("H", "W", "bh", "bw", "nby", "nbx", "nbox", "nlos", "nitems", "nseg", "lidx8"):
                setattr(d, k, int(P.get(k, 0)))
            for k, v in keep.items():
                setattr(d, k, v.data_ptr() if v.numel() else None)
            self._plan = (d, keep)
        return self._plan[0]

    def apply(self, x, mode):
        self._check_input(x, mode)
        v = x.val.reshape(-1).contiguous()
        plan = self._box_plan()
        if mode == self.TIMES:
            y = torch.empty(self._target.shape, dtype=v.dtype, device=v.device)
            _native.los_forward(plan, v, y)
            return Field(self._target, y)
        y = torch.empty(self._domain.shape, dtype=v.dtype, device=v.device)
        _native.los_adjoint(plan, v, y.view(-1))
        return Field(self._domain, y)

    def fused_middle(self, dr, c, fct=1.0):
        """Callable s -> fct * dr * R^T (c * R (dr * s)) on grid tensors: the
        middle of a sampling metric J^T D R^T C R D J with pixel-space diagonal
        dr (tensor or None) and data-space weight c (tensor or float) fused
        into the two SpMV kernels (column / row scales)."""
        nlos = self._target.shape[0]
        shape = self._domain.shape
        drf = None if dr is None else dr.reshape(-1).contiguous()
        scale = float(fct)
        cv = None
        if torch.is_tensor(c):
            cv = c.reshape(-1).expand(nlos).contiguous()
        else:
            scale *= float(c)

        plan = self._box_plan()

        npix = int(np.prod(shape))
        cast = {}

        def scales(dt):
            # fp32 CG storage (config.set_cg_precision): scales in the input's dtype
            if dt == torch.float64:
                return drf, cv
            if dt not in cast:
                cast[dt] = (None if drf is None else drf.to(dt), None if cv is None else cv.to(dt))
            return cast[dt]

        def middle(s, qpart=None, fold=None):
            """qpart (optional, (k, >= quad_blocks) fp64): per-block partials of
            the quadratic form s . middle(s), from the data space.  fold
            (optional, with qpart): an nft_fold_partials call (part, nb, nrhs,
            out address, out stride) that needs those partials, carried by
            the last adjoint launch (nft_los_adjoint_fold)"""
            drf, cv = scales(s.dtype)
            if qpart is not None:
                k = s.shape[0] if s.dim() > len(shape) else 1
                v = s.reshape(k, npix).contiguous()
                y = torch.empty((k, nlos), dtype=v.dtype, device=v.device)
                out = torch.empty((k,) + tuple(shape), dtype=v.dtype, device=v.device)
                for a in range(0, k, LOS_KMAX):
                    b = min(k, a + LOS_KMAX)
                    _native.los_forward_quad_batched(plan, v[a:b], y[a:b], qpart[a:b], colscale=drf, rowscale=cv,
                                                     scale=scale)
                    _native.los_adjoint_batched(plan, y[a:b], out[a:b].view(b - a, npix), rowscale=drf,
                                                fold=fold if b == k else None)
                return out if s.dim() > len(shape) else out[0]
            if s.dim() > len(shape):
                # batch of right-hand sides along a leading axis (batched CG):
                # the matrix is streamed once per launch for all of them
                k = s.shape[0]
                v = s.reshape(k, npix).contiguous()
                y = torch.empty((k, nlos), dtype=v.dtype, device=v.device)
                out = torch.empty((k,) + tuple(shape), dtype=v.dtype, device=v.device)
                for a in range(0, k, LOS_KMAX):
                    b = min(k, a + LOS_KMAX)
                    _native.los_forward_batched(plan, v[a:b], y[a:b], colscale=drf, rowscale=cv, scale=scale)
                    _native.los_adjoint_batched(plan, y[a:b], out[a:b].view(b - a, npix), rowscale=drf)
                return out
            v = s.reshape(-1).contiguous()
            y = torch.empty(nlos, dtype=v.dtype, device=v.device)
            _native.los_forward(plan, v, y, colscale=drf, rowscale=cv, scale=scale)
            out = torch.empty(shape, dtype=v.dtype, device=v.device)
            _native.los_adjoint(plan, y, out.view(-1), rowscale=drf)
            return out
        middle.supports_batch = True
        middle.supports_fp32 = True
        middle.supports_fold = _FOLD_IN_ADJ
        middle.quad_blocks = int(_native.load().nft_los_quad_blocks(ctypes.byref(plan)))
        return middle

    @property
    def coo(self):
        return self._coo
