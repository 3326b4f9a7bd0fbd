"""Line-of-sight response (src/library/los_response.py:34-233).

Construction (host, setup only): every line of sight is traversed through the
pixel grid (Amanatides-Woo style cell crossing distances), giving per-pixel
path lengths (optionally tapered by the parallax error function); entries are
ordered by 16x16 pixel boxes exactly as the reference orders its COO matrix.
The matrix is then stored on the device twice: CSR over lines of sight (for
R x) and CSR over pixels (= CSC, for R^T y), float32 weights as in the
reference, applied by csrc/nft_spmv.hip with fp64 accumulation."""
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


def _csr(rows, cols, w, nrows):
    """stable CSR (entries of a row keep their COO storage order)"""
    order = np.argsort(rows, kind="stable")
    cnt = np.bincount(rows, minlength=nrows)
    ptr = np.zeros(nrows + 1, dtype=np.int64)
    np.cumsum(cnt, out=ptr[1:])
    return ptr, cols[order].astype(np.int32), w[order].astype(np.float32)


class LOSResponse(LinearOperator):
    def __init__(self, domain, starts, ends, sigmas=None, truncation=3.):
        self._domain = DomainTuple.make(domain)
        self._capability = self.TIMES | self.ADJOINT_TIMES
        if (not isinstance(self.domain[0], RGSpace)) or (len(self._domain) != 1):
            raise TypeError("The domain must be exactly one RGSpace instance.")
        sp = self.domain[0]
        rows, cols, w, nlos = los_coo(sp.shape, sp.distances, starts, ends, sigmas, truncation)
        self._coo = (rows, cols, w)
        npix = sp.size
        dev = config.device()
        p, c, ww = _csr(rows, cols, w, nlos)
        self._fwd = tuple(torch.from_numpy(a).to(dev) for a in (p, c, ww))
        p, c, ww = _csr(cols, rows, w, npix)
        self._adj = tuple(torch.from_numpy(a).to(dev) for a in (p, c, ww))
        self._target = DomainTuple.make(UnstructuredDomain(nlos))

    def apply(self, x, mode):
        self._check_input(x, mode)
        v = x.val.reshape(-1).contiguous()
        if mode == self.TIMES:
            y = torch.empty(self._target.shape, dtype=v.dtype, device=v.device)
            _native.spmv_csr(*self._fwd, v, y)
            return Field(self._target, y)
        y = torch.empty(self._domain.shape, dtype=v.dtype, device=v.device)
        _native.spmv_csr(*self._adj, v, y.view(-1))
        return Field(self._domain, y)

    @property
    def coo(self):
        return self._coo
