"""Oracle: regular-grid harmonic geometry and power-spectrum binning.
Restates src/domains/rg_space.py:52-150 and src/domains/power_space.py:155-198.
TEST INFRASTRUCTURE ONLY."""
import numpy as np


def harmonic_distances(shape, pos_distances=None):
    """harmonic partner distances 1/(n d) of a position grid (rg_space.py:75-76, 183-192)"""
    shape = np.asarray(shape)
    if pos_distances is None:
        pos_distances = 1. / shape
    return 1. / (shape * np.asarray(pos_distances, dtype=np.float64))


def k_length_array(shape, hdist):
    """periodic |k| per pixel (rg_space.py:105-116)"""
    res = np.arange(shape[0], dtype=np.float64)
    res = np.minimum(res, shape[0] - res) * hdist[0]
    if len(shape) == 1:
        return res
    res *= res
    for i in range(1, len(shape)):
        tmp = np.arange(shape[i], dtype=np.float64)
        tmp = np.minimum(tmp, shape[i] - tmp) * hdist[i]
        tmp *= tmp
        res = np.add.outer(res, tmp)
    return np.sqrt(res)


def unique_k_lengths(shape, hdist):
    """(rg_space.py:123-150)"""
    d = len(shape)
    if d == 1:
        return np.arange(shape[0] // 2 + 1, dtype=np.float64) * hdist[0]
    if np.all(np.asarray(hdist) == hdist[0]):
        maxdist = np.asarray(shape) // 2
        tmp = np.zeros(int(np.sum(maxdist * maxdist)) + 1, dtype=bool)
        t2 = np.arange(maxdist[0] + 1, dtype=np.int64) ** 2
        for i in range(1, d):
            t2 = np.add.outer(t2, np.arange(maxdist[i] + 1, dtype=np.int64) ** 2)
        tmp[t2] = True
        return np.sqrt(np.nonzero(tmp)[0]) * hdist[0]
    tmp = np.unique(k_length_array(shape, hdist))
    tol = 1e-12 * tmp[-1]
    return tmp[np.diff(np.r_[tmp, 2 * tmp[-1]]) > tol]


def power_space(shape, hdist):
    """(pindex, k_lengths, dvol) of the natural binning (power_space.py:169-192)"""
    klen = k_length_array(shape, hdist)
    u = unique_k_lengths(shape, hdist)
    bb = 0.5 * (u[:-1] + u[1:])
    pindex = np.searchsorted(bb, klen)
    nbin = len(bb) + 1
    rho = np.bincount(pindex.ravel(), minlength=nbin)
    kl = np.bincount(pindex.ravel(), weights=klen.ravel(), minlength=nbin).astype(np.float64) / rho
    dvol = rho * float(np.prod(hdist))
    return pindex, kl, dvol


def power_distribute(v, pindex):
    """PowerDistributor TIMES (distributors.py:114-119)"""
    return v[pindex]


def power_collect(g, pindex, nbin):
    """PowerDistributor ADJOINT via bincount (distributors.py:105-112, utilities.py:223-242)"""
    return np.bincount(pindex.ravel(), weights=g.ravel(), minlength=nbin)
