"""Domains: regular grids, power spaces, unstructured spaces.

Host-side geometry (setup only; the hot path consumes the cached device
arrays these classes expose).  Behaviour follows
  src/domains/domain.py            (hash/equality by `_needed_for_hash`)
  src/domains/structured_domain.py (dvol / total_volume)
  src/domains/rg_space.py:52-214   (distances, codomain, |k| arrays)
  src/domains/power_space.py:155-198 (pindex / k_lengths / dvol binning)
  src/domains/unstructured_domain.py, src/domains/dof_space.py
"""
from functools import reduce

import numpy as np


class Domain:
    """Abstract domain; equality/hash use the attributes named in
    ``_needed_for_hash`` (src/domains/domain.py:22-80)."""
    _needed_for_hash = []

    def __hash__(self):
        try:
            return self._hash
        except AttributeError:
            v = vars(self)
            self._hash = reduce(lambda x, y: x ^ y, (hash(v[k]) for k in self._needed_for_hash), 0)
            return self._hash

    def __eq__(self, x):
        if self is x:
            return True
        if not isinstance(x, type(self)):
            return False
        return all(vars(self)[k] == vars(x)[k] for k in self._needed_for_hash)

    def __ne__(self, x):
        return not self.__eq__(x)

    @property
    def shape(self):
        raise NotImplementedError

    @property
    def size(self):
        return int(np.prod(self.shape, dtype=np.int64))


class StructuredDomain(Domain):
    @property
    def scalar_dvol(self):
        raise NotImplementedError

    @property
    def dvol(self):
        return self.scalar_dvol

    @property
    def total_volume(self):
        tmp = self.dvol
        return self.size * tmp if np.isscalar(tmp) else float(np.sum(tmp))

    @property
    def harmonic(self):
        raise NotImplementedError


class UnstructuredDomain(Domain):
    _needed_for_hash = ["_shape"]

    def __init__(self, shape):
        try:
            self._shape = tuple([int(i) for i in shape])
        except TypeError:
            self._shape = (int(shape),)

    def __repr__(self):
        return f"UnstructuredDomain(shape={self.shape})"

    @property
    def shape(self):
        return self._shape


class DOFSpace(StructuredDomain):
    """Degrees of freedom with explicit per-entry volume (src/domains/dof_space.py)."""
    _needed_for_hash = ["_dvol_key"]

    def __init__(self, dof_weights):
        self._dvol = np.asarray(dof_weights, dtype=np.float64).copy()
        self._dvol.flags.writeable = False
        self._dvol_key = hash(self._dvol.tobytes())

    @property
    def harmonic(self):
        return False

    @property
    def shape(self):
        return (self._dvol.shape[0],)

    @property
    def scalar_dvol(self):
        return None

    @property
    def dvol(self):
        return self._dvol

    def __repr__(self):
        return f"DOFSpace(size={self.size})"


class RGSpace(StructuredDomain):
    """Regular Cartesian grid, periodic (src/domains/rg_space.py:24-83)."""
    _needed_for_hash = ["_rdistances", "_shape", "_harmonic"]

    def __init__(self, shape, distances=None, harmonic=False, _realdistances=None):
        self._harmonic = bool(harmonic)
        if np.isscalar(shape):
            shape = (shape,)
        self._shape = tuple(int(i) for i in shape)
        if min(self._shape) < 0:
            raise ValueError("Negative number of pixels encountered")
        if _realdistances is not None:
            self._rdistances = _realdistances
        else:
            if distances is None:
                self._rdistances = tuple(1. / np.array(self._shape))
            elif np.isscalar(distances):
                if self._harmonic:
                    self._rdistances = tuple(1. / (np.array(self._shape) * float(distances)))
                else:
                    self._rdistances = (float(distances),) * len(self._shape)
            else:
                temp = np.empty(len(self._shape), dtype=np.float64)
                temp[:] = distances
                if self._harmonic:
                    temp = 1. / (np.array(self._shape) * temp)
                self._rdistances = tuple(temp)
        self._rdistances = tuple(float(d) for d in self._rdistances)
        self._hdistances = tuple(1. / (np.array(self._shape) * np.array(self._rdistances)))
        if min(self._rdistances) <= 0:
            raise ValueError("Non-positive distances encountered")
        self._dvol = float(reduce(lambda x, y: x * y, self.distances))

    def __repr__(self):
        return f"RGSpace(shape={self.shape}, distances={self.distances}, harmonic={self.harmonic})"

    @property
    def harmonic(self):
        return self._harmonic

    @property
    def shape(self):
        return self._shape

    @property
    def scalar_dvol(self):
        return self._dvol

    @property
    def distances(self):
        return self._hdistances if self._harmonic else self._rdistances

    def _dist_array(self):
        """|k| per pixel, periodic minimum distance (rg_space.py:105-116)."""
        res = np.arange(self.shape[0], dtype=np.float64)
        res = np.minimum(res, self.shape[0] - res) * self.distances[0]
        if len(self.shape) == 1:
            return res
        res *= res
        for i in range(1, len(self.shape)):
            tmp = np.arange(self.shape[i], dtype=np.float64)
            tmp = np.minimum(tmp, self.shape[i] - tmp) * self.distances[i]
            tmp *= tmp
            res = np.add.outer(res, tmp)
        return np.sqrt(res)

    def get_k_length_array(self):
        if not self.harmonic:
            raise NotImplementedError
        from ..field import Field
        return Field.from_raw(self, self._dist_array())

    def get_unique_k_lengths(self):
        """(rg_space.py:123-150) integer-norm shortcut for equal distances."""
        if not self.harmonic:
            raise NotImplementedError
        d = len(self.shape)
        if d == 1:
            return np.arange(self.shape[0] // 2 + 1, dtype=np.float64) * self.distances[0]
        if np.all(np.array(self.distances) == self.distances[0]):
            maxdist = np.asarray(self.shape) // 2
            tmp = np.zeros(int(np.sum(maxdist * maxdist)) + 1, dtype=bool)
            t2 = np.arange(maxdist[0] + 1, dtype=np.int64) ** 2
            for i in range(1, d):
                t3 = np.arange(maxdist[i] + 1, dtype=np.int64) ** 2
                t2 = np.add.outer(t2, t3)
            tmp[t2] = True
            return np.sqrt(np.nonzero(tmp)[0]) * self.distances[0]
        tmp = np.unique(self._dist_array())
        tol = 1e-12 * tmp[-1]
        return tmp[np.diff(np.r_[tmp, 2 * tmp[-1]]) > tol]

    def get_default_codomain(self):
        return RGSpace(self.shape, None, not self.harmonic, self._rdistances)

    def check_codomain(self, codomain):
        if not isinstance(codomain, RGSpace):
            raise TypeError("domain is not a RGSpace")
        if self.shape != codomain.shape:
            raise AttributeError("The shapes of domain and codomain must be identical.")
        if self.harmonic == codomain.harmonic:
            raise AttributeError("domain.harmonic and codomain.harmonic must not be the same.")
        if not np.all(abs(np.array(self.shape) * np.array(self.distances) *
                          np.array(codomain.distances) - 1) < 1e-7):
            raise AttributeError("The grid-distances of domain and codomain do not match.")

    @staticmethod
    def _kernel(x, sigma):
        return (x * x * (-2. * np.pi * np.pi * sigma * sigma)).ptw("exp")

    def get_fft_smoothing_kernel_function(self, sigma):
        if not self.harmonic:
            raise NotImplementedError
        return lambda x: self._kernel(x, sigma)


class PowerSpace(StructuredDomain):
    """Power-spectrum bins of a harmonic partner (power_space.py:24-198).

    ``pindex`` is computed exactly as the reference does (searchsorted of |k|
    against bin-bound midpoints) so the bin assignment is bit-identical."""
    _powerIndexCache = {}
    _needed_for_hash = ["_harmonic_partner", "_binbounds"]

    @staticmethod
    def linear_binbounds(nbin, first_bound, last_bound):
        nbin = int(nbin)
        if nbin < 3:
            raise ValueError("nbin must be at least 3")
        return np.linspace(float(first_bound), float(last_bound), nbin - 1)

    @staticmethod
    def logarithmic_binbounds(nbin, first_bound, last_bound):
        nbin = int(nbin)
        if nbin < 3:
            raise ValueError("nbin must be at least 3")
        return np.logspace(np.log(float(first_bound)), np.log(float(last_bound)), nbin - 1, base=np.e)

    def __init__(self, harmonic_partner, binbounds=None):
        if not (isinstance(harmonic_partner, StructuredDomain) and harmonic_partner.harmonic):
            raise ValueError("harmonic_partner must be a harmonic space.")
        if harmonic_partner.scalar_dvol is None:
            raise ValueError("harmonic partner must have scalar volume factors")
        self._harmonic_partner = harmonic_partner
        pdvol = harmonic_partner.scalar_dvol
        if binbounds is not None:
            binbounds = tuple(binbounds)
            if min(binbounds) < 0:
                raise ValueError("Negative binbounds encountered")
        key = (harmonic_partner, binbounds)
        if self._powerIndexCache.get(key) is None:
            klen = harmonic_partner._dist_array()
            if binbounds is None:
                tmp = harmonic_partner.get_unique_k_lengths()
                tbb = 0.5 * (tmp[:-1] + tmp[1:])
            else:
                tbb = binbounds
            pindex = np.searchsorted(tbb, klen)
            nbin = len(tbb) + 1
            rho = np.bincount(pindex.ravel(), minlength=nbin)
            if (rho == 0).any():
                raise ValueError("empty bins detected")
            kl = np.bincount(pindex.ravel(), weights=klen.ravel(),
                             minlength=nbin).astype(np.float64, copy=False) / rho
            for a in (kl, pindex):
                a.flags.writeable = False
            dvol = rho * pdvol
            dvol.flags.writeable = False
            self._powerIndexCache[key] = (binbounds, pindex, kl, dvol)
        self._binbounds, self._pindex, self._k_lengths, self._dvol = self._powerIndexCache[key]

    def __repr__(self):
        return f"PowerSpace(harmonic_partner={self.harmonic_partner}, binbounds={self._binbounds})"

    @property
    def harmonic(self):
        return False

    @property
    def shape(self):
        return self._k_lengths.shape

    @property
    def scalar_dvol(self):
        return None

    @property
    def dvol(self):
        return self._dvol

    @property
    def harmonic_partner(self):
        return self._harmonic_partner

    @property
    def binbounds(self):
        return self._binbounds

    @property
    def pindex(self):
        return self._pindex

    @property
    def k_lengths(self):
        return self._k_lengths


__all__ = ["Domain", "StructuredDomain", "UnstructuredDomain", "DOFSpace", "RGSpace", "PowerSpace"]
