"""DomainTuple / MultiDomain (src/domain_tuple.py, src/multi_domain.py).

Both are interned by ``make`` so that domain checks can use identity, as in
the reference (utilities.check_object_identity)."""
import numpy as np

from .domains import Domain


class DomainTuple:
    _tupleCache = {}
    _scalarDomain = None

    def __init__(self, domain, _callingfrommake=False):
        if not _callingfrommake:
            raise NotImplementedError("use DomainTuple.make")
        self._dom = self._parse_domain(domain)
        self._axtuple = self._get_axes_tuple()
        shape_tuple = tuple(sp.shape for sp in self._dom)
        self._shape = tuple(i for s in shape_tuple for i in s)
        self._size = int(np.prod(self._shape, dtype=np.int64)) if self._shape else 1

    def _get_axes_tuple(self):
        i = 0
        res = [None] * len(self._dom)
        for idx, thing in enumerate(self._dom):
            nax = len(thing.shape)
            res[idx] = tuple(range(i, i + nax))
            i += nax
        return tuple(res)

    def __reduce__(self):
        # unpickling goes through make(): identity-based domain checks keep
        # working for objects exchanged between ranks (domain_tuple.py:199-213)
        return (_unpickle_domain_tuple, (self._dom,))

    @staticmethod
    def make(domain):
        if isinstance(domain, DomainTuple):
            return domain
        from .multi_domain import MultiDomain
        if isinstance(domain, MultiDomain):
            raise TypeError("Got MultiDomain, expected DomainTuple")
        domain = DomainTuple._parse_domain(domain)
        obj = DomainTuple._tupleCache.get(domain)
        if obj is not None:
            return obj
        obj = DomainTuple(domain, _callingfrommake=True)
        DomainTuple._tupleCache[domain] = obj
        return obj

    @staticmethod
    def _parse_domain(domain):
        if domain is None:
            return ()
        if isinstance(domain, Domain):
            return (domain,)
        if not isinstance(domain, tuple):
            domain = tuple(domain)
        for d in domain:
            if not isinstance(d, Domain):
                raise TypeError("Given object contains something that is not an instance of Domain")
        return domain

    def __getitem__(self, i):
        return self._dom[i]

    @property
    def shape(self):
        return self._shape

    @property
    def size(self):
        return self._size

    def scalar_weight(self, spaces=None):
        from .utilities import parse_spaces
        if np.isscalar(spaces):
            return self._dom[spaces].scalar_dvol
        if spaces is None:
            spaces = range(len(self._dom))
        res = 1.
        for i in spaces:
            tmp = self._dom[i].scalar_dvol
            if tmp is None:
                return None
            res *= tmp
        return res

    def total_volume(self, spaces=None):
        if np.isscalar(spaces):
            return self._dom[spaces].total_volume
        if spaces is None:
            spaces = range(len(self._dom))
        res = 1.
        for i in spaces:
            res *= self._dom[i].total_volume
        return res

    @property
    def axes(self):
        return self._axtuple

    def __len__(self):
        return len(self._dom)

    def __hash__(self):
        return self._dom.__hash__()

    def __eq__(self, x):
        return (self is x) or (isinstance(x, DomainTuple) and self._dom == x._dom)

    def __ne__(self, x):
        return not self.__eq__(x)

    def __iter__(self):
        return iter(self._dom)

    def __repr__(self):
        return "DomainTuple:\n" + "\n".join(f"  {d}" for d in self._dom)

    @staticmethod
    def scalar_domain():
        if DomainTuple._scalarDomain is None:
            DomainTuple._scalarDomain = DomainTuple.make(())
        return DomainTuple._scalarDomain


def _unpickle_domain_tuple(dom):
    return DomainTuple.make(dom)
