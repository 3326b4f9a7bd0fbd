"""MultiDomain: ordered (sorted-key) dict of DomainTuples (src/multi_domain.py:24-144)."""
from .domain_tuple import DomainTuple


class MultiDomain:
    _domainCache = {}

    def __init__(self, dct, _callingfrommake=False):
        if not _callingfrommake:
            raise NotImplementedError("use MultiDomain.make")
        self._keys = tuple(sorted(dct.keys()))
        self._domains = tuple(dct[k] for k in self._keys)
        self._idx = {k: i for i, k in enumerate(self._keys)}

    def __reduce__(self):
        # see DomainTuple.__reduce__ (multi_domain.py:136-144)
        return (_unpickle_multi_domain, (dict(zip(self._keys, self._domains)),))

    @staticmethod
    def make(inp):
        if isinstance(inp, MultiDomain):
            return inp
        if not isinstance(inp, dict):
            raise TypeError("dict expected")
        tmp = {}
        for key, value in inp.items():
            if not isinstance(key, str):
                raise TypeError("keys must be strings")
            tmp[key] = DomainTuple.make(value)
        tmp = tuple(sorted(tmp.items()))
        obj = MultiDomain._domainCache.get(tmp)
        if obj is not None:
            return obj
        obj = MultiDomain(dict(tmp), _callingfrommake=True)
        MultiDomain._domainCache[tmp] = obj
        return obj

    def keys(self):
        return self._keys

    def values(self):
        return self._domains

    def domains(self):
        return self._domains

    @property
    def idx(self):
        return self._idx

    def items(self):
        return zip(self._keys, self._domains)

    def __getitem__(self, key):
        return self._domains[self._idx[key]]

    def __contains__(self, key):
        return key in self._idx

    def __len__(self):
        return len(self._keys)

    def __hash__(self):
        return self._keys.__hash__() ^ self._domains.__hash__()

    def __eq__(self, x):
        if self is x:
            return True
        return isinstance(x, MultiDomain) and list(self.items()) == list(x.items())

    def __ne__(self, x):
        return not self.__eq__(x)

    @property
    def size(self):
        return sum(d.size for d in self._domains)

    def __repr__(self):
        return "MultiDomain:\n" + "\n".join(f"  {k}: {d}" for k, d in self.items())

    @staticmethod
    def union(inp):
        res = {}
        for dd in inp:
            for key, subdom in zip(dd._keys, dd._domains):
                if key in res:
                    if res[key] is not subdom:
                        raise ValueError("domain mismatch")
                else:
                    res[key] = subdom
        return MultiDomain.make(res)


def _unpickle_multi_domain(dct):
    return MultiDomain.make(dct)
