"""ResidualSampleList: latent mean + (possibly distributed) residual samples
(src/minimization/sample_list.py:42-531, averaging :285-341).

Averages over samples use the deterministic pairwise sum of
utilities.allreduce_sum (bit-identical for any number of ranks)."""
import numpy as np

from .. import utilities
from ..multi_field import MultiField


class ResidualSampleList:
    def __init__(self, mean, residuals, neg, comm=None):
        self._m = mean
        self._r = tuple(residuals)
        self._n = tuple(neg)
        self._comm = comm
        if len(self._r) != len(self._n):
            raise ValueError("length mismatch")
        ntask, rank, _ = utilities.get_MPI_params_from_comm(comm)
        self._nlocal = len(self._r)
        if comm is None:
            self._ntotal = self._nlocal
            self._lo = 0
        else:
            counts = comm.allgather(self._nlocal)
            self._ntotal = int(sum(counts))
            self._lo = int(sum(counts[:rank]))

    @property
    def comm(self):
        return self._comm

    @property
    def n_samples(self):
        return self._ntotal

    @property
    def n_local_samples(self):
        return self._nlocal

    @property
    def domain(self):
        return self._m.domain

    @property
    def mean(self):
        return self._m

    def local_item(self, i):
        # residuals may live on a sub-domain of the mean (point estimates):
        # the missing keys get a zero residual (sample_list.py:486-487)
        r = self._r[i]
        if isinstance(self._m, MultiField) and self._m.domain is not r.domain:
            return self._m.flexible_addsub(r, self._n[i])
        return self._m - r if self._n[i] else self._m + r

    def local_iterator(self):
        for i in range(self._nlocal):
            yield self.local_item(i)

    def iterator(self, op=None):
        if self._comm is not None and self._comm.Get_size() > 1:
            raise NotImplementedError("iterator over distributed samples: use local_iterator")
        for s in self.local_iterator():
            yield s if op is None else op(s)

    def _average_tuple(self, func):
        """Average a tuple-valued function over all samples (sample_list.py:312-341)."""
        return self._average_results([func(s) for s in self.local_iterator()])

    def _average_results(self, res):
        """The reduction of _average_tuple on precomputed per-sample tuples."""
        n = self._ntotal
        out = []
        for k in range(len(res[0]) if res else 0):
            vals = [r[k] for r in res]
            tot = utilities.allreduce_sum(vals, self._comm)
            out.append(tot / n)
        return tuple(out)

    def average(self, op=None):
        res = [op(s) if op is not None else s for s in self.local_iterator()]
        return utilities.allreduce_sum(res, self._comm) / self._ntotal

    def at(self, mean):
        """sample_list.py:489-507: only the keys present in ``mean`` are
        updated."""
        if isinstance(self._m, MultiField) and self.domain is not mean.domain:
            mean = MultiField.union([self._m, mean])
        return ResidualSampleList(mean, self._r, self._n, self._comm)

    def sample_stat(self, op=None):
        mean = self.average(op)
        sq = self.average(lambda s: (op(s) if op is not None else s) ** 2)
        return mean, sq - mean ** 2
