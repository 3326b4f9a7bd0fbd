"""ResidualSampleList: latent mean + (possibly distributed) residual samples
(src/minimization/sample_list.py:42-531, averaging :285-341).

Averages over samples: per rank the reference's pairwise order, across ranks
ONE all-reduce of a packed buffer (utilities.allreduce_sum), or the
reference's global pairwise tree over point-to-point messages in
deterministic mode (bit-identical for any number of ranks)."""
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
            self._counts = None
            self._ntotal = self._nlocal
            self._lo = 0
        else:
            counts = [int(c) for c in comm.allgather(self._nlocal)]
            self._counts = counts
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

    def _average_tuple(self, func, template=None):
        """Average a tuple-valued function over all samples (sample_list.py:312-341)."""
        return self._average_results([func(s) for s in self.local_iterator()], template)

    def _average_results(self, res, template=None):
        """The reduction of _average_tuple on precomputed per-sample tuples:
        per rank the pairwise sum of every tuple element, then ONE all-reduce
        of all elements packed into one buffer (utilities.allreduce_sum).  A
        rank without samples contributes zeros of ``template()``'s layout
        (the reference splits off an active communicator instead and
        broadcasts, sample_list.py:62-70,327-341)."""
        n = self._ntotal
        if self._comm is None and not res:
            return None
        tot = utilities.allreduce_sum([tuple(r) for r in res], self._comm, counts=self._counts,
                                      template=template)
        return tuple(t / n for t in tot)

    def average(self, op=None):
        res = [op(s) if op is not None else s for s in self.local_iterator()]

        def template():
            # a rank without samples: the layout of op's result
            return 0 * (op(self._m) if op is not None else self._m)
        return utilities.allreduce_sum(res, self._comm, counts=self._counts, template=template) / self._ntotal

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
