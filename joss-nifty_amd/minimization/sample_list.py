"""ResidualSampleList: latent mean + (possibly distributed) residual samples
(src/minimization/sample_list.py:42-531, averaging :285-341).

Averages over samples: per rank the reference's pairwise order, across ranks
ONE all-reduce of a packed buffer (utilities.allreduce_sum), or the
reference's global pairwise tree over point-to-point messages in
deterministic mode (bit-identical for any number of ranks)."""
import glob
import os

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

    @property
    def local_indices(self):
        return range(self._lo, self._lo + self._nlocal)

    # ------------------------------------------------------------ disk
    # sample_list.py:510-531: one file per sample (global index) written by
    # its rank, the mean by the MPI master; data-only files (checkpoint.py)
    def save(self, file_name_base, overwrite=False):
        from .checkpoint import save_field
        for i, isample in enumerate(self.local_indices):
            save_field(f"{file_name_base}.{isample}.npz", self._r[i], {"neg": bool(self._n[i])}, overwrite)
        if utilities.get_MPI_params_from_comm(self._comm)[2]:
            save_field(f"{file_name_base}.mean.npz", self._m, None, overwrite)
        _barrier(self._comm)

    @classmethod
    def load(cls, file_name_base, comm=None, domain=None):
        """``domain``: the latent MultiDomain the fields belong to (else the
        domains are rebuilt from the files' descriptors)"""
        from .checkpoint import load_field
        _barrier(comm)
        mean, _ = load_field(f"{file_name_base}.mean.npz", domain)
        res, neg = [], []
        for f in _local_sample_files(file_name_base, comm):
            r, ex = load_field(f, domain)
            res.append(r)
            neg.append(bool(ex["neg"]))
        return cls(mean, res, neg, comm=comm)

    @classmethod
    def load_mean(cls, file_name_base, domain=None):
        from .checkpoint import load_field
        return load_field(f"{file_name_base}.mean.npz", domain)[0]


class SampleList:
    """Plain list of (possibly distributed) samples (sample_list.py:533-653);
    optimize_kl's result for maximum-a-posteriori iterations."""

    def __init__(self, samples, comm=None, domain=None):
        self._s = list(samples)
        self._comm = comm
        if domain is None:
            if not self._s:
                raise ValueError("SampleList without samples needs a domain")
            domain = self._s[0].domain
        self._domain = domain
        ntask, rank, _ = utilities.get_MPI_params_from_comm(comm)
        counts = [len(self._s)] if comm is None else [int(c) for c in comm.allgather(len(self._s))]
        self._counts = None if comm is None else counts
        self._lo = int(sum(counts[:rank]))

    @property
    def comm(self):
        return self._comm

    @property
    def domain(self):
        return self._domain

    @property
    def n_samples(self):
        return len(self._s) if self._counts is None else int(sum(self._counts))

    @property
    def n_local_samples(self):
        return len(self._s)

    @property
    def local_indices(self):
        return range(self._lo, self._lo + len(self._s))

    def local_item(self, i):
        return self._s[i]

    def local_iterator(self):
        return iter(self._s)

    def _template(self, op):
        """a zero object of op's result layout, for a rank without samples"""
        def template():
            from ..sugar import full
            z = full(self._domain, 0.)
            return 0 * (op(z) if op is not None else z)
        return template

    def average(self, op=None):
        res = [op(s) if op is not None else s for s in self._s]
        return utilities.allreduce_sum(res, self._comm, counts=self._counts,
                                       template=self._template(op)) / self.n_samples

    def sample_stat(self, op=None):
        mean = self.average(op)
        sq = self.average(lambda s: (op(s) if op is not None else s) ** 2)
        return mean, sq - mean ** 2

    def save(self, file_name_base, overwrite=False):
        from .checkpoint import save_field
        for s, isample in zip(self._s, self.local_indices):
            save_field(f"{file_name_base}.{isample}.npz", s, None, overwrite)
        _barrier(self._comm)

    @classmethod
    def load(cls, file_name_base, comm=None, domain=None):
        """``domain``: the samples' domain; a rank whose share of the files is
        empty (e.g. the one sample of a MAP iteration on two ranks) takes it
        from sample 0's file, so that every rank joins the constructor's
        collective"""
        from .checkpoint import load_domain, load_field
        _barrier(comm)
        files = _local_sample_files(file_name_base, comm)
        samples = [load_field(f, domain)[0] for f in files]
        if domain is None and not samples:
            domain = load_domain(f"{file_name_base}.0.npz")
        return cls(samples, comm=comm, domain=domain)


def _barrier(comm):
    if comm is not None:
        comm.Barrier()


def _local_sample_files(file_name_base, comm):
    """this rank's share (shareRange) of the sample files, in index order
    (sample_list.py:626-653)"""
    files = glob.glob(f"{file_name_base}.*.npz")
    idx = sorted(int(f[len(file_name_base) + 1:-4]) for f in files
                 if f[len(file_name_base) + 1:-4].isdigit())
    if idx != list(range(len(idx))):
        raise RuntimeError(f"sample files of {file_name_base} are not numbered 0..n-1")
    ntask, rank, _ = utilities.get_MPI_params_from_comm(comm)
    lo, hi = utilities.shareRange(len(idx), ntask, rank)
    return [f"{file_name_base}.{i}.npz" for i in range(lo, hi)]
