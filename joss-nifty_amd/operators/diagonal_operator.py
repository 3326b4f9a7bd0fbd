"""DiagonalOperator (src/operators/diagonal_operator.py:26-189); the diagonal
is a device tensor, broadcast over `spaces`."""
import numpy as np
import torch

from .. import utilities
from ..domain_tuple import DomainTuple
from ..field import Field
from .endomorphic_operator import EndomorphicOperator


class DiagonalOperator(EndomorphicOperator):
    def __init__(self, diagonal, domain=None, spaces=None, sampling_dtype=None):
        if not isinstance(diagonal, Field):
            raise TypeError("Field object required")
        self._dtype = sampling_dtype
        self._domain = diagonal.domain if domain is None else DomainTuple.make(domain)
        if spaces is None:
            self._spaces = None
            utilities.check_object_identity(diagonal.domain, self._domain)
        else:
            self._spaces = utilities.parse_spaces(spaces, len(self._domain))
            if len(self._spaces) != len(diagonal.domain):
                raise ValueError("spaces and domain must have the same length")
            for i, j in enumerate(self._spaces):
                if diagonal.domain[i] != self._domain[j]:
                    raise ValueError(f"Mismatch:\n{diagonal.domain[i]}\n{self._domain[j]}")
            if self._spaces == tuple(range(len(self._domain))):
                self._spaces = None
        if self._spaces is not None:
            active_axes = []
            for space_index in self._spaces:
                active_axes += self._domain.axes[space_index]
            self._reshaper = [shp if i in active_axes else 1 for i, shp in enumerate(self._domain.shape)]
            self._ldiag = diagonal.val.reshape(self._reshaper)
        else:
            self._ldiag = diagonal.val
        self._fill_rest()

    def _fill_rest(self):
        self._complex = self._ldiag.is_complex()
        self._capability = self._all_ops

    def _from_ldiag(self, spc, ldiag, sampling_dtype):
        res = DiagonalOperator.__new__(DiagonalOperator)
        res._dtype = sampling_dtype
        res._domain = self._domain
        if self._spaces is None or spc is None:
            res._spaces = None
        else:
            res._spaces = tuple(set(self._spaces) | set(spc))
        res._ldiag = ldiag
        res._fill_rest()
        return res

    def _scale(self, fct):
        if not np.isscalar(fct):
            raise TypeError("scalar value required")
        return self._from_ldiag((), self._ldiag * fct, self._dtype)

    def _add(self, sum_):
        if not np.isscalar(sum_):
            raise TypeError("scalar value required")
        return self._from_ldiag((), self._ldiag + sum_, self._dtype)

    def _combine_prod(self, op):
        dtype = self._dtype if self._dtype == op._dtype else None
        return self._from_ldiag(op._spaces, self._ldiag * op._ldiag, dtype)

    def _combine_sum(self, op, selfneg, opneg):
        tdiag = self._ldiag * (-1 if selfneg else 1) + op._ldiag * (-1 if opneg else 1)
        dtype = self._dtype if self._dtype == op._dtype else None
        return self._from_ldiag(op._spaces, tdiag, dtype)

    @property
    def diagonal_tensor(self):
        """full-shape diagonal (broadcast) as a device tensor"""
        return self._ldiag.expand(self._domain.shape)

    def apply(self, x, mode):
        self._check_input(x, mode)
        if mode == 1 or (not self._complex and mode == 2):
            return Field(x.domain, x.val * self._ldiag)
        xdiag = self._ldiag
        if self._complex and (mode & 10):
            xdiag = xdiag.conj()
        if mode & 3:
            return Field(x.domain, x.val * xdiag)
        return Field(x.domain, x.val / xdiag)

    def _flip_modes(self, trafo):
        if trafo == self.ADJOINT_BIT and not self._complex:
            return self
        xdiag = self._ldiag
        if self._complex and (trafo & self.ADJOINT_BIT):
            xdiag = xdiag.conj()
        if trafo & self.INVERSE_BIT:
            xdiag = 1. / xdiag
        return self._from_ldiag((), xdiag, self._dtype)

    def process_sample(self, samp, from_inverse):
        if self._complex:
            raise ValueError("operator not positive definite")
        dmin = float(self._ldiag.min().item())
        if dmin < 0. or (dmin == 0. and from_inverse):
            raise ValueError("operator not positive definite")
        if from_inverse:
            res = samp.val / torch.sqrt(self._ldiag)
        else:
            res = samp.val * torch.sqrt(self._ldiag)
        return Field(self._domain, res.expand(self._domain.shape).contiguous())

    def draw_sample(self, from_inverse=False):
        if self._dtype is None:
            raise RuntimeError("Need to specify dtype to be able to sample from this operator:\n" + repr(self))
        res = Field.from_random(domain=self._domain, random_type="normal", dtype=self._dtype)
        return self.process_sample(res, from_inverse)

    def get_sqrt(self):
        if self._complex or bool((self._ldiag < 0).any().item()):
            raise ValueError("get_sqrt() works only for positive definite operators.")
        return self._from_ldiag((), torch.sqrt(self._ldiag), self._dtype)

    def __repr__(self):
        return "DiagonalOperator"
