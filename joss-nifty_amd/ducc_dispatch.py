"""Numeric backend seam (mirror of src/ducc_dispatch.py:29-92).

Every function runs the hand-written HIP kernels of libnifty_amd.so on device
tensors; there is no CPU fallback (``_native.require_device`` raises)."""
import torch

from . import _native
from .config import hartley_convention_code

_nthreads = 1


def nthreads():
    return _nthreads


def set_nthreads(nthr):
    """Kept for API compatibility; GPU kernels ignore host thread counts."""
    global _nthreads
    _nthreads = int(nthr)


def _axes(a, axes):
    return tuple(range(a.ndim)) if axes is None else tuple(int(x) % a.ndim for x in axes)


def fftn(a, axes=None):
    if not a.is_complex():
        a = a.to(torch.complex128 if a.dtype == torch.float64 else torch.complex64)
    return _native.fft_c2c(a.contiguous(), _axes(a, axes), forward=True)


def ifftn(a, axes=None):
    if not a.is_complex():
        a = a.to(torch.complex128 if a.dtype == torch.float64 else torch.complex64)
    ax = _axes(a, axes)
    n = 1
    for x in ax:
        n *= a.shape[x]
    return _native.fft_c2c(a.contiguous(), ax, forward=False, scale=1. / n)


def hartley(a, axes=None, scale=1.0, out=None):
    return _native.hartley(a.contiguous(), _axes(a, axes), hartley_convention_code(), scale, out=out)


def vdot(a, b):
    """sum(conj(a) * b) as a 0-d fp64 device tensor (fp64 accumulation)."""
    if a.is_complex() or b.is_complex():
        a = a.to(torch.complex128)
        b = b.to(torch.complex128)
        ar, ai = torch.view_as_real(a.conj().resolve_conj().contiguous()).unbind(-1)
        br, bi = torch.view_as_real(b.contiguous()).unbind(-1)
        ar, ai, br, bi = (t.contiguous() for t in (ar, ai, br, bi))
        re = _native.dot(ar, br) - _native.dot(ai, bi)
        im = _native.dot(ar, bi) + _native.dot(ai, br)
        return torch.complex(re, im)
    if a.dtype != b.dtype:
        a = a.to(torch.float64)
        b = b.to(torch.float64)
    if not a.is_floating_point():
        a = a.to(torch.float64)
        b = b.to(torch.float64)
    return _native.dot(a.contiguous(), b.contiguous())
