"""Oracle: numeric seam (restates src/ducc_dispatch.py:38-58, scipy path).
TEST INFRASTRUCTURE ONLY.  ``workers=None``: scipy's default (1 thread) or the
count of an enclosing ``scipy.fft.set_workers`` block (bench.py's CPU
baseline runs on all host cores that way)."""
import numpy as np
import scipy.fft


def fftn(a, axes=None, workers=None):
    """ducc_dispatch._scipy_fftn (:38-39)"""
    return scipy.fft.fftn(a, axes=axes, workers=workers)


def ifftn(a, axes=None, workers=None):
    """ducc_dispatch._scipy_ifftn (:42-43): normalised by 1/N"""
    return scipy.fft.ifftn(a, axes=axes, workers=workers)


def hartley(a, axes=None, convention="non_canonical_hartley", workers=None):
    """ducc_dispatch._scipy_hartley (:46-50): Re F +/- Im F of the forward FFT"""
    tmp = scipy.fft.fftn(a, axes=axes, workers=workers)
    if convention == "non_canonical_hartley":
        return tmp.real + tmp.imag
    return tmp.real - tmp.imag


def vdot(a, b):
    """ducc_dispatch._scipy_vdot (:53-58)"""
    return np.vdot(a, b)
