"""Packed HBM layout for latent MultiFields.

The CG vectors of a sampling solve (x, r, d, q, b) are MultiFields over the
latent domain (sorted keys: scalars, 'spectrum', 'xi', ...).  For the fused
solver each vector is one contiguous device buffer; every key occupies an
aligned segment (multiple of ALIGN elements, zero padding) so that whole-vector
kernels (AXPY, dots) are single launches over 16-byte-aligned memory and the
grid segment ('xi') can be handed to the FFT kernels as a plain pointer."""
import torch

from .domain_tuple import DomainTuple
from .field import Field
from .multi_domain import MultiDomain
from .multi_field import MultiField

ALIGN = 64


class PackedLayout:
    def __init__(self, domain, dtype=torch.float64, device=None):
        from . import config
        self.domain = domain
        self.dtype = dtype
        self.device = config.device() if device is None else device
        self.multi = isinstance(domain, MultiDomain)
        items = list(domain.items()) if self.multi else [(None, domain)]
        self.keys, self.shapes, self.offsets, self.sizes = [], [], [], []
        off = 0
        for k, d in items:
            n = d.size
            self.keys.append(k)
            self.shapes.append(d.shape)
            self.offsets.append(off)
            self.sizes.append(n)
            off += (n + ALIGN - 1) // ALIGN * ALIGN
        self.size = max(off, ALIGN)

    def empty(self):
        return torch.zeros(self.size, dtype=self.dtype, device=self.device)

    def views(self, flat):
        return {k: flat[o:o + n].view(s) for k, s, o, n in zip(self.keys, self.shapes, self.offsets, self.sizes)}

    def view(self, flat, key):
        i = self.keys.index(key)
        return flat[self.offsets[i]:self.offsets[i] + self.sizes[i]].view(self.shapes[i])

    def pack(self, field, out=None):
        if out is None:
            out = self.empty()
        v = self.views(out)
        if self.multi:
            for k in self.keys:
                v[k].copy_(field[k].val)
        else:
            v[None].copy_(field.val)
        return out

    def unpack(self, flat, copy=True):
        v = self.views(flat)
        if self.multi:
            return MultiField(self.domain, tuple(Field(self.domain[k], v[k].clone() if copy else v[k])
                                                 for k in self.keys))
        return Field(self.domain, v[None].clone() if copy else v[None])
