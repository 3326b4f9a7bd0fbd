"""DOFDistributor / PowerDistributor (src/operators/distributors.py:28-157).

Forward (gather) and adjoint (deterministic segmented scatter, bit-identical
to np.bincount) run as native kernels (csrc/nft_cf.hip)."""
import os

import numpy as np
import torch

from .. import _native
from ..domain_tuple import DomainTuple
from ..domains import DOFSpace, PowerSpace
from ..field import Field
from ..utilities import infer_space
from .linear_operator import LinearOperator


def _chunk_bins(offs, nbin, npix, ch=None):
    """First bin owned by each chunk of ch (default nft_bin_chunk()) sorted
    positions (the first bin whose offset is >= c * chunk), last entry nbin
    (int32)."""
    if ch is None:
        ch = int(_native.load().nft_bin_chunk())
    nch = (npix + ch - 1) // ch
    cb = np.searchsorted(offs[:-1], np.arange(nch + 1, dtype=np.int64) * ch, side="left")
    cb[-1] = nbin
    return cb.astype(np.int32)


class _ILFold:
    """fold_into's result in cell order with the items interleaved (nf, pre)"""

    def __init__(self, t):
        self.t = t


class BinIndex:
    """Device-resident bin index: pindex (int32) plus the stable bin->pixel
    permutation and CSR offsets for the adjoint.  Built once on the host."""
    _cache = {}

    def __init__(self, dofdex, nbin, device, fold=False):
        grid = np.asarray(dofdex)
        dofdex = grid.ravel()
        self.npix = dofdex.size
        self.nbin = int(nbin)
        if self.npix >= 2 ** 31:
            raise ValueError("grids with >= 2^31 pixels are not supported")
        self._order = None
        self.fold = self._make_fold(grid, device) if fold and self.FOLD else None
        if self.fold is not None:
            # a folded index serves scatter() only: no full-grid permutation
            self.pindex = self.perm = self.offsets = None
            return
        perm = np.argsort(dofdex, kind="stable")
        cnt = np.bincount(dofdex, minlength=self.nbin)
        offs = np.zeros(self.nbin + 1, dtype=np.int64)
        np.cumsum(cnt, out=offs[1:])
        self.pindex = torch.from_numpy(dofdex.astype(np.int32)).to(device)
        self.perm = torch.from_numpy(perm.astype(np.int32)).to(device)
        self.offsets = torch.from_numpy(offs.astype(np.int32)).to(device)

    # Mirror-folded adjoint (nft_bin_fold + scatter over the fundamental cell,
    # 2^d fewer scattered gathers) for harmonic grids whose bins are invariant
    # under k_a -> -k_a on every axis.  Sums agree with np.bincount to rounding
    # (not bitwise), so only the fused CF Jacobian paths ask for it; the
    # PowerDistributor operator keeps the bit-exact scatter.
    FOLD = os.environ.get("NFT_BIN_FOLD", "1") != "0"

    def _make_fold(self, grid, device):
        shp = grid.shape
        if not (1 <= len(shp) <= 3) or self.npix < 4096:
            return None
        for ax in range(len(shp)):
            if not np.array_equal(grid, np.roll(np.flip(grid, ax), 1, ax)):
                return None
        f = np.ascontiguousarray(grid[tuple(slice(0, n // 2 + 1) for n in shp)]).ravel()
        perm = np.argsort(f, kind="stable")
        offs = np.zeros(self.nbin + 1, dtype=np.int64)
        np.cumsum(np.bincount(f, minlength=self.nbin), out=offs[1:])
        cb = _chunk_bins(offs, self.nbin, f.size)
        # the interleaved scatter's chunk -> first bin tables, made here on the
        # host (a first use inside a HIP-graph capture must not sync)
        lib = _native.load()
        il_cb = {pre: torch.from_numpy(_chunk_bins(offs, self.nbin, f.size,
                                                   int(lib.nft_bin_scatter_il_chunk(pre)))).to(device)
                 for pre in (2, 4, 8)}
        return dict(shape=tuple(int(n) for n in shp), nf=int(f.size), il_cb=il_cb,
                    pindex=torch.from_numpy(f.astype(np.int32)).to(device),   # cell -> bin
                    perm=torch.from_numpy(perm.astype(np.int32)).to(device),
                    offsets=torch.from_numpy(offs.astype(np.int32)).to(device),
                    order=(None, None, torch.from_numpy(cb).to(device)))

    def gather_folded(self, src, k, interleaved=True):
        """per-cell values of src on the fundamental cell: (nf, k) from the
        (B, k) bin-major src, or (k, nf) from a (k, B) src -- the forward
        Jacobian's bin gather done once per mirror class
        (nft_hartley_fuse.pro_folded reads it by the cell of each pixel)"""
        f = self.fold
        if interleaved:
            out = torch.empty((f["nf"], k), dtype=src.dtype, device=src.device)
            return _native.bin_gather(src, f["pindex"], out, 1, f["nf"], self.nbin, k)
        out = torch.empty((k, f["nf"]), dtype=src.dtype, device=src.device)
        return _native.bin_gather(src, f["pindex"], out, k, f["nf"], self.nbin, 1)

    def scatter(self, w, out, pre):
        """out[p, b] = sum over the pixels of bin b of w[p, :] (w: pre grids,
        contiguous).  Folded when available, else the bit-exact scatter."""
        f = self.fold
        if f is None:
            return _native.bin_scatter(w, self.perm, self.offsets, out, pre, self.npix, self.nbin, 1,
                                       order=self.gather_order)
        wf = torch.empty((pre, f["nf"]), dtype=w.dtype, device=w.device)
        _native.bin_fold(w, wf, pre, f["shape"])
        return _native.bin_scatter_folded(wf, f["perm"], f["offsets"], out, pre, f["nf"], self.nbin,
                                          chunk_bins=f["order"][2])

    # the half-grid fold with the items interleaved (bin_fold_half_sorted,
    # cpos None) + bin sums gathering all items of a cell at once
    # (nft_bin_scatter_il; NFT_BIN_IL=0: planar fold + per-item gathers) --
    # bitwise the same sums
    IL = os.environ.get("NFT_BIN_IL", "1") != "0"

    def fold_into(self, w, wf, pre, half=False):
        """first half of scatter: the mirror fold of w into wf (pre, nf);
        returns the operand of scatter_from (wf, or w without a fold).
        half: w holds point-mirror pair sums on the half grid
        (nft_hartley_fuse.epi_out2_pairs); then, for pre in (2, 4, 8), wf
        receives the fold with the items interleaved (nf, pre) and the operand
        is tagged so"""
        f = self.fold
        if f is None:
            if half:
                raise ValueError("pair sums need the folded bin index")
            return w
        if half and self.IL and pre in (2, 4, 8):
            _native.bin_fold_half_sorted(w, wf, None, pre, f["shape"])
            return _ILFold(wf)
        (_native.bin_fold_half if half else _native.bin_fold)(w, wf, pre, f["shape"])
        return wf

    def scatter_from(self, src, out, pre):
        """second half of scatter: the bin sums of fold_into's result"""
        f = self.fold
        if f is None:
            return _native.bin_scatter(src, self.perm, self.offsets, out, pre, self.npix, self.nbin, 1,
                                       order=self.gather_order)
        if isinstance(src, _ILFold):
            return _native.bin_scatter_il(src.t, f["perm"], f["offsets"], out, pre, f["nf"], self.nbin,
                                          chunk_bins=self._il_chunk_bins(pre))
        return _native.bin_scatter_folded(src, f["perm"], f["offsets"], out, pre, f["nf"], self.nbin,
                                          chunk_bins=f["order"][2])

    def _il_chunk_bins(self, pre):
        """the interleaved scatter's chunk -> first bin table of an item count
        (pre in 2, 4, 8; made with the plan, _make_fold)"""
        return self.fold["il_cb"][pre]

    @property
    def gather_order(self):
        """(None, None, chunk_bins int32) for nft_bin_scatter_ordered: the
        first bin owned by each chunk of nft_bin_chunk() sorted positions
        (pixel-ordered chunk gathers measured no faster at 2048^2: the chunk
        kernel is bound by its per-bin phase, not by gather divergence)."""
        if self._order is None:
            perm = self.perm
            offs = self.offsets.cpu().numpy().astype(np.int64)
            cbt = torch.from_numpy(_chunk_bins(offs, self.nbin, perm.numel())).to(perm.device)
            self._order = (None, None, cbt)
        return self._order

    @classmethod
    def get(cls, dofdex, nbin, device, fold=False):
        fold = bool(fold) and cls.FOLD
        key = (id(dofdex), int(nbin), str(device), fold)
        obj = cls._cache.get(key)
        if obj is None or obj._ref is not dofdex:
            obj = cls(dofdex, nbin, device, fold)
            obj._ref = dofdex
            cls._cache[key] = obj
        return obj


class DOFDistributor(LinearOperator):
    def __init__(self, dofdex, target=None, space=None):
        if target is None:
            target = dofdex.domain
        self._target = DomainTuple.make(target)
        space = infer_space(self._target, space)
        partner = self._target[space]
        if not isinstance(dofdex, Field):
            raise TypeError("dofdex must be a Field")
        ldat = dofdex.val_np()
        nbin = 0 if ldat.size == 0 else ldat.max()
        nbin = int(nbin) + 1
        if partner.scalar_dvol is not None:
            wgt = np.bincount(ldat.ravel(), minlength=nbin) * partner.scalar_dvol
        else:
            wgt = np.bincount(ldat.ravel(), minlength=nbin, weights=np.broadcast_to(partner.dvol, ldat.shape).ravel())
        wgt = wgt.astype(np.float64, copy=False)
        if (wgt == 0).any():
            raise ValueError("empty bins detected")
        self._init2(ldat, space, DOFSpace(wgt))

    def _init2(self, dofdex, space, other_space):
        from .. import config
        self._space = space
        dom = list(self._target)
        dom[self._space] = other_space
        self._domain = DomainTuple.make(dom)
        self._capability = self.TIMES | self.ADJOINT_TIMES
        firstaxis = self._target.axes[self._space][0]
        lastaxis = self._target.axes[self._space][-1]
        arrshape = self._target.shape
        self._pre = int(np.prod(arrshape[0:firstaxis], dtype=np.int64))
        self._post = int(np.prod(arrshape[lastaxis + 1:], dtype=np.int64))
        self._nbin = self._domain[self._space].shape[0]
        self._dofdex_np = dofdex
        self._bins = BinIndex.get(dofdex, self._nbin, config.device())

    def apply(self, x, mode):
        self._check_input(x, mode)
        v = x.val.contiguous()
        b = self._bins
        if mode == self.TIMES:
            out = torch.empty(self._target.shape, dtype=v.dtype, device=v.device)
            _native.bin_gather(v, b.pindex, out, self._pre, b.npix, self._nbin, self._post)
            return Field(self._target, out)
        out = torch.empty(self._domain.shape, dtype=v.dtype, device=v.device)
        _native.bin_scatter(v, b.perm, b.offsets, out, self._pre, b.npix, self._nbin, self._post)
        return Field(self._domain, out)


class PowerDistributor(DOFDistributor):
    def __init__(self, target, power_space=None, space=None):
        self._target = DomainTuple.make(target)
        self._space = infer_space(self._target, space)
        hspace = self._target[self._space]
        if not hspace.harmonic:
            raise ValueError("Operator requires harmonic target space")
        if power_space is None:
            power_space = PowerSpace(hspace)
        else:
            if not isinstance(power_space, PowerSpace):
                raise TypeError("power_space argument must be a PowerSpace")
            if power_space.harmonic_partner != hspace:
                raise ValueError("power_space does not match its partner")
        self._init2(power_space.pindex, self._space, power_space)
