"""SimpleCorrelatedField as one fused device model
(src/library/correlated_fields_simple.py:38-170).

    s(xi, theta) = offset_mean + c_h * HT[ A(theta)[pindex] * xi ]

with the non-parametric amplitude A(theta) of correlated_fields.py
(_TwoLogIntegrations, _SlopeRemover, _Normalization, fluctuation scaling,
zero-mode insertion, total-volume scaling) and HT the harmonic->position
Hartley transform with harmonic volume factor c_h.

Instead of the reference's operator tree (~40 nodes, each a separate pass
over its array) the model is one Operator whose Linearization carries a
single fused Jacobian node, CFJacobian:

    J [dxi, dtheta] = c_h HT[ A_full * dxi + xi0 * (dA(dtheta))[pindex] ]
    J^T g           = ( A_full * v ,  dA^T( bins(xi0 * v) ) ),  v = c_h HT g

whose grid work runs in the native kernels (Hartley passes, power-bin
gather/scatter) and whose B-sized amplitude Jacobian runs in the nft_amp_*
scan kernels on constants precomputed at the expansion point.  CFJacobian also implements ``sandwich_apply`` /
``metric_flat`` so that SandwichOperator and the fused CG can evaluate
J^T W J without materialising the operator tree."""
import os
import weakref

import numpy as np
import torch

from .. import _native, config
from ..domain_tuple import DomainTuple
from ..domains import PowerSpace, UnstructuredDomain
from ..ducc_dispatch import hartley_convention_code
from ..field import Field
from ..linearization import Linearization
from ..multi_domain import MultiDomain
from ..multi_field import MultiField
from ..operators.distributors import BinIndex
from ..operators.linear_operator import LinearOperator
from ..operators.operator import Operator
from ..packing import PackedLayout
from ..utilities import lognormal_moments
from .correlated_fields import (_log_vol, _relative_log_k_lengths, mode_multiplicity, slope_remove,
                                slope_remove_adjoint, twolog, twolog_adjoint)


# torch formulation of the amplitude JVP/VJP instead of the nft_amp kernels
# (A/B comparisons only; both run on the device)
_AMP_TORCH = os.environ.get("NFT_AMP_TORCH") is not None


def _t(a):
    return torch.as_tensor(np.ascontiguousarray(a), dtype=torch.float64, device=config.device())


# xi0 * v of the Jacobian adjoint stored as point-mirror pair sums on the half
# grid (NFT_O2_PAIRS=0: the full grid)
_O2_PAIRS = os.environ.get("NFT_O2_PAIRS", "1") != "0"

# amplitude forward + linearisation constants in native passes
# (NFT_AMP_NATIVE_FWD=0: the torch formulation, for A/B comparisons)
_AMP_NATIVE_FWD = os.environ.get("NFT_AMP_NATIVE_FWD", "1") != "0"

# folded prologue gather (NFT_PRO_FOLD=0 restores the per-pixel pindex gather)
_PRO_FOLD = os.environ.get("NFT_PRO_FOLD", "1") != "0"

# the CG curvature fold carried by the adjoint transform's R2C row pass
# (nft_hartley_fuse.fold_*; NFT_FOLD_R2C=0: its own launch between W and the
# adjoint)
_FOLD_R2C = os.environ.get("NFT_FOLD_R2C", "1") != "0"

# constant-scan tables for the two-phase amplitude kernels (nft_amp2_prepare:
# bitwise the same results with fewer scans); tests switch it off for A/B
AMP2_TABLE = True

class AmpLin:
    """Linearisation points of the amplitude made on the device
    (_AmplitudeModel.forward_rows): values a (k, B), the per-row constant
    vectors (buf) and k device nft_amp_const structs pointing into them.
    Stands in for the host AmpConst wherever the native JVP/VJP takes one:
    `host` carries B and the flags for the launch geometry, the kernels read
    every value from the device structs (item_consts)."""

    def __init__(self, amp, a, buf, dconst, k):
        import ctypes
        self.a, self.buf, self.dconst, self.k = a, buf, dconst, k
        self.keep = None
        self.size = ctypes.sizeof(_native.AmpConst)
        h = _native.AmpConst()
        h.B = amp.B
        h.has_flex, h.has_asp, h.has_zm = int(amp.has_flex), int(amp.has_asp), int(amp.has_zm)
        self.host = h
        self._rep = {}

    @property
    def B(self):
        return self.host.B

    def row_bytes(self, r):
        return self.dconst[r * self.size:(r + 1) * self.size]

    def items(self, k, row=0):
        """device pointer of k consecutive structs: row `row` shared by k
        right-hand sides"""
        if self.k == 1 and k == 1:
            return self.dconst.data_ptr()
        key = (k, row)
        if key not in self._rep:
            self._rep[key] = self.row_bytes(row).repeat(k)
        return self._rep[key].data_ptr()


class _AmplitudeModel:
    """Amplitude A(theta) on the PowerSpace, its JVP and VJP (B-sized math)."""

    def __init__(self, target, harmonic_partner, offset_std, fluctuations, flexibility, asperity,
                 loglogavgslope, prefix, zm_prefix=None):
        self.pspace = PowerSpace(harmonic_partner)
        self.B = self.pspace.shape[0]
        self.prefix = prefix
        p = prefix
        zp = prefix if zm_prefix is None else zm_prefix
        self.k_fl, self.k_sl = p + "fluctuations", p + "loglogavgslope"
        self.k_flex, self.k_asp = p + "flexibility", p + "asperity"
        self.k_spec, self.k_zm = p + "spectrum", zp + "zeromode"
        self.has_flex = flexibility is not None
        self.has_asp = asperity is not None
        self.has_zm = offset_std is not None
        self.lm_f, self.ls_f = (float(v) for v in lognormal_moments(*fluctuations))
        self.mu_s, self.sig_s = float(loglogavgslope[0]), float(loglogavgslope[1])
        if self.has_flex:
            self.lm_x, self.ls_x = (float(v) for v in lognormal_moments(*flexibility))
        if self.has_asp:
            self.lm_a, self.ls_a = (float(v) for v in lognormal_moments(*asperity))
        if self.has_zm:
            self.lm_o, self.ls_o = (float(v) for v in lognormal_moments(*offset_std))
        self.total_vol = float(target.total_volume)
        self.vslope = _t(_relative_log_k_lengths(self.pspace))
        rl = _relative_log_k_lengths(self.pspace)
        self.sc = _t(rl / float(rl[-1]))
        self.mult = _t(mode_multiplicity(self.pspace))
        if self.has_flex:
            lv = _log_vol(self.pspace)
            self.lv = _t(lv)
            self.sqrt_lv = _t(np.sqrt(lv))
            self.shift0 = _t(lv ** 2 / 12.)
        dom = {self.k_fl: DomainTuple.scalar_domain(), self.k_sl: DomainTuple.scalar_domain()}
        if self.has_flex:
            dom[self.k_flex] = DomainTuple.scalar_domain()
            dom[self.k_spec] = DomainTuple.make(UnstructuredDomain((2, self.B - 2)))
        if self.has_asp:
            dom[self.k_asp] = DomainTuple.scalar_domain()
        if self.has_zm:
            dom[self.k_zm] = DomainTuple.scalar_domain()
        self.domain_dict = dom

    # ------------------------------------------------------------- forward
    def forward(self, lat):
        """lat: dict key -> device tensor.  Returns (a, cache)."""
        c = {}
        fl = torch.exp(self.lm_f + self.ls_f * lat[self.k_fl])
        avgsl = self.mu_s + self.sig_s * lat[self.k_sl]
        apre = self.vslope * avgsl
        if self.has_flex:
            flex = torch.exp(self.lm_x + self.ls_x * lat[self.k_flex])
            sf = self.sqrt_lv * flex
            if self.has_asp:
                asp = torch.exp(self.lm_a + self.ls_a * lat[self.k_asp])
                sq0 = torch.sqrt(self.shift0 + asp)
                c["asp"] = asp
            else:
                sq0 = torch.sqrt(self.shift0)
            xs = lat[self.k_spec]
            at0 = xs[0] * sf * sq0
            at1 = xs[1] * sf
            apre = apre + slope_remove(twolog(at0, at1, self.lv), self.sc)
            c.update(flex=flex, sf=sf, sq0=sq0, xs=xs)
        spec = torch.exp(apre)
        S = torch.sum(self.mult * spec)
        An = torch.sqrt(spec * (1. / S))
        a = fl * An
        a = torch.cat([a.new_zeros(1), a[1:]])
        if self.has_zm:
            zm = torch.exp(self.lm_o + self.ls_o * lat[self.k_zm])
            a = a + torch.cat([zm.reshape(1), a.new_zeros(self.B - 1)])
            c["zm"] = zm
        a = a * self.total_vol
        c.update(fl=fl, spec=spec, S=S, An=An)
        return a, c

    def jvp(self, c, t):
        dfl = c["fl"] * self.ls_f * t[self.k_fl]
        dapre = self.vslope * (self.sig_s * t[self.k_sl])
        if self.has_flex:
            dsf = c["sf"] * (self.ls_x * t[self.k_flex])
            xs, ts, sf, sq0 = c["xs"], t[self.k_spec], c["sf"], c["sq0"]
            dat0 = ts[0] * sf * sq0 + xs[0] * dsf * sq0
            if self.has_asp:
                dsq0 = c["asp"] * self.ls_a * t[self.k_asp] / (2. * sq0)
                dat0 = dat0 + xs[0] * sf * dsq0
            dat1 = ts[1] * sf + xs[1] * dsf
            dapre = dapre + slope_remove(twolog(dat0, dat1, self.lv), self.sc)
        spec, S, An = c["spec"], c["S"], c["An"]
        dS = torch.sum(self.mult * spec * dapre)
        dAn = An * (dapre / 2. - dS / (2. * S))
        da = dfl * An + c["fl"] * dAn
        da = torch.cat([da.new_zeros(1), da[1:]])
        if self.has_zm:
            dzm = c["zm"] * self.ls_o * t[self.k_zm]
            da = da + torch.cat([dzm.reshape(1), da.new_zeros(self.B - 1)])
        return da * self.total_vol

    def vjp(self, c, g):
        """g: (B,) cotangent of a.  Returns dict key -> cotangent tensors."""
        out = {}
        g = g * self.total_vol
        if self.has_zm:
            out[self.k_zm] = c["zm"] * self.ls_o * g[0]
        gm = torch.cat([g.new_zeros(1), g[1:]])
        An, spec, S = c["An"], c["spec"], c["S"]
        out[self.k_fl] = c["fl"] * self.ls_f * torch.sum(gm * An)
        gAn = c["fl"] * gm
        gapre = An * gAn / 2. - self.mult * spec * (torch.sum(gAn * An) / (2. * S))
        out[self.k_sl] = self.sig_s * torch.sum(self.vslope * gapre)
        if self.has_flex:
            gtl = slope_remove_adjoint(gapre, self.sc)
            g0, g1 = twolog_adjoint(gtl, self.lv)
            xs, sf, sq0 = c["xs"], c["sf"], c["sq0"]
            out[self.k_spec] = torch.stack([g0 * sf * sq0, g1 * sf])
            gsf = g0 * xs[0] * sq0 + g1 * xs[1]
            out[self.k_flex] = c["flex"] * self.ls_x * torch.sum(gsf * self.sqrt_lv)
            if self.has_asp:
                gsq0 = g0 * xs[0] * sf
                out[self.k_asp] = c["asp"] * self.ls_a * torch.sum(gsq0 / (2. * sq0))
        return out

    # ------------------------------------------------- native linearisation
    def native_const(self, c):
        """Per-bin constants of the linearisation at the expansion point for
        the native JVP/VJP kernels (nft_amp_*, include/nifty_amd.h).  Returns
        (AmpConst, keep-alive dict of the device tensors it points to); an
        AmpLin from forward_rows is its own constant set."""
        if isinstance(c, AmpLin):
            return c, None
        keep = {}
        if self.has_flex:
            xs, sf, sq0 = c["xs"], c["sf"], c["sq0"]
            keep["c0"] = (sf * sq0).contiguous()
            keep["sf"] = sf.contiguous()
            keep["p0"] = (xs[0] * sf * (self.ls_x * sq0)).contiguous()
            keep["p2"] = (xs[1] * sf * self.ls_x).contiguous()
            keep["lv"] = self.lv
            keep["Qf"] = slope_remove(twolog(keep["p0"], keep["p2"], self.lv), self.sc).contiguous()
            if self.has_asp:
                keep["p1"] = (xs[0] * sf * c["asp"] * self.ls_a / (2. * sq0)).contiguous()
                keep["Qa"] = slope_remove(twolog(keep["p1"], torch.zeros_like(keep["p1"]), self.lv),
                                          self.sc).contiguous()
        keep["vslope"], keep["sc"] = self.vslope, self.sc
        keep["mspec"] = (self.mult * c["spec"]).contiguous()
        keep["An"] = c["An"].contiguous()
        k = _native.AmpConst()
        for name in ("c0", "sf", "p0", "p1", "p2", "lv", "vslope", "sc", "Qf", "Qa", "mspec", "An"):
            setattr(k, name, keep[name].data_ptr() if name in keep else None)
        k.fl, k.S = float(c["fl"]), float(c["S"])
        k.ls_f, k.sig_s = self.ls_f, self.sig_s
        k.zm = float(c["zm"]) if self.has_zm else 0.0
        k.ls_o = self.ls_o if self.has_zm else 0.0
        k.total_volume = self.total_vol
        k.B = self.B
        k.has_flex, k.has_asp, k.has_zm = int(self.has_flex), int(self.has_asp), int(self.has_zm)
        return k, keep

    # ------------------------------------------------- native forward
    def native_model(self):
        """nft_amp_model of this amplitude (fixed per-bin vectors + scalars)"""
        nm = getattr(self, "_nm", None)
        if nm is None:
            k = _native.AmpModel()
            keep = dict(vslope=self.vslope, sc=self.sc, mult=self.mult)
            if self.has_flex:
                keep.update(lv=self.lv, sqrt_lv=self.sqrt_lv, shift0=self.shift0)
            keep = {n: v.contiguous() for n, v in keep.items()}
            for n in ("vslope", "sc", "mult", "lv", "sqrt_lv", "shift0"):
                setattr(k, n, keep[n].data_ptr() if n in keep else None)
            k.lm_f, k.ls_f, k.mu_s, k.sig_s = self.lm_f, self.ls_f, self.mu_s, self.sig_s
            if self.has_flex:
                k.lm_x, k.ls_x = self.lm_x, self.ls_x
            if self.has_asp:
                k.lm_a, k.ls_a = self.lm_a, self.ls_a
            if self.has_zm:
                k.lm_o, k.ls_o = self.lm_o, self.ls_o
            k.total_volume = self.total_vol
            k.B = self.B
            k.has_flex, k.has_asp, k.has_zm = int(self.has_flex), int(self.has_asp), int(self.has_zm)
            nm = self._nm = (k, keep)
        return nm[0]

    def forward_rows(self, at, k, lat_stride, device):
        """Amplitude values and linearisation constants at k latent points in
        one native pass (nft_amp_forward_batched): at(key) -> device pointer of
        row 0's key or None, rows lat_stride elements apart.  Nothing is read
        back to the host."""
        import ctypes
        lib = _native.load()
        nbuf = int(lib.nft_amp_forward_buf(self.B))
        a = torch.empty((k, self.B), dtype=torch.float64, device=device)
        buf = torch.empty((k, nbuf), dtype=torch.float64, device=device)
        dconst = torch.empty(k * ctypes.sizeof(_native.AmpConst), dtype=torch.uint8, device=device)
        ws = _native.workspace(k * lib.nft_amp_workspace(self.B), device, "amp")
        P = ctypes.c_void_p
        _native._check(lib.nft_amp_forward_batched(
            ctypes.byref(self.native_model()), P(at(self.k_fl)), P(at(self.k_sl)), P(at(self.k_flex)),
            P(at(self.k_asp)), P(at(self.k_zm)), P(at(self.k_spec)), int(lat_stride), k, P(a.data_ptr()), self.B,
            P(buf.data_ptr()), nbuf, P(dconst.data_ptr()), P(ws.data_ptr()), _native.stream_ptr()))
        return AmpLin(self, a, buf, dconst, k)

    def forward_native(self, lat):
        """forward_rows at one latent point given as a dict key -> tensor"""
        vals = {kk: v.contiguous() for kk, v in lat.items() if kk in self.domain_dict}

        def at(key):
            return vals[key].data_ptr() if key in vals else None
        lin = self.forward_rows(at, 1, 0, next(iter(vals.values())).device)
        lin.keep = vals
        return lin

    def _ptrs(self, D, off):
        """base pointers of the amplitude keys of packed row 0 of D (or None)"""
        def at(key):
            if key not in off:
                return None
            return D[0, off[key]:].data_ptr()
        return at

    def _keys6(self):
        return (self.k_fl, self.k_sl, self.k_flex, self.k_asp, self.k_zm, self.k_spec)

    def _key_ptrs(self, T, off):
        """ctypes array of the 6 key pointers (fl, sl, flex, asp, zm, spec) of
        packed row 0 of T (NULL for absent keys), or NULL if T is None"""
        import ctypes
        if T is None:
            return None
        return (ctypes.c_void_p * 6)(*[T[0, off[kk]:].data_ptr() if kk in off else None for kk in self._keys6()])

    @staticmethod
    def _item_mode(const, item_consts):
        """(host AmpConst, item pointer, nft_amp2 item_mode): an AmpLin
        without per-item constants is ONE device constant set shared by every
        right-hand side (mode 2)"""
        if isinstance(const, AmpLin):
            if item_consts is None:
                return const.host, const.items(1), 2
            return const.host, item_consts, 1
        return const, item_consts, (1 if item_consts else 0)

    def amp2_table(self, const):
        """constant-scan table of the constant set `const` (nft_amp2_prepare),
        made once per set and kept on it; None for per-RHS constant sets, when
        switched off, or when first asked for during a graph capture"""
        import ctypes
        if not AMP2_TABLE:
            return None
        host, ic, mode = self._item_mode(const, None)
        if mode == 1:
            return None
        tab = getattr(const, "_amp2_tab", None)
        if tab is None:
            if torch.cuda.is_current_stream_capturing():
                return None
            lib = _native.load()
            n = int(lib.nft_amp2_tab_size(self.B))
            if n <= 0:
                return None
            tab = torch.empty(n, dtype=torch.float64, device=self.vslope.device)
            _native._check(lib.nft_amp2_prepare(ctypes.byref(host), ctypes.c_void_p(ic), mode,
                                                ctypes.c_void_p(tab.data_ptr()), _native.stream_ptr()))
            const._amp2_tab = tab
        return tab

    @staticmethod
    def _tab_ptr(tab):
        import ctypes
        return ctypes.c_void_p(tab.data_ptr() if tab is not None else None)

    def native_jvp_batched(self, const, D, off, da, interleave=False, item_consts=None):
        """da[b] = J_amp D[b] for the k rows of a packed batch D (k, size);
        interleave: da is (B, k), bin-major (one contiguous run per bin)."""
        import ctypes
        k, size = D.shape
        lib = _native.load()
        ws = _native.workspace(k * lib.nft_amp_workspace(self.B), D.device, "amp")
        P = ctypes.c_void_p
        host, ic, mode = self._item_mode(const, item_consts)
        if da.dtype != D.dtype:
            raise _native.NativeError("native_jvp_batched: da and D dtypes differ")
        tab = self.amp2_table(const) if item_consts is None else None
        st = lib.nft_amp2_jvp(ctypes.byref(host), P(ic), mode, self._key_ptrs(D, off), None, size, P(da.data_ptr()),
                              1 if interleave else self.B, k if interleave else 1, P(ws.data_ptr()), k, None, None,
                              0, 0.0, _native.dtype_code(D.dtype), self._tab_ptr(tab), _native.stream_ptr())
        if st != _native.AMP2_FALLBACK:
            _native._check(st)
            return da
        if D.dtype != torch.float64:
            raise _native.NativeError("the multi-kernel amplitude JVP is fp64 only (NFT_AMP2=0 with fp32 storage)")
        at = self._ptrs(D, off)
        if mode == 2:
            ic = const.items(k)
        _native._check(lib.nft_amp_jvp_batched(
            ctypes.byref(host), P(ic), P(at(self.k_fl)), P(at(self.k_sl)), P(at(self.k_flex)), P(at(self.k_asp)),
            P(at(self.k_zm)), P(at(self.k_spec)), P(da.data_ptr()), P(ws.data_ptr()), k, size,
            1 if interleave else self.B, k if interleave else 1, _native.stream_ptr()))
        return da

    def native_vjp_batched(self, const, g, Q, off, D=None, shift=0.0, item_consts=None):
        """Q[b] amplitude keys = shift * D[b] + J_amp^T g[b]."""
        import ctypes
        k, size = Q.shape
        lib = _native.load()
        ws = _native.workspace(k * lib.nft_amp_workspace(self.B), Q.device, "amp")
        P = ctypes.c_void_p
        host, ic, mode = self._item_mode(const, item_consts)
        dk = self._key_ptrs(D, off) if (D is not None and shift != 0.0) else None
        if g.dtype != Q.dtype or (D is not None and D.dtype != Q.dtype):
            raise _native.NativeError("native_vjp_batched: g, Q and D dtypes differ")
        tab = self.amp2_table(const) if item_consts is None else None
        st = lib.nft_amp2_vjp(ctypes.byref(host), P(ic), mode, P(g.data_ptr()), self.B, self._key_ptrs(Q, off), None,
                              dk, size, float(shift), P(ws.data_ptr()), k, None, None, 0, None, 0, 0, 0,
                              _native.dtype_code(Q.dtype), self._tab_ptr(tab), _native.stream_ptr())
        if st != _native.AMP2_FALLBACK:
            _native._check(st)
            return Q
        if Q.dtype != torch.float64:
            raise _native.NativeError("the multi-kernel amplitude VJP is fp64 only (NFT_AMP2=0 with fp32 storage)")
        if mode == 2:
            ic = const.items(k)
        atq = self._ptrs(Q, off)
        atd = self._ptrs(D, off) if (D is not None and shift != 0.0) else (lambda key: None)
        o = _native.AmpOut()
        for short, key in (("fl", self.k_fl), ("sl", self.k_sl), ("flex", self.k_flex), ("asp", self.k_asp),
                           ("zm", self.k_zm), ("spec", self.k_spec)):
            setattr(o, short, atq(key))
            setattr(o, "d" + short, atd(key))
        o.shift = float(shift)
        _native._check(lib.nft_amp_vjp_batched(ctypes.byref(host), ctypes.c_void_p(ic),
                                               ctypes.c_void_p(g.data_ptr()), ctypes.byref(o),
                                               ctypes.c_void_p(ws.data_ptr()), k, size, self.B,
                                               _native.stream_ptr()))
        return Q

    # ----- the amplitude keys' CG work carried by the two-phase kernels
    def amp2_tiles(self, const, k):
        """tile count of the two-phase JVP / VJP for k RHS (0: not applicable)"""
        _, _, mode = self._item_mode(const, None)
        return int(_native.load().nft_amp2_tiles(self.B, k, mode))

    def native_jvp_dir(self, const, D, R, off, da, SC, part, pstride, shift):
        """d = max(0, gamma/gprev) d + r on the amplitude keys of the k rows of
        D (in place), d.d partials per tile (times shift) into part, and
        da (B, k) = J_amp d, bin-major (nft_amp2_jvp with residual keys)."""
        import ctypes
        k, size = D.shape
        lib = _native.load()
        ws = _native.workspace(k * lib.nft_amp_workspace(self.B), D.device, "amp")
        P = ctypes.c_void_p
        host, ic, mode = self._item_mode(const, None)
        _native._check(lib.nft_amp2_jvp(ctypes.byref(host), P(ic), mode, self._key_ptrs(D, off),
                                        self._key_ptrs(R, off), size, P(da.data_ptr()), 1, k, P(ws.data_ptr()), k,
                                        P(SC.data_ptr()), P(part.data_ptr()), int(pstride), float(shift),
                                        _native.dtype_code(D.dtype), self._tab_ptr(self.amp2_table(const)),
                                        _native.stream_ptr()))
        return da

    def native_vjp_cg(self, const, g, X, R, D, off, SC, part, pstride, gpart, gp_stride, gp_row, ngp, shift):
        """the amplitude keys' CG update x -= alpha d, r -= alpha (J_amp^T g +
        shift d) and the iteration's finalize over their r.r / x.r partials
        and the grid segment's (nft_amp2_vjp with out2)"""
        import ctypes
        k, size = X.shape
        lib = _native.load()
        ws = _native.workspace(k * lib.nft_amp_workspace(self.B), X.device, "amp")
        P = ctypes.c_void_p
        host, ic, mode = self._item_mode(const, None)
        _native._check(lib.nft_amp2_vjp(ctypes.byref(host), P(ic), mode, P(g.data_ptr()), self.B,
                                        self._key_ptrs(X, off), self._key_ptrs(R, off), self._key_ptrs(D, off), size,
                                        float(shift), P(ws.data_ptr()), k, P(SC.data_ptr()), P(part.data_ptr()),
                                        int(pstride), P(gpart.data_ptr()), int(gp_stride), int(gp_row), int(ngp),
                                        _native.dtype_code(X.dtype), self._tab_ptr(self.amp2_table(const)),
                                        _native.stream_ptr()))

    def native_jvp(self, const, t, da):
        if isinstance(const, AmpLin):
            import ctypes
            lib = _native.load()
            ws = _native.workspace(lib.nft_amp_workspace(self.B), da.device, "amp")
            P = ctypes.c_void_p

            def ptr(key):
                v = t.get(key)
                return P(v.data_ptr() if v is not None else None)
            _native.require_device(da, *[v for v in t.values()])
            _native._check(lib.nft_amp_jvp_batched(
                ctypes.byref(const.host), P(const.items(1)), ptr(self.k_fl), ptr(self.k_sl), ptr(self.k_flex),
                ptr(self.k_asp), ptr(self.k_zm), ptr(self.k_spec), P(da.data_ptr()), P(ws.data_ptr()), 1, 0, 0, 1,
                _native.stream_ptr()))
            return da
        g = t.get
        _native.amp_jvp(const, g(self.k_fl), g(self.k_sl), g(self.k_flex), g(self.k_asp),
                        g(self.k_zm), g(self.k_spec), da)
        return da

    def native_vjp(self, const, g, out, d=None, shift=0.0):
        """out/d: dict key -> contiguous device tensors; out = shift*d + J^T g."""
        o = _native.AmpOut()
        names = (("fl", self.k_fl), ("sl", self.k_sl), ("flex", self.k_flex), ("asp", self.k_asp),
                 ("zm", self.k_zm), ("spec", self.k_spec))
        for short, key in names:
            if key in out:
                setattr(o, short, out[key].data_ptr())
                if d is not None and shift != 0.0:
                    setattr(o, "d" + short, d[key].data_ptr())
        o.shift = float(shift)
        if isinstance(const, AmpLin):
            import ctypes
            lib = _native.load()
            ws = _native.workspace(lib.nft_amp_workspace(self.B), g.device, "amp")
            _native.require_device(g)
            _native._check(lib.nft_amp_vjp_batched(
                ctypes.byref(const.host), ctypes.c_void_p(const.items(1)), ctypes.c_void_p(g.data_ptr()),
                ctypes.byref(o), ctypes.c_void_p(ws.data_ptr()), 1, 0, 0, _native.stream_ptr()))
            return out
        _native.amp_vjp(const, g, o)
        return out


class _AmplitudeJacobian(LinearOperator):
    def __init__(self, amp, cache, domain, target):
        self._amp, self._c = amp, cache
        self._domain, self._target = domain, target
        self._capability = self.TIMES | self.ADJOINT_TIMES

    def apply(self, x, mode):
        self._check_input(x, mode)
        if mode == self.TIMES:
            return Field(self._target, self._amp.jvp(self._c, {k: x[k].val for k in x.keys()}))
        g = self._amp.vjp(self._c, x.val)
        return MultiField(self._domain, tuple(Field(self._domain[k], g[k]) for k in self._domain.keys()))


class _AmplitudeOperator(Operator):
    """`op.amplitude` of the reference: latent (without xi) -> PowerSpace."""

    def __init__(self, amp, power=1):
        self._amp = amp
        self._domain = MultiDomain.make(amp.domain_dict)
        self._target = DomainTuple.make(amp.pspace)
        self._power = power

    def apply(self, x):
        self._check_input(x)
        lin = x.jac is not None
        v = x.val if lin else x
        a, c = self._amp.forward({k: v[k].val for k in self._domain.keys()})
        res = Field(self._target, a if self._power == 1 else a ** 2)
        if not lin:
            return res
        jac = _AmplitudeJacobian(self._amp, c, self._domain, self._target)
        if self._power == 2:
            from ..sugar import makeOp
            jac = makeOp(Field(self._target, 2. * a)) @ jac
        return x.new(res, jac)

    def force(self, x):
        return self.apply(x.extract(self._domain))


class CFJacobian(LinearOperator):
    """Fused Jacobian of the correlated field at an expansion point."""

    def __init__(self, model, cache, a, afull, xi0):
        self._m = model
        self._c = cache
        self._a = a
        self._afull = afull
        self._xi0 = xi0
        self._domain = model.domain
        self._target = model.target
        self._capability = self.TIMES | self.ADJOINT_TIMES
        self.device = afull.device
        self._k = None

    @property
    def layout(self):
        return self._m.layout

    # ---------------------------------------------------------- primitives
    def _const(self):
        if self._k is None:
            self._k = self._m.amp.native_const(self._c)
            self._m.amp.amp2_table(self._k[0])  # before any graph capture uses it
        return self._k[0]

    def _times_t(self, t):
        """t: dict key->tensor tangent.  Returns position-space grid tensor:
        c_h HT[A_full * t_xi + xi0 * dA[pindex]] in one fused native transform
        (the gather and the two products run inside its first pass)."""
        m = self._m
        if _AMP_TORCH:
            da = m.amp.jvp(self._c, t)
        else:
            da = torch.empty(m.amp.B, dtype=torch.float64, device=self.device)
            m.amp.native_jvp(self._const(), {k: v.contiguous() for k, v in t.items()}, da)
        out = torch.empty(self._afull.shape, dtype=self._afull.dtype, device=self.device)
        pro = dict(a=self._afull, x=t[m.k_xi].contiguous(), b=self._xi0, **self._pro_bins(da.contiguous(), 1))
        return _native.hartley_fused(out, range(out.ndim), m.c_h, pro=pro, convention=hartley_convention_code())

    def _pro_bins(self, da, k):
        """bin operand of the forward prologue: with mirror-symmetric bins the
        per-cell bin index of the fundamental cell (nft_hartley_fuse.pro_folded:
        dA gathered once per mirror class, 2^d fewer scattered gathers, no
        per-pixel index read), else the per-pixel pindex.  The values read
        are the same either way."""
        jb = self._m.jbins
        if _PRO_FOLD and jb.fold is not None:
            return dict(c=da, index=jb.fold["pindex"], fold=True)
        return dict(c=da, index=self._m.bins.pindex)

    def _adjoint_t(self, g, out=None, d=None, shift=0.0):
        """g: grid tensor.  Returns dict key->tensor, or fills the `out` views
        with shift * d + J^T g.  One fused transform produces both
        A_full * v (+ shift * d_xi) and xi0 * v, v = c_h HT g."""
        m = self._m
        b = m.bins
        grid = tuple(self._afull.shape)
        pairs = self._pairs(1)
        # with pair sums: the batched adjoint's layout (a batch of one), so
        # single and batched solves stay bitwise equal
        w = torch.empty(self._half(grid) if pairs else grid, dtype=self._afull.dtype, device=self.device)
        oxi = out[m.k_xi] if out is not None else torch.empty(grid, dtype=self._afull.dtype, device=self.device)
        epi = dict(a=self._afull, b=self._xi0, out2=w, pairs=pairs)
        if out is not None and shift != 0.0:
            epi.update(d=d[m.k_xi], shift=shift)
        if pairs:
            N = self._afull.numel()
            _native.hartley_fused(oxi, tuple(range(1, 1 + len(grid))), m.c_h, x=g.contiguous(), epi=epi,
                                  convention=hartley_convention_code(), shape=(1,) + grid,
                                  batch=dict(period=N, out=N, out2=w.numel(), d=N))
        else:
            _native.hartley_fused(oxi, range(len(grid)), m.c_h, x=g.contiguous(), epi=epi,
                                  convention=hartley_convention_code())
        ga = torch.empty(m.amp.B, dtype=w.dtype, device=w.device)
        if pairs:
            wf = torch.empty((1, m.jbins.fold["nf"]), dtype=w.dtype, device=w.device)
            m.jbins.scatter_from(m.jbins.fold_into(w, wf, 1, half=True), ga, 1)
        else:
            m.jbins.scatter(w, ga, 1)
        if out is None:
            if _AMP_TORCH:
                res = m.amp.vjp(self._c, ga)
            else:
                res = {k: torch.empty(self._domain[k].shape, dtype=torch.float64, device=self.device)
                       for k in m.amp.domain_dict}
                m.amp.native_vjp(self._const(), ga, res)
            res[m.k_xi] = oxi
            return res
        if _AMP_TORCH:
            res = m.amp.vjp(self._c, ga)
            for k, r in res.items():
                if shift != 0.0:
                    torch.add(r.reshape(out[k].shape), d[k], alpha=shift, out=out[k])
                else:
                    out[k].copy_(r.reshape(out[k].shape))
        else:
            m.amp.native_vjp(self._const(), ga, out, d, shift)
        return out

    def apply(self, x, mode):
        self._check_input(x, mode)
        if mode == self.TIMES:
            return Field(self._target, self._times_t({k: x[k].val for k in x.keys()}))
        res = self._adjoint_t(x.val)
        return MultiField(self._domain, tuple(Field(self._domain[k], res[k].reshape(self._domain[k].shape))
                                              for k in self._domain.keys()))

    def sandwich_apply(self, x, W):
        """J^T W J x for a latent MultiField x, W a grid tensor."""
        s = self._times_t({k: x[k].val for k in x.keys()})
        res = self._adjoint_t(W(s) if callable(W) else s * W)
        return MultiField(self._domain, tuple(Field(self._domain[k], res[k].reshape(self._domain[k].shape))
                                              for k in self._domain.keys()))

    def metric_flat_batch(self, D, Q, W, shift, qpart=None):
        """Q[b] = shift * D[b] + J^T W J D[b] for the k rows of D (k, size),
        every stage launched once for the whole batch (nft_*_batched; the LOS
        matrix is streamed once for all rows).  Per row bitwise equal to
        metric_flat."""
        if D.dtype == torch.float32 and not self.phases_fp32(D.shape[0]):
            if qpart is not None:
                raise NotImplementedError("data-space curvature partials: fp32 needs the two-phase amplitude kernels")
            return self._metric_flat_batch32(D, Q, W, shift)
        da = self.mv_amp_jvp(D)
        w = self.mv_grid(D, da, Q, W, shift, qpart)
        self.mv_amp_vjp(D, w, Q, shift)
        return Q

    # The three phases of metric_flat_batch.  Only mv_grid touches the grid
    # segment of D and Q; the amplitude phases read / write the amplitude keys
    # alone, so a caller may run them on a second stream next to the grid
    # segment's CG work (fused_cg.FusedCGBatch).  Their buffers persist per
    # batch size: no allocation is freed while another stream may use it.
    def _mv_bufs(self, k, dtype=torch.float64):
        """the phases' buffers for k rows of storage dtype (fp64, or fp32 for
        the fp32-storage CG: every grid operand and dA in fp32)"""
        bufs = getattr(self, "_mvb", None)
        if bufs is None or bufs["k"] != k or bufs["dt"] != dtype:
            grid = tuple(self._afull.shape)
            dt = dtype
            B = self._m.amp.B
            fold = self._m.jbins.fold
            wshape = self._half(grid) if self._pairs(k) else grid
            bufs = self._mvb = dict(k=k, dt=dtype, da=torch.empty((B, k), dtype=dt, device=self.device),
                                    s=torch.empty((k,) + grid, dtype=dt, device=self.device),
                                    w=torch.empty((k,) + wshape, dtype=dt, device=self.device),
                                    wf=torch.empty((k, fold["nf"]) if fold else (1,), dtype=dt,
                                                   device=self.device),
                                    ga=torch.empty((k, B), dtype=dt, device=self.device))
        return bufs

    def _grid_ops(self, dtype):
        """(A_full, xi0) in the storage dtype (fp32 copies made once)"""
        if dtype == self._afull.dtype:
            return self._afull, self._xi0
        c = self.__dict__.setdefault("_g32", {})
        if dtype not in c:
            c[dtype] = (self._afull.to(dtype), self._xi0.to(dtype))
        return c[dtype]

    def _weight(self, W, dtype):
        """a pointwise weight tensor in the storage dtype: ONE cached copy,
        keyed on the tensor object itself (a weak reference: a new W at a
        recycled address is not mistaken for the old one) and its version
        counter (an in-place update of W is seen)"""
        if not torch.is_tensor(W) or W.dtype == dtype:
            return W
        c = self.__dict__.get("_w32")
        if c is not None:
            ref, ver, dt, val = c
            if ref() is W and ver == W._version and dt == dtype:
                return val
        val = W.to(dtype).contiguous()
        self._w32 = (weakref.ref(W), W._version, dtype, val)
        return val

    def phases_fp32(self, k):
        """True if the phase methods (mv_*) run on fp32 storage: the
        two-phase amplitude kernels apply (nft_amp2_* with dtype 1)"""
        return self.amp2_tiles(k) > 0

    @staticmethod
    def _half(grid):
        return tuple(grid[:-1]) + (grid[-1] // 2 + 1,)

    def _pairs(self, k):
        """the adjoint stores xi0 * v as point-mirror pair sums on the half
        grid (nft_hartley_fuse.epi_out2_pairs): half the bytes of the second
        epilogue output and of the mirror fold's input"""
        return (_O2_PAIRS and self._m.jbins.fold is not None and len(self._afull.shape) >= 2
                and self.cg_blocks(k) > 0)

    def mv_amp_jvp(self, D):
        """dA (B, k) of the k rows of D, bin-major interleaved: the
        prologue's bin gather reads one contiguous run per pixel for all k"""
        m = self._m
        k = D.shape[0]
        da = self._mv_bufs(k, D.dtype)["da"]
        m.amp.native_jvp_batched(self._const(), D, dict(zip(self.layout.keys, self.layout.offsets)), da,
                                 interleave=True)
        return da

    def amp2_tiles(self, k):
        """tile count of the two-phase amplitude kernels (carried direction /
        update of the amplitude keys), 0 if they do not apply"""
        return self._m.amp.amp2_tiles(self._const(), k)

    def mv_amp_jvp_dir(self, D, R, SC, part, pstride, shift):
        """the amplitude keys' CG direction update (in place, d.d partials per
        tile) and dA (B, k) of the updated D, bin-major interleaved"""
        m = self._m
        k = D.shape[0]
        da = self._mv_bufs(k, D.dtype)["da"]
        return m.amp.native_jvp_dir(self._const(), D, R, dict(zip(self.layout.keys, self.layout.offsets)), da, SC,
                                    part, pstride, shift)

    def mv_amp_vjp_cg(self, X, R, D, w, SC, part, pstride, gpart, gp_stride, gp_row, ngp, shift):
        """bin sums of w, then the amplitude keys' CG update with J_amp^T and
        the iteration's finalize (no q is stored)"""
        m = self._m
        k = X.shape[0]
        ga = self._mv_bufs(k, X.dtype)["ga"]
        m.jbins.scatter_from(self.mv_fold(w), ga, k)
        m.amp.native_vjp_cg(self._const(), ga, X, R, D, dict(zip(self.layout.keys, self.layout.offsets)), SC, part,
                            pstride, gpart, gp_stride, gp_row, ngp, shift)

    def cg_blocks(self, k):
        """partial blocks per item of the CG-carrying adjoint epilogue at
        this grid (nft_hartley_cg_blocks), 0 if unsupported"""
        cache = self.__dict__.setdefault("_cgb", {})
        if k not in cache:
            grid = tuple(self._afull.shape)
            cache[k] = _native.hartley_cg_blocks((k,) + grid, tuple(range(1, 1 + len(grid))), self._afull.dtype)
        return cache[k]

    def pointwise_quad_blocks(self, W):
        """partials per RHS of (J d).W(J d) formed by the forward transform's
        epilogue for a pointwise weight W (a grid-shaped tensor of the grid's
        dtype), 0 where that epilogue does not apply"""
        if not (torch.is_tensor(W) and W.dtype in (torch.float64, torch.float32)
                and tuple(W.shape) == tuple(self._afull.shape) and W.is_contiguous() and W.device == self.device):
            return 0
        return self.cg_blocks(1)

    def lazy_ok(self, k):
        """the carried iteration can defer its iterate (nft_hartley_fuse.lazy_*):
        the direction is carried by the row-staged prologue"""
        grid = tuple(self._afull.shape)
        return self.dir_blocks(k) > 0 and 2 <= len(grid) <= 3 and grid[-1] // 2 + 1 <= 2556

    def grid_size(self):
        """elements of the grid key (the grid segment without its padding)"""
        return int(self._afull.numel())

    def dir_blocks(self, k):
        """d.d partial blocks of the CG direction carried by the folded
        prologue (nft_hartley_fuse.dir_*), 0 where the prologue is not folded"""
        jb = self._m.jbins
        if not (_PRO_FOLD and jb.fold is not None) or not (1 <= k <= 8):
            return 0
        return _native.hartley_dir_blocks(jb.fold["shape"])

    def mv_grid(self, D, da, Q, W, shift=0.0, qpart=None, after_w=None, cg=None, pro_dir=None):
        """forward transform (with the prologue), W, adjoint transform: the
        grid segment of Q and w = xi0 * v for the amplitude VJP.
        after_w: called between W and the adjoint (the curvature fold);
        cg: the grid segment's CG update carried by the adjoint's epilogue
        (nft_hartley_fuse.cg_*) -- Q's grid segment is then not written.
        pro_dir: the grid segment's CG direction update carried by the folded
        prologue (nft_hartley_fuse.dir_*): D's grid segment is updated in place."""
        m = self._m
        lay = self.layout
        k, size = D.shape
        bufs = self._mv_bufs(k, D.dtype)
        afull, xi0 = self._grid_ops(D.dtype)
        W = self._weight(W, D.dtype)
        grid = tuple(afull.shape)
        N = afull.numel()
        xo = dict(zip(lay.keys, lay.offsets))[m.k_xi]
        axes = tuple(range(1, 1 + len(grid)))
        conv = hartley_convention_code()
        s = bufs["s"]
        pro = dict(a=afull, x=D[0, xo:], b=xi0, **self._pro_bins(da, k))
        if pro_dir is not None:
            pro["dir"] = pro_dir
        bt = dict(period=N, x=size, c=1, c_elem=k)
        if qpart is not None and torch.is_tensor(W):
            # pointwise W inside the forward's last pass: s = W * (J d) and
            # the per-tile partials of (J d).W(J d) (nft_hartley_fuse.quad_*)
            _native.hartley_fused(s, axes, m.c_h, pro=pro, epi=dict(a=W), convention=conv, shape=s.shape,
                                  batch=bt, quad=dict(part=qpart, pstride=qpart.stride(0)))
            g = s
        else:
            _native.hartley_fused(s, axes, m.c_h, pro=pro, convention=conv, shape=s.shape, batch=bt)
            fspec = getattr(after_w, "spec", None)
            if fspec is not None and qpart is not None and callable(W) and getattr(W, "supports_fold", False):
                # the fold rides in W's last launch (it needs only W's partials)
                g = W(s, qpart=qpart, fold=fspec)
                after_w = None
            else:
                g = (W(s, qpart=qpart) if qpart is not None else W(s)) if callable(W) else s * W
            g = g.contiguous()
        fold = None
        if after_w is not None:
            fold = getattr(after_w, "spec", None) if _FOLD_R2C else None
            if fold is None:
                after_w()
        w = bufs["w"]
        pairs = self._pairs(k)
        epi = dict(a=afull, b=xi0, out2=w, pairs=pairs)
        bt = dict(period=N, out=size, out2=w[0].numel())
        if shift != 0.0:
            epi.update(d=D[0, xo:], shift=shift)
            bt["d"] = size
        _native.hartley_fused(Q[0, xo:], axes, m.c_h, x=g, epi=epi, convention=conv, shape=(k,) + grid, batch=bt,
                              cg=cg, fold=fold)
        return w

    def mv_fold(self, w):
        """the mirror fold of w (the bandwidth-bound half of the bin sums)"""
        k = w.shape[0]
        return self._m.jbins.fold_into(w, self._mv_bufs(k, w.dtype)["wf"], k, half=self._pairs(k))

    def mv_amp_vjp(self, D, w, Q, shift=0.0, folded=None):
        """bin sums of w (folded: mv_fold's result, if already formed) and the
        amplitude VJP into Q's amplitude keys"""
        m = self._m
        k = Q.shape[0]
        ga = self._mv_bufs(k, Q.dtype)["ga"]
        m.jbins.scatter_from(self.mv_fold(w) if folded is None else folded, ga, k)
        m.amp.native_vjp_batched(self._const(), ga, Q, dict(zip(self.layout.keys, self.layout.offsets)), D, shift)
        return Q

    def grid_segment(self):
        """[start, stop) of the grid key ('xi') in the packed layout, padding
        included: the amplitude keys lie outside it"""
        lay = self.layout
        i = lay.keys.index(self._m.k_xi)
        o = lay.offsets[i]
        stop = lay.offsets[i + 1] if i + 1 < len(lay.keys) else lay.size
        return o, stop

    supports_fp32 = True

    def _metric_flat_batch32(self, D, Q, W, shift):
        """metric_flat_batch on fp32 storage (config.set_cg_precision("fp32")):
        grid operands (A_full, xi0, the transforms, W, the bin sums) in fp32,
        the B-sized amplitude Jacobian in fp64 on fp64 copies of the (small)
        amplitude segments; every reduction accumulates in fp64."""
        m = self._m
        lay = self.layout
        k, size = D.shape
        amp = m.amp
        B = amp.B
        grid = tuple(self._afull.shape)
        N = self._afull.numel()
        off = dict(zip(lay.keys, lay.offsets))
        xo = off[m.k_xi]
        axes = tuple(range(1, 1 + len(grid)))
        conv = hartley_convention_code()
        const = self._const()
        c32 = getattr(self, "_c32", None)
        if c32 is None:
            c32 = self._c32 = dict(afull=self._afull.float(), xi0=self._xi0.float(), W={})
        segs = [(o, n) for kk, o, n in zip(lay.keys, lay.offsets, lay.sizes) if kk != m.k_xi]
        D64 = torch.zeros((k, size), dtype=torch.float64, device=D.device)
        for o, n in segs:
            D64[:, o:o + n] = D[:, o:o + n]
        da = torch.empty((B, k), dtype=torch.float64, device=self.device)
        amp.native_jvp_batched(const, D64, off, da, interleave=True)
        da32 = da.float()
        s = torch.empty((k,) + grid, dtype=torch.float32, device=self.device)
        pro = dict(a=c32["afull"], x=D[0, xo:], b=c32["xi0"], **self._pro_bins(da32, k))
        _native.hartley_fused(s, axes, m.c_h, pro=pro, convention=conv, shape=s.shape,
                              batch=dict(period=N, x=size, c=1, c_elem=k))
        if callable(W):
            g = W(s)
        else:
            if torch.is_tensor(W):
                key = W.data_ptr()
                if key not in c32["W"]:
                    c32["W"][key] = W.float()
                g = s * c32["W"][key]
            else:
                g = s * float(W)
        g = g.contiguous()
        w = torch.empty((k,) + grid, dtype=torch.float32, device=self.device)
        epi = dict(a=c32["afull"], b=c32["xi0"], out2=w)
        bt = dict(period=N, out=size, out2=N)
        if shift != 0.0:
            epi.update(d=D[0, xo:], shift=shift)
            bt["d"] = size
        _native.hartley_fused(Q[0, xo:], axes, m.c_h, x=g, epi=epi, convention=conv, shape=(k,) + grid, batch=bt)
        ga = torch.empty((k, B), dtype=torch.float32, device=self.device)
        m.jbins.scatter(w, ga, k)
        Q64 = torch.zeros((k, size), dtype=torch.float64, device=D.device)
        amp.native_vjp_batched(const, ga.double(), Q64, off, D64, shift)
        for o, n in segs:
            Q[:, o:o + n] = Q64[:, o:o + n]
        return Q

    # metric_flat(_batch) take qpart (data-space curvature partials, fused_cg)
    supports_quad = True

    def metric_flat(self, d, q, W, shift, qpart=None):
        """q = shift * d + J^T W J d on packed latent buffers (fused CG).
        qpart: partials of the quadratic form (J d).W(J d), from a middle W
        that supports it (W.quad_blocks)."""
        lay = self.layout
        dv = lay.views(d)
        s = self._times_t(dv)
        g = (W(s, qpart=qpart) if qpart is not None else W(s)) if callable(W) else s * W
        self._adjoint_t(g, lay.views(q), dv, shift)


class _CorrelatedFieldModel(Operator):
    """The fused correlated field.  `prefix` names the amplitude keys;
    `xi_prefix` (default: `prefix`) names 'xi' and 'zeromode', which the
    CorrelatedFieldMaker keys by the maker's prefix alone
    (correlated_fields.py:578-581,759,806)."""

    def __init__(self, target, harmonic_partner, offset_mean, offset_std, fluctuations, flexibility,
                 asperity, loglogavgslope, prefix, xi_prefix=None):
        xp = prefix if xi_prefix is None else xi_prefix
        self.amp = _AmplitudeModel(target, harmonic_partner, offset_std, fluctuations, flexibility,
                                   asperity, loglogavgslope, prefix, zm_prefix=xp)
        self.k_xi = xp + "xi"
        dom = dict(self.amp.domain_dict)
        dom[self.k_xi] = DomainTuple.make(harmonic_partner)
        self._domain = MultiDomain.make(dom)
        self._target = DomainTuple.make(target)
        self.harmonic_partner = harmonic_partner
        self.c_h = float(harmonic_partner.scalar_dvol)
        self.offset_mean = None if offset_mean is None else float(offset_mean)
        self.bins = BinIndex.get(self.amp.pspace.pindex, self.amp.B, config.device())
        # bin sums of the Jacobian adjoint: mirror-folded where the grid allows
        # (rounding-level parity); the value path keeps the bincount order
        self.jbins = BinIndex.get(self.amp.pspace.pindex, self.amp.B, config.device(), fold=True)
        self._layout = None
        self.amplitude = _AmplitudeOperator(self.amp)
        self.power_spectrum = _AmplitudeOperator(self.amp, power=2)

    @property
    def layout(self):
        if self._layout is None:
            self._layout = PackedLayout(self._domain)
        return self._layout

    def _value(self, lat):
        if _AMP_TORCH or not _AMP_NATIVE_FWD:
            a, c = self.amp.forward(lat)
        else:
            # amplitude and its linearisation constants on the device in one
            # pass (nft_amp_forward_batched), no host round trip
            c = self.amp.forward_native(lat)
            a = c.a[0]
        afull = torch.empty(self.harmonic_partner.shape, dtype=a.dtype, device=a.device)
        b = self.bins
        _native.bin_gather(a, b.pindex, afull, 1, b.npix, b.nbin, 1)
        s = _native.hartley_fused(torch.empty_like(afull), range(afull.ndim), self.c_h,
                                  pro=dict(a=afull, x=lat[self.k_xi].contiguous()),
                                  convention=hartley_convention_code())
        if self.offset_mean is not None:
            s = s + self.offset_mean
        return s, a, c, afull

    def apply(self, x):
        self._check_input(x)
        lin = x.jac is not None
        v = x.val if lin else x
        lat = {k: v[k].val for k in self._domain.keys()}
        s, a, c, afull = self._value(lat)
        res = Field(self._target, s)
        if not lin:
            return res
        jac = CFJacobian(self, c, a, afull, lat[self.k_xi])
        return x.new(res, jac)

    def __repr__(self):
        return f"SimpleCorrelatedField (fused) {self._target.shape}"


def SimpleCorrelatedField(target, offset_mean, offset_std, fluctuations, flexibility, asperity,
                          loglogavgslope, prefix="", harmonic_partner=None):
    """Same signature and latent keys as the reference
    (correlated_fields_simple.py:38-48)."""
    target = DomainTuple.make(target)
    if len(target) != 1:
        raise ValueError
    target = target[0]
    if harmonic_partner is None:
        harmonic_partner = target.get_default_codomain()
    else:
        target.check_codomain(harmonic_partner)
        harmonic_partner.check_codomain(target)
    for kk in (fluctuations, loglogavgslope):
        if len(kk) != 2:
            raise TypeError
    for kk in (offset_std, flexibility, asperity):
        if not (kk is None or len(kk) == 2):
            raise TypeError
    if flexibility is None and asperity is not None:
        raise ValueError
    return _CorrelatedFieldModel(target, harmonic_partner, offset_mean, offset_std, fluctuations,
                                 flexibility, asperity, loglogavgslope, prefix)
