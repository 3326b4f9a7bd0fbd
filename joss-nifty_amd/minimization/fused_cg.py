"""Fused conjugate gradient for sampling metrics  M = shift * 1 + J^T W J.

Same algorithm as ConjugateGradient.__call__ (src/minimization/
conjugate_gradient.py:48-126), on packed device vectors:

  q' = M' d                     fused model pipeline (core.metric_flat, M = shift + M')
  curv = d.(q' + shift d)       nft_cg_curv        -> sc[CURV]
  x -= a d ; r -= a (q' + s d)  nft_cg_update      -> sc[GAMMA]=r.r, x.r, x.b
  (every nreset-th step: r = M x - b exactly, nft_cg_residual)
The shift is applied element-wise inside the CG kernels (same arithmetic as
forming q = q' + shift d first), so the matvec never reads d a second time.
  host: guards + controller on (curv, gamma, value = (x.r - x.b)/2)
  d = max(0, g/g_prev) d + r    nft_cg_direction

All scalars stay on the device; one 16-double D2H read per iteration feeds the
host-side controller, exactly as the reference decides on host floats.
"""
import collections
import ctypes
import math
import os

import numpy as np
import torch

from .. import _native
from ..logger import logger
from ..packing import PackedLayout
from .conjugate_gradient import ConjugateGradient


USE_GRAPHS = os.environ.get("NFT_NO_GRAPH") is None
# iterations run eagerly before the loop body is captured: capturing costs a
# few ms, which short solves (NewtonCG directions, ~5 steps) never win back
GRAPH_AFTER = 4


def fusable_metric(A):
    """(core, W, shift) if A = shift*1 + Sandwich(fused core, W), else None."""
    from ..operators.sandwich_operator import SandwichOperator
    from ..operators.scaling_operator import ScalingOperator
    from ..operators.sum_operator import SumOperator
    if isinstance(A, SandwichOperator):
        if A.fused is None:
            return None
        return A.fused[0], A.fused[1], 0.0
    if isinstance(A, SumOperator):
        sand, shift = None, 0.0
        for op, neg in zip(A._ops, A._neg):
            if isinstance(op, SandwichOperator) and op.fused is not None and not neg and sand is None:
                sand = op
            elif isinstance(op, ScalingOperator) and complex(op._factor).imag == 0:
                shift += (-1 if neg else 1) * complex(op._factor).real
            else:
                return None
        if sand is None:
            return None
        return sand.fused[0], sand.fused[1], shift
    return None


class _State:
    """Energy-like view of the fused iterate for IterationControllers."""

    def __init__(self, value, gnorm, lazy):
        self._value = value
        self.gradient_norm = gnorm
        self._lazy = lazy

    @property
    def value(self):
        """the energy value (a callable is evaluated on first access)"""
        if callable(self._value):
            self._value = self._value()
        return self._value

    @property
    def position(self):
        return self._lazy()[0]

    @property
    def gradient(self):
        return self._lazy()[1]


def _stale():
    raise RuntimeError("CG energy value read after its iteration: the fused solve computes it "
                       "on demand only while the controller checks that iterate")


_CAPTURE_STREAM = None


def _capture(fn):
    """HIP graph of the launches fn makes.  Same capture as the
    torch.cuda.graph context manager, minus its device synchronize, gc.collect
    and empty_cache preamble (milliseconds per capture, paid per CG solve)."""
    global _CAPTURE_STREAM
    if _CAPTURE_STREAM is None:
        _CAPTURE_STREAM = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    cur = torch.cuda.current_stream()
    _CAPTURE_STREAM.wait_stream(cur)
    with torch.cuda.stream(_CAPTURE_STREAM):
        # thread-local capture: the background RNG thread may page-lock host
        # memory (random._pin) while the main thread captures
        g.capture_begin(capture_error_mode="thread_local")
        try:
            fn()
        finally:
            g.capture_end()
    cur.wait_stream(_CAPTURE_STREAM)
    return g


def _reads_value(ctl):
    """False for controllers that never look at the energy value
    (GradientNormController.check without a name and without an energy
    history, iteration_controllers.py:188-221).  A subclass may read it in an
    overridden check, so only the exact class qualifies.  (The decision trace
    reads values too, but from scalars recorded beside the iteration: it does
    not change which iteration runs.)"""
    from .iteration_controllers import GradientNormController
    return not (type(ctl) is GradientNormController and getattr(ctl, "_name", None) is None
                and getattr(ctl, "_history", None) is None)


# data-space curvature (nifty_amd.h "curvature from the data space"):
# shift * d.d summed while d is formed, (J d).W(J d) while the LOS forward
# reduces its lines -- no curvature pass over q and d (NFT_CURV_DATA=0: off)
CURV_DATA = os.environ.get("NFT_CURV_DATA", "1") != "0"
# ... also for value-driven controllers (energy deltas, gradient-norm
# tolerances; NFT_CURV_DATA_VALUE=1, off by default).  Equal in exact
# arithmetic, the data-space curvature rounds differently from the
# reference's d.(A d), and alpha = gamma / curv then no longer cancels d.r
# exactly in r -= alpha q: the CG energies leave the reference's trajectory
# (measured: demo64's AbsDelta(0.05) sampling CG agrees to 1e-12 for 12
# checks, then drifts -- 7e-7 relative at check 14 -- and stops after 24
# checks, the reference and its three 1e-15-perturbed runs after 28).
# Value-driven controllers therefore keep d.q, and with it the separate
# update pass (the carried update needs alpha before the adjoint).
CURV_DATA_VALUE = os.environ.get("NFT_CURV_DATA_VALUE", "0") == "1"


def _count_only(ctl):
    """True for a controller whose decisions depend on the iteration count
    alone (GradientNormController without tolerances)."""
    from .iteration_controllers import GradientNormController
    return (type(ctl) is GradientNormController and ctl._tol_abs_gradnorm is None
            and ctl._tol_rel_gradnorm is None)


def _count_silent(ctl):
    """a count-only controller that logs nothing and keeps no energy history:
    its checks read no energy"""
    return (_count_only(ctl) and ctl._name is None and ctl._iteration_limit is not None
            and getattr(ctl, "_history", None) is None)


class _CountOnlyState:
    """energy stand-in for the checks of a queued chunk: count-only
    controllers read nothing from it (any read fails loudly)"""

    def __getattr__(self, name):
        raise RuntimeError(f"count-only controller read energy.{name} in a queued CG chunk")


_COUNT_ONLY_STATE = _CountOnlyState()

# queued CG iterations between host reads (NFT_CG_CHUNK=0: one read per step)
CHUNK = os.environ.get("NFT_CG_CHUNK", "1") != "0"

def _quad_blocks(core, W, dtype, controllers=()):
    """partials per RHS of the metric's data-space quadratic form, or 0"""
    if not CURV_DATA or dtype not in (torch.float64, torch.float32):
        return 0
    if dtype == torch.float32 and not (hasattr(core, "phases_fp32") and core.phases_fp32(1)):
        # fp32 storage: the data-space curvature rides in the carried
        # iteration only (its amplitude keys in the two-phase kernels)
        return 0
    if not CURV_DATA_VALUE and not all(_count_only(c) for c in controllers):
        return 0
    if not getattr(core, "supports_quad", False):
        return 0
    if torch.is_tensor(W):
        # pointwise W (Gaussian / Poisson): the forward transform's epilogue
        f = getattr(core, "pointwise_quad_blocks", None)
        return int(f(W)) if f is not None else 0
    if not callable(W):
        return 0
    return int(getattr(W, "quad_blocks", 0) or 0)


def _worth_capturing(ctl, niter, min_left=4):
    """Capture only if the controller's iteration limit leaves at least
    `min_left` more iterations to replay (short solves, e.g. NewtonCG's first
    5-iteration direction, stay eager)."""
    lim = getattr(ctl, "_iteration_limit", None)
    return lim is None or lim - niter >= min_left


def fused_cg_or_none(energy, controller, nreset):
    from .quadratic_energy import QuadraticEnergy
    if type(energy) is not QuadraticEnergy:
        return None
    spec = fusable_metric(energy.metric)
    if spec is None:
        from ..lowering import lowered_metric
        lm = lowered_metric(energy.metric)
        if lm is None:
            return None
        spec = (lm, None, 0.0)
    core, W, shift = spec
    if energy.position.domain != core.domain or not core.device.type == "cuda":
        return None
    if mixed_precision(core, W):
        # fp32 storage runs in the batched loop (one right-hand side)
        return FusedCGBatch(core, W, shift, [controller], nreset).run([energy])[0]
    return FusedCG(core, W, shift, controller, nreset).run(energy)


def mixed_precision(core, W):
    """fp32 CG storage requested (config.set_cg_precision) and supported by
    the metric's native pipeline (else the solve stays fp64)."""
    from .. import config
    if config.cg_dtype() != torch.float32 or not getattr(core, "supports_fp32", False):
        return False
    return (not callable(W)) or getattr(W, "supports_fp32", False)


class FusedCG:
    """One fused solve: the batched loop (FusedCGBatch) with one right-hand
    side -- per RHS the batched kernels run exactly the single-solve
    arithmetic."""

    def __init__(self, core, W, shift, controller, nreset=20):
        self.core, self.W, self.shift = core, W, float(shift)
        self.controller = controller
        self.nreset = nreset
        self.layout = core.layout
        self.niter = 0

    def run(self, energy):
        cg = FusedCGBatch(self.core, self.W, self.shift, [self.controller], self.nreset)
        res = cg.run([energy])[0]
        self.niter = cg.niter
        self.path = getattr(cg, "path", None)
        return res


def batch_supported(core, W):
    """True if the fused metric can evaluate a batch of right-hand sides."""
    if not hasattr(core, "metric_flat_batch"):
        return False
    return (not callable(W)) or getattr(W, "supports_batch", False)


def fused_cg_batch_or_none(energies, controllers, nreset):
    """Solve several QuadraticEnergies with the SAME fused sampling metric in
    one batched loop (FusedCGBatch), or None if that does not apply."""
    from .quadratic_energy import QuadraticEnergy
    if len(energies) < 2 or any(type(e) is not QuadraticEnergy for e in energies):
        return None
    A = energies[0].metric
    if any(e.metric is not A for e in energies):
        return None
    if len({e._b is None for e in energies}) != 1:
        return None
    spec = fusable_metric(A)
    if spec is None:
        return None
    core, W, shift = spec
    if not batch_supported(core, W) or not core.device.type == "cuda":
        return None
    if any(e.position.domain != core.domain for e in energies):
        return None
    # at most MAX_BATCH right-hand sides per loop: the direction carried by
    # the folded prologue (and with it the rounding of the curvature) exists
    # for <= 8 items, so a rank holding 32 samples solves them in batches of
    # 8 with the per-RHS arithmetic of a rank holding 4 -- bit-identical KL
    # values on any rank count (test_mpi/test_kl.py:46-114,
    # tests/test_dist_ranks_gpu.py)
    out = []
    for i in range(0, len(energies), MAX_BATCH):
        out += FusedCGBatch(core, W, shift, controllers[i:i + MAX_BATCH], nreset).run(energies[i:i + MAX_BATCH])
    return out


MAX_BATCH = 8


# The grid segment's CG update carried by the adjoint transform's epilogue
# (data-space curvature: alpha is known before the adjoint): q's grid segment
# is neither stored nor read back (NFT_CG_CARRY=0: separate update pass)
_CARRY = os.environ.get("NFT_CG_CARRY", "1") != "0"
# ... and the grid segment's direction update inside the folded prologue
# (NFT_CG_CARRY_DIR=0: a separate direction pass)
_CARRY_DIR = os.environ.get("NFT_CG_CARRY_DIR", "1") != "0"
# the amplitude keys before and after the grid segment in one launch each for
# the direction and the update (nft_cg_*2_batched; NFT_CG_SEG2=0: two each)
_SEG2 = os.environ.get("NFT_CG_SEG2", "1") != "0"
# the amplitude keys' direction with the JVP and their update + the finalize
# with the VJP in the two-phase amplitude kernels (NFT_CG_AMP2=0: the
# separate direction / update / finalize launches)
_AMP2 = os.environ.get("NFT_CG_AMP2", "1") != "0"
# deferred iterate inside queued chunks of count-only solves
# (nft_hartley_fuse.lazy_*): the grid segment's directions go to ring slots,
# x is brought up to date once per chunk (nft_cg_lazy_flush, bitwise the
# per-step update); NFT_CG_LAZY=0: x updated every step
LAZY = os.environ.get("NFT_CG_LAZY", "1") != "0"


class _CarryIteration:
    """One CG iteration (k RHS, count-only controllers, no energy values)
    with the update of the grid segment G (the 'xi' key) inside the adjoint
    transform's last pass:

      dir + d.d partials | amplitude JVP | forward transform, W (LOS with the
      (R J d).C(R J d) partials), curvature fold | adjoint transform whose
      epilogue updates x, r on G and writes its r.r, x.r partials per tile |
      bin sums, amplitude VJP | update of the amplitude segments | finalize

    The per-element arithmetic is that of the separate update; the dot
    partials are [amplitude keys before G][G's tiles][keys after G], folded
    in that order.  The same for k = 1 (FusedCG) and k > 1 (FusedCGBatch)."""

    def __init__(self, lib, core, W, n, k, nq, shift):
        self.lib, self.core, self.W = lib, core, W
        self.n, self.k, self.nq, self.shift = n, k, nq, shift
        g0, g1 = core.grid_segment()
        self.g0 = g0
        tiles = core.cg_blocks(k)
        # the amplitude keys' direction / update carried by the two-phase
        # amplitude kernels (nft_amp2_*): partials [amplitude tiles][prologue
        # blocks] for d.d, [amplitude tiles] for r.r / x.r (each tile also
        # folds a slice of the grid epilogue's partials, GP)
        self.na = int(core.amp2_tiles(k)) if (_AMP2 and hasattr(core, "amp2_tiles")) else 0
        pb = core.dir_blocks(k) if (_CARRY_DIR and hasattr(core, "dir_blocks")) else 0
        if self.na and pb:
            dev = core.device
            self.tiles = tiles
            self.nbd = self.na + pb
            self.pro_blk0 = self.na
            self.PQ = torch.empty((k, self.nbd + nq), dtype=torch.float64, device=dev)
            self.UP = torch.empty((k, 2 * self.na), dtype=torch.float64, device=dev)
            self.GP = torch.empty((k, 3 * tiles), dtype=torch.float64, device=dev)
            return
        self.na = 0
        nb0 = int(lib.nft_cg_dd_blocks(g0)) if g0 > 0 else 0
        nb1 = int(lib.nft_cg_dd_blocks(n - g1)) if n > g1 else 0
        self.amp = [(o, e - o, blk) for (o, e), blk in (((0, g0), 0), ((g1, n), nb0 + tiles)) if e > o]
        self.tiles_blk0 = nb0
        self.nbtot = nb0 + tiles + nb1
        # the direction: the grid segment's inside the folded prologue when
        # available (d.d partials [keys before][prologue blocks][keys after]),
        # else one pass over the whole vector
        pb = core.dir_blocks(k) if (_CARRY_DIR and hasattr(core, "dir_blocks")) else 0
        if pb:
            self.dirs = [(o, e - o, blk) for (o, e), blk in (((0, g0), 0), ((g1, n), nb0 + pb)) if e > o]
            self.pro_blk0 = nb0
            self.nbd = nb0 + pb + nb1
        else:
            self.dirs = None
            self.nbd = int(lib.nft_cg_dd_blocks(n))
        dev = core.device
        self.PQ = torch.empty((k, self.nbd + nq), dtype=torch.float64, device=dev)
        self.UP = torch.empty((k, 3 * self.nbtot), dtype=torch.float64, device=dev)

    @staticmethod
    def supported(core, k, dtype=torch.float64):
        if not (_CARRY and hasattr(core, "cg_blocks") and core.cg_blocks(k) > 0):
            return False
        if dtype == torch.float64:
            return True
        # fp32 storage: only the two-phase amplitude flavour (its segment
        # kernels are dtype-generic; the separate segment passes are fp64)
        return (dtype == torch.float32 and _AMP2 and _CARRY_DIR and hasattr(core, "amp2_tiles")
                and core.amp2_tiles(k) > 0 and hasattr(core, "dir_blocks") and core.dir_blocks(k) > 0)

    def _call_amp2(self, X, Rr, D, Q, SC, lazy=None):
        core, lib = self.core, self.lib
        n, k, g0 = self.n, self.k, self.g0
        pstride = self.nbd + self.nq
        da = core.mv_amp_jvp_dir(D, Rr, SC, self.PQ, pstride, self.shift)
        pro_dir = dict(r=Rr[0, g0:], sc=SC, part=self.PQ, pstride=pstride, shift=self.shift, blk0=self.pro_blk0,
                       lazy=lazy)

        def fold():
            _native._check(lib.nft_fold_partials(_native.ptr(self.PQ), pstride, k,
                                                 ctypes.c_void_p(SC.data_ptr() + _native.CG_CURV * 8),
                                                 _native.CG_NSCALARS, _native.stream_ptr()))
        # the same call as arguments, for a W that carries it in its own launch
        fold.spec = (self.PQ, pstride, k, SC.data_ptr() + _native.CG_CURV * 8, _native.CG_NSCALARS)
        cg = dict(x=X[0, g0:], r=Rr[0, g0:], d=D[0, g0:], sc=SC, part=self.GP, stride=n, shift=self.shift,
                  nbtot=self.tiles, blk0=0, lazy=lazy)
        w = core.mv_grid(D, da, Q, self.W, 0.0, qpart=self.PQ[:, self.nbd:], after_w=fold, cg=cg,
                         pro_dir=pro_dir)
        core.mv_amp_vjp_cg(X, Rr, D, w, SC, self.UP, 2 * self.na, self.GP, 3 * self.tiles, self.tiles, self.tiles,
                           self.shift)

    def __call__(self, X, Rr, D, Q, SC, lazy=None):
        if self.na:
            return self._call_amp2(X, Rr, D, Q, SC, lazy)
        if lazy is not None:
            raise RuntimeError("the deferred iterate needs the two-phase amplitude kernels")
        core, lib = self.core, self.lib
        P = _native.ptr
        s_ = _native.stream_ptr()
        n, k = self.n, self.k
        Pv = ctypes.c_void_p
        pstride = self.nbd + self.nq
        pro_dir = None
        if self.dirs is None:
            _native._check(lib.nft_cg_direction_dd_batched(P(D), P(Rr), n, n, k, 0, P(SC), self.shift, P(self.PQ),
                                                           pstride, s_))
        elif _SEG2 and len(self.dirs) == 2 and self.dirs[0][0] == 0:
            (_, n1, _), (o2, n2, blk2) = self.dirs
            _native._check(lib.nft_cg_direction_dd2_batched(P(D), P(Rr), n1, o2, n2, n, k, 0, P(SC), self.shift,
                                                            P(self.PQ), blk2, pstride, s_))
        else:
            for o, ln, blk in self.dirs:
                _native._check(lib.nft_cg_direction_dd_batched(
                    Pv(D.data_ptr() + 8 * o), Pv(Rr.data_ptr() + 8 * o), ln, n, k, 0, P(SC), self.shift,
                    Pv(self.PQ.data_ptr() + 8 * blk), pstride, s_))
        if self.dirs is not None:
            pro_dir = dict(r=Rr[0, self.g0:], sc=SC, part=self.PQ, pstride=pstride, shift=self.shift,
                           blk0=self.pro_blk0)
        da = core.mv_amp_jvp(D)

        def fold():
            _native._check(lib.nft_fold_partials(P(self.PQ), self.nbd + self.nq, k,
                                                 ctypes.c_void_p(SC.data_ptr() + _native.CG_CURV * 8),
                                                 _native.CG_NSCALARS, _native.stream_ptr()))
        fold.spec = (self.PQ, self.nbd + self.nq, k, SC.data_ptr() + _native.CG_CURV * 8, _native.CG_NSCALARS)
        g0 = self.g0
        cg = dict(x=X[0, g0:], r=Rr[0, g0:], d=D[0, g0:], sc=SC, part=self.UP, stride=n, shift=self.shift,
                  nbtot=self.nbtot, blk0=self.tiles_blk0)
        w = core.mv_grid(D, da, Q, self.W, 0.0, qpart=self.PQ[:, self.nbd:], after_w=fold, cg=cg, pro_dir=pro_dir)
        core.mv_amp_vjp(D, w, Q, 0.0)
        if _SEG2 and len(self.amp) == 2 and self.amp[0][0] == 0:
            (_, n1, blk1), (o2, n2, blk2) = self.amp
            _native._check(lib.nft_cg_update_seg2_batched(P(X), P(Rr), P(D), P(Q), n1, blk1, o2, n2, blk2, n, k, 0,
                                                          self.shift, P(SC), P(self.UP), self.nbtot, s_))
        else:
            for o, ln, blk in self.amp:
                e = 8 * o
                _native._check(lib.nft_cg_update_seg_batched(
                    Pv(X.data_ptr() + e), Pv(Rr.data_ptr() + e), Pv(D.data_ptr() + e), Pv(Q.data_ptr() + e),
                    Pv(0), ln, n, k, 0, self.shift, P(SC), P(self.UP), self.nbtot, blk, s_))
        _native._check(lib.nft_cg_finalize_batched(P(self.UP), self.nbtot, k, P(SC), s_))


class FusedCGBatch(FusedCG):
    """k independent conjugate-gradient solves with the same metric, run in
    lock step: every iteration is ONE batched matvec (the LOS matrix, the FFT
    passes and the amplitude kernels each launched once for all right-hand
    sides) and ONE set of batched CG kernels.  Each right-hand side keeps its
    own scalars, guards and controller (a deep copy of the caller's, started
    on its own energy, exactly as a sequential solve would); once it stops,
    sc[DONE] freezes it on the device.  Per right-hand side the arithmetic is
    bitwise that of FusedCG (and of solving the systems one after another)."""

    def __init__(self, core, W, shift, controllers, nreset=20):
        super().__init__(core, W, shift, controllers[0], nreset)
        self.controllers = controllers

    def run(self, energies):
        k = len(energies)
        lay, core = self.layout, self.core
        n = lay.size
        dev = core.device
        dt = torch.float32 if mixed_precision(core, self.W) else torch.float64
        X = torch.zeros((k, n), dtype=dt, device=dev)
        Rr = torch.zeros_like(X)
        Bv = torch.zeros_like(X) if energies[0]._b is not None else None
        for j, e in enumerate(energies):
            lay.pack(e.position, out=X[j])
            lay.pack(e.gradient, out=Rr[j])
            if Bv is not None:
                lay.pack(e._b, out=Bv[j])
        A = energies[0].metric
        X, status = self.run_packed(X, Rr, Bv, energies)
        from .quadratic_energy import QuadraticEnergy
        results = []
        for j, e in enumerate(energies):
            st, moved = status[j]
            if moved is None:
                results.append((e, st))
            else:
                results.append((QuadraticEnergy(lay.unpack(X[j].double()), A, e._b,
                                                _grad=lay.unpack(Rr[j].double())), st))
        return results

    def run_packed(self, X, Rr, Bv, starts):
        """The batched loop on packed (k, n) buffers: X (iterates) and Rr
        (gradients A x - b) are updated in place, Bv is b (or None).
        `starts`: per RHS an energy-like object (value, gradient_norm) for the
        controller's start().  Returns (X, [(status, moved)]) -- moved is None
        for a RHS returned in its initial state.

        Once some right-hand sides have stopped, the live ones are compacted
        into smaller buffers (and a metric restricted to them, core.subset)
        when their controllers allow a few more iterations: the lock-step
        batch then stops paying matvecs for frozen rows.  Per RHS the
        arithmetic does not depend on the batch size (bitwise)."""
        k0 = X.shape[0]
        lay = self.layout
        n = lay.size
        results = [None] * k0
        active = []
        for j, (e, ctl) in enumerate(zip(starts, self.controllers)):
            st = ctl.start(e)
            if st != ctl.CONTINUE:
                results[j] = (st, None)
            else:
                active.append(j)
        if not active:
            return X, results
        core = self.core
        dev = core.device
        NS = _native.CG_NSCALARS
        lib = _native.load()
        dt = _native.dtype_code(X.dtype)
        P = _native.ptr
        sh = self.shift
        full_X, full_Rr = X, Rr
        rows = list(range(k0))          # buffer position -> original RHS index
        pos = {j: j for j in rows}      # original RHS index -> buffer position
        SC = torch.zeros((k0, NS), dtype=torch.float64, device=dev)
        host = torch.zeros((k0, NS), dtype=torch.float64).pin_memory()
        ws = _native.workspace(k0 * lib.nft_reduce_workspace(n), dev, "cgb")

        def chk(st):
            _native._check(st)

        def finish(j, status):
            results[j] = (status, True)
            SC[pos[j], _native.CG_DONE] = 1.0

        for j in range(k0):
            if results[j] is not None:
                SC[j, _native.CG_DONE] = 1.0
        chk(lib.nft_dot_batched(P(Rr), P(Rr), n, n, k0, dt, P(SC[:, _native.CG_GAMMA:]), NS, P(ws),
                                _native.stream_ptr()))
        host.copy_(SC)
        for j in list(active):
            g = float(host[j, _native.CG_GAMMA])
            if np.isnan(g):
                logger.error("Error: ConjugateGradient: previous_gamma==NaN")
                results[j] = (self.controllers[j].ERROR, None)
            elif g == 0:
                results[j] = (self.controllers[j].CONVERGED, None)
            if results[j] is not None:
                SC[j, _native.CG_DONE] = 1.0
                active.remove(j)
        if not active:
            return X, results

        # The energy value 0.5 (x.r - x.b) needs x.b: the update kernel sums
        # it while streaming b, or -- in the carried iteration, which has no
        # separate update -- one dot beside the iteration (reads x and b,
        # changes nothing).  Value-blind controllers (GradientNormController
        # without a name) get it on demand only.  The decision trace records
        # each step's scalars from the device (HIST), so tracing changes
        # neither the iteration nor the chunking.
        from . import trace
        tracing = trace.active()
        need_value = tracing or any(_reads_value(c) for c in self.controllers)
        nq = _quad_blocks(core, self.W, X.dtype, self.controllers)
        D = Rr.clone()
        st = {}
        # per step: gamma, x.r, x.b of every RHS (trace replay of queued chunks)
        HIST = torch.zeros((k0, self.nreset + 1, 3), dtype=torch.float64, device=dev) if tracing else None
        hsel = torch.tensor([_native.CG_GAMMA, _native.CG_XR, _native.CG_XB], device=dev)

        def setup(k):
            """the k-dependent iteration state (partials, carried iteration)"""
            st.clear()
            st["Q"] = torch.zeros_like(X)
            st["AX"] = None
            st["split"] = None
            carry = bool(nq) and _CarryIteration.supported(core, k, X.dtype)
            # x.b from the update kernel (b streamed) or from a dot beside
            # the carried iteration
            st["Bu"] = Bv if (need_value and not carry) else None
            st["xbdot"] = carry and need_value and Bv is not None
            if nq:
                st["nbd"] = int(lib.nft_cg_dd_blocks(n))
                st["PQ"] = torch.empty((k, st["nbd"] + nq), dtype=torch.float64, device=dev)
                if carry:
                    st["split"] = _CarryIteration(lib, core, self.W, n, k, nq, sh)
            # the deferred iterate: count-only chunks of the carried iteration
            # with the two-phase amplitude kernels (nothing reads x.r or x
            # between the chunk's host reads)
            st["lazy"] = None
            spl = st["split"]
            ring_bytes = self.nreset * k * n * X.element_size()
            if (LAZY and chunkable0 and HIST is None and not need_value and isinstance(spl, _CarryIteration)
                    and spl.na and getattr(core, "lazy_ok", lambda k: False)(k)
                    and ring_bytes <= 0.5 * torch.cuda.mem_get_info(dev)[0]):
                g0 = spl.g0
                ring = torch.empty((self.nreset, k, n), dtype=X.dtype, device=dev)
                alpha = torch.empty((k, self.nreset), dtype=torch.float64, device=dev)
                st["lazy"] = dict(ring=ring[0, 0, g0:], sstride=k * n, alpha=alpha, nslot=self.nreset,
                                  buf=ring, g0=g0, ng=core.grid_size())
        chunkable0 = CHUNK and all(_count_silent(self.controllers[j]) for j in active)
        setup(k0)

        def record():
            """HIST[r, ITER % (nreset + 1)] = (gamma, x.r, x.b) of every live
            RHS after this step (device ops only: graph-capturable)"""
            if HIST is None:
                return
            k = X.shape[0]
            idx = (SC[:, _native.CG_ITER].long() % HIST.shape[1])
            rows = torch.arange(k, device=dev)
            live = (SC[:, _native.CG_DONE] == 0.0).unsqueeze(1)
            cur = HIST[rows, idx]
            HIST[rows, idx] = torch.where(live, SC.index_select(1, hsel), cur)

        def body(with_dir, lazy=False):
            s_ = _native.stream_ptr()
            k = X.shape[0]
            split, Q, Bu = st["split"], st["Q"], st["Bu"]
            if st["xbdot"]:
                # the first (direction-less) step runs the separate update:
                # it streams b for x.b
                Bu = Bv
            if with_dir and isinstance(split, _CarryIteration):
                split(X, Rr, D, Q, SC, st["lazy"] if lazy else None)
                if st["xbdot"]:
                    chk(lib.nft_dot_batched(P(X), P(Bv), n, n, k, dt, P(SC[:, _native.CG_XB:]), NS, P(ws), s_))
                record()
                return
            if with_dir and nq:
                # curvature from the data space: shift * d.d partials while d is
                # formed, (J d).W(J d) partials in the LOS forward reduce
                nbd, PQ = st["nbd"], st["PQ"]
                chk(lib.nft_cg_direction_dd_batched(P(D), P(Rr), n, n, k, dt, P(SC), sh, P(PQ), nbd + nq, s_))
                core.metric_flat_batch(D, Q, self.W, 0.0, qpart=PQ[:, nbd:])
                chk(lib.nft_fold_partials(P(PQ), nbd + nq, k, P(SC[:, _native.CG_CURV:]), NS, s_))
            else:
                if with_dir:
                    chk(lib.nft_cg_direction_batched(P(D), P(Rr), n, n, k, dt, P(SC), s_))
                core.metric_flat_batch(D, Q, self.W, 0.0)
                chk(lib.nft_cg_curv_batched(P(D), P(Q), n, n, k, dt, sh, P(SC), P(ws), s_))
            chk(lib.nft_cg_update_batched(P(X), P(Rr), P(D), P(Q), P(Bu), n, n, k, dt, sh, P(SC), P(ws), s_))
            record()

        def compact():
            """restrict the buffers, the scalars and the metric to the live RHS"""
            nonlocal X, Rr, Bv, D, SC, host, core, rows, pos, graph, lgraph, eager, iter_seen, HIST
            keep = sorted(pos[j] for j in active)
            if X is not full_X:
                idx = torch.tensor(rows, device=dev)
                full_X.index_copy_(0, idx, X)
                full_Rr.index_copy_(0, idx, Rr)
            kt = torch.tensor(keep, device=dev)
            X, Rr, D, SC = (t.index_select(0, kt) for t in (X, Rr, D, SC))
            if Bv is not None:
                Bv = Bv.index_select(0, kt)
            if HIST is not None:
                HIST = HIST.index_select(0, kt)
            host = torch.zeros((len(keep), NS), dtype=torch.float64).pin_memory()
            iter_seen = iter_seen[keep]
            rows = [rows[p] for p in keep]
            pos = {j: p for p, j in enumerate(rows)}
            sub = getattr(core, "subset", None)
            if sub is not None:
                # per-RHS metrics (NewtonCG directions): the live rows' metric
                core = sub(rows)
            setup(len(rows))
            # one eager iteration warms the new batch size's caches, then the
            # loop body is captured again
            graph = None
            lgraph = None
            eager = 1

        # a core without `subset` applies one metric to every row; a per-RHS
        # metric compacts only if it can restrict itself (subset not None)
        can_compact = COMPACT and getattr(core, "subset", _shared) is not None
        graph = None
        lgraph = None
        eager = 0
        ii = 0
        first = True
        # several graph replays per host read while every live controller only
        # counts (_count_silent); a decision trace replays the queued steps'
        # checks with their recorded scalars (HIST)
        chunkable = CHUNK and all(_count_silent(self.controllers[j]) for j in active)
        # which iteration this solve runs (diagnostics: tools/demo_profile.py)
        self.path = ("carry" if isinstance(st["split"], _CarryIteration) else "quad" if nq else "plain") + \
            ("+chunk" if chunkable else "")
        self.compactions = 0
        iter_seen = np.zeros(k0)
        # value-driven controllers read the host every iteration and their
        # solves are short (NewtonCG directions: ~7 iterations): the loop body
        # stays eager (the one-off capture measured slower: demo step 858 ->
        # 834 ms eager, Newton-direction CG 788 -> 747 us per RHS iteration)
        eager_only = any(_reads_value(c) for c in self.controllers)
        while active:
            if chunkable and graph is not None and ii + 2 < self.nreset:
                m = min(min(self.controllers[j]._iteration_limit - self.controllers[j]._itcount for j in active),
                        self.nreset - 1 - ii)
                if m > 1:
                    lz = st["lazy"]
                    if lz is not None:
                        # the chunk with the deferred iterate: ring slots from 0,
                        # x brought up to date before the host read
                        if lgraph is None:
                            lgraph = _capture(lambda: body(True, lazy=True))
                        SC[:, _native.CG_LAZY] = 0.0

                        def flush(m=m, lz=lz):
                            g0 = lz["g0"]
                            _native.cg_lazy_flush(X[0, g0:], D[0, g0:], lz["ring"], lz["sstride"], lz["alpha"],
                                                  lz["nslot"], m, lz["ng"], n, X.shape[0])
                        iter_seen = self._chunk(lgraph, m, SC, host, iter_seen, active, finish, pos, HIST, flush)
                    else:
                        iter_seen = self._chunk(graph, m, SC, host, iter_seen, active, finish, pos, HIST)
                    STATS["chunks"] += 1
                    STATS["chunk_iters"] += m
                    if isinstance(st["split"], _CarryIteration):
                        STATS["carry_iters"] += m
                    ii += m
                    if can_compact and _worth_compacting(self.controllers, active, len(rows)):
                        compact()
                        self.compactions += 1
                        STATS["compactions"] += 1
                    continue
            self.niter += 1
            ConjugateGradient.iterations_total += len(active)
            ii += 1
            sp = _native.stream_ptr()
            if ii < self.nreset:
                if not first and isinstance(st["split"], _CarryIteration):
                    STATS["carry_iters"] += 1
                if first or not USE_GRAPHS or eager_only or self.niter <= GRAPH_AFTER or eager > 0:
                    body(not first)
                    eager = max(0, eager - 1)
                elif graph is None:
                    if any(_worth_capturing(self.controllers[j], self.niter) for j in active):
                        graph = _capture(lambda: body(True))
                        graph.replay()
                    else:
                        body(True)
                else:
                    graph.replay()
                first = False
            else:
                k = X.shape[0]
                Q, Bu = st["Q"], st["Bu"]
                if not first:
                    chk(lib.nft_cg_direction_batched(P(D), P(Rr), n, n, k, dt, P(SC), sp))
                first = False
                core.metric_flat_batch(D, Q, self.W, 0.0)
                chk(lib.nft_cg_curv_batched(P(D), P(Q), n, n, k, dt, sh, P(SC), P(ws), sp))
                gp = SC[:, _native.CG_GAMMA].clone()
                chk(lib.nft_cg_update_batched(P(X), P(Rr), P(D), P(Q), P(Bu), n, n, k, dt, sh, P(SC), P(ws), sp))
                if st["AX"] is None:
                    st["AX"] = torch.zeros_like(X)
                AX = st["AX"]
                core.metric_flat_batch(X, AX, self.W, 0.0)
                flag = SC[:, _native.CG_FLAG].clone()
                chk(lib.nft_cg_residual_batched(P(Rr), P(AX), P(X), P(Bv), n, n, k, dt, sh, P(SC), P(ws), sp))
                live = SC[:, _native.CG_DONE] == 0.0
                SC[:, _native.CG_GPREV] = torch.where(live, gp, SC[:, _native.CG_GPREV])
                SC[:, _native.CG_FLAG] = torch.where(live, flag, SC[:, _native.CG_FLAG])
                record()
                ii = 0
            host.copy_(SC, non_blocking=True)
            torch.cuda.current_stream().synchronize()
            h = host.numpy()
            iter_seen = h[:, _native.CG_ITER].copy()
            # x.b of this step on the device: streamed by the update kernel,
            # the dot beside the carried iteration, or the residual refresh
            xb_dev = st["Bu"] is not None or st["xbdot"] or ii == 0
            for j in list(active):
                ctl = self.controllers[j]
                p = pos[j]
                hj = h[p]
                status = None
                if hj[_native.CG_FLAG] != 0.0:
                    curv = hj[_native.CG_CURV]
                    if np.isnan(curv):
                        logger.error("Error: ConjugateGradient: curv==NaN")
                    elif curv == 0.:
                        logger.error("Error: ConjugateGradient: curv==0.")
                    else:
                        logger.error("Error: ConjugateGradient: alpha<0.")
                    status = ctl.ERROR
                else:
                    gamma = float(hj[_native.CG_GAMMA])
                    if np.isnan(gamma):
                        logger.error("Error: ConjugateGradient: gamma==NaN")
                        status = ctl.ERROR
                    elif gamma < 0:
                        logger.error("Positive definiteness of preconditioner violated!")
                        status = ctl.ERROR
                    elif gamma == 0:
                        status = ctl.CONVERGED
                    else:
                        cache = {}

                        def lazy(p=p, cache=cache, Xc=X, Rc=Rr):
                            if "v" not in cache:
                                cache["v"] = (lay.unpack(Xc[p].double()), lay.unpack(Rc[p].double()))
                            return cache["v"]
                        xr, xb = float(hj[_native.CG_XR]), float(hj[_native.CG_XB])
                        if not xb_dev and Bv is not None:
                            # x.b was not accumulated by the update kernel
                            def value(p=p, xr=xr, Xc=X, Bc=Bv):
                                xbj = float(torch.dot(Xc[p].double(), Bc[p].double()))
                                return 0.5 * (xr - xbj)
                        else:
                            value = 0.5 * (xr - xb)
                        state = _State(value, math.sqrt(gamma), lazy)
                        sts = ctl.check(state)
                        if callable(state._value):
                            # not read during the check: the buffers move on with the
                            # next iteration, so a later read would see another iterate
                            state._value = _stale
                        if sts != ctl.CONTINUE:
                            status = sts
                if status is not None:
                    finish(j, status)
                    active.remove(j)
            if active and can_compact and _worth_compacting(self.controllers, active, len(rows)):
                compact()
                self.compactions += 1
                STATS["compactions"] += 1
        if X is not full_X:
            idx = torch.tensor(rows, device=dev)
            full_X.index_copy_(0, idx, X)
            full_Rr.index_copy_(0, idx, Rr)
        return full_X, results

    def _chunk(self, graph, m, SC, host, iter_seen, active, finish, pos, HIST=None, flush=None):
        """m queued iterations (graph replays) and one host read.  A terminal
        step (guard tripped, gamma zero / negative / NaN) freezes its RHS on
        the device (NFT_CG_DONE = 2, with NFT_CG_AUTO set); every RHS's
        controller then sees exactly the checks a one-step loop would have
        made, in order -- count-only controllers read nothing but the count."""
        NS = _native
        SC[:, NS.CG_AUTO] = 1.0
        for _ in range(m):
            graph.replay()
        if flush is not None:
            flush()
        SC[:, NS.CG_AUTO] = 0.0
        self.niter += m
        host.copy_(SC, non_blocking=True)
        hh = HIST.cpu().numpy() if HIST is not None else None
        torch.cuda.current_stream().synchronize()
        h = host.numpy()
        for j in list(active):
            ctl = self.controllers[j]
            hj = h[pos[j]]
            p = int(round(hj[NS.CG_ITER] - iter_seen[pos[j]]))
            ConjugateGradient.iterations_total += p
            frozen = hj[NS.CG_DONE] == 2.0
            status = None
            for t in range(p - 1 if frozen else p):
                state = _COUNT_ONLY_STATE
                if hh is not None:
                    # the step's recorded scalars (decision trace)
                    g_, xr_, xb_ = hh[pos[j], (int(round(iter_seen[pos[j]])) + t + 1) % hh.shape[1]]
                    state = _State(0.5 * (float(xr_) - float(xb_)), math.sqrt(float(g_)), lambda: None)
                st = ctl.check(state)
                if st != ctl.CONTINUE:
                    if t != p - 1:
                        raise RuntimeError("count-only controller stopped inside a queued chunk")
                    status = st
            if frozen:
                if hj[NS.CG_FLAG] != 0.0:
                    curv = hj[NS.CG_CURV]
                    if np.isnan(curv):
                        logger.error("Error: ConjugateGradient: curv==NaN")
                    elif curv == 0.:
                        logger.error("Error: ConjugateGradient: curv==0.")
                    else:
                        logger.error("Error: ConjugateGradient: alpha<0.")
                    status = ctl.ERROR
                else:
                    gamma = float(hj[NS.CG_GAMMA])
                    if np.isnan(gamma):
                        logger.error("Error: ConjugateGradient: gamma==NaN")
                        status = ctl.ERROR
                    elif gamma < 0:
                        logger.error("Positive definiteness of preconditioner violated!")
                        status = ctl.ERROR
                    else:
                        status = ctl.CONVERGED
            if status is not None:
                finish(j, status)
                active.remove(j)
        return h[:, NS.CG_ITER].copy()


def _shared(rows):
    raise AssertionError("a shared metric is not restricted")


# which iterations the batched loop ran (tests assert the timed path ran)
STATS = collections.Counter()


# compaction of the lock-step batch once right-hand sides stop
# (NFT_CG_COMPACT=0: frozen rows ride along to the end)
COMPACT = os.environ.get("NFT_CG_COMPACT", "1") != "0"


def _worth_compacting(controllers, active, k, min_left=3):
    """fewer live RHS than rows, and some live controller allows at least
    `min_left` more iterations (a compaction re-captures the loop body)"""
    if len(active) >= k:
        return False
    for j in active:
        ctl = controllers[j]
        lim = getattr(ctl, "_iteration_limit", None)
        if lim is None or lim - getattr(ctl, "_itcount", 0) >= min_left:
            return True
    return False
