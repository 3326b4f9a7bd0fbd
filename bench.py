"""Benchmark: geoVI sample drawing on a 2048^2 CorrelatedField (MI355X).

Workload (BASELINE.json metric "geoVI samples-drawn/sec + CG-iter/sec, 2048^2
CorrelatedField"; config C3 of SURVEY.md §8(d)): 2048x2048 RGSpace
SimpleCorrelatedField with the getting_started_3 parameters, signal
sigmoid(cf), LOSResponse with 16384 random lines of sight, Gaussian noise
var 1e-3, synthetic mock data (seed 27).  One step = one draw_samples call
(geoVI: linear MGVI solve + NewtonCG refinement per sample, mirrored pairs)
at a fixed expansion point followed by the sampled-KL value/gradient mean
(the single all-reduce over ranks).  Controllers are fixed-iteration so GPU
and CPU do identical work.  Samples are sharded over ranks with shareRange:
per-GPU work is fixed (weak scaling).

Prints ONE JSON line (rank 0).  See DESIGN.md §Measurement for the roofline
and CPU-baseline definitions.
"""
import argparse
import collections
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CF_ARGS = dict(offset_mean=0, offset_std=(1e-3, 1e-6), fluctuations=(1., 0.8),
               loglogavgslope=(-3., 1), flexibility=(2, 1.), asperity=(0.5, 0.4))
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak, /opt/skills/guides/MI355X_MICROARCH.md

# BASELINE.json configs (SURVEY.md §8(d) synthetic inputs); `pairs`: mirrored
# pairs per GPU = the config's n_samples over its GPU count, per-GPU share
# measured on one GPU (C2 4, C4 2, C5 4 pairs)
CONFIGS = {
    "C2": dict(shape=(1024, 1024), lik="poisson", pairs=4, cg="fp64",
               desc="1024^2 SimpleCorrelatedField, exp, Poisson counts, geoVI mirrored"),
    "C3": dict(shape=(2048, 2048), lik="los", pairs=4, cg="fp64",
               desc="2048^2 SimpleCorrelatedField, sigmoid, LOSResponse, Gaussian 1e-3, geoVI mirrored"),
    "C4": dict(shape=(512, 512, 512), lik="gauss", pairs=2, cg="fp64",
               desc="512^3 SimpleCorrelatedField (no asperity), GeometryRemover, Gaussian 0.01, geoVI mirrored"),
    "C5": dict(shape=(4096, 4096), lik="gauss", pairs=4, cg="fp32",
               desc="4096^2 SimpleCorrelatedField, GeometryRemover, Gaussian 0.01, geoVI mirrored, "
                    "fp32-storage / fp64-accumulated CG"),
}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=2)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--config", choices=sorted(CONFIGS), default="C3",
                   help="BASELINE.json workload (the headline is C3; C2 / C4 / C5 are the other GPU configs' "
                        "per-GPU shares)")
    p.add_argument("--size", type=int, default=None, help="grid edge (default: the config's)")
    p.add_argument("--nlos", type=int, default=16384)
    # C3 (BASELINE.json configs[2]): geoVI n_samples=8 mirrored pairs across 2
    # GPUs -> 4 pairs (8 samples) per GPU, held fixed per GPU (weak scaling)
    p.add_argument("--samples-per-gpu", type=int, default=None, help="mirrored pairs per GPU (default: the config's)")
    p.add_argument("--lin-iters", type=int, default=100)
    p.add_argument("--newton-iters", type=int, default=2)
    p.add_argument("--newton-cg-max", type=int, default=50)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-pairs", type=int, default=1, help="mirrored pairs in the timed CPU oracle draw")
    p.add_argument("--cpu-lin-iters", type=int, default=None,
                   help="C2/C4/C5: linear-CG iterations of the timed CPU oracle run (default C2 200, C5 15, C4 2)")
    p.add_argument("--no-demo", action="store_true", help="skip the demo-controller line")
    p.add_argument("--deterministic-allreduce", action="store_true")
    p.add_argument("--backend", choices=["nccl", "gloo", "none"], default=None,
                   help="process-group backend (default: nccl = RCCL on a GPU, also at N = 1; gloo on CPU "
                        "at N > 1; none: no communicator, N = 1 only)")
    a = p.parse_args()
    cfg = CONFIGS[a.config]
    if a.size is None:
        a.size = cfg["shape"][0]
    if a.samples_per_gpu is None:
        a.samples_per_gpu = cfg["pairs"]
    if a.cpu_lin_iters is None:
        # about 10 s of host work on the GPU box's cores (C2 ~23, C5 ~1.3,
        # C4 ~0.15 oracle CG iterations per second there)
        a.cpu_lin_iters = {"C2": 200, "C5": 15, "C4": 2}.get(a.config, 3)
    return a


def launch_workers(n):
    """`--gpus N` without a launcher: start N ranks of this script (one per
    GPU, LOCAL_RANK = RANK) as child processes -- this process never touches
    the GPU -- forward rank 0's line and exit with the worst status."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    codes = [p.wait() for p in procs]
    bad = [c for c in codes if c != 0]
    return bad[0] if bad else 0


def setup_dist(backend=None):
    """One process per GPU.  On a GPU the process group is RCCL ("nccl")
    whatever the world size: at N = 1 a world-size-1 group on an in-process
    store, so the KL-mean all-reduce of the timed step runs through the same
    RCCL call as at N = 8 (`--backend none` at N = 1: no communicator)."""
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    lrank = int(os.environ.get("LOCAL_RANK", "0"))
    if torch.cuda.is_available():
        torch.cuda.set_device(lrank % torch.cuda.device_count())
    backend = backend or ("nccl" if torch.cuda.is_available() else ("gloo" if ws > 1 else "none"))
    if backend == "none":
        if ws > 1:
            raise SystemExit("bench.py: --backend none needs WORLD_SIZE 1")
        return ws, rank, lrank, False
    import torch.distributed as dist
    if ws > 1:
        dist.init_process_group(backend)
    else:
        dist.init_process_group(backend, store=dist.HashStore(), rank=0, world_size=1)
    return ws, rank, lrank, True


def barrier_sync(ws):
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    import torch.distributed as dist
    if dist.is_initialized():
        import torch.distributed as dist
        dist.barrier()
    if torch.cuda.is_available():
        torch.cuda.synchronize()


def build_problem(ift, n, nlos, config="C3"):
    """(cf, R or None, likelihood energy, expansion point, LOS geometry or
    None) of a BASELINE config, synthetic mock data from seed 27"""
    cfg = CONFIGS[config]
    if cfg["lik"] != "los":
        shape = (n,) * len(cfg["shape"])
        sp = ift.RGSpace(shape)
        cf = ift.SimpleCorrelatedField(sp, **(dict(CF_ARGS, asperity=None) if len(shape) == 3 else CF_ARGS))
        ift.random.push_sseq_from_seed(27)
        mock = ift.from_random(cf.domain, "normal")
        if cfg["lik"] == "poisson":
            sig = cf.exp()
            lam = sig(mock).val.cpu().numpy()
            counts = ift.random.current_rng().poisson(lam).astype(np.int64)
            pos = 0.1 * ift.from_random(cf.domain, "normal")
            lh = ift.PoissonianEnergy(ift.makeField(sp, counts)) @ sig
        else:
            R = ift.GeometryRemover(sp)
            N = ift.ScalingOperator(R.target, 0.01, np.float64)
            data = R(cf(mock)) + N.draw_sample()
            pos = 0.1 * ift.from_random(cf.domain, "normal")
            lh = ift.GaussianEnergy(data, inverse_covariance=N.inverse) @ (R @ cf)
        ift.random.pop_sseq()
        return cf, None, lh, pos, None
    sp = ift.RGSpace((n, n))
    cf = ift.SimpleCorrelatedField(sp, **CF_ARGS)
    signal = ift.sigmoid(cf)
    ift.random.push_sseq_from_seed(27)
    rng = ift.random.current_rng()
    starts = list(rng.random((nlos, 2)).T)
    ends = list(rng.random((nlos, 2)).T)
    R = ift.LOSResponse(sp, starts=starts, ends=ends)
    sr = R(signal)
    N = ift.ScalingOperator(R.target, 1e-3, np.float64)
    mock = ift.from_random(sr.domain, "normal")
    data = sr(mock) + N.draw_sample()
    pos = 0.1 * ift.from_random(sr.domain, "normal")
    ift.random.pop_sseq()
    lh = ift.GaussianEnergy(data, inverse_covariance=N.inverse) @ sr
    return cf, R, lh, pos, (starts, ends)


def probe_setup(ift, lh, pos, k):
    """The linear geoVI sampling metric exactly as draw_samples builds it
    (kl_energies.py:147-153, 1 + J^T J of the likelihood's transformation),
    its fused core, and k random right-hand-side buffers laid out like
    FusedCGBatch's (k, latent) blocks."""
    from nifty_amd.minimization.fused_cg import fusable_metric, mixed_precision
    dtype, f_lh = lh.get_transformation()
    fl = f_lh(ift.Linearization.make_var(pos))
    met = (ift.SandwichOperator.make(fl.jac, ift.ScalingOperator(f_lh.target, 1., dtype))
           + ift.ScalingOperator(fl.domain, 1., float))
    spec = fusable_metric(met)
    assert spec is not None, "bench metric did not fuse"
    core, W, shift = spec
    lay = core.layout
    # probe vectors: device normals in the packed layout (padding zero); the
    # values do not matter for timing, so the host PCG64 stream is not used
    # (C5: fp32 storage, as FusedCGBatch.run allocates them)
    dt = torch.float32 if mixed_precision(core, W) else torch.float64
    X = torch.zeros((3 * k, lay.size), dtype=dt, device=lay.device)
    g = torch.Generator(device=lay.device)
    g.manual_seed(1234)
    for key, o, n in zip(lay.keys, lay.offsets, lay.sizes):
        X[:, o:o + n] = torch.randn((3 * k, n), dtype=torch.float64, device=lay.device, generator=g).to(dt)
    return core, W, shift, X


_CARRY_CACHE = {}


def cg_iteration(lib, core, W, shift, bufs, k):
    """One batched CG iteration as FusedCGBatch.body runs it inside the timed
    loop: direction, batched matvec, curvature, update (+ their folds); the
    curvature from the data space when the metric supports it (fused_cg)."""
    from nifty_amd import _native
    from nifty_amd.minimization.fused_cg import _quad_blocks
    X, R, D, Q, SC, ws = bufs
    n = X.shape[1]
    P = _native.ptr
    s_ = _native.stream_ptr()
    dt = _native.dtype_code(X.dtype)
    nq = _quad_blocks(core, W, X.dtype)
    from nifty_amd.minimization.fused_cg import _CarryIteration
    if nq and _CarryIteration.supported(core, k, X.dtype):
        # FusedCGBatch's iteration: the grid segment's update inside the
        # adjoint transform's epilogue (no b stream: count-only controllers)
        key = (id(core), k, n)
        it = _CARRY_CACHE.get(key)
        if it is None:
            it = _CARRY_CACHE[key] = _CarryIteration(lib, core, W, n, k, nq, shift)
        it(X, R, D, Q, SC)
        return
    if nq:
        nbd = int(lib.nft_cg_dd_blocks(n))
        PQ = torch.empty((k, nbd + nq), dtype=torch.float64, device=X.device)
        _native._check(lib.nft_cg_direction_dd_batched(P(D), P(R), n, n, k, dt, P(SC), shift, P(PQ), nbd + nq, s_))
        core.metric_flat_batch(D, Q, W, 0.0, qpart=PQ[:, nbd:])
        _native._check(lib.nft_fold_partials(P(PQ), nbd + nq, k, P(SC[:, _native.CG_CURV:]), _native.CG_NSCALARS,
                                             s_))
    else:
        _native._check(lib.nft_cg_direction_batched(P(D), P(R), n, n, k, dt, P(SC), s_))
        core.metric_flat_batch(D, Q, W, 0.0)
        _native._check(lib.nft_cg_curv_batched(P(D), P(Q), n, n, k, dt, shift, P(SC), P(ws), s_))
    _native._check(lib.nft_cg_update_batched(P(X), P(R), P(D), P(Q), 0, n, n, k, dt, shift, P(SC), P(ws), s_))


def cg_iteration_wall(lib, core, W, shift, bufs, k, reps=20):
    """Wall time of one batched CG iteration exactly as the timed loop runs it:
    FusedCGBatch's iteration body captured in a HIP graph and replayed
    `reps` times between two events.  Every replay continues the CG from the
    previous one (the probe's scalars never freeze a right-hand side:
    CG_AUTO is 0 and the metric is positive definite), so every replay does
    the full update; the scalars are restored once afterwards."""
    from nifty_amd import _native
    from nifty_amd.minimization import fused_cg
    X, R, D, Q, SC, ws = bufs
    n = X.shape[1]
    SC0 = SC.clone()

    def body():
        cg_iteration(lib, core, W, shift, bufs, k)
    assert float(SC[:, _native.CG_AUTO].abs().sum()) == 0.0
    for _ in range(2):
        body()
    torch.cuda.synchronize()
    g = fused_cg._capture(body)
    g.replay()
    torch.cuda.synchronize()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    for _ in range(reps):
        g.replay()
    t1.record()
    torch.cuda.synchronize()
    if float(SC[:, _native.CG_DONE].abs().sum()) != 0.0:
        raise RuntimeError("cg_iteration_wall: a right-hand side froze during the replays")
    SC.copy_(SC0)
    return t0.elapsed_time(t1) * 1e3 / reps


def lazy_spec(core, k, n, dtype, nreset=20):
    """the deferred-iterate buffers of FusedCGBatch's count-only chunks
    (fused_cg.LAZY) for the probe's carried iteration, or None where the
    timed loop does not defer x"""
    from nifty_amd.minimization import fused_cg
    it = _CARRY_CACHE.get((id(core), k, n))
    if not (fused_cg.LAZY and it is not None and it.na and getattr(core, "lazy_ok", lambda k: False)(k)):
        return None
    ring = torch.empty((nreset, k, n), dtype=dtype, device=core.device)
    alpha = torch.empty((k, nreset), dtype=torch.float64, device=core.device)
    return dict(ring=ring[0, 0, it.g0:], sstride=k * n, alpha=alpha, nslot=nreset, buf=ring, g0=it.g0,
                ng=core.grid_size())


LAZY_CHUNK = 19   # count-only chunk length between residual refreshes (nreset 20)


def lazy_chunk(lib, core, W, shift, bufs, k, lz, m):
    """m eager steps of the carried iteration with the deferred iterate from
    ring slot 0, then the flush (the chunk of the timed loop, uncaptured)"""
    from nifty_amd import _native
    X, R, D, Q, SC, ws = bufs
    n = X.shape[1]
    it = _CARRY_CACHE[(id(core), k, n)]
    SC[:, _native.CG_LAZY] = 0.0
    for _ in range(m):
        it(X, R, D, Q, SC, lz)
    g0 = lz["g0"]
    _native.cg_lazy_flush(X[0, g0:], D[0, g0:], lz["ring"], lz["sstride"], lz["alpha"], lz["nslot"], m, lz["ng"], n, k)


def cg_iteration_lazy_wall(lib, core, W, shift, bufs, k, lz, m=LAZY_CHUNK):
    """Wall time per iteration of a count-only chunk as FusedCGBatch runs it
    with the deferred iterate: m replays of the captured iteration body
    (directions into ring slots, x untouched) and the flush that brings x up
    to date, between two events, divided by m (nreset = 20: chunks of 19)."""
    from nifty_amd import _native
    from nifty_amd.minimization import fused_cg
    X, R, D, Q, SC, ws = bufs
    n = X.shape[1]
    it = _CARRY_CACHE[(id(core), k, n)]
    SC0 = SC.clone()

    def body():
        it(X, R, D, Q, SC, lz)

    def flush(steps):
        g0 = lz["g0"]
        _native.cg_lazy_flush(X[0, g0:], D[0, g0:], lz["ring"], lz["sstride"], lz["alpha"], lz["nslot"], steps,
                              lz["ng"], n, k)
    SC[:, _native.CG_LAZY] = 0.0
    body()
    flush(1)
    torch.cuda.synchronize()
    g = fused_cg._capture(body)
    SC[:, _native.CG_LAZY] = 0.0
    torch.cuda.synchronize()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    for _ in range(m):
        g.replay()
    flush(m)
    t1.record()
    torch.cuda.synchronize()
    if float(SC[:, _native.CG_DONE].abs().sum()) != 0.0:
        raise RuntimeError("cg_iteration_lazy_wall: a right-hand side froze during the replays")
    SC.copy_(SC0)
    return t0.elapsed_time(t1) * 1e3 / m


def byte_model(cf, R, k, n_lat, dir_carried=False, pairs=False, s=8, lazy_m=0):
    """Algorithmic bytes per launch (every operand array counted once per
    launch; arrays shared by the k right-hand sides -- amplitude, xi0, pindex,
    the LOS matrix and its scales -- once).  s: bytes per value of the CG
    vectors and grid operands (8 fp64; 4 for C5's fp32 storage -- complex
    values 2s, indices 4 bytes, LOS weights 4 bytes either way).  DESIGN.md §3."""
    shape = cf.target.shape
    N = int(np.prod(shape))
    Hh = N // shape[-1] * (shape[-1] // 2 + 1)
    B = cf.amp.B
    if R is not None:
        P = R._plan_np
        nnz = int(P["box_ent"][-1])
        nseg = int(P["nseg"])
        nbox = int(P["nbox"])
        nlos = R.target.shape[0]
    else:   # no LOS pair (C2, C4, C5): its rows are not used
        nnz = nseg = nbox = nlos = 0
    # the Jacobian adjoint's bin sums run over the mirror-folded cell (N_f)
    fold = getattr(getattr(cf, "jbins", None), "fold", None)
    Nf = fold["nf"] if fold else N
    return {
        # prologue A*x + xi0*dA[pindex]: x (k), A, xi0, pindex, dA (k); half spectrum out (k)
        "fft_r2c+pro": s * k * N + s * N + s * N + 4 * N + s * k * B + 2 * s * k * Hh,
        # batched prologue as its own pass: x (k), A, xi0, pindex, dA (k) -> u (k)
        "pro_batch": s * k * N + s * N + s * N + 4 * N + s * k * B + s * k * N,
        # folded: the cell's bin (N_f), dA gathered per mirror class; no pindex
        "pro_fold": s * k * N + s * N + s * N + 4 * Nf + s * k * B + s * k * N,
        # ... carrying the grid segment's CG direction: d, r in, d out (k)
        "pro_fold+dir": 3 * s * k * N + s * N + s * N + 4 * Nf + s * k * B + s * k * N,
        # ... fused with the R2C row pass (nft_pro_r2c.hip): u is never stored;
        # the half spectrum out (k) instead
        "pro_r2c+dir": 3 * s * k * N + s * N + s * N + 4 * Nf + s * k * B + 2 * s * k * Hh,
        "fft_r2c": s * k * N + 2 * s * k * Hh,
        "fft_c2c": 2 * 2 * s * k * Hh,
        "fft_unpack": 2 * s * k * Hh + s * k * N,
        # + the pointwise weight (shared by the k items) and the per-tile
        # quadratic-form partials (negligible): W*h out (k)
        "fft_unpack+quad": 2 * s * k * Hh + s * N + s * k * N,
        # epilogue: out = A*v (k), out2 = xi0*v (k), reads A, xi0
        "fft_unpack+epi": 2 * s * k * Hh + 2 * s * N + s * k * N + s * k * (Hh if pairs else N),
        # 5 B per nonzero, 12 B segment descriptors, x (k) and the column scale, partials (k)
        "los_fwd_items": 5 * nnz + 12 * nseg + s * (k + 1) * N + 8 * k * nseg,   # fp64 partials
        "los_fwd_reduce": 8 * k * nseg + s * k * nlos,
        "los_adj_boxes": 5 * nnz + 4 * nseg + 2 * 257 * nbox + s * (k + 1) * N,
        # mirror fold: w (k) in -- the half grid of point-mirror pair sums
        # with epi_out2_pairs -- folded cell (k) out
        "bin_fold": s * k * (Hh if pairs else N) + s * k * Nf,
        # perm over the cell, cell values (k), bin offsets, sums (k)
        "bin_scatter": 4 * Nf + s * k * Nf + 4 * B + s * k * B,
        "cg_dir_kernel": 3 * s * k * n_lat,
        # whole vector, or (direction carried by the prologue) two launches
        # over the keys before / after the grid segment, half their bytes each
        "cg_dir_dd": 3 * s * k * (n_lat if not dir_carried else (n_lat - N) // 2),
        "curv_partial": 2 * s * k * n_lat,
        # x, r, d, q in; x, r out (b is not streamed: the probe passes none,
        # and the sampling CG's value-blind controllers skip it too)
        "cg_update_kernel": 6 * s * k * n_lat,
        # the amplitude keys' update (the grid segment's rides in the
        # epilogue): two launches, the keys before and after the grid
        # segment; per launch the model carries half of their bytes
        "cg_update_seg": 3 * s * k * (n_lat - N),
        # both amplitude segments in one launch (nft_cg_*2_batched)
        "cg_update_seg2": 6 * s * k * (n_lat - N),
        "cg_dir_dd2": 3 * s * k * (n_lat - N),
        # unpack + the grid segment's CG update: half spectrum (k), A, xi0;
        # x, r, d in (k), x, r and w = xi0*v out (k) -- q is not stored;
        # with the deferred iterate (lazy_m steps per chunk) r, d in and r
        # out: x is left to the flush
        "fft_unpack+cg": 2 * s * k * Hh + 2 * s * N + (3 if lazy_m else 5) * s * k * N + s * k * (Hh if pairs else N),
        # the flush of a chunk: its lazy_m direction slots and x in, x and
        # the last direction out (k)
        "cg_lazy_flush": (lazy_m + 3) * s * k * N,
    }


def kernel_probe(ift, cf, R, lh, pos, k, reps=10):
    """Per-kernel durations of the batched CG iteration of the timed loop
    (k right-hand sides = the local linear solves of one draw_samples call),
    measured with HIP events recorded on the launch stream before every
    hot-path launch (nft_prof_*; the same kernels with the same arguments as
    inside the timed region, run eagerly because events cannot be timed inside
    a HIP graph).

    Returns ({label: {"launches": per iteration, "avg_us", "bytes": algorithmic
    bytes per launch, "gbs"}}, iteration summary)."""
    from nifty_amd import _native
    lib = _native.load()
    core, W, shift, XS = probe_setup(ift, lh, pos, k)
    n_lat = XS.shape[1]
    X, Rr, D = XS[:k].clone(), XS[k:2 * k].clone(), XS[2 * k:].clone()
    Q = torch.zeros_like(X)
    SC = torch.zeros((k, _native.CG_NSCALARS), dtype=torch.float64, device=X.device)
    SC[:, _native.CG_GAMMA] = 1.0
    SC[:, _native.CG_GPREV] = 1.0
    ws = _native.workspace(k * lib.nft_reduce_workspace(n_lat), X.device, "cgb")
    bufs = (X, Rr, D, Q, SC, ws)
    for _ in range(3):
        cg_iteration(lib, core, W, shift, bufs, k)
    torch.cuda.synchronize()
    lz = lazy_spec(core, k, n_lat, X.dtype)
    # keep the GPU busy while the probe launches are queued, so that the
    # events bracket kernels and not host enqueue gaps
    torch.cuda._sleep(200_000_000)
    lazy_m = 0
    with _native.LaunchProfile() as prof:
        if lz is None:
            for _ in range(reps):
                cg_iteration(lib, core, W, shift, bufs, k)
        else:
            # the timed loop's count-only chunk: 19 steps with the deferred
            # iterate, then its flush (launches per iteration: 1 / 19 for it)
            lazy_m = reps = LAZY_CHUNK
            lazy_chunk(lib, core, W, shift, bufs, k, lz, lazy_m)
    acc = {}
    for lab, ms in prof.records:
        a = acc.setdefault(lab, [0, 0.0])
        a[0] += 1
        a[1] += ms
    from nifty_amd.minimization import fused_cg
    dcar = bool(fused_cg._CARRY and fused_cg._CARRY_DIR and getattr(core, "dir_blocks", lambda k: 0)(k) > 0
                and _CARRY_CACHE)
    model = byte_model(cf, R, k, n_lat, dir_carried=dcar, pairs=bool(getattr(core, "_pairs", lambda k: 0)(k)),
                       s=X.element_size(), lazy_m=lazy_m)
    out = {}
    tot_us, tot_b = 0.0, 0
    for lab, (cnt, tot) in acc.items():
        avg = tot / cnt * 1e3
        by = model.get(lab)
        per = cnt // reps if cnt % reps == 0 else round(cnt / reps, 4)
        out[lab] = {"launches": per, "avg_us": round(avg, 2), "bytes": by,
                    "gbs": round(by / (avg * 1e-6) / 1e9, 1) if by else None}
        tot_us += tot * 1e3 / reps
        tot_b += (by or 0) * per
    wall_us = cg_iteration_wall(lib, core, W, shift, bufs, k)
    timing = "HIP graph replay of the iteration body"
    eager_x_us = None
    if lz is not None:
        # the timed loop's count-only chunks defer x (fused_cg.LAZY): their
        # per-iteration time, flush included
        eager_x_us = wall_us
        wall_us = cg_iteration_lazy_wall(lib, core, W, shift, bufs, k, lz)
        timing = ("HIP graph replay of a 19-iteration count-only chunk with the deferred iterate and its flush "
                  "(as the timed loop runs it), per iteration")
    # the per-launch byte model of the kernel table (every operand array once
    # per launch), over the same iteration time -- a bandwidth, not a second
    # roofline fraction: the line's fraction is roofline.frac (SURVEY §8(d)
    # bytes) beside roofline.traffic_frac (PMC bytes)
    it = {"rhs": k, "us_per_iteration": round(wall_us, 1), "timing": timing,
          "us_sum_of_launches": round(tot_us, 1), "launch_model_bytes": tot_b,
          "launch_model_gbs": round(tot_b / (wall_us * 1e-6) / 1e9, 1)}
    if eager_x_us is not None:
        it["us_per_iteration_x_every_step"] = round(eager_x_us, 1)
    return out, it


def load_pmc(label, config="C3"):
    """Per-launch HBM traffic of `label` from the committed PMC summary of
    the config (tools/pmc_probe.py under rocprofv3 --pmc FETCH_SIZE /
    WRITE_SIZE, calibrated as MI355X_MICROARCH.md §HBM prescribes), or None."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json" if config == "C3" else f"pmc_traffic_{config}.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    e = d.get("kernels", {}).get(label)
    return None if e is None else e.get("traffic_bytes")


def survey_bytes_per_iteration(cf, R, config="C3"):
    """SURVEY.md §8(d)'s algorithmic bytes of one linear-CG iteration of one
    right-hand side: N [(4d + 13) s + 8] for the CF metric + CG update (s = 8
    fp64, 4 for C5's fp32 storage), + 2 s N for Poisson's per-pixel weights,
    + 2 s N + 16 nnz for the LOS pair."""
    cfg = CONFIGS[config]
    N = int(np.prod(cf.target.shape))
    d = len(cf.target.shape)
    s = 4 if cfg["cg"] == "fp32" else 8
    by = N * ((4 * d + 13) * s + 8)
    if cfg["lik"] == "poisson":
        by += 2 * s * N
    if R is not None:
        by += 2 * s * N + 16 * int(R._plan_np["box_ent"][-1])
    return by


def bytes_model_text(config):
    cfg = CONFIGS[config]
    s = "4" if cfg["cg"] == "fp32" else "8"
    extra = {"poisson": " + 2sN (Poisson weights)", "los": " + 2sN + 16 nnz (LOS pair)"}.get(cfg["lik"], "")
    return f"SURVEY §8(d): k x (N[(4d+13)s+8]{extra}), s = {s}, d = {len(cfg['shape'])}"


def roofline_of(kp, cgit, cf, R, config="C3"):
    """roofline of the FFT+CG matvec the north star targets: one batched CG
    iteration (k right-hand sides) as a unit -- §8(d) bytes x k over the
    measured iteration time (HIP-graph replay of the iteration body, timed
    with events on its stream; the per-kernel table beside it comes from
    single-stream launches bracketed by events).
    traffic: PMC HBM bytes of the same launches (profiles/pmc_traffic.json),
    when every kernel of the iteration has an entry."""
    k = cgit["rhs"]
    by = survey_bytes_per_iteration(cf, R, config) * k
    us = cgit["us_per_iteration"]
    ach = by / (us * 1e-6) / 1e9
    traffic = 0
    for lab, e in kp.items():
        t = load_pmc(lab, config)
        if t is None:
            traffic = None
            break
        traffic += t * e["launches"]
    dom = max(kp, key=lambda lab: kp[lab]["avg_us"] * kp[lab]["launches"])
    # the rocprof-achieved bandwidth north_star asks for: PMC HBM bytes of the
    # iteration's launches over the same iteration time
    tfrac = None if traffic is None else round(traffic / (us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)
    return {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_frac": tfrac,
            "traffic_source": "profiles/" + ("pmc_traffic.json" if config == "C3" else f"pmc_traffic_{config}.json"),
            "kernel": "cg_iteration",
            "rhs": k, "avg_launch_us": us, "algorithmic_bytes_per_launch": by,
            "bytes_model": bytes_model_text(config),
            "largest_kernel": {"label": dom, "avg_us": kp[dom]["avg_us"], "launches": kp[dom]["launches"],
                               "gbs": kp[dom]["gbs"]}}


def cpu_baseline(args, lat0, R, n, pairs):
    """The oracle's geoVI draw (oracle/geovi.py: numpy + scipy.fft on all host
    cores, scipy.sparse LOS) of `pairs` mirrored pair(s) with the bench's
    controllers, timed from the seed spawn to the last residual."""
    import scipy.fft
    from oracle.cf import CFOracle
    from oracle.geovi import LOSWhitened, draw_geovi
    from oracle.sampling import GradNormCtl
    ncores = os.cpu_count() or 1
    o = CFOracle((n, n), **CF_ARGS)
    rows, cols, w = R.coo
    lh = LOSWhitened(o, rows, cols, w, R.target.shape[0], 1e-3)
    with scipy.fft.set_workers(ncores):
        t = time.perf_counter()
        res, iters = draw_geovi(lh, lat0, pairs, True, np.random.SeedSequence(1000),
                                lambda: GradNormCtl(iteration_limit=args.lin_iters), args.newton_iters,
                                max_cg=args.newton_cg_max)
        el = time.perf_counter() - t
    return 2 * pairs / el, iters / el, ncores, el, iters


def cpu_baseline_config(args, lat0, n, gpu_iters, gpu_samples):
    """C2 / C4 / C5: a TIMED bounded run of the oracle (oracle/sampling.py's
    conjugate_gradient on oracle/geovi.py's sampling metric 1 + J0^T J0,
    numpy + scipy.fft on all host cores): `args.cpu_lin_iters` linear-CG
    iterations of one right-hand side b ~ N(0, 1) from x0 = 0, timed after one
    warm-up metric application (FFT plans, caches); the full geoVI draw would
    take minutes to hours on the host.  value = the measured CPU rate in CG
    iterations per second (compare with the line's cg_iter_per_s: GPU CG
    iterations of all right-hand sides per second); the samples/s the CPU
    would reach at that rate for the GPU run's CG iterations per sample is a
    separately labelled projection."""
    import scipy.fft
    from oracle.cf import CFOracle
    from oracle.geovi import GaussWhitened, PoissonWhitened
    from oracle.sampling import GradNormCtl, axpy, conjugate_gradient
    cfg = CONFIGS[args.config]
    shape = (n,) * len(cfg["shape"])
    ncores = os.cpu_count() or 1
    o = CFOracle(shape, **(dict(CF_ARGS, asperity=None) if len(shape) == 3 else CF_ARGS))
    lh = PoissonWhitened(o) if cfg["lik"] == "poisson" else GaussWhitened(o, 0.01)
    keys = sorted(lat0)

    def M(v):
        g = lh.vjp(lat0, lh.jvp(lat0, v))
        return axpy(1., v, {k: np.reshape(g[k], np.shape(v[k])) for k in keys})
    rng = np.random.default_rng(1000)
    b = {k: rng.normal(0., 1., np.shape(lat0[k])) for k in keys}
    zero = {k: np.zeros_like(b[k]) for k in keys}
    with scipy.fft.set_workers(ncores):
        M(b)
        t = time.perf_counter()
        _, _, iters = conjugate_gradient(M, zero, b, GradNormCtl(iteration_limit=args.cpu_lin_iters))
        el = time.perf_counter() - t
    cgps = iters / el
    return {"value": round(cgps, 4), "unit": "CG-iter/s", "cores": ncores, "kind": "port",
            "compare_with": "cg_iter_per_s (GPU CG iterations of all right-hand sides per second)",
            "projected_samples_per_s": round(gpu_samples / (gpu_iters / cgps), 6),
            "projection": (f"NOT measured: the GPU run's {gpu_iters} CG iterations for {gpu_samples} samples "
                           f"at the measured CPU rate"),
            "sample": (f"TIMED: oracle linear CG (oracle/sampling.py conjugate_gradient on oracle/geovi.py's "
                       f"sampling metric; numpy, scipy.fft workers={ncores}) on the same "
                       f"{'x'.join(map(str, shape))} problem, one right-hand side, {iters} iteration(s) "
                       f"(+ the initial metric application) in {el:.1f} s after one warm-up application")}


def demo_step(ift, lh, pos, nsamp, comm, R=None):
    """One step with SURVEY §8(d)'s demo controllers: sampling
    AbsDeltaEnergyController(0.05, iteration_limit=100), NewtonCG(
    AbsDeltaEnergyController(0.5, convergence_level=2, iteration_limit=15))."""
    H = ift.StandardHamiltonian(lh, ift.AbsDeltaEnergyController(deltaE=0.05, iteration_limit=100))
    mini = ift.NewtonCG(ift.AbsDeltaEnergyController(deltaE=0.5, convergence_level=2, iteration_limit=15))
    ift.random.push_sseq_from_seed(2000)

    def one():
        sl = ift.draw_samples(pos, H, mini, nsamp, True, comm=comm)
        ift.SampledKLEnergyClass(sl, H, [], None, True)
    # one untimed step first (its batch sizes' graph captures and caches),
    # then one timed step of the same seeded stream
    one()
    barrier_sync(1)
    it0 = ift.ConjugateGradient.iterations_total
    t = time.perf_counter()
    one()
    barrier_sync(1)
    el = time.perf_counter() - t
    cg_iters = int(ift.ConjugateGradient.iterations_total - it0)
    newton = newton_roofline(ift, one, R)
    ift.random.pop_sseq()
    return {"samples_per_s": round(2 * nsamp / el, 4), "ms_per_step": round(el * 1e3, 1),
            "cg_iters": cg_iters, "warmup_steps": 1,
            "controllers": "sampling AbsDelta(0.05, 100); NewtonCG(AbsDelta(0.5, convergence_level=2, 15))",
            "newton_cg": newton}


def newton_roofline(ift, one, R):
    """The geoVI Newton-direction CG of the demo controllers on the roofline:
    one more (untimed) demo step with every batched solve of the lowered
    Newton metric timed (device synchronised around it), SURVEY §8(d) bytes
    per right-hand-side iteration with the matvec term and the LOS pair
    doubled (M = B^T B, B = 1 + J0^T L0^T L J: 4 transforms, 2 LOS pairs):
    N [2 ((4d+3) s + 8) + 10 s] + 2 (2 s N + 16 nnz)."""
    from nifty_amd.minimization import fused_cg
    if not torch.cuda.is_available():
        return None
    rec = [0, 0, 0.0]
    paths = collections.Counter()
    orig = fused_cg.FusedCGBatch.run_packed

    def run_packed(self, X, Rr, Bv, starts):
        if type(self.core).__name__ != "_MetricCore":
            return orig(self, X, Rr, Bv, starts)
        torch.cuda.synchronize()
        it0 = ift.ConjugateGradient.iterations_total
        t = time.perf_counter()
        r = orig(self, X, Rr, Bv, starts)
        torch.cuda.synchronize()
        rec[0] += 1
        rec[1] += ift.ConjugateGradient.iterations_total - it0
        rec[2] += time.perf_counter() - t
        paths[getattr(self, "path", "?")] += 1
        return r
    fused_cg.FusedCGBatch.run_packed = run_packed
    try:
        one()
    finally:
        fused_cg.FusedCGBatch.run_packed = orig
    if rec[1] == 0:
        return None
    if R is None:
        return None
    shp = R.domain[0].shape
    N, s, d = int(np.prod(shp)), 8, len(shp)
    nnz = int(R._plan_np["box_ent"][-1])
    per = N * (2 * ((4 * d + 3) * s + 8) + 10 * s) + 2 * (2 * s * N + 16 * nnz)
    gbs = per * rec[1] / rec[2] / 1e9
    return {"solves": rec[0], "rhs_iters": rec[1], "ms": round(rec[2] * 1e3, 1),
            "us_per_rhs_iter": round(rec[2] * 1e6 / rec[1], 1), "bytes_per_rhs_iter": per,
            "achieved": round(gbs, 1), "peak": 8000.0, "unit": "GB/s", "frac": round(gbs / 8000.0, 4),
            "path": "separate direction / curvature d.q / update passes (value-driven controllers keep the "
                    "reference's d.q); solves by fused_cg path: " + ", ".join(f"{p} {n}" for p, n in sorted(paths.items()))}


class _TimedComm:
    """the communicator with its collectives timed (device-synchronised
    before and after each): the KL-mean all-reduce of one extra, untimed step"""

    def __init__(self, comm):
        self._c = comm
        self.calls = []

    def __getattr__(self, name):
        return getattr(self._c, name)

    def allreduce_tensor_(self, t):
        torch.cuda.synchronize() if t.is_cuda else None
        t0 = time.perf_counter()
        self._c.allreduce_tensor_(t)
        torch.cuda.synchronize() if t.is_cuda else None
        self.calls.append((time.perf_counter() - t0, t.numel() * t.element_size()))
        return t


def _json_stdout():
    """stdout carries ONE JSON line: RCCL prints a banner ("RCCL version :
    ...") to fd 1 when its first communicator comes up, and libraries may
    print too -- everything written to fd 1 from here on goes to stderr, the
    result line to a duplicate of the original stdout"""
    sys.stdout.flush()
    out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    return out


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_workers(args.gpus))
    result_out = _json_stdout()
    if int(os.environ.get("WORLD_SIZE", "1")) != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but the launcher's WORLD_SIZE is {os.environ.get('WORLD_SIZE')}",
              file=sys.stderr, flush=True)
        sys.exit(2)
    ws, rank, lrank, has_pg = setup_dist(args.backend)
    import nifty_amd as ift
    ift.config.set_device(f"cuda:{lrank % torch.cuda.device_count()}" if torch.cuda.is_available() else "cpu")
    if args.deterministic_allreduce:
        ift.utilities.DETERMINISTIC_ALLREDUCE = True
    comm = ift.TorchComm() if has_pg else None
    n = args.size
    cfg = CONFIGS[args.config]
    if cfg["cg"] == "fp32":
        ift.config.set_cg_precision("fp32")
    cf, R, lh, pos, _ = build_problem(ift, n, args.nlos, args.config)
    H = ift.StandardHamiltonian(lh, ift.GradientNormController(iteration_limit=args.lin_iters))
    mini = ift.NewtonCG(ift.GradientNormController(iteration_limit=args.newton_iters),
                        max_cg_iterations=args.newton_cg_max)
    nsamp = args.samples_per_gpu * ws

    # one seeded stream for the whole run, each step spawning its sample seeds
    # from it -- the way optimize_kl drives SampledKLEnergy (optimize_kl.py,
    # kl_energies.py:131)
    ift.random.push_sseq_from_seed(1000)

    def step(i):
        sl = ift.draw_samples(pos, H, mini, nsamp, True, comm=comm)
        kl = ift.SampledKLEnergyClass(sl, H, [], None, True)
        return kl

    for i in range(args.warmup):
        step(i)
    barrier_sync(ws)
    it0 = ift.ConjugateGradient.iterations_total
    t0 = time.perf_counter()
    for i in range(args.steps):
        kl = step(args.warmup + i)
    barrier_sync(ws)
    el = time.perf_counter() - t0
    iters = ift.ConjugateGradient.iterations_total - it0
    dist_info = None
    if has_pg:
        import torch.distributed as dist
        dev = "cuda" if torch.cuda.is_available() and dist.get_backend() != "gloo" else "cpu"
        t = torch.tensor([el, float(iters)], dtype=torch.float64, device=dev)
        dist.all_reduce(t[0:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(t[1:2], op=dist.ReduceOp.SUM)
        el, iters = float(t[0]), float(t[1])
        # every rank drew its share and holds the same KL: a rank that
        # disagrees fails the run (non-zero exit on every rank)
        per_rank = [int(c) for c in comm.allgather(kl.samples.n_local_samples)]
        vals = comm.allgather(float(kl.value))
        # the KL-mean all-reduce of one extra, untimed step, timed on its own
        tc = _TimedComm(comm)
        sl = ift.draw_samples(pos, H, mini, nsamp, True, comm=tc)
        ift.SampledKLEnergyClass(sl, H, [], None, True)
        ar = tc.calls
        ar_ms = comm.allgather(sum(c[0] for c in ar) * 1e3)
        dist_info = {"backend": dist.get_backend(), "samples_per_rank": per_rank,
                     "kl_allreduce": {"calls": len(ar), "bytes": sum(c[1] for c in ar),
                                      "ms_max_over_ranks": round(max(ar_ms), 4),
                                      "timing": "one extra untimed step, device-synchronised around each call"}}
        bad = []
        if sum(per_rank) != 2 * nsamp:
            bad.append(f"samples per rank {per_rank} do not add up to {2 * nsamp}")
        if any(v != vals[0] for v in vals):
            bad.append(f"KL values differ over ranks: {vals}")
        if bad:
            if rank == 0:
                print("bench.py: rank mismatch: " + "; ".join(bad), file=sys.stderr, flush=True)
            dist.destroy_process_group()
            sys.exit(3)
    samples = 2 * nsamp * args.steps
    sps = samples / el
    cgps = iters / el
    kp, cgit = kernel_probe(ift, cf, R, lh, pos, args.samples_per_gpu) if torch.cuda.is_available() \
        else (None, None)
    roof = roofline_of(kp, cgit, cf, R, args.config) if kp else None
    demo = None
    if not args.no_demo and torch.cuda.is_available() and args.config == "C3":
        demo = demo_step(ift, lh, pos, nsamp, comm, R)
    cpu = None
    if rank == 0 and ws == 1 and not args.no_cpu_baseline and args.config != "C3":
        lat0 = {k: pos[k].val.cpu().numpy() for k in cf.domain.keys()}
        cpu = cpu_baseline_config(args, lat0, n, int(iters), samples)
    elif rank == 0 and ws == 1 and not args.no_cpu_baseline:
        lat0 = {k: pos[k].val.cpu().numpy() for k in cf.domain.keys()}
        sps_c, cgps_c, ncores, cel, citers = cpu_baseline(args, lat0, R, n, args.cpu_pairs)
        cpu = {"value": round(sps_c, 6), "unit": "samples/s", "cores": ncores, "kind": "port",
               "cg_iter_per_s": round(cgps_c, 4),
               "sample": (f"oracle geoVI draw (oracle/geovi.py: numpy, scipy.fft workers={ncores}, "
                          f"scipy.sparse LOS) of {args.cpu_pairs} mirrored pair(s) on the same {n}^2 LOS "
                          f"problem with the bench's controllers: {2 * args.cpu_pairs} samples, {citers} CG "
                          f"iterations in {cel:.1f} s")}
    if rank == 0:
        if args.config == "C3":
            wl = (f"C3: {n}x{n} SimpleCorrelatedField, sigmoid, LOSResponse({args.nlos}), "
                  f"Gaussian 1e-3, geoVI mirrored, {args.samples_per_gpu} pair(s)/GPU, "
                  f"lin CG {args.lin_iters} it, NewtonCG {args.newton_iters} it "
                  f"(inner CG <= {args.newton_cg_max})")
            metric = "geoVI samples-drawn/sec (+ CG-iter/sec), 2048^2 CorrelatedField"
        else:
            shp = "x".join([str(n)] * len(cfg["shape"]))
            wl = (f"{args.config}: {cfg['desc'].replace(str(cfg['shape'][0]), str(n), 1)} "
                  f"({shp}), {args.samples_per_gpu} pair(s)/GPU, lin CG {args.lin_iters} it, "
                  f"NewtonCG {args.newton_iters} it (inner CG <= {args.newton_cg_max})")
            metric = f"geoVI samples-drawn/sec (+ CG-iter/sec), {args.config} per-GPU share"
        line = {"metric": metric,
                "value": round(sps, 6), "unit": "samples/s", "n_gpus": ws, "steps": args.steps,
                "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 3),
                "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
                "dtype": "f32 (fp64-accumulated CG)" if cfg["cg"] == "fp32" else "f64",
                "data": "synthetic",
                "config": {"workload": wl, "global_batch": samples // args.steps, "parallelism": f"sample-dp{ws}"},
                "cg_iter_per_s": round(cgps, 3), "cg_iters": int(iters),
                "roofline": roof, "cpu_baseline": cpu, "demo_controllers": demo,
                "cg_iteration": cgit, "kernels": kp, "distributed": dist_info}
        print(json.dumps(line), file=result_out, flush=True)
    if has_pg:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
