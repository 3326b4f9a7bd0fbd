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


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=2)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--size", type=int, default=2048)
    p.add_argument("--nlos", type=int, default=16384)
    p.add_argument("--samples-per-gpu", type=int, default=1, help="mirrored pairs per GPU")
    p.add_argument("--lin-iters", type=int, default=100)
    p.add_argument("--newton-iters", type=int, default=2)
    p.add_argument("--newton-cg-max", type=int, default=50)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-iters", type=int, default=20)
    p.add_argument("--deterministic-allreduce", action="store_true")
    return p.parse_args()


def setup_dist():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    lrank = int(os.environ.get("LOCAL_RANK", "0"))
    if torch.cuda.is_available():
        torch.cuda.set_device(lrank % torch.cuda.device_count())
    if ws > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl" if torch.cuda.is_available() else "gloo")
    return ws, rank, lrank


def barrier_sync(ws):
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    if ws > 1:
        import torch.distributed as dist
        dist.barrier()
    if torch.cuda.is_available():
        torch.cuda.synchronize()


def build_problem(ift, n, nlos):
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


def roofline_probe(ift, cf, n, reps=20):
    """Average duration of the dominant kernel family (the Hartley passes of
    the sampling-metric matvec: R2C rows + C2C/unpack columns at n x n fp64),
    timed with HIP events on the stream the kernels are launched on."""
    from nifty_amd import _native
    x = torch.randn((n, n), dtype=torch.float64, device="cuda")
    out = torch.empty_like(x)
    for _ in range(3):
        _native.hartley(x, (0, 1), out=out)
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        _native.hartley(x, (0, 1), out=out)
    e1.record(s)
    torch.cuda.synchronize()
    t_pair = e0.elapsed_time(e1) / reps * 1e-3          # one 2-D transform = 2 pass kernels
    N = n * n
    bytes_per_pass = N * 8 * 2                              # read N reals + write N/2 complex (= N reals)
    t_pass = t_pair / 2
    ach = bytes_per_pass / t_pass / 1e9
    return {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None,
            "kernel": "pass_kernel<double,*,R2C|UNPACK> (Hartley axis pass, 2048^2 fp64)",
            "avg_launch_us": round(t_pass * 1e6, 2), "algorithmic_bytes_per_launch": bytes_per_pass}


def cpu_baseline(cf_np_args, lat0, R, n, iters):
    """Oracle (numpy + scipy.fft on all host cores) sampling-metric CG on the
    same problem, bounded to `iters` CG iterations."""
    import scipy.fft
    from oracle.cf import CFOracle
    from oracle.sampling import LOSLikelihood, SamplingMetric, GradNormCtl, conjugate_gradient
    # the box's CPU share for one GPU (OMP_NUM_THREADS=16 there), not os.cpu_count()
    ncores = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    o = CFOracle((n, n), **cf_np_args)
    rows, cols, w = R.coo
    lh = LOSLikelihood(o, rows, cols, w, R.target.shape[0], 1e-3)
    with scipy.fft.set_workers(ncores):
        M = SamplingMetric(o, lat0, lh.middle(lat0))
        rng = np.random.default_rng(0)
        b = {k: rng.standard_normal(np.shape(v)) for k, v in lat0.items()}
        t = time.perf_counter()
        conjugate_gradient(M, {k: 0 * v for k, v in b.items()}, b, GradNormCtl(iteration_limit=iters))
        el = time.perf_counter() - t
    return iters / el, ncores, el


def main():
    args = parse()
    ws, rank, lrank = setup_dist()
    import nifty_amd as ift
    ift.config.set_device(f"cuda:{lrank}" if torch.cuda.is_available() else "cpu")
    if args.deterministic_allreduce:
        ift.utilities.DETERMINISTIC_ALLREDUCE = True
    comm = ift.TorchComm() if ws > 1 else None
    n = args.size
    cf, R, lh, pos, _ = build_problem(ift, n, args.nlos)
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
    if ws > 1:
        import torch.distributed as dist
        t = torch.tensor([el, float(iters)], dtype=torch.float64, device="cuda")
        dist.all_reduce(t[0:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(t[1:2], op=dist.ReduceOp.SUM)
        el, iters = float(t[0]), float(t[1])
    samples = 2 * nsamp * args.steps
    sps = samples / el
    cgps = iters / el
    roof = roofline_probe(ift, cf, n) if torch.cuda.is_available() else None
    cpu = None
    if rank == 0 and ws == 1 and not args.no_cpu_baseline:
        lat0 = {k: np.asarray(pos[k]) for k in cf.domain.keys()}
        cgi, ncores, cel = cpu_baseline(CF_ARGS, lat0, R, n, args.cpu_iters)
        cpu = {"value": round(cgi * sps / cgps, 6), "unit": "samples/s", "cores": ncores, "kind": "port",
               "cg_iter_per_s": round(cgi, 4),
               "sample": (f"oracle (numpy + scipy.fft workers={ncores}) sampling-metric CG on the same "
                          f"{n}^2 LOS problem, {args.cpu_iters} iterations in {cel:.1f}s; samples/s = "
                          f"cpu_cg_iter_per_s x (GPU samples per CG iteration)")}
    if rank == 0:
        line = {"metric": "geoVI samples-drawn/sec (+ CG-iter/sec), 2048^2 CorrelatedField",
                "value": round(sps, 6), "unit": "samples/s", "n_gpus": ws, "steps": args.steps,
                "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 3),
                "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
                "data": "synthetic",
                "config": {"workload": f"C3: {n}x{n} SimpleCorrelatedField, sigmoid, LOSResponse({args.nlos}), "
                                       f"Gaussian 1e-3, geoVI mirrored, {args.samples_per_gpu} pair(s)/GPU, "
                                       f"lin CG {args.lin_iters} it, NewtonCG {args.newton_iters} it "
                                       f"(inner CG <= {args.newton_cg_max})",
                           "global_batch": samples // args.steps, "parallelism": f"sample-dp{ws}"},
                "cg_iter_per_s": round(cgps, 3), "cg_iters": int(iters),
                "roofline": roof, "cpu_baseline": cpu}
        print(json.dumps(line), flush=True)
    if ws > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
