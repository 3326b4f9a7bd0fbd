"""Wall time of the phases of one bench step (draw_samples + SampledKLEnergy
at a bench config's size, C3 by default) and how busy the GPU is inside each: the phases are timed
with a device synchronisation at their ends, the GPU busy time is the union
of the kernel intervals torch.profiler records.  Usage:
python tools/step_phases.py [--demo] [--config C2|C3|C4|C5] [--phase LABEL]"""
import sys
import time
from collections import defaultdict

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402

WALL = defaultdict(float)
CNT = defaultdict(int)


PROFILE = {}      # label -> torch.profiler results of that phase (--phase LABEL)


def _busy(prof):
    ivs, by = [], defaultdict(lambda: [0, 0.0])
    for ev in prof.events():
        if ev.device_type == torch.autograd.DeviceType.CUDA and ev.time_range.elapsed_us() > 0:
            ivs.append((ev.time_range.start, ev.time_range.end))
            by[ev.name][0] += 1
            by[ev.name][1] += ev.time_range.elapsed_us()
    ivs.sort()
    busy, cur = 0.0, None
    for a, b in ivs:
        if cur is None or a > cur[1]:
            if cur:
                busy += cur[1] - cur[0]
            cur = [a, b]
        else:
            cur[1] = max(cur[1], b)
    if cur:
        busy += cur[1] - cur[0]
    return busy, len(ivs), by


def timed(obj, name, label):
    f = getattr(obj, name)

    def w(*a, **k):
        torch.cuda.synchronize()
        prof = None
        if PROFILE.get("want") and PROFILE["want"] in label and "done" not in PROFILE:
            from torch.profiler import ProfilerActivity, profile
            prof = profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA])
            prof.__enter__()
        t = time.perf_counter()
        r = f(*a, **k)
        if hasattr(r, "__next__"):     # generators (refine): drain them
            r = list(r)
        torch.cuda.synchronize()
        el = time.perf_counter() - t
        WALL[label] += el
        CNT[label] += 1
        if prof is not None:
            prof.__exit__(None, None, None)
            PROFILE["done"] = True
            busy, n, by = _busy(prof)
            print(f"[{label}] wall {el * 1e3:.1f} ms (profiled), GPU busy {busy / 1e3:.1f} ms, {n} kernels")
            for nm, (c, us) in sorted(by.items(), key=lambda kv: -kv[1][1])[:25]:
                print(f"    {us / 1e3:8.2f} ms {c:5d}  {nm[:90]}")
        return r
    setattr(obj, name, w)


def main():
    if "--phase" in sys.argv:
        PROFILE["want"] = sys.argv[sys.argv.index("--phase") + 1]
    import nifty_amd as ift
    from nifty_amd.minimization import geovi_batch
    ift.config.set_device("cuda:0")
    c = sys.argv[sys.argv.index("--config") + 1] if "--config" in sys.argv else "C3"
    cfg = bench.CONFIGS[c]
    if cfg["cg"] == "fp32":
        ift.config.set_cg_precision("fp32")
    cf, Rr, lh, pos, _ = bench.build_problem(ift, cfg["shape"][0], 16384, c)
    pairs = cfg["pairs"]
    print(f"config {c}: {cfg['desc']}, {pairs} mirrored pairs", flush=True)
    if "--demo" in sys.argv:     # SURVEY 8(d)'s demo controllers (bench.py demo_step)
        H = ift.StandardHamiltonian(lh, ift.AbsDeltaEnergyController(deltaE=0.05, iteration_limit=100))
        mini = ift.NewtonCG(ift.AbsDeltaEnergyController(deltaE=0.5, convergence_level=2, iteration_limit=15))
    else:
        H = ift.StandardHamiltonian(lh, ift.GradientNormController(iteration_limit=100))
        mini = ift.NewtonCG(ift.GradientNormController(iteration_limit=2), max_cg_iterations=50)
    ift.random.push_sseq_from_seed(1000)

    def step():
        sl = ift.draw_samples(pos, H, mini, pairs, True)
        ift.SampledKLEnergyClass(sl, H, [], None, True)
        torch.cuda.synchronize()
    step()
    step()
    timed(geovi_batch, "kl_batch", "kl_batch (KL value + gradient)")
    timed(geovi_batch, "plan", "geovi plan (f_lh at the position)")
    orig_plan = geovi_batch.plan

    def plan(*a, **k):
        gb = orig_plan(*a, **k)
        timed(gb, "refine", "geovi refine (NewtonCG, batched)")
        return gb
    geovi_batch.plan = plan
    timed(geovi_batch.GeoVIBatch, "_serve_dir", "  refine: Newton directions (batched CG)")
    timed(geovi_batch.GeoVIBatch, "_serve_at", "  refine: energies at trial points")
    timed(geovi_batch.GeoVIBatch, "_serve_dd", "  refine: directional derivatives")
    from nifty_amd.operators import sampling_enabler as se
    timed(se.SamplingEnabler, "solve_rhs", "linear sampling CG (batched)")
    timed(se.SamplingEnabler, "draw_rhs", "draw_rhs (sample right-hand sides)")
    from nifty_amd.minimization import sample_list
    # inside draw_rhs: waiting for the background RNG, host->device uploads,
    # the likelihood draw J^T xi and the gradient J^T J s
    import nifty_amd.random as rnd
    import nifty_amd.field as fld
    from nifty_amd.operators import sandwich_operator as sw
    timed(rnd, "_take", "  rng: wait for prefetched draws")
    timed(fld, "_to_tensor", "  host->device uploads (_to_tensor)")
    timed(sw.SandwichOperator, "draw_sample", "  likelihood draw (J^T xi)")
    timed(sw.SandwichOperator, "apply", "  SandwichOperator.apply")
    timed(sample_list.ResidualSampleList, "__init__", "ResidualSampleList")
    # one step without the profiler: the phase wall times
    torch.cuda.synchronize()
    t = time.perf_counter()
    step()
    print(f"unprofiled step {1e3 * (time.perf_counter() - t):.1f} ms")
    for k, v in WALL.items():
        print(f"  {k:40s} {v * 1e3:9.1f} ms  ({CNT.get(k, 1)} calls)")
    WALL.clear()
    CNT.clear()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        torch.cuda.synchronize()
        t = time.perf_counter()
        sl = ift.draw_samples(pos, H, mini, pairs, True)
        torch.cuda.synchronize()
        WALL["draw_samples total"] += time.perf_counter() - t
        t1 = time.perf_counter()
        ift.SampledKLEnergyClass(sl, H, [], None, True)
        torch.cuda.synchronize()
        WALL["SampledKLEnergy"] += time.perf_counter() - t1
    WALL["step"] = time.perf_counter() - t
    ivs = []
    by = defaultdict(float)
    for ev in prof.events():
        if ev.device_type == torch.autograd.DeviceType.CUDA and ev.time_range.elapsed_us() > 0:
            ivs.append((ev.time_range.start, ev.time_range.end))
            nm = ev.name
            grp = "nft" if ("nft" in nm or "los_" in nm or "amp_" in nm or "cg_" in nm or "fft" in nm
                            or "r2c" in nm or "c2c" in nm or "bin_" in nm) else "torch/other"
            by[grp] += ev.time_range.elapsed_us()
    ivs.sort()
    busy, cur = 0.0, None
    for a, b in ivs:
        if cur is None or a > cur[1]:
            if cur:
                busy += cur[1] - cur[0]
            cur = [a, b]
        else:
            cur[1] = max(cur[1], b)
    if cur:
        busy += cur[1] - cur[0]
    span = (ivs[-1][1] - ivs[0][0]) if ivs else 0
    print(f"step wall {WALL['step'] * 1e3:.1f} ms; GPU busy {busy / 1e3:.1f} ms of a {span / 1e3:.1f} ms kernel span "
          f"({len(ivs)} kernels); kernel time nft {by['nft'] / 1e3:.1f} ms, other {by['torch/other'] / 1e3:.1f} ms")
    for k, v in WALL.items():
        print(f"  {k:40s} {v * 1e3:9.1f} ms  ({CNT.get(k, 1)} calls)")


if __name__ == "__main__":
    main()
