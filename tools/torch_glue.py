"""Where the torch (non-native) GPU kernels of one bench step come from:
torch.profiler over draw_samples + SampledKLEnergy, aten ops grouped by the
innermost nifty_amd call site, with their GPU time."""
import sys
from collections import defaultdict

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402


def main():
    import nifty_amd as ift
    ift.config.set_device("cuda:0")
    cf, Rr, lh, pos, _ = bench.build_problem(ift, 2048, 16384)
    H = ift.StandardHamiltonian(lh, ift.GradientNormController(iteration_limit=100))
    mini = ift.NewtonCG(ift.GradientNormController(iteration_limit=2), max_cg_iterations=50)
    ift.random.push_sseq_from_seed(1000)

    def step():
        sl = ift.draw_samples(pos, H, mini, 4, True)
        ift.SampledKLEnergyClass(sl, H, [], None, True)
        torch.cuda.synchronize()
    step()
    step()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True,
                 experimental_config=torch._C._profiler._ExperimentalConfig(verbose=True)) as prof:
        step()
    agg = defaultdict(lambda: [0, 0.0])
    # leaf aten ops only (aten::to -> _to_copy -> copy_ would count thrice),
    # attributed to the innermost nifty_amd frame of their Python stack
    for ev in prof.events():
        if not ev.name.startswith("aten::") or ev.self_device_time_total <= 0:
            continue
        site = "?"
        for fr in (ev.stack or []):
            if "nifty_amd" in fr or "bench.py" in fr:
                site = fr.split("/")[-1]
                break
        key = (ev.name, site)
        agg[key][0] += 1
        agg[key][1] += ev.self_device_time_total
    tot = sum(v[1] for v in agg.values())
    print(f"aten GPU time in one step: {tot / 1e3:.1f} ms")
    for (name, site), (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:45]:
        print(f"{t / 1e3:8.2f} ms {n:6d}  {name:28s} {site}")


if __name__ == "__main__":
    main()
