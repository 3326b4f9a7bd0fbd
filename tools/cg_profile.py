"""Per-kernel device time of one batched sampling CG solve (4 right-hand
sides, the bench's metric) and of the Newton phase, per CG iteration
(nft_prof_* HIP events; graphs off so every launch is visible)."""
import os
import sys
import time
from collections import defaultdict

os.environ["NFT_NO_GRAPH"] = "1"
import torch  # noqa: E402

sys.path.insert(0, ".")
import bench  # noqa: E402


def main():
    import nifty_amd as ift
    from nifty_amd import _native
    from nifty_amd.minimization.conjugate_gradient import ConjugateGradient
    ift.config.set_device("cuda:0")
    cf, R, lh, pos, _ = bench.build_problem(ift, 2048, 16384)
    H = ift.StandardHamiltonian(lh, ift.GradientNormController(iteration_limit=100))
    mini = ift.NewtonCG(ift.GradientNormController(iteration_limit=2), max_cg_iterations=50)
    ift.random.push_sseq_from_seed(1000)
    ift.draw_samples(pos, H, mini, 4, True)
    torch.cuda.synchronize()
    torch.cuda._sleep(300_000_000)
    it0 = ConjugateGradient.iterations_total
    t0 = time.perf_counter()
    with _native.LaunchProfile(capacity=40000) as p:
        ift.draw_samples(pos, H, mini, 4, True)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    its = ConjugateGradient.iterations_total - it0
    acc, cnt = defaultdict(float), defaultdict(int)
    for lab, ms in p.records:
        acc[lab] += ms
        cnt[lab] += 1
    tot = sum(acc.values())
    print(f"draw_samples wall {wall * 1e3:.1f} ms, profiled device time {tot:.1f} ms, CG its {its}")
    for lab, ms in sorted(acc.items(), key=lambda kv: -kv[1]):
        print(f"   {lab:24s} {ms:8.2f} ms  launches {cnt[lab]:5d}  avg {ms / cnt[lab] * 1e3:7.1f} us")


if __name__ == "__main__":
    main()
