"""Where the demo-controller step's time goes: every batched / single fused
CG solve timed (device synchronised around it) with its metric kind, batch
size, iteration count and the iteration path it took (carried / queued /
per-iteration host read).  Usage: python tools/demo_profile.py [--steps N]"""
import os
import sys
import time
from collections import defaultdict

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    steps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 2
    import nifty_amd as ift
    from nifty_amd.minimization import fused_cg
    ift.config.set_device("cuda:0")
    cf, R, lh, pos, _ = bench.build_problem(ift, 2048, 16384)
    rec = defaultdict(lambda: [0, 0, 0.0])
    orig = fused_cg.FusedCGBatch.run_packed

    def run_packed(self, X, Rr, Bv, starts):
        torch.cuda.synchronize()
        it0 = ift.ConjugateGradient.iterations_total
        t = time.perf_counter()
        r = orig(self, X, Rr, Bv, starts)
        torch.cuda.synchronize()
        el = time.perf_counter() - t
        kind = type(self.core).__name__
        ctl = type(self.controllers[0]).__name__
        key = (kind, ctl, X.shape[0], getattr(self, "path", "?"))
        rec[key][0] += 1
        rec[key][1] += ift.ConjugateGradient.iterations_total - it0
        rec[key][2] += el
        return r
    fused_cg.FusedCGBatch.run_packed = run_packed
    for i in range(steps + 1):
        rec.clear()
        d = bench.demo_step(ift, lh, pos, 4, None)
        print(f"step {i}: {d}", flush=True)
    tot = 0.0
    for key, (n, it, el) in sorted(rec.items(), key=lambda kv: -kv[1][2]):
        tot += el
        print(f"  {el * 1e3:9.1f} ms  solves {n:4d}  rhs-iters {it:6d}  "
              f"{el * 1e6 / max(it, 1):8.1f} us/rhs-iter  {key}", flush=True)
    print(f"  {tot * 1e3:9.1f} ms in batched solves", flush=True)


if __name__ == "__main__":
    main()
