"""Wall-clock breakdown of one bench step on the GPU (host timers around the
phases of draw_samples; torch.cuda.synchronize at phase ends)."""
import sys
import time
from collections import defaultdict

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402


def main(steps=3):
    import nifty_amd as ift
    from nifty_amd import random as R
    from nifty_amd.minimization import descent_minimizers as DM
    from nifty_amd.operators import sampling_enabler as SE
    ift.config.set_device("cuda:0")
    cf, Rr, lh, pos, _ = bench.build_problem(ift, 2048, 16384)
    H = ift.StandardHamiltonian(lh, ift.GradientNormController(iteration_limit=100))
    mini = ift.NewtonCG(ift.GradientNormController(iteration_limit=2), max_cg_iterations=50)
    T = defaultdict(float)
    hits = [0, 0]

    def timed(name, f):
        def g(*a, **k):
            torch.cuda.synchronize()
            t = time.perf_counter()
            r = f(*a, **k)
            torch.cuda.synchronize()
            T[name] += time.perf_counter() - t
            return r
        return g
    R.Random.normal = staticmethod(timed("rng.normal", R.Random.normal))
    orig_take = R._take

    def take(ss):
        r = orig_take(ss)
        hits[0 if r is None else 1] += 1
        return r
    R._take = take
    SE.SamplingEnabler.special_draw_sample = timed("special_draw_sample", SE.SamplingEnabler.special_draw_sample)
    SE.SamplingEnabler.draw_rhs = timed("draw_rhs", SE.SamplingEnabler.draw_rhs)
    SE.SamplingEnabler.solve_rhs = timed("solve_rhs (batched CG)", SE.SamplingEnabler.solve_rhs)
    DM.DescentMinimizer.__call__ = timed("newton", DM.DescentMinimizer.__call__)
    DM.NewtonCG.get_descent_direction = timed("  newton direction (CG)", DM.NewtonCG.get_descent_direction)
    from nifty_amd.minimization import energy_adapter as EA, line_search as LS, conjugate_gradient as CGm
    EA.EnergyAdapter.__init__ = timed("  energy evaluations", EA.EnergyAdapter.__init__)
    LS.LineSearch.perform_line_search = timed("  line search", LS.LineSearch.perform_line_search)
    ncall = [0]
    orig_ea = EA.EnergyAdapter.__init__

    def ea_count(*a, **k):
        ncall[0] += 1
        return orig_ea(*a, **k)
    EA.EnergyAdapter.__init__ = ea_count
    ift.random.push_sseq_from_seed(1000)
    for i in range(steps + 1):
        if i == 1:
            T.clear()
            hits[:] = [0, 0]
            ncall[0] = 0
            it0 = CGm.ConjugateGradient.iterations_total
        torch.cuda.synchronize()
        t = time.perf_counter()
        sl = ift.draw_samples(pos, H, mini, 4, True)
        ift.SampledKLEnergyClass(sl, H, [], None, True)
        torch.cuda.synchronize()
        T["step"] += time.perf_counter() - t if i else 0
    for k, v in T.items():
        print(f"{k:24s} {v / steps * 1e3:8.1f} ms/step")
    print("prefetch misses/hits", hits)
    print("energy evaluations/step", ncall[0] / steps,
          "CG iterations/step", (CGm.ConjugateGradient.iterations_total - it0) / steps)


if __name__ == "__main__":
    main()
