"""cProfile of one bench step (draw_samples + KL energy) on the GPU: host-side
cost centres (Python overhead, syncs) of the sampling path."""
import cProfile
import pstats
import sys

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402


def main(sort="cumulative", n=70):
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
    pr = cProfile.Profile()
    pr.enable()
    step()
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats(sort).print_stats(n)
    st.sort_stats("tottime").print_stats(40)


if __name__ == "__main__":
    main()
