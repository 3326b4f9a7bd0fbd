"""The bench's batched CG iteration (C3, 4 RHS): graph-replayed wall time and
the per-kernel table (bench.kernel_probe), without the timed steps.  With
NFT_LIB pointing at an A/B build.  Usage: python tools/iter_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    import nifty_amd as ift
    ift.config.set_device("cuda:0")
    cf, R, lh, pos, _ = bench.build_problem(ift, 2048, 16384)
    kp, it = bench.kernel_probe(ift, cf, R, lh, pos, 4)
    print(f"{os.path.basename(os.environ.get('NFT_LIB', 'default'))}: iteration {it['us_per_iteration']} us "
          f"(sum of launches {it['us_sum_of_launches']})", flush=True)
    print("   " + " ".join(f"{k}={v['avg_us']:.1f}" for k, v in kp.items()), flush=True)


if __name__ == "__main__":
    main()
