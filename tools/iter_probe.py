"""The bench's batched CG iteration: graph-replayed wall time and the
per-kernel table (bench.kernel_probe), without the timed steps.  With
NFT_LIB pointing at an A/B build; PROBE_CONFIG = C2 / C3 (default) / C4 / C5.
Usage: python tools/iter_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    import nifty_amd as ift
    ift.config.set_device("cuda:0")
    c = os.environ.get("PROBE_CONFIG", "C3")
    cfg = bench.CONFIGS[c]
    if cfg["cg"] == "fp32":
        ift.config.set_cg_precision("fp32")
    cf, R, lh, pos, _ = bench.build_problem(ift, cfg["shape"][0], 16384, c)
    kp, it = bench.kernel_probe(ift, cf, R, lh, pos, cfg["pairs"])
    print(f"{c} {os.path.basename(os.path.dirname(os.environ.get('NFT_LIB', 'default/x')))}: "
          f"iteration {it['us_per_iteration']} us (sum of launches {it['us_sum_of_launches']})", flush=True)
    print("   " + " ".join(f"{k}={v['avg_us']:.1f}" for k, v in kp.items()), flush=True)


if __name__ == "__main__":
    main()
