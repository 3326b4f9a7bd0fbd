"""LOS adjoint ablations on the bench's plan (2048^2, 16384 lines, K = 4,
pixel-side row scale shared): NFT_LOS_ADJ_DBG bits 1 no output stores, 2 no
entry sums, 4 no line values, 8 no entry loads (tuning probe only).  The
ablation bits live in a probe build of los_adj_boxes (remap bits 4..7, read
from NFT_LOS_ADJ_DBG by adj_boxes_k; not in the product kernel, whose
registers they would cost): run with NFT_LIB pointing at that build."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from los_probe import timed  # noqa: E402


def main():
    import nifty_amd as ift
    from nifty_amd import _native as nat
    ift.config.set_device("cuda:0")
    cf, R, lh, pos, _ = bench.build_problem(ift, 2048, 16384)
    k = 4
    N = 2048 * 2048
    nlos = R.target.shape[0]
    Y = torch.randn((k, nlos), dtype=torch.float64, device="cuda")
    cs = torch.rand(N, dtype=torch.float64, device="cuda")
    out = torch.empty((k, N), dtype=torch.float64, device="cuda")
    plan = R._box_plan()
    for rep in range(2):
        for dbg in ("0", "1", "2", "4", "8", "3", "6", "14", "15"):
            os.environ["NFT_LOS_ADJ_DBG"] = dbg
            us = timed(lambda: nat.los_adjoint_batched(plan, Y, out, rowscale=cs))
            print(f"adj dbg={dbg} {us:.1f} us", flush=True)
    os.environ["NFT_LOS_ADJ_DBG"] = "0"


if __name__ == "__main__":
    main()
