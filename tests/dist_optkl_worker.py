"""One rank of the 2-rank optimize_kl run of test_optkl_dist_gpu.py (not a test
module): ranks share cuda:0 and a gloo group, samples are sharded over the
ranks (kl_energies.py:140-141), the KL means go through the deterministic
tree, and checkpoints are written per rank into one output directory.

    RANK=r WORLD_SIZE=2 MASTER_ADDR=127.0.0.1 MASTER_PORT=p \
        python tests/dist_optkl_worker.py OUT TOTAL RESUME RESULT.npz
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))


def main():
    out, total, resume, result = sys.argv[1], int(sys.argv[2]), sys.argv[3] == "1", sys.argv[4]
    import numpy as np
    import torch.distributed as dist
    dist.init_process_group("gloo")
    import nifty_amd as ift
    from nifty_amd import utilities
    from conftest import golden
    from test_optimize_kl_gpu import _problem, _run
    utilities.DETERMINISTIC_ALLREDUCE = True
    comm = ift.TorchComm()
    lh, pos = _problem(ift, golden("optkl32.npz"))
    means, sl, mean = _run(ift, lh, pos, total, comm=comm, output_directory=out, resume=resume)
    res = {f"it{i}_{k}": v for i, m in enumerate(means) for k, v in m.items()}
    res.update({f"final_{k}": mean[k].val.cpu().numpy() for k in mean.keys()})
    for i in range(sl.n_local_samples):
        s = sl.local_item(i)
        res.update({f"s{list(sl.local_indices)[i]}_{k}": s[k].val.cpu().numpy() for k in s.keys()})
    res["n_iters"] = np.array(len(means))
    res["n_samples"] = np.array([sl.n_samples, sl.n_local_samples])
    np.savez(result, **res)
    comm.Barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
