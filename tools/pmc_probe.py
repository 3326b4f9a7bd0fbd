"""Short GPU program for the rocprofv3 PMC passes (HBM traffic of the CG
iteration kernels, bench.py roofline `traffic`).

    rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 tools/pmc_probe.py [C?]
    rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python3 tools/pmc_probe.py [C?]
    python tools/pmc_summary.py gpurun_out

(C? = a bench.py config, default C3: its problem, RHS count and storage
type; the summary goes to profiles/pmc_traffic.json for C3,
profiles/pmc_traffic_C?.json otherwise.)

Runs (1) a calibration: nft_scale over a 1 GiB fp64 buffer (known bytes: 1 GiB
read + 1 GiB written, 8 B per lane, larger than the 256 MiB Infinity Cache),
then (2) `reps` batched CG iterations of the bench problem exactly as
bench.kernel_probe runs them, writing the launch labels (in dispatch order) to
gpurun_out/pmc_labels.json so the summary can name every dispatch."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main(config="C3", reps=3):
    import nifty_amd as ift
    from nifty_amd import _native
    ift.config.set_device("cuda:0")
    lib = _native.load()
    cfg = bench.CONFIGS[config]
    k = cfg["pairs"]
    if cfg["cg"] == "fp32":
        ift.config.set_cg_precision("fp32")   # as bench.py runs C5
    cf, R, lh, pos, _ = bench.build_problem(ift, cfg["shape"][0], 16384, config)
    ift.random.push_sseq_from_seed(5)
    core, W, shift, XS = bench.probe_setup(ift, lh, pos, k)
    n_lat = XS.shape[1]
    X, Rr, D = XS[:k].clone(), XS[k:2 * k].clone(), XS[2 * k:].clone()
    Q = torch.zeros_like(X)
    SC = torch.zeros((k, _native.CG_NSCALARS), dtype=torch.float64, device=X.device)
    SC[:, _native.CG_GAMMA] = 1.0
    SC[:, _native.CG_GPREV] = 1.0
    ws = _native.workspace(k * lib.nft_reduce_workspace(n_lat), X.device, "cgb")
    bufs = (X, Rr, D, Q, SC, ws)
    # calibration in the storage type of the run (fp32 loads are counted
    # differently from fp64 ones): 1 GiB each way
    cal_n = (1 << 30) // X.element_size()
    cal = torch.ones(cal_n, dtype=X.dtype, device=X.device)
    torch.cuda.synchronize()
    for _ in range(2):
        _native._check(lib.nft_scale(_native.ptr(cal), cal_n, _native.dtype_code(X.dtype), 1.0000001,
                                     _native.stream_ptr()))
    torch.cuda.synchronize()
    for _ in range(2):
        bench.cg_iteration(lib, core, W, shift, bufs, k)
    torch.cuda.synchronize()
    # the timed loop's count-only chunk when it defers x (bench.lazy_spec):
    # 19 steps and the flush, as bench.kernel_probe labels them
    lz = bench.lazy_spec(core, k, n_lat, X.dtype)
    lazy_m = bench.LAZY_CHUNK if lz is not None else 0
    with _native.LaunchProfile(capacity=4096) as p:
        if lz is None:
            for _ in range(reps):
                bench.cg_iteration(lib, core, W, shift, bufs, k)
        else:
            bench.lazy_chunk(lib, core, W, shift, bufs, k, lz, lazy_m)
    torch.cuda.synchronize()
    from nifty_amd.minimization import fused_cg
    dcar = bool(fused_cg._CARRY and fused_cg._CARRY_DIR and core.dir_blocks(k) > 0 and bench._CARRY_CACHE)
    model = bench.byte_model(cf, R, k, n_lat, dir_carried=dcar, pairs=bool(core._pairs(k)), s=X.element_size(),
                             lazy_m=lazy_m)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "pmc_labels.json"), "w") as f:
        json.dump({"labels": [lab for lab, _ in p.records], "calibration_bytes": X.element_size() * cal_n,
                   "calibration_launches": 2, "rhs": k, "model": model, "config": config}, f)
    print("pmc probe done:", len(p.records), "labelled launches")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "C3")
