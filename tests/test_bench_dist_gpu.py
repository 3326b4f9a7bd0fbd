"""bench.py's multi-rank path on the one-GPU box: `--gpus 3 --backend gloo`
on a tiny C3-shaped problem (128^2, 500 lines of sight, one mirrored pair
per rank).  launch_workers starts the three ranks as child processes (the
parent never touches the GPU), every rank draws its shareRange of the
samples, the KL mean is one all-reduce, the ranks agree on the KL value (a
disagreement exits non-zero) and rank 0 prints the driver's JSON line with
n_gpus = 3 and the whole job's samples.  The 8-GPU scaling run itself is the
driver's (one process per GPU over RCCL)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_three_ranks_gloo(dev):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3", "--backend", "gloo", "--size", "128",
           "--nlos", "500", "--samples-per-gpu", "1", "--lin-iters", "10", "--newton-iters", "1",
           "--newton-cg-max", "5", "--steps", "1", "--warmup", "1", "--no-cpu-baseline", "--no-demo"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=400, cwd=ROOT,
                       env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0"))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 3 and d["scaling"] == "weak"
    assert d["distributed"]["backend"] == "gloo"
    assert d["distributed"]["samples_per_rank"] == [2, 2, 2]
    assert d["config"]["global_batch"] == 6
    assert d["value"] > 0 and d["cg_iters"] > 0
