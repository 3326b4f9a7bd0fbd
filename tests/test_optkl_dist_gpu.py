"""GPU, two ranks: optimize_kl (optimize_kl.py:51-412) with the samples
sharded over a 2-process group (both ranks on the one GPU, gloo), the
deterministic KL-mean tree and per-rank checkpoint files -- an uninterrupted
run and one interrupted after iteration 1 then resumed give the same
iterates bit for bit, on both ranks, and match the one-process run."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _two_ranks(tmp, out, total, resume, tag):
    port = _port()
    procs, files = [], []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE="2",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        f = os.path.join(tmp, f"{tag}_{r}.npz")
        files.append(f)
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "dist_optkl_worker.py"), out,
                                       str(total), "1" if resume else "0", f], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    logs = []
    for p in procs:
        try:
            logs.append(p.communicate(timeout=240)[0])
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    if any(p.returncode for p in procs):
        raise AssertionError("\n".join(f"--- rank {r} (status {p.returncode})\n{log[-3000:]}"
                                        for r, (p, log) in enumerate(zip(procs, logs))))
    return [dict(np.load(f)) for f in files]


def test_two_rank_optimize_kl_resume(dev, tmp_path):
    import nifty_amd as ift
    from test_optimize_kl_gpu import _problem, _run
    full = _two_ranks(str(tmp_path), str(tmp_path / "a"), 3, False, "full")
    part = _two_ranks(str(tmp_path), str(tmp_path / "b"), 2, False, "part")
    assert (tmp_path / "b" / "last_finished_iteration").read_text() == "1"
    # per-rank sample files of iteration 0 were replaced by iteration 1's
    # single MAP position
    assert os.path.isfile(tmp_path / "b" / "pickle" / "last.0.npz")
    assert not os.path.isfile(tmp_path / "b" / "pickle" / "last.1.npz")
    res = _two_ranks(str(tmp_path), str(tmp_path / "b"), 3, True, "res")
    for r in range(2):
        assert int(full[r]["n_iters"]) == 3 and int(part[r]["n_iters"]) == 2 and int(res[r]["n_iters"]) == 1
        # mirrored pair sharded: one sample on each rank
        assert list(full[r]["n_samples"]) == [2, 1] and list(res[r]["n_samples"]) == [2, 1]
        for k in [k for k in full[0] if k.startswith("final_")]:
            np.testing.assert_array_equal(full[r][k], full[0][k], err_msg=(r, k))
            np.testing.assert_array_equal(res[r][k], full[r][k], err_msg=(r, k))
        for k in [k for k in full[r] if k.startswith("it2_")]:
            np.testing.assert_array_equal(res[r]["it0_" + k[4:]], full[r][k], err_msg=(r, k))
        for k in [k for k in full[r] if k[0] == "s"]:
            np.testing.assert_array_equal(res[r][k], full[r][k], err_msg=(r, k))
    # the one-process run: the same samples and, the deterministic tree
    # being the serial pairwise sum, the same KL means -- the same iterates
    # bit for bit (test_dist_gpu.py shows it for one KL evaluation)
    from nifty_amd import utilities
    G = golden("optkl32.npz")
    lh, pos = _problem(ift, G)
    utilities.DETERMINISTIC_ALLREDUCE = True
    try:
        means, sl, mean = _run(ift, lh, pos, 3)
    finally:
        utilities.DETERMINISTIC_ALLREDUCE = False
    for k in mean.keys():
        np.testing.assert_array_equal(full[0]["final_" + k], mean[k].val.cpu().numpy(), err_msg=k)
    for i in range(2):
        s = sl.local_item(i)
        for k in s.keys():
            np.testing.assert_array_equal(full[i][f"s{i}_{k}"], s[k].val.cpu().numpy(), err_msg=(i, k))


def test_bench_two_ranks(dev, tmp_path):
    """bench.py --gpus 2 without a launcher starts its own two ranks (both on
    the one GPU here, gloo): one line with n_gpus 2, both ranks' samples
    counted, the KL all-reduce timed; a launcher world size that disagrees
    with --gpus is refused"""
    import json
    root = os.path.dirname(HERE)
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--size", "256", "--nlos", "1024",
           "--samples-per-gpu", "1", "--steps", "1", "--warmup", "1", "--lin-iters", "5", "--newton-iters", "1",
           "--newton-cg-max", "5", "--backend", "gloo", "--no-demo", "--no-cpu-baseline"]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=400)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["config"]["global_batch"] == 4
    d = line["distributed"]
    assert d["backend"] == "gloo" and d["samples_per_rank"] == [2, 2]
    assert d["kl_allreduce"]["calls"] >= 1 and d["kl_allreduce"]["ms_max_over_ranks"] > 0
    # a launcher's WORLD_SIZE that disagrees with --gpus: refused before any work
    bad = subprocess.run(cmd[:2] + ["--gpus", "4"], env=dict(env, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"),
                         capture_output=True, text=True, timeout=120)
    assert bad.returncode == 2 and "WORLD_SIZE" in bad.stderr
