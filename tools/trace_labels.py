"""Per-label summary of the graph-replayed CG iteration from a rocprofv3
kernel trace (tools/replay_probe.py under rocprofv3 --kernel-trace): the last
REPLAYS iterations of the trace are split into their dispatches, every
dispatch is labelled as bench.py's kernel table labels it (by kernel name and,
for the two unpack passes, by order within the iteration), and per label the
mean duration and count per iteration are written, together with the
iteration's span (first start to last end) per replay.

    python tools/trace_labels.py TRACE.csv REPLAYS > summary.json"""
import csv
import json
import re
import sys
from collections import OrderedDict, defaultdict


def label(name, seen):
    n = name
    rules = [(r"cg_dir_dd_kernel", "cg_dir_dd2"), (r"jvp2a_kernel", "amp_jvp2a+dir"), (r"jvp2b_kernel", "amp_jvp2b"),
             (r"vjp2a_kernel", "amp_vjp2a+cg"), (r"vjp2b_kernel", "amp_vjp2b+cg"), (r"pro_fold_kernel|pro_rows_kernel", "pro_fold+dir"),
             (r"pro_r2c_kernel", "pro_r2c+dir"),
             (r"fast_kernel<double, \d+, \d+, 1, true", "fft_r2c"), (r"fast_kernel<double, \d+, \d+, 0, false", "fft_c2c"),
             (r"fin_kernel", "amp_fin"),
             (r"los_fwd_items|los_fwd_boxes|los_fwd_tiles", "los_fwd_items"), (r"los_fwd_reduce", "los_fwd_reduce"),
             (r"los_adj_boxes", "los_adj_boxes"), (r"fold_wide", "fold_partials"), (r"bin_fold", "bin_fold"),
             (r"bin_scatter", "bin_scatter"), (r"cg_update_kernel", "cg_update_seg2"),
             (r"cg_finalize_kernel", "cg_finalize_kernel")]
    # the strided unpack passes (kind 3), whatever their length and thread
    # count: the forward transform's, then the CG-carrying adjoint's
    if re.search(r"fast_kernel<double, \d+, \d+, 3, false", n):
        k = seen["unpack"]
        seen["unpack"] += 1
        return "fft_unpack" if k == 0 else "fft_unpack+cg"
    for pat, lab in rules:
        if re.search(pat, n):
            return lab
    return "other:" + n.split("(")[0][:60]


def main(path, reps):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    names = [r["Kernel_Name"] for r in rows]
    # period of the replayed tail: the smallest L with the last reps * L names
    # repeating every L, after at most a few trailing dispatches (the probe's
    # check of the scalars after the replays)
    L = None
    for skip in range(0, 9):
        n = len(names) - skip
        for cand in range(4, n // reps + 1):
            tail = names[n - reps * cand:n]
            if all(tail[i] == tail[i % cand] for i in range(len(tail))):
                L = cand
                break
        if L:
            break
    assert L, "no periodic tail found"
    tail = rows[n - reps * L:n]
    per = defaultdict(list)
    spans = []
    order = OrderedDict()
    for r in range(reps):
        it = tail[r * L:(r + 1) * L]
        seen = defaultdict(int)
        spans.append((int(it[-1]["End_Timestamp"]) - int(it[0]["Start_Timestamp"])) / 1e3)
        acc = defaultdict(float)
        for d in it:
            lab = label(d["Kernel_Name"], seen)
            order.setdefault(lab, 0)
            acc[lab] += (int(d["End_Timestamp"]) - int(d["Start_Timestamp"])) / 1e3
            if r == 0:
                order[lab] += 1
        for lab, us in acc.items():
            per[lab].append(us)
    out = {"source": path, "replays": reps, "dispatches_per_iteration": L,
           "iteration_span_us": round(sum(spans) / len(spans), 1),
           "labels": {lab: {"launches": order[lab], "avg_us": round(sum(per[lab]) / len(per[lab]), 2)}
                      for lab in order}}
    out["sum_of_label_us"] = round(sum(v["avg_us"] for v in out["labels"].values()), 1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 20)
