"""Per-kernel SQ counters of the CG iteration (tools/pmc_probe.py) from
rocprofv3 --pmc passes: every counter of every pass directory given, per
labelled kernel, averaged per launch; derived per-wave figures (cycles are
quad-cycles, MI355X_MICROARCH.md §PMC).

    bash tools/pmc_sq.sh C5          (on the GPU box: the passes + this summary)
    python tools/pmc_sq.py gpurun_out pmc_sq1 pmc_sq2 ..."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def read_pass(d):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        raise SystemExit(f"no counter_collection.csv under {d}")
    per = defaultdict(lambda: defaultdict(float))
    names = {}
    for row in csv.DictReader(open(f[0])):
        i = int(row["Dispatch_Id"])
        per[i][row["Counter_Name"]] += float(row["Counter_Value"])
        names[i] = row["Kernel_Name"]
    return [(names[i], per[i]) for i in sorted(per)]


def main(out_dir, subs):
    meta = json.load(open(os.path.join(out_dir, "pmc_labels.json")))
    labels = meta["labels"]
    acc = defaultdict(lambda: defaultdict(float))
    cnt = defaultdict(int)
    for sub in subs:
        disp = read_pass(os.path.join(out_dir, sub))
        nft = [(n, v) for n, v in disp if "nft::" in n and "scale_kernel" not in n][-len(labels):]
        assert len(nft) == len(labels), (len(nft), len(labels))
        for lab, (_, vals) in zip(labels, nft):
            if sub == subs[0]:
                cnt[lab] += 1
            for c, v in vals.items():
                acc[lab][c] += v
    res = {}
    for lab, vals in acc.items():
        n = cnt[lab]
        v = {c: x / n for c, x in vals.items()}
        w = v.get("SQ_WAVES")
        d = dict(v)
        if w:
            for c in list(v):
                if c != "SQ_WAVES":
                    d[c + "_per_wave"] = round(v[c] / w, 1)
        res[lab] = {c: (round(x, 1) if isinstance(x, float) else x) for c, x in d.items()}
    print(json.dumps({"config": meta.get("config"), "rhs": meta.get("rhs"), "kernels": res}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
