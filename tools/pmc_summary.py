"""Fold the two rocprofv3 PMC passes of tools/pmc_probe.py into
profiles/pmc_traffic.json: per labelled kernel the average FETCH_SIZE and
WRITE_SIZE per launch, corrected with the calibration dispatches.

Correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE/WRITE_SIZE are L2
memory-side request counts in KiB; on gfx950 a wide streaming read is
under-reported, so each counter is scaled by known_bytes / counted for the
nft_scale calibration over a 1 GiB buffer (8 B per lane, as most of the CG
kernels' loads).  Loads of other widths inside a kernel make the corrected
number approximate; the raw counter values are kept beside it."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def read_pass(d, counter):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        raise SystemExit(f"no counter_collection.csv under {d}")
    per = defaultdict(float)
    names = {}
    for row in csv.DictReader(open(f[0])):
        if row["Counter_Name"] != counter:
            continue
        i = int(row["Dispatch_Id"])
        per[i] += float(row["Counter_Value"])
        names[i] = row["Kernel_Name"]
    ids = sorted(per)
    return [(names[i], per[i] * 1024.0) for i in ids]  # counters are KiB


def main(out_dir):
    meta = json.load(open(os.path.join(out_dir, "pmc_labels.json")))
    labels = meta["labels"]
    res = {}
    for counter, sub in (("FETCH_SIZE", "pmc_fetch"), ("WRITE_SIZE", "pmc_write")):
        disp = read_pass(os.path.join(out_dir, sub), counter)
        cal = [v for n, v in disp if "scale_kernel" in n][-meta["calibration_launches"]:]
        nft = [(n, v) for n, v in disp if "nft::" in n and "scale_kernel" not in n]
        nft = nft[-len(labels):]
        assert len(nft) == len(labels), (len(nft), len(labels))
        res[counter] = (sum(cal) / len(cal), nft)
    fcal, fetch = res["FETCH_SIZE"]
    wcal, write = res["WRITE_SIZE"]
    known = meta["calibration_bytes"]
    fcorr, wcorr = known / fcal, known / wcal
    acc = defaultdict(lambda: [0, 0.0, 0.0, ""])
    for lab, (kn, fv), (_, wv) in zip(labels, fetch, write):
        a = acc[lab]
        a[0] += 1
        a[1] += fv
        a[2] += wv
        a[3] = kn[:120]
    kernels = {}
    for lab, (cnt, fv, wv, kn) in acc.items():
        f, w = fv / cnt, wv / cnt
        alg = meta["model"].get(lab)
        tr = f * fcorr + w * wcorr
        kernels[lab] = {"kernel": kn, "launches": cnt, "fetch_size_raw": round(f), "write_size_raw": round(w),
                        "traffic_bytes": round(tr), "algorithmic_bytes": alg,
                        "traffic_over_algorithmic": round(tr / alg, 3) if alg else None}
    config = meta.get("config", "C3")
    what = ("a 19-step count-only chunk with the deferred iterate and its flush (cg_lazy_flush: launches "
            "per iteration 1/19)" if "cg_lazy_flush" in acc else "batched CG iteration")
    out = {"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), tools/pmc_probe.py, "
                     f"{what} of the bench problem ({config}), {meta['rhs']} RHS",
           "calibration": {"kernel": "nft::scale_kernel over 1 GiB in the run's storage type",
                           "known_bytes_each_way": known,
                           "fetch_size_bytes": round(fcal), "write_size_bytes": round(wcal),
                           "fetch_correction": round(fcorr, 4), "write_correction": round(wcorr, 4)},
           "kernels": kernels}
    dst = os.path.join(ROOT, "profiles", "pmc_traffic.json" if config == "C3" else f"pmc_traffic_{config}.json")
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out"))
