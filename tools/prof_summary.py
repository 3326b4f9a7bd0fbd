"""Summarise a rocprofv3 kernel-stats CSV (and, if present, the kernel trace:
GPU-busy fraction of the last `window` ms)."""
import csv
import sys

import numpy as np


def main(d, window=None, top=25):
    r = list(csv.DictReader(open(f"{d}/run_kernel_stats.csv")))
    tot = sum(float(x["TotalDurationNs"]) for x in r)
    print(f"total kernel time {tot / 1e6:.2f} ms")
    for x in r[:top]:
        print(f"{float(x['TotalDurationNs']) / 1e6:8.2f}ms {int(x['Calls']):6d} "
              f"{float(x['AverageNs']) / 1e3:8.1f}us {float(x['Percentage']):5.1f}% {x['Name'][:100]}")
    if window:
        t = list(csv.DictReader(open(f"{d}/run_kernel_trace.csv")))
        S = np.array([int(x["Start_Timestamp"]) for x in t])
        E = np.array([int(x["End_Timestamp"]) for x in t])
        m = S > E.max() - window * 1e6
        print(f"last {window} ms: busy {(E[m] - S[m]).sum() / 1e6:.1f} ms, {m.sum()} kernels")


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else None)
