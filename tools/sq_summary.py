"""Per-kernel SQ stall breakdown from a rocprofv3 --pmc pass over
tools/pmc_probe.py (SQ_WAVE_CYCLES, SQ_WAIT_ANY, SQ_WAIT_INST_ANY,
SQ_ACTIVE_INST_ANY, SQ_WAIT_INST_LDS, SQ_LDS_BANK_CONFLICT, SQ_WAVES):
fractions of wave cycles parked on waitcnt/barriers (WAIT_ANY), stalled at
issue (WAIT_INST_ANY) and issuing (ACTIVE_INST_ANY).

    python tools/sq_summary.py gpurun_out/pmc_sq/run_counter_collection.csv"""
import csv
import sys
from collections import defaultdict


def main(path):
    acc = defaultdict(lambda: defaultdict(float))
    n = defaultdict(set)
    for row in csv.DictReader(open(path)):
        k = row["Kernel_Name"][:60]
        acc[k][row["Counter_Name"]] += float(row["Counter_Value"])
        n[k].add(row["Dispatch_Id"])
    for k, c in sorted(acc.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
        wc = c.get("SQ_WAVE_CYCLES", 0) or 1
        print(f"{k:60s} disp {len(n[k]):3d} waves/disp {c.get('SQ_WAVES', 0) / len(n[k]):9.0f} "
              f"wait {c.get('SQ_WAIT_ANY', 0) / wc:5.2f} issue-stall {c.get('SQ_WAIT_INST_ANY', 0) / wc:5.2f} "
              f"active {c.get('SQ_ACTIVE_INST_ANY', 0) / wc:5.2f} lds-stall {c.get('SQ_WAIT_INST_LDS', 0) / wc:5.2f} "
              f"bank-conf/disp {c.get('SQ_LDS_BANK_CONFLICT', 0) / len(n[k]):10.0f}")


if __name__ == "__main__":
    main(sys.argv[1])
