#!/usr/bin/env python3
"""Reduce the f4 profiles (tools/gpu_f4_prof.sh) to per-check numbers:
SQ_INSTS_VALU x 64 / checks per kernel and in total (lane-ops per check, the
VALU roofline's work figure), average kernel durations from the trace stats.
usage: pmc_pairing.py <prof dir> <checks per call>; prints JSON."""
import csv
import glob
import json
import sys
from collections import defaultdict


def main():
    d, n = sys.argv[1], int(sys.argv[2])
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(d + "/pmc/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            k = row.get("Kernel_Name", "")
            kern = ("prepare" if "g2_prepare" in k else "prepare_keys" if "g1_prepare" in k
                    else "miller" if "miller" in k
                    else "final_exp" if "final_exp_kernel" in k else None)
            if kern:
                vals[kern][row["Counter_Name"]].append(float(row["Counter_Value"]))
    per = {}
    # per call: every kernel's dispatches summed, over the number of calls (one
    # Miller launch per call; the G1 preparation runs twice per call when the
    # shares are prepared too -- keys and shares -- with different work)
    calls = max(1, len(vals.get("miller", {}).get("SQ_INSTS_VALU", [])))
    for kern, cs in vals.items():
        per[kern] = {c: sum(v) / calls for c, v in cs.items()}
    stats = {}
    for f in glob.glob(d + "/trace/**/*kernel_stats.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            k = row["Name"]
            kern = ("prepare" if "g2_prepare" in k else "prepare_keys" if "g1_prepare" in k
                    else "miller" if "miller" in k
                    else "final_exp" if "final_exp_kernel" in k else None)
            if kern:
                stats[kern] = float(row["AverageNs"]) / 1e6
    ops = {k: v["SQ_INSTS_VALU"] * 64 / n for k, v in per.items() if "SQ_INSTS_VALU" in v}
    out = {"checks_per_call": n, "counters_per_dispatch": per, "avg_ms": stats,
           "ops_per_check_by_kernel": ops, "ops_per_check": sum(ops.values()),
           "source": "rocprofv3 SQ_INSTS_VALU x 64 / %d checks (tools/gpu_f4_prof.sh)" % n}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
