#!/usr/bin/env python3
"""Per-round state-machine kernel times and per-wave SQ counters from the
rocprofv3 CSVs of tools/sm_bench.py (tools/gpu_r5t.sh): the trace's
sm_round dispatches in order (rounds 0.. of each run, N=64 runs first), and
the counter pass's per-dispatch values divided by SQ_WAVES.

usage: sm_rounds.py <trace dir> <pmc dir>"""
import collections
import csv
import glob
import re
import sys


def main():
    tr = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
    rows = sorted((r for r in csv.DictReader(open(tr)) if "sm_round" in r["Kernel_Name"]),
                  key=lambda r: int(r["Start_Timestamp"]))
    runs, cur = [], []
    for r in rows:
        m = re.search(r"sm_round_\w+<[^>]*>", r["Kernel_Name"])
        k = m.group(0) if m else r["Kernel_Name"][:40]
        us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        cur.append((k, us))
        if us < 12:    # the quiescent round ends a run
            runs.append(cur)
            cur = []
    print("kernel trace, us per round (runs of sm_bench: warm-up + reps, N=64 then N=128)")
    for run in runs:
        print("  ", " ".join("%.0f" % us for _, us in run), " total %.0f" % sum(u for _, u in run),
              " ", run[-2][0])
    pm = glob.glob(sys.argv[2] + "/**/*counter_collection.csv", recursive=True)[0]
    d = collections.defaultdict(dict)
    for r in csv.DictReader(open(pm)):
        if "sm_round" not in r["Kernel_Name"]:
            continue
        c = d[int(r["Dispatch_Id"])]
        c[r["Counter_Name"]] = c.get(r["Counter_Name"], 0) + float(r["Counter_Value"])
    print("SQ counters per wave, per round")
    for i in sorted(d):
        c = d[i]
        w = c.get("SQ_WAVES", 1)
        print("  ", " ".join("%s %.0f" % (k.replace("SQ_", ""), v / w)
                             for k, v in sorted(c.items()) if k != "SQ_WAVES"))


if __name__ == "__main__":
    main()
