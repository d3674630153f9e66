#!/usr/bin/env python3
"""Which hardware queue each HIP stream's dispatches used, and whether the
streams' kernels overlapped in time, from a rocprofv3 --kernel-trace CSV
(settle DESIGN's two-stream explanation from the trace).

usage: queue_map.py <kernel_trace.csv> [name filter]
"""
import collections
import csv
import json
import sys


def main():
    rows = [r for r in csv.DictReader(open(sys.argv[1]))
            if len(sys.argv) < 3 or sys.argv[2] in r["Kernel_Name"]]
    by_stream = collections.defaultdict(lambda: collections.Counter())
    spans = collections.defaultdict(list)
    for r in rows:
        by_stream[r["Stream_Id"]][r["Queue_Id"]] += 1
        spans[r["Stream_Id"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    streams = sorted(spans)
    # pairwise overlap: total ns during which a kernel of stream a and one of b both ran
    ov = {}
    for i, a in enumerate(streams):
        for b in streams[i + 1:]:
            tot = 0
            sb = sorted(spans[b])
            for s0, e0 in spans[a]:
                for s1, e1 in sb:
                    if s1 >= e0:
                        break
                    lo, hi = max(s0, s1), min(e0, e1)
                    if hi > lo:
                        tot += hi - lo
            ov["%s|%s" % (a, b)] = tot / 1e6
    busy = {s: sum(e - b for b, e in spans[s]) / 1e6 for s in streams}
    doc = {"dispatches_by_stream_and_queue": {s: dict(c) for s, c in by_stream.items()},
           "busy_ms_by_stream": busy, "overlap_ms_between_streams": ov}
    print(json.dumps(doc, indent=1))


if __name__ == "__main__":
    main()
