#!/usr/bin/env python3
"""One-screen summary of a bench.py JSON line (stdin)."""
import json
import sys

d = json.loads(sys.stdin.read())
print("head", round(d["value"], 2), "GB/s", round(d["ms_per_step"], 2), "ms",
      {k: round(v, 2) for k, v in d["stages_ms_per_step"].items()})
r = d.get("roofline") or {}
print("roofline", r.get("kernel"), round(r.get("frac", 0), 3), r.get("traffic"))
for k in ("leaf_reuse", "validators", "validators_cfg4", "cfg2", "cfg5", "threshold_decrypt"):
    v = d.get(k) or {}
    print(k, v.get("error") or (round(v.get("value", 0), 2), round(v.get("ms_per_step", 0), 2)))
for k in ("cfg2", "cfg5"):
    v = d.get(k) or {}
    if "stages_ms_per_step" in v:
        print(k, "stages", {a: round(b, 2) for a, b in v["stages_ms_per_step"].items()})
    if "encode_merkle" in v:
        print(k, "encode_merkle", round(v["encode_merkle"]["value"], 2), "GB/s")
