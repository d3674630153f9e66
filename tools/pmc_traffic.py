#!/usr/bin/env python3
"""Per-kernel HBM traffic from two rocprofv3 counter passes (FETCH_SIZE and
WRITE_SIZE, separate runs as MI355X_MICROARCH.md prescribes) of
`bench.py --steps 1 --warmup 1`.

FETCH_SIZE / WRITE_SIZE are in KB; on gfx950 FETCH_SIZE reports half the bytes
of a wide streaming read, so it is doubled.  Output: bytes per launch and per
instance for every hbrbc kernel, and the "cfg:stage" -> bytes-per-instance map
bench.py reads for roofline.traffic.

usage: pmc_traffic.py <profile dir> <config> <instances per launch> <out.json>
"""
import collections
import csv
import glob
import json
import re
import sys

STAGE = {"leaf_hash_kernel": "leaf_hash", "validate_kernel": "validate", "frame_kernel": "frame",
         "unframe_kernel": "unframe", "tree_level_kernel": "tree_levels", "proofs_kernel": "proofs",
         "decode_matrix_kernel": "decode_matrix"}


def kname(n):
    m = re.search(r"(hbrbc_enc_\w+|\w+_kernel(<[^>]*>)?)", n)
    return m.group(1) if m else n[:40]


def per_launch(path, counter):
    f = glob.glob(path + "/**/run_counter_collection.csv", recursive=True)[0]
    tot, cnt = collections.defaultdict(float), collections.defaultdict(set)
    for x in csv.DictReader(open(f)):
        if "hbrbc" not in x["Kernel_Name"] or x["Counter_Name"] != counter:
            continue
        k = kname(x["Kernel_Name"])
        tot[k] += float(x["Counter_Value"]) * 1024.0
        cnt[k].add(x["Dispatch_Id"])
    return {k: tot[k] / len(cnt[k]) for k in tot}


def main():
    d, cfg, inst, out = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
    fe, wr = per_launch(d + "/pmc_fetch", "FETCH_SIZE"), per_launch(d + "/pmc_write", "WRITE_SIZE")
    kernels = {}
    for k in sorted(set(fe) | set(wr)):
        f2 = 2.0 * fe.get(k, 0.0)
        kernels[k] = {"fetch_raw_bytes": fe.get(k, 0.0), "fetch_corrected_bytes": f2,
                      "write_bytes": wr.get(k, 0.0), "hbm_bytes": f2 + wr.get(k, 0.0),
                      "hbm_bytes_per_instance": (f2 + wr.get(k, 0.0)) / inst}
    traffic = {"%s:%s" % (cfg, STAGE[k]): v["hbm_bytes_per_instance"]
               for k, v in kernels.items() if k in STAGE}
    for k, v in kernels.items():
        if k.startswith("hbrbc_enc_") or k.startswith("gf_bitslice_kernel<14"):
            traffic["%s:encode" % cfg] = v["hbm_bytes_per_instance"]
    traffic["_note"] = ("HBM bytes per instance per launch: (2 x FETCH_SIZE + WRITE_SIZE) x 1024 "
                        "/ %d instances; source %s" % (inst, d))
    json.dump({"kernels": kernels, "traffic": traffic}, open(out, "w"), indent=1)
    print(json.dumps(traffic, indent=1))


if __name__ == "__main__":
    main()
