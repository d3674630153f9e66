#!/usr/bin/env python3
"""FETCH_SIZE / WRITE_SIZE calibration factors.

Reads the known byte counts printed by tools/fetch_calib (JSON on stdout) and
the rocprofv3 counter CSVs of its FETCH_SIZE and WRITE_SIZE passes, and writes
per access pattern: the raw counter bytes per launch (counter KB x 1024), the
known bytes, and raw / known.  pmc_traffic.py divides each kernel's raw
FETCH_SIZE by the factor of the pattern that kernel uses (instead of doubling
every kernel, which the guide documents only for 16-B/lane streaming reads).

usage: fetch_calib.py <known.json> <fetch dir> <write dir> <out.json>
"""
import collections
import csv
import glob
import json
import sys


def per_launch(d, counter):
    fs = glob.glob(d + "/**/*counter_collection.csv", recursive=True)
    tot, ids = collections.defaultdict(float), collections.defaultdict(set)
    for x in csv.DictReader(open(fs[0])):
        if x["Counter_Name"] != counter or "calib_" not in x["Kernel_Name"]:
            continue
        k = x["Kernel_Name"].split("(")[0].strip()
        tot[k] += float(x["Counter_Value"]) * 1024.0
        ids[k].add(x["Dispatch_Id"])
    return {k: tot[k] / len(ids[k]) for k in tot}


def main():
    known = json.load(open(sys.argv[1]))
    fe = per_launch(sys.argv[2], "FETCH_SIZE")
    wr = per_launch(sys.argv[3], "WRITE_SIZE")
    out = {}
    for k, kb in known.items():
        e = {"known_read_bytes": kb["read"], "known_write_bytes": kb["write"]}
        if k in fe:
            e["fetch_raw_bytes"] = fe[k]
            e["fetch_factor"] = fe[k] / kb["read"] if kb["read"] else None
        if k in wr:
            e["write_raw_bytes"] = wr[k]
            e["write_factor"] = wr[k] / kb["write"] if kb["write"] else None
        out[k] = e
    doc = {"patterns": out,
           "note": "factor = raw counter bytes (KB x 1024) per launch / known bytes per launch; "
                   "tools/fetch_calib.hip over a 4 GiB buffer (16x the Infinity Cache), mean of "
                   "3 launches per pattern, one rocprofv3 --pmc pass per counter",
           # which pattern each kernel family's loads follow (pmc_traffic.py)
           # first matching prefix wins (the V16 instantiations before the rest)
           "kernel_pattern": {"leaf_hash_kernel<true>": "calib_rows16",
                              "validate_kernel<true>": "calib_rows16",
                              "leaf_hash_kernel": "calib_rows8", "validate_kernel": "calib_rows8",
                              "leaf_hash_list": "calib_rows8", "gf_bitslice_kernel": "calib_gf16",
                              "hbrbc_enc_": "calib_gf16", "hbrbc_dec_": "calib_gf16",
                              "default": "calib_stream16"}}
    json.dump(doc, open(sys.argv[4], "w"), indent=1)
    print(json.dumps(doc, indent=1))


if __name__ == "__main__":
    main()
