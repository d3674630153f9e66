#!/usr/bin/env python3
"""Per-kernel HBM traffic and Keccak VALU ops from rocprofv3 counter passes
(FETCH_SIZE, WRITE_SIZE and SQ_INSTS_VALU, each its own run as
MI355X_MICROARCH.md prescribes) of `bench.py --steps 1 --warmup 1`, as
collected by tools/profile.sh.

FETCH_SIZE / WRITE_SIZE are in KB.  FETCH_SIZE is divided by the calibration
factor of the access pattern the kernel's loads follow
(profiles/fetch_calibration.json, tools/fetch_calib.hip: raw counter bytes /
known bytes on gfx950 -- 0.500 for 16- and 4-byte coalesced loads, 0.539 for
the sponges' one-lane-per-row 8-byte loads); WRITE_SIZE measured exact (1.00).  Output (out.json): bytes per
launch and per instance for every hbrbc kernel of every profiled config, and
the "cfg:stage" -> bytes-per-instance map bench.py reads for roofline.traffic.
With an SQ pass and a sponge geometry it also writes
profiles/valu_ops_per_perm.json[config]: 32-bit lane-ops per Keccak-f[1600] of
the leaf-hash kernel = SQ_INSTS_VALU x 64 / permutations per launch.

usage: pmc_traffic.py <out.json> <profile dir>:<config>:<instances per launch>
                      [:<n>:<shard_len>] ...
"""
import collections
import csv
import glob
import json
import os
import re
import sys

STAGE = {"leaf_hash_kernel": "leaf_hash", "validate_kernel": "validate", "frame_kernel": "frame",
         "unframe_kernel": "unframe", "tree_level_kernel": "tree_levels", "proofs_kernel": "proofs",
         "decode_matrix_kernel": "decode_matrix", "decode_check_kernel": "decode_check",
         "gf_bitslice_kernel": "reconstruct"}


def kname(n):
    m = re.search(r"(hbrbc_(?:enc|dec)_\w+|\w+_kernel(<[^>]*>)?)", n)
    return m.group(1) if m else n[:40]


def base(k):
    return k.split("<")[0]


CALIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles",
                     "fetch_calibration.json")


def fetch_factor(k, calib):
    """(raw / known factor, pattern name) of kernel k's loads."""
    pats, kp = calib["patterns"], calib["kernel_pattern"]
    for prefix, pat in kp.items():
        if prefix != "default" and k.startswith(prefix):
            return pats[pat]["fetch_factor"], pat
    return pats[kp["default"]]["fetch_factor"], kp["default"]


def per_launch(path, counter, scale):
    fs = glob.glob(path + "*/**/run_counter_collection.csv", recursive=True)
    if not fs:
        return {}
    tot, cnt = collections.defaultdict(float), collections.defaultdict(set)
    for x in csv.DictReader(open(fs[0])):
        if "hbrbc" not in x["Kernel_Name"] or x["Counter_Name"] != counter:
            continue
        k = kname(x["Kernel_Name"])
        tot[k] += float(x["Counter_Value"]) * scale
        cnt[k].add(x["Dispatch_Id"])
    return {k: tot[k] / len(cnt[k]) for k in tot}


def main():
    out = sys.argv[1]
    try:
        doc = json.load(open(out))
    except (OSError, ValueError):
        doc = {}
    kernels_all, traffic = doc.get("kernels", {}), doc.get("traffic", {})
    calib = json.load(open(CALIB))
    for spec in sys.argv[2:]:
        parts = spec.split(":")
        d, cfg, inst = parts[0], parts[1], int(parts[2])
        fe = per_launch(d + "/pmc_fetch", "FETCH_SIZE", 1024.0)
        wr = per_launch(d + "/pmc_write", "WRITE_SIZE", 1024.0)
        kernels = {}
        for k in sorted(set(fe) | set(wr)):
            fac, pat = fetch_factor(k, calib)
            f2 = fe.get(k, 0.0) / fac
            kernels[k] = {"fetch_raw_bytes": fe.get(k, 0.0), "fetch_corrected_bytes": f2,
                          "fetch_factor": fac, "fetch_pattern": pat,
                          "write_bytes": wr.get(k, 0.0), "hbm_bytes": f2 + wr.get(k, 0.0),
                          "hbm_bytes_per_instance": (f2 + wr.get(k, 0.0)) / inst}
        kernels_all[cfg] = kernels
        # a stage = the sum of its kernels (the specialised encoder / decoder
        # programs of one matrix run one after another on the same rows)
        stage_bytes = collections.defaultdict(float)
        for k, v in kernels.items():
            if base(k) in STAGE:
                stage_bytes[STAGE[base(k)]] += v["hbm_bytes_per_instance"]
            elif k.startswith("hbrbc_enc_"):
                stage_bytes["encode"] += v["hbm_bytes_per_instance"]
            elif k.startswith("hbrbc_dec_"):
                stage_bytes["reconstruct"] += v["hbm_bytes_per_instance"]
        for st, b in stage_bytes.items():
            traffic["%s:%s" % (cfg, st)] = b
        if len(parts) >= 5:
            n, S = int(parts[3]), int(parts[4])
            sq = per_launch(d + "/pmc_sq", "SQ_INSTS_VALU", 1.0)
            leaf = [v for k, v in sq.items() if base(k) == "leaf_hash_kernel"]
            if leaf:
                perms = inst * n * ((S + 1 + 135) // 136)
                ops = leaf[0] * 64.0 / perms
                # keyed by config: the bench line of config c uses c's own pass
                vp = os.path.join(os.path.dirname(out), "valu_ops_per_perm.json")
                try:
                    vdoc = json.load(open(vp))
                except (OSError, ValueError):
                    vdoc = {}
                if "leaf_hash_kernel" in vdoc:   # the round-3 flat form
                    vdoc = {}
                vdoc[cfg] = {"leaf_hash_kernel": ops, "sq_insts_valu_per_launch": leaf[0],
                             "perms_per_launch": perms,
                             "source": "%s, %s: SQ_INSTS_VALU %.0f x 64 / %d permutations per "
                                       "launch" % (os.path.basename(d), cfg, leaf[0], perms)}
                json.dump(vdoc, open(vp, "w"), indent=1, sort_keys=True)
                print("%s leaf_hash lane-ops per permutation: %.1f" % (cfg, ops))
    traffic["_note"] = ("HBM bytes per instance per launch: (FETCH_SIZE / factor + WRITE_SIZE) x "
                        "1024 / instances per launch (rocprofv3 --pmc passes, tools/profile.sh); "
                        "factor = the calibrated raw/known ratio of the kernel's load pattern, "
                        "profiles/fetch_calibration.json (tools/fetch_calib.hip)")
    json.dump({"kernels": kernels_all, "traffic": traffic}, open(out, "w"), indent=1)
    print(json.dumps(traffic, indent=1))


if __name__ == "__main__":
    main()
