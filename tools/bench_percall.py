#!/usr/bin/env python3
"""Latency of the per-call drop-in path (include/hbrbc.h layer 1) against the
CPU restatement of the reference, call by call: what the unchanged
`Broadcast` pays at broadcast.rs:193 (Coding::encode), 204/580
(MerkleTree::from_vec), 569 (Coding::reconstruct_shards) and 605
(Proof::validate).  One instance per call, host buffers in and out (the
shims stage through pinned memory: one DMA each way, one synchronisation).

Prints one JSON object per (op, N, shard length): median microseconds of the
HIP shim and of the oracle (oracle/rbc_oracle.c, one core), and the ratio.
usage: python tools/bench_percall.py [out.jsonl]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import hbbft_amd as hb  # noqa: E402
from oracle import pyoracle as orc  # noqa: E402


def median_us(fn, reps):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return ts[len(ts) // 2] * 1e6


def main():
    out = open(sys.argv[1], "w") if len(sys.argv) > 1 else None
    rng = np.random.default_rng(5)
    rows = []
    for n, S in [(4, 514), (16, 4096), (64, 1024), (64, 11916), (64, 65536), (128, 5958),
                 (250, 49933)]:
        f = (n - 1) // 3
        k, m = n - 2 * f, 2 * f
        reps = 50 if S * n < 4 << 20 else 10
        coding = hb.Coding(k, m)
        data = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)]
        gpu = [d.copy() for d in data] + [np.zeros(S, np.uint8) for _ in range(m)]
        cpu = [d.copy() for d in data] + [np.zeros(S, np.uint8) for _ in range(m)]
        res = {"encode": (median_us(lambda: coding.encode(gpu), reps),
                          median_us(lambda: orc.rs_encode(k, m, cpu), reps))}
        shards = [bytes(x) for x in cpu]
        res["merkle_from_vec"] = (median_us(lambda: hb.MerkleTree.from_vec(shards), reps),
                                  median_us(lambda: orc.merkle_build(shards), reps))
        nodes = orc.merkle_build(shards)
        dig = orc.merkle_proof(nodes, n, 1)
        p = hb.Proof(shards[1], 1, [d.tobytes() for d in dig], nodes[-1].tobytes())
        res["proof_validate"] = (median_us(lambda: p._validate_one(n), reps),
                                 median_us(lambda: orc.proof_validate(shards[1], 1, dig,
                                                                      nodes[-1], n), reps))
        erased = rng.permutation(n)[:f]
        opt = [None if i in set(erased.tolist()) else shards[i] for i in range(n)]

        def rec_gpu():
            o = list(opt)
            coding.reconstruct_shards(o)

        opt_np = [None if x is None else np.frombuffer(x, np.uint8) for x in opt]
        res["reconstruct"] = (median_us(rec_gpu, reps),
                              median_us(lambda: orc.coding_reconstruct(k, m, list(opt_np)), reps))
        for op, (g, c) in res.items():
            row = {"op": op, "n": n, "shard_len": S, "hip_us": g, "cpu_us": c,
                   "cpu_over_hip": c / g}
            rows.append(row)
            line = json.dumps(row)
            print(line, flush=True)
            if out:
                out.write(line + "\n")
    if out:
        out.close()


if __name__ == "__main__":
    main()
