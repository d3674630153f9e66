#!/usr/bin/env python3
"""Times hbrbc_pairing_check_batch (f4) on the GPU: `--n` checks e(a,b) ==
e(c,d) in the verify_decryption_share shape, from a small pool of points
built by the CPU restatement (dev tooling; bench.py's f4 leg generates its
own inputs).  Prints one JSON line; HBRBC_PAIR_WAVES picks the kernel
occupancy variant (read once per process)."""
import argparse
import json
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=16384)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import numpy as np
    import torch
    from oracle import bls_oracle as B
    from hbbft_amd import threshold as T
    rng = random.Random(3)
    pool = []
    for _ in range(8):
        pool.append(B.decryption_share_case(rng.randrange(1, B.R), rng.randrange(1, B.R),
                                            rng.randrange(1, B.R), tamper=rng.random() < 0.25))
    g1 = np.empty((2 * a.n, 96), np.uint8)
    g2 = np.empty((2 * a.n, 192), np.uint8)
    expect = []
    enc = [(B.g1_bytes(s), B.g2_bytes(h), B.g1_bytes(pk), B.g2_bytes(w)) for s, h, pk, w in pool]
    good = [B.pairing_check(*c) for c in pool]
    for i in range(a.n):
        j = i % len(pool)
        g1[2 * i] = np.frombuffer(enc[j][0], np.uint8)
        g2[2 * i] = np.frombuffer(enc[j][1], np.uint8)
        g1[2 * i + 1] = np.frombuffer(enc[j][2], np.uint8)
        g2[2 * i + 1] = np.frombuffer(enc[j][3], np.uint8)
        expect.append(1 if good[j] else 0)
    d1 = torch.from_numpy(g1).cuda()
    d2 = torch.from_numpy(g2).cuda()
    ws = T.workspace(2 * a.n)
    ok = T.pairing_check_batch(d1, d2, ws)       # warm-up (+ module load)
    torch.cuda.synchronize()
    assert ok.cpu().tolist() == expect, "check outcomes differ from the oracle"
    times = []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        T.pairing_check_batch(d1, d2, ws)
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    t = sorted(times)[len(times) // 2]
    print(json.dumps({"n_checks": a.n, "waves": os.environ.get("HBRBC_PAIR_WAVES", "default"),
                      "ms": t * 1e3, "checks_per_s": a.n / t, "pairings_per_s": 2 * a.n / t,
                      "outcomes_exact": True}), flush=True)


if __name__ == "__main__":
    main()
