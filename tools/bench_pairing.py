#!/usr/bin/env python3
"""Times hbrbc_pairing_check_batch (f4) on the GPU: `--n` checks e(a,b) ==
e(c,d) in the verify_decryption_share shape, from a small pool of points
built by the CPU restatement (dev tooling; bench.py's f4 leg generates its
own inputs).  Prints one JSON line; HBRBC_PAIR_MULTI=0 selects one lane per
pairing instead of the multi-Miller check kernel."""
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
    ap.add_argument("--prepared", action="store_true",
                    help="grouped checks against prepared G2 points (64 shares per ciphertext)")
    ap.add_argument("--keys", type=int, default=2,
                    help="with --prepared: 2 = key shares and shares from prepared G1 tables, "
                         "the shares' beside the G2 preparation (the bench's f4 leg); 1 = key "
                         "shares only; 0 = both decoded per check")
    a = ap.parse_args()
    if a.prepared:
        return prepared(a)
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
    print(json.dumps({"n_checks": a.n, "mode": "plain",
                      "ms": t * 1e3, "checks_per_s": a.n / t, "pairings_per_s": 2 * a.n / t,
                      "outcomes_exact": True}), flush=True)


def prepared(a):
    """a.n checks in groups of 64 shares per ciphertext (the fixture groups of
    tests/golden/bls_vectors.json tiled): each step prepares the H and W of
    every group (inside the timing) and checks its shares against them."""
    import numpy as np
    import torch
    from hbbft_amd import threshold as T
    groups = json.load(open(os.path.join(ROOT, "tests", "golden", "bls_vectors.json")))["bench_groups"]
    ng = a.n // 64
    g2 = np.empty((2 * ng, 192), np.uint8)
    g1 = np.empty((2 * a.n, 96), np.uint8)
    expect = []
    for q in range(ng):
        grp = groups[q % len(groups)]
        g2[2 * q] = np.frombuffer(bytes.fromhex(grp["hash"]), np.uint8)
        g2[2 * q + 1] = np.frombuffer(bytes.fromhex(grp["w"]), np.uint8)
        for s, sh in enumerate(grp["shares"]):
            i = q * 64 + s
            g1[2 * i] = np.frombuffer(bytes.fromhex(sh["share"]), np.uint8)
            g1[2 * i + 1] = np.frombuffer(bytes.fromhex(sh["pk"]), np.uint8)
            expect.append(1 if sh["expect"] else 0)
    d1, d2 = torch.from_numpy(g1).cuda(), torch.from_numpy(g2).cuda()
    ib = torch.arange(a.n, dtype=torch.int32, device="cuda") // 64 * 2
    idd = ib + 1
    ws = T.workspace(a.n)
    shares = d1[0::2].contiguous()
    keys_h = np.stack([np.frombuffer(bytes.fromhex(sh["pk"]), np.uint8)
                       for grp in groups for sh in grp["shares"]])
    dkeys = torch.from_numpy(keys_h).cuda()
    ic = torch.from_numpy(np.array([(q % len(groups)) * 64 + s for q in range(ng)
                                    for s in range(64)], np.int32)).cuda()

    main = torch.cuda.current_stream()
    side = torch.cuda.Stream()

    def run():
        if a.keys >= 2:
            side.wait_stream(main)
            with torch.cuda.stream(side):
                keys = T.g1_prepare(dkeys)
                sprep = T.g1_prepare(shares)
            prep = T.g2_prepare(d2)
            main.wait_stream(side)
            keys.record_stream(main)
            sprep.record_stream(main)
            return T.pairing_check_prepared_pts(sprep, a.n, keys, dkeys.shape[0], ic, prep, 2 * ng,
                                                ib, idd, ws)
        prep = T.g2_prepare(d2)
        if not a.keys:
            return T.pairing_check_prepared(d1, prep, 2 * ng, ib, idd, ws)
        keys = T.g1_prepare(dkeys)
        return T.pairing_check_prepared_keys(shares, keys, dkeys.shape[0], ic, prep, 2 * ng, ib,
                                             idd, ws)
    ok = run()
    torch.cuda.synchronize()
    assert ok.cpu().tolist() == expect, "check outcomes differ from the fixtures"
    times = []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        run()
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    t = sorted(times)[len(times) // 2]
    print(json.dumps({"n_checks": a.n, "mode": "prepared" + ("+keys+shares" if a.keys >= 2 else "+keys" if a.keys else ""),
                      "groups": ng, "ms": t * 1e3,
                      "checks_per_s": a.n / t, "outcomes_exact": True}), flush=True)


if __name__ == "__main__":
    main()
