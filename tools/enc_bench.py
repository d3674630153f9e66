#!/usr/bin/env python3
"""Frame + encode alone (hbrbc_frame_encode_batch, the specialised encoder of
the bench's context) over a cfg3-sized batch already in HBM: ms per launch
(HIP events, median of --reps), for A/B of encoder code-object variants
(HBRBC_RT_SPEC, HBRBC_JIT_WPE, ... as in tools/build_variants.py).

usage: python tools/enc_bench.py [--n 64] [--count 16384] [--plen 262144]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=64)
    ap.add_argument("--count", type=int, default=16384)
    ap.add_argument("--plen", type=int, default=256 << 10)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    import torch

    import hbbft_amd as hb
    dev = torch.device("cuda", 0)
    rb = hb.RbcBatch(a.n, device=0)
    S = hb.shard_len(a.plen, rb.k)
    pay = torch.randint(0, 256, (a.count, (a.plen + 15) // 16 * 16), dtype=torch.uint8, device=dev)
    slab = torch.empty((a.count, a.n, rb.stride_for(S)), dtype=torch.uint8, device=dev)
    for _ in range(2):
        rb.frame_encode(pay, a.plen, slab)
    torch.cuda.synchronize()
    ts = []
    for _ in range(a.reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        rb.frame_encode(pay, a.plen, slab)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    alg = a.count * (a.plen + a.n * S)
    print(json.dumps({"n": a.n, "count": a.count, "kernel": rb.coding.encode_kernel(),
                      "ms_median": ts[len(ts) // 2], "ms_min": ts[0],
                      "alg_TBps": alg / (ts[len(ts) // 2] * 1e-3) / 1e12,
                      "env": {k: v for k, v in os.environ.items() if k.startswith("HBRBC_")}}),
          flush=True)


if __name__ == "__main__":
    main()
