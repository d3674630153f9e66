"""Sponge rate against residency rounds: times hbrbc_merkle_batch (leaf
hashes + levels) at cfg3 shape (N=64, S=11916) for 16384, 8192, 6144, 4096
and 2048 instances (4, 2, 1.5, 1 and 0.5 residency rounds of 4 waves per
SIMD).  Prints one JSON line per case with the rate in G permutations/s."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import hbbft_amd as hb  # noqa: E402


def run(rb, slab, S, nodes, reps=5):
    rb.merkle(slab, S, nodes)
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        rb.merkle(slab, S, nodes)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return sorted(ts)[len(ts) // 2]


def main():
    n, f, S = 64, 21, 11916
    rb = hb.RbcBatch(n, f, device=0)
    perms_row = S // 136 + 1
    for count in (16384, 8192, 6144, 4096, 2048):
        slab = rb.alloc_slab(count, S)
        slab.random_(0, 256)
        nodes = rb.alloc_nodes(count)
        ms = run(rb, slab, S, nodes)
        perms = count * n * perms_row + count * (n - 1)
        print(json.dumps({"instances": count, "rounds": count * n / (1024 * 4 * 64), "ms": ms,
                          "G_perm_per_s": perms / ms / 1e6}), flush=True)
        del slab, nodes
        torch.cuda.empty_cache()

if __name__ == "__main__":
    main()
