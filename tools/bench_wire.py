#!/usr/bin/env python3
"""Measures the wire-format kernels: bincode Value messages
for every proof of `count` cfg3 instances (N=64, 256 KiB), then their
deserialisation.  Prints one JSON line per kernel with its HBM roofline
(algorithmic bytes = bytes read + bytes written per launch / live launch
time, HIP events on the launch stream)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import hbbft_amd as hb
    n, plen = 64, 256 << 10
    count = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    rb = hb.RbcBatch(n, device=0)
    S = hb.shard_len(plen, rb.k)
    g = torch.Generator(device="cuda").manual_seed(1)
    payloads = torch.randint(0, 256, (count, plen), dtype=torch.uint8, device="cuda", generator=g)
    slab = rb.alloc_slab(count, S)
    nodes = rb.alloc_nodes(count)
    digests = torch.zeros((count, n, rb.dslots, 32), dtype=torch.uint8, device="cuda")
    ndig = torch.zeros((count, n), dtype=torch.uint8, device="cuda")
    rb.frame(payloads, plen, slab)
    rb.encode(slab, S)
    rb.merkle(slab, S, nodes)
    rb.proofs(nodes, digests, ndig)
    slot = rb.wire_slot(S)
    nmsg = count * n
    out = torch.empty((nmsg, slot), dtype=torch.uint8, device="cuda")
    mlen = torch.empty(nmsg, dtype=torch.int32, device="cuda")
    stride = rb.stride_for(S)
    vals = torch.empty((nmsg, stride), dtype=torch.uint8, device="cuda")
    vlen, idx, var, st = (torch.empty(nmsg, dtype=torch.int32, device="cuda") for _ in range(4))
    dg = torch.empty((nmsg, rb.dslots, 32), dtype=torch.uint8, device="cuda")
    ndo = torch.empty(nmsg, dtype=torch.uint8, device="cuda")
    rts = torch.empty((nmsg, 32), dtype=torch.uint8, device="cuda")

    def enc():
        rb.wire_encode(slab, S, digests, ndig, nodes[:, -1, :], out, mlen)

    def dec():
        rb.wire_decode(out, mlen, vals, vlen, idx, dg, ndo, rts, var, st)

    def timeit(fn, reps=5):
        fn()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) / reps / 1e3

    t_enc, t_dec = timeit(enc), timeit(dec)
    assert bool((st == 0).all()) and torch.equal(vals.view(count, n, stride)[:, :, :S], slab[:, :, :S])
    msg_bytes = float(mlen.to(torch.int64).sum())
    dig_bytes = float(ndig.to(torch.int64).sum()) * 32
    # encode reads values + digests (+ roots, indices), writes the messages;
    # decode reads the messages, writes values (padded rows) + digests + roots
    enc_alg = nmsg * S + dig_bytes + msg_bytes
    dec_alg = msg_bytes + nmsg * stride + dig_bytes + nmsg * 32
    for name, t, alg in [("wire_encode", t_enc, enc_alg), ("wire_decode", t_dec, dec_alg)]:
        print(json.dumps({"kernel": name, "messages": nmsg, "workload": "cfg3 Value messages, "
                          "N=64, 256 KiB payloads, %d instances" % count, "ms": t * 1e3,
                          "messages_per_s": nmsg / t, "roofline": {
                              "bound": "hbm", "achieved": alg / t / 1e9, "peak": 8000.0,
                              "unit": "GB/s", "frac": alg / t / 8e12, "alg_bytes": alg}}))


if __name__ == "__main__":
    main()
