#!/usr/bin/env python3
"""How much of the sponge kernels' time is memory?  Runs hbrbc_validate_batch
at the cfg3 size (16384 instances x 64 proofs of 11,916-byte values) twice:
with the real row strides (every lane streams its own row) and with zero
strides (every lane reads the same row: broadcast loads that hit in L1).  The
Keccak work is identical (each proof hashes its value and walks its digests),
so the difference is the cost of the row traffic.  Prints one JSON line."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import hbbft_amd as hb  # noqa: E402


def main():
    n, S, count = 64, 11916, int(os.environ.get("COUNT", "16384"))
    rb = hb.RbcBatch(n, device=0)
    stride = rb.stride_for(S)
    dev = torch.device("cuda", 0)
    slab = torch.randint(0, 256, (count, n, stride), dtype=torch.uint8, device=dev)
    dig = torch.zeros((count, n, rb.dslots, 32), dtype=torch.uint8, device=dev)
    ndig = torch.full((count, n), rb.dslots, dtype=torch.uint8, device=dev)
    roots = torch.zeros((count, 32), dtype=torch.uint8, device=dev)
    idx = torch.arange(n, dtype=torch.int32, device=dev).repeat(count, 1).contiguous()
    ok = torch.zeros((count, n), dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream(dev)

    def run(vs, vis):
        hb._check(hb.lib().hbrbc_validate_batch(
            rb.coding.handle, slab.data_ptr(), S, vs, vis, n, idx.data_ptr(), dig.data_ptr(),
            ndig.data_ptr(), roots.data_ptr(), roots.stride(0), n, count, ok.data_ptr(),
            hb.ctypes.c_void_p(st.cuda_stream)))

    out = {}
    for name, vs, vis in (("rows", slab.stride(1), slab.stride(0)), ("broadcast", 0, 0),
                          ("rows_again", slab.stride(1), slab.stride(0))):
        run(vs, vis)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(5):
            run(vs, vis)
        b.record()
        torch.cuda.synchronize()
        out[name + "_ms"] = a.elapsed_time(b) / 5
    perms = count * n * ((S + 1 + 135) // 136 + rb.dslots)
    out.update({"perms_per_launch": perms,
                "rows_Gperm_s": perms / out["rows_ms"] / 1e6,
                "broadcast_Gperm_s": perms / out["broadcast_ms"] / 1e6})
    print(json.dumps(out))


if __name__ == "__main__":
    main()
