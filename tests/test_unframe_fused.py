"""Fused unframe (the generic reconstruct kernel writes the payload bytes of
the data rows; decode_check + a zero-fill fixup finish decode_from_shards,
broadcast.rs:563-601) against the separate unframe kernel and the oracle:
whole payload slots, lengths and statuses identical, for all-present, f and 2f
erasures, too few shards, a tampered shard, a lying length prefix, and shard
lengths that are not a multiple of 4 (byte-aligned payload stores in the
generic kernel; with a specialised decoder such a call unframes separately)."""
import os

import numpy as np
import pytest

from oracle import pyoracle as orc

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available(), "gpu tests need an MI355X"
    return torch


def _decode(torch, rb, slab, S, present, roots, env):
    old = os.environ.get("HBRBC_UNFRAME_FUSED")
    os.environ["HBRBC_UNFRAME_FUSED"] = env
    try:
        count = slab.shape[0]
        work = slab.clone()
        work[present == 0] = 0xA5                     # garbage in the erased rows
        nodes2 = rb.alloc_nodes(count)
        out = torch.full((count, (rb.k * S + 15) // 16 * 16), 0x5A, dtype=torch.uint8,
                         device="cuda")                # stale bytes everywhere
        plen_out = torch.zeros(count, dtype=torch.int32, device="cuda")
        status = torch.zeros(count, dtype=torch.int32, device="cuda")
        rb.decode(work, S, present, roots, nodes2, out, plen_out, status)
        torch.cuda.synchronize()
        return out.cpu().numpy(), plen_out.cpu().numpy(), status.cpu().numpy()
    finally:
        if old is None:
            del os.environ["HBRBC_UNFRAME_FUSED"]
        else:
            os.environ["HBRBC_UNFRAME_FUSED"] = old


@pytest.mark.parametrize("n,plen", [(16, 2396), (16, 2380), (64, 262144), (7, 1000), (4, 8),
                                    (64, 16380), (31, 5000)])
@pytest.mark.parametrize("gf", ["bitslice", "bitslice_x2"])
def test_fused_unframe_matches_separate_and_oracle(torch_cuda, monkeypatch, n, plen, gf):
    """(gf: the generic reconstruct form, one input or input pairs per step)"""
    torch = torch_cuda
    import hbbft_amd as hb
    monkeypatch.setenv("HBRBC_GF", gf)
    f = (n - 1) // 3
    count = 8
    rb = hb.RbcBatch(n, f, device=0)
    S = hb.shard_len(plen, rb.k)
    pay = np.stack([orc.gen_payload(11, i, plen) for i in range(count)])
    stride_p = (plen + 15) // 16 * 16
    payloads = torch.zeros((count, stride_p), dtype=torch.uint8, device="cuda")
    payloads[:, :plen] = torch.from_numpy(pay).cuda()
    slab = rb.alloc_slab(count, S)
    rb.frame(payloads, plen, slab)
    lie = max(0, plen - 100)
    slab[6, 0, :4] = torch.tensor(list(lie.to_bytes(4, "big")), dtype=torch.uint8)  # lying prefix
    rb.encode(slab, S)
    nodes = rb.alloc_nodes(count)
    rb.merkle(slab, S, nodes)
    roots = nodes[:, -1, :].clone()
    rng = np.random.default_rng(n * 1000 + plen)
    present = np.ones((count, n), np.uint8)
    for i in (1, 5, 7):
        present[i, rng.choice(n, f, replace=False)] = 0
    present[2, : 2 * f] = 0 if f else 1             # worst case: first 2f rows gone
    if f:
        present[3, : 2 * f + 1] = 0                 # too few
        present[5, 0] = 0                           # row 0 (the length prefix) rebuilt
    slab[4, n - 1, 0] ^= 1                          # tampered shard -> root mismatch
    pres = torch.from_numpy(present).cuda()
    a = _decode(torch, rb, slab, S, pres, roots, "1")
    b = _decode(torch, rb, slab, S, pres, roots, "0")
    for x, y in zip(a, b):
        assert np.array_equal(x, y)
    out, plo, st = a
    slot = (rb.k * S - 4 + 15) // 16 * 16       # unframe defines the chunks covering k*S - 4
    slab_h = slab.cpu().numpy()
    roots_h = roots.cpu().numpy()
    for i in range(count):
        sh = slab_h[i, :, :S].copy()
        sh[present[i] == 0] = 0xA5
        ref, _, _ = orc.decode_from_shards(n, f, sh, present[i], roots_h[i].tobytes())
        if ref is None:
            assert st[i] != 0 and (out[i, :slot] == 0).all(), i
        else:
            assert st[i] == 0 and plo[i] == len(ref), i
            assert out[i, :len(ref)].tobytes() == ref and (out[i, len(ref):slot] == 0).all(), i
    if f:
        assert st[3] == 10 and st[4] == 65
    assert plo[6] == lie or st[6] != 0


@pytest.mark.parametrize("n,plen", [(16, 2396), (64, 20050), (16, 2380), (31, 5000)])
def test_fused_unframe_in_specialised_decoder(torch_cuda, n, plen):
    """Instances of a pattern with a specialised (JIT) decoder write their
    payload from that decoder (first program: present data rows; every
    program: rebuilt data rows); instances of other patterns from the generic
    kernel.  Whole slots equal the separate unframe's and the oracle's.  With S
    % 4 != 0 the _uf programs do not apply and the call unframes separately."""
    torch = torch_cuda
    import hbbft_amd as hb
    f = (n - 1) // 3
    count = 6
    rb = hb.RbcBatch(n, f, device=0)
    S = hb.shard_len(plen, rb.k)
    pay = np.stack([orc.gen_payload(13, i, plen) for i in range(count)])
    stride_p = (plen + 15) // 16 * 16
    payloads = torch.zeros((count, stride_p), dtype=torch.uint8, device="cuda")
    payloads[:, :plen] = torch.from_numpy(pay).cuda()
    slab = rb.alloc_slab(count, S)
    rb.frame(payloads, plen, slab)
    rb.encode(slab, S)
    nodes = rb.alloc_nodes(count)
    rb.merkle(slab, S, nodes)
    roots = nodes[:, -1, :].clone()
    pattern = np.ones(n, np.uint8)
    pattern[[0, 2, n - 1] + list(range(5, 5 + f - 3))] = 0      # row 0 (the length) missing
    rb.specialise_decoder(pattern)
    present = np.tile(pattern, (count, 1))
    rng = np.random.default_rng(n)
    present[4] = 1
    present[4, rng.choice(n, f, replace=False)] = 0              # another pattern: generic
    present[5] = 1                                               # all present
    pres = torch.from_numpy(present).cuda()
    a = _decode(torch, rb, slab, S, pres, roots, "1")
    b = _decode(torch, rb, slab, S, pres, roots, "0")
    for x, y in zip(a, b):
        assert np.array_equal(x, y)
    out, plo, st = a
    slot = (rb.k * S - 4 + 15) // 16 * 16
    assert (st == 0).all() and (plo == plen).all()
    for i in range(count):
        assert out[i, :plen].tobytes() == pay[i].tobytes() and (out[i, plen:slot] == 0).all(), i
