"""Wire format (bincode 1.x of broadcast::Message, message.rs:13-24) on the GPU:
hbrbc_wire_encode_batch / hbrbc_wire_decode_batch against the oracle's
restatement of bincode and the golden N=4 'Foo' messages.  Byte work:
bit-exact."""
import json
import os

import numpy as np
import pytest

import hbbft_amd as hb
from oracle import pyoracle as orc

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden")


def proposer_side(torch, n, plen, count, seed):
    rb = hb.RbcBatch(n, device=0)
    S = hb.shard_len(plen, rb.k)
    pay = np.stack([orc.gen_payload(seed, i, plen) for i in range(count)])
    payloads = torch.zeros((count, max(16, (plen + 15) // 16 * 16)), dtype=torch.uint8, device="cuda")
    payloads[:, :plen] = torch.from_numpy(pay).cuda()
    slab = rb.alloc_slab(count, S)
    nodes = rb.alloc_nodes(count)
    rb.frame(payloads, plen, slab)
    rb.encode(slab, S)
    rb.merkle(slab, S, nodes)
    ds = max(rb.dslots, 1)
    digests = torch.zeros((count, n, ds, 32), dtype=torch.uint8, device="cuda")
    ndig = torch.zeros((count, n), dtype=torch.uint8, device="cuda")
    rb.proofs(nodes, digests, ndig)
    return rb, S, pay, slab, nodes, digests, ndig


def encode_all(torch, rb, S, slab, nodes, digests, ndig, variant=0):
    count, n = slab.shape[0], rb.n
    slot = rb.wire_slot(S)
    out = torch.full((count * n, slot), 0xEE, dtype=torch.uint8, device="cuda")
    mlen = torch.zeros(count * n, dtype=torch.int32, device="cuda")
    rb.wire_encode(slab, S, digests, ndig, nodes[:, -1, :], out, mlen, variant=variant)
    return out, mlen


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available()
    return torch


def test_wire_golden_foo(torch_cuda):
    torch = torch_cuda
    w = json.load(open(os.path.join(G, "wire_vectors.json")))
    rb = hb.RbcBatch(4, device=0)
    payloads = torch.zeros((1, 16), dtype=torch.uint8, device="cuda")
    payloads[0, :3] = torch.tensor(list(b"Foo"), dtype=torch.uint8)
    S = hb.shard_len(3, rb.k)
    slab = rb.alloc_slab(1, S)
    nodes = rb.alloc_nodes(1)
    rb.frame(payloads, 3, slab)
    rb.encode(slab, S)
    rb.merkle(slab, S, nodes)
    digests = torch.zeros((1, 4, rb.dslots, 32), dtype=torch.uint8, device="cuda")
    ndig = torch.zeros((1, 4), dtype=torch.uint8, device="cuda")
    rb.proofs(nodes, digests, ndig)
    out, mlen = encode_all(torch, rb, S, slab, nodes, digests, ndig)
    torch.cuda.synchronize()
    o, ml = out.cpu().numpy(), mlen.cpu().numpy()
    for j in range(4):
        assert o[j, : ml[j]].tobytes().hex() == w["value_msgs"][str(j)]
        assert not o[j, ml[j]:].any(), "slot padding must be zero"


@pytest.mark.parametrize("n,plen,count,variant", [(4, 1000, 3, 0), (7, 333, 2, 1), (16, 6001, 2, 0),
                                                  (64, 20000, 2, 1), (250, 5000, 1, 0),
                                                  (1, 17, 2, 0)])
def test_wire_encode_decode_vs_oracle(torch_cuda, n, plen, count, variant):
    torch = torch_cuda
    rb, S, pay, slab, nodes, digests, ndig = proposer_side(torch, n, plen, count, 31 + n)
    out, mlen = encode_all(torch, rb, S, slab, nodes, digests, ndig, variant)
    torch.cuda.synchronize()
    o, ml = out.cpu().numpy(), mlen.cpu().numpy()
    sl, nd = slab.cpu().numpy(), nodes.cpu().numpy()
    for i in range(count):
        root = nd[i, -1].tobytes()
        for j in range(n):
            p = orc.merkle_proof(nd[i], n, j)
            ref = orc.bincode_message(variant, sl[i, j, :S].tobytes(), j, [d.tobytes() for d in p],
                                      root)
            g = i * n + j
            assert ml[g] == len(ref) and o[g, : ml[g]].tobytes() == ref, (n, i, j)
    # decode back into slab-shaped rows and the proof fields
    nmsg = count * n
    stride = rb.stride_for(S)
    vals = torch.full((nmsg, stride), 0x77, dtype=torch.uint8, device="cuda")
    vlen, idx, var, st = (torch.zeros(nmsg, dtype=torch.int32, device="cuda") for _ in range(4))
    dg = torch.zeros((nmsg, max(rb.dslots, 1), 32), dtype=torch.uint8, device="cuda")
    ndo = torch.zeros(nmsg, dtype=torch.uint8, device="cuda")
    rts = torch.zeros((nmsg, 32), dtype=torch.uint8, device="cuda")
    rb.wire_decode(out, mlen, vals, vlen, idx, dg, ndo, rts, var, st)
    torch.cuda.synchronize()
    assert (st.cpu() == 0).all() and (var.cpu() == variant).all() and (vlen.cpu() == S).all()
    assert np.array_equal(idx.cpu().numpy(), np.tile(np.arange(n), count))
    v = vals.cpu().numpy().reshape(count, n, stride)
    assert np.array_equal(v[:, :, :S], sl[:, :, :S]) and not v[:, :, S:].any()
    assert np.array_equal(ndo.cpu().numpy().reshape(count, n), ndig.cpu().numpy())
    if rb.dslots:
        d = dg.cpu().numpy().reshape(count, n, rb.dslots, 32)
        ref_d = digests.cpu().numpy()
        for i in range(count):
            for j in range(n):
                k = int(ndig[i, j])
                assert np.array_equal(d[i, j, :k], ref_d[i, j, :k])
    assert np.array_equal(rts.cpu().numpy().reshape(count, n, 32),
                          np.repeat(nd[:, -1][:, None, :], n, axis=1))


def test_wire_decode_errors_and_digest_variants(torch_cuda):
    torch = torch_cuda
    n = 16
    rb, S, pay, slab, nodes, digests, ndig = proposer_side(torch, n, 3000, 1, 5)
    out, mlen = encode_all(torch, rb, S, slab, nodes, digests, ndig)
    slot = out.shape[1]
    ml = mlen.clone()
    ml[0] -= 1                                   # truncated root
    out[1, 0] = 9                                # unknown variant
    out[2, 20 + S] = rb.dslots + 1               # more digests than levels
    ml[3] = 30                                   # truncated inside the value
    root = nodes[0, -1].cpu().numpy().tobytes()
    for g, name in [(4, "Ready"), (5, "CanDecode"), (6, "EchoHash")]:
        m = orc.bincode_message(name, root=root)
        out[g].zero_()
        out[g, : len(m)] = torch.tensor(list(m), dtype=torch.uint8)
        ml[g] = len(m)
    nmsg = n

    def decode(msgs, lens, stride):
        vals = torch.zeros((nmsg, stride), dtype=torch.uint8, device="cuda")
        vlen, idx, var, st = (torch.zeros(nmsg, dtype=torch.int32, device="cuda") for _ in range(4))
        dg = torch.zeros((nmsg, rb.dslots, 32), dtype=torch.uint8, device="cuda")
        ndo = torch.zeros(nmsg, dtype=torch.uint8, device="cuda")
        rts = torch.zeros((nmsg, 32), dtype=torch.uint8, device="cuda")
        rb.wire_decode(msgs, lens, vals, vlen, idx, dg, ndo, rts, var, st)
        torch.cuda.synchronize()
        return st.cpu().tolist(), var.cpu().tolist(), rts.cpu().numpy()

    s, var, rts = decode(out, ml, rb.stride_for(S))
    assert s[0] == 70 and s[1] == 71 and s[2] == 72 and s[3] == 70
    assert s[4:7] == [0, 0, 0] and var[4:7] == [2, 3, 4]
    for g in (4, 5, 6):
        assert rts[g].tobytes() == root
    assert all(x == 0 for x in s[7:]), s
    # a value longer than the batch's rows is reported, not truncated
    pristine, plen_ = encode_all(torch, rb, S, slab, nodes, digests, ndig)
    s, _, _ = decode(pristine, plen_, rb.stride_for(S) - 16)
    assert s == [72] * n
    assert slot % 16 == 0
