"""GPU parity of the round-2 entry points (include/hbrbc.h): blocked row
layouts (hbrbc_*_rows), Merkle leaves out of Proof::validate and decodes that
reuse them (known_leaves), the decode-matrix cache (rse's per-pattern
decode-matrix LRU, behind broadcast.rs:684) and pattern-specialised decoders.
Every comparison is bit-exact against the plain layout, the oracle
(oracle/pyoracle.py) or a round trip."""
import numpy as np
import pytest

import hbbft_amd as hb
from oracle import pyoracle as orc

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available(), "gpu tests need an MI355X"
    return torch


def payloads(torch, seed, count, plen):
    pay = np.stack([orc.gen_payload(seed, i, plen) for i in range(count)])
    t = torch.zeros((count, max(16, (plen + 15) // 16 * 16)), dtype=torch.uint8, device="cuda")
    t[:, :plen] = torch.from_numpy(pay).cuda()
    return pay, t


def random_present(rng, count, n, n_erase):
    pres = np.ones((count, n), np.uint8)
    for i in range(count):
        pres[i, rng.permutation(n)[:n_erase]] = 0
    return pres


def blocked(torch, rb, count, S, R):
    """A [G][count][R][stride] slab and its (shard_stride, rpb, block_stride, inst_stride)."""
    st = rb.stride_for(S)
    G = -(-rb.n // R)
    buf = torch.full((G, count, R, st), 0x5A, dtype=torch.uint8, device="cuda")
    return buf, (st, R, count * R * st, R * st)


def row(buf, j, i, R):
    return buf[j // R, i, j % R]


@pytest.mark.parametrize("n,R,plen,count", [(64, 8, 20000, 3), (64, 32, 777, 4), (10, 3, 1500, 3),
                                            (128, 16, 6000, 2), (16, 5, 4099, 3)])
def test_blocked_layout_matches_plain(torch_cuda, n, R, plen, count):
    """frame+encode, Merkle, validate (with leaves out) and decode (with and
    without known leaves) in a blocked layout give the plain layout's bytes."""
    torch = torch_cuda
    f = (n - 1) // 3
    rb = hb.RbcBatch(n, f, device=0)
    S = hb.shard_len(plen, rb.k)
    pay, p = payloads(torch, 31, count, plen)
    plain = rb.alloc_slab(count, S)
    nodes = rb.alloc_nodes(count)
    rb.frame_encode(p, plen, plain)
    rb.merkle(plain, S, nodes)
    buf, (st, rpb, bst, ist) = blocked(torch, rb, count, S, R)
    rb.frame_encode_rows(p, plen, buf, count, st, rpb, bst, ist)
    nodes_b = rb.alloc_nodes(count)
    rb.merkle_rows(buf, S, count, st, rpb, bst, ist, nodes_b)
    torch.cuda.synchronize()
    for i in range(count):
        for j in range(n):
            assert torch.equal(row(buf, j, i, R)[:S], plain[i, j, :S]), (i, j)
            assert not row(buf, j, i, R)[S:].any(), "padding must be zero"
    assert torch.equal(nodes_b, nodes)
    # proofs, then validate every row of the blocked slab with leaves out
    ds = max(rb.dslots, 1)
    dig = torch.zeros((count, n, ds, 32), dtype=torch.uint8, device="cuda")
    ndig = torch.zeros((count, n), dtype=torch.uint8, device="cuda")
    rb.proofs(nodes, dig, ndig)
    ok = torch.zeros((count, n), dtype=torch.uint8, device="cuda")
    leaves = rb.alloc_nodes(count)
    leaves.fill_(0xEE)
    rows = torch.arange(n, dtype=torch.int32, device="cuda")
    rb.validate_layout(buf, S, count, n, st, rpb, bst, ist, dig, ndig, n, nodes[:, -1, :], ok,
                       rows=rows, leaf_out=leaves)
    torch.cuda.synchronize()
    assert ok.all()
    assert torch.equal(leaves[:, :n], nodes[:, :n])
    # decode from f random erasures (garbage in the erased rows), both ways
    rng = np.random.default_rng(n + R)
    pres = random_present(rng, count, n, f)
    pres_d = torch.from_numpy(pres).cuda()
    ostride = max(16, (rb.k * S + 15) // 16 * 16)
    for known in (False, True):
        rec = buf.clone()
        for i in range(count):
            for j in range(n):
                if not pres[i, j]:
                    row(rec, j, i, R)[:S] = 0xA5
        nodes2 = rb.alloc_nodes(count)
        nodes2.fill_(0x33)
        if known:   # the leaves the receiver computed when it validated the present rows
            nodes2[:, :n] = torch.where(pres_d.bool()[:, :, None], leaves[:, :n], nodes2[:, :n])
        out = torch.full((count, ostride), 0xEE, dtype=torch.uint8, device="cuda")
        plo = torch.zeros(count, dtype=torch.int32, device="cuda")
        status = torch.zeros(count, dtype=torch.int32, device="cuda")
        rb.decode_rows(rec, S, count, st, rpb, bst, ist, pres_d, nodes[:, -1, :].clone(), nodes2,
                       out, plo, status, known_leaves=known)
        torch.cuda.synchronize()
        assert (status.cpu() == 0).all() and (plo.cpu() == plen).all()
        assert torch.equal(out[:, :plen].cpu(), torch.from_numpy(pay))
        assert torch.equal(rec, buf) and torch.equal(nodes2, nodes), known


def test_unframe_zero_fills_past_payload(torch_cuda):
    """Every byte of a payload row past the decoded length is written 0, and a
    failed instance's whole row is 0 (hbrbc.h, decode_from_shards)."""
    torch = torch_cuda
    n, plen, count = 16, 3001, 3
    f = 5
    rb = hb.RbcBatch(n, f, device=0)
    S = hb.shard_len(plen, rb.k)
    pay, p = payloads(torch, 5, count, plen)
    slab = rb.alloc_slab(count, S)
    nodes = rb.alloc_nodes(count)
    rb.frame_encode(p, plen, slab)
    rb.merkle(slab, S, nodes)
    roots = nodes[:, -1, :].clone()
    roots[2, 0] ^= 1                       # instance 2: root mismatch
    present = torch.ones((count, n), dtype=torch.uint8, device="cuda")
    ostride = (rb.k * S + 15) // 16 * 16 + 64
    out = torch.full((count, ostride), 0xEE, dtype=torch.uint8, device="cuda")
    plo = torch.zeros(count, dtype=torch.int32, device="cuda")
    status = torch.zeros(count, dtype=torch.int32, device="cuda")
    rb.decode(slab, S, present, roots, rb.alloc_nodes(count), out, plo, status)
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    need = (rb.k * S - 4 + 15) // 16 * 16
    assert status.cpu().tolist() == [0, 0, 65]
    assert np.array_equal(o[0, :plen], pay[0]) and not o[0, plen:need].any()
    assert not o[2, :need].any()
    assert (o[:, need:] == 0xEE).all()     # nothing past the documented row


def test_decode_cache_reuses_one_pattern(torch_cuda):
    """Instances that share an erasure pattern share one decode matrix, within
    a call and across calls; a new pattern takes a new slot."""
    torch = torch_cuda
    n, plen, count = 64, 5000, 64
    f = 21
    rb = hb.RbcBatch(n, f, device=0)
    k = rb.k
    S = hb.shard_len(plen, k)
    pay, p = payloads(torch, 8, count, plen)
    slab = rb.alloc_slab(count, S)
    nodes = rb.alloc_nodes(count)
    rb.frame_encode(p, plen, slab)
    rb.merkle(slab, S, nodes)
    rb.reserve(count)
    rb.decode_cache_clear()
    ostride = (k * S + 15) // 16 * 16

    def decode(pres_np):
        pres = torch.from_numpy(pres_np).cuda()
        rec = slab.clone()
        rec[pres == 0] = 0xA5
        out = torch.zeros((count, ostride), dtype=torch.uint8, device="cuda")
        plo = torch.zeros(count, dtype=torch.int32, device="cuda")
        st = torch.zeros(count, dtype=torch.int32, device="cuda")
        nodes2 = rb.alloc_nodes(count)
        rb.decode(rec, S, pres, nodes[:, -1, :].clone(), nodes2, out, plo, st)
        torch.cuda.synchronize()
        assert (st.cpu() == 0).all()
        assert torch.equal(out[:, :plen].cpu(), torch.from_numpy(pay))
        assert torch.equal(rec, slab) and torch.equal(nodes2, nodes)

    worst = np.zeros((count, n), np.uint8)
    worst[:, k:2 * k] = 1                  # every data row and 20 parity rows missing
    decode(worst)
    assert rb.decode_cache_fill() == 1
    decode(worst)
    assert rb.decode_cache_fill() == 1     # reused across calls
    other = worst.copy()
    other[: count // 2, 0] = 1             # half the instances: a second pattern
    decode(other)
    assert rb.decode_cache_fill() == 2


def test_decode_cache_full_table_uses_private_slots(torch_cuda):
    """Once the shared table is half full new patterns are decoded in
    per-instance private slots, still bit-exact (round trip)."""
    torch = torch_cuda
    n, plen, count = 64, 600, 1024
    f = 21
    rb = hb.RbcBatch(n, f, device=0)
    S = hb.shard_len(plen, rb.k)
    pay, p = payloads(torch, 12, count, plen)
    slab = rb.alloc_slab(count, S)
    nodes = rb.alloc_nodes(count)
    rb.frame_encode(p, plen, slab)
    rb.merkle(slab, S, nodes)
    rb.reserve(count)                      # 2048 shared slots
    rb.decode_cache_clear()
    rng = np.random.default_rng(3)
    ostride = (rb.k * S + 15) // 16 * 16
    fills = []
    for _ in range(3):
        pres = torch.from_numpy(random_present(rng, count, n, f)).cuda()
        rec = slab.clone()
        rec[pres == 0] = 0
        out = torch.zeros((count, ostride), dtype=torch.uint8, device="cuda")
        plo = torch.zeros(count, dtype=torch.int32, device="cuda")
        st = torch.zeros(count, dtype=torch.int32, device="cuda")
        nodes2 = rb.alloc_nodes(count)
        rb.decode(rec, S, pres, nodes[:, -1, :].clone(), nodes2, out, plo, st)
        torch.cuda.synchronize()
        assert (st.cpu() == 0).all()
        assert torch.equal(out[:, :plen].cpu(), torch.from_numpy(pay))
        assert torch.equal(rec, slab)
        fills.append(rb.decode_cache_fill())
    assert fills[0] == count and fills[1] == count and fills[2] == count


@pytest.mark.parametrize("n,pattern", [(250, "worst"), (16, "f"), (64, "right")])
def test_specialised_decoder_vs_generic(torch_cuda, monkeypatch, tmp_path, n, pattern):
    """A pattern-specialised XOR-network decoder (hbrbc_decoder_specialise)
    writes the generic kernel's bytes; instances of other patterns in the same
    call still take the generic kernel."""
    torch = torch_cuda
    if pattern != "worst":
        monkeypatch.setenv("HBRBC_JIT_DIR", str(tmp_path))   # compiled here
    f = (n - 1) // 3
    k = n - 2 * f
    plen, count = 4000, 6
    rng = np.random.default_rng(n)
    if pattern == "worst":
        pat = np.array([1 if k <= i < 2 * k else 0 for i in range(n)], np.uint8)
    elif pattern == "f":
        pat = np.ones(n, np.uint8)
        pat[rng.permutation(n)[:f]] = 0
    else:
        pat = np.array([0 if 1 <= i <= f else 1 for i in range(n)], np.uint8)
    results = []
    for spec in (True, False):
        rb = hb.RbcBatch(n, f, device=0)
        if spec:
            rb.specialise_decoder(pat)
        S = hb.shard_len(plen, rb.k)
        pay, p = payloads(torch, 21, count, plen)
        slab = rb.alloc_slab(count, S)
        nodes = rb.alloc_nodes(count)
        rb.frame_encode(p, plen, slab)
        rb.merkle(slab, S, nodes)
        pres = np.tile(pat, (count, 1))
        pres[count - 2:] = random_present(rng, 2, n, f)   # two other patterns
        pres_d = torch.from_numpy(pres).cuda()
        rec = slab.clone()
        rec[pres_d == 0] = 0x11
        st = torch.zeros(count, dtype=torch.int32, device="cuda")
        rb.reconstruct(rec, S, pres_d, st)
        torch.cuda.synchronize()
        assert (st.cpu() == 0).all()
        assert torch.equal(rec[:, :, :S], slab[:, :, :S])
        results.append(rec.cpu())
    assert torch.equal(results[0], results[1])


def test_validate_rows_subset_with_indices(torch_cuda):
    """A row list validates only the listed rows; the claimed index comes
    from `indices`; leaves of listed rows only are written."""
    torch = torch_cuda
    n, plen, count = 16, 999, 3
    rb = hb.RbcBatch(n, 5, device=0)
    S = hb.shard_len(plen, rb.k)
    pay, p = payloads(torch, 2, count, plen)
    slab = rb.alloc_slab(count, S)
    nodes = rb.alloc_nodes(count)
    rb.frame_encode(p, plen, slab)
    rb.merkle(slab, S, nodes)
    dig = torch.zeros((count, n, rb.dslots, 32), dtype=torch.uint8, device="cuda")
    ndig = torch.zeros((count, n), dtype=torch.uint8, device="cuda")
    rb.proofs(nodes, dig, ndig)
    sel = [1, 4, 9, 15]
    rows = torch.tensor(sel, dtype=torch.int32, device="cuda")
    idx = torch.tensor([sel] * count, dtype=torch.int32, device="cuda")
    idx[1, 2] = 8                          # claims another index: rejected
    ok = torch.zeros((count, len(sel)), dtype=torch.uint8, device="cuda")
    leaves = rb.alloc_nodes(count)
    leaves.zero_()
    st = rb.stride_for(S)
    rb.validate_layout(slab, S, count, len(sel), st, 0, 0, n * st, dig, ndig, n,
                       nodes[:, -1, :], ok, rows=rows, indices=idx, leaf_out=leaves)
    torch.cuda.synchronize()
    exp = np.ones((count, len(sel)), np.uint8)
    exp[1, 2] = 0
    assert np.array_equal(ok.cpu().numpy(), exp)
    lv = leaves.cpu().numpy()
    nd = nodes.cpu().numpy()
    for j in range(n):
        if j in sel:
            assert np.array_equal(lv[:, j], nd[:, j])
        else:
            assert not lv[:, j].any()


@pytest.mark.parametrize("count,n_erase", [(2, 21), (1500, 42), (3000, 30), (3000, 42), (6000, 42)])
def test_rebuilt_row_list_lengths(torch_cuda, count, n_erase):
    """A decode with known leaves re-hashes only the rebuilt rows, through
    the balanced list kernel (leaf_hash_list_mix_kernel, kernels.hip) below
    2^18 listed rows of the worst case.  The list lengths here take each of its
    branches per CU share: pair-lane only (<= 128), one-lane only (129..256),
    one round plus a pair-lane remainder (<= 384), and the long-list form
    (> 384 per CU: one-lane rounds of 512 on all eight waves, ~490 and ~980
    per CU here).  The decode tree must come out as the proposer's tree."""
    torch = torch_cuda
    n, f, plen = 64, 21, 2000
    rb = hb.RbcBatch(n, f, device=0)
    S = hb.shard_len(plen, rb.k)
    pay, p = payloads(torch, 77, count, plen)
    slab = rb.alloc_slab(count, S)
    nodes = rb.alloc_nodes(count)
    rb.frame_encode(p, plen, slab)
    rb.merkle(slab, S, nodes)
    rng = np.random.default_rng(count + n_erase)
    pres = np.ones((count, n), np.uint8)
    np.put_along_axis(pres, np.argsort(rng.random((count, n)), axis=1)[:, :n_erase], 0, axis=1)
    pres_d = torch.from_numpy(pres).cuda()
    keep = pres_d.bool()
    rec = slab.clone()
    rec[~keep] = 0xA5                              # garbage in the erased rows
    nodes2 = rb.alloc_nodes(count)
    nodes2.fill_(0x33)
    nodes2[:, :n] = torch.where(keep[:, :, None], nodes[:, :n], nodes2[:, :n])
    ostride = max(16, (rb.k * S + 15) // 16 * 16)
    out = torch.zeros((count, ostride), dtype=torch.uint8, device="cuda")
    plo = torch.zeros(count, dtype=torch.int32, device="cuda")
    status = torch.ones(count, dtype=torch.int32, device="cuda")
    rb.decode(rec, S, pres_d, nodes[:, -1, :].clone(), nodes2, out, plo, status, known_leaves=True)
    torch.cuda.synchronize()
    assert (status == 0).all() and (plo == plen).all()
    assert torch.equal(rec, slab) and torch.equal(nodes2, nodes)
    assert torch.equal(out[:, :plen].cpu(), torch.from_numpy(pay))
