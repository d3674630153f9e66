"""GPU parity of the f4 path (threshold-decrypt share verification,
hbbft_amd/csrc/pairing.hip) against the BLS12-381 restatement
(oracle/bls_oracle.py) and its golden vectors: GT values bit-exact, check
outcomes exact, invalid encodings rejected per item."""
import json
import os
import random

import numpy as np
import pytest

from oracle import bls_oracle as B

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = json.load(open(os.path.join(ROOT, "tests", "golden", "bls_vectors.json")))

pytestmark = pytest.mark.gpu


def _t(rows, width):
    import torch
    a = np.frombuffer(b"".join(rows), np.uint8).reshape(len(rows), width)
    return torch.from_numpy(a.copy()).to("cuda:0")


def test_pairing_batch_matches_golden():
    from hbbft_amd import threshold as T
    vs = GOLD["pairings"]
    g1 = _t([bytes.fromhex(v["g1"]) for v in vs], 96)
    g2 = _t([bytes.fromhex(v["g2"]) for v in vs], 192)
    gt, st = T.pairing_batch(g1, g2)
    assert st.cpu().tolist() == [0] * len(vs)
    for i, v in enumerate(vs):
        assert bytes(gt[i].cpu().numpy()).hex() == v["gt"], i


def test_pairing_batch_infinity_and_invalid():
    from hbbft_amd import threshold as T
    one = B.gt_bytes(B.F12_ONE)
    e = B.gt_bytes(B.pairing(B.G1_GEN, B.G2_GEN))
    g1_ok, g2_ok = B.g1_bytes(B.G1_GEN), B.g2_bytes(B.G2_GEN)
    off_curve = bytearray(g1_ok)
    off_curve[-1] ^= 1
    big = bytes.fromhex("%096x" % B.P) + g1_ok[48:]          # x = p: not canonical
    compressed = bytes([g1_ok[0] | 0x80]) + g1_ok[1:]
    inf_dirty = b"\x40" + b"\0" * 94 + b"\x01"
    cases = [(g1_ok, g2_ok, e, 0), (B.g1_bytes(None), g2_ok, one, 0),
             (g1_ok, B.g2_bytes(None), one, 0), (bytes(off_curve), g2_ok, one, 2),
             (big, g2_ok, one, 2), (compressed, g2_ok, one, 2), (inf_dirty, g2_ok, one, 2)]
    g1 = _t([c[0] for c in cases], 96)
    g2 = _t([c[1] for c in cases], 192)
    gt, st = T.pairing_batch(g1, g2)
    assert st.cpu().tolist() == [c[3] for c in cases]
    for i, c in enumerate(cases):
        assert bytes(gt[i].cpu().numpy()) == c[2], i


def test_check_batch_golden_and_mixed():
    from hbbft_amd import threshold as T
    cs = GOLD["checks"]
    items = [(bytes.fromhex(c["a"]), bytes.fromhex(c["c"]), bytes.fromhex(c["b"]),
              bytes.fromhex(c["d"])) for c in cs]
    assert T.verify_decryption_shares(items) == [c["expect"] for c in cs]
    for c in cs:
        assert T.pairing_check(*(bytes.fromhex(c[k]) for k in "abcd")) == c["expect"]


def test_ciphertext_verify_shape():
    from hbbft_amd import threshold as T
    r_enc, h = 0x1234, 0x99
    H = B.g2_mul(B.G2_GEN, h)
    U = B.g1_mul(B.G1_GEN, r_enc)
    W = B.g2_mul(H, r_enc)
    W_bad = B.g2_mul(H, r_enc + 1)
    got = T.verify_ciphertexts([(B.g1_bytes(U), B.g2_bytes(W), B.g2_bytes(H)),
                                (B.g1_bytes(U), B.g2_bytes(W_bad), B.g2_bytes(H))])
    assert got == [True, False]


def test_check_batch_bilinearity_at_size():
    """4096 checks e(a P_i, b Q_j) == e(b P_i, a Q_j) (true) and with b+1 on one
    side (false), from small pools of oracle-built points; exact outcomes."""
    from hbbft_amd import threshold as T
    rng = random.Random(7)
    sa = [rng.randrange(1, B.R) for _ in range(4)]
    sb = [rng.randrange(1, B.R) for _ in range(4)]
    P = B.g1_mul(B.G1_GEN, rng.randrange(1, B.R))
    Q = B.g2_mul(B.G2_GEN, rng.randrange(1, B.R))
    g1p = {s: B.g1_bytes(B.g1_mul(P, s)) for s in sa + sb + [x + 1 for x in sb]}
    g2p = {s: B.g2_bytes(B.g2_mul(Q, s)) for s in sa + sb}
    items, expect = [], []
    for i in range(4096):
        a, b = sa[i % 4], sb[(i // 4) % 4]
        good = (i // 16) % 3 != 0
        c_s = b if good else b + 1
        items.append((g1p[a], g2p[b], g1p[c_s], g2p[a]))
        expect.append(good)
    g1 = _t([x for it in items for x in (it[0], it[2])], 96)
    g2 = _t([x for it in items for x in (it[1], it[3])], 192)
    ok = T.pairing_check_batch(g1, g2).cpu().tolist()
    assert ok == [1 if e else 0 for e in expect]


def test_per_call_rejects_invalid_point():
    from hbbft_amd import RseError
    from hbbft_amd import threshold as T
    bad = bytearray(B.g1_bytes(B.G1_GEN))
    bad[-1] ^= 1
    with pytest.raises(RseError):
        T.pairing_check(bytes(bad), B.g2_bytes(B.G2_GEN), B.g1_bytes(B.G1_GEN),
                        B.g2_bytes(B.G2_GEN))


@pytest.mark.parametrize("multi", ["1", "0"])
def test_check_batch_infinity_and_invalid(monkeypatch, multi):
    """Checks whose points include infinity (that pairing is 1) or an invalid
    encoding (outcome 2), on the one-lane-per-check multi-Miller kernel
    (default) and on one lane per pairing (HBRBC_PAIR_MULTI=0)."""
    from hbbft_amd import threshold as T
    monkeypatch.setenv("HBRBC_PAIR_MULTI", multi)
    P, Q = B.g1_mul(B.G1_GEN, 3), B.g2_mul(B.G2_GEN, 5)
    P15 = B.g1_mul(B.G1_GEN, 15)
    inf1, inf2 = B.g1_bytes(None), B.g2_bytes(None)
    bad = bytearray(B.g1_bytes(P))
    bad[-1] ^= 1
    cases = [
        ((B.g1_bytes(P), B.g2_bytes(Q), B.g1_bytes(P15), B.g2_bytes(B.G2_GEN)), 1),
        ((inf1, B.g2_bytes(Q), B.g1_bytes(P), inf2), 1),          # 1 == 1
        ((B.g1_bytes(P), B.g2_bytes(Q), inf1, B.g2_bytes(Q)), 0),  # e(P,Q) != 1
        ((inf1, inf2, inf1, inf2), 1),
        ((bytes(bad), B.g2_bytes(Q), B.g1_bytes(P), B.g2_bytes(Q)), 2),
        ((B.g1_bytes(P), B.g2_bytes(Q), B.g1_bytes(P), B.g2_bytes(Q)), 1),
    ]
    g1 = _t([x for (a, b, c, d), _ in cases for x in (a, c)], 96)
    g2 = _t([x for (a, b, c, d), _ in cases for x in (b, d)], 192)
    assert T.pairing_check_batch(g1, g2).cpu().tolist() == [e for _, e in cases]


def test_pairing_batch_at_size_vs_c_restatement():
    """4096 GT values (a 64 x 64 grid of pool points) bit-exact against the C
    restatement (oracle/bls_pairing.c, itself pinned to the Python oracle's
    golden bytes in tests/test_bls_oracle.py)."""
    import os
    from hbbft_amd import threshold as T
    from oracle import bls_c
    rng = random.Random(11)
    P = [B.g1_bytes(B.g1_mul(B.G1_GEN, rng.randrange(1, B.R))) for _ in range(64)]
    Q = [B.g2_bytes(B.g2_mul(B.G2_GEN, rng.randrange(1, B.R))) for _ in range(64)]
    g1b = b"".join(P[i % 64] for i in range(4096))
    g2b = b"".join(Q[i // 64] for i in range(4096))
    gt, st = T.pairing_batch(_t([g1b[96 * i:96 * i + 96] for i in range(4096)], 96),
                             _t([g2b[192 * i:192 * i + 192] for i in range(4096)], 192))
    ref_gt, ref_st = bls_c.pairing_batch(g1b, g2b, 4096, min(16, os.cpu_count() or 1))
    assert st.cpu().numpy().tobytes() == ref_st == b"\0" * 4096
    assert gt.cpu().numpy().tobytes() == ref_gt


def test_prepared_checks_match_plain_checks():
    """Checks against prepared G2 points (the crate's G2Prepared, shared by all
    shares of a ciphertext) give exactly the outcomes of the plain checks:
    valid and tampered shares, several ciphertexts, infinity and invalid
    points, and the grouped verify_decryption_shares helper."""
    from hbbft_amd import threshold as T
    rng = random.Random(21)
    cts, shares, expect = [], [], []
    for j in range(3):
        h, r_enc = rng.randrange(1, B.R), rng.randrange(1, B.R)
        H = B.g2_mul(B.G2_GEN, h)
        U = B.g1_mul(B.G1_GEN, r_enc)
        W = B.g2_mul(H, r_enc)
        cts.append((B.g2_bytes(H), B.g2_bytes(W)))
        for s in range(5):
            sk = rng.randrange(1, B.R)
            share = B.g1_mul(U, sk)
            good = (s + j) % 3 != 0
            if not good:
                share = B.g1_add(share, B.G1_GEN)
            shares.append((j, B.g1_bytes(share), B.g1_bytes(B.g1_mul(B.G1_GEN, sk))))
            expect.append(good)
    # interleave the ciphertexts so grouping has work to do
    perm = list(range(len(shares)))
    rng.shuffle(perm)
    shares = [shares[i] for i in perm]
    expect = [expect[i] for i in perm]
    assert T.verify_decryption_shares_grouped(cts, shares) == expect
    plain = T.verify_decryption_shares([(s, pk, cts[j][0], cts[j][1]) for j, s, pk in shares])
    assert plain == expect
    # infinity / invalid prepared points and G1 points
    bad2 = bytearray(B.g2_bytes(B.G2_GEN))
    bad2[-1] ^= 1
    g2 = _t([B.g2_bytes(B.G2_GEN), B.g2_bytes(None), bytes(bad2)], 192)
    prep = T.g2_prepare(g2)
    P = B.g1_bytes(B.g1_mul(B.G1_GEN, 7))
    inf1 = B.g1_bytes(None)
    import torch
    g1 = _t([P, P, inf1, P, P, inf1, P, P], 96)
    ib = torch.tensor([0, 1, 0, 2], dtype=torch.int32, device="cuda:0")
    idd = torch.tensor([0, 0, 0, 0], dtype=torch.int32, device="cuda:0")
    # e(P,G)==e(P,G): 1;  e(inf,..)=1 vs e(P,G) != 1: 0;  e(P,G) vs e(inf,G)=1: 0;  invalid: 2
    assert T.pairing_check_prepared(g1, prep, 3, ib, idd).cpu().tolist() == [1, 0, 0, 2]
    # indices past the table (as uint32: -1 is 2^32-1) are invalid inputs, not reads
    ib2 = torch.tensor([0, 3, -1, 0], dtype=torch.int32, device="cuda:0")
    assert T.pairing_check_prepared(g1, prep, 3, ib2, idd).cpu().tolist() == [1, 2, 2, 1]


def test_g2_prepare_across_blocks():
    """The G2 preparation checks a point's order (block 2j) and computes its
    lines (block 2j + 1) in different waves (HB_G2_SPLIT): 130 points, so
    three block pairs and a ragged last one, with an off-curve, an
    off-subgroup and an infinity point at the block edges (63, 64, 129) and
    valid points elsewhere.  Prepared checks give exactly the plain checks'
    outcomes for every point, against a valid and a tampered G1 side."""
    import torch
    from hbbft_amd import threshold as T
    rng = random.Random(41)
    base = [B.g2_mul(B.G2_GEN, rng.randrange(1, B.R)) for _ in range(5)]
    pts = [B.g2_bytes(base[i % 5]) for i in range(130)]
    bad = bytearray(pts[63])
    bad[-1] ^= 1                                      # off the curve
    pts[63] = bytes(bad)
    _, (q0, _) = _off_subgroup_points()
    pts[64] = B.g2_bytes(q0)                          # on E', not in the subgroup
    pts[129] = B.g2_bytes(None)                       # infinity
    prep = T.g2_prepare(_t(pts, 192))
    a = B.g1_mul(B.G1_GEN, 5)
    P, P2 = B.g1_bytes(a), B.g1_bytes(B.g1_add(a, B.G1_GEN))
    idx = [0, 1, 62, 63, 64, 65, 127, 128, 129]
    # odd checks e(P, Q_k) == e(P, Q_k); even ones e(P, Q_k) == e(P + G, Q_(k+1))
    dix = [k if n % 2 else (k + 1) % 130 for n, k in enumerate(idx)]
    g1 = _t([x for n, k in enumerate(idx) for x in (P, P if n % 2 else P2)], 96)
    dev = "cuda:0"
    ib = torch.tensor(idx, dtype=torch.int32, device=dev)
    idd = torch.tensor(dix, dtype=torch.int32, device=dev)
    got = T.pairing_check_prepared(g1, prep, len(pts), ib, idd).cpu().tolist()
    g2 = _t([x for k, d in zip(idx, dix) for x in (pts[k], pts[d])], 192)
    ref = T.pairing_check_batch(g1, g2).cpu().tolist()
    assert got == ref == [0, 1, 2, 2, 2, 1, 0, 1, 0]


def test_prepared_keys_match_prepared_checks():
    """Checks against a table of prepared G1 keys (hbbft's pk_i, decoded and
    checked once) give exactly the outcomes of the same checks with both G1
    points decoded per check: valid and tampered shares, keys that are
    infinity, off the subgroup or non-canonical, and indices past either
    table (as uint32: -1 is 2^32-1), which are invalid inputs, not reads."""
    import torch
    from hbbft_amd import threshold as T
    rng = random.Random(33)
    cts, rows = [], []
    keys_sk = [rng.randrange(1, B.R) for _ in range(6)]
    keys = [B.g1_bytes(B.g1_mul(B.G1_GEN, sk)) for sk in keys_sk]
    (p0, _), _ = _off_subgroup_points()
    noncanon = bytearray(B.g1_bytes(B.g1_mul(B.G1_GEN, 3)))
    noncanon[0] = (noncanon[0] & 0xE0) | 0x1F   # x >= p (p's top byte is 0x1a; flags kept)
    keys += [B.g1_bytes(None), B.g1_bytes(p0), bytes(noncanon)]   # keys 6, 7, 8
    for j in range(2):
        h, r_enc = rng.randrange(1, B.R), rng.randrange(1, B.R)
        H = B.g2_mul(B.G2_GEN, h)
        U = B.g1_mul(B.G1_GEN, r_enc)
        W = B.g2_mul(H, r_enc)
        cts += [B.g2_bytes(H), B.g2_bytes(W)]
        for i in range(len(keys)):
            share = B.g1_mul(U, keys_sk[i] if i < 6 else 5)
            if (i + j) % 4 == 1:
                share = B.g1_add(share, B.G1_GEN)   # tampered
            rows.append((B.g1_bytes(share), i, 2 * j, 2 * j + 1))
    rows.append((rows[0][0], 9, 0, 1))            # key index past the table
    rows.append((rows[0][0], -1, 0, 1))
    rows.append((rows[0][0], 0, 4, 1))            # G2 index past the table
    prep = T.g2_prepare(_t(cts, 192))
    ktab = T.g1_prepare(_t(keys, 96))
    dev = "cuda:0"
    ib = torch.tensor([r[2] for r in rows], dtype=torch.int32, device=dev)
    idd = torch.tensor([r[3] for r in rows], dtype=torch.int32, device=dev)
    ic = torch.tensor([r[1] for r in rows], dtype=torch.int32, device=dev)
    got = T.pairing_check_prepared_keys(_t([r[0] for r in rows], 96), ktab, len(keys), ic, prep,
                                        len(cts), ib, idd).cpu().tolist()
    # the same checks with the key decoded per check (the key index clamped
    # for the rows whose index is out of range: their outcome must be 2)
    g1 = _t([x for r in rows for x in (r[0], keys[r[1] if 0 <= r[1] < len(keys) else 0])], 96)
    ref = T.pairing_check_prepared(g1, prep, len(cts), ib, idd).cpu().tolist()
    n = len(rows)
    assert got[:n - 3] == ref[:n - 3] and got[n - 3:] == [2, 2, 2]
    # the shares decoded beforehand too (hbrbc_pairing_check_prepared_pts):
    # the same outcomes, including invalid shares (off the subgroup,
    # non-canonical, infinity) decoded into the table
    bad_shares = [B.g1_bytes(p0), bytes(noncanon), B.g1_bytes(None)]
    sh = [r[0] for r in rows] + bad_shares
    ib2 = torch.cat([ib, torch.zeros(3, dtype=torch.int32, device=dev)])
    idd2 = torch.cat([idd, torch.ones(3, dtype=torch.int32, device=dev)])
    ic2 = torch.cat([ic, torch.zeros(3, dtype=torch.int32, device=dev)])
    sprep = T.g1_prepare(_t(sh, 96))
    pts = T.pairing_check_prepared_pts(sprep, len(sh), ktab, len(keys), ic2, prep, len(cts), ib2,
                                       idd2).cpu().tolist()
    ref2 = T.pairing_check_prepared_keys(_t(sh, 96), ktab, len(keys), ic2, prep, len(cts), ib2,
                                         idd2).cpu().tolist()
    assert pts == ref2 and pts[:n] == got and pts[n:n + 2] == [2, 2]
    assert ref[n - 1] == 2
    # valid keys: 1 unless tampered; invalid keys (infinity on one side gives 1
    # against a non-1 value, off-subgroup and non-canonical are invalid)
    for r, v in zip(rows[:n - 3], got[:n - 3]):
        i, j = r[1], r[2] // 2
        if i < 6:
            assert v == (0 if (i + j) % 4 == 1 else 1), (i, j, v)
        elif i == 6:
            assert v == 0
        else:
            assert v == 2


def _off_subgroup_points():
    """On-curve points outside the order-r subgroups (the crate's into_affine
    rejects them): a plain curve point of E / E', and a subgroup point plus a
    point of cofactor order ([r] of a curve point)."""
    p0, q0 = B.g1_curve_point(0x5EED), B.g2_curve_point(0x5EED)
    t1, t2 = B._smul(B.g1_add, p0, B.R), B._smul(B.g2_add, q0, B.R)
    p1 = B.g1_add(B.g1_mul(B.G1_GEN, 11), t1)
    q1 = B.g2_add(B.g2_mul(B.G2_GEN, 13), t2)
    for pt in (p0, p1):
        assert B.g1_on_curve(pt) and not B.g1_in_subgroup(pt)
    for pt in (q0, q1):
        assert B.g2_on_curve(pt) and not B.g2_in_subgroup(pt)
    return [p0, p1], [q0, q1]


@pytest.mark.parametrize("multi", ["1", "0"])
def test_points_outside_subgroup_are_invalid(monkeypatch, multi):
    """a point on the curve but outside the order-r subgroup (e.g.
    share + T, T of cofactor order) is an invalid input (status / outcome 2)
    in every form -- GT values, plain and multi-Miller checks, prepared G2
    points and the G1 points checked against them -- as the crate's
    deserialisation rejects it before any pairing."""
    import torch
    from hbbft_amd import threshold as T
    monkeypatch.setenv("HBRBC_PAIR_MULTI", multi)
    (p0, p1), (q0, q1) = _off_subgroup_points()
    G, Q = B.g1_bytes(B.g1_mul(B.G1_GEN, 5)), B.g2_bytes(B.g2_mul(B.G2_GEN, 7))
    one = B.gt_bytes(B.F12_ONE)
    rows = [(G, Q, 0), (B.g1_bytes(p0), Q, 2), (B.g1_bytes(p1), Q, 2), (G, B.g2_bytes(q0), 2),
            (G, B.g2_bytes(q1), 2)]
    gt, st = T.pairing_batch(_t([r[0] for r in rows], 96), _t([r[1] for r in rows], 192))
    assert st.cpu().tolist() == [r[2] for r in rows]
    for i in range(1, len(rows)):
        assert bytes(gt[i].cpu().numpy()) == one
    # checks e(a, b) == e(c, d): a valid pair, then one bad point in each slot
    good = (G, Q, G, Q)
    cases = [good]
    for slot, pt in ((0, B.g1_bytes(p1)), (1, B.g2_bytes(q1)), (2, B.g1_bytes(p0)),
                     (3, B.g2_bytes(q0))):
        c = list(good)
        c[slot] = pt
        cases.append(tuple(c))
    g1 = _t([x for a, b, c, d in cases for x in (a, c)], 96)
    g2 = _t([x for a, b, c, d in cases for x in (b, d)], 192)
    assert T.pairing_check_batch(g1, g2).cpu().tolist() == [1, 2, 2, 2, 2]
    # prepared: an off-subgroup G2 point is flagged at preparation, an
    # off-subgroup share when its check runs
    prep = T.g2_prepare(_t([Q, B.g2_bytes(q1)], 192))
    g1 = _t([G, G, G, G, B.g1_bytes(p1), G], 96)
    ib = torch.tensor([0, 1, 0], dtype=torch.int32, device="cuda:0")
    idd = torch.tensor([0, 0, 0], dtype=torch.int32, device="cuda:0")
    assert T.pairing_check_prepared(g1, prep, 2, ib, idd).cpu().tolist() == [1, 2, 2]
    # the helpers hbbft's callers use return False for such a share
    # (items are (share, pk_i, H, W): e(share, H) == e(pk_i, W))
    assert T.verify_decryption_shares([(B.g1_bytes(p1), G, Q, Q), (G, G, Q, Q)]) == [False, True]
