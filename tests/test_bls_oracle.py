"""CPU checks of the BLS12-381 restatement (oracle/bls_oracle.py) that the
f4 GPU parity tests compare against: generator coordinates,
field and Frobenius identities, the final-exponentiation chain against its
specification, bilinearity, and the committed golden vectors."""
import json
import os
import random

import pytest

from oracle import bls_oracle as B

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = json.load(open(os.path.join(ROOT, "tests", "golden", "bls_vectors.json")))


def test_generators_on_curve_and_in_r_torsion():
    assert B.g1_on_curve(B.G1_GEN) and B.g2_on_curve(B.G2_GEN)
    assert B.g1_mul(B.G1_GEN, B.R) is None
    assert B.g2_mul(B.G2_GEN, B.R) is None
    assert B.P % 6 == 1 and B.P % 4 == 3      # sextic twist, u^2 = -1 non-residue


def test_fp12_identities():
    rng = random.Random(1)
    a = [rng.randrange(B.P) for _ in range(12)]
    assert B.f12mul(a, B.f12inv(a)) == B.F12_ONE
    assert B.f12frob(a, 1) == B.f12pow(a, B.P)
    assert B.f12frob(a, 6) == B.f12conj(a)
    assert B.from_tower(B.to_tower(a)) == a


def test_final_exponentiation_chain_is_cube_of_reduced_pairing():
    """The crate's hard-part chain evaluates f^(3 (p^12-1)/r)."""
    rng = random.Random(2)
    f = [rng.randrange(B.P) for _ in range(12)]
    assert B.final_exponentiation(f) == B.final_exponentiation_plain(f, 3)
    assert B.final_exponentiation(f) != B.final_exponentiation_plain(f, 1)


def test_bilinear_nondegenerate_order_r():
    e = B.pairing(B.G1_GEN, B.G2_GEN)
    assert e != B.F12_ONE
    assert B.f12pow(e, B.R) == B.F12_ONE
    e6 = B.pairing(B.g1_mul(B.G1_GEN, 2), B.g2_mul(B.G2_GEN, 3))
    assert e6 == B.f12pow(e, 6)
    assert B.pairing(None, B.G2_GEN) == B.F12_ONE
    assert B.pairing(B.g1_neg(B.G1_GEN), B.G2_GEN) == B.f12inv(e)


def test_decryption_share_shapes():
    share, H, pk, W = B.decryption_share_case(5, 9, 3)
    assert B.pairing_check(share, H, pk, W)
    share, H, pk, W = B.decryption_share_case(5, 9, 3, tamper=True)
    assert not B.pairing_check(share, H, pk, W)


@pytest.mark.parametrize("idx", [0, 3])
def test_oracle_reproduces_golden(idx):
    v = GOLD["pairings"][idx]
    p1 = B.g1_mul(B.G1_GEN, v["g1_scalar"])
    q2 = B.g2_mul(B.G2_GEN, v["g2_scalar"])
    assert B.g1_bytes(p1).hex() == v["g1"] and B.g2_bytes(q2).hex() == v["g2"]
    assert B.gt_bytes(B.pairing(p1, q2)).hex() == v["gt"]


def test_golden_g1_encoding_of_generator_matches_product_constant():
    from hbbft_amd import threshold
    assert threshold.G1_ONE == B.g1_bytes(B.G1_GEN)


def test_c_restatement_matches_golden_and_python():
    """oracle/bls_pairing.c (the bench's f4 CPU baseline) against the golden GT
    bytes of the Python restatement, the check outcomes, and the same
    encoding rejections as the product."""
    from oracle import bls_c
    for v in GOLD["pairings"]:
        gt, st = bls_c.pairing(bytes.fromhex(v["g1"]), bytes.fromhex(v["g2"]))
        assert st == 0 and gt.hex() == v["gt"]
    for c in GOLD["checks"] + GOLD["bench_pool"][:8]:
        assert bls_c.check(*(bytes.fromhex(c[k]) for k in "abcd")) == (1 if c["expect"] else 0)
    g1, g2 = B.g1_bytes(B.G1_GEN), B.g2_bytes(B.G2_GEN)
    bad = bytearray(g1)
    bad[-1] ^= 1
    assert bls_c.check(bytes(bad), g2, g1, g2) == 2
    assert bls_c.check(bytes([g1[0] | 0x80]) + g1[1:], g2, g1, g2) == 2
    gt, st = bls_c.pairing(B.g1_bytes(None), g2)
    assert st == 0 and gt == B.gt_bytes(B.F12_ONE)


def test_endomorphism_subgroup_tests_match_r_torsion():
    """The HIP decoders test subgroup membership with Scott's endomorphism
    checks (phi(P) == -[x^2] P on G1, psi(Q) == [x] Q on G2); the crate checks
    [r] P == O.  Both agree on subgroup points and on on-curve points outside
    the subgroup (plain curve points, and subgroup points plus a point of
    cofactor order); beta is the cube root the generator selects."""
    rng = random.Random(5)
    assert B.g1_endo_test(B.G1_GEN) and B.g2_endo_test(B.G2_GEN)
    other_beta = B.BETA * B.BETA % B.P
    assert (other_beta * B.G1_GEN[0] % B.P, B.G1_GEN[1]) != B.g1_neg(
        B._smul(B.g1_add, B.G1_GEN, B.X_ABS * B.X_ABS))
    for _ in range(2):
        p = B.g1_mul(B.G1_GEN, rng.randrange(1, B.R))
        q = B.g2_mul(B.G2_GEN, rng.randrange(1, B.R))
        assert B.g1_in_subgroup(p) and B.g1_endo_test(p)
        assert B.g2_in_subgroup(q) and B.g2_endo_test(q)
    for seed in (1, 0x5EED):
        p0, q0 = B.g1_curve_point(seed), B.g2_curve_point(seed)
        t1, t2 = B._smul(B.g1_add, p0, B.R), B._smul(B.g2_add, q0, B.R)
        p1 = B.g1_add(B.g1_mul(B.G1_GEN, 11), t1)
        q1 = B.g2_add(B.g2_mul(B.G2_GEN, 13), t2)
        for pt in (p0, p1):
            assert B.g1_on_curve(pt)
            assert not B.g1_in_subgroup(pt) and not B.g1_endo_test(pt)
        for pt in (q0, q1):
            assert B.g2_on_curve(pt)
            assert not B.g2_in_subgroup(pt) and not B.g2_endo_test(pt)


def test_c_restatement_rejects_points_outside_subgroup():
    """oracle/bls_pairing.c (the CPU baseline) decodes points as the crate does,
    [r] P == O included: an on-curve point outside the subgroup is invalid (2)."""
    from oracle import bls_c
    p0, q0 = B.g1_curve_point(0x5EED), B.g2_curve_point(0x5EED)
    G, Q = B.g1_bytes(B.g1_mul(B.G1_GEN, 5)), B.g2_bytes(B.g2_mul(B.G2_GEN, 7))
    items = [(G, Q, G, Q), (B.g1_bytes(p0), Q, G, Q), (G, B.g2_bytes(q0), G, Q),
             (G, Q, B.g1_bytes(p0), Q), (G, Q, G, B.g2_bytes(q0))]
    g1 = b"".join(a + c for a, b, c, d in items)
    g2 = b"".join(b + d for a, b, c, d in items)
    assert bls_c.check_batch(g1, g2, len(items), 1) == bytes([1, 2, 2, 2, 2])
