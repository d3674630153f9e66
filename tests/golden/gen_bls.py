"""Writes tests/golden/bls_vectors.json: BLS12-381 pairing vectors from the
CPU restatement (oracle/bls_oracle.py) for the f4 parity tests.

Run from the repo root: python tests/golden/gen_bls.py.  Each vector holds
the uncompressed point encodings and the GT bytes (576, tower order) of
the `pairing` crate's e(P, Q) = f^(3 (p^12-1)/r) (see the oracle header for
what pins that); `checks` hold threshold-decrypt shaped checks with their
expected outcomes.  Scalars are fixed, so the file is reproducible.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import bls_oracle as B  # noqa: E402

SCALARS_1 = [1, 2, 3, 0x1234567, B.R - 1, 0x5eed_1e55_0f_c0ffee]
SCALARS_2 = [1, 5, 0xabcdef, B.R - 2]


def main():
    pairs = [(1, 1), (2, 1), (1, 2), (3, 5), (0x1234567, 0xabcdef), (B.R - 1, 1),
             (0x5eed_1e55_0f_c0ffee, B.R - 2)]
    vectors = []
    for a, b in pairs:
        p1 = B.g1_mul(B.G1_GEN, a)
        q2 = B.g2_mul(B.G2_GEN, b)
        gt = B.pairing(p1, q2)
        vectors.append({"g1_scalar": a, "g2_scalar": b, "g1": B.g1_bytes(p1).hex(),
                        "g2": B.g2_bytes(q2).hex(), "gt": B.gt_bytes(gt).hex()})
    checks = []
    for sk, r_enc, h, tamper in [(7, 11, 13, False), (7, 11, 13, True),
                                 (0xdead_beef, 0x1234_5678_9abc, 0x42, False),
                                 (B.R - 3, 99, 0x77, True)]:
        share, H, pk, W = B.decryption_share_case(sk, r_enc, h, tamper)
        checks.append({"a": B.g1_bytes(share).hex(), "b": B.g2_bytes(H).hex(),
                       "c": B.g1_bytes(pk).hex(), "d": B.g2_bytes(W).hex(),
                       "expect": not tamper, "kind": "verify_decryption_share"})
    # bench pool (bench.py's f4 leg tiles these): 32 checks, one in four tampered
    import random
    rng = random.Random(0x48424246)
    pool = []
    for i in range(32):
        share, H, pk, W = B.decryption_share_case(rng.randrange(1, B.R), rng.randrange(1, B.R),
                                                  rng.randrange(1, B.R), tamper=(i % 4 == 3))
        pool.append({"a": B.g1_bytes(share).hex(), "b": B.g2_bytes(H).hex(),
                     "c": B.g1_bytes(pk).hex(), "d": B.g2_bytes(W).hex(),
                     "expect": i % 4 != 3, "kind": "verify_decryption_share"})
    # grouped bench pool (bench.py's f4 leg): 4 ciphertexts x 64 decryption shares,
    # every share of a ciphertext checked against its H and W; one in eight tampered
    groups = []
    for g in range(4):
        h, r_enc = rng.randrange(1, B.R), rng.randrange(1, B.R)
        H = B.g2_mul(B.G2_GEN, h)
        U = B.g1_mul(B.G1_GEN, r_enc)
        W = B.g2_mul(H, r_enc)
        sh = []
        for s in range(64):
            sk = rng.randrange(1, B.R)
            share = B.g1_mul(U, sk)
            good = (s + g) % 8 != 7
            if not good:
                share = B.g1_add(share, B.G1_GEN)
            sh.append({"share": B.g1_bytes(share).hex(),
                       "pk": B.g1_bytes(B.g1_mul(B.G1_GEN, sk)).hex(), "expect": good})
        groups.append({"hash": B.g2_bytes(H).hex(), "w": B.g2_bytes(W).hex(), "shares": sh})
    out = {"source": "oracle/bls_oracle.py (restatement of the pairing crate's BLS12-381)",
           "pairings": vectors, "checks": checks, "bench_pool": pool, "bench_groups": groups}
    path = os.path.join(ROOT, "tests", "golden", "bls_vectors.json")
    with open(path, "w") as fh:
        json.dump(out, fh, indent=1)
    print("wrote", path, len(vectors), "pairings", len(checks), "checks")


if __name__ == "__main__":
    main()
