#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/.

This is an INDEPENDENT second restatement (pure Python + numpy + hashlib) of
the reference's Reliable-Broadcast data path; it shares no code with the C
oracle (oracle/rbc_oracle.c) or with the HIP path.  What anchors it:

* SHA3-256: Python's hashlib.sha3_256 (FIPS-202), identical to
  tiny-keccak 2.0 `Sha3::v256()` used at /root/reference/src/broadcast/merkle.rs:143-150.
  Cross-checked against the NIST FIPS-202 example digests for "" and "abc".
* GF(2^8) Reed-Solomon: the published known-answer tests of the upstream
  crate `reed-solomon-erasure` 4.0.x (galois_8 `mul`/`exp`/`mul_slice` tests
  and the 5+5 `encode` vector it shares with Backblaze JavaReedSolomon).  The
  crate's source is not in this container; the values below are
  recorded as data and this restatement must reproduce every one of them
  before any fixture is written.
* Merkle tree / proof / framing: restated from merkle.rs:20-103 and
  broadcast.rs:170-189, 563-601.

Run:  python tests/golden/gen_golden.py   (writes *.json next to this file)
"""
import hashlib
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
MASK64 = (1 << 64) - 1

# --------------------------------------------------------------------------
# Upstream known-answer tests (data).
# --------------------------------------------------------------------------
MUL_SLICE_INPUT = [0, 1, 2, 3, 4, 5, 6, 10, 50, 100, 150, 174, 201, 255, 99, 32, 67, 85, 200, 199,
                   198, 197, 196, 195, 194, 193, 192, 191, 190, 189, 188, 187, 186, 185]
RS_KAT = {
    "source": "reed-solomon-erasure 4.0.x src/galois_8.rs test_galois / src/tests; Backblaze "
              "JavaReedSolomon GaloisTest + ReedSolomonTest.testOneEncode (published tests; "
              "recorded as data)",
    "mul": [[3, 4, 12], [7, 7, 21], [23, 45, 41]],
    "exp": [[2, 2, 4], [5, 20, 235], [13, 7, 43]],
    "mul_slice": {
        "input": MUL_SLICE_INPUT,
        "25": [0x0, 0x19, 0x32, 0x2b, 0x64, 0x7d, 0x56, 0xfa, 0xb8, 0x6d, 0xc7, 0x85, 0xc3, 0x1f,
               0x22, 0x7, 0x25, 0xfe, 0xda, 0x5d, 0x44, 0x6f, 0x76, 0x39, 0x20, 0xb, 0x12, 0x11,
               0x8, 0x23, 0x3a, 0x75, 0x6c, 0x47],
        "177": [0x0, 0xb1, 0x7f, 0xce, 0xfe, 0x4f, 0x81, 0x9e, 0x3, 0x6, 0xe8, 0x75, 0xbd, 0x40,
                0x36, 0xa3, 0x95, 0xcb, 0xc, 0xdd, 0x6c, 0xa2, 0x13, 0x23, 0x92, 0x5c, 0xed, 0x1b,
                0xaa, 0x64, 0xd5, 0xe5, 0x54, 0x9a],
    },
    "encode_5_5": {
        "data": [[0, 1], [4, 5], [2, 3], [6, 7], [8, 9]],
        "parity": [[12, 13], [10, 11], [14, 15], [90, 91], [94, 95]],
    },
}

NIST_SHA3_256 = {
    "": "a7ffc6f8bf1ed76651c14756a061d662f580ff4de43b49fa82d80a4b80f8434a",
    "abc": "3a985da74fe225b2045c172d6bd390bd855f086e3e9d525b46bfe24511431532",
}

# --------------------------------------------------------------------------
# GF(2^8) (poly 0x11D, generator 2) -- second, independent restatement.
# --------------------------------------------------------------------------
EXP = [0] * 512
LOG = [0] * 256
_x = 1
for _i in range(255):
    EXP[_i] = _x
    LOG[_x] = _i
    _x <<= 1
    if _x & 0x100:
        _x ^= 0x11D
for _i in range(255, 512):
    EXP[_i] = EXP[_i - 255]

MUL = np.zeros((256, 256), dtype=np.uint8)
for _a in range(1, 256):
    for _b in range(1, 256):
        MUL[_a, _b] = EXP[LOG[_a] + LOG[_b]]


def gmul(a, b):
    return int(MUL[a, b])


def gexp(a, n):
    if n == 0:
        return 1
    if a == 0:
        return 0
    return EXP[(LOG[a] * n) % 255]


def ginv(a):
    return EXP[(255 - LOG[a]) % 255]


def mat_inv(m):
    n = len(m)
    a = [list(r) + [1 if i == j else 0 for j in range(n)] for i, r in enumerate(m)]
    for c in range(n):
        p = next(r for r in range(c, n) if a[r][c])
        a[c], a[p] = a[p], a[c]
        s = ginv(a[c][c])
        a[c] = [gmul(s, v) for v in a[c]]
        for r in range(n):
            if r != c and a[r][c]:
                f = a[r][c]
                a[r] = [v ^ gmul(f, w) for v, w in zip(a[r], a[c])]
    return [r[n:] for r in a]


def mat_mul(a, b):
    out = []
    for r in a:
        row = []
        for c in range(len(b[0])):
            acc = 0
            for j in range(len(b)):
                acc ^= gmul(r[j], b[j][c])
            row.append(acc)
        out.append(row)
    return out


def build_matrix(k, total):
    v = [[gexp(r, c) for c in range(k)] for r in range(total)]
    return mat_mul(v, mat_inv(v[:k]))


def apply_rows(rows, inputs):
    """GF matrix (list of rows) times list of byte arrays."""
    outs = []
    for row in rows:
        acc = np.zeros_like(inputs[0])
        for c, x in zip(row, inputs):
            if c:
                acc ^= MUL[c][x]
        outs.append(acc)
    return outs


def rs_encode(k, m, data):
    mat = build_matrix(k, k + m)
    return apply_rows(mat[k:], data)


def rs_reconstruct(k, m, shards):
    """rse reconstruct semantics on a list of Optional arrays; returns list."""
    total = k + m
    present = [i for i, s in enumerate(shards) if s is not None]
    if len(present) == total:
        return list(shards)
    if len(present) < k:
        raise ValueError("TooFewShardsPresent")
    mat = build_matrix(k, total)
    valid = present[:k]
    dm = mat_inv([mat[i] for i in valid])
    sub = [shards[i] for i in valid]
    out = list(shards)
    for d in range(k):
        if out[d] is None:
            out[d] = apply_rows([dm[d]], sub)[0]
    for p in range(k, total):
        if out[p] is None:
            out[p] = apply_rows([mat[p]], out[:k])[0]
    return out


# --------------------------------------------------------------------------
# SHA3 / Merkle / framing (merkle.rs, broadcast.rs)
# --------------------------------------------------------------------------
def H(b):
    return hashlib.sha3_256(bytes(b)).digest()


def merkle_levels(values):
    lvl = [H(v) for v in values]
    levels = [lvl]
    while len(lvl) > 1:
        lvl = [H(lvl[i] + lvl[i + 1]) if i + 1 < len(lvl) else lvl[i] for i in range(0, len(lvl), 2)]
        levels.append(lvl)
    return levels


def merkle_proof(levels, index):
    d, i = [], index
    for lvl in levels[:-1]:
        if (i ^ 1) < len(lvl):
            d.append(lvl[i ^ 1])
        i //= 2
    return d


def validate(value, index, digests, root, n):
    d = H(value)
    i, ln, it = index, n, iter(digests)
    while ln > 1:
        if (i ^ 1) < ln:
            s = next(it, None)
            if s is None:
                return False
            d = H(s + d) if i & 1 else H(d + s)
        i //= 2
        ln = (ln + 1) // 2
    if next(it, None) is not None:
        return False
    return d == root


def frame(payload, n, f):
    m = 2 * f
    k = n - m
    buf = len(payload).to_bytes(4, "big") + bytes(payload)
    S = (len(buf) + k - 1) // k
    buf = buf + bytes(S * n - len(buf))
    return [np.frombuffer(buf[i * S:(i + 1) * S], dtype=np.uint8).copy() for i in range(n)], S


def send_shards(payload, n, f):
    shards, S = frame(payload, n, f)
    m = 2 * f
    k = n - m
    if m:
        shards[k:] = rs_encode(k, m, shards[:k])
    return shards, S


def unframe(shards, k):
    b = b"".join(bytes(s) for s in shards[:k])
    if len(b) < 4:
        return None
    ln = int.from_bytes(b[:4], "big")
    return b[4:4 + ln]


# --------------------------------------------------------------------------
# Synthetic workload (same counter PRNG as oracle/rbc_oracle.c, HIP bench)
# --------------------------------------------------------------------------
C1 = 0xD6E8FEB86659FD93
C2 = 0xA0761D6478BD642F


def mix64(z):
    z = (z + 0x9E3779B97F4A7C15) & MASK64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK64
    return z ^ (z >> 31)


def gen_payload(seed, inst, length):
    base = (seed * C1 + inst * C2) & MASK64
    out = bytearray()
    q = 0
    while len(out) < length:
        out += mix64((base + q) & MASK64).to_bytes(8, "little")
        q += 1
    return bytes(out[:length])


def gen_present(seed, inst, n, n_erase):
    base = (((seed ^ 0x5EED5EED5EED5EED) * C1) + inst * C2) & MASK64
    present = [1] * n
    for t in range(min(n_erase, n)):
        r = mix64((base + t) & MASK64) % (n - t)
        for i in range(n):
            if not present[i]:
                continue
            if r == 0:
                present[i] = 0
                break
            r -= 1
    return present


# --------------------------------------------------------------------------
def check_kats():
    for a, b, c in RS_KAT["mul"]:
        assert gmul(a, b) == c, (a, b, c)
    for a, n, c in RS_KAT["exp"]:
        assert gexp(a, n) == c, (a, n, c)
    inp = np.array(MUL_SLICE_INPUT, dtype=np.uint8)
    for c in ("25", "177"):
        assert MUL[int(c)][inp].tolist() == RS_KAT["mul_slice"][c], c
    data = [np.array(r, dtype=np.uint8) for r in RS_KAT["encode_5_5"]["data"]]
    par = rs_encode(5, 5, data)
    assert [p.tolist() for p in par] == RS_KAT["encode_5_5"]["parity"]
    for msg, hx in NIST_SHA3_256.items():
        assert H(msg.encode()).hex() == hx


def main():
    check_kats()
    with open(os.path.join(HERE, "rs_kat.json"), "w") as fh:
        json.dump(RS_KAT, fh, indent=1)

    # SHA3 across the rate boundary (0..300 bytes); input byte i = (7*i+3) & 0xff
    sha = {"nist": NIST_SHA3_256, "pattern": "byte i = (7*i + 3) & 0xff",
           "digests": [H(bytes((7 * i + 3) & 0xFF for i in range(L))).hex() for L in range(301)]}
    with open(os.path.join(HERE, "sha3_kat.json"), "w") as fh:
        json.dump(sha, fh, indent=0)

    # merkle.rs:152-166 test_merkle shapes, leaves vec![i as u8]
    shapes = {}
    for n in (1, 2, 3, 4, 5, 7, 8, 9, 17, 33):
        levels = merkle_levels([bytes([i]) for i in range(n)])
        root = levels[-1][0]
        proofs = [[d.hex() for d in merkle_proof(levels, i)] for i in range(n)]
        for i in range(n):
            assert validate(bytes([i]), i, [bytes.fromhex(x) for x in proofs[i]], root, n)
        shapes[str(n)] = {"root": root.hex(), "proofs": proofs}
    with open(os.path.join(HERE, "merkle_shapes.json"), "w") as fh:
        json.dump(shapes, fh, indent=0)

    # Whole-path vectors: send_shards -> digests/root/proofs; decode with erasures.
    vec = {"seed": 0x48424246, "cases": []}
    seed = vec["seed"]
    cases = [(1, [0, 3, 100]), (2, [0, 5, 77]), (3, [0, 9, 1000]), (4, [0, 1, 3, 1024]),
             (5, [2, 300]), (7, [128, 1001]), (8, [32, 4099]), (10, [500]), (16, [0, 1000, 6001]),
             (31, [777]), (64, [0, 3, 5000, 11916 * 22 - 4]), (100, [2048]), (128, [3000, 10000]),
             (250, [0, 17, 20000]), (256, [1234])]
    for n, plens in cases:
        f = (n - 1) // 3
        m, k = 2 * f, n - 2 * f
        for inst, plen in enumerate(plens):
            payload = gen_payload(seed, inst, plen)
            shards, S = send_shards(payload, n, f)
            levels = merkle_levels([s.tobytes() for s in shards])
            root = levels[-1][0]
            idxs = sorted({0, n // 2, n - 1})
            case = {
                "n": n, "f": f, "inst": inst, "plen": plen, "S": S,
                "shard_sha3": [H(s).hex() for s in shards],
                "root": root.hex(),
                "proofs": {str(i): [d.hex() for d in merkle_proof(levels, i)] for i in idxs},
                "decodes": [],
            }
            for pat in range(2):
                n_erase = f if pat == 0 else m  # f random, or 2f = worst case allowed
                present = gen_present(seed + pat, inst, n, n_erase)
                opt = [s if p else None for s, p in zip(shards, present)]
                if m:
                    rec = rs_reconstruct(k, m, opt)
                else:
                    rec = opt if all(present) else None
                out = None
                if rec is not None:
                    assert all(np.array_equal(a, b) for a, b in zip(rec, shards))
                    out = unframe(rec, k)
                    assert out == payload
                case["decodes"].append({
                    "seed": seed + pat, "n_erase": n_erase, "present": present,
                    "ok": out is not None,
                    "payload_sha3": H(out).hex() if out is not None else None,
                })
            vec["cases"].append(case)
    # The N=4 "Foo" vector spelled out byte for byte (tests/broadcast.rs:261-281 payload)
    shards, S = send_shards(b"Foo", 4, 1)
    lv = merkle_levels([s.tobytes() for s in shards])
    vec["foo_n4"] = {"shards": [s.tobytes().hex() for s in shards], "root": lv[-1][0].hex(),
                     "matrix": build_matrix(2, 4)}
    with open(os.path.join(HERE, "broadcast_vectors.json"), "w") as fh:
        json.dump(vec, fh, indent=0)
    print("golden fixtures written")


if __name__ == "__main__":
    main()
