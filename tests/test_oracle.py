"""The CPU oracle (oracle/liborc.so) pinned against the golden fixtures.

The fixtures come from tests/golden/gen_golden.py: an independent Python
restatement anchored on hashlib.sha3_256 and the upstream reed-solomon-erasure
known-answer tests.  Only once these pass is the oracle trusted as the
checker for the HIP path.
"""
import json
import os

import numpy as np
import pytest

from oracle import pyoracle as orc

G = os.path.join(os.path.dirname(__file__), "golden")


def load(name):
    with open(os.path.join(G, name)) as fh:
        return json.load(fh)


@pytest.fixture(scope="module", autouse=True)
def _built():
    orc.build()


def test_gf_kats():
    kat = load("rs_kat.json")
    for a, b, c in kat["mul"]:
        assert orc.gf_mul(a, b) == c
    for a, n, c in kat["exp"]:
        assert orc.gf_exp(a, n) == c
    inp = np.array(kat["mul_slice"]["input"], np.uint8)
    for c in ("25", "177"):
        assert orc.gf_mul_slice(int(c), inp).tolist() == kat["mul_slice"][c]


def test_rs_encode_5_5_kat():
    kat = load("rs_kat.json")["encode_5_5"]
    shards = [np.array(r, np.uint8) for r in kat["data"]] + [np.zeros(2, np.uint8) for _ in range(5)]
    st, out = orc.rs_encode(5, 5, shards)
    assert st == 0
    assert [o.tolist() for o in out[5:]] == kat["parity"]


def test_build_matrix_systematic_and_foo():
    v = load("broadcast_vectors.json")
    assert orc.build_matrix(2, 4).tolist() == v["foo_n4"]["matrix"]
    for k, m in [(6, 10), (22, 42), (44, 84), (84, 166)]:
        mat = orc.build_matrix(k, k + m)
        assert np.array_equal(mat[:k], np.eye(k, dtype=np.uint8))


def test_sha3_kat():
    kat = load("sha3_kat.json")
    for msg, hx in kat["nist"].items():
        assert orc.sha3_256(msg.encode()).hex() == hx
    for L, hx in enumerate(kat["digests"]):
        data = bytes((7 * i + 3) & 0xFF for i in range(L))
        assert orc.sha3_256(data).hex() == hx, L


def test_merkle_shapes():
    """merkle.rs:152-166 test_merkle, plus its digests pinned by hashlib."""
    shapes = load("merkle_shapes.json")
    for n_s, case in shapes.items():
        n = int(n_s)
        nodes = orc.merkle_build([bytes([i]) for i in range(n)])
        assert nodes[-1].tobytes().hex() == case["root"]
        for i in range(n):
            p = orc.merkle_proof(nodes, n, i)
            assert [d.tobytes().hex() for d in p] == case["proofs"][i]
            assert orc.proof_validate(bytes([i]), i, p, nodes[-1].tobytes(), n)
        assert orc.merkle_proof(nodes, n, n) is None


def test_proof_rejects_tampering():
    n = 9
    nodes = orc.merkle_build([bytes([i]) for i in range(n)])
    root = nodes[-1].tobytes()
    p = orc.merkle_proof(nodes, n, 3)
    assert orc.proof_validate(bytes([3]), 3, p, root, n)
    assert not orc.proof_validate(bytes([4]), 3, p, root, n)        # wrong value
    assert not orc.proof_validate(bytes([3]), 2, p, root, n)        # wrong index
    assert not orc.proof_validate(bytes([3]), 3, p[:-1], root, n)   # too few digests
    assert not orc.proof_validate(bytes([3]), 3, np.concatenate([p, p[:1]]), root, n)  # too many
    assert not orc.proof_validate(bytes([3]), 3, p, root, 2 * n)    # wrong n (deeper tree)
    bad = p.copy()
    bad[0, 0] ^= 1
    assert not orc.proof_validate(bytes([3]), 3, bad, root, n)


def test_foo_vector():
    v = load("broadcast_vectors.json")["foo_n4"]
    shards, nodes = orc.send_shards(4, 1, b"Foo")
    assert [s.tobytes().hex() for s in shards] == v["shards"]
    assert nodes[-1].tobytes().hex() == v["root"]


def test_broadcast_vectors():
    v = load("broadcast_vectors.json")
    seed = v["seed"]
    for c in v["cases"]:
        n, f, plen = c["n"], c["f"], c["plen"]
        payload = orc.gen_payload(seed, c["inst"], plen).tobytes()
        shards, nodes = orc.send_shards(n, f, payload)
        assert shards.shape[1] == c["S"]
        root = nodes[-1].tobytes()
        assert root.hex() == c["root"], (n, plen)
        assert [orc.sha3_256(s).hex() for s in shards] == c["shard_sha3"]
        for i_s, dig in c["proofs"].items():
            i = int(i_s)
            p = orc.merkle_proof(nodes, n, i)
            assert [d.tobytes().hex() for d in p] == dig
            assert orc.proof_validate(shards[i], i, p, root, n)
        for d in c["decodes"]:
            present = orc.gen_present(d["seed"], c["inst"], n, d["n_erase"])
            assert present.tolist() == d["present"]
            erased = shards.copy()
            erased[present == 0] = 0
            out, code, rec = orc.decode_from_shards(n, f, erased, present, root)
            assert (out is not None) == d["ok"], (n, plen, code)
            if out is not None:
                assert out == payload
                assert np.array_equal(rec, shards)


def test_reconstruct_error_semantics():
    """rse reconstruct error order + hbbft Coding::Trivial (broadcast.rs:682-693)."""
    k, m = 4, 2
    sh = [np.arange(8, dtype=np.uint8) + i for i in range(6)]
    st, _ = orc.coding_reconstruct(k, m, [sh[0], None, None, None, sh[4], sh[5]])
    assert st == 10  # TooFewShardsPresent
    st, _ = orc.coding_reconstruct(k, m, [sh[0], sh[1][:4], None, sh[3], sh[4], sh[5]])
    assert st == 9   # IncorrectShardSize
    st, _ = orc.coding_reconstruct(k, m, [sh[0][:0], None, sh[2], sh[3], sh[4], sh[5]])
    assert st == 11  # EmptyShard
    st, _ = orc.coding_reconstruct(k, m, sh[:5])
    assert st == 1   # TooFewShards
    # Trivial coding (m == 0): Ok iff all present
    assert orc.coding_reconstruct(3, 0, sh[:3])[0] == 0
    assert orc.coding_reconstruct(3, 0, [sh[0], None, sh[2]])[0] == 10


def test_unframe_truncates_and_rejects_short():
    # payload_len larger than available bytes -> take() truncates silently
    shards, nodes = orc.send_shards(4, 1, b"Foo")
    bad = shards.copy()
    bad[0, :4] = [0, 0, 1, 0]  # claims 256 bytes
    out, code, _ = orc.decode_from_shards(4, 1, bad, np.ones(4, np.uint8), nodes[-1].tobytes())
    assert out is None and code == -2  # root no longer matches (proposer faulty)


def test_bench_pipeline_small():
    t, ok = orc.bench_pipeline(16, 5, 4096, 8, 5, 1, 2)
    assert ok == 8 and t > 0


def test_bincode_wire_vectors():
    """Wire format of broadcast::Message (bincode 1.x), golden N=4 'Foo' messages."""
    w = load("wire_vectors.json")
    sh, nd = orc.send_shards(4, 1, b"Foo")
    root = nd[-1].tobytes()
    assert root.hex() == w["root"]
    for j_s, hx in w["value_msgs"].items():
        j = int(j_s)
        p = orc.merkle_proof(nd, 4, j)
        msg = orc.bincode_message("Value", sh[j].tobytes(), j, [d.tobytes() for d in p], root)
        assert msg.hex() == hx
        v, value, index, digests, r = orc.bincode_parse(msg)
        assert (v, value, index, r) == (0, sh[j].tobytes(), j, root)
        assert digests == [d.tobytes() for d in p]
    assert orc.bincode_message("Ready", root=root).hex() == w["ready"]
    for bad in [b"\x00\x00\x00", b"\x05\x00\x00\x00" + bytes(32), bytes.fromhex(w["value_msgs"]["0"])[:-1]]:
        with pytest.raises(ValueError):
            orc.bincode_parse(bad)
