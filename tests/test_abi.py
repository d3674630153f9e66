"""CPU-side checks of the C ABI (no GPU compute): the library builds, loads and
exports every symbol include/hbrbc.h declares; pure host helpers agree with
the oracle; compute entry points fail loudly (no CPU fallback) without a GPU."""
import ctypes
import os
import re

import numpy as np
import pytest

import __graft_entry__
import hbbft_amd as hb
from oracle import pyoracle as orc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module", autouse=True)
def _built():
    __graft_entry__.build()


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "hbrbc.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(hbrbc_[a-z0-9_]+)\s*\(", src)))


def test_exports_every_declared_symbol():
    syms = declared_symbols()
    assert len(syms) >= 25
    L = ctypes.CDLL(hb.LIB_PATH)
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing


def test_library_is_gfx950_code_object():
    data = open(hb.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_host_helpers_match_oracle():
    L = hb.lib()
    assert L.hbrbc_version().startswith(b"hbrbc")
    for n in [1, 2, 3, 4, 5, 7, 8, 9, 17, 64, 128, 250, 256, 1000]:
        assert L.hbrbc_merkle_node_count(n) == orc.merkle_node_count(n) == hb.merkle_node_count(n)
        assert L.hbrbc_merkle_max_proof_len(n) == hb.max_proof_len(n)
    for plen, k in [(0, 1), (1024, 2), (1 << 20, 6), (256 << 10, 22), (4 << 20, 84)]:
        assert L.hbrbc_shard_len(plen, k) == orc.shard_len(plen, k) == hb.shard_len(plen, k)
    assert [L.hbrbc_stage_name(i).decode() for i in range(9)] == hb.STAGES


def test_library_built_from_this_tree():
    """Provenance: hbrbc_version() carries the hash of the sources the library
    was compiled from (hbbft_amd/srchash.py via the Makefile); it must be the
    hash of the sources in this tree."""
    from hbbft_amd.srchash import source_hash, source_files
    v = hb.lib().hbrbc_version().decode()
    assert v.startswith("hbrbc ") and " gfx950 " in v
    assert v.endswith("src=" + source_hash()), (v, source_hash())
    files = source_files()
    assert "hbbft_amd/csrc/kernels.hip" in files and "include/hbrbc.h" in files


def test_merkle_proof_is_host_data_movement():
    """MerkleTree::proof only copies sibling digests: checkable without a GPU."""
    for n in [1, 4, 7, 9, 17, 64, 250]:
        values = [bytes([i % 256, i // 256]) for i in range(n)]
        nodes = orc.merkle_build(values)
        for i in range(n):
            dig = np.zeros((64, 32), np.uint8)
            nd = ctypes.c_size_t(0)
            st = hb.lib().hbrbc_merkle_proof(nodes.ctypes.data, n, i, dig.ctypes.data,
                                             ctypes.byref(nd))
            assert st == 0
            assert np.array_equal(dig[: nd.value], orc.merkle_proof(nodes, n, i))
        nd = ctypes.c_size_t(0)
        assert hb.lib().hbrbc_merkle_proof(nodes.ctypes.data, n, n, None, ctypes.byref(nd)) == 13


def test_rse_constructor_errors_precede_device():
    """ReedSolomon::new argument errors are reported before any device use."""
    h = ctypes.c_void_p()
    assert hb.lib().hbrbc_coding_new(0, 3, -1, ctypes.byref(h)) == 3      # TooFewDataShards
    assert hb.lib().hbrbc_coding_new(200, 57, -1, ctypes.byref(h)) == 2   # TooManyShards


def test_no_cpu_fallback_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(hb.HbrbcUnavailable):   # HBRBC_E_NO_DEVICE (102): fails loudly,
        hb.Coding(4, 2)                         # never computes on the host
    assert hb.lib().hbrbc_coding_new(4, 2, -1, ctypes.byref(ctypes.c_void_p())) == 102
    with pytest.raises(hb.HbrbcUnavailable):
        hb.RbcBatch(16)


def test_state_machine_block_size():
    """hbrbc_sm_state_bytes (include/hbrbc.h): per node, the echo/ready entry
    of every sender (two bytes per sender with several roots; with one root
    four 32-sender bitmasks -- hash, full, tampered, ready -- per 32 senders),
    can_decode and (several roots) full-Echo masks, counters and flags,
    rounded to 16 bytes; rbc_sim.sm_state_bytes_host mirrors it."""
    from hbbft_amd.rbc_sim import sm_state_bytes_host
    L = hb.lib()
    L.hbrbc_sm_state_bytes.restype = ctypes.c_size_t
    L.hbrbc_sm_state_bytes.argtypes = [ctypes.c_size_t, ctypes.c_size_t]
    for n in (1, 4, 16, 31, 64, 128, 250):
        w = (n + 31) // 32
        for roots in (1, 2, 3):
            er = 16 * w if roots == 1 else 2 * n
            full = 0 if roots == 1 else 4 * w
            want = (er + 4 * roots * w + full + 6 * roots + 4 + 6 + 15) & ~15
            got = L.hbrbc_sm_state_bytes(n, roots)
            assert got == want and got % 16 == 0, (n, roots, got, want)
            assert sm_state_bytes_host(n, roots) == got
