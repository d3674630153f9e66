"""ctypes wrapper for the CPU oracle (oracle/liborc.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, as the checker -- never by the product path
(hbbft_amd/).  See rbc_oracle.h for what is restated and from where.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liborc.so")
_lib = None

c_size_t = ctypes.c_size_t
c_u8p = ctypes.POINTER(ctypes.c_uint8)


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.orc_gf_mul.restype = ctypes.c_uint8
        L.orc_gf_mul.argtypes = [ctypes.c_uint8, ctypes.c_uint8]
        L.orc_gf_div.restype = ctypes.c_uint8
        L.orc_gf_div.argtypes = [ctypes.c_uint8, ctypes.c_uint8]
        L.orc_gf_exp.restype = ctypes.c_uint8
        L.orc_gf_exp.argtypes = [ctypes.c_uint8, c_size_t]
        L.orc_gf_mul_slice.argtypes = [ctypes.c_uint8, ctypes.c_void_p, ctypes.c_void_p, c_size_t]
        L.orc_gf_invert.argtypes = [c_size_t, ctypes.c_void_p]
        L.orc_build_matrix.argtypes = [c_size_t, c_size_t, ctypes.c_void_p]
        L.orc_rs_encode.argtypes = [c_size_t, c_size_t, ctypes.c_void_p, ctypes.c_void_p, c_size_t]
        L.orc_rs_reconstruct.argtypes = [c_size_t, c_size_t, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_void_p, c_size_t]
        L.orc_coding_reconstruct.argtypes = L.orc_rs_reconstruct.argtypes
        L.orc_sha3_256.argtypes = [ctypes.c_void_p, c_size_t, ctypes.c_void_p]
        L.orc_merkle_node_count.restype = c_size_t
        L.orc_merkle_node_count.argtypes = [c_size_t]
        L.orc_merkle_build.argtypes = [c_size_t, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.orc_merkle_proof.argtypes = [c_size_t, ctypes.c_void_p, c_size_t, ctypes.c_void_p,
                                       ctypes.POINTER(c_size_t)]
        L.orc_proof_validate.argtypes = [ctypes.c_void_p, c_size_t, c_size_t, ctypes.c_void_p,
                                         c_size_t, ctypes.c_void_p, c_size_t]
        L.orc_shard_len.restype = c_size_t
        L.orc_shard_len.argtypes = [c_size_t, c_size_t]
        L.orc_frame.argtypes = [ctypes.c_void_p, c_size_t, c_size_t, c_size_t, c_size_t,
                                ctypes.c_void_p]
        L.orc_unframe.restype = ctypes.c_long
        L.orc_unframe.argtypes = [ctypes.c_void_p, c_size_t, c_size_t, ctypes.c_void_p]
        L.orc_send_shards.argtypes = [c_size_t, c_size_t, ctypes.c_void_p, c_size_t,
                                      ctypes.c_void_p, ctypes.c_void_p]
        L.orc_decode_from_shards.restype = ctypes.c_long
        L.orc_decode_from_shards.argtypes = [c_size_t, c_size_t, ctypes.c_void_p, c_size_t,
                                             ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.orc_mix64.restype = ctypes.c_uint64
        L.orc_mix64.argtypes = [ctypes.c_uint64]
        L.orc_gen_payload.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p, c_size_t]
        L.orc_gen_present.argtypes = [ctypes.c_uint64, ctypes.c_uint64, c_size_t, c_size_t,
                                      ctypes.c_void_p]
        L.orc_bench_pipeline.restype = ctypes.c_double
        L.orc_bench_pipeline.argtypes = [c_size_t, c_size_t, c_size_t, c_size_t, c_size_t,
                                         ctypes.c_uint64, ctypes.c_int, ctypes.POINTER(c_size_t)]
        _lib = L
    return _lib


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _ptr_array(rows):
    arr = (ctypes.c_void_p * len(rows))()
    for i, r in enumerate(rows):
        arr[i] = r.ctypes.data
    return arr


# ---- GF / matrix ---------------------------------------------------------
def gf_mul(a, b):
    return lib().orc_gf_mul(a, b)


def gf_exp(a, n):
    return lib().orc_gf_exp(a, n)


def gf_mul_slice(c, data):
    data = np.ascontiguousarray(data, dtype=np.uint8)
    out = np.empty_like(data)
    lib().orc_gf_mul_slice(c, _ptr(data), _ptr(out), data.size)
    return out


def build_matrix(k, total):
    out = np.zeros((total, k), dtype=np.uint8)
    st = lib().orc_build_matrix(k, total, _ptr(out))
    assert st == 0
    return out


# ---- RS ------------------------------------------------------------------
def rs_encode(k, m, shards):
    """shards: list of np.uint8 arrays (modified in place).  Returns status."""
    shards = [np.ascontiguousarray(s) for s in shards]
    lens = np.array([s.size for s in shards], dtype=np.uint64)
    st = lib().orc_rs_encode(k, m, _ptr_array(shards), _ptr(lens), len(shards))
    return st, shards


def coding_reconstruct(k, m, shards):
    """shards: list of Optional[np.uint8 array] (hbbft Coding::reconstruct_shards).
    Returns (status, list)."""
    lens = np.array([0 if s is None else s.size for s in shards], dtype=np.uint64)
    present = np.array([s is not None for s in shards], dtype=np.uint8)
    L = int(max([s.size for s in shards if s is not None], default=0))
    bufs = [np.ascontiguousarray(s).copy() if s is not None else np.zeros(max(L, 1), np.uint8)
            for s in shards]
    st = lib().orc_coding_reconstruct(k, m, _ptr_array(bufs), _ptr(lens), _ptr(present), len(bufs))
    if st != 0:
        return st, shards
    return st, [b[:L] if s is None else b for b, s in zip(bufs, shards)]


# ---- hashing / Merkle ----------------------------------------------------
def sha3_256(data):
    data = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else data
    data = np.ascontiguousarray(data, dtype=np.uint8)
    out = np.zeros(32, np.uint8)
    lib().orc_sha3_256(_ptr(data) if data.size else None, data.size, _ptr(out))
    return out.tobytes()


def merkle_node_count(n):
    return lib().orc_merkle_node_count(n)


def merkle_build(values):
    vals = [np.ascontiguousarray(np.frombuffer(bytes(v), np.uint8) if not isinstance(v, np.ndarray)
                                 else v, dtype=np.uint8) for v in values]
    vals = [v if v.size else np.zeros(1, np.uint8)[:0] for v in vals]
    keep = [np.concatenate([v, np.zeros(1, np.uint8)]) for v in vals]  # non-null pointers
    lens = np.array([v.size for v in vals], dtype=np.uint64)
    n = len(vals)
    nodes = np.zeros((merkle_node_count(n), 32), np.uint8)
    lib().orc_merkle_build(n, _ptr_array(keep), _ptr(lens), _ptr(nodes))
    return nodes


def merkle_proof(nodes, n, index):
    dig = np.zeros((64, 32), np.uint8)
    nd = c_size_t(0)
    ok = lib().orc_merkle_proof(n, _ptr(nodes), index, _ptr(dig), ctypes.byref(nd))
    if not ok:
        return None
    return dig[: nd.value].copy()


def proof_validate(value, index, digests, root, n):
    v = np.ascontiguousarray(np.frombuffer(bytes(value), np.uint8) if not isinstance(value, np.ndarray)
                             else value, dtype=np.uint8)
    v = np.concatenate([v, np.zeros(1, np.uint8)])
    d = np.ascontiguousarray(digests, dtype=np.uint8).reshape(-1, 32)
    d = np.concatenate([d, np.zeros((1, 32), np.uint8)])
    r = np.frombuffer(bytes(root), np.uint8).copy()
    return bool(lib().orc_proof_validate(_ptr(v), v.size - 1, index, _ptr(d), d.shape[0] - 1,
                                         _ptr(r), n))


# ---- framing / whole path -------------------------------------------------
def shard_len(plen, k):
    return lib().orc_shard_len(plen, k)


def send_shards(n, f, payload):
    """frame + encode + tree -> (shards[N,S], nodes[T,32])."""
    p = np.concatenate([np.frombuffer(bytes(payload), np.uint8), np.zeros(1, np.uint8)])
    k = n - 2 * f
    S = shard_len(len(payload), k)
    shards = np.zeros((n, S), np.uint8)
    nodes = np.zeros((merkle_node_count(n), 32), np.uint8)
    st = lib().orc_send_shards(n, f, _ptr(p), len(payload), _ptr(shards), _ptr(nodes))
    assert st == 0, st
    return shards, nodes


def decode_from_shards(n, f, shards, present, root):
    """Returns (payload bytes | None, code, reconstructed shards)."""
    sh = np.ascontiguousarray(shards, dtype=np.uint8).copy()
    S = sh.shape[1]
    pres = np.ascontiguousarray(present, dtype=np.uint8)
    k = n - 2 * f
    out = np.zeros(k * S + 1, np.uint8)
    r = np.frombuffer(bytes(root), np.uint8).copy()
    L = lib().orc_decode_from_shards(n, f, _ptr(sh), S, _ptr(pres), _ptr(r), _ptr(out))
    if L < 0:
        return None, int(L), sh
    return out[:L].tobytes(), 0, sh


# ---- synthetic workload ----------------------------------------------------
def gen_payload(seed, inst, length):
    out = np.zeros(max(length, 1), np.uint8)
    lib().orc_gen_payload(seed, inst, _ptr(out), length)
    return out[:length]


def gen_present(seed, inst, n, n_erase):
    out = np.zeros(n, np.uint8)
    lib().orc_gen_present(seed, inst, n, n_erase, _ptr(out))
    return out


def bench_pipeline(n, f, plen, count, n_erase, seed, threads):
    ok = c_size_t(0)
    t = lib().orc_bench_pipeline(n, f, plen, count, n_erase, seed, threads, ctypes.byref(ok))
    return t, ok.value


# ---- bincode wire format of broadcast::Message ------------------------------
# bincode 1.x defaults (Cargo.toml:24 `bincode = "1.2.0"`; serialize at
# examples/simulation.rs:132): little-endian fixed-width integers, enum
# variant as u32, Vec length and usize as u64, [u8; 32] as 32 raw bytes.
# Field order of Proof: value, index, digests, root_hash (merkle.rs:72-78);
# variants in declaration order (message.rs:13-24).  Plain struct packing:
# restated from the bincode 1.x specification, no reference fixture exists.
import struct as _struct

WIRE_VARIANTS = {"Value": 0, "Echo": 1, "Ready": 2, "CanDecode": 3, "EchoHash": 4}


def bincode_message(variant, value=b"", index=0, digests=(), root=b"\0" * 32):
    v = WIRE_VARIANTS[variant] if isinstance(variant, str) else variant
    if v >= 2:
        return _struct.pack("<I", v) + bytes(root)
    digests = [bytes(d) for d in digests]
    return (_struct.pack("<IQ", v, len(value)) + bytes(value) + _struct.pack("<QQ", index, len(digests))
            + b"".join(digests) + bytes(root))


def bincode_parse(msg):
    """-> (variant, value, index, digests, root) or raises ValueError (truncated /
    bad variant), as bincode::deserialize::<Message> would fail."""
    msg = bytes(msg)
    if len(msg) < 4:
        raise ValueError("truncated")
    (v,) = _struct.unpack_from("<I", msg, 0)
    if v > 4:
        raise ValueError("bad variant")
    if v >= 2:
        if len(msg) < 36:
            raise ValueError("truncated")
        return v, b"", 0, [], msg[4:36]
    if len(msg) < 12:
        raise ValueError("truncated")
    (L,) = _struct.unpack_from("<Q", msg, 4)
    if len(msg) < 28 + L:
        raise ValueError("truncated")
    value = msg[12:12 + L]
    index, d = _struct.unpack_from("<QQ", msg, 12 + L)
    if len(msg) < 60 + L + 32 * d:
        raise ValueError("truncated")
    digests = [msg[28 + L + 32 * t: 60 + L + 32 * t] for t in range(d)]
    root = msg[28 + L + 32 * d: 60 + L + 32 * d]
    return v, value, index, digests, root
