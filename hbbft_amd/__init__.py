"""hbbft_amd -- MI355X-native Reliable-Broadcast data path for hbbft.

Python host-side mirror of the reference's `Coding` / `MerkleTree` / `Proof`
surface (/root/reference/src/broadcast/broadcast.rs:639-694,
src/broadcast/merkle.rs) over the C ABI in include/hbrbc.h, plus thin
wrappers of the batched device entry points that take torch tensors.

Every computation runs in hbbft_amd/libhbrbc.so (HIP kernels for gfx950).
There is no CPU fallback: importing works anywhere, but the first call that
needs the library raises `HbrbcUnavailable` when it is not built or no GPU is
visible.
"""
import ctypes
import os

__all__ = [
    "RseError", "HbrbcUnavailable", "Coding", "MerkleTree", "Proof", "RbcBatch",
    "shard_len", "merkle_node_count", "max_proof_len", "lib", "LIB_PATH", "STAGES",
    "jit_build_encode", "jit_file_name", "WIRE_VARIANTS", "validate_proofs", "VALIDATE_STATS",
    "send_shards_batch", "SEND_STATS", "jit_decode_groups", "jit_build_decode",
    "jit_decode_file_name", "jit_encode_groups",
]

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("HBRBC_LIB") or os.path.join(_HERE, "libhbrbc.so")  # A/B builds

STATUS_NAMES = {
    0: "Ok", 1: "TooFewShards", 2: "TooManyShards", 3: "TooFewDataShards",
    4: "TooManyDataShards", 5: "TooFewParityShards", 6: "TooManyParityShards",
    7: "TooFewBufferShards", 8: "TooManyBufferShards", 9: "IncorrectShardSize",
    10: "TooFewShardsPresent", 11: "EmptyShard", 12: "InvalidShardFlags", 13: "InvalidIndex",
    64: "SingularMatrix", 65: "RootMismatch", 66: "NoPayloadLen",
    70: "WireTruncated", 71: "WireBadVariant", 72: "WireTooLarge",
    100: "InvalidArgument", 101: "DeviceError", 102: "NoDevice",
}
WIRE_VARIANTS = {"Value": 0, "Echo": 1, "Ready": 2, "CanDecode": 3, "EchoHash": 4}
STAGES = ["frame", "encode", "leaf_hash", "tree_levels", "proofs", "validate",
          "decode_matrix", "reconstruct", "unframe"]


class HbrbcUnavailable(RuntimeError):
    """libhbrbc.so is missing or no HIP device is visible (no fallback exists)."""


class RseError(Exception):
    """A `reed_solomon_erasure::Error` (or library error) returned by the ABI."""

    def __init__(self, code, msg=""):
        self.code = code
        self.msg = msg
        self.name = STATUS_NAMES.get(code, "Status%d" % code)
        super().__init__("%s%s" % (self.name, (": " + msg) if msg else ""))

    def __reduce__(self):   # picklable across process pools (build() workers)
        return (RseError, (self.code, self.msg))


_lib = None
_P = ctypes.c_void_p
_S = ctypes.c_size_t


def lib():
    """Load libhbrbc.so (raises HbrbcUnavailable if it is not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise HbrbcUnavailable("%s not built (run __graft_entry__.build())" % LIB_PATH)
    L = ctypes.CDLL(LIB_PATH)
    sig = {
        "hbrbc_last_error": (ctypes.c_char_p, []),
        "hbrbc_version": (ctypes.c_char_p, []),
        "hbrbc_coding_new": (ctypes.c_int, [_S, _S, ctypes.c_int, ctypes.POINTER(_P)]),
        "hbrbc_coding_free": (None, [_P]),
        "hbrbc_data_shard_count": (_S, [_P]),
        "hbrbc_parity_shard_count": (_S, [_P]),
        "hbrbc_encoding_matrix": (ctypes.c_int, [_P, _P]),
        "hbrbc_stream": (_P, [_P]),
        "hbrbc_encode": (ctypes.c_int, [_P, _P, _P, _S]),
        "hbrbc_reconstruct": (ctypes.c_int, [_P, _P, _P, _P, _S]),
        "hbrbc_merkle_node_count": (_S, [_S]),
        "hbrbc_merkle_max_proof_len": (_S, [_S]),
        "hbrbc_merkle_build": (ctypes.c_int, [_P, _P, _S, _P]),
        "hbrbc_merkle_proof": (ctypes.c_int, [_P, _S, _S, _P, ctypes.POINTER(_S)]),
        "hbrbc_proof_validate": (ctypes.c_int, [_P, _S, _S, _P, _S, _P, _S,
                                                ctypes.POINTER(ctypes.c_int)]),
        "hbrbc_shard_len": (_S, [_S, _S]),
        "hbrbc_frame_batch": (ctypes.c_int, [_P, _P, _S, _S, _S, _P, _S, _S, _S, _P]),
        "hbrbc_encode_batch": (ctypes.c_int, [_P, _P, _S, _S, _S, _S, _P]),
        "hbrbc_frame_encode_batch": (ctypes.c_int, [_P, _P, _S, _S, _S, _P, _S, _S, _S, _P]),
        "hbrbc_merkle_batch": (ctypes.c_int, [_P, _P, _S, _S, _S, _S, _P, _S, _P]),
        "hbrbc_proofs_batch": (ctypes.c_int, [_P, _P, _S, _S, _P, _P, _P]),
        "hbrbc_validate_batch": (ctypes.c_int, [_P, _P, _S, _S, _S, _S, _P, _P, _P, _P, _S, _S,
                                                _S, _P, _P]),
        "hbrbc_reconstruct_batch": (ctypes.c_int, [_P, _P, _S, _S, _S, _P, _S, _P, _P]),
        "hbrbc_decode_batch": (ctypes.c_int, [_P, _P, _S, _S, _S, _P, _S, _P, _S, _P, _S, _P, _S,
                                              _P, _P, _P]),
        "hbrbc_reserve": (ctypes.c_int, [_P, _S]),
        "hbrbc_profile_enable": (ctypes.c_int, [_P, ctypes.c_int]),
        "hbrbc_profile_reset": (ctypes.c_int, [_P]),
        "hbrbc_profile_read": (ctypes.c_int, [_P, _P, _P]),
        "hbrbc_stage_name": (ctypes.c_char_p, [ctypes.c_int]),
        "hbrbc_encode_kernel": (ctypes.c_char_p, [_P]),
        "hbrbc_wire_proof_message_len": (_S, [_S, _S]),
        "hbrbc_wire_encode_batch": (ctypes.c_int, [_P, ctypes.c_uint32, _P, _S, _S, _S, _S, _P, _P,
                                                   _P, _P, _S, _S, _P, _S, _P, _P]),
        "hbrbc_wire_decode_batch": (ctypes.c_int, [_P, _P, _S, _P, _S, _P, _S, _P, _P, _P, _P, _P,
                                                   _P, _P, _P]),
        "hbrbc_jit_build_encode": (ctypes.c_int, [_S, _S, ctypes.c_char_p]),
        "hbrbc_jit_encode_groups": (_S, [_S, _S]),
        "hbrbc_jit_build_encode_group": (ctypes.c_int, [_S, _S, _S, ctypes.c_char_p]),
        "hbrbc_jit_file_name": (ctypes.c_int, [_S, _S, _S, ctypes.c_char_p, _S]),
        "hbrbc_frame_encode_rows": (ctypes.c_int, [_P, _P, _S, _S, _S, _P, _S, _S, _S, _S, _S, _P]),
        "hbrbc_frame_encode_ragged": (ctypes.c_int, [_P, _P, _S, _P, _S, _S, _P, _S, _S, _P]),
        "hbrbc_merkle_ragged": (ctypes.c_int, [_P, _P, _P, _S, _S, _S, _P, _S, _P]),
        "hbrbc_merkle_rows": (ctypes.c_int, [_P, _P, _S, _S, _S, _S, _S, _S, _P, _S, _P]),
        "hbrbc_validate_rows": (ctypes.c_int, [_P, _P, _S, _S, _S, _S, _S, _S, _P, _P, _P, _P, _S,
                                               _P, _S, _S, _S, _P, _P, _S, _P]),
        "hbrbc_reconstruct_rows": (ctypes.c_int, [_P, _P, _S, _S, _S, _S, _S, _P, _S, _P, _P]),
        "hbrbc_decode_rows": (ctypes.c_int, [_P, _P, _S, _S, _S, _S, _S, _P, _S, _P, _S, _P, _S,
                                             ctypes.c_int, _P, _S, _P, _P, _P]),
        "hbrbc_decode_cache_clear": (ctypes.c_int, [_P]),
        "hbrbc_decode_cache_fill": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_uint32)]),
        "hbrbc_decoder_specialise": (ctypes.c_int, [_P, _P, _S]),
        "hbrbc_jit_build_encode_rows": (ctypes.c_int, [_S, _S, _S, _S, ctypes.c_char_p]),
        "hbrbc_jit_encode_file_name": (ctypes.c_int, [_S, _S, _S, _S, ctypes.c_char_p, _S]),
        "hbrbc_jit_decode_groups": (_S, [_S, _S, _P]),
        "hbrbc_jit_build_decode": (ctypes.c_int, [_S, _S, _P, _S, _S, ctypes.c_char_p]),
        "hbrbc_jit_decode_file_name": (ctypes.c_int, [_S, _S, _P, _S, _S, ctypes.c_char_p, _S]),
        "hbrbc_jit_build_decode_variant": (ctypes.c_int, [_S, _S, _P, _S, _S, ctypes.c_int,
                                                          ctypes.c_char_p]),
        "hbrbc_jit_decode_variant_file_name": (ctypes.c_int, [_S, _S, _P, _S, _S, ctypes.c_int,
                                                              ctypes.c_char_p, _S]),
        "hbrbc_unframe_fused": (ctypes.c_int, [_P, _S, _S, _S]),
        "hbrbc_drop_rows": (ctypes.c_int, [_P, _P, _S, _S, _S, _S, _P, _S, ctypes.c_uint8, _P]),
        "hbrbc_pairing_workspace_size": (_S, [_S]),
        "hbrbc_g2_prepared_size": (_S, [_S]),
        "hbrbc_g2_prepare": (ctypes.c_int, [_P, _S, _P, _P]),
        "hbrbc_pairing_check_prepared": (ctypes.c_int, [_P, _P, _S, _P, _P, _S, _P, _P, _P]),
        "hbrbc_pairing_batch": (ctypes.c_int, [_P, _P, _S, _P, _P, _P, _P]),
        "hbrbc_pairing_check_batch": (ctypes.c_int, [_P, _P, _S, _P, _P, _P]),
        "hbrbc_g1_prepared_size": (_S, [_S]),
        "hbrbc_g1_prepare": (ctypes.c_int, [_P, _S, _P, _P]),
        "hbrbc_pairing_check_prepared_keys": (ctypes.c_int, [_P, _P, _S, _P, _P, _S, _P, _P, _S, _P,
                                                             _P, _P]),
        "hbrbc_pairing_check_prepared_pts": (ctypes.c_int, [_P, _P, _S, _P, _P, _S, _P, _P, _S, _P,
                                                            _P, _P]),
        "hbrbc_pairing_check": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p,
                                               ctypes.c_char_p, ctypes.POINTER(ctypes.c_int)]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def _check(code):
    if code == 102:   # HBRBC_E_NO_DEVICE: no silent fallback exists
        raise HbrbcUnavailable(lib().hbrbc_last_error().decode(errors="replace") or "no HIP device")
    if code != 0:
        raise RseError(code, lib().hbrbc_last_error().decode(errors="replace"))


def jit_build_encode(data_shards, parity_shards, directory=None, group=None, rows_per_block=0):
    """Generate + compile (hiprtc, gfx950; no GPU needed) the specialised RS
    encoder for this matrix into the code-object cache (jit.hip): every
    parity-row group, or just `group`; rows_per_block < n builds the variant
    for that blocked row layout."""
    d = directory.encode() if directory else None
    groups = range(jit_encode_groups(data_shards, parity_shards)) if group is None else [group]
    for g in groups:
        _check(lib().hbrbc_jit_build_encode_rows(data_shards, parity_shards, g, rows_per_block, d))


def jit_file_name(data_shards, parity_shards, group=0, rows_per_block=0):
    """Cache file name of one group's specialised-encoder code object."""
    buf = ctypes.create_string_buffer(256)
    _check(lib().hbrbc_jit_encode_file_name(data_shards, parity_shards, group, rows_per_block,
                                            buf, 256))
    return buf.value.decode()


def _mask_buffer(present):
    import numpy as np
    return np.ascontiguousarray(np.asarray(present, dtype=np.uint8) != 0, dtype=np.uint8)


def jit_decode_groups(data_shards, parity_shards, present):
    """Code objects (output-row groups) of the decoder specialised for an
    erasure pattern (present: n flags)."""
    m = _mask_buffer(present)
    return lib().hbrbc_jit_decode_groups(data_shards, parity_shards, m.ctypes.data)


def jit_build_decode(data_shards, parity_shards, present, group, rows_per_block=0,
                     directory=None, fused_unframe=False):
    """Compile one group of the pattern-specialised decoder (or of its
    fused-unframe variant) into the cache."""
    m = _mask_buffer(present)
    d = directory.encode() if directory else None
    _check(lib().hbrbc_jit_build_decode_variant(data_shards, parity_shards, m.ctypes.data,
                                                rows_per_block, group, int(fused_unframe), d))


def jit_decode_file_name(data_shards, parity_shards, present, group=0, rows_per_block=0,
                         fused_unframe=False):
    m = _mask_buffer(present)
    buf = ctypes.create_string_buffer(256)
    _check(lib().hbrbc_jit_decode_variant_file_name(data_shards, parity_shards, m.ctypes.data,
                                                    rows_per_block, group, int(fused_unframe),
                                                    buf, 256))
    return buf.value.decode()


def jit_encode_groups(data_shards, parity_shards):
    """Number of code objects (parity-row groups) of the specialised encoder."""
    return lib().hbrbc_jit_encode_groups(data_shards, parity_shards)


def shard_len(payload_len, data_shards):
    """broadcast.rs:182 -- ceil((len + 4) / data_shards)."""
    return (payload_len + 4 + data_shards - 1) // data_shards


def merkle_node_count(n):
    total, sz = 0, n
    while True:
        total += sz
        if sz <= 1:
            return total
        sz = (sz + 1) // 2


def max_proof_len(n):
    d, sz = 0, n
    while sz > 1:
        d += 1
        sz = (sz + 1) // 2
    return d


def _as_buffer(b):
    """A writable contiguous uint8 buffer for bytes-like / numpy input."""
    import numpy as np
    if isinstance(b, np.ndarray):
        assert b.dtype == np.uint8 and b.flags.c_contiguous
        return b
    if isinstance(b, bytearray):
        return np.frombuffer(b, dtype=np.uint8)
    return np.frombuffer(bytearray(b), dtype=np.uint8)


def _addr(a):
    return a.ctypes.data if a.size else 0


# --------------------------------------------------------------------------
# Mirror of `Coding` (broadcast.rs:639-694)
# --------------------------------------------------------------------------
class Coding:
    """`Coding::new(data_shard_num, parity_shard_num)`; parity 0 = Trivial."""

    def __init__(self, data_shard_num, parity_shard_num, device=-1):
        h = _P()
        _check(lib().hbrbc_coding_new(data_shard_num, parity_shard_num, device, ctypes.byref(h)))
        self._h = h

    @classmethod
    def for_validators(cls, n, device=-1):
        """Broadcast::new (broadcast.rs:98-101): f = (n-1)/3, parity 2f, data n-2f."""
        f = (n - 1) // 3
        return cls(n - 2 * f, 2 * f, device)

    @property
    def handle(self):
        return self._h

    def close(self):
        if self._h:
            lib().hbrbc_coding_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def data_shard_count(self):
        return lib().hbrbc_data_shard_count(self._h)

    def encode_kernel(self):
        """Which encode kernel this context runs: specialised / bitslice / trivial."""
        return lib().hbrbc_encode_kernel(self._h).decode()

    def parity_shard_count(self):
        return lib().hbrbc_parity_shard_count(self._h)

    def encoding_matrix(self):
        import numpy as np
        k, m = self.data_shard_count(), self.parity_shard_count()
        out = np.zeros((k + m, k), np.uint8)
        _check(lib().hbrbc_encoding_matrix(self._h, out.ctypes.data))
        return out

    def encode(self, shards):
        """`Coding::encode(&mut [&mut [u8]])`: parity shards overwritten in place."""
        import numpy as np
        bufs = [_as_buffer(s) for s in shards]
        for s, b in zip(shards, bufs):
            if not isinstance(s, (np.ndarray, bytearray)):
                raise TypeError("encode needs mutable shards (bytearray / np.uint8)")
        ptrs = (ctypes.c_void_p * max(len(bufs), 1))(*[_addr(b) for b in bufs])
        lens = (ctypes.c_size_t * max(len(bufs), 1))(*[b.size for b in bufs])
        _check(lib().hbrbc_encode(self._h, ptrs, lens, len(bufs)))

    def reconstruct_shards(self, shards):
        """`Coding::reconstruct_shards(&mut [Option<Box<[u8]>>])`: None entries are
        replaced by the rebuilt shard (bytes) in place."""
        import numpy as np
        present = [s is not None for s in shards]
        lens = [len(s) if s is not None else 0 for s in shards]
        L = max([l for l, p in zip(lens, present) if p], default=0)
        bufs = [np.frombuffer(bytes(s), np.uint8).copy() if s is not None else
                np.zeros(max(L, 1), np.uint8) for s in shards]
        ptrs = (ctypes.c_void_p * max(len(bufs), 1))(*[_addr(b) for b in bufs])
        lns = (ctypes.c_size_t * max(len(bufs), 1))(*lens)
        pres = (ctypes.c_uint8 * max(len(bufs), 1))(*[1 if p else 0 for p in present])
        _check(lib().hbrbc_reconstruct(self._h, ptrs, lns, pres, len(bufs)))
        for i, p in enumerate(present):
            if not p:
                shards[i] = bufs[i][:L].tobytes()


# --------------------------------------------------------------------------
# Mirror of `MerkleTree` / `Proof` (merkle.rs)
# --------------------------------------------------------------------------
class Proof:
    """`Proof<T>` (merkle.rs:72-78); field order value, index, digests, root_hash."""

    __slots__ = ("_value", "_index", "_digests", "_root", "_valid")

    def __init__(self, value, index, digests, root_hash):
        self._value = bytes(value)
        self._index = int(index)
        self._digests = [bytes(d) for d in digests]
        self._root = bytes(root_hash)
        self._valid = {}   # n -> result: validate is a pure function of the proof

    def validate(self, n):
        """`Proof::validate(n)` (merkle.rs:83-103), on the GPU.  One result per
        (proof, n): a proof delivered to many receivers is hashed once, here or
        in a batch by `validate_proofs`."""
        r = self._valid.get(n)
        if r is None:
            r = self._valid[n] = self._validate_one(n)
            VALIDATE_STATS["single"] += 1
        return r

    def _validate_one(self, n):
        v = _as_buffer(self._value) if self._value else None
        dig = b"".join(self._digests)
        d = _as_buffer(dig) if dig else None
        r = _as_buffer(self._root)
        ok = ctypes.c_int(0)
        _check(lib().hbrbc_proof_validate(_addr(v) if v is not None else 0, len(self._value),
                                          self._index, _addr(d) if d is not None else 0,
                                          len(self._digests), _addr(r), n, ctypes.byref(ok)))
        return bool(ok.value)

    def index(self):
        return self._index

    def root_hash(self):
        return self._root

    def value(self):
        return self._value

    def digests(self):
        return list(self._digests)

    def into_value(self):
        return self._value

    def __eq__(self, other):
        return (isinstance(other, Proof) and self._value == other._value and
                self._index == other._index and self._digests == other._digests and
                self._root == other._root)

    def __repr__(self):
        return "Proof(index=%d, root=%s, %d digests)" % (self._index, self._root.hex()[:10],
                                                         len(self._digests))


VALIDATE_STATS = {"single": 0, "batched": 0, "launches": 0}
_VALIDATE_CTX = {}


def validate_proofs(proofs, n, device=0):
    """`Proof::validate(n)` for many proofs at once: one hbrbc_validate_batch
    launch per distinct value length (normally one: every shard of a
    broadcast has the same length).  Results are memoised on each Proof, so
    the state machine's own `validate` calls then cost nothing.  Proofs that
    do not fit the batched layout (empty value, more digests than a tree over
    n leaves has levels) take the per-call path."""
    import numpy as np
    import torch
    todo, seen = [], set()
    for p in proofs:
        if n not in p._valid and id(p) not in seen:
            seen.add(id(p))
            todo.append(p)
    ds = max_proof_len(n)
    groups = {}
    for p in todo:
        if not p._value or len(p._digests) > ds or p._index > 0xFFFFFFFF:
            p.validate(n)
        else:
            groups.setdefault(len(p._value), []).append(p)
    if not groups:
        return
    ctx = _VALIDATE_CTX.get(device)
    if ctx is None:
        with torch.cuda.device(device):
            ctx = _VALIDATE_CTX[device] = Coding(1, 0, device)
    dev = torch.device("cuda", device)
    for L, ps in groups.items():
        cnt, stride = len(ps), (L + 15) // 16 * 16
        vals = np.zeros((cnt, 1, stride), np.uint8)
        dig = np.zeros((cnt, 1, max(ds, 1), 32), np.uint8)
        ndig = np.zeros((cnt, 1), np.uint8)
        roots = np.zeros((cnt, 32), np.uint8)
        idx = np.zeros((cnt, 1), np.uint32)
        for i, p in enumerate(ps):
            vals[i, 0, :L] = np.frombuffer(p._value, np.uint8)
            for d, dg in enumerate(p._digests):
                dig[i, 0, d] = np.frombuffer(dg, np.uint8)
            ndig[i, 0] = len(p._digests)
            roots[i] = np.frombuffer(p._root, np.uint8)
            idx[i, 0] = p._index
        t = [torch.from_numpy(a).to(dev) for a in (vals, dig, ndig, roots, idx.view(np.int32))]
        ok = torch.zeros((cnt, 1), dtype=torch.uint8, device=dev)
        stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        _check(lib().hbrbc_validate_batch(ctx.handle, t[0].data_ptr(), L, t[0].stride(1),
                                          t[0].stride(0), 1, t[4].data_ptr(), t[1].data_ptr(),
                                          t[2].data_ptr(), t[3].data_ptr(), t[3].stride(0), n, cnt,
                                          ok.data_ptr(), stream))
        res = ok.cpu().numpy()[:, 0]
        for p, r in zip(ps, res):
            p._valid[n] = bool(r)
        VALIDATE_STATS["batched"] += cnt
        VALIDATE_STATS["launches"] += 1


class MerkleTree:
    """`MerkleTree<T>` (merkle.rs:12-69) built on the GPU."""

    def __init__(self, values, nodes):
        self._values = values
        self._nodes = nodes  # numpy [node_count, 32]

    @classmethod
    def from_vec(cls, values):
        import numpy as np
        values = [bytes(v) for v in values]
        n = len(values)
        if n == 0:
            raise RseError(100, "MerkleTree::from_vec of an empty vector panics in the reference")
        bufs = [np.frombuffer(v, np.uint8) if v else np.zeros(1, np.uint8) for v in values]
        ptrs = (ctypes.c_void_p * n)(*[b.ctypes.data for b in bufs])
        lens = (ctypes.c_size_t * n)(*[len(v) for v in values])
        nodes = np.zeros((merkle_node_count(n), 32), np.uint8)
        _check(lib().hbrbc_merkle_build(ptrs, lens, n, nodes.ctypes.data))
        return cls(values, nodes)

    def proof(self, index):
        """`MerkleTree::proof(index)` -> Proof or None."""
        import numpy as np
        n = len(self._values)
        dig = np.zeros((max(max_proof_len(n), 1), 32), np.uint8)
        nd = ctypes.c_size_t(0)
        st = lib().hbrbc_merkle_proof(self._nodes.ctypes.data, n, index, dig.ctypes.data,
                                      ctypes.byref(nd))
        if st == 13:
            return None
        _check(st)
        return Proof(self._values[index], index, [dig[i].tobytes() for i in range(nd.value)],
                     self.root_hash())

    def root_hash(self):
        return self._nodes[-1].tobytes()

    def values(self):
        return list(self._values)

    def into_values(self):
        return self._values

    def levels(self):
        """Leaf digests and every level above them (merkle.rs:13)."""
        out, off, sz = [], 0, len(self._values)
        while True:
            out.append([self._nodes[off + i].tobytes() for i in range(sz)])
            if sz <= 1:
                return out
            off += sz
            sz = (sz + 1) // 2


# --------------------------------------------------------------------------
# Batched device path over torch CUDA tensors
# --------------------------------------------------------------------------
def _ptr(t):
    return t.data_ptr() if t is not None else 0


class RbcBatch:
    """Batched broadcast data path for `count` instances of one (N, f) on one
    GPU.  Owns nothing but the `Coding` context; every buffer is a torch tensor
    on the context's device.  Calls are asynchronous on `stream` (a
    torch.cuda.Stream; default: torch's current stream)."""

    def __init__(self, n, f=None, device=0):
        import torch
        if not torch.cuda.is_available():
            raise HbrbcUnavailable("no GPU visible: the RBC path has no CPU fallback")
        self.n = n
        self.f = (n - 1) // 3 if f is None else f
        self.m = 2 * self.f
        self.k = n - self.m
        self.device = torch.device("cuda", device)
        with torch.cuda.device(self.device):
            self.coding = Coding(self.k, self.m, device)
        self.node_count = merkle_node_count(n)
        self.dslots = max_proof_len(n)

    # -- layout helpers -----------------------------------------------------
    # row slot alignment of the slabs (bytes; A/B knob HBRBC_ROW_ALIGN, a
    # multiple of 16): rows are S bytes rounded up to it
    ROW_ALIGN = int(os.environ.get("HBRBC_ROW_ALIGN", "16"))

    @staticmethod
    def stride_for(S):
        a = RbcBatch.ROW_ALIGN
        return (S + a - 1) // a * a

    def alloc_slab(self, count, S):
        import torch
        stride = self.stride_for(S)
        return torch.empty((count, self.n, stride), dtype=torch.uint8, device=self.device)

    def alloc_nodes(self, count):
        import torch
        return torch.empty((count, self.node_count, 32), dtype=torch.uint8, device=self.device)

    def _stream(self, stream):
        import torch
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        return ctypes.c_void_p(s.cuda_stream)

    # -- entry points ----------------------------------------------------------
    def frame(self, payloads, plen, slab, stream=None):
        count = slab.shape[0]
        S = shard_len(plen, self.k)
        _check(lib().hbrbc_frame_batch(self.coding.handle, _ptr(payloads), payloads.stride(0),
                                       plen, count, _ptr(slab), S, slab.stride(1),
                                       slab.stride(0), self._stream(stream)))

    def frame_encode(self, payloads, plen, slab, stream=None):
        """frame + encode in one pass when the specialised encoder is loaded."""
        count = slab.shape[0]
        S = shard_len(plen, self.k)
        _check(lib().hbrbc_frame_encode_batch(self.coding.handle, _ptr(payloads), payloads.stride(0),
                                              plen, count, _ptr(slab), S, slab.stride(1),
                                              slab.stride(0), self._stream(stream)))

    def encode(self, slab, S, stream=None):
        _check(lib().hbrbc_encode_batch(self.coding.handle, _ptr(slab), S, slab.stride(1),
                                        slab.stride(0), slab.shape[0], self._stream(stream)))

    def merkle(self, slab, S, nodes, stream=None):
        _check(lib().hbrbc_merkle_batch(self.coding.handle, _ptr(slab), S, slab.stride(1),
                                        slab.stride(0), slab.shape[0], _ptr(nodes),
                                        nodes.stride(0), self._stream(stream)))

    def proofs(self, nodes, digests, ndig, stream=None):
        """digests: uint8 [count, n, max(dslots,1), 32]; ndig: uint8 [count, n]."""
        _check(lib().hbrbc_proofs_batch(self.coding.handle, _ptr(nodes), nodes.stride(0),
                                        nodes.shape[0], _ptr(digests), _ptr(ndig),
                                        self._stream(stream)))

    def validate(self, slab, S, digests, ndig, nodes, ok, indices=None, leaf_out=None,
                 stream=None):
        """Validate all n proofs of every instance against its own root.
        leaf_out: a node slab [count, node_count, 32] whose level 0 receives
        each validated row's Merkle leaf (hbrbc_validate_rows), for a decode
        with known_leaves."""
        count = slab.shape[0]
        root = nodes[:, -1, :]
        if leaf_out is not None:
            self.validate_layout(slab, S, count, self.n, slab.stride(1), 0, 0, slab.stride(0),
                                 digests, ndig, self.n, root, ok, indices=indices,
                                 leaf_out=leaf_out, stream=stream)
            return
        _check(lib().hbrbc_validate_batch(self.coding.handle, _ptr(slab), S, slab.stride(1),
                                          slab.stride(0), self.n, _ptr(indices), _ptr(digests),
                                          _ptr(ndig), _ptr(root), nodes.stride(0), self.n,
                                          count, _ptr(ok), self._stream(stream)))

    def validate_rows(self, values, S, per_inst, indices, digests, ndig, roots, ok, stream=None):
        """Proof::validate for proofs laid out as [count][per_inst] rows: values
        uint8 [count, per_inst, >=S] (any row/instance stride that is a multiple of
        8), indices int32 [count, per_inst] (the index each proof claims and
        the receiver expects), digests uint8 [count, per_inst, dslots, 32],
        ndig uint8 [count, per_inst], roots uint8 [count, >=32], ok uint8
        [count, per_inst].  Trees have self.n leaves."""
        count = values.shape[0]
        for t in (indices, digests, ndig, ok):
            assert t.is_contiguous() and t.shape[0] == count and t.shape[1] == per_inst
        _check(lib().hbrbc_validate_batch(self.coding.handle, _ptr(values), S, values.stride(1),
                                          values.stride(0), per_inst, _ptr(indices), _ptr(digests),
                                          _ptr(ndig), _ptr(roots), roots.stride(0), self.n, count,
                                          _ptr(ok), self._stream(stream)))

    # -- ragged batches (hbrbc.h): proposals of different lengths, one launch per stage
    def frame_encode_ragged(self, payloads, plens, max_plen, slab, stream=None):
        """payloads [count, >=max_plen]; plens int32 device [count]; slab [count, n, stride]
        with stride >= round_up(shard_len(max_plen), 16)."""
        _check(lib().hbrbc_frame_encode_ragged(self.coding.handle, _ptr(payloads),
                                               payloads.stride(0), _ptr(plens), max_plen,
                                               slab.shape[0], _ptr(slab), slab.stride(1),
                                               slab.stride(0), self._stream(stream)))

    def merkle_ragged(self, slab, slens, nodes, stream=None):
        _check(lib().hbrbc_merkle_ragged(self.coding.handle, _ptr(slab), _ptr(slens),
                                         slab.stride(1), slab.stride(0), slab.shape[0],
                                         _ptr(nodes), nodes.stride(0), self._stream(stream)))

    # -- blocked row layouts (hbrbc.h "*_rows"): row j of instance i at
    #    base + i*inst_stride + (j // rpb)*block_stride + (j % rpb)*shard_stride
    def frame_encode_rows(self, payloads, plen, base, count, shard_stride, rows_per_block,
                          block_stride, inst_stride, stream=None):
        S = shard_len(plen, self.k)
        _check(lib().hbrbc_frame_encode_rows(self.coding.handle, _ptr(payloads), payloads.stride(0),
                                             plen, count, _ptr(base), S, shard_stride,
                                             rows_per_block, block_stride, inst_stride,
                                             self._stream(stream)))

    def merkle_rows(self, base, S, count, shard_stride, rows_per_block, block_stride, inst_stride,
                    nodes, stream=None):
        _check(lib().hbrbc_merkle_rows(self.coding.handle, _ptr(base), S, shard_stride,
                                       rows_per_block, block_stride, inst_stride, count,
                                       _ptr(nodes), nodes.stride(0), self._stream(stream)))

    def validate_layout(self, base, S, count, per_inst, shard_stride, rows_per_block, block_stride,
                        inst_stride, digests, ndig, digest_rows, roots, ok, rows=None,
                        indices=None, leaf_out=None, stream=None):
        """Proof::validate of `per_inst` rows (`rows`: int32 device list, or
        0..per_inst-1) of every instance in a (blocked) row layout; digests
        [count, digest_rows, dslots, 32], ndig [count, digest_rows]; leaf_out:
        node slab [count, node_count, 32] whose level 0 receives the leaves."""
        _check(lib().hbrbc_validate_rows(
            self.coding.handle, _ptr(base), S, shard_stride, rows_per_block, block_stride,
            inst_stride, per_inst, _ptr(rows), _ptr(indices), _ptr(digests), _ptr(ndig),
            digest_rows, _ptr(roots), roots.stride(0), self.n, count, _ptr(ok), _ptr(leaf_out),
            leaf_out.stride(0) if leaf_out is not None else 0, self._stream(stream)))

    def decode_rows(self, base, S, count, shard_stride, rows_per_block, block_stride, inst_stride,
                    present, roots, nodes, payload_out, plen_out, status, known_leaves=False,
                    stream=None):
        _check(lib().hbrbc_decode_rows(
            self.coding.handle, _ptr(base), S, shard_stride, rows_per_block, block_stride,
            inst_stride, _ptr(present), count, _ptr(roots), roots.stride(0), _ptr(nodes),
            nodes.stride(0), 1 if known_leaves else 0, _ptr(payload_out), payload_out.stride(0),
            _ptr(plen_out), _ptr(status), self._stream(stream)))

    def specialise_decoder(self, present, rows_per_block=0):
        """hbrbc_decoder_specialise: an XOR-network decoder for one erasure
        pattern (present: n flags) in layouts with this rows_per_block."""
        m = _mask_buffer(present)
        assert m.size == self.n
        _check(lib().hbrbc_decoder_specialise(self.coding.handle, m.ctypes.data, rows_per_block))

    def decode_cache_clear(self):
        _check(lib().hbrbc_decode_cache_clear(self.coding.handle))

    def decode_cache_fill(self):
        v = ctypes.c_uint32(0)
        _check(lib().hbrbc_decode_cache_fill(self.coding.handle, ctypes.byref(v)))
        return v.value

    def reconstruct(self, slab, S, present, status, stream=None):
        _check(lib().hbrbc_reconstruct_batch(self.coding.handle, _ptr(slab), S, slab.stride(1),
                                             slab.stride(0), _ptr(present), slab.shape[0],
                                             _ptr(status), self._stream(stream)))

    def drop_rows(self, slab, present, fill=0xA5, stream=None):
        """Overwrite every row with present == 0 (whole slot) with `fill`: the
        rows a receiver never got (hbrbc_drop_rows); slab [count][n][stride]."""
        _check(lib().hbrbc_drop_rows(self.coding.handle, _ptr(slab), slab.stride(1), 0, 0,
                                     slab.stride(0), _ptr(present), slab.shape[0], fill,
                                     self._stream(stream)))

    def unframe_fused(self, S, payload_stride, rows_per_block=0):
        """Whether decode writes the payload from the reconstruct kernel (same
        outputs either way; where the bytes move, for accounting)."""
        return bool(lib().hbrbc_unframe_fused(self.coding.handle, S, payload_stride,
                                              rows_per_block))

    def decode(self, slab, S, present, roots, nodes, payload_out, plen_out, status,
               known_leaves=False, stream=None):
        """roots: uint8 [count, >=32] (row stride multiple of 16).  known_leaves:
        level 0 of `nodes` already holds the leaves of the present rows (from
        validate(leaf_out=nodes)); only the rebuilt rows are hashed again."""
        if known_leaves:
            self.decode_rows(slab, S, slab.shape[0], slab.stride(1), 0, 0, slab.stride(0),
                             present, roots, nodes, payload_out, plen_out, status,
                             known_leaves=True, stream=stream)
            return
        _check(lib().hbrbc_decode_batch(self.coding.handle, _ptr(slab), S, slab.stride(1),
                                        slab.stride(0), _ptr(present), slab.shape[0],
                                        _ptr(roots), roots.stride(0), _ptr(nodes),
                                        nodes.stride(0), _ptr(payload_out),
                                        payload_out.stride(0), _ptr(plen_out), _ptr(status),
                                        self._stream(stream)))

    # -- bincode wire format of broadcast::Message (message.rs:13-24) -------------
    def wire_slot(self, S):
        """Message slot bytes for Value/Echo messages of S-byte shards."""
        return (lib().hbrbc_wire_proof_message_len(S, self.dslots) + 15) // 16 * 16

    def wire_encode(self, values, S, digests, ndig, roots, out, msg_len, variant=0, indices=None,
                    stream=None):
        """Value (variant 0) or Echo (1) messages of proofs laid out as for
        validate_rows: values [count, per_inst, >=S] (16-aligned rows), digests
        [count, per_inst, dslots, 32], ndig [count, per_inst], roots [count, >=32];
        out uint8 [count*per_inst, slot], msg_len int32 [count*per_inst]."""
        count, per_inst = values.shape[0], values.shape[1]
        _check(lib().hbrbc_wire_encode_batch(self.coding.handle, variant, _ptr(values), S,
                                             values.stride(1), values.stride(0), per_inst,
                                             _ptr(indices), _ptr(digests), _ptr(ndig),
                                             _ptr(roots), roots.stride(0), count, _ptr(out),
                                             out.stride(0), _ptr(msg_len), self._stream(stream)))

    def wire_decode(self, msgs, msg_len, values, value_len, index, digests, ndig, roots, variant,
                    status, stream=None):
        """Parse msgs uint8 [nmsg, slot] (msg_len int32 [nmsg]) into values
        [nmsg, stride], value_len/index/variant/status int32 [nmsg], digests
        [nmsg, dslots, 32], ndig uint8 [nmsg], roots [nmsg, 32]."""
        _check(lib().hbrbc_wire_decode_batch(self.coding.handle, _ptr(msgs), msgs.stride(0),
                                             _ptr(msg_len), msgs.shape[0], _ptr(values),
                                             values.stride(0), _ptr(value_len), _ptr(index),
                                             _ptr(digests), _ptr(ndig), _ptr(roots), _ptr(variant),
                                             _ptr(status), self._stream(stream)))

    def own_stream(self):
        """The context's own HIP stream (created with the context, so the
        contexts of one process sit on successive hardware queues) wrapped as a
        torch stream."""
        import torch
        return torch.cuda.ExternalStream(lib().hbrbc_stream(self.coding.handle), device=self.device)

    def reserve(self, count):
        _check(lib().hbrbc_reserve(self.coding.handle, count))

    # -- profiling ---------------------------------------------------------
    def profile(self, enable=True):
        _check(lib().hbrbc_profile_enable(self.coding.handle, 1 if enable else 0))

    def profile_reset(self):
        _check(lib().hbrbc_profile_reset(self.coding.handle))

    def profile_read(self):
        ms = (ctypes.c_double * len(STAGES))()
        cnt = (ctypes.c_uint64 * len(STAGES))()
        _check(lib().hbrbc_profile_read(self.coding.handle, ms, cnt))
        return {STAGES[i]: (ms[i], cnt[i]) for i in range(len(STAGES))}


# --------------------------------------------------------------------------
# Epoch batching: every proposer's send_shards in one pass
# --------------------------------------------------------------------------
SEND_STATS = {"trees": 0, "launches": 0}
_SEND_BATCH = {}


def send_shards_batch(items, device=0):
    """The proposer half of `Broadcast::send_shards` (broadcast.rs:170-225:
    BE32 length prefix, zero pad to N shards of ceil((P+4)/k) bytes, encode,
    `MerkleTree::from_vec`) for many proposals at once, e.g. the N
    contributions of one Subset / HoneyBadger epoch (subset/proposal_state.rs
    :69-113, honey_badger/epoch_state.rs:223-236), or many epochs.
    items: [(n, value bytes)].  Proposals with the same validator count share
    one frame+encode launch and one tree launch whatever their lengths
    (hbrbc_frame_encode_batch / hbrbc_merkle_batch when the lengths agree,
    the ragged forms when they do not); returns one `MerkleTree` per item,
    equal to the per-call from_vec over the encoded shards."""
    import numpy as np
    import torch
    if not torch.cuda.is_available():
        raise HbrbcUnavailable("no GPU visible: the RBC path has no CPU fallback")
    out = [None] * len(items)
    groups = {}
    for i, (n, value) in enumerate(items):
        groups.setdefault(int(n), []).append(i)
    dev = torch.device("cuda", device)
    for n, idx in groups.items():
        rb = _SEND_BATCH.get((n, device))
        if rb is None:
            rb = _SEND_BATCH[(n, device)] = RbcBatch(n, device=device)
        count = len(idx)
        lens = [len(items[i][1]) for i in idx]
        pmax = max(lens)
        Ss = [shard_len(L, rb.k) for L in lens]
        pay = np.zeros((count, max(16, (pmax + 15) // 16 * 16)), np.uint8)
        for r, i in enumerate(idx):
            if lens[r]:
                pay[r, :lens[r]] = np.frombuffer(bytes(items[i][1]), np.uint8)
        payloads = torch.from_numpy(pay).to(dev)
        nodes = rb.alloc_nodes(count)
        if len(set(lens)) == 1:
            S = Ss[0]
            slab = rb.alloc_slab(count, S)
            if rb.m:
                rb.frame_encode(payloads, pmax, slab)
            else:   # Coding::Trivial (N <= 3): no parity
                rb.frame(payloads, pmax, slab)
            rb.merkle(slab, S, nodes)
        else:       # ragged: one launch per stage for every length
            slab = rb.alloc_slab(count, shard_len(pmax, rb.k))
            rb.frame_encode_ragged(payloads, torch.tensor(lens, dtype=torch.int32, device=dev),
                                   pmax, slab)
            rb.merkle_ragged(slab, torch.tensor(Ss, dtype=torch.int32, device=dev), nodes)
        sl, nd = slab.cpu().numpy(), nodes.cpu().numpy()
        for r, i in enumerate(idx):
            out[i] = MerkleTree([sl[r, j, :Ss[r]].tobytes() for j in range(n)], nd[r].copy())
        SEND_STATS["trees"] += count
        SEND_STATS["launches"] += 1
    return out


# --------------------------------------------------------------------------
# Deferred decodes of many Broadcast instances
# --------------------------------------------------------------------------
DECODE_STATS = {"decodes": 0, "launches": 0}
_DECODE_BATCH = {}


def decode_shards_batch(requests, device=0):
    """`Broadcast::decode_from_shards` (broadcast.rs:563-601) for many
    instances at once: requests [(n, leaf_values, root)] with leaf_values a
    list of n shards (bytes, or None when missing) -> [payload bytes or None].
    Shards of one instance must share one non-zero length, else rse's
    reconstruct fails (IncorrectShardSize / EmptyShard) and so does the decode;
    the rest go through hbrbc_decode_batch, one launch per (n, shard length):
    reconstruct, re-tree over all n shards, root compare, BE32 length,
    truncating take -- None for every rse error, root mismatch or missing
    length, as in the reference."""
    import numpy as np
    import torch
    if not torch.cuda.is_available():
        raise HbrbcUnavailable("no GPU visible: the RBC path has no CPU fallback")
    out = [None] * len(requests)
    groups = {}
    for i, (n, leaves, root) in enumerate(requests):
        lens = {len(v) for v in leaves if v is not None}
        if len(leaves) != n or len(lens) != 1 or 0 in lens:
            continue   # TooFewShardsPresent (nothing present) / IncorrectShardSize / EmptyShard
        groups.setdefault((int(n), lens.pop()), []).append(i)
    dev = torch.device("cuda", device)
    for (n, S), idx in groups.items():
        rb = _DECODE_BATCH.get((n, device))
        if rb is None:
            rb = _DECODE_BATCH[(n, device)] = RbcBatch(n, device=device)
        cnt, stride = len(idx), RbcBatch.stride_for(S)
        slab = np.zeros((cnt, n, stride), np.uint8)
        present = np.zeros((cnt, n), np.uint8)
        roots = np.zeros((cnt, 32), np.uint8)
        for r, i in enumerate(idx):
            _, leaves, root = requests[i]
            for j, v in enumerate(leaves):
                if v is not None:
                    slab[r, j, :S] = np.frombuffer(bytes(v), np.uint8)
                    present[r, j] = 1
            roots[r] = np.frombuffer(bytes(root), np.uint8)
        t_slab = torch.from_numpy(slab).to(dev)
        t_pres = torch.from_numpy(present).to(dev)
        t_roots = torch.from_numpy(roots).to(dev)
        nodes = rb.alloc_nodes(cnt)
        prow = max(16, (rb.k * S + 15) // 16 * 16)
        pay = torch.empty((cnt, prow), dtype=torch.uint8, device=dev)
        plen = torch.zeros(cnt, dtype=torch.int32, device=dev)
        status = torch.zeros(cnt, dtype=torch.int32, device=dev)
        rb.decode(t_slab, S, t_pres, t_roots, nodes, pay, plen, status)
        st, pl, py = status.cpu().numpy(), plen.cpu().numpy(), pay.cpu().numpy()
        for r, i in enumerate(idx):
            if st[r] == 0:
                out[i] = py[r, :pl[r]].tobytes()
        DECODE_STATS["decodes"] += cnt
        DECODE_STATS["launches"] += 1
    return out
