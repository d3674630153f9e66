"""Checker backend for hbbft_amd.broadcast.Broadcast: `Coding`, `MerkleTree`
and `Proof` over the CPU oracle (oracle/liborc.so).

TEST INFRASTRUCTURE ONLY.  It lets the CPU suite run the Broadcast state
machine (the host-side caller logic) without a GPU; the product default is the
HIP backend, and the GPU tests run the same scenarios through libhbrbc.so.
"""
import numpy as np

from oracle import pyoracle as orc


class RseError(Exception):
    def __init__(self, code):
        super().__init__("rse error %d" % code)
        self.code = code


class Coding:
    """`Coding` (broadcast.rs:639-694) on the oracle (rse 4.0.x restatement)."""

    def __init__(self, data_shard_num, parity_shard_num):
        if data_shard_num == 0:
            raise RseError(3)   # TooFewDataShards
        if data_shard_num + parity_shard_num > 256:
            raise RseError(2)   # TooManyShards
        self.k, self.m = data_shard_num, parity_shard_num

    def data_shard_count(self):
        return self.k

    def parity_shard_count(self):
        return self.m

    def encode(self, shards):
        if self.m == 0:
            return
        st, out = orc.rs_encode(self.k, self.m, [np.frombuffer(bytes(s), np.uint8).copy()
                                                 for s in shards])
        if st:
            raise RseError(st)
        for s, o in zip(shards, out):
            s[:] = o.tobytes()

    def reconstruct_shards(self, shards):
        if self.m == 0:
            if all(s is not None for s in shards):
                return
            raise RseError(10)  # TooFewShardsPresent
        st, out = orc.coding_reconstruct(
            self.k, self.m, [None if s is None else np.frombuffer(bytes(s), np.uint8) for s in shards])
        if st:
            raise RseError(st)
        for i, s in enumerate(shards):
            if s is None:
                shards[i] = out[i].tobytes()


STATS = {"single": 0, "batched": 0, "launches": 0}


class Proof:
    __slots__ = ("_value", "_index", "_digests", "_root", "_valid")

    def __init__(self, value, index, digests, root_hash):
        self._value = bytes(value)
        self._index = int(index)
        self._digests = [bytes(d) for d in digests]
        self._root = bytes(root_hash)
        self._valid = {}

    def validate(self, n):
        r = self._valid.get(n)
        if r is None:
            r = self._valid[n] = self._check(n)
            STATS["single"] += 1
        return r

    def _check(self, n):
        dig = np.frombuffer(b"".join(self._digests), np.uint8).reshape(-1, 32)
        return orc.proof_validate(self._value, self._index, dig, self._root, n)


    def index(self):
        return self._index

    def root_hash(self):
        return self._root

    def value(self):
        return self._value

    def digests(self):
        return list(self._digests)

    def __eq__(self, other):
        return (self._value == other._value and self._index == other._index and
                self._digests == other._digests and self._root == other._root)


def validate_proofs(proofs, n, device=0):
    """Checker twin of hbbft_amd.validate_proofs (one 'launch' per call)."""
    todo = {id(p): p for p in proofs if n not in p._valid}
    for p in todo.values():
        p._valid[n] = p._check(n)
    if todo:
        STATS["batched"] += len(todo)
        STATS["launches"] += 1


class MerkleTree:
    def __init__(self, values, nodes):
        self._values = values
        self._nodes = nodes

    @classmethod
    def from_vec(cls, values):
        values = [bytes(v) for v in values]
        return cls(values, orc.merkle_build(values))

    def proof(self, index):
        n = len(self._values)
        if index >= n:
            return None
        dig = orc.merkle_proof(self._nodes, n, index)
        return Proof(self._values[index], index, [d.tobytes() for d in dig], self.root_hash())

    def root_hash(self):
        return self._nodes[-1].tobytes()

    def values(self):
        return list(self._values)

    def into_values(self):
        return self._values


SEND_STATS = {"trees": 0, "launches": 0}


def send_shards_batch(items, device=0):
    """Checker twin of hbbft_amd.send_shards_batch: orc.send_shards per item
    (frame + encode + tree of broadcast.rs:170-204)."""
    out = []
    for n, value in items:
        shards, nodes = orc.send_shards(n, (n - 1) // 3, bytes(value))
        out.append(MerkleTree([shards[j].tobytes() for j in range(n)], nodes))
    SEND_STATS["trees"] += len(items)
    SEND_STATS["launches"] += 1
    return out
