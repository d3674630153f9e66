"""Host mirror of `broadcast::Broadcast` over the HIP data path.

The RBC message state machine of /root/reference/src/broadcast/broadcast.rs
(Value / Echo / EchoHash / CanDecode / Ready handling, thresholds, targeting)
restated line by line in Python, so the caller logic the reference keeps on
the host runs unchanged on top of this repository's `Coding`, `MerkleTree` and
`Proof` (hbbft_amd/__init__.py -> libhbrbc.so).  Every data operation of the
path -- encode (broadcast.rs:193), tree (204), proofs (213), validate (605),
reconstruct (569), re-tree (580) -- goes through those classes; this module
only does the bookkeeping and the framing byte shuffles.

`backend` is the object supplying `Coding`, `MerkleTree` and `Proof`; it
defaults to the HIP classes (there is no CPU fallback: without a GPU,
`Coding` raises `HbrbcUnavailable`).  Tests substitute a checker backend.
"""
import enum
import struct

__all__ = ["ValidatorSet", "Target", "TargetedMessage", "Message", "Fault", "FaultKind", "Step",
           "BroadcastError", "ErrorKind", "Broadcast", "prevalidate", "broadcast_many"]


# --------------------------------------------------------------------------
# L1 plumbing the state machine needs (network_info.rs, messaging.rs,
# fault_log.rs, traits.rs)
# --------------------------------------------------------------------------
class ValidatorSet:
    """`ValidatorSet` (network_info.rs:12-85): ids sorted, index = sorted
    position (this is the shard index, broadcast.rs:212), f = (N-1)/3
    (util.rs:22-25)."""

    def __init__(self, ids):
        self._ids = sorted(set(ids))
        if not self._ids:
            raise ValueError("empty validator set")
        self._index = {v: i for i, v in enumerate(self._ids)}
        self._f = (len(self._ids) - 1) // 3

    def contains(self, node_id):
        return node_id in self._index

    def index(self, node_id):
        return self._index.get(node_id)

    def num(self):
        return len(self._ids)

    def num_faulty(self):
        return self._f

    def num_correct(self):
        return len(self._ids) - self._f

    def all_ids(self):
        return list(self._ids)

    def all_indices(self):
        return list(self._index.items())


class Target:
    """`Target::{Nodes, AllExcept}` (messaging.rs:15-23)."""

    __slots__ = ("all_except", "ids")

    def __init__(self, all_except, ids):
        self.all_except = bool(all_except)
        self.ids = frozenset(ids)

    @classmethod
    def nodes(cls, ids):
        return cls(False, ids)

    @classmethod
    def node(cls, node_id):
        return cls(False, (node_id,))

    @classmethod
    def all_except_ids(cls, ids):
        return cls(True, ids)

    @classmethod
    def all(cls):
        return cls(True, ())

    def contains(self, node_id):
        return (node_id not in self.ids) if self.all_except else (node_id in self.ids)

    def message(self, msg):
        return TargetedMessage(self, msg)

    def __repr__(self):
        return "%s(%s)" % ("AllExcept" if self.all_except else "Nodes", sorted(self.ids))


class TargetedMessage:
    __slots__ = ("target", "message")

    def __init__(self, target, message):
        self.target = target
        self.message = message


class Message:
    """`broadcast::Message` (message.rs:13-24): kind is one of VALUE, ECHO
    (payload: Proof), READY, CAN_DECODE, ECHO_HASH (payload: 32-byte digest).
    The variant numbers are the bincode tags (hbbft_amd/csrc/wire.hip)."""

    VALUE, ECHO, READY, CAN_DECODE, ECHO_HASH = range(5)
    _NAMES = ("Value", "Echo", "Ready", "CanDecode", "EchoHash")
    __slots__ = ("kind", "payload")

    def __init__(self, kind, payload):
        self.kind = kind
        self.payload = payload if kind <= Message.ECHO else bytes(payload)

    @classmethod
    def value(cls, proof):
        return cls(cls.VALUE, proof)

    @classmethod
    def echo(cls, proof):
        return cls(cls.ECHO, proof)

    @classmethod
    def ready(cls, digest):
        return cls(cls.READY, digest)

    @classmethod
    def can_decode(cls, digest):
        return cls(cls.CAN_DECODE, digest)

    @classmethod
    def echo_hash(cls, digest):
        return cls(cls.ECHO_HASH, digest)

    def __eq__(self, other):
        return isinstance(other, Message) and self.kind == other.kind and \
            self.payload == other.payload

    def __repr__(self):
        if self.kind <= Message.ECHO:
            return "%s(%r)" % (self._NAMES[self.kind], self.payload)
        return "%s(%s)" % (self._NAMES[self.kind], self.payload.hex()[:10])


class FaultKind(enum.Enum):
    """`broadcast::FaultKind` (error.rs:28-50)."""
    ReceivedValueFromNonProposer = 0
    MultipleValues = 1
    MultipleEchos = 2
    MultipleEchoHashes = 3
    MultipleReadys = 4
    InvalidProof = 5
    BroadcastDecoding = 6


class ErrorKind(enum.Enum):
    """`broadcast::Error` (error.rs:5-21)."""
    InvalidNodeCount = 0
    InstanceCannotPropose = 1
    MultipleInputs = 2
    ProofConstructionFailed = 3
    UnknownSender = 4


class BroadcastError(Exception):
    def __init__(self, kind):
        super().__init__(kind.name)
        self.kind = kind


class Fault:
    """`Fault { node_id, kind }` (fault_log.rs:13-30)."""
    __slots__ = ("node_id", "kind")

    def __init__(self, node_id, kind):
        self.node_id = node_id
        self.kind = kind

    def __repr__(self):
        return "Fault(%r, %s)" % (self.node_id, self.kind.name)


class Step:
    """`Step { output, fault_log, messages }` (traits.rs:64-161)."""
    __slots__ = ("output", "fault_log", "messages")

    def __init__(self):
        self.output = []
        self.fault_log = []
        self.messages = []

    @classmethod
    def from_fault(cls, node_id, kind):
        s = cls()
        s.fault_log.append(Fault(node_id, kind))
        return s

    @classmethod
    def from_message(cls, tmsg):
        s = cls()
        s.messages.append(tmsg)
        return s

    def extend(self, other):
        self.output.extend(other.output)
        self.fault_log.extend(other.fault_log)
        self.messages.extend(other.messages)

    def join(self, other):
        self.extend(other)
        return self


# --------------------------------------------------------------------------
# The Reliable Broadcast state machine (broadcast.rs:23-629)
# --------------------------------------------------------------------------
def _default_backend():
    import hbbft_amd
    return hbbft_amd


class _EchoHash:
    """`EchoContent::Hash` (broadcast.rs:696-721); `EchoContent::Full` is the Proof itself."""
    __slots__ = ("digest",)

    def __init__(self, digest):
        self.digest = digest


def _echo_hash(content):
    return content.digest if isinstance(content, _EchoHash) else content.root_hash()


def _echo_proof(content):
    return None if isinstance(content, _EchoHash) else content


class Broadcast:
    """`Broadcast<N>` (broadcast.rs:23-55, 90-629)."""

    def __init__(self, our_id, val_set, proposer_id, backend=None, device=-1):
        """`Broadcast::new` (broadcast.rs:93-120)."""
        self._be = backend if backend is not None else _default_backend()
        self.our_id = our_id
        self.val_set = val_set if isinstance(val_set, ValidatorSet) else ValidatorSet(val_set)
        self.proposer_id = proposer_id
        parity = 2 * self.val_set.num_faulty()
        data = self.val_set.num() - parity
        try:
            self.coding = self._be.Coding(data, parity, device) if device != -1 \
                else self._be.Coding(data, parity)
        except self._be.RseError as e:   # rse TooManyShards etc. (broadcast.rs:101)
            if getattr(e, "code", 0) >= 100:
                raise
            raise BroadcastError(ErrorKind.InvalidNodeCount)
        self._k, self._m = data, parity
        self.device = device if device >= 0 else 0   # batched helpers run on this GPU
        self.value_sent = False
        self.echo_sent = False
        self.ready_sent = False
        self.echo_hash_sent = False
        self.can_decode_sent = set()
        self.decided = False
        self.fault_estimate = self.val_set.num_faulty()
        self.echos = {}         # sender -> Proof | _EchoHash
        self.can_decodes = {}   # digest -> set(sender)
        self.readys = {}        # sender -> digest
        # deferred decoding (run_lockstep): a list the decode requests go to
        # instead of decoding at once; resolve_decodes() completes them
        self.decode_sink = None
        self._decode_pending = None

    # -- ConsensusProtocol (broadcast.rs:60-88) ------------------------------
    def handle_input(self, value):
        return self.broadcast(value)

    def terminated(self):
        return self.decided

    def validator_set(self):
        return self.val_set

    def broadcast(self, value, _mtree=None):
        """broadcast.rs:123-137.  `_mtree`: the tree of this value's shards,
        already built by `broadcast_many`."""
        if self.our_id != self.proposer_id:
            raise BroadcastError(ErrorKind.InstanceCannotPropose)
        if self.value_sent:
            raise BroadcastError(ErrorKind.MultipleInputs)
        self.value_sent = True
        proof, step = self._send_shards(bytes(value), _mtree)
        return step.join(self._handle_value(self.our_id, proof))

    def handle_message(self, sender_id, message):
        """broadcast.rs:142-153."""
        if not self.val_set.contains(sender_id):
            raise BroadcastError(ErrorKind.UnknownSender)
        if self._decode_pending is not None:
            # a deferred decode decides this instance's next state: the caller
            # must resolve it first (decode_sink is run_lockstep's contract:
            # one message per instance per round, then resolve_decodes)
            raise RuntimeError("%r: message delivered while a deferred decode is pending; "
                               "call resolve_decodes() first" % (self,))
        k = message.kind
        if k == Message.VALUE:
            return self._handle_value(sender_id, message.payload)
        if k == Message.ECHO:
            return self._handle_echo(sender_id, message.payload)
        if k == Message.READY:
            return self._handle_ready(sender_id, message.payload)
        if k == Message.CAN_DECODE:
            return self._handle_can_decode(sender_id, message.payload)
        return self._handle_echo_hash(sender_id, message.payload)

    # -- proposer ---------------------------------------------------------------
    def _send_shards(self, value, mtree=None):
        """broadcast.rs:170-225: BE32 length prefix, shard_len = ceil(len/k),
        zero pad to (k+m) shards, encode parity in place, tree, one proof per
        validator."""
        if mtree is None:
            k, m = self._k, self._m
            framed = struct.pack(">I", len(value) & 0xFFFFFFFF) + value
            shard_len = (len(framed) + k - 1) // k
            buf = bytearray(framed) + bytearray(shard_len * (k + m) - len(framed))
            shards = [bytearray(buf[i * shard_len:(i + 1) * shard_len]) for i in range(k + m)]
            self.coding.encode(shards)
            mtree = self._be.MerkleTree.from_vec([bytes(s) for s in shards])
        assert self.val_set.num() == len(mtree.values())
        step = Step()
        result = None
        for node_id, index in self.val_set.all_indices():
            proof = mtree.proof(index)
            if proof is None:
                raise BroadcastError(ErrorKind.ProofConstructionFailed)
            if node_id == self.our_id:
                result = proof
            else:
                step.messages.append(Target.node(node_id).message(Message.value(proof)))
        if result is None:
            raise BroadcastError(ErrorKind.ProofConstructionFailed)
        return result, step

    # -- handlers ---------------------------------------------------------------
    def _handle_value(self, sender_id, p):
        """broadcast.rs:228-263."""
        if sender_id != self.proposer_id:
            return Step.from_fault(sender_id, FaultKind.ReceivedValueFromNonProposer)
        ours = self.echos.get(self.our_id)
        if ours is not None:
            if _echo_hash(ours) != p.root_hash():
                return Step.from_fault(sender_id, FaultKind.MultipleValues)
            if _echo_proof(ours) is not None and ours == p:
                return Step()   # Value received twice (warn! only)
        if not self._validate_proof(p, self.our_id):
            return Step.from_fault(sender_id, FaultKind.InvalidProof)
        echo_hash_steps = self._send_echo_hash(p.root_hash())
        echo_steps = self._send_echo_left(p)
        return echo_steps.join(echo_hash_steps)

    def _handle_echo(self, sender_id, p):
        """broadcast.rs:266-320."""
        old = self.echos.get(sender_id)
        if old is not None and _echo_proof(old) is not None:
            if old == p:
                return Step()
            return Step.from_fault(sender_id, FaultKind.MultipleEchos)
        if old is not None and old.digest != p.root_hash():
            return Step.from_fault(sender_id, FaultKind.MultipleEchos)
        if not self._validate_proof(p, sender_id):
            return Step.from_fault(sender_id, FaultKind.InvalidProof)
        h = p.root_hash()
        self.echos[sender_id] = p
        step = Step()
        if h not in self.can_decode_sent and self._count_echos_full(h) >= self._k:
            step.extend(self._send_can_decode(h))
        if not self.ready_sent and self._count_echos(h) >= self.val_set.num_correct():
            step.extend(self._send_ready(h))
        if self.ready_sent:
            step.extend(self._compute_output(h))
        return step

    def _handle_echo_hash(self, sender_id, h):
        """broadcast.rs:322-355."""
        old = self.echos.get(sender_id)
        if old is not None:
            if _echo_proof(old) is None:
                if old.digest == h:
                    return Step()
                return Step.from_fault(sender_id, FaultKind.MultipleEchoHashes)
            if old.root_hash() == h:
                return Step()
            return Step.from_fault(sender_id, FaultKind.MultipleEchoHashes)
        self.echos[sender_id] = _EchoHash(h)
        if self.ready_sent or self._count_echos(h) < self.val_set.num_correct():
            return self._compute_output(h)
        return self._send_ready(h)

    def _handle_can_decode(self, sender_id, h):
        """broadcast.rs:358-375."""
        self.can_decodes.setdefault(h, set()).add(sender_id)
        return Step()

    def _handle_ready(self, sender_id, h):
        """broadcast.rs:378-410."""
        old = self.readys.get(sender_id)
        if old is not None:
            if old == h:
                return Step()
            return Step.from_fault(sender_id, FaultKind.MultipleReadys)
        self.readys[sender_id] = h
        step = Step()
        f = self.val_set.num_faulty()
        if self._count_readys(h) == f + 1 and not self.ready_sent:
            step.extend(self._send_ready(h))
        if self._count_readys(h) == 2 * f + 1:
            step.extend(self._send_echo_remaining(h))
        return step.join(self._compute_output(h))

    # -- senders ------------------------------------------------------------------
    def _send_echo_left(self, p):
        """broadcast.rs:413-425."""
        if not self.val_set.contains(self.our_id):
            return Step()
        step = Step.from_message(Target.all_except_ids(self._right_nodes()).message(Message.echo(p)))
        return step.join(self._handle_echo(self.our_id, p))

    def _send_echo_remaining(self, h):
        """broadcast.rs:428-453."""
        self.echo_sent = True
        if not self.val_set.contains(self.our_id):
            return Step()
        p = self.echos.get(self.our_id)
        if p is None or _echo_proof(p) is None or p.root_hash() != h:
            return Step()
        senders = self.can_decodes.get(h)
        right = [i for i in self._right_nodes() if senders is None or i not in senders]
        return Step.from_message(Target.nodes(right).message(Message.echo(p)))

    def _send_echo_hash(self, h):
        """broadcast.rs:456-468."""
        self.echo_hash_sent = True
        if not self.val_set.contains(self.our_id):
            return Step()
        step = Step.from_message(Target.nodes(self._right_nodes()).message(Message.echo_hash(h)))
        return step.join(self._handle_echo_hash(self.our_id, h))

    def _right_nodes(self):
        """broadcast.rs:476-485: the ids after ours on the circle, skipping the
        first N-2f+fault_estimate (us included); f of them."""
        ids = self.val_set.all_ids()
        n = len(ids)
        start = ids.index(self.our_id)
        skip = self.val_set.num_correct() - self.val_set.num_faulty() + self.fault_estimate
        return [ids[(start + j) % n] for j in range(skip, n)]

    def _send_can_decode(self, h):
        """broadcast.rs:488-510."""
        self.can_decode_sent.add(h)
        if not self.val_set.contains(self.our_id):
            return Step()
        recipients = [i for i in self.val_set.all_ids()
                      if i != self.our_id and _echo_proof(self.echos.get(i, _EchoHash(b""))) is None]
        step = Step.from_message(Target.nodes(recipients).message(Message.can_decode(h)))
        return step.join(self._handle_can_decode(self.our_id, h))

    def _send_ready(self, h):
        """broadcast.rs:513-522."""
        self.ready_sent = True
        if not self.val_set.contains(self.our_id):
            return Step()
        step = Step.from_message(Target.all().message(Message.ready(h)))
        return step.join(self._handle_ready(self.our_id, h))

    # -- output -------------------------------------------------------------------
    def _compute_output(self, h):
        """broadcast.rs:526-558."""
        if (self.decided or self._count_readys(h) <= 2 * self.val_set.num_faulty()
                or self._count_echos_full(h) < self._k):
            return Step()
        if self._decode_pending is not None:
            # a second attempt within the same message: same inputs, same outcome
            # (nothing on success, another decoding fault on failure)
            if self._decode_pending["root"] != h:
                raise RuntimeError("%r: second decode for another root while one is pending"
                                   % (self,))
            self._decode_pending["repeat"] += 1
            return Step()
        leaf_values = []
        for i in self.val_set.all_ids():
            p = _echo_proof(self.echos[i]) if i in self.echos else None
            leaf_values.append(p.value() if p is not None and p.root_hash() == h else None)
        if self.decode_sink is not None:
            self._decode_pending = {"bc": self, "leaf_values": leaf_values, "root": h, "repeat": 0}
            self.decode_sink.append(self._decode_pending)
            return Step()
        value = self._decode_from_shards(leaf_values, h)
        if value is not None:
            self.decided = True
            s = Step()
            s.output.append(value)
            return s
        return Step.from_fault(self.proposer_id, FaultKind.BroadcastDecoding)

    def _decode_from_shards(self, leaf_values, root_hash):
        """broadcast.rs:563-601: reconstruct (rse errors -> None), re-tree
        over all shards, root compare, BE32 length, take(len)."""
        try:
            self.coding.reconstruct_shards(leaf_values)
        except self._be.RseError as e:
            if getattr(e, "code", 0) >= 100:   # device / library failure, not an rse outcome
                raise
            return None
        shards = [bytes(v) for v in leaf_values if v is not None]
        mtree = self._be.MerkleTree.from_vec(shards)
        if mtree.root_hash() != root_hash:
            return None
        data = b"".join(mtree.into_values()[:self._k])
        if len(data) < 4:
            return None
        (plen,) = struct.unpack(">I", data[:4])
        return data[4:4 + plen]

    def _validate_proof(self, p, node_id):
        """broadcast.rs:604-606."""
        return self.val_set.index(node_id) == p.index() and p.validate(self.val_set.num())

    def _count_echos_full(self, h):
        return sum(1 for c in self.echos.values() if _echo_proof(c) is not None and c.root_hash() == h)

    def _count_echos(self, h):
        return sum(1 for c in self.echos.values() if _echo_hash(c) == h)

    def _count_readys(self, h):
        return sum(1 for r in self.readys.values() if r == h)

    def __repr__(self):
        return "%r Broadcast(%r)" % (self.our_id, self.proposer_id)


def resolve_decodes(requests, backend=None):
    """Complete the decodes that Broadcast instances with a `decode_sink`
    deferred: every `decode_from_shards` (broadcast.rs:563-601)
    of the batch in one reconstruct + re-tree + root check + unframe launch per
    (validator count, shard length) through the backend's
    `decode_shards_batch`, or one call each without it.  Returns [(Broadcast,
    Step)]: the output (and `decided`) on success, the decoding fault(s) on
    failure -- what `compute_output` would have returned.  Exact as long as
    an instance handles no message between its request and this call (one
    crank per network per round)."""
    be = backend if backend is not None else _default_backend()
    if not requests:
        return []
    fn = getattr(be, "decode_shards_batch", None)
    if fn is not None:
        by_dev = {}
        for r in requests:
            by_dev.setdefault(r["bc"].device, []).append(r)
        values = {}
        for dev, rs in by_dev.items():
            out = fn([(r["bc"].val_set.num(), r["leaf_values"], r["root"]) for r in rs], device=dev)
            for r, v in zip(rs, out):
                values[id(r)] = v
    else:
        values = {id(r): r["bc"]._decode_from_shards(list(r["leaf_values"]), r["root"])
                  for r in requests}
    res = []
    for r in requests:
        bc, v = r["bc"], values[id(r)]
        bc._decode_pending = None
        if v is not None:
            bc.decided = True
            s = Step()
            s.output.append(v)
        else:
            s = Step()
            for _ in range(1 + r["repeat"]):
                s.fault_log.append(Fault(bc.proposer_id, FaultKind.BroadcastDecoding))
        res.append((bc, s))
    return res


def prevalidate(messages, n, backend=None, device=0):
    """Validate the proofs of many pending Value / Echo messages (of any number
    of Broadcast instances over n validators) in one batched launch on
    `device` before they are delivered.  `Proof::validate` is a pure function
    of the proof, so the results, memoised on each Proof, are exactly what
    every receiver's `validate_proof` (broadcast.rs:604-606) would compute; the
    receiver's index check stays in the state machine."""
    be = backend if backend is not None else _default_backend()
    fn = getattr(be, "validate_proofs", None)
    if fn is not None:
        fn([m.payload for m in messages if m.kind <= Message.ECHO], n, device=device)


def broadcast_many(inputs, backend=None):
    """`Broadcast::broadcast` (broadcast.rs:123-137) of many proposer instances
    at once -- the N contributions of a Subset / HoneyBadger epoch
    (subset/proposal_state.rs:69-113) or several epochs.
    inputs: [(Broadcast, value)] -> [Step], in order.  The proposers' framing,
    encode and tree go through the backend's `send_shards_batch` (one launch
    per validator count and payload length); each instance then sends its
    proofs exactly as `broadcast` does.  Error checks stay per instance and
    come first, as in `broadcast`."""
    be = backend if backend is not None else _default_backend()
    # all-or-nothing: every input is checked before any instance changes state,
    # so an error leaves every instance able to propose again
    seen = set()
    for bc, _ in inputs:
        if bc.our_id != bc.proposer_id:
            raise BroadcastError(ErrorKind.InstanceCannotPropose)
        if bc.value_sent or id(bc) in seen:
            raise BroadcastError(ErrorKind.MultipleInputs)
        seen.add(id(bc))
    fn = getattr(be, "send_shards_batch", None)
    todo = [(bc, bytes(v)) for bc, v in inputs]
    trees = {}
    if fn is not None and todo:
        by_dev = {}
        for bc, v in todo:   # each instance's trees are built on its own GPU
            by_dev.setdefault(bc.device, []).append((bc, v))
        for dev, group in by_dev.items():
            for (bc, v), t in zip(group, fn([(bc.val_set.num(), v) for bc, v in group],
                                            device=dev)):
                trees[id(bc)] = t
    return [bc.broadcast(v, trees.get(id(bc))) for bc, v in todo]
