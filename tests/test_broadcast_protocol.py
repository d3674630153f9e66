"""The Reliable Broadcast state machine (hbbft_amd/broadcast.py) run the way
the reference's own tests run it:

* the doc-test of src/broadcast/mod.rs:140-220 (7 nodes, proposer 3, 128 random
  bytes, every node outputs the payload exactly once);
* the seven proptests of tests/broadcast.rs:187-286 (sizes 1..5, rand[6,20),
  rand[30,50); Reordering / NodeOrder / Propose(+drop) / Random adversaries;
  the N=8 equal-leaves case), through tests/virtual_net.py;
* unit checks of every fault and error the state machine reports
  (broadcast.rs:123-153, 228-410, 526-558; error.rs).

Each scenario runs twice: on the CPU against the oracle backend
(tests/oracle_backend.py, the checker) and, marked `gpu`, with the product
backend -- every encode / tree / proof / validate / reconstruct through
libhbrbc.so on the MI355X.
"""
import random
import struct

import pytest

import virtual_net as vn
from hbbft_amd.broadcast import (Broadcast, BroadcastError, ErrorKind, FaultKind, Message,
                                 Target, ValidatorSet, broadcast_many)


def _oracle_backend():
    import oracle_backend
    return oracle_backend


def _hip_backend():
    import torch

    import hbbft_amd
    if not torch.cuda.is_available():
        pytest.fail("GPU test without a visible GPU")
    return hbbft_amd


BACKENDS = [pytest.param("oracle", id="oracle"),
            pytest.param("hip", id="hip", marks=pytest.mark.gpu)]


@pytest.fixture(params=BACKENDS)
def backend(request):
    return _oracle_backend() if request.param == "oracle" else _hip_backend()


# ---- src/broadcast/mod.rs:140-220 --------------------------------------------
def test_doc_example_seven_nodes(backend):
    rng = random.Random(140)
    n, proposer = 7, 3
    vals = ValidatorSet(range(n))
    nodes = {i: Broadcast(i, vals, proposer, backend=backend) for i in range(n)}
    payload = bytes(rng.randrange(256) for _ in range(128))
    queue, finished = [], set()

    def on_step(node_id, step):
        queue.extend((node_id, tm) for tm in step.messages)
        if step.output:
            assert step.output == [payload]
            assert node_id not in finished     # at most once
            finished.add(node_id)

    on_step(proposer, nodes[proposer].broadcast(payload))
    while queue:
        src, tm = queue.pop(0)
        for i, node in nodes.items():
            if tm.target.contains(i):
                on_step(i, node.handle_message(src, tm.message))
    assert finished == set(nodes)             # ... and at least once


# ---- tests/broadcast.rs ---------------------------------------------------------
def test_8_broadcast_equal_leaves_silent(backend):
    """tests/broadcast.rs:235-258: 32 spaces, so every data shard is equal."""
    rng = random.Random(235)
    size, proposer = 8, rng.randrange(8)
    ids = list(range(size))
    net = vn.VirtualNet(ids, 0, lambda i: Broadcast(i, ids, proposer, backend=backend),
                        vn.ReorderingAdversary(), rng, message_limit=10_000 * size)
    vn.run_broadcast(net, b" " * 32, proposer)


def test_broadcast_random_delivery_silent(backend):
    rng = random.Random(260)
    vn.broadcast_different_sizes(vn.ReorderingAdversary, b"Foo", rng, backend)


def test_broadcast_first_delivery_silent(backend):
    rng = random.Random(264)
    vn.broadcast_different_sizes(vn.NodeOrderAdversary, b"Foo", rng, backend)


def test_broadcast_first_delivery_adv_propose(backend):
    rng = random.Random(268)
    vn.broadcast_different_sizes(
        lambda: vn.ProposeAdversary(vn.ProposeAdversary.SORT_ASCENDING, False, backend),
        b"Foo", rng, backend)


def test_broadcast_random_delivery_adv_propose(backend):
    rng = random.Random(273)
    vn.broadcast_different_sizes(
        lambda: vn.ProposeAdversary(vn.ProposeAdversary.RANDOM_PICK, False, backend),
        b"Foo", rng, backend)


def test_broadcast_random_delivery_adv_propose_and_drop(backend):
    rng = random.Random(278)
    vn.broadcast_different_sizes(
        lambda: vn.ProposeAdversary(vn.ProposeAdversary.RANDOM_PICK, True, backend),
        b"Foo", rng, backend)


def test_broadcast_random_adversary(backend):
    rng = random.Random(283)
    vn.broadcast_different_sizes(lambda: vn.RandomAdversary(0.2, 0.2, backend), b"RandomFoo",
                                 rng, backend)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_broadcast_payload_sizes(backend, seed):
    """Ragged payloads across the shard-length rounding (broadcast.rs:182), an
    empty payload, and a faulty proposer under the reordering adversary."""
    rng = random.Random(seed)
    for size in (4, 7, 10):
        for plen in (0, 1, 5, rng.randrange(6, 300)):
            proposer = rng.randrange(size)
            ids = list(range(size))
            net = vn.VirtualNet(ids, vn.max_faulty(size),
                                lambda i: Broadcast(i, ids, proposer, backend=backend),
                                vn.ReorderingAdversary(), rng, message_limit=10_000 * size)
            vn.run_broadcast(net, bytes(rng.randrange(256) for _ in range(plen)), proposer)


# ---- faults and errors -------------------------------------------------------------
def _proposal(backend, n, proposer, payload):
    """The proposer's step: Value proofs keyed by recipient, plus its own."""
    bc = Broadcast(proposer, range(n), proposer, backend=backend)
    step = bc.broadcast(payload)
    values = {}
    for tm in step.messages:
        if tm.message.kind == Message.VALUE:
            (to,) = tm.target.ids
            values[to] = tm.message.payload
    return bc, step, values


def test_errors(backend):
    with pytest.raises(BroadcastError) as e:
        Broadcast(0, range(4), 1, backend=backend).broadcast(b"x")
    assert e.value.kind == ErrorKind.InstanceCannotPropose
    bc = Broadcast(1, range(4), 1, backend=backend)
    bc.broadcast(b"x")
    with pytest.raises(BroadcastError) as e:
        bc.broadcast(b"y")
    assert e.value.kind == ErrorKind.MultipleInputs
    with pytest.raises(BroadcastError) as e:
        bc.handle_message(9, Message.ready(b"\0" * 32))
    assert e.value.kind == ErrorKind.UnknownSender
    with pytest.raises(BroadcastError) as e:     # rse: more than 256 shards
        Broadcast(0, range(257), 0, backend=backend)
    assert e.value.kind == ErrorKind.InvalidNodeCount


def test_value_faults(backend):
    n, proposer = 4, 2
    _, _, values = _proposal(backend, n, proposer, b"payload")
    p0 = values[0]
    node = Broadcast(0, range(n), proposer, backend=backend)
    # Value from someone other than the proposer
    st = node.handle_message(1, Message.value(p0))
    assert [f.kind for f in st.fault_log] == [FaultKind.ReceivedValueFromNonProposer]
    # a proof for another index (validate_proof: index must be ours)
    st = node.handle_message(proposer, Message.value(values[1]))
    assert [f.kind for f in st.fault_log] == [FaultKind.InvalidProof]
    # a tampered value byte
    bad = backend.Proof(bytes([p0.value()[0] ^ 1]) + p0.value()[1:], p0.index(), p0.digests(),
                        p0.root_hash())
    st = node.handle_message(proposer, Message.value(bad))
    assert [f.kind for f in st.fault_log] == [FaultKind.InvalidProof]
    # the genuine one: Echo to the left nodes, EchoHash to the f right nodes
    st = node.handle_message(proposer, Message.value(p0))
    assert not st.fault_log
    kinds = [tm.message.kind for tm in st.messages]
    assert kinds == [Message.ECHO, Message.ECHO_HASH]
    assert st.messages[0].target.all_except and st.messages[0].target.ids == {3}
    assert not st.messages[1].target.all_except and st.messages[1].target.ids == {3}
    # the same Value again: ignored; a Value of a different tree: MultipleValues
    assert not node.handle_message(proposer, Message.value(p0)).fault_log
    _, _, other = _proposal(backend, n, proposer, b"another payload")
    st = node.handle_message(proposer, Message.value(other[0]))
    assert [f.kind for f in st.fault_log] == [FaultKind.MultipleValues]


def test_echo_ready_faults(backend):
    n, proposer = 4, 0
    _, _, values = _proposal(backend, n, proposer, b"echoes")
    _, _, other = _proposal(backend, n, proposer, b"other tree")
    node = Broadcast(3, range(n), proposer, backend=backend)
    assert not node.handle_message(1, Message.echo(values[1])).fault_log
    assert not node.handle_message(1, Message.echo(values[1])).fault_log   # duplicate: ignored
    st = node.handle_message(1, Message.echo(other[1]))
    assert [f.kind for f in st.fault_log] == [FaultKind.MultipleEchos]
    st = node.handle_message(2, Message.echo(values[1]))                   # wrong index
    assert [f.kind for f in st.fault_log] == [FaultKind.InvalidProof]
    # EchoHash then a conflicting EchoHash / Echo
    h = values[2].root_hash()
    assert not node.handle_message(2, Message.echo_hash(h)).fault_log
    st = node.handle_message(2, Message.echo_hash(other[2].root_hash()))
    assert [f.kind for f in st.fault_log] == [FaultKind.MultipleEchoHashes]
    st = node.handle_message(2, Message.echo(other[2]))
    assert [f.kind for f in st.fault_log] == [FaultKind.MultipleEchos]
    st = node.handle_message(1, Message.echo_hash(other[1].root_hash()))
    assert [f.kind for f in st.fault_log] == [FaultKind.MultipleEchoHashes]
    # Ready twice (ignored), then a different Ready (MultipleReadys)
    assert not node.handle_message(0, Message.ready(h)).fault_log
    assert not node.handle_message(0, Message.ready(h)).fault_log
    st = node.handle_message(0, Message.ready(other[1].root_hash()))
    assert [f.kind for f in st.fault_log] == [FaultKind.MultipleReadys]


def test_decode_fault_on_inconsistent_shards(backend):
    """A proposer whose parity shards are not a codeword of its data: proofs
    validate, but the rebuilt shard changes the root (broadcast.rs:551-557,
    583-585) -> BroadcastDecoding blamed on the proposer, no output."""
    n, proposer = 7, 0                      # f = 2, k = 3, m = 4
    k, S = 3, 6
    framed = struct.pack(">I", 10) + bytes(range(10))
    shards = [bytearray(framed[i * S:(i + 1) * S].ljust(S, b"\0")) for i in range(k)]
    shards += [bytearray(bytes([0x5A + i]) * S) for i in range(n - k)]   # not parity
    tree = backend.MerkleTree.from_vec([bytes(s) for s in shards])
    proofs = [tree.proof(i) for i in range(n)]
    node = Broadcast(6, range(n), proposer, backend=backend)
    # Echoes from 1..5 (shard 0 missing -> it is rebuilt from garbage), Readys from 2f+1
    for i in range(1, 6):
        assert not node.handle_message(i, Message.echo(proofs[i])).fault_log
    faults = []
    for i in range(1, 6):
        st = node.handle_message(i, Message.ready(tree.root_hash()))
        faults += st.fault_log
        assert not st.output
    assert FaultKind.BroadcastDecoding in [f.kind for f in faults]
    assert all(f.node_id == proposer for f in faults if f.kind == FaultKind.BroadcastDecoding)
    assert not node.terminated()


def test_decode_all_shards_present_outputs_data(backend):
    """All N leaves present: rse reconstruct is a no-op, so the re-tree matches
    and the data shards are output even though the parity is not a codeword
    (the reference's behaviour, broadcast.rs:569-600)."""
    n, proposer = 4, 0
    k, S = 2, 5
    framed = struct.pack(">I", 3) + b"abc"
    shards = [bytearray(framed[i * S:(i + 1) * S].ljust(S, b"\0")) for i in range(k)]
    shards += [bytearray(b"\x11" * S), bytearray(b"\x22" * S)]
    tree = backend.MerkleTree.from_vec([bytes(s) for s in shards])
    node = Broadcast(3, range(n), proposer, backend=backend)
    for i in range(n):
        node.handle_message(i, Message.echo(tree.proof(i)))
    out = []
    for i in range(n):
        out += node.handle_message(i, Message.ready(tree.root_hash())).output
    assert out == [b"abc"]


def test_right_nodes_and_targets():
    """broadcast.rs:476-485 on the circle of sorted ids (no backend needed)."""

    class _Stub:
        class RseError(Exception):
            pass

        class Coding:
            def __init__(self, k, m):
                pass

    for n in (1, 4, 7, 10):
        for me in range(n):
            bc = Broadcast(me, range(n), 0, backend=_Stub)
            f = (n - 1) // 3
            assert bc._right_nodes() == [(me + j) % n for j in range(n - f, n)]
    t = Target.all_except_ids([2])
    assert t.contains(1) and not t.contains(2)
    assert Target.nodes([]).contains(1) is False


def test_trivial_coding_single_node(backend):
    """N=1..3: f=0, Coding::Trivial (broadcast.rs:639-693)."""
    for n in (1, 2, 3):
        ids = list(range(n))
        net = vn.VirtualNet(ids, 0, lambda i: Broadcast(i, ids, n - 1, backend=backend),
                            vn.NullAdversary(), random.Random(n))
        vn.run_broadcast(net, b"trivial", n - 1)


def test_default_backend_has_no_cpu_fallback():
    """The product backend is libhbrbc.so: without a GPU, Broadcast::new fails loudly."""
    import torch

    import hbbft_amd
    if torch.cuda.is_available():
        assert Broadcast(0, range(4), 0).coding.encode_kernel()   # HIP context
        return
    with pytest.raises(hbbft_amd.HbrbcUnavailable):
        Broadcast(0, range(4), 0)


def _validate_stats(backend):
    return getattr(backend, "VALIDATE_STATS", None) or backend.STATS


def test_lockstep_batched_validation(backend):
    """Several networks cranked in lockstep with their pending proofs validated
    in batched launches (f2): every node's outputs and fault log equal the
    one-network-at-a-time run of the same seeds, under the random adversary."""
    sizes = [4, 7, 10, 16, 16, 31]

    def make(i, size):
        rng = random.Random(1000 + i)
        proposer = rng.randrange(size)
        ids = list(range(size))
        net = vn.VirtualNet(ids, vn.max_faulty(size),
                            lambda j: Broadcast(j, ids, proposer, backend=backend),
                            vn.RandomAdversary(0.2, 0.2, backend), rng, message_limit=10_000 * size)
        return net, b"lockstep %d" % i, proposer

    seq = [make(i, s) for i, s in enumerate(sizes)]
    for net, value, proposer in seq:
        vn.run_broadcast(net, value, proposer)
    st = _validate_stats(backend)
    before = dict(st)
    lock = [make(i, s) for i, s in enumerate(sizes)]
    vn.run_lockstep(lock, backend)
    for (a, _, _), (b, _, _) in zip(seq, lock):
        for na, nb in zip(a.nodes.values(), b.nodes.values()):
            assert na.outputs == nb.outputs
            assert [(f.node_id, f.kind) for f in na.faults] == [(f.node_id, f.kind) for f in nb.faults]
        assert a.crank_count == b.crank_count
    launches = st["launches"] - before["launches"]
    batched = st["batched"] - before["batched"]
    assert launches > 0 and batched > launches      # several proofs per launch
    assert st["single"] - before["single"] < batched  # only adversary-injected proofs go alone



def test_lockstep_batched_decodes(backend):
    """f2: networks cranked in lockstep with every node's `decode_from_shards`
    deferred and completed for all networks together after each round
    (resolve_decodes; on the HIP backend one hbrbc_decode_batch launch per
    validator count and shard length).  Outputs, fault logs and crank counts
    equal the one-network-at-a-time run of the same seeds."""
    # networks of one validator count and value length decode together
    sizes = [7] * 6 + [16] * 6 + [4, 31]

    def make(i, size):
        rng = random.Random(2000 + i)
        proposer = rng.randrange(size)
        ids = list(range(size))
        net = vn.VirtualNet(ids, vn.max_faulty(size),
                            lambda j: Broadcast(j, ids, proposer, backend=backend),
                            vn.RandomAdversary(0.2, 0.2, backend), rng, message_limit=10_000 * size)
        return net, b"decode lockstep %03d" % i * size, proposer

    seq = [make(i, s) for i, s in enumerate(sizes)]
    for net, value, proposer in seq:
        vn.run_broadcast(net, value, proposer)
    st = getattr(backend, "DECODE_STATS", None)
    before = dict(st) if st is not None else None
    lock = [make(i, s) for i, s in enumerate(sizes)]
    vn.run_lockstep(lock, backend, batched_decode=True)
    outputs = 0
    for (a, _, _), (b, _, _) in zip(seq, lock):
        for na, nb in zip(a.nodes.values(), b.nodes.values()):
            assert na.outputs == nb.outputs
            assert [(f.node_id, f.kind) for f in na.faults] == [(f.node_id, f.kind) for f in nb.faults]
            outputs += len(nb.outputs)
        assert a.crank_count == b.crank_count
    if st is not None:   # HIP backend: decodes went through the batched launches
        decodes = st["decodes"] - before["decodes"]
        launches = st["launches"] - before["launches"]
        assert decodes >= outputs > 0 and decodes > launches > 0


def test_deferred_decode_refuses_interleaved_messages():
    """decode_sink is run_lockstep's contract: once compute_output
    has filed a decode, another message before resolve_decodes is an error,
    not a silent extra BroadcastDecoding fault; after the resolution the
    instance proceeds as the reference's does."""
    from hbbft_amd.broadcast import resolve_decodes
    backend = _oracle_backend()
    n, proposer = 4, 0
    k, S = 2, 4
    framed = (struct.pack(">I", 3) + b"Foo").ljust(k * S, b"\0")
    shards = [bytearray(framed[i * S:(i + 1) * S]) for i in range(k)] + [bytearray(S) for _ in range(2)]
    backend.Coding(k, 2).encode(shards)
    tree = backend.MerkleTree.from_vec([bytes(s) for s in shards])
    node = Broadcast(3, range(n), proposer, backend=backend)
    node.decode_sink = sink = []
    for i in range(3):
        node.handle_message(i, Message.echo(tree.proof(i)))
    i = 0
    while not sink:   # N - f Echoes sent our Ready; > 2f Readys file the decode
        node.handle_message(i, Message.ready(tree.root_hash()))
        i += 1
    assert len(sink) == 1 and not node.terminated()
    with pytest.raises(RuntimeError):
        node.handle_message(i, Message.ready(tree.root_hash()))
    ((bc, step),) = resolve_decodes(sink, backend)
    assert bc is node and step.output == [b"Foo"] and node.terminated()


def _epoch_value(n, p):
    # ragged contributions: several proposers share a length (one batch), one
    # is empty, the rest differ
    return bytes((7 * p + i) & 0xFF for i in range(0 if p == 1 else 40 * (p % 3) + 3 * (p // 3 % 2)))


def test_epoch_batched_inputs(backend):
    """one epoch in which every validator proposes (Subset runs
    N broadcasts, subset/proposal_state.rs:69-113), all proposers' framing,
    encode and trees built by `broadcast_many` in a few batched launches;
    every node's outputs, faults and crank counts equal the one-input-at-a-time
    run of the same seeds."""
    def make(n, p, seed):
        rng = random.Random(seed)
        ids = list(range(n))
        net = vn.VirtualNet(ids, vn.max_faulty(n), lambda j: Broadcast(j, ids, p, backend=backend),
                            vn.RandomAdversary(0.2, 0.2, backend), rng, message_limit=10_000 * n)
        return net, _epoch_value(n, p), p

    plan = [(n, p, 7000 + 100 * n + p) for n in (3, 4, 7) for p in range(n)]
    seq = [make(*x) for x in plan]
    for net, value, p in seq:
        vn.run_broadcast(net, value, p)
    st = backend.SEND_STATS
    before = dict(st)
    lock = [make(*x) for x in plan]
    vn.run_lockstep(lock, backend, batched_input=True)
    for (a, _, _), (b, _, _) in zip(seq, lock):
        for na, nb in zip(a.nodes.values(), b.nodes.values()):
            assert na.outputs == nb.outputs
            assert [(f.node_id, f.kind) for f in na.faults] == [(f.node_id, f.kind) for f in nb.faults]
        assert a.crank_count == b.crank_count
    assert st["trees"] - before["trees"] == len(plan)
    assert st["launches"] - before["launches"] < len(plan)


def test_broadcast_many_errors(backend):
    """`broadcast_many` keeps `broadcast`'s per-instance errors
    (broadcast.rs:123-137): a non-proposer raises InstanceCannotPropose, a
    second input MultipleInputs."""
    ids = list(range(4))
    prop = Broadcast(0, ids, 0, backend=backend)
    other = Broadcast(1, ids, 0, backend=backend)
    with pytest.raises(BroadcastError) as e:
        broadcast_many([(other, b"x")], backend)
    assert e.value.kind == ErrorKind.InstanceCannotPropose
    steps = broadcast_many([(prop, b"abc")], backend)
    fresh = Broadcast(0, ids, 0, backend=backend).broadcast(b"abc")
    assert [(repr(t.target), t.message) for t in steps[0].messages] == \
        [(repr(t.target), t.message) for t in fresh.messages]   # 3 Values, Echo, EchoHash
    with pytest.raises(BroadcastError) as e:
        broadcast_many([(prop, b"abc")], backend)
    assert e.value.kind == ErrorKind.MultipleInputs


def test_broadcast_many_is_all_or_nothing(backend):
    """A failing input anywhere in the list (a non-proposer, the same instance
    twice) raises before any instance changes state, so the valid proposers
    can still broadcast afterwards (no stalled instances)."""
    ids = list(range(4))
    a = Broadcast(0, ids, 0, backend=backend)
    b = Broadcast(2, ids, 2, backend=backend)
    other = Broadcast(1, ids, 0, backend=backend)
    with pytest.raises(BroadcastError) as e:
        broadcast_many([(a, b"one"), (b, b"two"), (other, b"x")], backend)
    assert e.value.kind == ErrorKind.InstanceCannotPropose
    assert not a.value_sent and not b.value_sent
    with pytest.raises(BroadcastError) as e:
        broadcast_many([(a, b"one"), (a, b"again")], backend)
    assert e.value.kind == ErrorKind.MultipleInputs
    assert not a.value_sent
    steps = broadcast_many([(a, b"one"), (b, b"two")], backend)
    assert a.value_sent and b.value_sent and len(steps) == 2
    fresh = Broadcast(2, ids, 2, backend=backend).broadcast(b"two")
    assert [(repr(t.target), t.message) for t in steps[1].messages] == \
        [(repr(t.target), t.message) for t in fresh.messages]


@pytest.mark.gpu
def test_send_shards_batch_matches_oracle():
    """hbbft_amd.send_shards_batch (batched frame+encode+tree on the MI355X)
    against the oracle's send_shards for ragged payloads at N = 1..64 -- each
    N one ragged launch per stage: every shard, every tree node and every
    proof bit-exact."""
    hb = _hip_backend()
    orb = _oracle_backend()
    items = [(n, bytes((13 * n + 5 * i + j) & 0xFF for j in range(L)))
             for n in (1, 2, 3, 4, 7, 16, 64) for i, L in enumerate((0, 1, 5, 5, 100, 1000, 4099, 1000))]
    before = dict(hb.SEND_STATS)
    got = hb.send_shards_batch(items)
    # one frame+encode and one tree launch per validator count, whatever the lengths (f3)
    assert hb.SEND_STATS["launches"] - before["launches"] == 7
    want = orb.send_shards_batch(items)
    for (n, _), g, w in zip(items, got, want):
        assert g.values() == w.values()
        assert g.root_hash() == w.root_hash()
        for i in range(n):
            pg, pw = g.proof(i), w.proof(i)
            assert (pg.value(), pg.index(), pg.digests(), pg.root_hash()) == \
                (pw.value(), pw.index(), pw.digests(), pw.root_hash())
        assert g.proof(n) is None
