"""In-process test network for hbbft_amd.broadcast.Broadcast.

TEST INFRASTRUCTURE: a restatement of hbbft_testing's `VirtualNet` crank loop
(/root/reference/hbbft_testing/src/lib.rs:223-283 process_step, 869-884
send_input, 908-996 crank; faulty nodes are the first f by index, 775-800)
and of the adversaries the reference's tests/broadcast.rs uses
(hbbft_testing/src/adversary.rs:372-450 sort_ascending / swap_random /
sort_by_random_node, 484-531 NodeOrder / Reordering, 540-607 Random;
tests/broadcast.rs:33-98 ProposeAdversary).  Python's `random.Random` stands
in for the reference's seeded XorShiftRng: the schedules differ, the
properties asserted are the reference's.
"""
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from hbbft_amd.broadcast import (Broadcast, Message, Step, Target, TargetedMessage,  # noqa: E402
                                 broadcast_many, prevalidate, resolve_decodes)


class CrankError(AssertionError):
    pass


class NetMessage:
    __slots__ = ("frm", "to", "payload")

    def __init__(self, frm, payload, to):
        self.frm, self.payload, self.to = frm, payload, to


class Node:
    def __init__(self, node_id, algo, faulty):
        self.id = node_id
        self.algo = algo
        self.faulty = faulty
        self.outputs = []
        self.faults = []


class VirtualNet:
    def __init__(self, ids, num_faulty, make_algo, adversary, rng, message_limit=None,
                 error_on_fault=True):
        ids = sorted(ids)
        assert 3 * num_faulty < len(ids)
        self.nodes = collections.OrderedDict(
            (i, Node(i, make_algo(i), idx < num_faulty)) for idx, i in enumerate(ids))
        self.adversary = adversary
        self.rng = rng
        self.messages = collections.deque()
        self.message_limit = message_limit
        self.message_count = 0
        self.crank_count = 0
        self.error_on_fault = error_on_fault
        self.pending = []   # Value / Echo messages queued since the last batched validation

    def correct_nodes(self):
        return [n for n in self.nodes.values() if not n.faulty]

    def faulty_nodes(self):
        return [n for n in self.nodes.values() if n.faulty]

    def send_input(self, node_id, value):
        step = self.nodes[node_id].algo.handle_input(value)
        self.process_step(node_id, step)
        return step

    def dispatch_message(self, msg):
        return self.nodes[msg.to].algo.handle_message(msg.frm, msg.payload)

    def process_step(self, stepped_id, step):
        """lib.rs:223-283: expand targets in node-id order, store outputs, fail
        when a correct node blames a correct node."""
        node = self.nodes[stepped_id]
        for tm in step.messages:
            if tm.message.kind <= Message.ECHO:
                self.pending.append(tm.message)
            if not node.faulty:
                assert stepped_id not in tm.target.ids   # targets never name the sender
            for to in self.nodes:
                if to != stepped_id and tm.target.contains(to):
                    if not node.faulty:
                        self.message_count += 1
                    self.messages.append(NetMessage(stepped_id, tm.message, to))
        node.outputs.extend(step.output)
        node.faults.extend(step.fault_log)
        if self.error_on_fault and not node.faulty:
            for fault in step.fault_log:
                other = self.nodes.get(fault.node_id)
                if other is not None and not other.faulty:
                    raise CrankError("%r blamed correct node %r: %s"
                                     % (stepped_id, fault.node_id, fault.kind.name))

    def crank(self):
        if self.message_limit is not None and self.message_count >= self.message_limit:
            raise CrankError("message limit %d exceeded" % self.message_limit)
        self.adversary.pre_crank(self)
        if not self.messages:
            return None
        msg = self.messages.popleft()
        if self.nodes[msg.to].faulty:
            step = self.adversary.tamper(self, msg)
        else:
            step = self.dispatch_message(msg)
        self.process_step(msg.to, step)
        self.crank_count += 1
        return msg.to, step

    def crank_expect(self):
        r = self.crank()
        if r is None:
            raise CrankError("queue empty before every node terminated")
        return r


# ---- adversaries (adversary.rs) ---------------------------------------------
def sort_ascending(net):
    net.messages = collections.deque(sorted(net.messages, key=lambda m: m.to))


def swap_random(net, rng):
    n = len(net.messages)
    if n:
        j = rng.randrange(n)
        net.messages[0], net.messages[j] = net.messages[j], net.messages[0]


def random_node(net, rng):
    ids = list(net.nodes)
    return ids[rng.randrange(len(ids))] if ids else None


def sort_by_random_node(net, rng):
    picked = random_node(net, rng)
    if picked is not None:
        net.messages = collections.deque(
            sorted(net.messages, key=lambda m: (m.to != picked, m.to)))


class NullAdversary:
    def pre_crank(self, net):
        pass

    def tamper(self, net, msg):
        return net.dispatch_message(msg)


class NodeOrderAdversary(NullAdversary):
    def pre_crank(self, net):
        sort_ascending(net)


class ReorderingAdversary(NullAdversary):
    def pre_crank(self, net):
        swap_random(net, net.rng)


class ProposeAdversary(NullAdversary):
    """tests/broadcast.rs:33-98: once, every faulty node proposes "Fake news"
    through a fresh Broadcast of its own; optionally drops every other message
    faulty nodes send."""

    RANDOM_PICK, SORT_ASCENDING = 0, 1

    def __init__(self, strategy, drop_messages, backend=None):
        self.strategy = strategy
        self.drop = drop_messages
        self.has_sent = False
        self.backend = backend

    def pre_crank(self, net):
        if self.strategy == self.RANDOM_PICK:
            swap_random(net, net.rng)
        else:
            sort_ascending(net)

    def tamper(self, net, msg):
        step = net.dispatch_message(msg)
        if self.drop:
            step.messages.clear()
        if not self.has_sent:
            self.has_sent = True
            for fnode in net.faulty_nodes():
                fake = Broadcast(fnode.id, fnode.algo.validator_set(), fnode.id,
                                 backend=self.backend).handle_input(b"Fake news")
                step.messages.extend(fake.messages)
        return step


class RandomAdversary(NullAdversary):
    """adversary.rs:540-607 (replay to a random node, inject random messages
    from message.rs:28-50 -- whose can_decode / echo_hash samples are Ready)."""

    def __init__(self, p_replay, p_inject, backend):
        self.p_replay = p_replay
        self.p_inject = p_inject
        self.backend = backend

    def pre_crank(self, net):
        sort_by_random_node(net, net.rng)

    def random_message(self, rng):
        kind = rng.choice(["value", "echo", "ready", "can_decode", "echo_hash"])
        buf = bytes(rng.randrange(256) for _ in range(32))
        proof = self.backend.MerkleTree.from_vec([buf]).proof(0)
        if kind == "value":
            return Message.value(proof)
        if kind == "echo":
            return Message.echo(proof)
        return Message.ready(b"r" * 32)

    def tamper(self, net, msg):
        rng = net.rng
        if rng.random() < self.p_replay:
            picked = random_node(net, rng)
            if picked is not None:
                net.messages.append(NetMessage(msg.to, msg.payload, picked))
        while rng.random() < self.p_inject:
            sender = msg.to
            m = self.random_message(rng)
            for nid in net.nodes:
                if nid != sender:
                    net.messages.append(NetMessage(sender, m, nid))
        return net.dispatch_message(msg)


def max_faulty(n):
    """util.rs:22-25."""
    return (n - 1) // 3


def run_broadcast(net, value, proposer_id):
    """tests/broadcast.rs:101-147 (test_broadcast)."""
    proposer_faulty = net.nodes[proposer_id].faulty
    net.send_input(proposer_id, value)
    while not all(n.algo.terminated() for n in net.nodes.values()):
        if proposer_faulty and not net.messages:
            break
        net.crank_expect()
    return check_outcome(net, value, proposer_id)


def check_outcome(net, value, proposer_id):
    """The assertions of tests/broadcast.rs:127-146."""
    if net.nodes[proposer_id].faulty:
        first = net.correct_nodes()[0].outputs
        assert all(n.outputs == first for n in net.nodes.values())
    else:
        assert all(n.outputs == [bytes(value)] for n in net.nodes.values()), \
            [(n.id, n.outputs) for n in net.nodes.values()]
    return net


def run_lockstep(items, backend, batched_input=False, batched_decode=False):
    """Many broadcast networks cranked in lockstep, one crank per network per
    round.  Before every round the Value / Echo proofs all networks queued
    since the previous round are validated together, one batched launch per
    tree size (hbbft_amd.broadcast.prevalidate); the state machines then find
    every result memoised.  Each network's schedule depends only on its own
    RNG and state, so outcomes equal those of `run_broadcast`.
    batched_input: the proposers' inputs go through `broadcast_many` (one
    frame+encode+tree launch per size) instead of one
    `send_input` each.
    batched_decode: every node defers `decode_from_shards` to a shared sink
    and the decodes of all networks are completed together after each round
    (hbbft_amd.broadcast.resolve_decodes: one launch per validator count and
    shard length); a node handles one message per round, so
    its decode completes before its next message.  items: [(net, value,
    proposer)]."""
    sink, owner = [], {}
    if batched_decode:
        for net, _, _ in items:
            for nid, nd in net.nodes.items():
                nd.algo.decode_sink = sink
                owner[id(nd.algo)] = (net, nid)
    if batched_input:
        steps = broadcast_many([(net.nodes[p].algo, v) for net, v, p in items], backend)
        for (net, _, proposer), step in zip(items, steps):
            net.process_step(proposer, step)
    else:
        for net, value, proposer in items:
            net.send_input(proposer, value)
    live = list(items)
    while live:
        by_n = {}
        for net, _, _ in live:
            by_n.setdefault(len(net.nodes), []).extend(net.pending)
            net.pending.clear()
        for n, msgs in by_n.items():
            prevalidate(msgs, n, backend)
        nxt = []
        for it in live:
            net, _, proposer = it
            if all(nd.algo.terminated() for nd in net.nodes.values()):
                continue
            if net.nodes[proposer].faulty and not net.messages:
                continue
            net.crank_expect()
            nxt.append(it)
        for bc, step in resolve_decodes(sink, backend):
            net, nid = owner[id(bc)]
            net.process_step(nid, step)
        sink.clear()
        live = nxt
    for net, value, proposer in items:
        check_outcome(net, value, proposer)
    return [it[0] for it in items]


def broadcast_different_sizes(new_adversary, value, rng, backend, sizes=None):
    """tests/broadcast.rs:149-185: N in 1..5, rand[6,20), rand[30,50); f =
    max_faulty(N) faulty nodes (the first f), random proposer."""
    if sizes is None:
        sizes = list(range(1, 6)) + [rng.randrange(6, 20), rng.randrange(30, 50)]
    nets = []
    for size in sizes:
        nf = max_faulty(size)
        proposer = rng.randrange(size)
        ids = list(range(size))
        net = VirtualNet(ids, nf, lambda i: Broadcast(i, ids, proposer, backend=backend),
                         new_adversary(), rng, message_limit=10_000 * size)
        nets.append(run_broadcast(net, value, proposer))
    return nets


# ---- synchronous rounds (the schedule of the GPU state machine) -------------
def codeword_tree(backend, n, value):
    """send_shards (broadcast.rs:170-204) of `value` over n validators."""
    f = max_faulty(n)
    k, m = n - 2 * f, 2 * f
    framed = len(value).to_bytes(4, "big") + bytes(value)
    S = max(1, (len(framed) + k - 1) // k)
    buf = framed.ljust(S * n, b"\0")
    shards = [bytearray(buf[i * S:(i + 1) * S]) for i in range(n)]
    backend.Coding(k, m).encode(shards)
    return backend.MerkleTree.from_vec([bytes(s) for s in shards])


def run_rounds(inst, backend, max_rounds=64):
    """The host restatement of hbbft_amd/rbc_sim.py's schedule for one
    scenario instance (hbbft_amd.rbc_sim.Instance): hbbft_amd/broadcast.py
    nodes exchange messages in synchronous rounds -- what a node emits in
    round t is delivered in round t + 1, each node handling its inbox in
    (sender index, emission order).  Round 0 is the proposer's broadcast()
    with its per-recipient Values (value_root / value_tamper).  Roles filter
    what a node sends after handling a message: SILENT drops everything (the
    ProposeAdversary with drop, tests/broadcast.rs:66-71), CORRUPT_ECHO
    sends the tampered copy of every Echo proof, WITHHOLD_ECHO no Echo.  After
    its first handled message, inst.fake_from sends the broadcasts of every
    node in inst.fake_list (tests/broadcast.rs:73-97), unfiltered.
    Returns ({node: [outputs]}, {node: [(blamed, FaultKind name)]}, rounds)."""
    from hbbft_amd.rbc_sim import CORRUPT_ECHO, NONE, SILENT, WITHHOLD_ECHO, tampered
    n, p = inst.n, inst.proposer
    ids = list(range(n))
    nodes = {i: Broadcast(i, ids, p, backend=backend) for i in ids}
    outputs = {i: [] for i in ids}
    faults = {i: [] for i in ids}
    trees = [codeword_tree(backend, n, v) for v in inst.values]

    def record(i, st):
        outputs[i].extend(st.output)
        faults[i].extend((fl.node_id, fl.kind.name) for fl in st.fault_log)

    def sent(i, msgs, first_round=False):
        role = inst.role[i]
        if role == SILENT and not first_round:
            return []
        out = []
        for tm in msgs:
            if tm.message.kind == Message.ECHO:
                if role == WITHHOLD_ECHO:
                    continue
                if role == CORRUPT_ECHO:
                    tm = TargetedMessage(tm.target, Message.echo(tampered(tm.message.payload)))
            out.append(tm)
        return out

    def proof(c, j, t):
        pr = trees[c].proof(j)
        return tampered(pr) if t else pr

    # round 0: broadcast() with the scenario's Values (broadcast.rs:123-137, 212-222)
    bc = nodes[p]
    bc.value_sent = True
    step = Step()
    for j in ids:
        if j != p and inst.value_root[j] != NONE:
            step.messages.append(Target.node(j).message(
                Message.value(proof(inst.value_root[j], j, inst.value_tamper[j]))))
    step = step.join(bc._handle_value(p, proof(inst.value_root[p], p, inst.value_tamper[p])))
    record(p, step)
    outbox = {i: [] for i in ids}
    outbox[p] = sent(p, step.messages, first_round=True)
    fake_done = False
    rounds = 1
    while any(outbox.values()):
        if rounds >= max_rounds:
            raise CrankError("no quiescence in %d rounds" % max_rounds)
        inbox = {r: [] for r in ids}
        for s in ids:
            for tm in outbox[s]:
                for r in ids:
                    if r != s and tm.target.contains(r):
                        inbox[r].append((s, tm.message))
        nxt = {i: [] for i in ids}
        for r in ids:
            for s, msg in inbox[r]:
                st = nodes[r].handle_message(s, msg)
                record(r, st)
                nxt[r].extend(sent(r, st.messages))
                if inst.fake_from == r and not fake_done:
                    fake_done = True
                    for F in inst.fake_list:
                        fake = Broadcast(F, ids, F, backend=backend).handle_input(
                            inst.values[inst.fake_root])
                        nxt[r].extend(fake.messages)
        outbox = nxt
        rounds += 1
    return outputs, faults, rounds
