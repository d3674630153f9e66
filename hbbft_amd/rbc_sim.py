"""The Reliable-Broadcast state machine of many instances and nodes on the GPU
(SURVEY.md §8 row f2), sharded over ranks like the validator-sharded
simulation (hbbft_amd/sharded.py).

Control plane.  `hbrbc_sm_round` (hbbft_amd/csrc/sim.hip) runs
/root/reference/src/broadcast/broadcast.rs:228-558 -- handle_value,
handle_echo, handle_echo_hash, handle_can_decode, handle_ready, the senders
and compute_output -- for every hosted (instance, node) in synchronous rounds:
what a node emits in round t is delivered in round t + 1, handled in (sender,
emission) order.  Every node's Echo / EchoHash / Ready / CanDecode state and
counters live on the GPU; each round's messages (records of kind, root, proof
index, tamper flag and an N-bit recipient mask) are all-gathered between the
ranks -- one all-gather per round for all of a rank's sub-batches, with their
emitted counts and overflow flags (`_run_rounds_dist`) -- the
Ready/EchoHash/CanDecode fan-out of SURVEY §5.

Data plane.  Messages carry proofs by reference (root slot c, index j,
tampered copy or not).  `data_plane` encodes each instance's codewords
(send_shards_batch), validates every proof and its tampered copy
(validate_proofs) and decodes each root once (decode_shards_batch): Proof::
validate is a pure function of the proof, and a codeword decodes from any k
of its rows, so the state machine looks the outcomes up (broadcast.rs:254,
291, 551-557).

Scenarios (`Scenario`): a proposer that sends different codewords, tampered
proofs or nothing to some validators; faulty nodes that drop what they would
send (tests/broadcast.rs:33-98 ProposeAdversary with drop), corrupt or
withhold their Echoes; and the ProposeAdversary's injected broadcasts of the
faulty nodes' own value.  tests/test_rbc_sim.py checks every node's output and
fault log against the host restatement (hbbft_amd/broadcast.py driven by
tests/virtual_net.py RoundNet) on the same scenarios.
"""
import ctypes

import torch

from . import _check, decode_shards_batch, lib, send_shards_batch, validate_proofs
from . import RbcBatch

NONE = 0xFF
HONEST, SILENT, CORRUPT_ECHO, WITHHOLD_ECHO = 0, 1, 2, 3
# FaultKind (broadcast/error.rs:28-50), in declaration order
FAULT_KINDS = ["ReceivedValueFromNonProposer", "MultipleValues", "MultipleEchos",
               "MultipleEchoHashes", "MultipleReadys", "InvalidProof", "BroadcastDecoding"]
MSG_KINDS = ["Value", "Echo", "Ready", "CanDecode", "EchoHash", "Fake"]

_P = ctypes.c_void_p


class SmArgs(ctypes.Structure):
    """struct hbrbc_sm_args (include/hbrbc.h)."""
    _fields_ = [("count", ctypes.c_size_t), ("node_lo", ctypes.c_uint32),
                ("nodes", ctypes.c_uint32), ("rows_per_rank", ctypes.c_uint32),
                ("roots", ctypes.c_uint32), ("max_out", ctypes.c_uint32),
                ("max_faults", ctypes.c_uint32), ("round", ctypes.c_int32)] + [
        (name, _P) for name in (
            "proposer", "role", "value_root", "value_tamper", "proof_ok", "decode_ok",
            "fake_from", "fake_root", "fake_list", "in_", "in_count", "out", "out_count",
            "state", "output_root", "faults", "fault_count", "emitted", "active")] + [
        ("flags", ctypes.c_uint32)]


SM_NO_FAKE = 1   # hbrbc_sm_args.flags: no instance injects broadcasts (HBRBC_SM_NO_FAKE)


def sm_state_bytes_host(n, roots):
    """hbrbc_sm_state_bytes without the library (hbbft_amd/csrc/launchers.hpp
    sm_state_bytes): per node, with several roots a u16 echo/ready entry per
    sender, can_decode masks per root, a full-Echo mask; with one root four
    bitmasks per 32 senders and the can_decode mask; counters and flags;
    rounded to 16 bytes."""
    w = (n + 31) // 32
    er = 16 * w if roots == 1 else 2 * n
    full = 0 if roots == 1 else 4 * w
    return (er + 4 * roots * w + full + 6 * roots + 4 + 6 + 15) & ~15


def _bind():
    L = lib()
    if not getattr(L, "_sm_bound", False):
        L.hbrbc_sm_state_bytes.restype = ctypes.c_size_t
        L.hbrbc_sm_state_bytes.argtypes = [ctypes.c_size_t, ctypes.c_size_t]
        L.hbrbc_sm_round.restype = ctypes.c_int
        L.hbrbc_sm_round.argtypes = [_P, ctypes.POINTER(SmArgs), _P]
        L._sm_bound = True
    return L


# ------------------------------------------------------------------ scenario --
class Instance:
    """One broadcast instance: `values[c]` is the payload of root slot c (c = 0
    the proposer's value); value_root[j] / value_tamper[j] what the proposer's
    Value to node j carries (NONE: no Value); role[j] the node's behaviour;
    fake_from (or None) the node that injects the broadcasts of the nodes in
    fake_list, whose value is values[fake_root]."""

    def __init__(self, n, proposer, values, value_root=None, value_tamper=None, role=None,
                 fake_from=None, fake_list=(), fake_root=None):
        self.n, self.proposer, self.values = n, proposer, [bytes(v) for v in values]
        assert len(set(self.values)) == len(self.values), "root slots need distinct values"
        self.value_root = list(value_root) if value_root is not None else [0] * n
        self.value_tamper = list(value_tamper) if value_tamper is not None else [0] * n
        self.role = list(role) if role is not None else [HONEST] * n
        self.fake_from, self.fake_list, self.fake_root = fake_from, sorted(fake_list), fake_root
        assert self.value_root[proposer] != NONE, "the proposer handles its own Value"
        if fake_from is not None:
            assert fake_root is not None and fake_list


class Scenario:
    """`count` instances of one validator count n (roots: codeword slots)."""

    def __init__(self, n, instances):
        self.n = n
        self.instances = list(instances)
        assert all(i.n == n for i in self.instances)
        self.roots = max(len(i.values) for i in self.instances)
        assert self.roots <= 8

    @property
    def count(self):
        return len(self.instances)

    def tensors(self, device):
        n, cnt = self.n, self.count
        W = (n + 31) // 32
        u8 = dict(dtype=torch.uint8)
        prop = torch.tensor([i.proposer for i in self.instances], **u8)
        role = torch.tensor([i.role for i in self.instances], **u8).view(cnt, n)
        vr = torch.tensor([i.value_root for i in self.instances], **u8).view(cnt, n)
        vt = torch.tensor([i.value_tamper for i in self.instances], **u8).view(cnt, n)
        ff = torch.tensor([NONE if i.fake_from is None else i.fake_from for i in self.instances], **u8)
        fr = torch.tensor([0 if i.fake_root is None else i.fake_root for i in self.instances], **u8)
        import numpy as np
        flw = np.zeros((cnt, W), np.uint32)
        for r, i in enumerate(self.instances):
            for F in i.fake_list:
                flw[r, F // 32] |= np.uint32(1 << (F % 32))
        fl = torch.from_numpy(flw.view(np.int32))   # bit patterns (uint32 words)
        return {k: v.to(device) for k, v in dict(proposer=prop, role=role, value_root=vr,
                                                value_tamper=vt, fake_from=ff, fake_root=fr,
                                                fake_list=fl).items()}


def honest_tensors(n, proposers, device):
    """Scenario tensors of honest instances: proposers [count] (a tensor or
    list), every node honest, every Value from codeword 0, no injection."""
    dev = torch.device("cuda", device) if isinstance(device, int) else device
    prop = torch.as_tensor(proposers, dtype=torch.uint8).to(dev)
    cnt = prop.shape[0]
    W = (n + 31) // 32
    z = torch.zeros((cnt, n), dtype=torch.uint8, device=dev)
    return dict(proposer=prop, role=z, value_root=z, value_tamper=z,
                fake_from=torch.full((cnt,), NONE, dtype=torch.uint8, device=dev),
                fake_root=torch.zeros(cnt, dtype=torch.uint8, device=dev),
                fake_list=torch.zeros((cnt, W), dtype=torch.int32, device=dev))


def tampered(p):
    """The corrupted copy of a proof a CORRUPT_ECHO node (or a tampering
    proposer) sends: first value byte flipped, index / digests / root kept."""
    v = p.value()
    return type(p)(bytes([v[0] ^ 1]) + v[1:], p.index(), p.digests(), p.root_hash())


def data_plane(scn, device=0):
    """Encode every root slot's codeword (one batched launch per stage),
    validate every proof and its tampered copy, decode each root once.
    Returns proof_ok [count][roots][2][n], decode_ok [count][roots] (uint8,
    on `device`), the decoded payloads {(inst, c): bytes} and the trees."""
    n, cnt, C = scn.n, scn.count, scn.roots
    items, keys = [], []
    for r, inst in enumerate(scn.instances):
        for c, v in enumerate(inst.values):
            items.append((n, v))
            keys.append((r, c))
    trees = dict(zip(keys, send_shards_batch(items, device=device)))
    proofs = {}
    for (r, c), t in trees.items():
        for j in range(n):
            p = t.proof(j)
            proofs[(r, c, 0, j)] = p
            proofs[(r, c, 1, j)] = tampered(p)
    validate_proofs(list(proofs.values()), n, device=device)
    ok = torch.zeros((cnt, C, 2, n), dtype=torch.uint8)
    for (r, c, t, j), p in proofs.items():
        ok[r, c, t, j] = 1 if p.validate(n) else 0
    # decode_from_shards of each root from n - f of its rows (a codeword
    # decodes from any k of its rows; the last f are dropped so the
    # reconstruct runs)
    f = (n - 1) // 3
    reqs = [(n, [v if j < n - f else None for j, v in enumerate(t.values())], t.root_hash())
            for t in trees.values()]
    outs = decode_shards_batch(reqs, device=device)
    dec = torch.zeros((cnt, C), dtype=torch.uint8)
    payloads = {}
    for key, o in zip(trees, outs):
        if o is not None:
            dec[key] = 1
            payloads[key] = o
    return ok.to(device), dec.to(device), payloads, trees


# ------------------------------------------------------------- one rank -----
class StateMachineRank:
    """The hosted nodes [node_lo, node_lo + R) of rank `rank` of `world` for
    `count` instances (R = ceil(n / world)).  `sc`: the scenario tensors
    (Scenario.tensors or honest_tensors); ok / dec: the data plane's
    proof_ok [count][roots][2][n] and decode_ok [count][roots]."""

    def __init__(self, n, count, roots, sc, rank, world, device=0, max_out=24, max_faults=32,
                 ok=None, dec=None, max_rounds=64):
        self.n, self.count, self.roots = n, count, roots
        self.rank, self.world = rank, world
        self.R = -(-n // world)
        # every rank hosts at least one node (sharded.Topology's rule): with
        # n=10, world=8 ranks 5..7 would start at node 10..14
        if world < 1 or (world - 1) * self.R >= n:
            raise ValueError("world %d leaves rank %d without nodes at n=%d"
                             % (world, world - 1, n))
        if not 0 <= rank < world:
            raise ValueError("rank %d outside world %d" % (rank, world))
        self.node_lo = rank * self.R
        self.W = (n + 31) // 32
        self.rec = 1 + self.W
        self.max_out, self.max_faults = max_out, max_faults
        self.rb = RbcBatch(n, device=device)
        dev = self.rb.device
        self.device = dev
        L = _bind()
        sb = L.hbrbc_sm_state_bytes(n, roots)
        R, cnt = self.R, count
        self.sc = sc
        # no fake_from node anywhere: rounds >= 2 run the kernels without the
        # Value / Fake handlers (sim.hip Sm::deliver, LEAN)
        self.flags = SM_NO_FAKE if bool((sc["fake_from"] == NONE).all()) else 0
        self.ok, self.dec = ok, dec
        self.state = torch.zeros((cnt, R, sb), dtype=torch.uint8, device=dev)
        self.out = torch.zeros((cnt, R, max_out, self.rec), dtype=torch.int32, device=dev)
        self.out_count = torch.zeros((cnt, R), dtype=torch.int32, device=dev)
        self.output_root = torch.full((cnt, R), NONE, dtype=torch.uint8, device=dev)
        self.faults = torch.zeros((cnt, R, max(1, max_faults)), dtype=torch.int16, device=dev)
        self.fault_count = torch.zeros((cnt, R), dtype=torch.int32, device=dev)
        # per round: records emitted, overflow flag (hbrbc_sm_args.emitted of round r)
        self.max_rounds = max_rounds
        self.hist = torch.zeros((max_rounds, 2), dtype=torch.int32, device=dev)
        # every sender's records of the previous round, [G][count][R][E][rec]
        self.inbox = torch.zeros((world, cnt, R, max_out, self.rec), dtype=torch.int32, device=dev)
        self.inbox_count = torch.zeros((world, cnt, R), dtype=torch.int32, device=dev)
        self.records = 0   # records emitted over the last run (all rounds)

    @classmethod
    def from_scenario(cls, scn, rank, world, device=0, max_out=24, max_faults=32, ok=None,
                      dec=None):
        dev = torch.device("cuda", device) if isinstance(device, int) else device
        return cls(scn.n, scn.count, scn.roots, scn.tensors(dev), rank, world, device, max_out,
                   max_faults, ok, dec)

    def reset(self):
        """Fresh nodes (before round 0 of another run)."""
        self.state.zero_()
        self.hist.zero_()
        self.out_count.zero_()
        self.inbox_count.zero_()
        self.output_root.fill_(NONE)
        self.fault_count.zero_()
        self.records = 0

    def swap_local(self):
        """One rank: this round's records become the next round's inbox."""
        self.inbox, self.out = self.out.unsqueeze(0), self.inbox[0]
        self.inbox_count, self.out_count = self.out_count.unsqueeze(0), self.inbox_count[0]

    def round(self, r, active=None, stream=None):
        """Handle round r's inbox (round 0: the proposers' broadcast()).
        active: None, or a device int32 scalar tensor -- the records every
        sender emitted in round r - 1; the kernel returns at once when it is
        0 (quiescent), so rounds can be enqueued without reading back."""
        if r >= self.max_rounds:
            raise RuntimeError("state machine: round %d past max_rounds %d" % (r, self.max_rounds))
        s = self.sc
        a = SmArgs(count=self.count, node_lo=self.node_lo, nodes=self.R, rows_per_rank=self.R,
                   roots=self.roots, max_out=self.max_out, max_faults=self.max_faults, round=r,
                   flags=self.flags)
        for name in ("proposer", "role", "value_root", "value_tamper", "fake_from", "fake_root",
                     "fake_list"):
            setattr(a, name, s[name].data_ptr())
        a.proof_ok, a.decode_ok = self.ok.data_ptr(), self.dec.data_ptr()
        a.in_, a.in_count = self.inbox.data_ptr(), self.inbox_count.data_ptr()
        a.out, a.out_count = self.out.data_ptr(), self.out_count.data_ptr()
        a.state, a.output_root = self.state.data_ptr(), self.output_root.data_ptr()
        a.faults, a.fault_count = self.faults.data_ptr(), self.fault_count.data_ptr()
        a.emitted = self.hist[r].data_ptr()
        a.active = None if active is None else active.data_ptr()
        st = stream if stream is not None else torch.cuda.current_stream(self.device)
        _check(_bind().hbrbc_sm_round(self.rb.coding.handle, ctypes.byref(a),
                                      ctypes.c_void_p(st.cuda_stream)))

    def emitted(self, r):
        """Device int32 scalar: records this rank emitted in round r."""
        return self.hist[r, 0]

    def exchange(self, ex, async_op=False):
        """All-gather of this round's records (the Ready / EchoHash / CanDecode
        and Echo-reference fan-out) into every rank's inbox."""
        return [ex.all_gather(self.inbox, self.out, async_op, name="sm_messages"),
                ex.all_gather(self.inbox_count, self.out_count, async_op, name="sm_counts")]

    # -- results -------------------------------------------------------------
    def outputs(self):
        """[count][hosted] decided root slot or NONE."""
        return self.output_root.cpu().numpy()

    def fault_logs(self):
        """{(inst, node): [(blamed node, FaultKind name)]} of the hosted nodes."""
        fc = self.fault_count.cpu().numpy()
        fl = self.faults.cpu().numpy().astype("uint16")
        out = {}
        for i in range(self.count):
            for r in range(self.R):
                node = self.node_lo + r
                if node >= self.n:
                    continue
                cnt = int(fc[i, r])
                if cnt > self.max_faults:
                    raise RuntimeError("fault log overflow at (%d, %d): %d records" % (i, node, cnt))
                out[(i, node)] = [(int(v) >> 8, FAULT_KINDS[int(v) & 0xFF]) for v in fl[i, r, :cnt]]
        return out


class LoopbackExchange:
    """The all-gather of `world` virtual ranks living in one process."""

    def __init__(self, ranks):
        self.ranks = ranks

    def gather(self):
        outs = torch.stack([r.out for r in self.ranks])
        cnts = torch.stack([r.out_count for r in self.ranks])
        for r in self.ranks:
            r.inbox.copy_(outs)
            r.inbox_count.copy_(cnts)


ROUND_BATCH = 6   # rounds enqueued per read-back (honest runs quiesce after 5)


def _check_batch(ranks, h, r0, own=None):
    """h [ranks][rounds][2] (host) of rounds r0..: records per round and the
    overflow flags; returns the number of rounds run if one of them was
    quiescent (no records anywhere), else None.  own: the records of THIS
    rank per (sub-batch, round) where h holds every rank's totals."""
    for i in range(h.shape[1]):
        fl = int(h[:, i, 1].max())
        if fl & 2:
            raise RuntimeError("state machine: a Value / Fake record or a fake_from node reached "
                               "a round run without those handlers (hbrbc_sm_args.flags)")
        if fl:
            raise RuntimeError("state machine: a node emitted more than %d messages in a round"
                               % ranks[0].max_out)
        mine = h[:, i, 0] if own is None else own[:, i]
        for sm, c in zip(ranks, mine):
            sm.records += int(c)
        if int(h[:, i, 0].sum()) == 0:
            return r0 + i + 1
    return None


class LocalRounds:
    """The rounds of the StateMachineRank objects of one process with no
    process group -- the virtual ranks of a loopback topology (loopback=True:
    their records are gathered between rounds) or independent objects each
    talking to itself -- split into enqueue and read-back so a caller can
    overlap them with other work: `launch()` enqueues the first ROUND_BATCH
    rounds on `stream` (default: the current stream) and returns at once;
    `wait()` reads the per-round counts back (one host read, synchronising
    that stream only), enqueues and reads further batches until the network
    is quiescent, and returns the number of rounds.

    Round r gets the device total of round r - 1's records as `active` and
    returns at once when it is 0, so the rounds past quiescence cost an empty
    launch (round 3 read the counts back after every round: ~0.3 ms of host
    gaps per step in the validator-sharded bench objects)."""

    def __init__(self, ranks, loopback, max_rounds=64, stream=None):
        self.ranks = ranks
        self.max_rounds = min(max_rounds, min(sm.max_rounds for sm in ranks))
        self.loop = LoopbackExchange(ranks) if loopback and len(ranks) > 1 else None
        self.stream = stream
        dev = ranks[0].device
        # with a loopback the next round's flag is the total over all ranks
        self.act = torch.zeros(self.max_rounds + 1, dtype=torch.int32, device=dev) \
            if self.loop is not None else None
        self.next = 0

    def _enqueue(self, r, hi):
        ranks, act = self.ranks, self.act
        for rr in range(r, hi):
            for sm in ranks:
                if rr == 0:
                    sm.round(0)
                else:   # own count (independent objects) or the device total
                    sm.round(rr, active=sm.emitted(rr - 1) if act is None else act[rr])
            if act is not None:
                act[rr + 1].copy_(torch.stack([sm.emitted(rr) for sm in ranks]).sum())
            if self.loop is not None:
                self.loop.gather()
            else:
                for sm in ranks:
                    sm.swap_local()
        self.next = hi

    def _ctx(self):
        return torch.cuda.stream(self.stream) if self.stream is not None else _nullctx()

    def launch(self):
        """Every run starts from fresh nodes: the per-round counts (hist) are
        accumulated by the kernel, and the inbox of the rounds after the last
        quiescent one still holds records, so a run never continues another."""
        with self._ctx():
            for sm in self.ranks:
                sm.reset()
            self._enqueue(0, min(self.max_rounds, ROUND_BATCH))
        return self

    def wait(self):
        r = 0   # first round whose count has not been read
        with self._ctx():
            while True:
                hi = self.next
                h = torch.stack([sm.hist[r:hi] for sm in self.ranks]).cpu()   # one read
                done = _check_batch(self.ranks, h, r)
                if done is not None:
                    return done
                if hi >= self.max_rounds:
                    raise RuntimeError("state machine did not quiesce in %d rounds"
                                       % self.max_rounds)
                self._enqueue(hi, min(self.max_rounds, hi + ROUND_BATCH))
                r = hi


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def run_rounds(ranks, exchange=None, max_rounds=64):
    """Drive the state machine until no node emits a message.  `ranks`: the
    StateMachineRank objects of this process -- all virtual ranks of one
    topology for a loopback run (exchange None), or independent objects of
    this rank (e.g. pipelined sub-batches) with a DistExchange / SoloExchange
    `exchange`, whose world they share.  Returns the number of rounds
    (LocalRounds / _run_rounds_dist: batches of rounds, one read-back per
    batch).  Every run starts from fresh nodes (StateMachineRank.reset)."""
    if exchange is not None and exchange.world > 1:
        return _run_rounds_dist(ranks, exchange, max_rounds)
    return LocalRounds(ranks, loopback=exchange is None, max_rounds=max_rounds).launch().wait()


class DistRounds:
    """run_rounds over a process group, split into enqueue and read-back like
    LocalRounds so a caller can overlap the rounds with other work (the
    validator-sharded step pipelines at world > 1, sharded.OverlapPipe):
    `launch()` enqueues the first ROUND_BATCH rounds on `stream` and returns;
    `wait()` reads the gathered tails back once per batch (synchronising that
    stream only), enqueues further batches until quiescence and returns the
    number of rounds.  ONE all-gather per round carries every sub-batch's
    records and counts plus each one's emitted count and overflow flag
    (instead of an all-reduce and two all-gathers per sub-batch); the next
    round's `active` is the device sum of the gathered counts.  Every rank
    reads the same tails, so every rank makes the same enqueue decisions and
    the collectives of `ex` stay in the same order on every rank.  Give `ex`
    a process group of its own when other collectives (the data plane's) run
    concurrently on another stream."""

    def __init__(self, ranks, ex, max_rounds=64, stream=None):
        self.ranks, self.ex, self.stream = ranks, ex, stream
        self.max_rounds = min(max_rounds, min(sm.max_rounds for sm in ranks))
        self.next = 0

    def _ctx(self):
        return torch.cuda.stream(self.stream) if self.stream is not None else _nullctx()

    def _enqueue(self, r, hi):
        ranks, ex = self.ranks, self.ex
        send, recv, body, k = self.send, self.recv, self.body, len(ranks)
        for rr in range(r, hi):
            for sm in ranks:
                sm.round(rr, active=None if rr == 0 else self.act[rr])
            off = 0
            for sm, (a, b) in zip(ranks, self.parts):
                send[off:off + a].copy_(sm.out.view(-1))
                send[off + a:off + a + b].copy_(sm.out_count.view(-1))
                off += a + b
            hist = torch.stack([sm.hist[rr] for sm in ranks])       # [k][2]
            send[body:body + k].copy_(hist[:, 0])
            send[body + k:].copy_(hist[:, 1].amax().view(1))
            ex.all_gather(recv, send, name="sm_round")
            self.tails[rr].copy_(recv[:, body:])
            self.act[rr + 1].copy_(recv[:, body:body + k].sum())
            off = 0
            for sm, (a, b) in zip(ranks, self.parts):
                sm.inbox.view(ex.world, a).copy_(recv[:, off:off + a])
                sm.inbox_count.view(ex.world, b).copy_(recv[:, off + a:off + a + b])
                off += a + b
        self.next = hi

    def launch(self):
        """Fresh nodes (every run), then the first batch of rounds."""
        ranks, ex = self.ranks, self.ex
        dev = ranks[0].device
        with self._ctx():
            for sm in ranks:
                sm.reset()
            self.parts = [(sm.out.numel(), sm.out_count.numel()) for sm in ranks]
            k = len(ranks)
            self.body = sum(a + b for a, b in self.parts)
            self.send = torch.zeros(self.body + k + 1, dtype=torch.int32, device=dev)
            self.recv = torch.empty((ex.world, self.body + k + 1), dtype=torch.int32, device=dev)
            self.tails = torch.zeros((self.max_rounds, ex.world, k + 1), dtype=torch.int32,
                                     device=dev)
            self.act = torch.zeros(self.max_rounds + 1, dtype=torch.int32, device=dev)
            self._enqueue(0, min(self.max_rounds, ROUND_BATCH))
        return self

    def wait(self):
        ranks, ex, k = self.ranks, self.ex, len(self.ranks)
        r = 0
        with self._ctx():
            while True:
                hi = self.next
                t = self.tails[r:hi].cpu()                          # [rounds][world][k + 1]
                # every rank's per-round totals (records of all ranks, overflow of any)
                h = torch.stack([t[:, :, :k].sum(dim=1).sum(dim=1), t[:, :, k].amax(dim=1)], dim=1)
                own = t[:, ex.rank, :k].transpose(0, 1)             # [k][rounds]
                done = _check_batch(ranks, h.unsqueeze(0), r, own=own)
                if done is not None:
                    return done
                if hi >= self.max_rounds:
                    raise RuntimeError("state machine did not quiesce in %d rounds"
                                       % self.max_rounds)
                self._enqueue(hi, min(self.max_rounds, hi + ROUND_BATCH))
                r = hi


def _run_rounds_dist(ranks, ex, max_rounds):
    """run_rounds over a process group (DistRounds, enqueued and read back in
    one call)."""
    return DistRounds(ranks, ex, max_rounds).launch().wait()


def simulate(scn, world=1, device=0, max_out=24, max_faults=None):
    """Every node of every instance of `scn` over `world` virtual ranks on one
    GPU.  Returns ({(inst, node): output bytes or None}, {(inst, node): fault
    list}, rounds)."""
    if max_faults is None:   # the ProposeAdversary costs a node ~2 faults per faulty node
        max_faults = max(32, 4 * scn.n)
    ok, dec, payloads, _ = data_plane(scn, device)
    ranks = [StateMachineRank.from_scenario(scn, g, world, device, max_out, max_faults, ok, dec)
             for g in range(world)]
    rounds = run_rounds(ranks)
    outputs, faults = {}, {}
    for sm in ranks:
        oc = sm.outputs()
        for i in range(scn.count):
            for r in range(sm.R):
                node = sm.node_lo + r
                if node < scn.n:
                    c = int(oc[i, r])
                    outputs[(i, node)] = None if c == NONE else payloads[(i, c)]
        faults.update(sm.fault_logs())
    return outputs, faults, rounds
