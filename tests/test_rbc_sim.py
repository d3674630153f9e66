"""the Broadcast state machine on the GPU (hbbft_amd/rbc_sim.py,
hbbft_amd/csrc/sim.hip) under the reference's adversaries.

Every scenario runs twice: through the GPU state machine (every node of every
instance, Echo/EchoHash/Ready/CanDecode counters on the device, over 1..8
virtual ranks whose per-round messages are all-gathered) and through the host
restatement -- hbbft_amd/broadcast.py nodes driven round by round by
tests/virtual_net.py run_rounds on the CPU oracle backend.  Every node's
outputs, fault log (blamed node and FaultKind, in order) and the round count
must be equal.

Adversaries: tests/broadcast.rs:33-98 ProposeAdversary (the first f nodes
inject their own "Fake news" broadcasts, with and without dropping everything
else they send), a proposer sending two codewords / tampered proofs / nothing
to different validators, faulty validators corrupting or withholding their
Echoes, and mixtures of these.
"""
import os
import random
import socket

import pytest
import torch

import virtual_net as vn
from hbbft_amd.rbc_sim import (CORRUPT_ECHO, HONEST, NONE, SILENT, WITHHOLD_ECHO, Instance,
                               Scenario)


def _oracle():
    import oracle_backend
    return oracle_backend


def _faulty(n):
    return list(range(vn.max_faulty(n)))


KINDS = ("honest", "propose", "propose_drop", "equivocate", "equivocate_2of3", "corrupt_echo",
         "withhold_echo", "partial_values", "tampered_values", "mixed")
BAD_PROPOSER = ("equivocate", "equivocate_2of3", "partial_values", "tampered_values", "mixed")


def make_instances(n, rng, seed_tag=0):
    """Scenario instances of one validator count covering every adversary."""
    f = vn.max_faulty(n)
    out = []

    def value(tag):
        return b"%s-%d-%d-" % (tag, n, seed_tag) + bytes(rng.randrange(256) for _ in range(rng.randrange(0, 40)))

    for kind in KINDS:
        # a misbehaving proposer is one of the f faulty nodes (the first f), so
        # at most f nodes misbehave and the reference's guarantees apply
        bad_proposer = kind in BAD_PROPOSER
        if bad_proposer and not f:
            kind, bad_proposer = "honest", False
        p = rng.randrange(f) if bad_proposer else rng.randrange(n)
        vals = [value(b"A")]
        role = [HONEST] * n
        vr, vt = [0] * n, [0] * n
        fake_from, fake_list, fake_root = None, (), None
        if kind in ("propose", "propose_drop") and f:
            vals.append(b"Fake news")
            fake_list = _faulty(n)
            cand = [F for F in fake_list if F != p]
            fake_from = cand[0] if cand else p
            fake_root = 1
            if kind == "propose_drop":
                for F in fake_list:
                    role[F] = SILENT
        elif kind.startswith("equivocate"):
            vals.append(value(b"B"))
            share = 2 if kind == "equivocate" else 3
            for j in range(n):
                vr[j] = 1 if (j + p) % share == 0 else 0
            vr[p] = 0
        elif kind == "corrupt_echo":
            for F in _faulty(n):
                role[F] = CORRUPT_ECHO
        elif kind == "withhold_echo":
            for F in _faulty(n):
                role[F] = WITHHOLD_ECHO
        elif kind == "partial_values":
            for j in rng.sample(range(n), min(n - 1, f + 1)):
                if j != p:
                    vr[j] = NONE
        elif kind == "tampered_values":
            for j in rng.sample(range(n), min(n, f + 1)):
                vt[j] = 1
        elif kind == "mixed" and f:
            vals.append(value(b"B"))
            vals.append(b"Fake news")
            fake_list = _faulty(n)
            fake_from, fake_root = fake_list[-1], 2
            for j in range(n):
                vr[j] = rng.choice([0, 0, 0, 1, NONE])
                vt[j] = 1 if rng.random() < 0.1 else 0
            vr[p], vt[p] = 0, 0
            for F in fake_list:
                role[F] = rng.choice([HONEST, SILENT, CORRUPT_ECHO, WITHHOLD_ECHO])
        out.append(Instance(n, p, vals, vr, vt, role, fake_from, fake_list, fake_root))
    return out


SINGLE_KINDS = ("honest", "silent", "corrupt_echo", "withhold_echo", "partial_values",
                "tampered_values", "faulty_mix")


def make_single_root_instances(n, rng, seed_tag=0):
    """Scenario instances with ONE codeword each (Scenario.roots == 1), the
    form the validator-sharded runs use (sim.hip Sm<true>: Echo / Ready
    entries as four 32-sender bitmasks, counters and flags in registers):
    every adversary that
    needs no second value -- silent faulty nodes (the ProposeAdversary's drop
    without its injected broadcasts), corrupted or withheld Echoes, a faulty
    proposer that sends nothing or tampered proofs to some validators, and a
    mixture of those."""
    f = vn.max_faulty(n)
    out = []
    for kind in SINGLE_KINDS:
        bad_proposer = kind in ("partial_values", "tampered_values", "faulty_mix") and f > 0
        p = rng.randrange(f) if bad_proposer else rng.randrange(n)
        val = b"S-%d-%d-%s-" % (n, seed_tag, kind.encode()) + bytes(
            rng.randrange(256) for _ in range(rng.randrange(0, 64)))
        role = [HONEST] * n
        vr, vt = [0] * n, [0] * n
        if kind == "silent":
            for F in _faulty(n):
                role[F] = SILENT
        elif kind == "corrupt_echo":
            for F in _faulty(n):
                role[F] = CORRUPT_ECHO
        elif kind == "withhold_echo":
            for F in _faulty(n):
                role[F] = WITHHOLD_ECHO
        elif kind == "partial_values" and f:
            for j in rng.sample(range(n), min(n - 1, f + 1)):
                if j != p:
                    vr[j] = NONE
        elif kind == "tampered_values" and f:
            for j in rng.sample(range(n), min(n, f + 1)):
                vt[j] = 1
        elif kind == "faulty_mix" and f:
            for j in range(n):
                vr[j] = rng.choice([0, 0, 0, 0, NONE])
                vt[j] = 1 if rng.random() < 0.15 else 0
            vr[p], vt[p] = 0, 0
            for F in _faulty(n):
                role[F] = rng.choice([HONEST, SILENT, CORRUPT_ECHO, WITHHOLD_ECHO])
        out.append(Instance(n, p, [val], vr, vt, role))
    return out


def host_run(inst):
    outs, faults, rounds = vn.run_rounds(inst, _oracle())
    return outs, faults, rounds


# ------------------------------------------------------------------ CPU ----
def test_round_schedule_honest_and_propose_adversary():
    """The round driver itself reproduces the reference's test assertions
    (tests/broadcast.rs:127-146): with a correct proposer every node outputs the
    value exactly once; otherwise all correct nodes (index >= f) agree."""
    rng = random.Random(3)
    for n in (1, 2, 4, 7, 10):
        f = vn.max_faulty(n)
        for inst in make_instances(n, rng):
            outs, faults, _ = host_run(inst)
            honest_p = (inst.proposer >= f and all(v == 0 for v in inst.value_root)
                        and not any(inst.value_tamper))
            if honest_p:
                assert all(outs[i] == [inst.values[0]] for i in range(n)), (n, outs)
            else:
                assert len({tuple(outs[i]) for i in range(f, n)}) == 1, (n, outs)
            # a correct node never blames a correct one
            for i in range(f, n):
                assert all(b < f or (b == inst.proposer and not honest_p) for b, _ in faults[i]), \
                    (n, i, faults[i])


def _gloo_sm_worker(rank, world, port, q):
    """The state machine's per-round exchange shape: every rank's records
    [count][R][E][1 + W] (and counts [count][R]) all-gathered into the
    blocked inbox [G][count][R][E][1 + W] the kernel reads (sender s at block
    s // R, row s % R)."""
    import torch.distributed as dist

    from hbbft_amd.sharded import DistExchange
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n, count, E = 10, 3, 4
        R, rec = -(-n // world), 1 + (n + 31) // 32
        out = torch.zeros((count, R, E, rec), dtype=torch.int32)
        cnt = torch.zeros((count, R), dtype=torch.int32)
        for i in range(count):
            for r in range(R):
                s = rank * R + r
                cnt[i, r] = (s + i) % E
                for e in range(E):
                    out[i, r, e, 0] = s * 1000 + i * 10 + e
        inbox = torch.empty((world, count, R, E, rec), dtype=torch.int32)
        icnt = torch.empty((world, count, R), dtype=torch.int32)
        ex = DistExchange()
        for h in [ex.all_gather(inbox, out, True, name="sm_messages"),
                  ex.all_gather(icnt, cnt, True, name="sm_counts")]:
            h.wait()
        good = True
        for s in range(world * R):
            for i in range(count):
                blk = inbox[s // R, i, s % R]
                good &= int(icnt[s // R, i, s % R]) == (s + i) % E
                good &= [int(blk[e, 0]) for e in range(E)] == [s * 1000 + i * 10 + e for e in range(E)]
        q.put((rank, "ok" if good else "mismatch"))
    except Exception as e:  # pragma: no cover
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def test_gloo_state_machine_exchange_shape():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = [ctx.Process(target=_gloo_sm_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(60)
    assert res == {0: "ok", 1: "ok"}, res


# ------------------------------------------------------------------ GPU ----
@pytest.mark.gpu
@pytest.mark.parametrize("n,worlds", [(4, (1, 2)), (7, (1, 3)), (10, (1, 4)), (16, (1, 2, 8)),
                                      (31, (1, 4)), (64, (8,))])
def test_state_machine_matches_host_restatement(n, worlds):
    """Per node: outputs, fault log (blamed node + kind, in order) and the
    number of rounds equal the host state machine on the same schedule."""
    from hbbft_amd.rbc_sim import simulate
    rng = random.Random(1000 + n)
    insts = make_instances(n, rng) + make_instances(n, rng, seed_tag=1)
    if n == 64:
        insts = insts[:10]
    scn = Scenario(n, insts)
    ref = [host_run(inst) for inst in insts]
    for world in worlds:
        outs, faults, rounds = simulate(scn, world=world)
        assert rounds == max(r[2] for r in ref), (world, rounds, [r[2] for r in ref])
        for i, (ho, hf, _) in enumerate(ref):
            for node in range(n):
                got = [] if outs[(i, node)] is None else [outs[(i, node)]]
                assert got == ho[node], (world, i, node, got, ho[node])
                assert faults[(i, node)] == hf[node], (world, i, node, faults[(i, node)], hf[node])


_HOST_CACHE = {}


def _single_root_case(n):
    """The single-root scenario of validator count n and its host results
    (computed once per n for all kernel forms and worlds)."""
    if n not in _HOST_CACHE:
        rng = random.Random(5000 + n)
        insts = make_single_root_instances(n, rng) + make_single_root_instances(n, rng, 1)
        scn = Scenario(n, insts)
        assert scn.roots == 1
        _HOST_CACHE[n] = (scn, [host_run(inst) for inst in insts])
    return _HOST_CACHE[n]


# the launch forms of hbrbc_sm_round (sim.hip launch_sm_round): the staged
# kernel at 4 waves/SIMD (128 VGPRs, spills) and at the default budget, and the
# global form; max_out 8 keeps the N=128 staged image under 64 KiB
SM_FORMS = {"staged_w4": {"HBRBC_SM_W4": "1"}, "staged_w3": {"HBRBC_SM_W4": "0"},
            "global": {"HBRBC_SM_STAGED": "0"},
            # the global-records kernel forced on (n = 64: two instances per
            # block, one per wave) and off (n = 128: the staged records)
            "grec_on": {"HBRBC_SM_GREC": "1"}, "grec_off": {"HBRBC_SM_GREC": "0"},
            # every round through the kernels with the Value / Fake handlers
            # (default: rounds >= 2 of a batch without injection run without them)
            "lean_off": {"HBRBC_SM_LEAN": "0"},
            # LDS-staged records read per lane even where every wave holds one
            # instance (default at nodes % 64 == 0: scalar dispatch)
            "wi_off": {"HBRBC_SM_WI": "0"}}


def test_single_root_scenarios_on_host():
    """CPU: the single-root scenarios are well formed (one root) and the host
    restatement keeps the reference's guarantees on them."""
    rng = random.Random(11)
    for n in (4, 7, 16):
        f = vn.max_faulty(n)
        insts = make_single_root_instances(n, rng)
        assert Scenario(n, insts).roots == 1
        for inst in insts:
            outs, faults, _ = host_run(inst)
            correct = [outs[i] for i in range(f, n)]
            assert len({tuple(o) for o in correct}) == 1
            for i in range(f, n):
                assert all(b < f or b == inst.proposer for b, _ in faults[i]), (i, faults[i])


@pytest.mark.gpu
@pytest.mark.parametrize("form", sorted(SM_FORMS))
@pytest.mark.parametrize("n", [4, 16, 64, 128])
def test_single_root_state_machine_matches_host(n, form, monkeypatch):
    """The one-root kernels (Sm<true>) the validator-sharded bench runs, in
    each launch form, per node against the host restatement: outputs, fault
    logs (blamed node + kind, in order) and round count, over worlds 1, 2, 8
    (the worlds that leave every rank a node)."""
    from hbbft_amd.rbc_sim import simulate
    for k, v in SM_FORMS[form].items():
        monkeypatch.setenv(k, v)
    scn, ref = _single_root_case(n)
    worlds = [w for w in (1, 2, 8) if (w - 1) * -(-n // w) < n]
    for world in worlds:
        outs, faults, rounds = simulate(scn, world=world, max_out=8)
        assert rounds == max(r[2] for r in ref), (world, rounds, [r[2] for r in ref])
        for i, (ho, hf, _) in enumerate(ref):
            for node in range(n):
                got = [] if outs[(i, node)] is None else [outs[(i, node)]]
                assert got == ho[node], (form, world, i, node, got, ho[node])
                assert faults[(i, node)] == hf[node], (form, world, i, node, faults[(i, node)],
                                                       hf[node])


@pytest.mark.gpu
@pytest.mark.parametrize("n,worlds", [(7, (1, 3)), (16, (1, 2)), (64, (1, 8))])
def test_lean_rounds_multi_root_match_host(n, worlds):
    """Batches without injected broadcasts (flags HBRBC_SM_NO_FAKE) run rounds
    >= 2 through the lean kernels (sim.hip Sm::deliver<LEAN>); with several
    roots (equivocating proposers, Sm<false>) every node's output, fault log
    and the round count still equal the host restatement."""
    from hbbft_amd.rbc_sim import SM_NO_FAKE, StateMachineRank, simulate
    rng = random.Random(2000 + n)
    insts = [i for i in make_instances(n, rng) + make_instances(n, rng, seed_tag=1)
             if i.fake_from is None]
    scn = Scenario(n, insts)
    assert scn.roots > 1
    assert StateMachineRank.from_scenario(scn, 0, 1).flags == SM_NO_FAKE
    ref = [host_run(inst) for inst in insts]
    for world in worlds:
        outs, faults, rounds = simulate(scn, world=world)
        assert rounds == max(r[2] for r in ref), (world, rounds)
        for i, (ho, hf, _) in enumerate(ref):
            for node in range(n):
                got = [] if outs[(i, node)] is None else [outs[(i, node)]]
                assert got == ho[node], (world, i, node, got, ho[node])
                assert faults[(i, node)] == hf[node], (world, i, node)


@pytest.mark.gpu
def test_lean_round_rejects_injected_records(monkeypatch):
    """A batch WITH a fake_from node marked HBRBC_SM_NO_FAKE anyway: its Fake
    node reaches a round run without the Fake handler, which reports it
    (emitted[1] bit 1), and the driver raises instead of dropping the
    injection."""
    from hbbft_amd.rbc_sim import SM_NO_FAKE, StateMachineRank, data_plane, run_rounds
    monkeypatch.delenv("HBRBC_SM_LEAN", raising=False)   # (=0 would run the full set)
    n = 7
    insts = [i for i in make_instances(n, random.Random(3)) if i.fake_from is not None]
    scn = Scenario(n, insts)
    ok, dec, _, _ = data_plane(scn, 0)
    sm = StateMachineRank.from_scenario(scn, 0, 1, 0, 24, 64, ok, dec)
    assert sm.flags == 0
    sm.flags = SM_NO_FAKE
    with pytest.raises(RuntimeError, match="without those handlers"):
        run_rounds([sm])


@pytest.mark.gpu
def test_state_machine_counters_at_size():
    """128 honest N=64 instances and 128 ProposeAdversary-with-drop
    instances on 8 virtual ranks: every correct node decides the proposer's
    value (honest proposer), and the fault logs blame only faulty nodes."""
    from hbbft_amd.rbc_sim import simulate
    n, f = 64, 21
    rng = random.Random(7)
    insts = []
    for i in range(256):
        p = rng.randrange(f, n)          # a correct proposer
        vals = [b"value %d" % i]
        if i % 2:
            role = [SILENT] * f + [HONEST] * (n - f)
            insts.append(Instance(n, p, vals + [b"Fake news"], role=role, fake_from=0,
                                  fake_list=range(f), fake_root=1))
        else:
            insts.append(Instance(n, p, vals))
    outs, faults, rounds = simulate(Scenario(n, insts), world=8)
    for i, inst in enumerate(insts):
        for node in range(n):
            assert outs[(i, node)] == inst.values[0]
            assert all(b < f for b, _ in faults[(i, node)])
    assert rounds <= 8


class _FakeSm:
    """A StateMachineRank stand-in with the buffers _run_rounds_dist moves:
    round r of rank g, sub-batch b writes records tagged (g, b, r) and emits
    until round 2 (rank 1's sub-batch 1 until round 3); like the kernel, a
    round whose `active` total is 0 returns at once."""

    def __init__(self, rank, world, b, count=3, R=2, E=2, rec=2, max_rounds=16):
        self.rank, self.b, self.max_out = rank, b, E
        self.device = torch.device("cpu")
        self.max_rounds = max_rounds
        self.out = torch.zeros((count, R, E, rec), dtype=torch.int32)
        self.out_count = torch.zeros((count, R), dtype=torch.int32)
        self.inbox = torch.zeros((world, count, R, E, rec), dtype=torch.int32)
        self.inbox_count = torch.zeros((world, count, R), dtype=torch.int32)
        self.hist = torch.zeros((max_rounds, 2), dtype=torch.int32)
        self.records = 0
        self.last = 2 if (rank, b) != (1, 1) else 3
        self.ran = []

    def reset(self):
        self.hist.zero_()
        self.out_count.zero_()
        self.inbox_count.zero_()
        self.records = 0
        self.ran = []

    def round(self, r, active=None):
        if active is not None and int(active) == 0:
            return
        self.ran.append(r)
        emits = r <= self.last
        self.out.fill_(self.rank * 10000 + self.b * 1000 + r)
        self.out_count.fill_(1 if emits else 0)
        self.hist[r, 0] = self.out_count.numel() if emits else 0


def _gloo_dist_rounds_worker(rank, world, port, q):
    import torch.distributed as dist

    from hbbft_amd.rbc_sim import _run_rounds_dist
    from hbbft_amd.sharded import DistExchange
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sms = [_FakeSm(rank, world, b) for b in range(2)]
        rounds = _run_rounds_dist(sms, DistExchange(), 16)
        good = rounds == 5   # the last emission (round 3) is delivered, round 4 is silent
        for sm in sms:
            # rounds 0..4 ran; round 5 (enqueued in the same batch) saw active 0
            good &= sm.ran == [0, 1, 2, 3, 4]
            # the inbox holds every rank's records of round 4, the silent one
            for g in range(world):
                good &= bool((sm.inbox[g] == g * 10000 + sm.b * 1000 + 4).all())
                good &= bool((sm.inbox_count[g] == 0).all())
            good &= sm.records == sm.out_count.numel() * (sm.last + 1)
        q.put((rank, "ok" if good else "mismatch rounds=%d" % rounds))
    except Exception as e:  # pragma: no cover
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def test_gloo_fused_round_exchange():
    """_run_rounds_dist (one all-gather per round for all sub-batches, emitted
    counts and overflow flags in the tail) on a gloo world of 2: termination
    round, every rank's records in every sub-batch's inbox, record counts."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = [ctx.Process(target=_gloo_dist_rounds_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(60)
    assert res == {0: "ok", 1: "ok"}, res


class _FakeLocalSm(_FakeSm):
    """_FakeSm with what LocalRounds drives on one rank: reset, emitted,
    swap_local; like the kernel, a round ADDS its records into hist[r]."""

    def __init__(self, **kw):
        super().__init__(0, 1, 0, **kw)
        self.last = 3

    def round(self, r, active=None):
        if active is not None and int(active) == 0:
            return
        self.ran.append(r)
        emits = r <= self.last
        self.out_count.fill_(1 if emits else 0)
        self.hist[r, 0] += self.out_count.numel() if emits else 0   # accumulated, not stored

    def emitted(self, r):
        return self.hist[r, 0]

    def swap_local(self):
        self.inbox, self.out = self.out.unsqueeze(0), self.inbox[0]
        self.inbox_count, self.out_count = self.out_count.unsqueeze(0), self.inbox_count[0]


def test_local_rounds_run_twice_from_fresh_nodes():
    """a second run of the same objects must not add to the first
    run's per-round counts (the kernel accumulates into hist) or deliver the
    records left after quiescence: every run starts from reset nodes and
    gives the same rounds and record count."""
    from hbbft_amd.rbc_sim import LocalRounds, run_rounds
    sm = _FakeLocalSm()
    first = LocalRounds([sm], loopback=False).launch().wait()
    rec1, ran1 = sm.records, list(sm.ran)
    second = LocalRounds([sm], loopback=False).launch().wait()
    assert (first, sm.records, sm.ran) == (second, rec1, ran1) == (5, 4 * sm.out_count.numel(),
                                                                   [0, 1, 2, 3, 4])
    assert run_rounds([sm]) == 5 and sm.records == rec1


def test_round_flags_raise_distinct_errors():
    """CPU: the per-round flags the kernels OR into emitted[1] -- bit 0 a node
    emitted more than max_out records, bit 1 a record kind (or a fake_from
    node) that the launch's handler set leaves out (hbrbc_sm_args.flags) --
    raise their own errors in the read-back; a clean quiescent batch returns
    the round count."""
    import torch

    from hbbft_amd.rbc_sim import _check_batch

    class _R:
        max_out = 4
        records = 0

    ranks = [_R()]
    ok = torch.tensor([[[5, 0], [3, 0], [0, 0]]], dtype=torch.int32)   # [ranks][rounds][2]
    assert _check_batch(ranks, ok, 0) == 3 and ranks[0].records == 8
    with pytest.raises(RuntimeError, match="more than 4 messages"):
        _check_batch(ranks, torch.tensor([[[5, 1]]], dtype=torch.int32), 0)
    with pytest.raises(RuntimeError, match="without those handlers"):
        _check_batch(ranks, torch.tensor([[[5, 2]]], dtype=torch.int32), 0)
    with pytest.raises(RuntimeError, match="without those handlers"):
        _check_batch(ranks, torch.tensor([[[5, 3]]], dtype=torch.int32), 0)
