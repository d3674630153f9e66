"""Validator-sharded simulation (hbbft_amd/sharded.py).

CPU (gloo, world 2 and 3): the topology, and that the Value all-to-all of a
destination-major slab followed by the Echo all-gather leaves every rank with
every row of every instance in the blocked layout the decoder reads.
GPU: G virtual ranks in one process (loopback exchange) run the whole step
through libhbrbc.so and are checked against the oracle; a 2-rank gloo run
shares cuda:0 (step and pipelined schedule)."""
import os
import socket

import numpy as np
import pytest
import torch

from hbbft_amd.sharded import (CommTimer, DistExchange, ShardedBroadcast, SoloExchange, Topology,
                               pipelined_step)
from oracle import pyoracle as orc


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


# ------------------------------------------------------------------ CPU ----
def test_topology():
    t = Topology(10, 4)
    assert t.rpg == 3 and t.npad == 12 and t.rows_per_block == 3
    assert [list(t.validators(r)) for r in range(4)] == [[0, 1, 2], [3, 4, 5], [6, 7, 8], [9]]
    assert t.proposers(3, 3) == [9, 9, 9] and t.proposers(1, 4) == [3, 4, 5, 3]
    with pytest.raises(ValueError):
        Topology(9, 4)   # the last rank would host no validator
    # receiver r0 = g*R misses Echoes from r0+1..r0+f (broadcast.rs:476-485), f = 3
    assert [t.receiver(r) for r in range(4)] == [0, 3, 6, 9]
    assert t.receiver_present(0) == [1, 0, 0, 0, 1, 1, 1, 1, 1, 1]
    assert t.receiver_present(3) == [0, 0, 0, 1, 1, 1, 1, 1, 1, 1]   # 10, 11, 12 wrap to 0, 1, 2
    assert all(sum(t.receiver_present(r)) == 10 - 3 for r in range(4))
    # Echo rows: received and from other ranks' validators
    assert t.echo_rows(0) == [4, 5, 6, 7, 8, 9]
    assert t.echo_rows(3) == [3, 4, 5, 6, 7, 8]
    assert Topology(64, 1).rows_per_block == 0 and Topology(64, 8).rows_per_block == 8


def blocked_row(buf, j, t, R, stride):
    """Row j of instance t of a blocked slab [blocks][instances][R][stride]."""
    return buf[j // R, t, j % R, :stride]


def _gloo_worker(rank, world, port, n, count, plen, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        t = Topology(n, world)
        R = t.rpg
        ex = DistExchange()
        f = t.f
        S = orc.shard_len(plen, n - 2 * f)

        def shards_of(r, i):
            sh, _ = orc.send_shards(n, f, orc.gen_payload(100 + r, i, plen).tobytes())
            return torch.from_numpy(sh)

        # what the encoder writes: the destination-major slab [G][C][R][S]
        slab = torch.zeros((world, count, R, S), dtype=torch.uint8)
        for i in range(count):
            sh = shards_of(rank, i)
            for j in range(n):
                slab[j // R, i, j % R] = sh[j]
        recv = torch.empty_like(slab)
        ex.all_to_all(recv, slab)
        # Value: block s = this rank's validators' rows of rank s's instances
        for s in range(world):
            for i in range(count):
                sh = shards_of(s, i)
                for r in range(len(t.validators(rank))):
                    assert torch.equal(recv[s, i, r], sh[rank * R + r])
        roots = torch.full((count, 32), rank, dtype=torch.uint8)
        allr = torch.empty((world, count, 32), dtype=torch.uint8)
        ex.all_gather(allr, roots)
        assert [int(allr[s, 0, 0]) for s in range(world)] == list(range(world))
        # Echo all-gather: [G_v][G*C][R][S]; instance (s, i) = s*C + i, row j in block j // R
        echo = torch.empty((world, world * count, R, S), dtype=torch.uint8)
        ex.all_gather(echo, recv)
        for s in range(world):
            for i in range(count):
                sh = shards_of(s, i)
                for j in range(n):
                    assert torch.equal(blocked_row(echo, j, s * count + i, R, S), sh[j])
        # the async form the pipelined schedule uses (handles waited after
        # every collective of a group is issued) gives the same bytes, and the
        # per-collective byte counts are what this rank sends
        ex.reset_stats()
        recv2, echo2 = torch.empty_like(recv), torch.empty_like(echo)
        hs = [ex.all_to_all(recv2, slab, async_op=True, name="value_shards"),
              ex.all_gather(echo2, recv, async_op=True, name="echo_shards")]
        for h in hs:
            h.wait()
        assert torch.equal(recv2, recv) and torch.equal(echo2, echo)
        nb = slab.numel()
        assert ex.stats == {"value_shards": {"calls": 1, "bytes_sent": nb * (world - 1) // world},
                            "echo_shards": {"calls": 1, "bytes_sent": nb * (world - 1)}}, ex.stats
        q.put((rank, "ok"))
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n,world", [(10, 2), (16, 2), (7, 3)])
def test_gloo_value_all_to_all_and_echo_all_gather(n, world):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_gloo_worker, args=(r, world, port, n, 3, 333, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(60)
    assert res == {r: "ok" for r in range(world)}, res


# ---- the overlapped schedule at world > 1, on CPU (gloo, fake kernels) ----
class _NoStream:
    """torch.cuda stream / event stand-ins: on the CPU every op is already
    ordered, so the schedule's control flow and collectives run unchanged."""

    def __init__(self, *a, **k):
        pass

    def wait_event(self, e):
        pass

    def wait_stream(self, s):
        pass

    def record(self, stream=None):
        pass

    def elapsed_time(self, other):
        return 0.0

    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def _no_cuda_streams():
    torch.cuda.Stream = _NoStream
    torch.cuda.Event = _NoStream
    torch.cuda.stream = _NoStream
    torch.cuda.current_stream = lambda *a: _NoStream()


class _FakeSm:
    """A StateMachineRank stand-in whose rounds depend on the data plane's
    outcomes (`ok`) and on every rank's records: each round adds the
    gathered records to `acc` and emits ok * (r + 1) + rank for 3 rounds."""

    def __init__(self, rank, world, count):
        self.rank, self.count = rank, count
        self.device = torch.device("cpu")
        self.max_rounds, self.max_out = 16, 1
        self.ok = torch.zeros(count, dtype=torch.int32)
        self.out = torch.zeros((count, 1, 1, 2), dtype=torch.int32)
        self.out_count = torch.zeros((count, 1), dtype=torch.int32)
        self.inbox = torch.zeros((world, count, 1, 1, 2), dtype=torch.int32)
        self.inbox_count = torch.zeros((world, count, 1), dtype=torch.int32)
        self.hist = torch.zeros((16, 2), dtype=torch.int32)
        self.acc = torch.zeros(count, dtype=torch.int64)
        self.records = 0

    def reset(self):
        self.hist.zero_()
        self.out_count.zero_()
        self.inbox_count.zero_()
        self.acc.zero_()
        self.records = 0

    def round(self, r, active=None):
        if active is not None and int(active) == 0:
            return
        if r > 0:
            self.acc += (self.inbox[:, :, 0, 0, 0] * self.inbox_count[:, :, 0]).sum(0)
        emit = r < 3
        self.out[:, 0, 0, 0] = self.ok * (r + 1) + self.rank
        self.out_count.fill_(1 if emit else 0)
        self.hist[r, 0] += self.count if emit else 0


class _FakeShardedBroadcast:
    """The data plane of a step: Value / Echo collectives over `ex` whose
    results feed the current slot's state machine; `history` = every
    finished step's outputs, in step order."""

    def __init__(self, rank, world, count):
        self.rank, self.world, self.count = rank, world, count
        self.sms = [_FakeSm(rank, world, count) for _ in range(2)]
        self.slot, self.sm_rounds, self.sm_timing = 0, 0, None
        self.history = []

    @property
    def sm(self):
        return self.sms[self.slot]

    def encode_phase(self, payloads):
        self.pay = payloads.clone()

    def rest_phase(self, ex, xspans=None):
        g = torch.zeros((self.world, self.count), dtype=torch.int32)
        ex.all_gather(g, self.pay, name="value")                       # Value / Echo fan-out
        roots = torch.zeros((self.world, self.count), dtype=torch.int32)
        ex.all_to_all(roots, (g * (self.rank + 2)).contiguous(), name="echo")
        self.sm.ok.copy_(g.sum(0) + roots.sum(0))

    def data_step(self, payloads, ex):
        self.encode_phase(payloads)
        self.rest_phase(ex)

    def finish(self):
        self.history.append(self.sm.acc.clone())


def _gloo_schedule_worker(rank, world, port, q):
    import torch.distributed as dist

    from hbbft_amd.sharded import (OverlapPipe, interleaved_steps, run_state_machines)
    _no_cuda_streams()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ex = DistExchange()
        sm_ex = DistExchange(dist.new_group(list(range(world))))
        count, steps = 5, 5

        def pay(i):
            return torch.arange(count, dtype=torch.int32) * 7 + 100 * i + 13 * rank
        # serial: data plane, then the rounds over the data group, step by step
        ser = _FakeShardedBroadcast(rank, world, count)
        for i in range(steps):
            ser.data_step(pay(i), ex)
            ser.sm_rounds = run_state_machines([ser], ex)
        # overlapped: step i's rounds (own group) beside step i + 1's data plane
        ov = _FakeShardedBroadcast(rank, world, count)
        pipe = OverlapPipe(ov, ex, _NoStream(), main=_NoStream(), sm_ex=sm_ex)
        for i in range(steps):
            pipe.step(pay(i))
        pipe.finish()
        # two pipelines, step i on pipe i % 2
        pp = [_FakeShardedBroadcast(rank, world, count) for _ in range(2)]
        pipes = [OverlapPipe(o, ex, _NoStream(), main=_NoStream(), sm_ex=sm_ex) for o in pp]
        payl = [None, None]

        class _Feed:   # interleaved_steps passes payloads[i % 2]: feed each step's own
            def __getitem__(self, j):
                return payl[j]
        feed = _Feed()
        for i in range(steps):
            payl[i % 2] = pay(i)
            pipes[i % 2].step(feed[i % 2])
        for p in pipes:
            p.finish()
        inter = [pp[i % 2].history[i // 2] for i in range(steps)]
        good = len(ser.history) == len(ov.history) == steps
        good &= all(torch.equal(a, b) for a, b in zip(ser.history, ov.history))
        good &= all(torch.equal(a, b) for a, b in zip(ser.history, inter))
        good &= all(bool(h.any()) for h in ser.history) and ser.sm_rounds == ov.sm_rounds == 4
        # the state machine's group refuses to be the data group
        try:
            OverlapPipe(_FakeShardedBroadcast(rank, world, count), ex, _NoStream(), sm_ex=ex)
            good = False
        except ValueError:
            pass
        q.put((rank, "ok" if good else "mismatch %s / %s / %s" % (
            [h.tolist() for h in ser.history], [h.tolist() for h in ov.history],
            [h.tolist() for h in inter])))
    except Exception as e:  # pragma: no cover
        import traceback
        q.put((rank, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_overlapped_schedule_equals_serial(world):
    """the overlapped validator schedule at world > 1 --
    each step's state machine beside the next step's data plane, its
    per-round all-gathers over a process group of their own, and two such
    pipelines interleaved -- gives every step the same state-machine
    outputs as the serial schedule (data plane, then the rounds, step by
    step), on gloo over CPU with the kernels replaced by deterministic
    stand-ins that depend on every rank's data and records."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_gloo_schedule_worker, args=(r, world, port, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(60)
    assert res == {r: "ok" for r in range(world)}, res


# ------------------------------------------------------------------ GPU ----
def _payloads(seed, count, plen, dev):
    pay = np.stack([orc.gen_payload(seed, i, plen) for i in range(count)])
    t = torch.zeros((count, max(16, (plen + 15) // 16 * 16)), dtype=torch.uint8, device=dev)
    t[:, :plen] = torch.from_numpy(pay).to(dev)
    return pay, t


def run_loopback(n, world, count, plen, tamper=None, specialise=True):
    """One step of `world` virtual ranks in this process; the collectives are
    the loopback copies an all-to-all / all-gather would make."""
    ranks = [ShardedBroadcast(n, count, plen, r, world, device=0, specialise=specialise)
             for r in range(world)]
    pays = []
    for r, sb in enumerate(ranks):
        pay, t = _payloads(500 + r, count, plen, sb.device)
        pays.append(pay)
        sb.propose(t)
        sb.pack_value()
    if world == 1:
        ranks[0].exchange_value(SoloExchange())
    else:
        for d, dst in enumerate(ranks):           # Value all-to-all
            for s, src in enumerate(ranks):
                dst.recv_sh[s].copy_(src.slab[d])
                dst.recv_dg[s].copy_(src.send_dg[d])
                dst.roots_all[s].copy_(src.roots())
    if tamper:
        tamper(ranks)
    for sb in ranks:
        sb.validate_values()
    if world > 1:
        for dst in ranks:                         # Echo all-gather
            for v, src in enumerate(ranks):
                dst.echo_sh[v].copy_(src.recv_sh.view(dst.echo_sh[v].shape))
                dst.echo_dg[v].copy_(src.recv_dg.view(dst.echo_dg[v].shape))
                dst.okv_all[v].copy_(src.ok_pad)
    for sb in ranks:
        sb.validate_echoes()
        sb.decode()
    # the state machine of every validator, the virtual ranks' messages
    # all-gathered (loopback) each round
    from hbbft_amd.rbc_sim import run_rounds
    rounds = run_rounds([sb.sm for sb in ranks])
    for sb in ranks:
        sb.finish()
        sb.sm_rounds = rounds
    torch.cuda.synchronize()
    return ranks, pays


@pytest.mark.gpu
@pytest.mark.parametrize("n,world,count,plen", [(16, 2, 3, 5000), (10, 4, 2, 777), (64, 8, 2, 20000),
                                                (7, 3, 4, 100), (128, 4, 2, 6000), (64, 1, 3, 9000)])
def test_sharded_loopback_vs_oracle(n, world, count, plen):
    ranks, pays = run_loopback(n, world, count, plen)
    t = ranks[0].topo
    R = t.rpg
    for r, sb in enumerate(ranks):
        S = sb.S
        slab = sb.slab.cpu()
        nodes = sb.nodes.cpu().numpy()
        for i in range(count):
            sh, nd = orc.send_shards(n, t.f, pays[r][i].tobytes())
            for j in range(n):   # the encoder wrote the destination-major slab
                row = blocked_row(slab, j, i, R, S) if world > 1 else slab[0, i, j, :S]
                assert np.array_equal(row.numpy(), sh[j]), (r, i, j)
            assert np.array_equal(nodes[i], nd)
        assert sb.ok_v.cpu().numpy().all()             # every Value validates
        if sb.echo_rows:
            assert sb.ok_e.cpu().numpy()[:, : len(sb.echo_rows)].all()
        # the receiver saw exactly N - f Echoes and decoded every payload of every rank
        assert (sb.present.cpu().numpy().sum(axis=1) == n - t.f).all()
        assert (sb.status.cpu().numpy() == 0).all()
        assert (sb.plen_out.cpu().numpy() == plen).all()
        assert sb.decided.cpu().all()                    # Ready quorum and CanDecode met
        assert (sb.echo_senders.cpu().numpy() == n).all()
        assert (sb.full_echos.cpu().numpy() == n - t.f).all()
        out = sb.out.cpu().numpy()
        dn = sb.dec_nodes.cpu().numpy()
        for s in range(world):
            for i in range(count):
                assert np.array_equal(out[s * count + i, :plen], pays[s][i])
                # the decode tree (reused leaves + rebuilt rows) is the proposer's tree
                assert np.array_equal(dn[s * count + i], ranks[s].nodes[i].cpu().numpy())


@pytest.mark.gpu
def test_sharded_generic_decoder_matches_specialised():
    """The pattern-specialised decoder and the generic kernel give the same bytes."""
    a, pa = run_loopback(16, 2, 2, 3000, specialise=True)
    b, pb = run_loopback(16, 2, 2, 3000, specialise=False)
    for x, y in zip(a, b):
        assert torch.equal(x.echo_sh, y.echo_sh)
        assert torch.equal(x.out, y.out)


@pytest.mark.gpu
def test_sharded_faulty_rows():
    """A shard corrupted in transit fails its Value validation, so that
    validator sends no Echo (broadcast.rs:254-256) and every receiver's Echo
    validation of it fails too; receivers still decode from the rest, and with
    too few rows left report TooFewShardsPresent."""
    n, world, count, plen = 16, 2, 2, 3000
    f = (n - 1) // 3   # 5; receivers 0 and 8 miss 1..5 and 9..13

    def tamper(ranks):
        # instance 0 of rank 1: validator 6 (rank 0) gets a corrupted row
        ranks[0].recv_sh[1, 0, 6, 5] ^= 0x40
        # instance 1 of rank 1: validators 0..7 all corrupted -> receiver 8 keeps 3 < k = 6
        for r in range(8):
            ranks[0].recv_sh[1, 1, r, 0] ^= 1

    ranks, pays = run_loopback(n, world, count, plen, tamper)
    ok = ranks[0].ok_v.cpu().numpy()          # [G*C][R]: instance (1, i) = row 2 + i
    assert ok[2, 6] == 0 and ok[2, :6].all() and ok[2, 7]
    assert not ok[3].any()
    for sb in ranks:
        pres = sb.present.cpu().numpy()
        assert pres[2, 6] == 0
    st0, st1 = ranks[0].status.cpu().numpy(), ranks[1].status.cpu().numpy()
    assert (st0 == 0).all()                   # receiver 0 keeps rows 8..15 of instance (1, 1)
    assert st1[2] == 0 and st1[3] == 10       # receiver 8: 16 - 5 - 8 = 3 rows of (1, 1)
    for sb in ranks:
        assert np.array_equal(sb.out.cpu().numpy()[2, :plen], pays[1][0])
    assert not ranks[1].out.cpu().numpy()[3].any()   # a failed instance's row is all zero
    # the state machine's thresholds: instance (1, 1) has 8 < N - f = 11 Echo
    # senders, so no Ready quorum forms and no node decides it, although
    # receiver 0 could rebuild it; instance (1, 0) keeps 15 senders
    for sb in ranks:
        assert sb.echo_senders.cpu().tolist() == [16, 16, 15, 8]
        assert sb.decided.cpu().tolist() == [True, True, True, False]


@pytest.mark.gpu
def test_sharded_single_rank_step():
    n, count, plen = 64, 4, 11916 * 22 - 4
    sb = ShardedBroadcast(n, count, plen, 0, 1, device=0)
    pay, t = _payloads(9, count, plen, sb.device)
    sb.step(t, SoloExchange())
    torch.cuda.synchronize()
    assert (sb.status.cpu().numpy() == 0).all()
    assert np.array_equal(sb.out.cpu().numpy()[:, :plen], pay)


@pytest.mark.gpu
def test_sharded_overlapped_and_interleaved_steps():
    """The one-rank schedules the bench runs: each step's state machine on a
    side stream beside the next step's data plane (two state-machine slots),
    and two such step pipelines side by side on their own streams.  Every
    object decodes its own payloads and every instance is decided."""
    from hbbft_amd.sharded import OverlapPipe, interleaved_steps, overlapped_steps
    n, count, plen = 64, 4, 11916 * 22 - 4
    sb = ShardedBroadcast(n, count, plen, 0, 1, device=0, sm_slots=2)
    pay, t = _payloads(21, count, plen, sb.device)
    timing = []
    overlapped_steps(sb, t, SoloExchange(), 3, torch.cuda.Stream(sb.device), timing)
    torch.cuda.synchronize()
    assert len(timing) == 3 and sb.sm_rounds > 0
    assert (sb.status.cpu().numpy() == 0).all() and sb.decided.cpu().all()
    assert np.array_equal(sb.out.cpu().numpy()[:, :plen], pay)
    objs = [ShardedBroadcast(n, count, plen, 0, 1, device=0, sm_slots=2) for _ in range(2)]
    pays = [_payloads(40 + i, count, plen, objs[i].device) for i in range(2)]
    pipes = [OverlapPipe(o, SoloExchange(), torch.cuda.Stream(o.device), main=torch.cuda.Stream(o.device))
             for o in objs]
    interleaved_steps(pipes, [p[1] for p in pays], 5)   # pipe 0: steps 0, 2, 4; pipe 1: 1, 3
    torch.cuda.synchronize()
    assert [p.steps for p in pipes] == [3, 2]
    for o, (p, _) in zip(objs, pays):
        assert (o.status.cpu().numpy() == 0).all() and o.decided.cpu().all()
        assert np.array_equal(o.out.cpu().numpy()[:, :plen], p)


def _gloo_gpu_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n, count, plen = 16, 3, 4000
        sb = ShardedBroadcast(n, count, plen, rank, world, device=0)
        pay, t = _payloads(700 + rank, count, plen, sb.device)
        sb.step(t, DistExchange())
        torch.cuda.synchronize()
        allpay = [_payloads(700 + s, count, plen, sb.device)[0] for s in range(world)]
        out = sb.out.cpu().numpy()
        good = bool((sb.status.cpu() == 0).all()) and all(
            np.array_equal(out[s * count:(s + 1) * count, :plen], allpay[s]) for s in range(world))
        # the pipelined schedule over two sub-batches gives the same result
        subs = [ShardedBroadcast(n, 2, plen, rank, world, device=0) for _ in range(2)]
        pays = [_payloads(800 + 10 * i + rank, 2, plen, subs[i].device) for i in range(2)]
        timer = CommTimer(subs[0].device)
        timer.timing = True
        pipelined_step(subs, [p[1] for p in pays], DistExchange(), timer)
        torch.cuda.synchronize()
        for i, sub in enumerate(subs):
            o = sub.out.cpu().numpy()
            for s in range(world):
                exp = _payloads(800 + 10 * i + s, 2, plen, sub.device)[0]
                good = good and np.array_equal(o[2 * s:2 * s + 2, :plen], exp)
            good = good and bool((sub.status.cpu() == 0).all())
        good = good and len(timer.spans) == 4 and timer.elapsed_ms() > 0
        # the overlapped schedule the bench runs at every world size: two step
        # pipelines, each step's state machine on a side stream beside the
        # next step's data plane, its all-gathers over a group of their own;
        # same payloads as the serial step above -> same outputs and flags
        from hbbft_amd.sharded import OverlapPipe, interleaved_steps
        sm_ex = DistExchange(dist.new_group(list(range(world))))
        objs = [ShardedBroadcast(n, count, plen, rank, world, device=0, sm_slots=2)
                for _ in range(2)]
        xs = []
        pipes = [OverlapPipe(o, DistExchange(), torch.cuda.Stream(o.device),
                             main=torch.cuda.Stream(o.device), sm_ex=sm_ex, xspans=xs)
                 for o in objs]
        interleaved_steps(pipes, [t, t], 5)   # pipe 0: steps 0, 2, 4; pipe 1: 1, 3
        torch.cuda.synchronize()
        good = good and [p.steps for p in pipes] == [3, 2] and len(xs) == 2 * 5
        for o in objs:
            oo = o.out.cpu().numpy()
            good = good and bool((o.status.cpu() == 0).all()) and bool(o.decided.cpu().all())
            good = good and torch.equal(o.decided.cpu(), sb.decided.cpu())
            good = good and o.sm_rounds == sb.sm_rounds
            good = good and all(np.array_equal(oo[s * count:(s + 1) * count, :plen], allpay[s])
                                for s in range(world))
        q.put((rank, "ok" if good else "mismatch %s" % sb.status.cpu().tolist()))
    except Exception as e:  # pragma: no cover
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_sharded_two_ranks_gloo_on_one_gpu():
    """Two ranks sharing cuda:0 over gloo: the serial step, the sub-batch
    pipelined step, and the overlapped two-pipeline schedule (state machine
    on its own process group), all against every rank's payloads."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_gloo_gpu_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=200) for _ in procs)
    for p in procs:
        p.join(60)
    assert res == {0: "ok", 1: "ok"}, res


def test_loop_exchange_issues_one_rank_collectives(tmp_path):
    """DistExchange(loop=True) on a one-rank group calls the collectives (and
    counts them) instead of copying; the default copies (CPU, gloo)."""
    import torch.distributed as dist
    store = dist.FileStore(str(tmp_path / "store"), 1)
    dist.init_process_group("gloo", store=store, rank=0, world_size=1)
    try:
        for loop in (False, True):
            ex = DistExchange(loop=loop)
            inp = torch.arange(2 * 3 * 5, dtype=torch.uint8).view(1, 6, 5)
            out = torch.zeros_like(inp)
            ex.all_to_all(out, inp, name="a2a")
            assert torch.equal(out, inp)
            got = torch.zeros((1, 30), dtype=torch.uint8)
            h = ex.all_gather(got, inp.view(-1), async_op=loop, name="ag")
            if h is not None:
                h.wait()
            assert torch.equal(got.view(-1), inp.view(-1))
            assert sorted(ex.stats) == (["a2a", "ag"] if loop else [])
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_rccl_one_rank_calls():
    """Every collective call of the multi-GPU bench (Value all-to-all, Echo
    all-gather, async handles waited on CommTimer's side stream, the state
    machine's own communicator, the agreement / max-over-ranks all-reduces,
    all_gather_object, barrier) on a one-rank RCCL group on the box's GPU
    (tests/rccl_one_rank.py): the RCCL side of the calls the gloo tests run
    multi-rank."""
    import subprocess
    import sys
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), RANK="0",
               LOCAL_RANK="0", WORLD_SIZE="1", LOCAL_WORLD_SIZE="1")
    script = os.path.join(os.path.dirname(os.path.abspath(__file__)), "rccl_one_rank.py")
    r = subprocess.run([sys.executable, "-u", script], env=env, capture_output=True, text=True,
                       timeout=150)
    assert r.returncode == 0 and "rccl one-rank: ok" in r.stdout, (r.returncode, r.stdout[-2000:],
                                                                   r.stderr[-4000:])


# ----------------------------------------------------------- HBM footprint --
BENCH_OBJECTS = [("cfg3", 64, 256 << 10, 8192), ("cfg4", 128, 256 << 10, 4096)]


@pytest.mark.parametrize("cfg,n,plen,count", BENCH_OBJECTS)
def test_rank_footprint_fits_hbm(cfg, n, plen, count):
    """Every rank of the bench's validator-sharded objects fits one MI355X
    (288 GB) at 1, 2, 4 and 8 GPUs: echo slab [G][G*C][R][stride], proposer
    slab, decode trees, state machine inboxes [G][G*C][R][E][1+W] and the
    library's reconstruct workspace (upper bound)."""
    from hbbft_amd.sharded import HBM_PER_GPU, rank_footprint
    prev = 0
    for world in (1, 2, 4, 8):
        for rank in (0, world - 1):
            fp = rank_footprint(n, count, plen, world, rank)
            assert fp["total_bytes"] < HBM_PER_GPU, (cfg, world, rank, fp["total_bytes"])
            assert all(v > 0 for v in fp["buffers"].values())
            # the bench's schedule at every world size: two step pipelines,
            # each with two state-machine slots
            fp2 = rank_footprint(n, count, plen, world, rank, sm_slots=2)
            assert fp2["total_bytes"] > fp["total_bytes"]
            assert 2 * fp2["total_bytes"] < HBM_PER_GPU, (cfg, world, rank, fp2["total_bytes"])
        # the all-gathered echo slab grows with the world (every rank decodes all)
        assert fp["torch_bytes"] > prev
        prev = fp["torch_bytes"]
    fp8 = rank_footprint(n, count, plen, 8, 0)
    # the G=8 echo slab dominates: G * G*C * R * stride bytes
    R = -(-n // 8)
    assert fp8["buffers"]["echo_sh"] == 8 * 8 * count * R * ((-(-(plen + 4) // (n - 2 * ((n - 1) // 3))) + 15) // 16 * 16)


@pytest.mark.gpu
@pytest.mark.parametrize("n,world,count,plen", [(64, 1, 64, 50000), (64, 8, 16, 50000),
                                                (128, 4, 16, 30000)])
def test_rank_footprint_matches_allocation(n, world, count, plen):
    """rank_footprint's torch buffers equal what ShardedBroadcast allocates
    (torch.cuda.memory_allocated delta; ranks of a larger world can be built
    on one GPU -- no collective runs)."""
    import torch

    from hbbft_amd.sharded import ShardedBroadcast, rank_footprint

    def requested():
        # bytes the tensors asked for (before the caching allocator rounds
        # them up or hands out a whole unsplit segment tail)
        return torch.cuda.memory_stats(0).get("requested_bytes.all.current")

    torch.cuda.synchronize()
    before = requested()
    sb = ShardedBroadcast(n, count, plen, 0, world, device=0, specialise=False)
    torch.cuda.synchronize()
    got = requested() - before
    want = rank_footprint(n, count, plen, world, 0)["torch_bytes"]
    assert got == want, (got, want, got - want)
    del sb
