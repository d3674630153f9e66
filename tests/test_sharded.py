"""Validator-sharded simulation (hbbft_amd/sharded.py).

CPU (gloo, world 2): the topology, the destination-major regrouping and the
two all-to-alls move every shard row to the rank hosting its validator and
back.  GPU: G virtual ranks in one process (loopback exchange) run the whole
step through libhbrbc.so and are checked against the oracle; a 2-rank gloo
run shares cuda:0."""
import os
import socket

import numpy as np
import pytest
import torch

from hbbft_amd.sharded import (DistExchange, ShardedBroadcast, SoloExchange, Topology,
                               loopback_all_to_all, pack_rows, pipelined_step, unpack_rows)
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
    assert t.rpg == 3 and t.npad == 12
    assert [list(t.validators(r)) for r in range(4)] == [[0, 1, 2], [3, 4, 5], [6, 7, 8], [9]]
    assert t.proposers(3, 3) == [9, 9, 9] and t.proposers(1, 4) == [3, 4, 5, 3]
    with pytest.raises(ValueError):
        Topology(9, 4)   # the last rank would host no validator
    # receiver p misses Echoes from p+1..p+f (broadcast.rs:476-485), f = 3
    m = t.echo_received([0, 8]).numpy()
    assert m[0].tolist() == [1, 0, 0, 0, 1, 1, 1, 1, 1, 1]
    assert m[1].tolist() == [0, 0, 1, 1, 1, 1, 1, 1, 1, 0]   # 9, 0, 1 wrap around
    assert m.sum(axis=1).tolist() == [7, 7]


def test_pack_unpack_roundtrip():
    g = torch.Generator().manual_seed(1)
    slab = torch.randint(0, 256, (5, 12, 48), dtype=torch.uint8, generator=g)
    buf = torch.empty((4, 5, 3, 48), dtype=torch.uint8)
    pack_rows(slab, 4, 3, buf)
    for d in range(4):
        assert torch.equal(buf[d], slab[:, 3 * d: 3 * d + 3])
    back = torch.empty_like(slab)
    assert torch.equal(unpack_rows(buf, back), slab)


def _gloo_worker(rank, world, port, n, count, plen, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        t = Topology(n, world)
        ex = DistExchange()
        f = t.f
        S = orc.shard_len(plen, n - 2 * f)

        def slab_of(r):   # what rank r's proposer side holds (oracle shards)
            out = torch.zeros((count, t.npad, S), dtype=torch.uint8)
            for i in range(count):
                sh, _ = orc.send_shards(n, f, orc.gen_payload(100 + r, i, plen).tobytes())
                out[i, :n] = torch.from_numpy(sh)
            return out

        mine = slab_of(rank)
        send = pack_rows(mine, world, t.rpg, torch.empty((world, count, t.rpg, S), dtype=torch.uint8))
        recv = torch.empty_like(send)
        ex.all_to_all(recv, send)
        # Value: block s = this rank's validators' rows of rank s's instances
        for s in range(world):
            assert torch.equal(recv[s], slab_of(s)[:, rank * t.rpg:(rank + 1) * t.rpg])
        roots = torch.full((count, 32), rank, dtype=torch.uint8)
        allr = torch.empty((world, count, 32), dtype=torch.uint8)
        ex.all_gather(allr, roots)
        assert [int(allr[s, 0, 0]) for s in range(world)] == list(range(world))
        # Echo back to the proposer's rank, then regroup = the original slab
        echo = torch.empty_like(recv)
        ex.all_to_all(echo, recv)
        assert torch.equal(unpack_rows(echo, torch.empty_like(mine)), mine)
        q.put((rank, "ok"))
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n,world", [(10, 2), (16, 2), (7, 3)])
def test_gloo_value_and_echo_exchange(n, world):
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


# ------------------------------------------------------------------ GPU ----
def _payloads(seed, count, plen, dev):
    pay = np.stack([orc.gen_payload(seed, i, plen) for i in range(count)])
    t = torch.zeros((count, max(16, (plen + 15) // 16 * 16)), dtype=torch.uint8, device=dev)
    t[:, :plen] = torch.from_numpy(pay).to(dev)
    return pay, t


def run_loopback(n, world, count, plen, tamper=None):
    ranks = [ShardedBroadcast(n, count, plen, r, world, device=0) for r in range(world)]
    pays = []
    for r, sb in enumerate(ranks):
        pay, t = _payloads(500 + r, count, plen, sb.device)
        pays.append(pay)
        sb.propose(t)
        sb.pack_value()
    loopback_all_to_all([sb.recv_sh for sb in ranks], [sb.send_sh for sb in ranks])
    loopback_all_to_all([sb.recv_dg for sb in ranks], [sb.send_dg for sb in ranks])
    for sb in ranks:
        for s, src in enumerate(ranks):
            sb.roots_all[s].copy_(src.roots())
    if tamper:
        tamper(ranks)
    for sb in ranks:
        sb.validate_values()
    loopback_all_to_all([sb.echo_sh for sb in ranks], [sb.recv_sh for sb in ranks])
    loopback_all_to_all([sb.echo_ok for sb in ranks], [sb.ok_v for sb in ranks])
    for sb in ranks:
        sb.decode()
    torch.cuda.synchronize()
    return ranks, pays


@pytest.mark.gpu
@pytest.mark.parametrize("n,world,count,plen", [(16, 2, 3, 5000), (10, 4, 2, 777), (64, 8, 2, 20000),
                                                (7, 3, 4, 100), (128, 4, 2, 6000)])
def test_sharded_loopback_vs_oracle(n, world, count, plen):
    ranks, pays = run_loopback(n, world, count, plen)
    t = ranks[0].topo
    for r, sb in enumerate(ranks):
        S = sb.S
        slab = sb.slab.cpu().numpy()
        nodes = sb.nodes.cpu().numpy()
        for i in range(count):
            sh, nd = orc.send_shards(n, t.f, pays[r][i].tobytes())
            assert np.array_equal(slab[i, :n, :S], sh)
            assert np.array_equal(nodes[i], nd)
        # every real row this rank validated is valid
        ok = sb.ok_v.cpu().numpy()
        real = len(t.validators(r))
        assert ok[:, :, :real].all()
        # the receiver saw exactly N - f Echoes and decoded every payload
        assert (sb.present.cpu().numpy().sum(axis=1) == n - t.f).all()
        assert (sb.status.cpu().numpy() == 0).all()
        assert (sb.plen_out.cpu().numpy() == plen).all()
        assert np.array_equal(sb.out.cpu().numpy()[:, :plen], pays[r])
        assert np.array_equal(sb.nodes2.cpu().numpy(), nodes)


@pytest.mark.gpu
def test_sharded_faulty_rows():
    """A shard corrupted in transit fails its Value validation, so that
    validator sends no Echo; the receiver still decodes from the rest, and
    with more than f missing it reports TooFewShardsPresent."""
    n, world, count, plen = 16, 2, 2, 3000
    f = (n - 1) // 3

    def tamper(ranks):
        # rank 0 hosts validators 0..7; instance 0 of rank 1 (proposer 8):
        # corrupt validator 0's row -> 1 more missing row (f + 1 total)
        ranks[0].recv_sh[1, 0, 0, 5] ^= 0x40
        # instance 1 of rank 1 (proposer 9): corrupt f + 1 more rows -> too few
        for r in range(f + 1):
            ranks[0].recv_sh[1, 1, r, 0] ^= 1

    ranks, pays = run_loopback(n, world, count, plen, tamper)
    ok = ranks[0].ok_v.cpu().numpy()
    assert ok[1, 0, 0] == 0 and ok[1, 0, 1:].all()
    assert not ok[1, 1, : f + 1].any()
    st = ranks[1].status.cpu().numpy()
    assert st[0] == 0 and st[1] == 10
    assert np.array_equal(ranks[1].out.cpu().numpy()[0, :plen], pays[1][0])
    assert (ranks[0].status.cpu().numpy() == 0).all()


@pytest.mark.gpu
def test_sharded_single_rank_step():
    n, count, plen = 64, 4, 11916 * 22 - 4
    sb = ShardedBroadcast(n, count, plen, 0, 1, device=0)
    pay, t = _payloads(9, count, plen, sb.device)
    sb.step(t, SoloExchange())
    torch.cuda.synchronize()
    assert (sb.status.cpu().numpy() == 0).all()
    assert np.array_equal(sb.out.cpu().numpy()[:, :plen], pay)


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
        good = bool((sb.status.cpu() == 0).all()) and \
            np.array_equal(sb.out.cpu().numpy()[:, :plen], pay)
        # the pipelined schedule over two sub-batches gives the same result
        subs = [ShardedBroadcast(n, 2, plen, rank, world, device=0) for _ in range(2)]
        pays = [_payloads(800 + 10 * i + rank, 2, plen, subs[i].device) for i in range(2)]
        pipelined_step(subs, [p[1] for p in pays], DistExchange())
        torch.cuda.synchronize()
        for sub, (pp, _) in zip(subs, pays):
            good = good and bool((sub.status.cpu() == 0).all()) and \
                np.array_equal(sub.out.cpu().numpy()[:, :plen], pp)
        q.put((rank, "ok" if good else "mismatch %s" % sb.status.cpu().tolist()))
    except Exception as e:  # pragma: no cover
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_sharded_two_ranks_gloo_on_one_gpu():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_gloo_gpu_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=100) for _ in procs)
    for p in procs:
        p.join(60)
    assert res == {0: "ok", 1: "ok"}, res
