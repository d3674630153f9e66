"""One-rank RCCL run of every collective call the multi-GPU bench makes.

The validator-sharded objects exchange shards over RCCL at world > 1, which
only the driver's 8-GPU node has; every multi-rank test here runs gloo.  This
script runs the same calls, with the same arguments, on a one-rank "nccl"
(= RCCL) process group on the test box's one GPU, so the RCCL side of them --
process-group creation with `device_id` and a timeout, device tensors in
`all_to_all_single` / `all_gather_into_tensor`, the async handles' `wait()`
on a side stream (`CommTimer`), a second communicator on its own stream
(`bench.sm_exchange`, the overlapped schedule), the device-tensor MIN / MAX
all-reduces of `bench.Phases.agree` / `bench.max_over_ranks`,
`all_gather_object`, `barrier` and teardown -- has run at least once before
the 8-GPU run.  What one rank cannot show (ordering across ranks, xGMI
bandwidth) stays with that run.  Prints "rccl one-rank: ok" on success.

Run by tests/test_sharded.py::test_rccl_one_rank_calls (GPU) as
    MASTER_ADDR=127.0.0.1 MASTER_PORT=<port> RANK=0 WORLD_SIZE=1 \
        python tests/rccl_one_rank.py
"""
import datetime
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import torch.distributed as dist

    import bench
    from hbbft_amd.sharded import CommTimer, DistExchange

    assert torch.cuda.is_available(), "needs a GPU"
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    bench.PG_TIMEOUT[0] = datetime.timedelta(seconds=60)
    # bench.main's call at world > 1
    dist.init_process_group("nccl", device_id=dev, timeout=bench.PG_TIMEOUT[0])
    assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
    g = torch.Generator(device=dev)
    g.manual_seed(0x48424246)

    def rnd(*shape):
        return torch.randint(0, 256, shape, dtype=torch.uint8, device=dev, generator=g)

    ex = DistExchange(loop=True)
    assert ex.backend == "nccl" and not ex.staged
    G, C, R, stride, dsz = 1, 3, 16, 11920, 6 * 32 + 16
    # Value exchange (ShardedBroadcast.exchange_value): slab [G][C][R][stride],
    # digests [G][C][R][dsz], roots [C][32] -> [G][C][32]; synchronous form
    slab, recv = rnd(G, C, R, stride), torch.empty((G, C, R, stride), dtype=torch.uint8,
                                                   device=dev)
    assert ex.all_to_all(recv, slab, name="value_shards") is None
    assert torch.equal(recv, slab)
    roots, roots_all = rnd(C, 32), torch.empty((G, C, 32), dtype=torch.uint8, device=dev)
    ex.all_gather(roots_all, roots, name="roots")
    assert torch.equal(roots_all[0], roots)
    # the serial schedule's form (pipelined_step): async handles waited on a
    # side stream (CommTimer), the compute stream waits for its event
    timer = CommTimer(dev)
    timer.timing = True
    for _ in range(3):
        slab = rnd(G, C, R, stride)
        dg = rnd(G, C, R, dsz)
        roots = rnd(C, 32)
        slab.add_(1)   # a kernel on the compute stream the exchange must follow
        r_sh = torch.empty_like(slab)
        r_dg = torch.empty_like(dg)
        r_roots = torch.empty((G, C, 32), dtype=torch.uint8, device=dev)
        ev = timer.run(lambda: [ex.all_to_all(r_sh, slab, True, name="value_shards"),
                                ex.all_to_all(r_dg, dg, True, name="value_proofs"),
                                ex.all_gather(r_roots, roots, True, name="roots")])
        torch.cuda.current_stream(dev).wait_event(ev)
        # Echo all-gather into [G][G*C][R][stride] from [G*C][R][stride]
        e_sh = torch.empty((G, G * C, R, stride), dtype=torch.uint8, device=dev)
        ev = timer.run(lambda: [ex.all_gather(e_sh, r_sh.view(G * C, R, stride), True,
                                              name="echo_shards")])
        torch.cuda.current_stream(dev).wait_event(ev)
        assert torch.equal(r_sh, slab) and torch.equal(r_dg, dg)
        assert torch.equal(r_roots[0], roots) and torch.equal(e_sh.view(-1), slab.view(-1))
    torch.cuda.synchronize(dev)
    assert len(timer.spans) == 6 and timer.elapsed_ms() > 0
    assert ex.stats["value_shards"]["calls"] == 4
    # the overlapped schedule: the state machine's communicator (its own
    # process group, bench.sm_exchange) issuing on a side stream while the
    # data plane's group issues on the main stream
    sm = bench.sm_exchange()
    sm.loop = True
    side = torch.cuda.Stream(dev)
    inbox = rnd(4096, 64)
    gathered = torch.empty((1, 4096, 64), dtype=torch.uint8, device=dev)
    big, big_out = rnd(G, 8, R, stride), torch.empty((G, 8, R, stride), dtype=torch.uint8,
                                                     device=dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        h = sm.all_gather(gathered, inbox, True, name="sm_records")
        h.wait()
    w = ex.all_to_all(big_out, big, True, name="value_shards")
    w.wait()
    torch.cuda.synchronize(dev)
    assert torch.equal(gathered[0], inbox) and torch.equal(big_out, big)
    # Phases.agree (MIN) and max_over_ranks (MAX) as the multi-rank bench calls
    # them: device tensors on the nccl group (world passed as > 1 so neither
    # takes its one-rank shortcut)
    P = bench.Phases(2, 0, dev, 0, lambda res: None, False)
    assert P.agree(True) is True and P.agree(False) is False
    assert bench.max_over_ranks(1.25, 2, dev) == 1.25
    per_rank = [None]
    dist.all_gather_object(per_rank, {"rank": 0, "backend": ex.backend})
    assert per_rank == [{"rank": 0, "backend": "nccl"}]
    dist.barrier()
    dist.destroy_process_group()
    print("rccl one-rank: ok", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
