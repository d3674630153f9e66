#!/usr/bin/env python3
"""Benchmark: hbbft Reliable-Broadcast data path on MI355X.

One step = the whole RBC data path over one batch of `count` independent
broadcast instances already resident in HBM:
  frame (broadcast.rs:174-189) -> RS encode (193) -> Merkle tree (204) ->
  N proofs (212-222) -> validate all N proofs (254/291, merkle.rs:83-103) ->
  decode_from_shards with f random erasures per instance (563-601: decode
  matrix + reconstruct, re-tree, root compare, unframe).
value = payload bytes of every instance on every rank / max-over-ranks wall
time of the K timed steps (GB/s, 1e9).  Multi-GPU: instances are sharded
across ranks with no data-path collective (weak scaling).
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
VALU_PEAK_OPS = 78.6e12        # 256 CU x 4 SIMD x 32 lanes x 2.4 GHz (32-bit lane-ops/s)
KECCAK_OPS_PER_PERM = 4320     # ~180 VALU ops/round x 24 rounds
# measured ceiling of the Keccak-f[1600] round code itself (register-only loop,
# 4 waves/SIMD, profiles/r1_valu_microbench.txt): v_alignbit issues at half rate
KECCAK_CEILING_PERMS = 10.48e9

CONFIGS = {
    # name: (N, payload bytes, instances per GPU, erasures)
    "cfg2": (16, 1 << 20, 4096, "f"),
    "cfg3": (64, 256 << 10, 16384, "f"),
    "cfg4": (128, 256 << 10, 8192, "f"),
    "cfg5": (250, 4 << 20, 1024, "worst"),
}
METRIC = "RBC encode+Merkle+decode payload GB/s, N=64, 1/8 GPUs; fraction of HBM peak"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="cfg3", choices=sorted(CONFIGS))
    ap.add_argument("--count", type=int, default=0, help="instances per GPU (default: config)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--streams", type=int, default=1,
                    help="sub-batches per step, each on its own HIP stream (overlap)")
    ap.add_argument("--own-streams", action="store_true",
                    help="run each sub-batch on its context's own HIP stream")
    ap.add_argument("--mode", choices=["instances", "validators"], default=None,
                    help="instances: every rank runs whole instances, no collective (default "
                         "except cfg4); validators: simulated validators sharded over the ranks, "
                         "Value/Echo exchanged by all-to-all (hbbft_amd/sharded.py; default for cfg4)")
    return ap.parse_args()


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    import hbbft_amd as hb

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("HBRBC_BENCH_REHEARSE") == "1":
        # multi-rank rehearsal on a box with fewer GPUs than ranks: gloo, ranks
        # share the visible devices (the real N > 1 runs use RCCL, one GPU each)
        local = local % torch.cuda.device_count()
        if world > 1:
            torch.cuda.set_device(local)
            dist.init_process_group("gloo")
    elif world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    n, plen, count, erase = CONFIGS[args.config]
    if args.count:
        count = args.count
    mode = args.mode or ("validators" if args.config == "cfg4" else "instances")
    if mode == "validators":
        return run_validators(args, n, plen, count, rank, world, local, dev)
    nsub = max(1, min(args.streams, count))
    f = (n - 1) // 3
    # one Coding context per sub-batch: each owns its reconstruct workspace
    subs_rb = [hb.RbcBatch(n, f, device=local) for _ in range(nsub)]
    rb = subs_rb[0]
    k, m = rb.k, rb.m
    S = hb.shard_len(plen, k)
    stride = rb.stride_for(S)
    n_erase = f if erase == "f" else m

    # ---- inputs resident in HBM before timing ---------------------------
    g = torch.Generator(device=dev)
    g.manual_seed(0x48424246 + rank)
    pstride = (plen + 15) // 16 * 16
    payloads = torch.randint(0, 256, (count, pstride), dtype=torch.uint8, device=dev, generator=g)
    if erase == "f":
        order = torch.rand((count, n), device=dev, generator=g).argsort(dim=1)
        present = torch.ones((count, n), dtype=torch.uint8, device=dev)
        present.scatter_(1, order[:, :n_erase], 0)
    else:  # worst case: only the first k parity shards survive
        present = torch.zeros((count, n), dtype=torch.uint8, device=dev)
        present[:, k:2 * k] = 1
    slab = torch.empty((count, n, stride), dtype=torch.uint8, device=dev)
    nodes = torch.empty((count, rb.node_count, 32), dtype=torch.uint8, device=dev)
    nodes2 = torch.empty_like(nodes)
    roots = torch.empty((count, 32), dtype=torch.uint8, device=dev)
    ds = max(rb.dslots, 1)
    digests = torch.empty((count, n, ds, 32), dtype=torch.uint8, device=dev)
    ndig = torch.empty((count, n), dtype=torch.uint8, device=dev)
    ok = torch.empty((count, n), dtype=torch.uint8, device=dev)
    ostride = (k * S + 15) // 16 * 16
    out = torch.empty((count, ostride), dtype=torch.uint8, device=dev)
    plen_out = torch.empty(count, dtype=torch.int32, device=dev)
    status = torch.empty(count, dtype=torch.int32, device=dev)

    # sub-batches: contiguous instance ranges, one stream each, so one
    # sub-batch's VALU-bound hashing overlaps another's HBM-bound copies and
    # the grid tails of every stage fill (the work per step is unchanged)
    bounds = [(i * count) // nsub for i in range(nsub + 1)]
    main = torch.cuda.current_stream(dev)
    subs = []
    for i in range(nsub):
        lo, hi = bounds[i], bounds[i + 1]
        sb = subs_rb[i]
        sb.reserve(hi - lo)
        subs.append((sb, (sb.own_stream() if args.own_streams else torch.cuda.Stream(dev))
                     if nsub > 1 else main, slice(lo, hi)))

    def run_sub(sb, sl):
        sb.frame_encode(payloads[sl], plen, slab[sl])   # frame folded into the encoder
        sb.merkle(slab[sl], S, nodes[sl])
        sb.proofs(nodes[sl], digests[sl], ndig[sl])
        sb.validate(slab[sl], S, digests[sl], ndig[sl], nodes[sl], ok[sl])
        roots[sl].copy_(nodes[sl, -1, :])      # what the Echo/Ready quorum agreed on
        sb.decode(slab[sl], S, present[sl], roots[sl], nodes2[sl], out[sl], plen_out[sl],
                  status[sl])

    # Sub-batch streams are joined only where the host synchronises (after the
    # warm-up and after the timed steps): each stream runs its own sub-batch
    # step after step, ordered by the stream alone.  After every join the
    # streams are re-staggered by one stage (stream i starts once stream i-1
    # has finished its frame+encode), so one sub-batch's HBM-bound stages run
    # beside another's VALU-bound Keccak instead of in lockstep with it.
    restagger = [True]

    def step():
        if nsub == 1:
            run_sub(subs[0][0], subs[0][2])
            return
        first = restagger[0]
        restagger[0] = False
        ev = None
        if first:
            ev = torch.cuda.Event()
            ev.record(main)
        for sb, st, sl in subs:
            if first:
                st.wait_event(ev)
            with torch.cuda.stream(st):
                sb.frame_encode(payloads[sl], plen, slab[sl])
                if first:
                    ev = torch.cuda.Event()
                    ev.record(st)
                sb.merkle(slab[sl], S, nodes[sl])
                sb.proofs(nodes[sl], digests[sl], ndig[sl])
                sb.validate(slab[sl], S, digests[sl], ndig[sl], nodes[sl], ok[sl])
                roots[sl].copy_(nodes[sl, -1, :])
                sb.decode(slab[sl], S, present[sl], roots[sl], nodes2[sl], out[sl],
                          plen_out[sl], status[sl])

    def join():
        torch.cuda.synchronize(dev)
        restagger[0] = True

    for _ in range(args.warmup):
        step()
    join()
    if not args.no_verify:
        assert bool((ok == 1).all()), "a valid proof was rejected"
        assert bool((status == 0).all()), "decode failed"
        assert bool((plen_out == plen).all())
        assert torch.equal(out[:, :plen], payloads[:, :plen]), "decoded payload differs"

    for sb in subs_rb:
        sb.profile(True)
        sb.profile_reset()
    if world > 1:
        dist.barrier()
    join()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    join()
    t1 = time.perf_counter()
    for sb in subs_rb:
        sb.profile(False)
    elapsed = t1 - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        dist.barrier()
    stages = {}
    for sb in subs_rb:
        for st_name, (ms, cnt) in sb.profile_read().items():
            a0, c0 = stages.get(st_name, (0.0, 0))
            stages[st_name] = (a0 + ms, c0 + cnt)

    total_payload = float(count) * plen * world * args.steps
    value = total_payload / elapsed / 1e9
    per_launch = count / nsub          # instances processed by one launch

    # ---- roofline of the dominant kernel (per launch, live HIP events) ---
    L = (S + 1 + 135) // 136  # Keccak blocks per leaf (S bytes + pad)
    # algorithmic bytes per launch (SURVEY 8d per-instance figures x instances per launch)
    alg_bytes = {s_: per_launch * v_ for s_, v_ in {
        "frame": plen + k * S,
        # frame folded into the specialised encoder: the encode launch also reads the payload
        "encode": (k + m) * S + (plen if stages.get("frame", (0.0, 0))[1] == 0 else 0),
        "leaf_hash": n * (S + 32),
        "tree_levels": (rb.node_count - n) * 96,   # one record = all levels of one tree batch
        "proofs": n * rb.dslots * 32 * 2 + n,
        "validate": n * (S + 32 * (rb.dslots + 1) + 1),
        "decode_matrix": n + m * k * 16,
        "reconstruct": (k + n_erase) * S,
        "unframe": k * S + plen,
    }.items()}
    dom = max(stages, key=lambda s: stages[s][0])
    dom_ms, dom_launches = stages[dom]
    per_launch_s = dom_ms / 1e3 / max(dom_launches, 1)
    achieved = alg_bytes[dom] / per_launch_s / 1e9 if per_launch_s > 0 else 0.0
    perms = {"leaf_hash": per_launch * n * L, "validate": per_launch * (n * L + n * rb.dslots),
             "tree_levels": per_launch * (n - 1)}
    valu = None
    if dom in perms:
        ops = perms[dom] * KECCAK_OPS_PER_PERM / per_launch_s
        pps = perms[dom] / per_launch_s
        valu = {"achieved_ops": ops, "peak_ops": VALU_PEAK_OPS, "frac": ops / VALU_PEAK_OPS,
                "ops_per_perm": KECCAK_OPS_PER_PERM, "perms_per_launch": perms[dom],
                "perms_per_s": pps, "measured_ceiling_perms_per_s": KECCAK_CEILING_PERMS,
                "frac_of_measured_ceiling": pps / KECCAK_CEILING_PERMS}
    step_bytes = sum(alg_bytes[s] * (stages[s][1] / max(args.steps, 1)) for s in stages)
    roofline = {
        "kernel": dom, "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": achieved / HBM_PEAK_GBS, "traffic": None, "launch_ms": per_launch_s * 1e3,
        "valu": valu,
        "pipeline_alg_bytes_per_step": step_bytes,
        "pipeline_hbm_frac": step_bytes / (elapsed / args.steps) / 1e9 / HBM_PEAK_GBS,
    }
    prof = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(prof):
        try:
            pm = json.load(open(prof)).get("traffic", {})
            key = "%s:%s" % (args.config, dom)
            if key in pm:   # HBM bytes per instance from the PMC pass x instances per launch
                roofline["traffic"] = pm[key] * per_launch
        except Exception:
            pass

    # ---- CPU baseline: the oracle (reference algorithm) on host cores -----
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        from oracle import pyoracle as orc
        threads = max(1, min(16, len(os.sched_getaffinity(0))))
        orc.build()
        cal = max(threads, 2)
        t_cal, ok_cal = orc.bench_pipeline(n, f, plen, cal, n_erase, 1, threads)
        sample = int(max(cal, min(4096, args.cpu_seconds / max(t_cal, 1e-6) * cal)))
        t_cpu, ok_cpu = orc.bench_pipeline(n, f, plen, sample, n_erase, 2, threads)
        cpu = {"value": sample * plen / t_cpu / 1e9, "unit": "GB/s", "cores": threads,
               "kind": "port",
               "sample": "%d instances of %s (N=%d, %d B payload) through the same pipeline in "
                         "oracle/rbc_oracle.c on %d pthreads, %.1f s, %d/%d decoded ok"
                         % (sample, args.config, n, plen, threads, t_cpu, ok_cpu, sample)}

    if rank == 0:
        line = {
            "metric": METRIC, "value": value, "unit": "GB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (uniform random payloads resident in HBM; random erasures)",
            "config": {"workload": "%s: N=%d f=%d (%d+%d shards), %d B payloads, %d instances/GPU, "
                                   "%s erasures" % (args.config, n, f, k, m, plen, count,
                                                    "f random" if erase == "f" else "worst-case"),
                       "n": n, "f": f, "payload_bytes": plen, "shard_len": S,
                       "instances_per_gpu": count, "global_batch": count * world,
                       "parallelism": "instance-sharded x%d" % world,
                       "streams_per_gpu": nsub},
            "roofline": roofline, "cpu_baseline": cpu,
            "stages_ms_per_step": {s: stages[s][0] / args.steps for s in stages},
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def run_validators(args, n, plen, count, rank, world, local, dev):
    """Validator-sharded simulation: each rank proposes `count`
    instances and hosts N/world validators; Value and Echo rows cross ranks
    in two all-to-alls (RCCL over xGMI), roots in an all-gather."""
    import torch
    import torch.distributed as dist

    from hbbft_amd.sharded import DistExchange, ShardedBroadcast, SoloExchange, pipelined_step

    # more than one rank: 4 pipelined sub-batches unless --streams says otherwise
    nsub = max(1, min(args.streams if args.streams > 1 else 4, count)) if world > 1 else 1
    bounds = [(i * count) // nsub for i in range(nsub + 1)]
    subs = [ShardedBroadcast(n, bounds[i + 1] - bounds[i], plen, rank, world, device=local)
            for i in range(nsub)]
    sb = subs[0]
    ex = DistExchange() if world > 1 else SoloExchange()
    g = torch.Generator(device=dev)
    g.manual_seed(0x48424246 + rank)
    pstride = (plen + 15) // 16 * 16
    payloads = torch.randint(0, 256, (count, pstride), dtype=torch.uint8, device=dev, generator=g)
    pay_sub = [payloads[bounds[i]:bounds[i + 1]] for i in range(nsub)]
    xev = []   # (start, end) events around the two exchanges, on torch's stream

    def step(timed=False):
        if nsub > 1:   # sub-batches with every exchange in flight behind compute
            pipelined_step(subs, pay_sub, ex)
            return
        sb.propose(payloads)
        sb.pack_value()
        a = torch.cuda.Event(enable_timing=True) if timed else None
        if a:
            a.record()
        sb.exchange_value(ex)
        if a:
            b = torch.cuda.Event(enable_timing=True)
            b.record()
            xev.append((a, b))
        sb.validate_values()
        a = torch.cuda.Event(enable_timing=True) if timed else None
        if a:
            a.record()
        sb.exchange_echo(ex)
        if a:
            b = torch.cuda.Event(enable_timing=True)
            b.record()
            xev.append((a, b))
        sb.decode()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if not args.no_verify:
        real = len(sb.topo.validators(rank))
        for i, s_ in enumerate(subs):
            assert bool((s_.ok_v[:, :, :real] == 1).all()), "a valid Value proof was rejected"
            assert bool((s_.status == 0).all()), "decode failed"
            assert bool((s_.plen_out == plen).all())
            assert torch.equal(s_.out[:, :plen], pay_sub[i][:, :plen]), "decoded payload differs"
    for s_ in subs:
        s_.rb.profile(True)
        s_.rb.profile_reset()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(timed=True)
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    for s_ in subs:
        s_.rb.profile(False)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        dist.barrier()
    stages = {}
    for s_ in subs:
        for st_name, (ms, cnt) in s_.rb.profile_read().items():
            a0, c0 = stages.get(st_name, (0.0, 0))
            stages[st_name] = (a0 + ms, c0 + cnt)
    count_launch = count // nsub
    xms = sum(a.elapsed_time(b) for a, b in xev)
    S, k, m = sb.S, sb.rb.k, sb.rb.m
    L = (S + 1 + 135) // 136
    alg_bytes = {"frame": plen + k * S, "encode": (k + m) * S, "leaf_hash": n * (S + 32),
                 "validate": n * (S + 32 * (sb.rb.dslots + 1) + 1), "reconstruct": (k + sb.topo.f) * S,
                 "unframe": k * S + plen}
    dom = max(alg_bytes, key=lambda s_: stages[s_][0])
    dom_ms, dom_launches = stages[dom]
    per_launch_s = dom_ms / 1e3 / max(dom_launches, 1)
    achieved = alg_bytes[dom] * count_launch / per_launch_s / 1e9 if per_launch_s > 0 else 0.0
    perms = {"leaf_hash": count_launch * n * L,
             "validate": count_launch * (n * L + n * sb.rb.dslots)}
    valu = None
    if dom in perms:
        ops = perms[dom] * KECCAK_OPS_PER_PERM / per_launch_s
        pps = perms[dom] / per_launch_s
        valu = {"achieved_ops": ops, "peak_ops": VALU_PEAK_OPS, "frac": ops / VALU_PEAK_OPS,
                "ops_per_perm": KECCAK_OPS_PER_PERM, "perms_per_launch": perms[dom],
                "perms_per_s": pps, "measured_ceiling_perms_per_s": KECCAK_CEILING_PERMS,
                "frac_of_measured_ceiling": pps / KECCAK_CEILING_PERMS}
    xbytes = 2 * (world - 1) / world * count * sb.topo.npad * sb.stride
    value = float(count) * plen * world * args.steps / elapsed / 1e9
    if rank == 0:
        line = {
            "metric": METRIC, "value": value, "unit": "GB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (uniform random payloads resident in HBM)",
            "config": {"workload": "%s: N=%d f=%d (%d+%d shards), %d B payloads, %d proposals/GPU, "
                                   "validators sharded over %d GPUs (%d each), Value + Echo "
                                   "all-to-all, receiver misses its f right-hand Echoes"
                                   % (args.config, n, sb.topo.f, k, m, plen, count, world,
                                      sb.topo.rpg),
                       "n": n, "f": sb.topo.f, "payload_bytes": plen, "shard_len": S,
                       "instances_per_gpu": count, "global_batch": count * world,
                       "parallelism": "validator-sharded x%d" % world,
                       "pipelined_sub_batches": nsub},
            "roofline": {"kernel": dom, "bound": "hbm", "achieved": achieved,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                         "traffic": None, "launch_ms": per_launch_s * 1e3, "valu": valu},
            "exchange": {"ms_per_step": xms / args.steps, "bytes_per_step_per_gpu": xbytes,
                         "GBps_per_gpu": xbytes / (xms / args.steps / 1e3) / 1e9 if xms else None},
            "cpu_baseline": None,
            "stages_ms_per_step": {s_: stages[s_][0] / args.steps for s_ in stages},
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
