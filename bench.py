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

CONFIGS = {
    # name: (N, payload bytes, instances per GPU, erasures)
    "cfg2": (16, 1 << 20, 4096, "f"),
    "cfg3": (64, 256 << 10, 8192, "f"),
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
    return ap.parse_args()


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    import hbbft_amd as hb

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    n, plen, count, erase = CONFIGS[args.config]
    if args.count:
        count = args.count
    f = (n - 1) // 3
    rb = hb.RbcBatch(n, f, device=local)
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
    rb.reserve(count)
    stream = torch.cuda.current_stream(dev)

    def step():
        rb.frame(payloads, plen, slab)
        rb.encode(slab, S)
        rb.merkle(slab, S, nodes)
        rb.proofs(nodes, digests, ndig)
        rb.validate(slab, S, digests, ndig, nodes, ok)
        roots.copy_(nodes[:, -1, :])           # what the Echo/Ready quorum agreed on
        rb.decode(slab, S, present, roots, nodes2, out, plen_out, status)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if not args.no_verify:
        assert bool((ok == 1).all()), "a valid proof was rejected"
        assert bool((status == 0).all()), "decode failed"
        assert bool((plen_out == plen).all())
        assert torch.equal(out[:, :plen], payloads[:, :plen]), "decoded payload differs"

    rb.profile(True)
    rb.profile_reset()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    rb.profile(False)
    elapsed = t1 - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        dist.barrier()
    stages = rb.profile_read()

    total_payload = float(count) * plen * world * args.steps
    value = total_payload / elapsed / 1e9

    # ---- roofline of the dominant kernel (per launch, live HIP events) ---
    L = (S + 1 + 135) // 136  # Keccak blocks per leaf (S bytes + pad)
    alg_bytes = {
        "frame": count * (plen + k * stride),
        "encode": count * (k + m) * stride,
        "leaf_hash": count * n * (S + 32),
        "tree_levels": count * (rb.node_count - n) * 96,
        "proofs": count * (n * rb.dslots * 32 * 2 + n),
        "validate": count * n * (S + 32 * (rb.dslots + 1) + 1),
        "decode_matrix": count * (n + m * k * 16),
        "reconstruct": count * (k + n_erase) * stride,
        "unframe": count * (k * S + plen),
    }
    dom = max(stages, key=lambda s: stages[s][0])
    dom_ms, dom_launches = stages[dom]
    per_launch_s = dom_ms / 1e3 / max(dom_launches, 1)
    achieved = alg_bytes[dom] / per_launch_s / 1e9 if per_launch_s > 0 else 0.0
    perms = {"leaf_hash": count * n * L, "validate": count * (n * L + n * rb.dslots),
             "tree_levels": count * (n - 1)}
    valu = None
    if dom in perms:
        ops = perms[dom] * KECCAK_OPS_PER_PERM / per_launch_s
        valu = {"achieved_ops": ops, "peak_ops": VALU_PEAK_OPS, "frac": ops / VALU_PEAK_OPS,
                "ops_per_perm": KECCAK_OPS_PER_PERM, "perms_per_launch": perms[dom]}
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
            pm = json.load(open(prof))
            key = "%s:%s:%d" % (args.config, dom, count)
            if key in pm:
                roofline["traffic"] = pm[key]
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
                       "parallelism": "instance-sharded x%d" % world},
            "roofline": roofline, "cpu_baseline": cpu,
            "stages_ms_per_step": {s: stages[s][0] / args.steps for s in stages},
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
