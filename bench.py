#!/usr/bin/env python3
"""Benchmark: hbbft Reliable-Broadcast data path on MI355X.

Headline (instance mode).  One step = the whole RBC data path over one batch
of `count` independent broadcast instances already resident in HBM:
  frame (broadcast.rs:174-189) -> RS encode (193) -> Merkle tree (204) ->
  N proofs (212-222) -> validate all N proofs (254/291, merkle.rs:83-103) ->
  decode_from_shards with f random erasures per instance (563-601: decode
  matrix + reconstruct, re-tree, root compare, unframe).
value = payload bytes of every instance on every rank / max-over-ranks wall
time of the K timed steps (GB/s, 1e9), without the HIP-event-timed erase fill
that stands in for transport (value_incl_erase keeps it).  Multi-GPU:
instances are sharded across ranks with no data-path collective (weak
scaling).

Rank 0 prints ONE compact JSON line of at most LINE_CAP bytes (the driver
keeps the last ~8 KB of stdout): the contract's fields, the dominant kernel's
roofline, the CPU baseline and each object's rate; --detail PATH writes the
full record.  Objects run in order -- headline, cfg2, cfg5, f4, then the
validator-sharded ones -- each secondary one guarded and under a deadline
(Phases), so a failure or a stuck collective costs only that object.

Validator-sharded simulation (the `validators` object of the same line, or
the headline with --mode validators): the N validators are split over the
ranks, Value is an all-to-all and Echo an all-gather over RCCL (xGMI), every
rank decodes every instance for the receivers it hosts (hbbft_amd/sharded.py).

`python bench.py --gpus N` without torch.distributed.run launches the N rank
processes itself (before any GPU call); under torch.distributed.run the
ranks come from the environment.  Inputs are generated on the device from the
same counter PRNG as the CPU baseline (oracle/rbc_oracle.c orc_gen_payload /
orc_gen_present), so both legs see identical payloads and erasure patterns.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
HBM_COPY_GBS = 6290.0          # MI355X_MICROARCH.md: 6.29 TB/s measured float4 copy
VALU_PEAK_OPS = 78.6e12        # 256 CU x 4 SIMD x 32 lanes x 2.4 GHz (32-bit lane-ops/s)
KECCAK_OPS_PER_PERM = 4320     # static count: 180 VALU per round x 24 rounds
# measured ceiling of the Keccak-f[1600] round code itself (register-only loop,
# 4 waves/SIMD, profiles/r1_valu_microbench.txt): v_alignbit issues at half rate
KECCAK_CEILING_PERMS = 10.48e9
SEED = 0x48424246              # "HBBF"
GARBAGE64 = -0x5A5A5A5A5A5A5A5B  # 0xA5A5A5A5A5A5A5A5 as int64: the erase stage's fill

CONFIGS = {
    # name: (N, payload bytes, instances per GPU, erasures, validator-mode proposals per GPU)
    "cfg2": (16, 1 << 20, 4096, "f", 512),
    # cfg3: 32768 instances = 8 residency rounds of 4 waves/SIMD per sponge launch
    # (16384: 4 rounds, ~2 % slower per instance -- ramp and tail,
    # profiles/r4y_count_ab.txt, r4t_sponge_residency.txt)
    # validator objects: 8192 / 4096 proposals per GPU (+2.6 / +2.8 % over 4096 / 2048
    # on one GPU, profiles/r4aa_vcount_ab.txt; G=8 footprint 0.3 of HBM, tests/test_sharded.py)
    "cfg3": (64, 256 << 10, 32768, "f", 8192),
    "cfg4": (128, 256 << 10, 16384, "f", 4096),
    # cfg2 keeps BASELINE's batch of 4096; cfg4 / cfg5 name none: 16384 / 4096
    # instances (cfg4 +1 % over 8192, profiles/r4ac_count_ab.txt; cfg5 4096:
    # 86.8 vs 84.1-84.6 GB/s at 2048, profiles/r6k_cfg5_batch_pipes_ab.txt --
    # four residency rounds of the sponge launches instead of two; ~90 GB)
    "cfg5": (250, 4 << 20, 4096, "worst", 128),
}
METRIC = "RBC encode+Merkle+decode payload GB/s, N=64, 1/8 GPUs; fraction of HBM peak"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="cfg3", choices=sorted(CONFIGS))
    ap.add_argument("--count", type=int, default=0, help="instances per GPU (default: config)")
    ap.add_argument("--vcount", type=int, default=0,
                    help="validator mode: proposals per GPU per step (default: config)")
    ap.add_argument("--cpu-reps", type=int, default=5)
    ap.add_argument("--cpu-seconds", type=float, default=2.0, help="target seconds per CPU rep")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--f4-checks", type=int, default=F4_CHECKS,
                    help="f4 leg: pairing checks per GPU per step (0 = skip the leg)")
    ap.add_argument("--f4-steps", type=int, default=3)
    ap.add_argument("--no-cfg4", action="store_true",
                    help="skip the cfg4 validator-sharded object of the default cfg3 line")
    ap.add_argument("--no-riders", action="store_true",
                    help="skip the cfg2 / cfg5 instance-mode objects of the default cfg3 line")
    ap.add_argument("--rider-count", type=int, default=0,
                    help="instances per GPU of the cfg2 / cfg5 objects (default: their config)")
    ap.add_argument("--streams", type=int, default=1,
                    help="instance mode: sub-batches per step, each on its own HIP stream")
    ap.add_argument("--ipipes", type=int, default=1,
                    help="instance mode (headline): step pipelines, each with its own buffers "
                         "and HIP stream, step i on pipe i %% ipipes")
    ap.add_argument("--rider-pipes", type=int, default=2,
                    help="step pipelines of the cfg2 object (its 65,536-sponge launches fill one "
                         "wave per SIMD; two pipelines run two side by side)")
    ap.add_argument("--stagger", action="store_true",
                    help="with --streams > 1: each sub-batch starts after the previous one's encode")
    ap.add_argument("--no-leaf-reuse", action="store_true",
                    help="skip the instance-mode leaf_reuse variant (labelled, not the headline)")
    ap.add_argument("--no-sm-overlap", action="store_true",
                    help="validator mode on one rank: run each step's state machine after its "
                         "decode instead of beside the next step's data plane")
    ap.add_argument("--sm-overlap", action="store_true",
                    help="validator mode with >1 rank: run the overlapped schedule (state machine "
                         "on a side stream with its own process group) instead of the serial one")
    ap.add_argument("--pg-timeout", type=float, default=120.0,
                    help="seconds: timeout of every process group (a stuck collective ends the "
                         "run instead of running into the driver's limit)")
    ap.add_argument("--phase-budget", type=float, default=100.0,
                    help="seconds: a validator-sharded object still running after this long is "
                         "recorded as an error and the line is printed without it")
    ap.add_argument("--detail", default="",
                    help="write the full per-object record (stage tables, per-rank exchange "
                         "records, footprints, prose) to this JSON file; stdout gets the compact line")
    ap.add_argument("--vpipes", type=int, default=int(os.environ.get("HBRBC_BENCH_VPIPES", "2")),
                    help="one rank: step pipelines on their own HIP streams, step i on pipe "
                         "i %% vpipes (each with its own buffers and state machines)")
    ap.add_argument("--vsubs", type=int, default=4,
                    help="validator mode with >1 rank: pipelined sub-batches per step")
    ap.add_argument("--mode", choices=["instances", "validators", "both"], default="both",
                    help="instances: headline only; validators: the validator-sharded simulation "
                         "as the headline; both (default): instance headline + a `validators` "
                         "object measured in the same run")
    return ap.parse_args()


# ----------------------------------------------------------------- launcher --
def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn(args):
    """`--gpus N` outside torch.distributed.run: start N rank processes (this
    process has touched no GPU) and exit with the worst of their codes."""
    port = str(free_port())
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable] + sys.argv, env=env,
                                      stdout=None if r == 0 else subprocess.DEVNULL))
    rcs = [p.wait() for p in procs]
    bad = [rc for rc in rcs if rc != 0]
    return bad[0] if bad else 0


# ---------------------------------------------------------- synthetic inputs --
GEN_C1 = 0xD6E8FEB86659FD93
GEN_C2 = 0xA0761D6478BD642F
M64 = (1 << 64) - 1


def _s64(x):
    x &= M64
    return x - (1 << 64) if x >> 63 else x


def _srl(torch, x, s):
    """Logical right shift of int64 tensors holding uint64 bit patterns."""
    return (x >> s) & ((1 << (64 - s)) - 1)


def _mix64(torch, z):
    """orc_mix64 (SplitMix64 finaliser) on int64 tensors, wrapping like uint64."""
    z = z + _s64(0x9E3779B97F4A7C15)
    z = (z ^ _srl(torch, z, 30)) * _s64(0xBF58476D1CE4E5B9)
    z = (z ^ _srl(torch, z, 27)) * _s64(0x94D049BB133111EB)
    return z ^ _srl(torch, z, 31)


def gen_payloads(torch, seed, first, count, plen, stride, dev):
    """orc_gen_payload(seed, first + i, ., plen) for i < count, on the device:
    [count][stride] uint8, bytes past plen zero."""
    out = torch.zeros((count, stride), dtype=torch.uint8, device=dev)
    words = (plen + 7) // 8
    if words == 0:
        return out
    chunk = max(1, (1 << 26) // words)
    q = torch.arange(words, dtype=torch.int64, device=dev).view(1, -1)
    for lo in range(0, count, chunk):
        hi = min(count, lo + chunk)
        inst = torch.arange(first + lo, first + hi, dtype=torch.int64, device=dev).view(-1, 1)
        base = _s64(seed * GEN_C1) + inst * _s64(GEN_C2)
        v = _mix64(torch, base + q)
        b = v.contiguous().view(torch.uint8).view(hi - lo, words * 8)   # little-endian bytes
        out[lo:hi, :plen] = b[:, :plen]
    return out


def gen_present(torch, seed, first, count, n, n_erase, dev):
    """orc_gen_present(seed, first + i, n, n_erase, .): erase the r-th still
    present index, r = mix64(base + t) mod (n - t), for t < n_erase."""
    pres = torch.ones((count, n), dtype=torch.uint8, device=dev)
    inst = torch.arange(first, first + count, dtype=torch.int64, device=dev)
    base = _s64((seed ^ 0x5EED5EED5EED5EED) * GEN_C1) + inst * _s64(GEN_C2)
    for t in range(min(n_erase, n)):
        v = _mix64(torch, base + t)
        d = n - t
        hi, lo = _srl(torch, v, 32), v & 0xFFFFFFFF
        r = ((hi % d) * ((1 << 32) % d) + lo % d) % d        # uint64 v mod d
        cum = torch.cumsum(pres.to(torch.int64), dim=1) - 1     # rank among present
        hit = (cum == r.view(-1, 1)) & (pres == 1)
        pres[hit] = 0
    return pres


# --------------------------------------------------------------- accounting --
def roofline_of(stages, steps, per_launch, n, k, m, S, plen, nc, dslots, n_erase, elapsed,
                config, unframe_fused=False, pipes=1):
    """Roofline of the dominant kernel from live per-stage HIP-event times.
    Sponge kernels are VALU-bound (Keccak-f[1600]); the HBM view is reported
    beside it."""
    L = (S + 1 + 135) // 136  # Keccak blocks per leaf (S bytes + pad)
    # algorithmic bytes per launch (SURVEY 8d per-instance figures x instances per launch)
    alg = {s_: per_launch * v_ for s_, v_ in {
        "frame": plen + k * S,
        # frame folded into the specialised encoder: the encode launch also reads the payload
        "encode": (k + m) * S + (plen if stages.get("frame", (0.0, 0))[1] == 0 else 0),
        "leaf_hash": n * (S + 32),
        "tree_levels": (nc - n) * 96,   # one record = all levels of one tree batch
        "proofs": n * dslots * 32 * 2 + n,
        "validate": n * (S + 32 * (dslots + 1) + 1),
        "decode_matrix": n + m * k,
        # fused unframe: the reconstruct kernel also writes the payload; the
        # unframe stage is then decode_check + the zero-fill past the length
        "reconstruct": (k + n_erase) * S + (plen if unframe_fused else 0),
        "unframe": (32 + max(0, k * S - 4 - plen)) if unframe_fused else k * S + plen,
    }.items()}
    perms = {"leaf_hash": per_launch * n * L, "validate": per_launch * (n * L + n * dslots),
             "tree_levels": per_launch * (n - 1)}
    live = {s: v for s, v in stages.items() if v[1] > 0}
    dom = max(live, key=lambda s: live[s][0])
    if pipes > 1 and any(s_ in perms for s_ in live):
        # concurrent pipelines stretch every launch's span by the other
        # pipeline's kernels, so spans no longer rank the stages: the sponge
        # launches carry the step's work (the one-pipeline profile's ranking)
        dom = max((s_ for s_ in live if s_ in perms), key=lambda s_: live[s_][0])
    dom_ms, dom_launches = live[dom]
    t = dom_ms / 1e3 / max(dom_launches, 1)
    hbm_gbs = alg[dom] / t / 1e9
    traffic = None
    prof = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(prof):
        try:
            pm = json.load(open(prof)).get("traffic", {})
            if "%s:%s" % (config, dom) in pm:   # HBM bytes per instance (PMC) x instances
                traffic = pm["%s:%s" % (config, dom)] * per_launch
        except (ValueError, OSError):
            traffic = None
    step_bytes = sum(alg[s] * (stages[s][1] / max(steps, 1)) for s in stages if s in alg)
    # every stage's HBM view (algorithmic bytes per launch / live launch time),
    # with the PMC traffic ratio where a counter pass exists for this config
    per_stage = {}
    pm_all = {}
    if os.path.exists(prof):
        try:
            pm_all = json.load(open(prof)).get("traffic", {})
        except (ValueError, OSError):
            pm_all = {}
    for s_, (ms_, nl_) in live.items():
        if s_ not in alg or nl_ == 0:
            continue
        tl = ms_ / 1e3 / nl_
        e = {"ms_per_launch": tl * 1e3, "alg_bytes_per_launch": alg[s_],
             "achieved_GBps": alg[s_] / tl / 1e9, "hbm_frac": alg[s_] / tl / 1e9 / HBM_PEAK_GBS}
        key = "%s:%s" % (config, s_)
        if key in pm_all and alg[s_] > 0:
            e["traffic_over_alg"] = pm_all[key] * per_launch / alg[s_]
        per_stage[s_] = e
    r = {"kernel": dom, "launch_ms": t * 1e3, "traffic": traffic,
         "hbm": {"achieved": hbm_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                 "frac": hbm_gbs / HBM_PEAK_GBS, "alg_bytes_per_launch": alg[dom]},
         "pipeline_alg_bytes_per_step": step_bytes, "stages": per_stage,
         "pipeline_hbm_frac": step_bytes / (elapsed / steps) / 1e9 / HBM_PEAK_GBS,
         "pipeline_frac_of_measured_copy": step_bytes / (elapsed / steps) / 1e9 / HBM_COPY_GBS}
    if pipes > 1:
        # launches of concurrent pipelines overlap: a launch's span includes
        # the other pipeline's kernels, so the per-launch rate understates the
        # kernel.  `aggregate`: the permutations of EVERY sponge launch of the
        # timed steps (tree, validate, re-tree, tree levels) over the whole
        # wall time -- a lower bound of the sponge kernels' rate, since the
        # wall time also holds the encode and reconstruct
        r["concurrent_pipes"] = pipes
        tot = sum(perms[s_] * stages[s_][1] for s_ in perms if s_ in stages)
        r["aggregate"] = {"perms_per_s": tot / elapsed,
                          "scope": "all sponge launches' permutations / wall time"}
    if dom in perms:
        opp, src = valu_ops_per_perm(config)
        pps = perms[dom] / t
        ops = pps * opp / 1e12
        if pipes > 1:
            r["aggregate"]["frac"] = r["aggregate"]["perms_per_s"] * opp / VALU_PEAK_OPS
        r.update({"bound": "valu", "achieved": ops, "peak": VALU_PEAK_OPS / 1e12,
                  "unit": "T lane-ops/s", "frac": ops * 1e12 / VALU_PEAK_OPS,
                  "perms_per_launch": perms[dom], "perms_per_s": pps,
                  "ops_per_perm": opp, "ops_per_perm_source": src,
                  "measured_ceiling_perms_per_s": KECCAK_CEILING_PERMS,
                  "frac_of_measured_ceiling": pps / KECCAK_CEILING_PERMS,
                  "sustained_clock": sustained_clock(dom, pps),
                  "profiled": profiled_frac(config, perms[dom], opp, per_launch, pipes)})
        if pipes > 1:
            # the line's `frac` is the aggregate (the per-launch figure stays
            # beside it): with two pipelines a launch's span is shared
            r["per_launch_frac"] = r["frac"]
            r["achieved"] = r["aggregate"]["perms_per_s"] * opp / 1e12
            r["frac"] = r["aggregate"]["frac"]
    else:
        r.update({"bound": "hbm", "achieved": hbm_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                  "frac": hbm_gbs / HBM_PEAK_GBS})
    return r


def sustained_clock(kernel, pps):
    """The Keccak ceiling scaled to the clock the sponge kernels hold inside
    the pipeline (profiles/effective_clock.json: GRBM_GUI_ACTIVE per dispatch
    over its duration; the ceiling's register-only loop ran at 2.38 GHz, the
    pipeline's sponges at 2.17): how close this kernel is to what the
    power-managed clock allows.  None without the committed record."""
    try:
        c = json.load(open(os.path.join(ROOT, "profiles", "effective_clock.json")))
        ghz = c["pipeline_ghz"]["leaf_hash_kernel" if kernel == "leaf_hash" else "validate_kernel"]
        ceil = c["keccak_ceiling_perms_per_s_4_waves"] * ghz / c["keccak_ceiling_loop_ghz"]
    except (OSError, ValueError, KeyError):
        return None
    return {"kernel_ghz": ghz, "ceiling_loop_ghz": c["keccak_ceiling_loop_ghz"],
            "ceiling_perms_per_s_at_kernel_clock": ceil, "frac": pps / ceil,
            "source": "profiles/effective_clock.json"}


def profiled_frac(config, perms_per_launch, opp, per_launch, pipes=1):
    """The same roofline from committed files only: the dominant kernel's
    average duration in the rocprofv3 --kernel-trace --stats summary named by
    profiles/roofline_sources.json[config], and the SQ_INSTS_VALU counter of
    profiles/valu_ops_per_perm.json[config] -- so `frac` can be recomputed
    from profiles/ (the live `frac` above uses this run's HIP events)."""
    import csv
    try:
        src = json.load(open(os.path.join(ROOT, "profiles", "roofline_sources.json")))[config]
        path = os.path.join(ROOT, src["kernel_stats"])
        avg_ns = None
        for row in csv.DictReader(open(path)):
            if src["kernel"] in row["Name"]:
                avg_ns = float(row["AverageNs"])
                break
        if avg_ns is None:
            return None
        if int(src["instances"]) != int(per_launch) or int(src.get("pipes", 1)) != int(pipes):
            # a different batch per launch (--count / --streams) or a different
            # number of step pipelines: the committed profile is not this
            # line's configuration
            return None
    except (OSError, ValueError, KeyError):
        return None
    pps = perms_per_launch / (avg_ns * 1e-9)
    return {"kernel_stats": src["kernel_stats"], "kernel": src["kernel"],
            "avg_ms": avg_ns / 1e6, "perms_per_s": pps, "ops_per_perm": opp,
            "lane_ops_per_s": pps * opp, "frac": pps * opp / VALU_PEAK_OPS,
            "instances_per_launch": src["instances"]}


def valu_ops_per_perm(config):
    """32-bit lane-ops per Keccak-f[1600] of the sponge kernel: SQ_INSTS_VALU x 64
    / permutations from the committed counter pass of THIS config
    (profiles/valu_ops_per_perm.json, keyed by config), else the static count."""
    p = os.path.join(ROOT, "profiles", "valu_ops_per_perm.json")
    try:
        d = json.load(open(p))[config]
        return float(d["leaf_hash_kernel"]), "rocprofv3 SQ_INSTS_VALU (%s)" % d["source"]
    except (OSError, ValueError, KeyError, TypeError):
        return float(KECCAK_OPS_PER_PERM), "static: 180 VALU/round x 24"


# ------------------------------------------------------------- CPU baseline --
def cpu_quota():
    """CPUs of this process's cgroup quota (cgroup v2 cpu.max), or None."""
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else float(q) / float(p)
    except (OSError, ValueError):
        return None


def cpu_baseline(args, n, f, plen, n_erase, config):
    """The same pipeline in oracle/rbc_oracle.c (the reference's algorithm: table
    GF MACs like pure-Rust galois_8, scalar Keccak like tiny-keccak) on every
    CPU this process may use and on one, median of --cpu-reps repetitions over
    the same counter-PRNG payloads and erasure patterns as the GPU leg."""
    from oracle import pyoracle as orc
    orc.build()
    cpus = len(os.sched_getaffinity(0))
    quota = cpu_quota()
    threads = max(1, min(cpus, int(quota)) if quota else cpus)

    def measure(th, target_s, cap):
        t1, _ = orc.bench_pipeline(n, f, plen, th, n_erase, SEED, th)   # calibration
        per = max(t1, 1e-6)
        sample = int(max(th, min(cap, target_s / per * th)))
        times, oks = [], []
        for _ in range(args.cpu_reps):
            t, ok = orc.bench_pipeline(n, f, plen, sample, n_erase, SEED, th)
            times.append(t)
            oks.append(ok)
        times.sort()
        med = times[len(times) // 2]
        return sample, med, min(oks), times

    sample, med, ok, times = measure(threads, args.cpu_seconds, 4096)
    s1, med1, ok1, _ = measure(1, args.cpu_seconds / 2, 256)
    return {"value": sample * plen / med / 1e9, "unit": "GB/s", "cores": threads,
            "kind": "port", "reps": args.cpu_reps, "host_cpus": os.cpu_count(),
            "affinity_cpus": cpus, "cgroup_cpu_quota": quota,
            "sample_short": "%d instances of %s through oracle/rbc_oracle.c (the reference's "
                            "algorithm), %d threads, median of %d reps, %d/%d decoded ok"
                            % (sample, config, threads, args.cpu_reps, ok, sample),
            "single_core": {"value": s1 * plen / med1 / 1e9, "unit": "GB/s", "cores": 1,
                            "sample": "%d instances, median of %d" % (s1, args.cpu_reps)},
            "sample": "%d instances of %s (N=%d, %d B payload, %s) through the same pipeline in "
                      "oracle/rbc_oracle.c on %d threads; median of %d reps %.2f s (min %.2f, "
                      "max %.2f); %d/%d decoded ok; inputs orc_gen_payload/orc_gen_present("
                      "seed 0x%X, instance i) = the GPU leg's instances 0..%d"
                      % (sample, config, n, plen, "f random erasures" if n_erase == f else
                         "%d random erasures" % n_erase, threads, args.cpu_reps, med, times[0],
                         times[-1], ok, sample, SEED, sample - 1)}


# -------------------------------------------------------------- instance mode --
def run_instances(args, n, plen, count, erase, rank, world, dev, local, config=None,
                  streams=None, leaf_reuse=True, encode_merkle=False, pipes=None):
    """One instance-mode object: `config` labels it (default --config); the
    headline passes streams / leaf_reuse from the command line, the riders
    (cfg2, cfg5) run one stream without the leaf-reuse variant, and cfg2 adds
    BASELINE's encode+Merkle rate (`encode_merkle`)."""
    import torch
    import torch.distributed as dist

    import hbbft_amd as hb
    config = config or args.config
    nsub = max(1, min(args.streams if streams is None else streams, count))
    f = (n - 1) // 3
    subs_rb = [hb.RbcBatch(n, f, device=local) for _ in range(nsub)]
    rb = subs_rb[0]
    k, m = rb.k, rb.m
    S = hb.shard_len(plen, k)
    stride = rb.stride_for(S)
    n_erase = f if erase == "f" else m

    # ---- inputs resident in HBM before timing (global instance ids) ------
    pstride = (plen + 15) // 16 * 16 + int(os.environ.get("HBRBC_BENCH_PPAD", "0"))
    first = rank * count
    payloads = gen_payloads(torch, SEED, first, count, plen, pstride, dev)
    if erase == "f":
        # fresh random patterns every step (seed SEED + step): a repeating set
        # would be served by the decode-matrix cache and hide its cost
        npat = args.warmup + args.steps
        pool = [gen_present(torch, SEED + s, first, count, n, n_erase, dev) for s in range(npat)]
        present = pool[0]
    else:  # worst case: only the first k parity shards survive
        present = torch.zeros((count, n), dtype=torch.uint8, device=dev)
        present[:, k:2 * k] = 1
        for sb in subs_rb:   # one fixed pattern: its specialised decoder (rse's cached matrix)
            sb.specialise_decoder(present[0].cpu().numpy())
        pool = [present]
    # step pipelines (--ipipes / `pipes`): each with its own buffers, context
    # and HIP stream, step i on pipe i % npipe -- two whole batches in flight,
    # so a sponge launch that fills one wave per SIMD (cfg2: 65,536 sponges)
    # runs beside the other pipe's (every step still does all its work)
    npipe = max(1, args.ipipes if pipes is None else pipes)
    assert npipe == 1 or nsub == 1, "step pipelines and sub-batch streams do not combine"
    ds = max(rb.dslots, 1)
    ostride = (k * S + 15) // 16 * 16

    def buffers():
        nodes_ = torch.empty((count, rb.node_count, 32), dtype=torch.uint8, device=dev)
        return {"slab": torch.empty((count, n, stride), dtype=torch.uint8, device=dev),
                "nodes": nodes_, "nodes2": torch.empty_like(nodes_),
                "roots": torch.empty((count, 32), dtype=torch.uint8, device=dev),
                "digests": torch.empty((count, n, ds, 32), dtype=torch.uint8, device=dev),
                "ndig": torch.empty((count, n), dtype=torch.uint8, device=dev),
                "ok": torch.empty((count, n), dtype=torch.uint8, device=dev),
                "out": torch.empty((count, ostride), dtype=torch.uint8, device=dev),
                "plen_out": torch.empty(count, dtype=torch.int32, device=dev),
                "status": torch.empty(count, dtype=torch.int32, device=dev)}
    bufs = [buffers() for _ in range(npipe)]
    B0 = bufs[0]
    slab, nodes, nodes2, roots = B0["slab"], B0["nodes"], B0["nodes2"], B0["roots"]
    digests, ndig, ok, out = B0["digests"], B0["ndig"], B0["ok"], B0["out"]
    plen_out, status = B0["plen_out"], B0["status"]
    pipe_rb = [rb] + [hb.RbcBatch(n, f, device=local) for _ in range(npipe - 1)]
    if erase != "f":
        for sb in pipe_rb[1:]:
            sb.specialise_decoder(present[0].cpu().numpy())
    warm = max(args.warmup, npipe)      # every pipe has stepped before the check
    if erase == "f" and warm > args.warmup:
        pool += [gen_present(torch, SEED + s, first, count, n, n_erase, dev)
                 for s in range(len(pool), warm + args.steps)]

    # Transport: the receiver never holds the rows its pattern erases.  Every
    # step overwrites them with garbage (the "erase" stage: one row fill,
    # f x stride bytes per instance) after validation and before the decode,
    # so every timed decode really rebuilds them and the fused unframe really
    # writes the payload from rebuilt rows (the decode never runs on rows
    # that still hold the right bytes).  The row ids of every pattern (and
    # sub-batch) are built here, outside the timed region.
    # The fill simulates transport, not reference work: its HIP-event spans
    # (same stream, between the validate and the decode) are taken out of the
    # timed region's wall time for `value`; `value_incl_erase` keeps them.
    bounds = [(i * count) // nsub for i in range(nsub + 1)]
    erase_spans = []

    def erase_rows(i, q, sb=None, B=None):
        sl = slice(bounds[q], bounds[q + 1])
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        (sb or subs_rb[q]).drop_rows((B or B0)["slab"][sl], pool[i % len(pool)][sl], 0xA5)
        e1.record()
        if timing_erase[0] is not None:
            timing_erase[0].append((e0, e1))
    timing_erase = [None]

    main = torch.cuda.current_stream(dev)
    subs = []
    for i in range(nsub):
        lo, hi = bounds[i], bounds[i + 1]
        sb = subs_rb[i]
        sb.reserve(hi - lo)
        subs.append((sb, torch.cuda.Stream(dev) if nsub > 1 else main, slice(lo, hi)))
    for sb in pipe_rb[1:]:
        sb.reserve(count)
    # each pipeline on its context's own stream: the contexts' streams are
    # created one after the other, so they sit on successive hardware queues
    # (two torch pool streams can share one queue, and then never overlap:
    # DESIGN.md section 4, rejected list)
    pipe_streams = [main] if npipe == 1 else [sb.own_stream() for sb in pipe_rb]

    def run_sub(sb, sl, pres, i, q, after_encode=None, B=None):
        B = B or B0
        slab_, nodes_ = B["slab"], B["nodes"]
        sb.frame_encode(payloads[sl], plen, slab_[sl])   # frame folded into the encoder
        if after_encode is not None:
            after_encode()
        sb.merkle(slab_[sl], S, nodes_[sl])
        sb.proofs(nodes_[sl], B["digests"][sl], B["ndig"][sl])
        sb.validate(slab_[sl], S, B["digests"][sl], B["ndig"][sl], nodes_[sl], B["ok"][sl])
        B["roots"][sl].copy_(nodes_[sl, -1, :])      # what the Echo/Ready quorum agreed on
        erase_rows(i, q, sb, B)
        sb.decode(slab_[sl], S, pres[sl], B["roots"][sl], B["nodes2"][sl], B["out"][sl],
                  B["plen_out"][sl], B["status"][sl])

    def step(i):
        pres = pool[i % len(pool)]
        if npipe > 1:
            p_ = i % npipe
            with torch.cuda.stream(pipe_streams[p_]):
                run_sub(pipe_rb[p_], slice(None), pres, i, 0, B=bufs[p_])
            return
        if nsub == 1:
            run_sub(subs[0][0], subs[0][2], pres, i, 0)
            return
        ev = torch.cuda.Event()
        ev.record(main)
        prev = ev
        for q, (sb, st, sl) in enumerate(subs):
            st.wait_event(prev)
            with torch.cuda.stream(st):
                if args.stagger:
                    # the next sub-batch starts when this one's encode is done:
                    # its encode (HBM-heavy) runs beside this one's sponges
                    nxt = torch.cuda.Event()
                    run_sub(sb, sl, pres, i, q, after_encode=lambda: nxt.record(st))
                    prev = nxt
                else:
                    run_sub(sb, sl, pres, i, q)
        for _, st, _ in subs:
            main.wait_stream(st)

    def check(what, pipes_run):
        """Every proof valid, every decode Ok, every payload byte, and the
        decode trees equal to the proposer's -- the rebuilt rows hash to the
        same leaves, so every rebuilt byte is right."""
        for p_ in pipes_run:
            B = bufs[p_]
            assert bool((B["ok"] == 1).all()), "%s: a valid proof was rejected" % what
            assert bool((B["status"] == 0).all()), "%s: decode failed" % what
            assert bool((B["plen_out"] == plen).all()), what
            assert torch.equal(B["out"][:, :plen], payloads[:, :plen]), \
                "%s: decoded payload differs" % what
            assert torch.equal(B["nodes2"], B["nodes"]), "%s: rebuilt rows differ" % what

    def begin():   # side streams start after everything queued on the main one
        for st in pipe_streams[1:] if npipe > 1 else []:
            st.wait_stream(main)
    begin()
    for i in range(warm):
        step(i)
    torch.cuda.synchronize(dev)
    if not args.no_verify:
        check("warm-up", range(npipe))
        # the last warm-up step's erased rows were garbage before its decode:
        # poison the payload buffer too, so the timed steps' outputs are theirs
        for B in bufs:
            B["out"].fill_(0x5A)
            B["nodes2"].fill_(0x5A)

    all_rb = list(subs_rb) + pipe_rb[1:]
    for sb in all_rb:
        sb.profile(True)
        sb.profile_reset()
    timing_erase[0] = erase_spans
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    begin()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(warm + i)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    timing_erase[0] = None
    for sb in all_rb:
        sb.profile(False)
    erase_s = sum(a.elapsed_time(b) for a, b in erase_spans) / 1e3
    # one stream: the erase spans are serial with the reference work and come
    # out of the wall time; sub-batches or pipelines on several streams
    # overlap them, so nothing is subtracted there
    serial = nsub == 1 and npipe == 1
    work = elapsed - (erase_s if serial else 0.0)
    elapsed_all = max_over_ranks(elapsed, world, dev)
    elapsed = max_over_ranks(work, world, dev)
    verified = False
    if not args.no_verify:
        # the outputs of each pipe's last timed step, from garbage rows
        check("last timed step", sorted({(warm + j) % npipe for j in range(args.steps)}))
        verified = True
    stages = {}
    for sb in all_rb:
        for st_name, (ms, cnt) in sb.profile_read().items():
            a0, c0 = stages.get(st_name, (0.0, 0))
            stages[st_name] = (a0 + ms, c0 + cnt)
    stages["erase"] = (erase_s * 1e3, len(erase_spans))
    value = float(count) * plen * world * args.steps / elapsed / 1e9
    lr = None
    if leaf_reuse and not args.no_leaf_reuse and nsub == 1 and npipe == 1 and erase == "f":
        lr = run_leaf_reuse(args, rb, payloads, plen, pool, slab, nodes, nodes2, roots, digests,
                            ndig, ok, out, plen_out, status, S, n, f, world, dev,
                            erase_rows, timing_erase)
    em = None
    if encode_merkle:
        em = run_encode_merkle(args, pipe_rb, payloads, plen, bufs, pipe_streams, S, world,
                               dev, count)
    roof = roofline_of(stages, args.steps, count / nsub, n, k, m, S, plen, rb.node_count,
                       rb.dslots, n_erase, elapsed, config,
                       unframe_fused=rb.unframe_fused(S, out.stride(0)), pipes=npipe)
    roof["unframe_fused"] = rb.unframe_fused(S, out.stride(0))
    r = {
        "value": value, "unit": "GB/s", "ms_per_step": elapsed / args.steps * 1e3,
        "value_incl_erase": float(count) * plen * world * args.steps / elapsed_all / 1e9,
        "ms_per_step_incl_erase": elapsed_all / args.steps * 1e3,
        "roofline": roof,
        "stages_ms_per_step": {s: stages[s][0] / args.steps for s in stages},
        "config": {"workload": "%s: N=%d f=%d (%d+%d shards), %d B payloads, %d instances/GPU, "
                               "%s erasures" % (config, n, f, k, m, plen, count,
                                                "f random" if erase == "f" else "worst-case"),
                   "n": n, "f": f, "payload_bytes": plen, "shard_len": S,
                   "instances_per_gpu": count, "global_batch": count * world,
                   "parallelism": "instance-sharded x%d" % world, "streams_per_gpu": nsub,
                   "step_pipelines": npipe},
        "n_erase": n_erase, "f": f, "leaf_reuse": lr,
        "verified_last_timed_step": verified,
        "decode_input": ("every step overwrites the %d erased rows of each instance with garbage "
                         "after validation (stage `erase`, transport: its HIP-event time is "
                         "outside `value`, inside `value_incl_erase`), so each timed decode "
                         "rebuilds them; the last timed step's payloads and decode trees are "
                         "checked" % n_erase),
    }
    if em is not None:
        r["encode_merkle"] = em
    return r


def run_leaf_reuse(args, rb, payloads, plen, pool, slab, nodes, nodes2, roots, digests, ndig,
                   ok, out, plen_out, status, S, n, f, world, dev, erase_rows, timing_erase):
    """Labelled variant of the instance step, NOT the headline: validate
    writes each validated row's Merkle leaf into the decode tree
    (hbrbc_validate_rows leaf_out), and the decode hashes only the rows the
    reconstruct rebuilds (known_leaves).  A node can do exactly this with
    the Echoes it validated (broadcast.rs:291 validate_proof, then 580
    MerkleTree::from_vec over the same rows); the reference hashes them
    again.  Same inputs, same erasure patterns, same outputs; like the
    headline, every step's erased rows are garbage before its decode, and so
    are their leaves (the receiver never validated those Echoes)."""
    import torch
    count = slab.shape[0]
    nc = nodes2.shape[1]
    leaf_words = nodes2.view(torch.int64).view(count * nc, 4)
    # leaf slot of erased row (i, j) = i * nc + j (built outside the timed region)
    leaf_ids = []
    for p_ in pool:
        e = torch.nonzero(p_.view(-1) == 0).view(-1)
        leaf_ids.append((e // n) * nc + e % n)

    def step(i):
        pres = pool[i % len(pool)]
        rb.frame_encode(payloads, plen, slab)
        rb.merkle(slab, S, nodes)
        rb.proofs(nodes, digests, ndig)
        rb.validate(slab, S, digests, ndig, nodes, ok, leaf_out=nodes2)
        roots.copy_(nodes[:, -1, :])
        erase_rows(i, 0)
        leaf_words.index_fill_(0, leaf_ids[i % len(pool)], GARBAGE64)
        rb.decode(slab, S, pres, roots, nodes2, out, plen_out, status, known_leaves=True)

    def check(what):
        assert bool((ok == 1).all()) and bool((status == 0).all()), what
        assert torch.equal(out[:, :plen], payloads[:, :plen]), "leaf reuse %s: payload differs" % what
        assert torch.equal(nodes2, nodes), "leaf reuse %s: rows/tree differ" % what

    for i in range(max(1, args.warmup)):
        step(i)
    torch.cuda.synchronize(dev)
    verified = False
    if not args.no_verify:
        check("warm-up")
        out.fill_(0x5A)
    rb.profile(True)
    rb.profile_reset()
    spans = []
    timing_erase[0] = spans
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - t0
    timing_erase[0] = None
    # like the headline: the erase fill (transport) is outside `value`
    erase_s = sum(a.elapsed_time(b) for a, b in spans) / 1e3
    elapsed = max_over_ranks(wall - erase_s, world, dev)
    rb.profile(False)
    if not args.no_verify:
        check("last timed step")
        verified = True
    stages = {k_: v_[0] / args.steps for k_, v_ in rb.profile_read().items()}
    stages["erase"] = erase_s * 1e3 / args.steps
    bl = (S + 1 + 135) // 136          # Keccak blocks per leaf (SHA3-256 rate 136)
    depth = max(1, (n - 1).bit_length())
    tree = n * bl + (n - 1)
    faithful = tree + n * (bl + depth) + tree
    executed = tree + n * (bl + depth) + f * bl + (n - 1)
    return {"value": float(count) * plen * world * args.steps / elapsed / 1e9, "unit": "GB/s",
            "ms_per_step": elapsed / args.steps * 1e3, "stages_ms_per_step": stages,
            "verified_last_timed_step": verified,
            "keccak_perms_per_instance": {"faithful": faithful, "executed": executed},
            "note": "labelled variant, not the headline: validate emits the Merkle leaf of each "
                    "validated row and the decode re-hashes only the f rebuilt rows (erased rows "
                    "and their leaves are garbage before every decode)"}


def run_encode_merkle(args, rbs, payloads, plen, bufs, streams, S, world, dev, count):
    """BASELINE cfg2's own metric: encode + Merkle only -- the proposer half
    of send_shards (broadcast.rs:170-225: frame, Coding::encode,
    MerkleTree::from_vec, one proof per shard) over the same batch, timed
    like the headline (step i on pipeline i % len(rbs), each with its own
    buffers and stream); the trees and proofs are checked against the full
    step's (which validated every proof)."""
    import torch
    npipe = len(rbs)
    refs = [B["nodes"].clone() for B in bufs]
    main = torch.cuda.current_stream(dev)

    def step(i):
        p_ = i % npipe
        B, rb = bufs[p_], rbs[p_]
        with torch.cuda.stream(streams[p_]):
            rb.frame_encode(payloads, plen, B["slab"])
            rb.merkle(B["slab"], S, B["nodes"])
            rb.proofs(B["nodes"], B["digests"], B["ndig"])

    def begin():
        for st in streams:
            if st != main:
                st.wait_stream(main)

    def check(what):
        for B, ref in zip(bufs, refs):
            assert torch.equal(B["nodes"], ref), "encode+Merkle %s: trees differ" % what
    warm = max(1, args.warmup, npipe)
    for B in bufs:
        B["nodes"].fill_(0x5A)
    begin()
    for i in range(warm):
        step(i)
    torch.cuda.synchronize(dev)
    if not args.no_verify:
        check("warm-up")
    for rb in rbs:
        rb.profile(True)
        rb.profile_reset()
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    torch.cuda.synchronize(dev)
    begin()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(warm + i)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = max_over_ranks(time.perf_counter() - t0, world, dev)
    stages = {}
    for rb in rbs:
        rb.profile(False)
        for k_, v_ in rb.profile_read().items():
            if v_[1]:
                stages[k_] = stages.get(k_, 0.0) + v_[0] / args.steps
    if not args.no_verify:
        check("after the timed steps")
    del refs
    return {"metric": "RBC encode+Merkle payload GB/s (frame, encode, tree, N proofs)",
            "value": float(count) * plen * world * args.steps / elapsed / 1e9, "unit": "GB/s",
            "ms_per_step": elapsed / args.steps * 1e3, "stages_ms_per_step": stages,
            "step_pipelines": npipe}


def max_over_ranks(x, world, dev):
    if world == 1:
        return x
    import torch
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


# ------------------------------------------------------------ validator mode --
def run_validators(args, n, plen, count, rank, world, dev, local, config=None):
    """Validator-sharded simulation: each rank proposes `count`
    instances per step and hosts N/world validators; Value rows cross ranks in
    an all-to-all, Echo rows in an all-gather (RCCL over xGMI), and every rank
    decodes every instance for its receivers."""
    import torch
    import torch.distributed as dist

    from hbbft_amd.sharded import (CommTimer, DistExchange, OverlapPipe, ShardedBroadcast,
                                   SoloExchange, interleaved_steps, overlapped_steps,
                                   pipelined_step)

    # the state machine of step i on a side stream beside the data plane of
    # step i + 1 (two state-machine slots).  One rank: the default.  More
    # ranks: opt-in (--sm-overlap; its per-round all-gathers then run over a
    # process group of their own, concurrently with the data plane's
    # collectives, which has never run on RCCL); the default there is the
    # serial schedule -- one communicator, one stream, sub-batches pipelined
    overlap = not args.no_sm_overlap and (world == 1 or args.sm_overlap)
    # serial schedule at world > 1: sub-batches with every exchange in flight
    nsub = max(1, min(args.vsubs, count)) if world > 1 and not overlap else 1
    bounds = [(i * count) // nsub for i in range(nsub + 1)]
    subs = [ShardedBroadcast(n, bounds[i + 1] - bounds[i], plen, rank, world, device=local,
                             sm_slots=2 if overlap else 1)
            for i in range(nsub)]
    sb = subs[0]
    ex = DistExchange() if world > 1 else SoloExchange()
    sm_ex = sm_exchange() if world > 1 and overlap else None
    timer = CommTimer(dev)
    pstride = (plen + 15) // 16 * 16 + int(os.environ.get("HBRBC_BENCH_PPAD", "0"))
    # instance (rank s, local i) is global instance s * count + i
    pay_sub = [gen_payloads(torch, SEED, rank * count + bounds[i], bounds[i + 1] - bounds[i], plen,
                            pstride, dev) for i in range(nsub)]

    side = torch.cuda.Stream(dev) if overlap else None
    # vpipes > 1: whole-step pipelines side by side on their own streams (each
    # its own ShardedBroadcast: buffers, library context, two state-machine
    # slots), step i on pipe i % vpipes; at world > 1 one pipe's exchanges
    # overlap the other's compute (what the serial schedule's sub-batches do)
    npipe = max(1, args.vpipes) if overlap else 1
    pipe_sbs = [sb] + [ShardedBroadcast(n, count, plen, rank, world, device=local, sm_slots=2)
                       for _ in range(npipe - 1)]
    if os.environ.get("HBRBC_BENCH_OWNQ", "0") == "1":
        # A/B: each pipeline's data plane on its context's own stream (the
        # contexts' streams sit on successive hardware queues)
        pipe_streams = [(p_.rb.own_stream(), torch.cuda.Stream(dev)) for p_ in pipe_sbs]
    else:
        pipe_streams = [(torch.cuda.Stream(dev), torch.cuda.Stream(dev)) for _ in range(npipe)]

    def step():
        if world > 1:   # sub-batches with every exchange in flight behind compute
            pipelined_step(subs, pay_sub, ex, timer)
        else:
            sb.step(pay_sub[0], ex)

    xspans = [] if world > 1 else None

    def run_steps(k, timing=None):
        if overlap and npipe > 1:
            pipes = [OverlapPipe(p_, ex, s_[1], main=s_[0], timing=timing, sm_ex=sm_ex,
                                 xspans=xspans if timing is not None else None)
                     for p_, s_ in zip(pipe_sbs, pipe_streams)]
            interleaved_steps(pipes, [pay_sub[0]] * npipe, k)
        elif overlap:
            pipe = OverlapPipe(sb, ex, side, timing=timing, sm_ex=sm_ex,
                               xspans=xspans if timing is not None else None)
            for _ in range(k):
                pipe.step(pay_sub[0])
            pipe.finish()
        else:
            for _ in range(k):
                step()

    run_steps(max(args.warmup, npipe))   # every pipe has stepped before the check
    torch.cuda.synchronize(dev)
    if not args.no_verify:
        for i, s_ in enumerate(subs + pipe_sbs[1:]):
            i = min(i, len(bounds) - 2)
            c = bounds[i + 1] - bounds[i]
            assert bool((s_.ok_v == 1).all()), "a valid Value proof was rejected"
            assert bool((s_.status == 0).all()), "decode failed"
            assert bool(s_.decided.all()), "an instance missed its Ready quorum / CanDecode"
            assert bool((s_.plen_out == plen).all())
            for src in range(world):   # every rank decoded every rank's instances
                exp = gen_payloads(torch, SEED, src * count + bounds[i], c, plen, pstride, dev)
                assert torch.equal(s_.out[src * c:(src + 1) * c, :plen], exp[:, :plen]), \
                    "decoded payload differs"
    for s_ in subs + pipe_sbs[1:]:
        s_.rb.profile(True)
        s_.rb.profile_reset()
    timer.reset()
    timer.timing = world > 1
    ex.reset_stats()
    sb.sm_timing = []
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    sm_side = [] if overlap else None
    run_steps(args.steps, sm_side)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    for s_ in subs + pipe_sbs[1:]:
        s_.rb.profile(False)
    if overlap:   # spans on the side stream, beside the next step's data plane
        sm_ms = sum(e0.elapsed_time(e1) for e0, e1 in sm_side) / args.steps
    else:
        sm_ms = sum(e0.elapsed_time(e1) for e0, e1 in sb.sm_timing) / args.steps
    sb.sm_timing = None
    elapsed = max_over_ranks(elapsed, world, dev)
    if world > 1 and overlap:   # spans of the exchanges on the pipes' main streams
        xms = sum(a.elapsed_time(b) for a, b in xspans) / args.steps
    else:
        xms = timer.elapsed_ms() / args.steps if world > 1 else 0.0
    timer.timing = False
    # per-rank record of the exchange: world, backend, and per collective the
    # calls and bytes this rank sent during the timed steps (rank 0 prints all)
    mine = {"rank": rank, "world": world, "backend": ex.backend,
            "device": str(dev), "exchange_ms_per_step": xms,
            "collectives": {k_: {"calls_per_step": v_["calls"] / args.steps,
                                 "bytes_sent_per_step": v_["bytes_sent"] / args.steps}
                            for k_, v_ in sorted(ex.stats.items())}}
    if world > 1:
        per_rank = [None] * world
        dist.all_gather_object(per_rank, mine)
    else:
        per_rank = [mine]
    stages = {}
    counts = {}
    for s_ in subs + pipe_sbs[1:]:
        for st_name, (ms, cnt) in s_.rb.profile_read().items():
            a0, c0 = stages.get(st_name, (0.0, 0))
            stages[st_name] = (a0 + ms, c0 + cnt)
        if s_ is not sb and s_ in pipe_sbs:
            continue   # a step runs on one pipe: its work is one object's
        for key, v in s_.counts().items():
            # sub-batches run their state machines in lockstep: rounds are shared
            counts[key] = max(counts.get(key, 0), v) if key == "state_machine_rounds" \
                else counts.get(key, 0) + v
    t = sb.topo
    # bytes each rank moves per step: Value all-to-all sends (G-1)/G of its
    # slab + digests; the Echo all-gather brings in the other ranks' rows of
    # every instance; the roots all-gather is 32 B per instance
    xbytes = ((world - 1) / world * count * t.npad * (sb.stride + sb.dsz)
              + (world - 1) * count * t.npad * (sb.stride + sb.dsz)
              + (world - 1) * count * 32) if world > 1 else 0.0
    value = float(count) * plen * world * args.steps / elapsed / 1e9
    return {
        "value": value, "unit": "GB/s", "ms_per_step": elapsed / args.steps * 1e3,
        "scaling": "weak in proposals (every rank decodes all world x count instances)",
        "schedule": "%s, %d pipe(s), %d sub-batch(es)" % ("overlapped" if overlap else "serial",
                                                          npipe, nsub),
        "scaling_model": ("every node outputs every broadcast, so each rank decodes all world x "
                          "count instances while its proposals stay fixed: time(G) ~ count x "
                          "(encode + tree + Value validate) + G x count x (Echo validate + decode) "
                          "+ exchange; with leaf reuse at N=64 the payload rate is expected to rise "
                          "about 2.4x from 1 to 8 GPUs, not 8x (DESIGN.md section 6) -- the "
                          "protocol's replicated decode, not a communication limit"),
        "config": {"workload": "%s validator-sharded: N=%d f=%d (%d+%d shards), %d B payloads, %d "
                               "proposals/GPU/step, validators in blocks of %d over %d GPUs, Value "
                               "all-to-all + Echo all-gather, every GPU decodes every instance"
                               % (config or args.config, n, t.f, sb.rb.k, sb.rb.m, plen, count, t.rpg,
                                  world),
                   "proposals_per_gpu": count, "instances_per_step": count * world,
                   "parallelism": "validator-sharded x%d" % world,
                   "pipelined_sub_batches": nsub,
                   "step_pipelines": npipe,
                   # per-rank device bytes of this object at 1/2/4/8 GPUs (rank 0;
                   # hbbft_amd.sharded.rank_footprint, torch buffers + reconstruct
                   # workspace bound), against 288 GB of HBM per MI355X
                   "hbm_footprint_per_rank": footprint_summary(n, count, plen,
                                                               2 if overlap else 1, npipe),
                   "state_machine_group": ("its own process group (one RCCL communicator for the "
                                           "rounds' all-gathers, one for the data plane)"
                                           if sm_ex is not None else None)},
        "exchange": {"ms_per_step": xms, "bytes_per_step_per_gpu": xbytes,
                     "GBps_per_gpu": xbytes / (xms / 1e3) / 1e9 if xms > 0 else None,
                     "backend": ex.backend, "per_rank": per_rank},
        "work_per_step_rank0": counts,
        "stages_ms_per_step": dict({s: stages[s][0] / args.steps for s in stages},
                                   **({"state_machine_overlapped": sm_ms} if overlap
                                      else {"state_machine": sm_ms})),
        **({"stages_note": "%d step pipelines run side by side: a stage's span includes the "
                           "other pipelines' kernels (--vpipes 1 gives the serial split)" % npipe}
           if npipe > 1 else {}),
        # the same string at every world size (the world shows in config.parallelism)
        "state_machine_schedule": ("step i's rounds on a second HIP stream beside step i + 1's "
                                   "data plane (two state-machine slots); every step's rounds "
                                   "complete inside the timed region" if overlap else
                                   "after each step's decode")
                                  + ("; %d step pipelines side by side on their own streams, "
                                     "step i on pipe i %% %d (stage times overlap)" % (npipe, npipe)
                                     if npipe > 1 else ""),
    }


_SM_EX = []
PG_TIMEOUT = [None]    # datetime.timedelta of every process group (main() sets it)


def sm_exchange():
    """The state machine's own process group (created once, collectively, by
    every rank in the same order): its per-round all-gathers run on a side
    stream beside the data plane's collectives, and a communicator of their
    own keeps the two from interleaving differently on different ranks."""
    import torch.distributed as dist

    from hbbft_amd.sharded import DistExchange
    if not _SM_EX:
        _SM_EX.append(DistExchange(dist.new_group(list(range(dist.get_world_size())),
                                                  timeout=PG_TIMEOUT[0])))
    return _SM_EX[0]


def footprint_summary(n, count, plen, sm_slots=1, pipes=1):
    from hbbft_amd.sharded import HBM_PER_GPU, rank_footprint
    out = {}
    for g in (1, 2, 4, 8):
        # the schedule is the same at every world size: sm_slots state-machine
        # slots per pipeline, `pipes` pipelines
        fp = rank_footprint(n, count, plen, g, 0, sm_slots=sm_slots)
        k = pipes
        out["G%d" % g] = {"bytes": k * fp["total_bytes"], "frac_of_288GB": k * fp["frac_of_hbm"],
                          "echo_slab_bytes": fp["buffers"].get("echo_sh", fp["buffers"]["slab"])}
    assert all(v["bytes"] < HBM_PER_GPU for v in out.values()), out
    return out


# --------------------------------------------------------------------- main --
# ------------------------------------------------ f4: threshold-decrypt checks --
F4_CHECKS = 262144     # 64 epochs x 64 ciphertexts x 64 decryption shares (N=64)
F4_METRIC = "threshold-decrypt share verifications/s (BLS12-381 pairing checks)"


def pairing_ops_per_check():
    """32-bit lane-ops per check (2 Miller loops + 1 final exponentiation):
    SQ_INSTS_VALU x 64 / checks from the committed counter pass, or None."""
    p = os.path.join(ROOT, "profiles", "pairing_valu_ops.json")
    try:
        d = json.load(open(p))
        return float(d["ops_per_check"]), d["source"]
    except (OSError, ValueError, KeyError):
        return None, None


def f4_cpu_check(item):
    """One fixture check through the pure-Python restatement (tests use it)."""
    from oracle import bls_oracle as B
    a, b, c, d = (bytes.fromhex(item[k]) for k in "abcd")

    def g1(x):
        return None if x[0] & 0x40 else (int.from_bytes(x[:48], "big"), int.from_bytes(x[48:], "big"))

    def g2(x):
        if x[0] & 0x40:
            return None
        v = [int.from_bytes(x[i:i + 48], "big") for i in range(0, 192, 48)]
        return ((v[1], v[0]), (v[3], v[2]))
    return B.pairing_check(g1(a), g2(b), g1(c), g2(d)) == item["expect"]


def f4_cpu_baseline(pool, reps, target_s=2.0):
    """oracle/bls_pairing.c (C restatement of the pairing crate: 6 x 64-bit
    Montgomery limbs, Karatsuba tower, sparse lines, the crate's final
    exponentiation) on the cgroup's cores and on one core, over the fixture
    pool tiled, median of reps; outcomes checked against the fixtures."""
    from oracle import bls_c
    cpus = len(os.sched_getaffinity(0))
    quota = cpu_quota()
    threads = max(1, min(cpus, int(quota)) if quota else cpus)
    g1 = b"".join(bytes.fromhex(c["a"]) + bytes.fromhex(c["c"]) for c in pool)
    g2 = b"".join(bytes.fromhex(c["b"]) + bytes.fromhex(c["d"]) for c in pool)
    want = bytes(1 if c["expect"] else 0 for c in pool)

    def measure(th):
        t0 = time.perf_counter()
        ok = bls_c.check_batch(g1, g2, len(pool), th)        # calibration + outcome check
        per = (time.perf_counter() - t0) / len(pool)
        assert ok == want, "C restatement disagrees with the fixture outcomes"
        tiles = max(1, int(target_s / per / len(pool)))
        times = []
        for _ in range(reps):
            t0 = time.perf_counter()
            ok = bls_c.check_batch(g1 * tiles, g2 * tiles, len(pool) * tiles, th)
            times.append(time.perf_counter() - t0)
            assert ok == want * tiles
        times.sort()
        return len(pool) * tiles, times[len(times) // 2]

    n, med = measure(threads)
    n1, med1 = measure(1)
    return {"value": n / med, "unit": "checks/s", "cores": threads, "kind": "port",
            "reps": reps, "single_core": {"value": n1 / med1, "unit": "checks/s", "cores": 1,
                                          "sample": "%d checks, median of %d" % (n1, reps)},
            "sample": "%d checks (the 32-check fixture pool tiled) through oracle/bls_pairing.c, "
                      "a C restatement of the pairing crate (the Rust crate cannot be built "
                      "here), %d threads; median of %d reps %.2f s" % (n, threads, reps, med)}


def run_threshold(args, rank, world, dev):
    """f4 leg: F4_CHECKS verify_decryption_share checks per GPU per step in
    hbbft's shape -- groups of 64 shares checked against one ciphertext's H and
    W (threshold_decrypt.rs:204-229) -- e(share, H) == e(pk_i, W): every step
    prepares each ciphertext's H and W (hbrbc_g2_prepare), decodes and checks
    the key shares pk_i (hbrbc_g1_prepare: once, as the crate holds them as
    points) and the received shares (hbrbc_g1_prepare, beside the G2
    preparation on a side stream), and checks the shares against them
    (hbrbc_pairing_check_prepared_pts).  Inputs tile the 4
    committed fixture groups (tests/golden/bls_vectors.json, one share in
    eight tampered); outcomes are checked exactly after warm-up.  The plain
    per-check form (hbrbc_pairing_check_batch) is timed beside it."""
    import numpy as np
    import torch
    import torch.distributed as dist
    from hbbft_amd import threshold as T
    groups = json.load(open(os.path.join(ROOT, "tests", "golden", "bls_vectors.json")))["bench_groups"]
    n = args.f4_checks // 64 * 64
    ng = n // 64
    g2 = np.empty((2 * ng, 192), np.uint8)
    g1 = np.empty((2 * n, 96), np.uint8)
    enc = [(np.frombuffer(bytes.fromhex(g["hash"]), np.uint8),
            np.frombuffer(bytes.fromhex(g["w"]), np.uint8),
            np.stack([np.frombuffer(bytes.fromhex(s["share"]), np.uint8) for s in g["shares"]]),
            np.stack([np.frombuffer(bytes.fromhex(s["pk"]), np.uint8) for s in g["shares"]]),
            [1 if s["expect"] else 0 for s in g["shares"]]) for g in groups]
    expect = []
    ic = np.empty(n, np.int32)
    for q in range(ng):
        e = (q + rank) % len(enc)
        h, w, sh, pk, ex = enc[e]
        g2[2 * q], g2[2 * q + 1] = h, w
        g1[2 * q * 64:2 * (q + 1) * 64:2] = sh
        g1[2 * q * 64 + 1:2 * (q + 1) * 64:2] = pk
        ic[q * 64:(q + 1) * 64] = e * 64 + np.arange(64)   # the sender's pk_i in the key table
        expect += ex
    expect = torch.tensor(expect, dtype=torch.uint8)
    d1, d2 = torch.from_numpy(g1).to(dev), torch.from_numpy(g2).to(dev)
    shares = d1[0::2].contiguous()
    # the validator sets' key shares pk_i (64 per fixture group), as the crate
    # holds them: decoded and checked once per step, then indexed per share
    dkeys = torch.from_numpy(np.concatenate([e_[3] for e_ in enc])).to(dev)
    dic = torch.from_numpy(ic).to(dev)
    ib = torch.arange(n, dtype=torch.int32, device=dev) // 64 * 2
    idd = ib + 1
    ws = T.workspace(n, dev.index)
    stream = torch.cuda.current_stream(dev)

    # the G2 preparation fills few SIMDs (one lane per point: 8192 points, a
    # serial chain each): the key shares and the received shares are decoded
    # and checked (order r) on a side stream beside it, and the Miller loops
    # only load them (hbrbc_pairing_check_prepared_pts).  HBRBC_BENCH_F4_SIDE:
    # 3 (default) the key shares on a stream of their own too (their 256
    # points are 4 waves, a latency-bound chain like the G2 points'), 2 keys
    # then shares on one side stream, 1 keys only (shares decoded inside the
    # Miller kernel), 0 everything in order on one stream; 4 (A/B) the keys
    # on the main stream before the G2 points; 5 (A/B) the G2 points on a
    # side stream too and no wait for the previous step (the host runs
    # ahead: every step's preparations pile up beside the first Miller loop;
    # +0.8 %, profiles/r6aj_f4_prep_streams_ab.txt); 6 (A/B) as 3 with the
    # G2 points on a side stream, and step i + 1's preparations enqueued
    # when step i's Miller loop is, so they run beside it and no further
    # (-3.5 %: the Miller kernel's two residency rounds become three).
    mode = int(os.environ.get("HBRBC_BENCH_F4_SIDE", "3"))
    side = torch.cuda.Stream(dev) if mode > 0 else None
    kside = torch.cuda.Stream(dev) if mode in (3, 5, 6) else stream if mode == 4 else side
    gside = torch.cuda.Stream(dev) if mode in (5, 6) else stream
    pending = []

    def prepare():
        if mode != 5:   # from this point of the main stream on
            side.wait_stream(stream)
            kside.wait_stream(stream)
            gside.wait_stream(stream)
        with torch.cuda.stream(kside):
            keys = T.g1_prepare(dkeys)
        with torch.cuda.stream(side):
            sprep = T.g1_prepare(shares) if mode >= 2 else None
        with torch.cuda.stream(gside):
            prep = T.g2_prepare(d2)
        return keys, sprep, prep

    def step(prefetch=False):
        if side is None:
            prep = T.g2_prepare(d2)
            keys = T.g1_prepare(dkeys)
            return T.pairing_check_prepared_keys(shares, keys, dkeys.shape[0], dic, prep, 2 * ng,
                                                 ib, idd, ws)
        keys, sprep, prep = pending.pop() if pending else prepare()
        stream.wait_stream(side)
        stream.wait_stream(kside)
        if gside is not stream:
            stream.wait_stream(gside)
            prep.record_stream(stream)
        keys.record_stream(stream)
        if prefetch:   # the next step's, beside this step's Miller loop
            pending.append(prepare())
        if sprep is None:
            return T.pairing_check_prepared_keys(shares, keys, dkeys.shape[0], dic, prep, 2 * ng,
                                                 ib, idd, ws)
        sprep.record_stream(stream)
        return T.pairing_check_prepared_pts(sprep, n, keys, dkeys.shape[0], dic, prep, 2 * ng, ib,
                                            idd, ws)
    for _ in range(max(1, args.warmup)):
        ok = step()
    torch.cuda.synchronize(dev)
    if not torch.equal(ok.cpu(), expect):
        raise AssertionError("bench f4: check outcomes differ from the fixtures")
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    for j in range(args.f4_steps):
        step(prefetch=mode == 6 and j + 1 < args.f4_steps)
    e1.record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    wall = max_over_ranks(time.perf_counter() - t0, world, dev)
    ev_ms = e0.elapsed_time(e1)
    # the plain form on the same checks: each check carries its own G2 points
    g2p = np.empty((2 * n, 192), np.uint8)
    g2p[0::2] = np.repeat(g2[0::2], 64, axis=0)
    g2p[1::2] = np.repeat(g2[1::2], 64, axis=0)
    d2p = torch.from_numpy(g2p).to(dev)
    wsp = T.workspace(2 * n, dev.index)
    okp = T.pairing_check_batch(d1, d2p, wsp)
    torch.cuda.synchronize(dev)
    assert torch.equal(okp.cpu(), expect)
    p0, p1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    p0.record(stream)
    for _ in range(args.f4_steps):
        T.pairing_check_batch(d1, d2p, wsp)
    p1.record(stream)
    torch.cuda.synchronize(dev)
    plain_ms = p0.elapsed_time(p1) / args.f4_steps
    del d2p, wsp
    checks = world * n * args.f4_steps
    ops, src = pairing_ops_per_check()
    roof = None
    if ops is not None:
        rate = n * args.f4_steps / (ev_ms / 1e3) * ops
        roof = {"bound": "valu", "achieved": rate / 1e12, "peak": VALU_PEAK_OPS / 1e12,
                "unit": "T lane-ops/s", "frac": rate / VALU_PEAK_OPS, "traffic": None,
                "ops_per_check": ops, "ops_per_check_source": src,
                "note": "g2_prepare_kernel + g1_prepare_kernel + miller_prepared_kernel + "
                        "final_exp_kernel, timed "
                        "with HIP events on the launch stream; ~55% of the mix issues at half "
                        "rate (v_mad_u64_u32, v_addc_co_u32; profiles/r2c_valu_microbench.txt)"}
    return {"metric": F4_METRIC, "value": checks / wall, "unit": "checks/s",
            "ms_per_step": wall / args.f4_steps * 1e3, "steps": args.f4_steps,
            "device_ms_per_step": ev_ms / args.f4_steps, "g2_points_prepared_per_step": 2 * ng,
            "plain_checks": {"checks_per_s": n / (plain_ms / 1e3), "ms_per_step": plain_ms,
                             "note": "hbrbc_pairing_check_batch, G2 points per check"},
            "scaling": "weak", "dtype": "u32 (12-limb Montgomery Fp)",
            "config": {"workload": "f4: verify_decryption_share e(share, H) == e(pk_i, W), "
                                   "%d checks per GPU per step (%d ciphertexts x 64 shares, N=64; "
                                   "each ciphertext's H and W and each key share prepared once "
                                   "per step)" % (n, ng),
                       "checks_per_gpu": n},
            "data": "the 4 fixture groups of tests/golden/bls_vectors.json tiled "
                    "(one share in eight tampered); outcomes verified exactly",
            "roofline": roof}

# ------------------------------------------------------------ the line --
LINE_CAP = 8000   # bytes: the driver keeps the last ~8 KB of stdout


def _sig(x, d=4):
    """Round floats to d significant digits (the compact line)."""
    if isinstance(x, float):
        if x != x or x in (float("inf"), float("-inf")) or x == 0.0:
            return x
        from math import floor, log10
        return round(x, max(0, d - 1 - int(floor(log10(abs(x))))))
    if isinstance(x, dict):
        return {k: _sig(v, d) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [_sig(v, d) for v in x]
    return x


def _get(d, *path):
    for p_ in path:
        if not isinstance(d, dict) or p_ not in d:
            return None
        d = d[p_]
    return d


def _compact_obj(o, extra=()):
    """One secondary object: value, time, workload, roofline fraction and the
    verification flag (errors pass through, truncated)."""
    if o is None:
        return None
    if "error" in o:
        return {"error": str(o["error"])[:300]}
    r = {"value": o.get("value"), "unit": o.get("unit"), "ms_per_step": o.get("ms_per_step"),
         "workload": _get(o, "config", "workload"), "roofline_frac": _get(o, "roofline", "frac"),
         "roofline_kernel": _get(o, "roofline", "kernel"),
         "verified_last_timed_step": o.get("verified_last_timed_step")}
    for key, path in extra:
        r[key] = _get(o, *path)
    return {k: v for k, v in r.items() if v is not None}


def compact_line(full, detail_path=None):
    """The line rank 0 prints: the contract's fields, the dominant kernel's
    roofline and the CPU baseline in full, and per secondary object only its
    rate, time, workload, roofline fraction and verification flag; everything
    else (stage tables, per-rank records, footprints, prose) is in the
    --detail file.  At most LINE_CAP bytes."""
    keep = ["metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
            "higher_is_better", "scaling", "vs_baseline", "dtype", "data"]
    line = {k: full.get(k) for k in keep}
    cfg = full.get("config") or {}
    line["config"] = {k: cfg[k] for k in ("workload", "n", "f", "payload_bytes", "shard_len",
                                          "instances_per_gpu", "global_batch", "parallelism",
                                          "proposals_per_gpu") if k in cfg}
    ro = full.get("roofline")
    if ro:
        line["roofline"] = {
            "kernel": ro.get("kernel"), "bound": ro.get("bound"), "achieved": ro.get("achieved"),
            "peak": ro.get("peak"), "unit": ro.get("unit"), "frac": ro.get("frac"),
            "traffic": ro.get("traffic"), "launch_ms": ro.get("launch_ms"),
            "hbm_frac": _get(ro, "hbm", "frac"), "pipeline_hbm_frac": ro.get("pipeline_hbm_frac"),
            "profiled_frac": _get(ro, "profiled", "frac"),
            "frac_of_sustained_clock_ceiling": _get(ro, "sustained_clock", "frac")}
    else:
        line["roofline"] = None
    cb = full.get("cpu_baseline")
    line["cpu_baseline"] = None if cb is None else {
        "value": cb.get("value"), "unit": cb.get("unit"), "cores": cb.get("cores"),
        "kind": cb.get("kind"), "single_core": _get(cb, "single_core", "value"),
        "sample": cb.get("sample_short", cb.get("sample", ""))[:200]}
    if "cpu_baseline_note" in full:
        line["cpu_baseline_note"] = full["cpu_baseline_note"]
    for k in ("value_incl_erase", "stages_ms_per_step"):
        if k in full:
            line[k] = full[k]
    if "encode_merkle" in full:   # --config cfg2: BASELINE's encode+Merkle rate
        line["encode_merkle"] = _get(full, "encode_merkle", "value")
    objs = [("leaf_reuse", ()),
            ("cfg2", (("encode_merkle", ("encode_merkle", "value")),
                      ("encode_merkle_ms", ("encode_merkle", "ms_per_step")),
                      ("pipes", ("config", "step_pipelines")),
                      ("roofline_aggregate_frac", ("roofline", "aggregate", "frac")))),
            ("cfg5", ()),
            ("threshold_decrypt", (("cpu_baseline", ("cpu_baseline", "value")),
                                   ("cpu_cores", ("cpu_baseline", "cores")))),
            ("validators", (("exchange_ms", ("exchange", "ms_per_step")),
                            ("schedule", ("schedule",)))),
            ("validators_cfg4", (("exchange_ms", ("exchange", "ms_per_step")),
                                 ("schedule", ("schedule",))))]
    for key, extra in objs:
        if key in full:
            line[key] = _compact_obj(full[key], extra)
    line["detail"] = detail_path
    line = _sig(line)
    # hard cap: drop the optional fields, largest first, until the line fits
    for drop in ("stages_ms_per_step", "leaf_reuse", "data"):
        if len(json.dumps(line)) <= LINE_CAP:
            break
        line.pop(drop, None)
    assert len(json.dumps(line)) <= LINE_CAP, len(json.dumps(line))
    return line


def assemble(args, world, res, cpu):
    """The full record (what --detail writes) from the phase results."""
    head = res.get("head")
    vobj = res.get("validators")
    if head is not None and "error" not in head:
        line = {
            "metric": METRIC, "value": head["value"], "unit": "GB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": head["ms_per_step"],
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (counter-PRNG payloads and f-erasure patterns generated in "
                    "HBM, identical to the CPU baseline's)",
            "config": head["config"], "roofline": head["roofline"], "cpu_baseline": cpu,
            "stages_ms_per_step": head["stages_ms_per_step"],
        }
        for k in ("value_incl_erase", "ms_per_step_incl_erase", "decode_input", "encode_merkle"):
            if k in head:
                line[k] = head[k]
        if head.get("leaf_reuse") is not None:
            line["leaf_reuse"] = head["leaf_reuse"]
        if cpu is None and world > 1:
            line["cpu_baseline_note"] = ("measured on rank 0 of the N=1 run only (bench "
                                         "contract); see that line's cpu_baseline")
    elif vobj is not None and "error" not in vobj and args.mode == "validators":
        line = {
            "metric": METRIC, "value": vobj["value"], "unit": "GB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": vobj["ms_per_step"],
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (counter-PRNG payloads generated in HBM)",
            "config": vobj["config"], "roofline": None, "cpu_baseline": cpu,
        }
    else:
        line = {"metric": METRIC, "value": None, "unit": "GB/s", "n_gpus": world,
                "steps": args.steps, "warmup": args.warmup, "ms_per_step": None,
                "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
                "config": {}, "roofline": None, "cpu_baseline": cpu,
                "error": str((head or vobj or {}).get("error", "no headline"))[:300]}
    for key in ("validators", "validators_cfg4", "cfg2", "cfg5", "threshold_decrypt"):
        if res.get(key) is not None:
            line[key] = res[key]
    return line


class Phases:
    """Runs the bench's objects in order on every rank and keeps the line.

    Secondary objects are guarded: an exception becomes {"error": ...}; at
    world > 1 the ranks then agree (MIN all-reduce of a success flag) so that
    none runs the next object's collectives alone.  Every secondary object
    runs under a deadline (a rank that failed before a collective its peers
    are waiting in, or an RCCL schedule that stalls): if it is still running
    after `budget` seconds, rank 0 prints the line with what has been
    measured and that object as an error, and every rank ends its process
    (os._exit) -- the headline, measured first, is never lost."""

    def __init__(self, world, rank, dev, budget, emit, backend_cpu):
        import threading
        self.world, self.rank, self.dev, self.budget = world, rank, dev, budget
        self.emit = emit                # emit(results) -> prints the line on rank 0
        self.backend_cpu = backend_cpu  # gloo: the flag tensor lives on the host
        self.res = {}
        self.lock = threading.Lock()
        self.fired = False

    def agree(self, ok):
        if self.world == 1:
            return ok
        import torch
        import torch.distributed as dist
        t = torch.tensor([1 if ok else 0], dtype=torch.int32,
                         device="cpu" if self.backend_cpu else self.dev)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return bool(t.item())

    def _expire(self, name):
        with self.lock:
            if self.fired is not None:   # the phase finished in time (or already fired)
                return
            self.fired = True
            self.res[name] = {"error": "timeout: still running after %.0f s (phase budget); "
                                       "the process ended here" % self.budget}
            try:
                self.emit(self.res)
            finally:
                sys.stdout.flush()
                sys.stderr.write("bench: %s exceeded its %.0f s budget; line printed, exiting\n"
                                 % (name, self.budget))
                sys.stderr.flush()
                os._exit(0)

    def run(self, name, fn, required=False, watch=False):
        import threading
        timer = None
        if watch and self.budget > 0:
            with self.lock:
                self.fired = None
            timer = threading.Timer(self.budget, self._expire, args=(name,))
            timer.daemon = True
            timer.start()
        ok, val = True, None
        try:
            val = fn()
        except Exception as e:  # noqa: BLE001
            if required:
                raise
            ok = False
            val = {"error": "%s: %s" % (type(e).__name__, e)}
            print("bench: %s failed: %r" % (name, e), file=sys.stderr)
        finally:
            if timer is not None:
                with self.lock:
                    if self.fired is None:
                        self.fired = False
                timer.cancel()
        if not self.agree(ok) and ok:
            val = {"error": "failed on another rank (this rank completed it)"}
        self.res[name] = val
        return val


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return spawn(args)
    import datetime

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("bench: WORLD_SIZE=%d but --gpus %d" % (world, args.gpus))
    rehearse = os.environ.get("HBRBC_BENCH_REHEARSE") == "1"
    if rehearse:
        # multi-rank rehearsal on a box with fewer GPUs than ranks: gloo, ranks
        # share the visible devices (the real N > 1 runs use RCCL, one GPU each)
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    PG_TIMEOUT[0] = datetime.timedelta(seconds=args.pg_timeout)
    if world > 1:
        if rehearse:
            dist.init_process_group("gloo", timeout=PG_TIMEOUT[0])
        else:
            dist.init_process_group("nccl", device_id=dev, timeout=PG_TIMEOUT[0])
        assert dist.get_world_size() == args.gpus
        assert rehearse or dist.get_backend() == "nccl", "multi-GPU runs use RCCL"
    return run_bench(args, world, rank, dev, local, real_phases(args, world, rank, dev, local),
                     backend_cpu=rehearse)


def real_phases(args, world, rank, dev, local):
    """name -> callable of every object of the line, in the order they run:
    the instance-mode objects (headline, cfg2, cfg5, f4: no data-path
    collective) first, then the validator-sharded ones (RCCL exchanges)."""
    import torch
    n, plen, count, erase, vcount = CONFIGS[args.config]
    count = args.count or count
    vcount = args.vcount or vcount
    both = args.mode == "both" and args.config == "cfg3"
    ph = []

    def fresh(fn):
        def run():
            torch.cuda.empty_cache()
            return fn()
        return run
    if args.mode in ("instances", "both"):
        ph.append(("head", lambda: run_instances(args, n, plen, count, erase, rank, world, dev,
                                                 local, encode_merkle=args.config == "cfg2")))
    if both and not args.no_riders:
        # BASELINE's other GPU configs, instance-sharded over the ranks like the
        # headline: cfg2 (N=16, 1 MiB x 4096, with its own encode+Merkle
        # metric) and cfg5 (N=250, 4 MiB, worst-case decode)
        for cfg in ("cfg2", "cfg5"):
            n_, plen_, cnt_, er_, _ = CONFIGS[cfg]
            ph.append((cfg, fresh(lambda n_=n_, plen_=plen_, cnt_=cnt_, er_=er_, cfg=cfg:
                                  run_instances(args, n_, plen_, args.rider_count or cnt_, er_,
                                                rank, world, dev, local, config=cfg, streams=1,
                                                leaf_reuse=False, encode_merkle=cfg == "cfg2",
                                                pipes=args.rider_pipes if cfg == "cfg2" else 1))))
    if args.f4_checks > 0:
        ph.append(("threshold_decrypt", fresh(lambda: run_threshold(args, rank, world, dev))))
    if args.mode in ("validators", "both"):
        ph.append(("validators", fresh(lambda: run_validators(args, n, plen, vcount, rank, world,
                                                              dev, local))))
    if both and not args.no_cfg4:
        # cfg4 (N=128, validators sharded over the ranks, RCCL all-to-all + all-gather)
        n4, plen4, _, _, vcount4 = CONFIGS["cfg4"]
        ph.append(("validators_cfg4", fresh(lambda: run_validators(
            args, n4, plen4, args.vcount or vcount4, rank, world, dev, local, config="cfg4"))))
    return ph


WATCHED = ("validators", "validators_cfg4")   # CPU baselines are taken before these


def run_bench(args, world, rank, dev, local, phases, backend_cpu=False, cpu_fn=None):
    """Run the phases in order (instance objects first, validator-sharded
    last, each watched), take the CPU baselines on rank 0 of a one-rank run
    before the watched phases, and print one compact line on rank 0."""
    n, plen, count, erase, vcount = CONFIGS[args.config]
    state = {"cpu": None}

    def emit(res):
        if rank != 0:
            return
        full = assemble(args, world, res, state["cpu"])
        if args.detail:
            try:
                os.makedirs(os.path.dirname(os.path.abspath(args.detail)), exist_ok=True)
                with open(args.detail, "w") as fh:
                    json.dump(full, fh, indent=1, default=str)
            except OSError as e:
                print("bench: --detail not written: %r" % (e,), file=sys.stderr)
        print(json.dumps(compact_line(full, args.detail or None)), flush=True)

    P = Phases(world, rank, dev, args.phase_budget, emit, backend_cpu)
    headline = args.mode in ("instances", "both") and "head" or "validators"
    cpu_done = False
    for name, fn in phases:
        if name in WATCHED and not cpu_done:
            state["cpu"] = cpu_fn() if cpu_fn else take_cpu_baselines(args, rank, world, P.res,
                                                                        n, plen, erase)
            cpu_done = True
        P.run(name, fn, required=name == headline, watch=name != headline)
    if not cpu_done:
        state["cpu"] = cpu_fn() if cpu_fn else take_cpu_baselines(args, rank, world, P.res, n,
                                                                    plen, erase)
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    emit(P.res)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()
    return 0


def take_cpu_baselines(args, rank, world, res, n, plen, erase):
    """Rank 0 of a one-rank run: the pipeline's CPU baseline, and the f4
    leg's (added to its object)."""
    if rank != 0 or world != 1 or args.no_cpu:
        return None
    f4 = res.get("threshold_decrypt")
    if f4 is not None and "error" not in f4:
        gold = json.load(open(os.path.join(ROOT, "tests", "golden", "bls_vectors.json")))
        pool = [{"a": s["share"], "b": g["hash"], "c": s["pk"], "d": g["w"],
                 "expect": s["expect"]} for g in gold["bench_groups"] for s in g["shares"][:8]]
        f4["cpu_baseline"] = f4_cpu_baseline(pool, 3)
    f = (n - 1) // 3
    return cpu_baseline(args, n, f, plen, f if erase == "f" else 2 * f, args.config)


if __name__ == "__main__":
    sys.exit(main())
