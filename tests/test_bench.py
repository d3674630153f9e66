"""bench.py's host logic on CPU: the device-side input generators restate the
oracle's counter PRNG (orc_gen_payload / orc_gen_present), so the GPU leg and
the CPU baseline see identical payloads and erasure patterns; the launcher
refuses a rank count that disagrees with --gpus."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

import bench
from oracle import pyoracle as orc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_payload_generator_matches_oracle():
    for plen, first, count in [(262144, 0, 3), (1000, 17, 4), (7, 5, 2), (0, 0, 2), (4096, 1 << 20, 2)]:
        out = bench.gen_payloads(torch, bench.SEED, first, count, plen, max(16, plen + 9),
                                 "cpu").numpy()
        for i in range(count):
            assert np.array_equal(out[i, :plen], orc.gen_payload(bench.SEED, first + i, plen))
            assert not out[i, plen:].any()


def test_present_generator_matches_oracle():
    for n, n_erase, first, count in [(64, 21, 0, 50), (16, 5, 1000, 30), (250, 166, 3, 5),
                                     (4, 1, 0, 20), (128, 42, 99, 10)]:
        pres = bench.gen_present(torch, bench.SEED, first, count, n, n_erase, "cpu").numpy()
        for i in range(count):
            assert np.array_equal(pres[i], orc.gen_present(bench.SEED, first + i, n, n_erase)), \
                (n, i)


def test_world_size_must_match_gpus():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "WORLD_SIZE=1 but --gpus 2" in r.stderr


def test_f4_leg_host_helpers():
    """The f4 leg's CPU check decodes the fixture encodings and agrees with the
    fixture outcomes (one valid, one tampered); the VALU work per check comes
    from the committed counter pass."""
    import json
    pool = json.load(open(os.path.join(ROOT, "tests", "golden", "bls_vectors.json")))["bench_pool"]
    assert len(pool) == 32 and sum(c["expect"] for c in pool) == 24
    assert bench.f4_cpu_check(pool[0]) and bench.f4_cpu_check(pool[3])
    ops, src = bench.pairing_ops_per_check()
    assert ops is not None and 1e6 < ops < 1e8 and "SQ_INSTS_VALU" in src


@pytest.mark.gpu
def test_bench_line_small(tmp_path):
    """The whole default line at small sizes on the GPU, as the driver runs it
    (one process, N=1): instance mode with its leaf-reuse variant, the cfg2 /
    cfg5 objects, the f4 leg, then both validator objects on the one-rank
    schedule (state machine beside the next step, two step pipelines).
    bench.py checks every decoded payload itself; here the printed line must
    fit the driver's tail (LINE_CAP) and carry every object, none of them an
    error, and --detail the full record."""
    detail = str(tmp_path / "detail.json")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--count", "512",
                        "--vcount", "256", "--rider-count", "64", "--steps", "2", "--warmup", "2",
                        "--no-cpu", "--detail", detail,
                        "--f4-checks", "4096", "--f4-steps", "1"],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1 and len(lines[0]) <= bench.LINE_CAP, len(lines[-1])
    line = json.loads(lines[0])
    assert line["value"] > 0 and line["n_gpus"] == 1 and line["config"]["instances_per_gpu"] == 512
    assert line["leaf_reuse"]["value"] > 0 and line["leaf_reuse"]["verified_last_timed_step"]
    # the erase fill (transport) is timed but outside `value`
    assert line["stages_ms_per_step"]["erase"] > 0 and line["value_incl_erase"] < line["value"]
    assert line["roofline"]["frac"] > 0 and line["roofline"]["bound"] in ("valu", "hbm")
    # BASELINE's cfg2 (with its encode+Merkle rate) and cfg5 ride along
    for key, n in (("cfg2", 16), ("cfg5", 250)):
        v = line[key]
        assert "error" not in v, v.get("error")
        assert v["value"] > 0 and ("N=%d " % n) in v["workload"] and v["verified_last_timed_step"]
        assert v["roofline_kernel"] and v["ms_per_step"] > 0
    assert line["cfg2"]["encode_merkle"] > line["cfg2"]["value"]
    for key in ("validators", "validators_cfg4"):
        v = line[key]
        assert "error" not in v, v.get("error")
        assert v["value"] > 0 and v["schedule"].startswith("overlapped, 2 pipe")
    assert "error" not in line["threshold_decrypt"]
    full = json.load(open(detail))
    assert "state_machine_overlapped" in full["validators"]["stages_ms_per_step"]
    assert full["validators"]["config"]["step_pipelines"] == 2
    assert "stages" in full["roofline"] and "encode_merkle" in full["cfg2"]


# ------------------------------------------------ the line and its phases --
def _run_phase_driver(scenario, extra_env=None, world=2):
    """World-2 gloo run of tests/bench_phase_driver.py; rank 0's stdout."""
    port = str(bench.free_port())
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port, **(extra_env or {}))
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests",
                                                                   "bench_phase_driver.py"),
                                       scenario], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=240) for p in procs]
    return [p.returncode for p in procs], outs


def _line(stdout):
    lines = [ln for ln in stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, stdout[-2000:]
    assert len(lines[0]) <= bench.LINE_CAP, len(lines[0])
    return json.loads(lines[0])


def test_compact_line_of_full_size_record_fits():
    """The full record of a real full-size run (profiles/r5ac_bench.json,
    21.4 KB, which the driver could not parse) compacts to at most LINE_CAP
    bytes and keeps the contract's fields, the dominant kernel's roofline,
    the CPU baseline and every object's rate."""
    full = json.load(open(os.path.join(ROOT, "profiles", "r5ac_bench.json")))
    assert len(json.dumps(full)) > 20000
    line = bench.compact_line(full, "gpurun_out/detail.json")
    text = json.dumps(line)
    assert len(text) <= bench.LINE_CAP
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "dtype",
              "config", "roofline", "cpu_baseline", "higher_is_better", "scaling", "vs_baseline"):
        assert k in line, k
    ro = line["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic", "launch_ms", "hbm_frac",
              "pipeline_hbm_frac", "profiled_frac"):
        assert k in ro, k
    assert abs(ro["frac"] - full["roofline"]["frac"]) < 1e-3
    cb = line["cpu_baseline"]
    assert cb["value"] > 0 and cb["cores"] >= 1 and cb["kind"] == "port" and cb["sample"]
    assert cb["single_core"] > 0
    for key in ("leaf_reuse", "validators", "validators_cfg4", "cfg2", "cfg5",
                "threshold_decrypt"):
        assert line[key]["value"] > 0 and line[key]["ms_per_step"] > 0, key
    assert line["cfg2"]["encode_merkle"] > line["cfg2"]["value"]
    assert line["cfg2"]["roofline_frac"] > 0 and line["cfg5"]["verified_last_timed_step"]
    assert line["threshold_decrypt"]["cpu_baseline"] > 0
    # an object that failed keeps only its (truncated) error
    full["validators"] = {"error": "RuntimeError: " + "x" * 5000}
    line = bench.compact_line(full)
    assert line["validators"]["error"].startswith("RuntimeError") and \
        len(json.dumps(line)) <= bench.LINE_CAP


def test_phases_validator_failure_keeps_the_line(tmp_path):
    """World 2 over gloo: the validator phase raises on every rank; the line
    still carries the headline, the instance objects and the validators'
    error, and --detail holds the full record."""
    detail = str(tmp_path / "detail.json")
    rcs, outs = _run_phase_driver("raise_validators", {"DETAIL": detail})
    assert rcs == [0, 0], [o[1][-2000:] for o in outs]
    line = _line(outs[0][0])
    assert "{" not in outs[1][0]                       # only rank 0 prints the line
    assert line["value"] > 0 and line["roofline"]["frac"] > 0 and line["n_gpus"] == 2
    assert line["cfg2"]["value"] > 0 and line["cfg5"]["value"] > 0
    assert line["threshold_decrypt"]["value"] > 0
    assert "injected failure" in line["validators"]["error"]
    assert line["validators_cfg4"]["value"] > 0      # the next phase still ran, on both ranks
    full = json.load(open(detail))
    assert "stages" in full["roofline"] and line["detail"] == detail


def test_phases_one_rank_failure_is_agreed():
    """cfg2 raises on rank 1 only: both ranks record it as failed and go on
    to the next phase together (no rank runs its collectives alone)."""
    rcs, outs = _run_phase_driver("raise_cfg2_rank1")
    assert rcs == [0, 0], [o[1][-2000:] for o in outs]
    line = _line(outs[0][0])
    assert "another rank" in line["cfg2"]["error"]
    assert line["cfg5"]["value"] > 0 and line["validators"]["value"] > 0


def test_phases_stuck_collective_prints_the_line():
    """Rank 1 blocks in a collective rank 0 never joins during the validator
    phase: after the phase budget rank 0 prints the line with the headline and
    the validators' timeout, and both processes end (exit 0) well before the
    process-group timeout."""
    import time
    t0 = time.time()
    rcs, outs = _run_phase_driver("hang_validators", {"BUDGET": "4"})
    assert time.time() - t0 < 50
    assert rcs == [0, 0], [o[1][-2000:] for o in outs]
    line = _line(outs[0][0])
    assert line["value"] > 0 and line["cfg2"]["value"] > 0
    assert "timeout" in line["validators"]["error"]
    assert "validators_cfg4" not in line


def test_roofline_with_step_pipelines():
    """With two step pipelines the launch spans overlap: the encode's span can
    exceed the sponges', yet the dominant kernel stays a sponge stage and the
    line's `frac` is the aggregate rate (every sponge launch's permutations
    over the wall time), the per-launch figure kept beside it."""
    n, k, m, plen, count, steps = 16, 6, 10, 1 << 20, 4096, 10
    S = (plen + 4 + k - 1) // k
    L = (S + 1 + 135) // 136
    nc, dsl = 31, 4
    # stage: (ms summed over the timed steps, launches)
    stages = {"encode": (600.0, 2 * steps), "leaf_hash": (550.0, 2 * steps),
              "validate": (300.0, steps), "tree_levels": (3.0, 2 * steps),
              "proofs": (1.0, steps), "reconstruct": (50.0, steps), "frame": (0.0, 0)}
    elapsed = 0.33
    r = bench.roofline_of(stages, steps, count, n, k, m, S, plen, nc, dsl, 5, elapsed, "cfgX",
                          pipes=2)
    assert r["kernel"] == "leaf_hash" and r["bound"] == "valu" and r["concurrent_pipes"] == 2
    perms = (count * n * L * 2 * steps + count * (n * L + n * dsl) * steps
             + count * (n - 1) * 2 * steps)
    opp, _ = bench.valu_ops_per_perm("cfgX")
    assert abs(r["aggregate"]["perms_per_s"] - perms / elapsed) < 1e-6 * perms / elapsed
    assert abs(r["frac"] - perms / elapsed * opp / bench.VALU_PEAK_OPS) < 1e-9
    assert r["per_launch_frac"] < r["frac"] and r["profiled"] is None
    one = bench.roofline_of(stages, steps, count, n, k, m, S, plen, nc, dsl, 5, elapsed, "cfgX")
    assert one["kernel"] == "encode" and "aggregate" not in one   # one pipeline: spans rank
