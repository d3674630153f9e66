"""bench.py's host logic on CPU: the device-side input generators restate the
oracle's counter PRNG (orc_gen_payload / orc_gen_present), so the GPU leg and
the CPU baseline see identical payloads and erasure patterns; the launcher
refuses a rank count that disagrees with --gpus."""
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
def test_bench_line_small():
    """The whole default line at small sizes on the GPU, as the driver runs it
    (one process, N=1): instance mode with its leaf-reuse variant, both
    validator objects on the one-rank schedule (state machine beside the next
    step, two step pipelines), the f4 leg.  bench.py checks every decoded
    payload itself after the warm-up; here the line must carry every object,
    none of them an error."""
    import json
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--count", "512",
                        "--vcount", "256", "--rider-count", "64", "--steps", "2", "--warmup", "2",
                        "--no-cpu",
                        "--f4-checks", "4096", "--f4-steps", "1"],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["value"] > 0 and line["n_gpus"] == 1 and line["config"]["instances_per_gpu"] == 512
    assert line["leaf_reuse"]["value"] > 0 and line["leaf_reuse"]["verified_last_timed_step"]
    assert line["stages_ms_per_step"]["erase"] > 0
    # BASELINE's cfg2 (with its encode+Merkle rate) and cfg5 ride along
    for key, n in (("cfg2", 16), ("cfg5", 250)):
        v = line[key]
        assert "error" not in v, v.get("error")
        assert v["value"] > 0 and v["config"]["n"] == n and v["verified_last_timed_step"]
        assert v["roofline"]["kernel"] and v["ms_per_step"] > 0
    assert line["cfg2"]["encode_merkle"]["value"] > line["cfg2"]["value"]
    for key in ("validators", "validators_cfg4"):
        v = line[key]
        assert "error" not in v, v.get("error")
        assert v["value"] > 0 and v["config"]["step_pipelines"] == 2
        assert "state_machine_overlapped" in v["stages_ms_per_step"]
    assert "error" not in line["threshold_decrypt"]
