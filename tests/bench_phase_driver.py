"""One rank of bench.py's phase orchestration with stand-in phases (CPU, gloo).

tests/test_bench.py starts WORLD_SIZE of these (RANK etc. in the
environment) and reads rank 0's stdout: bench.run_bench runs the phases in
order, guards the secondary ones, makes the ranks agree on failures, watches
the validator-sharded ones, and prints one compact line.  The stand-in
results are the objects of a real full-size line (profiles/r5ac_bench.json),
so the size of the printed line is the size the driver would see.

usage: python tests/bench_phase_driver.py SCENARIO
  raise_validators  -- the validator phase raises on every rank
  raise_cfg2_rank1  -- cfg2 raises on rank 1 only (the ranks must agree)
  hang_validators   -- rank 1 blocks in a collective, rank 0 keeps working:
                       the phase budget ends both with the line printed
  ok                -- every phase returns
"""
import argparse
import datetime
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def main():
    scenario = sys.argv[1]
    import torch.distributed as dist
    world = int(os.environ["WORLD_SIZE"])
    rank = int(os.environ["RANK"])
    dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=60))
    full = json.load(open(os.path.join(ROOT, "profiles", "r5ac_bench.json")))
    head = {k: full[k] for k in ("value", "ms_per_step", "config", "roofline",
                                 "stages_ms_per_step", "leaf_reuse")}
    args = argparse.Namespace(config="cfg3", mode="both", steps=2, warmup=1,
                              detail=os.environ.get("DETAIL", ""),
                              phase_budget=float(os.environ.get("BUDGET", "100")), no_cpu=False)

    def ok(key):
        def run():
            dist.barrier()     # every phase has collectives, like the real ones
            return full[key]
        return run

    def boom(key, ranks):
        def run():
            dist.barrier()     # the phase's collectives, then a failing check()
            if rank in ranks:
                raise RuntimeError("injected failure in %s" % key)
            return full[key]
        return run

    def hang(key):
        def run():
            if rank == 1:
                dist.barrier()          # rank 0 never joins: stuck collective
            else:
                time.sleep(60)          # rank 0 still busy in its own work
            return full[key]
        return run

    def run_head():
        dist.barrier()
        return head

    phases = [("head", run_head),
              ("cfg2", ok("cfg2")), ("cfg5", ok("cfg5")),
              ("threshold_decrypt", ok("threshold_decrypt")),
              ("validators", ok("validators")), ("validators_cfg4", ok("validators_cfg4"))]
    if scenario == "raise_validators":
        phases[4] = ("validators", boom("validators", {0, 1}))
    elif scenario == "raise_cfg2_rank1":
        phases[1] = ("cfg2", boom("cfg2", {1}))
    elif scenario == "hang_validators":
        phases[4] = ("validators", hang("validators"))
    sys.exit(bench.run_bench(args, world, rank, "cpu", 0, phases, backend_cpu=True,
                             cpu_fn=lambda: full["cpu_baseline"]))


if __name__ == "__main__":
    main()
