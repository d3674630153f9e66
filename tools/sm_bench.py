#!/usr/bin/env python3
"""State-machine rounds alone (hbbft_amd/rbc_sim.py over sim.hip), honest
instances as the validator-sharded bench objects run them: N=64 x 4096 and
N=128 x 2048 instances on one rank, every proof valid, every decode Ok.
Prints one JSON line per N: ms per run (all rounds, read-backs included),
rounds, and the kernel forms' environment.  For A/B of libhbrbc builds
(HBRBC_LIB) and launch forms (HBRBC_SM_W4, HBRBC_SM_STAGED).

usage: python tools/sm_bench.py [--reps 5]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import torch

    from hbbft_amd.rbc_sim import StateMachineRank, honest_tensors, run_rounds
    dev = torch.device("cuda", 0)
    for n, count in ((64, 4096), (128, 2048)):
        R = n
        props = [i % n for i in range(count)]
        ok = torch.zeros((count, 1, 2, n), dtype=torch.uint8, device=dev)
        ok[:, 0, 0, :] = 1
        dec = torch.ones((count, 1), dtype=torch.uint8, device=dev)
        sm = StateMachineRank(n, count, 1, honest_tensors(n, props, dev), 0, 1, device=0,
                              max_out=4, max_faults=4, ok=ok, dec=dec)
        rounds = run_rounds([sm])            # warm-up
        assert bool((sm.output_root[:, :R] == 0).all()), "an honest node did not decide"
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            rounds = run_rounds([sm])
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        ts.sort()
        print(json.dumps({"n": n, "instances": count, "nodes": count * n, "rounds": rounds,
                          "ms_median": ts[len(ts) // 2], "ms_min": ts[0],
                          "lib": os.path.basename(os.environ.get("HBRBC_LIB", "libhbrbc.so")),
                          "w4": os.environ.get("HBRBC_SM_W4", "auto"),
                          "staged": os.environ.get("HBRBC_SM_STAGED", "1")}), flush=True)


if __name__ == "__main__":
    main()
