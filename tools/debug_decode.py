import sys, numpy as np, torch
sys.path.insert(0, '.')
sys.path.insert(0, 'tests')
from test_gpu_parity import run_pipeline
from oracle import pyoracle as orc
for n, plen, count in [(8, 4099, 3), (8, 1000, 3), (10, 500, 3), (16, 6001, 4), (64, 5000, 4)]:
    f = (n - 1) // 3
    r = run_pipeline(torch, n, f, plen, count, seed=0x48424246, erase_seed=11, n_erase=f)
    S = r["S"]
    for i in range(count):
        sh, nd = orc.send_shards(n, f, r["pay"][i].tobytes())
        bad = [j for j in range(n) if not np.array_equal(r["recv"][i, j, :S], sh[j])]
        erased = np.where(r["present"][i] == 0)[0].tolist()
        print(n, plen, i, "status", r["status"][i], "erased", erased, "bad rows", bad,
              "padbad", [j for j in range(n) if r["recv"][i, j, S:].any()])
        for j in bad[:2]:
            d = np.where(r["recv"][i, j, :S] != sh[j])[0]
            print("   row", j, "ndiff", len(d), "first", d[:8].tolist())
