#!/usr/bin/env python3
"""Build A/B variants of the specialised encoders / decoders (hiprtc code
objects under hbbft_amd/jit/) with environment knobs, one fresh process per
code object so no knob leaks from one build into the next.

usage: python tools/build_variants.py 'ENV=V[,ENV=V...]' [...] --n 64 [--dec] [-j 8]
  each positional argument is one variant, e.g. HBRBC_RT_SPEC=8 or
  HBRBC_RT_SPEC=14,HBRBC_JIT_FDEPTH=4; --n picks the validator count (f =
  (n-1)//3); --dec also builds the decoders of the bench's fixed patterns for n,
  --uf their fused-unframe variants.
"""
import argparse
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

ONE = r"""
import sys, json
sys.path.insert(0, %r)
import hbbft_amd as hb
kind, k, m, g, pres = json.loads(sys.argv[1])
if kind == "enc":
    hb.jit_build_encode(k, m, group=g)
else:
    hb.jit_build_decode(k, m, pres, g, fused_unframe=kind == "decuf")
"""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--n", type=int, default=64)
    ap.add_argument("--dec", action="store_true")
    ap.add_argument("--uf", action="store_true", help="also the fused-unframe (_uf) decoders")
    ap.add_argument("-j", type=int, default=8)
    a = ap.parse_args()
    sys.path.insert(0, ROOT)
    import json
    f = (a.n - 1) // 3
    k, m = a.n - 2 * f, 2 * f
    pres = [1 if k <= i < 2 * k else 0 for i in range(a.n)]
    jobs = []
    for v in a.variants:
        env = dict(os.environ)
        env.update(dict(kv.split("=", 1) for kv in v.split(",")))
        probe = subprocess.run([sys.executable, "-c",
                                "import sys, json; sys.path.insert(0, %r); import hbbft_amd as hb; "
                                "print(json.dumps([hb.jit_encode_groups(%d, %d), "
                                "hb.jit_decode_groups(%d, %d, %r)]))" % (ROOT, k, m, k, m, pres)],
                               env=env, check=True, capture_output=True, text=True)
        ne, nd = json.loads(probe.stdout)
        jobs += [(env, v, ["enc", k, m, g, None]) for g in range(ne)]
        if a.dec:
            jobs += [(env, v, ["dec", k, m, g, pres]) for g in range(nd)]
        if a.uf:
            jobs += [(env, v, ["decuf", k, m, g, pres]) for g in range(nd)]

    def run(job):
        env, v, t = job
        r = subprocess.run([sys.executable, "-c", ONE % ROOT, json.dumps(t)], env=env,
                           capture_output=True, text=True)
        return v, t[0], t[3], r.returncode, r.stderr[-300:]

    with ThreadPoolExecutor(a.j) as ex:
        for v, kind, g, rc, err in ex.map(run, jobs):
            print(v, kind, g, "ok" if rc == 0 else "FAILED rc=%d %s" % (rc, err), flush=True)


if __name__ == "__main__":
    main()
