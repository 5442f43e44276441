"""Diagnostic: the IPOPT-mode generic bench batches (tools/generic_bench.py draws, seed 0) solved on the device;
per-horizon status / iterations / objective saved to gpurun_out/ipopt_fail_<case>.npz with the starts, so the
non-converged starts can be re-solved by the host IPM (oracle) on the CPU.

    python tools/ipopt_failures.py [--batch 512] [--cases c3,c4]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--cases", default="c3,c4")
    ap.add_argument("--max-iter", type=int, default=0, help="override IPOPT_KW's max_iter")
    a = ap.parse_args()
    from generic_bench import IPOPT_KW, _golden_q0
    from mpc_fatigue_amd import problems as PR
    from mpc_fatigue_amd.gocp import GOCP
    rng = np.random.default_rng(0)
    q0b = _golden_q0()
    sp3 = PR.box_shared_fatigue(N=100, q0=q0b)
    X3 = np.hstack([q0b[None] + rng.uniform(-0.01, 0.01, (a.batch, 12)), np.tile(sp3["T0"], (a.batch, 1))])
    sp4 = PR.centauro(N=50, T=2.0)
    q0c = np.asarray(sp4["q0"])
    X4 = np.hstack([q0c[None] + rng.uniform(-0.02, 0.02, (a.batch, 14)), np.tile(sp4["T0"], (a.batch, 1))])
    for case, spec, X in (("c3", sp3, X3), ("c4", sp4, X4)):
        if case not in a.cases:
            continue
        kw = dict(IPOPT_KW, **({"max_iter": a.max_iter} if a.max_iter else {}))
        r = GOCP(spec).solve(x0=X, **kw)
        st = np.asarray(r.status)
        vals, cnt = np.unique(st, return_counts=True)
        print(case, dict(zip(vals.tolist(), cnt.tolist())), "mean iters", float(np.mean(r.iters)), flush=True)
        np.savez(os.path.join(ROOT, "gpurun_out", f"ipopt_fail_{case}{'_' + str(a.max_iter) if a.max_iter else ''}.npz"), X=X, status=st, iters=np.asarray(r.iters),
                 obj=np.asarray(r.obj), kkt=np.asarray(r.kkt), w=np.asarray(r.w))
