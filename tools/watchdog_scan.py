"""Find IPOPT-mode solves in which a backtracking search after StopWatchDog fails (the oracle's counter
mfg_wdfail_count, oracle/mf_ocp.c ipm_filter) -- the path the device handles with its GP_WDSOFT re-evaluation round
(csrc/gipm.hip) -- among the bench starts of C2 (pilz6_batch_q0(64, seed 0), line reference fk(q0)), C3 shared budget
and C4 (tools/generic_bench.py's draws).  Host IPM with the product's node functions (oracle/libmfcpu.so), the device's
Riccati elimination.

Run:  python tools/watchdog_scan.py [c2|c3|c4] [count]
"""
import os
import sys
from multiprocessing import Pool

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from mpc_fatigue_amd import problems as PR  # noqa: E402


def spec_of(case, i):
    if case == "c2":
        from oracle import pin_np as P
        from oracle.urdf_np import load_urdf_file
        base = PR.pilz6_bench(N=100)
        q0 = PR.pilz6_batch_q0(64, seed=0)[i]
        lr = P.forward_kinematics(load_urdf_file(PR.urdf_path(base["urdf"])), q0, "prbt_link_5")[0][:2]
        return PR.pilz6_bench(N=100, q0=q0, line_ref=lr)
    from generic_bench import _golden_q0
    rng = np.random.default_rng(0)
    q0b = _golden_q0()
    sp3 = PR.box_shared_fatigue(N=100, q0=q0b)
    X3 = np.hstack([q0b[None] + rng.uniform(-0.01, 0.01, (64, 12)), np.tile(sp3["T0"], (64, 1))])
    if case == "c3":
        return dict(sp3, q0=list(X3[i, :12]), T0=list(X3[i, 12:]))
    sp4 = PR.centauro(N=50, T=2.0)
    X4 = np.hstack([np.asarray(sp4["q0"])[None] + rng.uniform(-0.02, 0.02, (64, 14)), np.tile(sp4["T0"], (64, 1))])
    return dict(sp4, q0=list(X4[i, :14]), T0=list(X4[i, 14:]))


def run(job):
    from oracle import cpu_fast as CF
    from oracle import generic as G
    case, i = job
    spec = spec_of(case, i)
    fk = CF.FastNodes(spec)
    L = G.bind(CF.lib())
    L.mfg_wdfail_count.argtypes = [G.C.c_int]
    L.mfg_wdfail_count(1)
    _, R = G.solve_batch([spec], nthreads=1, L=L, init_zero=True, filter=True, bound_relax=1e-8, max_iter=3000,
                         max_soc=4, riccati=2, **fk.opts_kw())
    return case, i, L.mfg_wdfail_count(1), R[0].status, R[0].iter


if __name__ == "__main__":
    os.environ.setdefault("OMP_NUM_THREADS", "1")
    case = sys.argv[1] if len(sys.argv) > 1 else "c2"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    with Pool(8) as p:
        for c, i, k, st, it in p.imap_unordered(run, [(case, i) for i in range(n)]):
            if k:
                print(f"{c} start {i}: {k} failed search(es) after StopWatchDog; status {st}, {it} iterations", flush=True)
