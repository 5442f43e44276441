"""C3 shared-budget bench starts (tools/generic_bench.py's draw: the G1 start + U(-0.01, 0.01), default_rng(0)) solved
by the host IPM in IPOPT mode (oracle/mf_ocp.c with the product's node functions, oracle/libmfcpu.so; the device's
Riccati elimination, riccati = 2) with the two restoration problems: the dynamics rows exact (resto_hard_dyn, the
build's variant before round 5) and IPOPT's (elastic p, n on every row).  Prints status, iterations, objective,
line-search failures (restoration entries), inertia corrections per iteration, and, with --trace i, the number of
restoration iterations of start i (the oracle's verbose trace).

Run:  python tools/resto_variant_probe.py [starts] > profiles/r05_c3_resto_variants.txt
"""
import os
import sys
import time
from multiprocessing import Pool

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from mpc_fatigue_amd import problems as PR  # noqa: E402
from generic_bench import _golden_q0  # noqa: E402

Q0B = _golden_q0()
SP3 = PR.box_shared_fatigue(N=100, q0=Q0B)
X3 = np.hstack([Q0B[None] + np.random.default_rng(0).uniform(-0.01, 0.01, (64, 12)), np.tile(SP3["T0"], (64, 1))])


def run(job):
    from oracle import cpu_fast as CF
    from oracle import generic as G
    i, hard = job
    spec = dict(SP3, q0=list(X3[i, :12]), T0=list(X3[i, 12:]))
    fk = CF.FastNodes(spec)
    t = time.time()
    w, R = G.solve_batch([spec], nthreads=1, L=CF.lib(), init_zero=True, filter=True, bound_relax=1e-8, max_iter=3000,
                         max_soc=4, riccati=2, resto_hard_dyn=hard, **fk.opts_kw())
    r = R[0]
    return i, hard, r.status, r.iter, r.obj, r.n_ls_fail, r.n_inertia_fix / max(1, r.iter), time.time() - t


if __name__ == "__main__":
    os.environ.setdefault("OMP_NUM_THREADS", "1")
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    print("| start | restoration | status | iterations | objective | line-search failures | inertia corrections / iter |")
    print("|---|---|---|---|---|---|---|")
    with Pool(8) as p:
        res = sorted(p.imap_unordered(run, [(i, h) for i in range(n) for h in (True, False)]), key=lambda r: (r[0], not r[1]))
    for i, hard, st, it, obj, lsf, ic, _ in res:
        print(f"| {i} | {'dynamics exact' if hard else 'IPOPT (elastic dynamics)'} | {st} | {it} | {obj:.8f} | {lsf} | {ic:.2f} |")
