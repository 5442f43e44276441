"""G3 (plotter/Result_4/solution.csv: Box_Pilz_6DOF.py with LeftConst, N = 80) solved cold as the reference solves it
(IPOPT from x0 = 0, L455-456) in the oracle (oracle/mf_ocp.c, IPOPT mode), with each remaining deviation from IPOPT
toggled: where does the cold solve end, and how far from Result_4?

  resto      hard: the restoration problem keeps x_{k+1} = f(x_k, u_k) exact; ipopt: IpRestoIpoptNLP's elastic p, n on
             every row, the dynamics rows included (the device's default since round 5)
  rows       eq_from = 2: the distance rows |E1 - E2|^2 = L of nodes 0 and 1 dropped (they involve only the fixed q_0,
             and q_1 = q_0 + h qd_0, which is fixed too); eq_from = 0: kept, as the reference's transcription has them
             (Box_Pilz_6DOF.py:279-282 inside `for k in range(N)`)
  delta_c    singular: IPOPT's delta_c = 1e-8 mu^(1/4) only when a factorisation is singular; always: from the first
             factorisation on every constraint row (IPOPT's treatment once it has flagged the Jacobian degenerate)
  kkt        banded: block-tridiagonal Bunch-Kaufman (the checker); riccati: the device's Riccati elimination

y_0: IPOPT's least-square multiplier estimate needs the system [[I, J^T], [J, 0]], singular for this transcription at
x0 = 0 (the fixed-node rows), where IPOPT itself falls back to y_0 = 0 -- the oracle's start; not a toggle.

Run:  python tools/g3_deviation_table.py > profiles/r05_g3_deviations.txt   (about 10 min on 8 processes)
"""
import itertools
import os
import sys
import time
from multiprocessing import Pool

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from mpc_fatigue_amd import problems as PR  # noqa: E402

N = 80
G3 = np.loadtxt(os.path.join(ROOT, "tests", "golden", "G3_box_N80_solution.csv"), delimiter=",")


def q_traj(w):
    nx, nu = 12, 18
    return np.array([w[:nx]] + [w[nx + k * (nu + nx) + nu: nx + (k + 1) * (nu + nx)] for k in range(N)])


def g3_objective():
    from oracle import generic as G
    one = PR.box_dual(N=1, q0=G3[:12], left_const=True)
    return sum(G.node_derivs(one, G3[k * 30:k * 30 + 30], np.zeros(18), np.zeros(1), np.zeros(12))[0][0]
               for k in range(N))


def run(job):
    from oracle import generic as G
    resto, eqf, dc, ric = job
    spec = dict(PR.box_dual(q0=G3[:12], N=N, left_const=True), eq_from=eqf)
    t = time.time()
    w, r = G.solve(spec, init_zero=True, bound_relax=1e-8, max_iter=3000, max_soc=4, filter=True,
                   resto_hard_dyn=(resto == "hard"), dc_all=dc, riccati=(0 if ric == "banded" else 2))
    dq = float(np.abs(q_traj(w) - q_traj(G3)).max())
    return job, r.status, r.iter, r.obj, dq, time.time() - t


if __name__ == "__main__":
    os.environ.setdefault("OMP_NUM_THREADS", "1")
    f3 = g3_objective()
    jobs = list(itertools.product(["hard", "ipopt"], [2, 0], [False, True], ["banded", "riccati"]))
    with Pool(8) as p:
        res = sorted(p.imap_unordered(run, jobs), key=lambda r: jobs.index(r[0]))
    print(f"G3 = Result_4: objective {f3:.6f}")
    print("| restoration | k = 0, 1 rows | delta_c | KKT | status | iterations | objective | max |q - q_G3| (rad) |")
    print("|---|---|---|---|---|---|---|---|")
    for (resto, eqf, dc, ric), st, it, obj, dq, _ in res:
        print(f"| {resto} | {'kept' if eqf == 0 else 'dropped'} | {'always' if dc else 'singular'} | {ric} | {st} | "
              f"{it} | {obj:.6f} | {dq:.2e} |")
