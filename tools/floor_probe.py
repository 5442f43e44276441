"""How tight can C2's fatigue floor be?  The reference's 15 Nm is infeasible even statically (16.64 Nm,
tests/test_problems.py); the bench uses 30 Nm (problems.BENCH_FLOOR).  This solves the first 16 horizons of the C5 batch
(q0 = IK + U(-0.05, 0.05), line reference fk(q0)) at a range of floors with the specialised solver's restatement
(oracle/mf_oracle.c, l1-merit mode from the held state, 300-iteration cap: the headline's algorithm) and, for the
floors just below, the first 4 with IPOPT mode (filter globalisation and IPOPT's restoration, x0 = 0, 3000-iteration
cap; the oracle's IPM with the product's node functions), whose statuses 4 / 5 say the restoration phase could not
find a feasible point.

Run:  python tools/floor_probe.py > profiles/r05_fatigue_floor_probe.txt
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mpc_fatigue_amd import problems as PR  # noqa: E402
from oracle import oracle as O  # noqa: E402
from oracle import pin_np as P  # noqa: E402
from oracle.urdf_np import load_urdf_file  # noqa: E402

if __name__ == "__main__":
    ref = load_urdf_file(PR.urdf_path(PR.pilz6_bench()["urdf"]))
    Q0 = PR.pilz6_batch_q0(16, seed=0)
    LR = [P.forward_kinematics(ref, q, "prbt_link_5")[0][:2] for q in Q0]
    print("| floor (Nm) | solver | horizons | converged | statuses | mean iterations |")
    print("|---|---|---|---|---|---|")
    for fl in (17.0, 20.0, 25.0, 27.0, 28.0, 29.0, 30.0):
        specs = [PR.pilz6_force(N=100, q0=Q0[i], line_ref=LR[i], tau_floor=fl) for i in range(16)]
        _, R = O.solve_batch(ref, specs, nthreads=8, tol=1e-8, constr_viol_tol=1e-8, max_iter=300, mu_init=0.1,
                             F_init=PR.BENCH_F_INIT)
        st = [r.status for r in R]
        print(f"| {fl:g} | merit (headline) | 16 | {sum(s == 0 for s in st)} | {sorted(set(st))} | "
              f"{np.mean([r.iter for r in R]):.1f} |", flush=True)
    from oracle import cpu_fast as CF
    from oracle import generic as G
    for fl in (25.0, 28.0):
        specs = [PR.pilz6_force(N=100, q0=Q0[i], line_ref=LR[i], tau_floor=fl) for i in range(4)]
        t = time.time()
        _, R = G.solve_batch(specs, nthreads=4, L=G.bind(CF.lib()), init_zero=True, filter=True, bound_relax=1e-8,
                             max_iter=3000, max_soc=4, riccati=2, **CF.FastNodes(specs[0]).opts_kw())
        st = [r.status for r in R]
        print(f"| {fl:g} | IPOPT mode | 4 | {sum(s == 0 for s in st)} | {st} | {np.mean([r.iter for r in R]):.1f} |",
              flush=True)
