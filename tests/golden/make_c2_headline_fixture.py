"""Fixture generator (test data, run in the build container): the oracle's IPOPT-mode solves of the headline
workload's first horizons -- C2 as the reference solves it (force_optimization_pilz_6DOF.py:195-197: nlpsol('ipopt')
at its defaults from x0 = 0) on horizons 0..B-1 of the C5 batch (problems.pilz6_bench, q0 = IK + U(-0.05, 0.05) with
default_rng(0), line reference = FK(q0)[0:2]), N = 100, IPOPT's globalisation with the device's elimination
(riccati = 2), max_iter 3000.  Writes tests/golden/c2_headline_ipopt_oracle.npz: w (B x 1306), status, iters, obj.

    python tests/golden/make_c2_headline_fixture.py [B] [threads]
"""
from __future__ import annotations

import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

IPOPT_MODE = dict(init_zero=True, filter=True, bound_relax=1e-8, max_iter=3000, max_soc=4)


def main():
    from mpc_fatigue_amd import problems as PR
    from oracle import generic as G
    from oracle import pin_np as P
    from oracle.urdf_np import load_urdf_file
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    nt = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    base = PR.pilz6_bench(N=100)
    ref = load_urdf_file(PR.urdf_path(base["urdf"]))
    Q0 = PR.pilz6_batch_q0(B, seed=0)
    LR = np.array([P.forward_kinematics(ref, q, "prbt_link_5")[0][:2] for q in Q0])
    specs = [PR.pilz6_bench(N=100, q0=Q0[b], line_ref=LR[b]) for b in range(B)]
    t = time.time()
    W, R = G.solve_batch(specs, nthreads=nt, riccati=2, **IPOPT_MODE)
    print(f"{B} oracle solves in {time.time() - t:.1f} s")
    np.savez_compressed(os.path.join(HERE, "c2_headline_ipopt_oracle.npz"), w=W,
                        status=np.array([r.status for r in R], np.int32), iters=np.array([r.iter for r in R], np.int32),
                        obj=np.array([r.obj for r in R]), q0=Q0, line_ref=LR)
    print("status", np.unique([r.status for r in R], return_counts=True), "iters", [r.iter for r in R])


if __name__ == "__main__":
    main()
