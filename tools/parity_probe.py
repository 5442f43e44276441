"""Diagnostic: GPU solve vs oracle solve, per horizon (iterations, objective, max |dq|).

    python tools/parity_probe.py [N] [B] [seed]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from mpc_fatigue_amd import problems as PR  # noqa: E402
from mpc_fatigue_amd.ocp import OCP  # noqa: E402
from oracle import oracle as O  # noqa: E402
from oracle import pin_np as P  # noqa: E402
from oracle.urdf_np import load_urdf_file  # noqa: E402


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    seed = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    opts = dict(tol=1e-8, constr_viol_tol=1e-8, max_iter=300, mu_init=0.1)
    base = PR.pilz6_bench(N=N)
    ocp = OCP(base)
    ref = load_urdf_file(PR.urdf_path(base["urdf"]))
    Q0 = PR.pilz6_batch_q0(B, seed=seed)
    LR = np.array([P.forward_kinematics(ref, q, "prbt_link_5")[0][:2] for q in Q0])
    res = ocp.solve(Q0, line_ref=LR, F_init=PR.BENCH_F_INIT, **opts)
    specs = [PR.pilz6_bench(N=N, q0=Q0[b], line_ref=LR[b]) for b in range(B)]
    W, R = O.solve_batch(ref, specs, F_init=PR.BENCH_F_INIT, **opts)
    for b in range(B):
        qg, _, Fg = ocp.unpack(res.w[b])
        qr, _, Fr = ocp.unpack(W[b])
        print(f"b={b} st {res.status[b]}/{R[b].status} it {res.iters[b]}/{R[b].iter} "
              f"obj {res.obj[b]:.10g}/{R[b].obj:.10g} max|dq| {np.abs(qg - qr).max():.3e} "
              f"max|dF| {np.abs(Fg - Fr).max():.3e}")


if __name__ == "__main__":
    main()
