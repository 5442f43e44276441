"""Diagnostic: the receding-horizon parity case of tests/test_gpu_mpc.py, printing per step and
horizon the GPU and oracle status, iterations and max |w_gpu - w_oracle| instead of asserting."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mpc_fatigue_amd import problems as PR  # noqa: E402
from mpc_fatigue_amd.mpc import RecedingHorizon, next_initial_state  # noqa: E402
from oracle import oracle as O  # noqa: E402
from oracle import pin_np as P  # noqa: E402
from oracle.urdf_np import load_urdf_file  # noqa: E402

OPTS = dict(tol=1e-8, constr_viol_tol=1e-8, max_iter=300, mu_init=0.1, F_init=PR.BENCH_F_INIT)
N, B, steps = 20, 4, 3
spec = PR.pilz6_bench(N=N)
ref = load_urdf_file(PR.urdf_path(spec["urdf"]))
Q0 = PR.pilz6_batch_q0(B, seed=5)
LR = np.array([P.forward_kinematics(ref, q, "prbt_link_5")[0][:2] for q in Q0])
gpu = RecedingHorizon(spec, carry_velocity=False, **OPTS).run(Q0, steps, line_ref=LR)
for b in range(B):
    q0, qd0, w0 = Q0[b], np.zeros(6), None
    for s in range(steps):
        sp = PR.pilz6_bench(N=N, q0=q0, line_ref=LR[b])
        sp["qd0"] = qd0
        w, r = O.solve(ref, sp, w0=w0, **OPTS)
        print(f"b={b} s={s} status gpu/oracle {gpu[s].status[b]}/{r.status} iters {gpu[s].iters[b]}/{r.iter} "
              f"max|dw| {np.abs(gpu[s].w[b] - w).max():.2e} obj gpu/oracle {gpu[s].obj[b]:.10g}/{r.obj:.10g}", flush=True)
        qN, _ = next_initial_state(gpu[s].w[b], 6, 1, N)
        q0, qd0, w0 = qN[0], np.zeros(6), gpu[s].w[b].copy()
