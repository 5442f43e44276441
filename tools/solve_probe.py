"""Diagnostic (GPU): one batched C2 bench solve (B horizons, N=100) with a given max_iter, for profiling
the full-occupancy iterations under rocprofv3."""
import sys
import time

sys.path.insert(0, ".")
import numpy as np  # noqa: E402

from mpc_fatigue_amd import problems as PR  # noqa: E402
from mpc_fatigue_amd.ocp import OCP  # noqa: E402
from oracle import pin_np as P  # noqa: E402
from oracle.urdf_np import load_urdf_file  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
MI = int(sys.argv[2]) if len(sys.argv) > 2 else 40
REP = int(sys.argv[3]) if len(sys.argv) > 3 else 2
spec = PR.pilz6_bench(N=100)
ocp = OCP(spec)
ref = load_urdf_file(PR.urdf_path(spec["urdf"]))
Q0 = PR.pilz6_batch_q0(B, seed=0)
LR = np.array([P.forward_kinematics(ref, q, "prbt_link_5")[0][:2] for q in Q0])
for r in range(REP):
    t = time.time()
    res = ocp.solve(Q0, line_ref=LR, F_init=PR.BENCH_F_INIT, max_iter=MI)
    print(f"rep {r} {time.time() - t:.3f} s  converged {int((res.status == 0).sum())}/{B} mean iters "
          f"{res.iters.mean():.1f}", flush=True)
