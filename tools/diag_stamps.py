"""Diagnostic: per-phase cycle shares of k_ipm_iter (build with -DMF_PHASE_STAMPS).

Usage: python tools/diag_stamps.py [batch]   (needs mpc_fatigue_amd/libmpcfatigue_stamps.so)
Phase slots: 0 opt-error+mu, 1 barrier, 2 KKT factor (all inertia tries), 3 back-subst+recovery,
4 FTB+merit0+gdot, 5 line search, 6 update; counters: 8 tries, 9 line-search trials, 10 iterations.
"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mpc_fatigue_amd import _lib  # noqa: E402

_lib.LIB_PATH = os.path.join(ROOT, "mpc_fatigue_amd", os.environ.get("MF_LIB", "libmpcfatigue_stamps.so"))
from mpc_fatigue_amd import problems as PR  # noqa: E402
from mpc_fatigue_amd.ocp import OCP  # noqa: E402
from oracle import pin_np as P  # noqa: E402
from oracle.urdf_np import load_urdf_file  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
spec = PR.pilz6_bench(N=100)
ocp = OCP(spec)
ref = load_urdf_file(PR.urdf_path(spec["urdf"]))
Q0 = PR.pilz6_batch_q0(B, seed=0)
LR = np.array([P.forward_kinematics(ref, q, "prbt_link_5")[0][:2] for q in Q0])
res = ocp.solve(Q0, line_ref=LR, tol=1e-8, constr_viol_tol=1e-8, max_iter=300, F_init=PR.BENCH_F_INIT)
L = _lib.lib()
buf = (C.c_ulonglong * (32 * B))()
L.mf_debug_phase_stamps(buf, B)
a = np.array(buf, dtype=np.float64).reshape(B, 32)[:min(B, 4096)]  # the stamp buffer holds 4096 problems
# KKT sub-phases (per stage, summed): 18 end of stage to loop top, 19 the wait for the prefetched
# stage block, 7 H to LDS, 11 s=Pc+p + slot stores, 12 block assembly,
# 13 Bunch-Kaufman factor, 14 solve, 15 P update; slot 2 keeps the rest of the KKT phase
cols = [0, 1, 2, 18, 19, 7, 11, 12, 13, 14, 15, 3, 4, 5, 6]
names = ["opt-err+mu", "barrier", "kkt-other", " kkt:loop-top", " kkt:wait-sgr", " kkt:H->LDS", " kkt:s+slot", " kkt:assemble", " kkt:BK-factor",
         " kkt:BK-solve", " kkt:P-update", "backsub+recover", "ftb+merit0+gdot", "linesearch", "update"]
a_ = a
a = a_[:, cols]
tot = a.sum(1)
print("status", np.bincount(res.status), "mean iters", res.iters.mean())
it = a_[:, 10]
print("per-iteration cycles (median over problems):", np.median(tot / it))
for i, nm in enumerate(names):
    print(f"{nm:18s} {np.median(a[:, i] / it):12.0f} cyc/iter  {100 * a[:, i].sum() / tot.sum():5.1f}%")
print("inertia tries / iter", np.mean(a_[:, 8] / it), " line-search trials / iter", np.mean(a_[:, 9] / it))
print("stage factorisations / iter", np.mean(a_[:, 17] / it), " pivoted fallbacks / iter", np.mean(a_[:, 16] / it))
stage = a_[:, [18, 19, 7, 11, 12, 13, 14, 15]].sum(1)
print("Riccati stage loop: cycles per stage factorisation (median over problems):", np.median(stage / a_[:, 17]))

