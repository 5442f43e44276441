"""Diagnostic: where the C3 shared-budget horizons that do not converge spend an iteration (the tail of the bench's
generic figure).  Runs the homotopy stages pos_toll 1 and 1e-2 (caps 150, 300), then the reference stage 1e-4 for
`iters` iterations with the phase stamps (libmpcfatigue_gstamps.so) and prints, for the horizons that converged and
for those still running at the cap, the per-iteration cycles of each phase and the counters.

    python tools/gdiag_tail.py [batch] [iters]
"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mpc_fatigue_amd import _lib  # noqa: E402

_lib.LIB_PATH = os.path.join(ROOT, "mpc_fatigue_amd", os.environ.get("MF_LIB", "libmpcfatigue_gstamps.so"))
from mpc_fatigue_amd import problems as PR  # noqa: E402
from mpc_fatigue_amd.gocp import GOCP  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
IT = int(sys.argv[2]) if len(sys.argv) > 2 else 300
rng = np.random.default_rng(0)
g1 = np.loadtxt(os.path.join(ROOT, "tests", "golden", "G1_box_N50_solution.csv"), delimiter=",")[:12]
sp = PR.box_shared_fatigue(N=100, q0=g1)
X = np.hstack([g1[None] + rng.uniform(-0.01, 0.01, (B, 12)), np.tile(sp["T0"], (B, 1))])
kw = dict(u_init=PR.box_u_init(sp), max_soc=4)
L = _lib.lib()
w = None
for tol, cap in ((1.0, 150), (1e-2, 300)):
    r = GOCP(dict(sp, pos_toll=tol)).solve(x0=X, w0=w, max_iter=cap, **kw)
    w = r.w
L.mf_debug_gstamps_reset()
r = GOCP(dict(sp, pos_toll=1e-4)).solve(x0=X, w0=w, max_iter=IT, **kw)
n = min(B, 1024)
buf = (C.c_ulonglong * (32 * n))()
L.mf_debug_gstamps(buf, n)
a = np.array(buf, dtype=np.float64).reshape(n, 32)
it = np.maximum(r.iters[:n], 1).astype(float)
cols = [0, 1, 8, 9, 10, 11, 12, 13, 14, 2, 19, 23, 24, 25, 26, 17, 18, 4, 5, 15, 6, 7]
names = ["opt-err+mu", "barrier+resid", " f:stage loads", " f:H assembly", " f:PB,PA", " f:stage block", " f:BK factor",
         " f:BK solve+st", " f:P update", " f:rest", " d:stage loads", " d:vx,tv", " d:zv", " d:solve", " d:pvs+loop",
         " d:forward", " d:tail", "ftb+merit0+pHp", "trial merits", "SOC rest", "post-LS", "update"]
print("stage pos_toll 1e-4 from the capped homotopy: status", {int(s): int((r.status == s).sum()) for s in np.unique(r.status)},
      "iterations p50/p90/max", np.percentile(r.iters, [50, 90, 100]).tolist())
for label, m in (("converged", r.status[:n] == 0), ("not converged", r.status[:n] != 0)):
    if not m.any():
        continue
    tot = a[m][:, cols].sum(1)
    print(f"--- {label}: {int(m.sum())} horizons, per-iteration cycles (median) {np.median(tot / it[m]):.0f}")
    for c, nm in zip(cols, names):
        print(f"{nm:18s} {np.median(a[m][:, c] / it[m]):12.0f} cyc/iter")
    print("factorisations / iter", np.mean(a[m][:, 20] / it[m]), " trial merits / iter", np.mean(a[m][:, 21] / it[m]),
          " SOC directions / iter", np.mean(a[m][:, 22] / it[m]))
