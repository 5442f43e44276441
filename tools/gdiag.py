"""Diagnostic (GPU): iterate-by-iterate comparison of the generic device solver with the generic oracle.
Runs both with max_iter = k for k = 1..K and prints the max |w_gpu - w_oracle| per k."""
import sys

import numpy as np

sys.path.insert(0, ".")
from mpc_fatigue_amd import problems as PR  # noqa: E402
from mpc_fatigue_amd.gocp import GOCP  # noqa: E402
from oracle import generic as G  # noqa: E402

case = sys.argv[1] if len(sys.argv) > 1 else "c2"
K = int(sys.argv[2]) if len(sys.argv) > 2 else 12
if case == "c2":
    spec, kw = PR.pilz6_bench(N=20), dict(F_init=PR.BENCH_F_INIT)
elif case == "thermal":
    spec, kw = PR.pilz6_thermal(N=20, T0=79.0), dict(F_init=PR.BENCH_F_INIT)
else:
    spec = dict(PR.box_dual(N=50), pos_toll=1.0)
    kw = dict(u_init=PR.box_u_init(spec))
ocp = GOCP(spec)
step = int(sys.argv[3]) if len(sys.argv) > 3 else 1
k0 = int(sys.argv[4]) if len(sys.argv) > 4 else step
for k in range(k0, K + 1, step):
    r = ocp.solve(max_iter=k, max_soc=4, **kw)
    w, ro = G.solve(spec, max_iter=k, max_soc=4, **kw)
    d = np.abs(r.w[0] - w)
    print(f"k={k} status gpu {int(r.status[0])} oracle {ro.status} max|dw| {d.max():.3e} at {int(d.argmax())} "
          f"kkt gpu {r.kkt[0]:.3e} oracle {ro.kkt:.3e}", flush=True)

# dual comparison at the step where they part
if len(sys.argv) > 5:
    import ctypes as C
    from mpc_fatigue_amd import _lib
    kk = int(sys.argv[5])
    r = ocp.solve(max_iter=kk, max_soc=4, **kw)
    dg = np.zeros(200000)
    n = _lib.check(_lib.lib().mf_gdebug_duals(ocp.handle, 0, _lib.dptr(dg)))
    do = np.zeros(200000)
    w, ro = G.solve(spec, max_iter=kk, max_soc=4, dual_out=do, **kw)
    N, nx, nu, ni, ne = spec["N"], ocp.nx, ocp.nu, ocp.ni, max(ocp.ne, 1)
    names = [("lam", N * nx), ("yi", N * ni), ("ye", N * ne), ("zxL", (N + 1) * nx), ("zxU", (N + 1) * nx),
             ("zuL", N * nu), ("zuU", N * nu), ("vL", N * ni), ("vU", N * ni), ("mu", 1)]
    o = 0
    for nm, ln in names:
        a, b = dg[o:o + ln], do[o:o + ln]
        d = np.abs(a - b)
        print(f"  {nm}: max|d| {d.max():.3e} at {int(d.argmax())} (gpu {a[d.argmax()]:.6e} oracle {b[d.argmax()]:.6e})")
        o += ln
