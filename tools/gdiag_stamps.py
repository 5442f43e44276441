"""Diagnostic: per-phase cycle shares of the generic solver's k_giter (build with -DMF_GSTAMPS:
mpc_fatigue_amd/libmpcfatigue_gstamps.so, `make -C mpc_fatigue_amd libmpcfatigue_gstamps.so`).

Usage: python tools/gdiag_stamps.py [batch] [iters] [case] [mode]    case: c3 (shared budget, pos_toll 1) | c4 | c2 (chain);
mode: merit (default) | ipopt (x0 = 0, filter globalisation, the reference problem at pos_toll 1e-4)
Slots: 0 opt-error+mu, 1 barrier/residuals, 2 factor rest, 8 stage loads, 9 H assembly, 10 PB / PA,
11 stage block, 12 BK factor, 13 BK solve + stores, 14 P update; direction (both calls): 19 stage loads,
23 vx / tv, 24 zv, 25 solve, 26 pvs and loop top, 17 forward sweep, 18 slack rows and bound multipliers; 3 rest, 4 ftb+merit0+gdot/pHp,
5 trial merits, 15 second-order corrections, 6 after the line search, 7 update; counters 20 factorisation
tries, 21 trial merits, 22 SOC directions.
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

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
IT = int(sys.argv[2]) if len(sys.argv) > 2 else 12
case = sys.argv[3] if len(sys.argv) > 3 else "c3"
rng = np.random.default_rng(0)
if case == "c3":
    g1 = np.loadtxt(os.path.join(ROOT, "tests", "golden", "G1_box_N50_solution.csv"), delimiter=",")[:12]
    sp = PR.box_shared_fatigue(N=100, q0=g1)
    X = np.hstack([g1[None] + rng.uniform(-0.01, 0.01, (B, 12)), np.tile(sp["T0"], (B, 1))])
    spec, kw = dict(sp, pos_toll=1.0), dict(u_init=PR.box_u_init(sp), max_soc=4)
elif case == "c2":  # the chain family (C2 instance of the C5 batch, merit globalisation from the line IK start)
    from mpc_fatigue_amd import pin
    spec = PR.pilz6_bench(N=100)
    X = PR.pilz6_batch_q0(B, seed=0)
    LR = pin.generate_forward_kin(PR.read_urdf(spec["urdf"]), spec["frame"]).batch(X)[0][:, :2]
    kw = dict(max_soc=4, line_ref=np.ascontiguousarray(LR))
else:
    spec = PR.centauro(N=50, T=2.0)
    q0 = np.asarray(spec["q0"])
    X = np.hstack([q0[None] + rng.uniform(-0.02, 0.02, (B, 14)), np.tile(spec["T0"], (B, 1))])
    kw = dict(u_init=PR.centauro_u_init(spec), max_soc=4)
if len(sys.argv) > 4 and sys.argv[4] == "ipopt":
    spec = dict(spec, pos_toll=1e-4) if case == "c3" else spec
    kw = dict(init_zero=True, filter=True, bound_relax=1e-8, max_soc=4)
g = GOCP(spec)
L = _lib.lib()
g.solve(x0=X, max_iter=1, **kw)  # warm-up
L.mf_debug_gstamps_reset()
res = g.solve(x0=X, max_iter=IT, **kw)
n = min(B, 1024)
buf = (C.c_ulonglong * (32 * n))()
L.mf_debug_gstamps(buf, n)
a = np.array(buf, dtype=np.float64).reshape(n, 32)
it = np.maximum(res.iters[:n], 1).astype(float)
cols = [0, 1, 8, 9, 10, 11, 12, 13, 14, 2, 19, 23, 24, 25, 26, 17, 18, 3, 4, 5, 15, 6, 7]
names = ["opt-err+mu", "barrier+resid", " f:stage loads", " f:H assembly", " f:PB,PA", " f:stage block", " f:BK factor",
         " f:BK solve+st", " f:P update", " f:rest", " d:stage loads", " d:vx,tv", " d:zv", " d:solve", " d:pvs+loop",
         " d:forward", " d:tail", "direction rest", "ftb+merit0+pHp", "trial merits", "SOC rest", "post-LS", "update"]
tot = a[:, cols].sum(1)
print(f"{case} batch {B}: status", {int(s): int((res.status == s).sum()) for s in np.unique(res.status)},
      "mean iters", res.iters.mean())
print("per-iteration cycles (median over problems):", np.median(tot / it))
for c, nm in zip(cols, names):
    print(f"{nm:18s} {np.median(a[:, c] / it):12.0f} cyc/iter  {100 * a[:, c].sum() / tot.sum():5.1f}%")
print("factorisations / iter", np.mean(a[:, 20] / it), " trial merits / iter", np.mean(a[:, 21] / it),
      " SOC directions / iter", np.mean(a[:, 22] / it))
ev = a[:, 30].sum() + a[:, 31].sum()
print(f"k_geval block cycles / iter (sum over blocks, per problem): models+sweeps {a[:, 30].sum() / it.sum():.0f}, "
      f"record assembly {a[:, 31].sum() / it.sum():.0f} ({100 * a[:, 31].sum() / max(ev, 1):.1f}% of k_geval)")
nf = a[:, 28].sum()
if nf > 0:
    print("register Bunch-Kaufman failures / iter", np.mean(a[:, 28] / it), " mean failing column", a[:, 27].sum() / nf,
          " share in the control rows", a[:, 29].sum() / nf)
