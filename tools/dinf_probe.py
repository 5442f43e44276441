"""Diagnostic: after `iters` GPU iterations (trace build), recompute the dual-infeasibility rows
on the host from the GPU's multipliers with the GPU's and with the oracle's node derivatives.

    python tools/dinf_probe.py [N] [iters]
"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mpc_fatigue_amd import _lib  # noqa: E402

_lib.LIB_PATH = os.path.join(ROOT, "mpc_fatigue_amd", "libmpcfatigue_trace.so")
from mpc_fatigue_amd import problems as PR  # noqa: E402
from mpc_fatigue_amd.ocp import OCP  # noqa: E402
from oracle import oracle as O  # noqa: E402
from oracle import pin_np as P  # noqa: E402
from oracle.urdf_np import load_urdf_file  # noqa: E402

NAMES = ["q", "qd", "F", "s", "yc", "yl", "yd", "zqL", "zqU", "zdL", "zdU", "vL", "vU", "tau", "Jt", "Jl", "W", "gf",
         "line", "cost"]


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    base = PR.pilz6_bench(N=N)
    ocp = OCP(base)
    ref = load_urdf_file(PR.urdf_path(base["urdf"]))
    Q0 = PR.pilz6_batch_q0(1, seed=5)
    LR = np.array([P.forward_kinematics(ref, q, "prbt_link_5")[0][:2] for q in Q0])
    ocp.solve(Q0, line_ref=LR, F_init=PR.BENCH_F_INIT, tol=1e-8, constr_viol_tol=1e-8, max_iter=iters, mu_init=0.1)
    L = _lib.lib()
    L.mf_debug_array.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_double), C.c_long]
    n, nv, nl = 6, 13, 2
    sizes = dict(q=(N + 1) * n, qd=N * n, F=N, s=N * n, yc=N * n, yl=N * nl, yd=N * n, zqL=(N + 1) * n,
                 zqU=(N + 1) * n, zdL=N * n, zdU=N * n, vL=N * n, vU=N * n, tau=N * n, Jt=N * n * nv, Jl=N * nl * n,
                 W=N * nv * nv, gf=N * nv, line=N * nl, cost=N)
    G = {}
    for i, nm in enumerate(NAMES):
        a = np.zeros(sizes[nm])
        assert L.mf_debug_array(ocp.handle, i, a.ctypes.data_as(C.POINTER(C.c_double)), a.size) == 0
        G[nm] = a
    q = G["q"].reshape(N + 1, n); qd = G["qd"].reshape(N, n); F = G["F"].reshape(N, 1)
    Jt = G["Jt"].reshape(N, n, nv); Jl = G["Jl"].reshape(N, nl, n); gf = G["gf"].reshape(N, nv)
    yc = G["yc"].reshape(N, n); yd = G["yd"].reshape(N, n); yl = G["yl"].reshape(N, nl)
    spec = PR.pilz6_bench(N=N, q0=Q0[0], line_ref=LR[0])
    # oracle derivatives at the GPU iterate
    mx = dict(Jt=0, Jl=0, tau=0, W=0)
    Jt_o = np.zeros_like(Jt); Jl_o = np.zeros_like(Jl)
    for k in range(N):
        tau, J, pf, Jp, H = O.node_derivs(ref, spec, q[k], qd[k], F[k], yd[k], yl[k])
        Jt_o[k] = J; Jl_o[k] = Jp[:2]
        mx["Jt"] = max(mx["Jt"], np.abs(J - Jt[k]).max())
        mx["Jl"] = max(mx["Jl"], np.abs(Jp[:2] - Jl[k]).max())
        mx["tau"] = max(mx["tau"], np.abs(tau - G["tau"].reshape(N, n)[k]).max())
    print("max |GPU - oracle| at the GPU iterate:", mx)

    def rows(Jt_, Jl_):
        out = {}
        rq = np.zeros((N, n))
        for k in range(1, N + 1):
            if k < N:
                r = gf[k, :n] + yc[k] - yc[k - 1] + Jl_[k].T @ yl[k] + Jt_[k][:, :n].T @ yd[k]
            else:
                r = -yc[N - 1].copy()
            r += -G["zqL"].reshape(N + 1, n)[k] + G["zqU"].reshape(N + 1, n)[k]
            rq[k - 1] = r
        out["q"] = np.abs(rq).max(axis=1)
        rqd = np.zeros((N, n))
        for k in range(1, N):
            rqd[k] = gf[k, n:2 * n] + base["h"] * yc[k] + Jt_[k][:, n:2 * n].T @ yd[k] - G["zdL"].reshape(N, n)[k] + \
                G["zdU"].reshape(N, n)[k]
        out["qd"] = np.abs(rqd).max(axis=1)
        rF = np.array([gf[k, 12] + Jt_[k][:, 12] @ yd[k] for k in range(N)])
        out["F"] = np.abs(rF)
        rs = -yd - G["vL"].reshape(N, n) + G["vU"].reshape(N, n)
        out["s"] = np.abs(rs).max(axis=1)
        return out
    for lab, (a, b) in [("GPU derivs", (Jt, Jl)), ("oracle derivs", (Jt_o, Jl_o))]:
        r = rows(a, b)
        print(lab, {k: (float(v.max()), int(v.argmax())) for k, v in r.items()})


if __name__ == "__main__":
    main()
