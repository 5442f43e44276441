"""Diagnostic: per-iteration trajectory of the GPU solver (trace build) beside the oracle's.

    make -C mpc_fatigue_amd diag
    python tools/trace_probe.py [N] [problem] [seed] > trace.txt

GPU columns (libmpcfatigue_trace.so, -DMF_TRACE): dinf pinf compl mu(start) mu(after update)
dFr dw dc tries alpha_primal alpha_dual alpha accepted nu f.  The oracle's verbose log
(stderr of oracle/libmforacle.so) follows for the same horizon.
"""
import os
import sys
import tempfile

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


def main():
    import ctypes as C
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    pb = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    seed = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    opts = dict(tol=1e-8, constr_viol_tol=1e-8, max_iter=300, mu_init=0.1)
    base = PR.pilz6_bench(N=N)
    ocp = OCP(base)
    ref = load_urdf_file(PR.urdf_path(base["urdf"]))
    B = pb + 1
    Q0 = PR.pilz6_batch_q0(B, seed=seed)
    LR = np.array([P.forward_kinematics(ref, q, "prbt_link_5")[0][:2] for q in Q0])
    res = ocp.solve(Q0, line_ref=LR, F_init=PR.BENCH_F_INIT, **opts)
    L = _lib.lib()
    buf = np.zeros(16 * 512 * 16)
    L.mf_debug_trace.argtypes = [C.POINTER(C.c_double), C.c_int]
    L.mf_debug_trace(buf.ctypes.data_as(C.POINTER(C.c_double)), 16)
    T = buf.reshape(16, 512, 16)[pb]
    print(f"GPU problem {pb}: status {res.status[pb]} iters {res.iters[pb]} obj {res.obj[pb]:.10g}")
    for it in range(int(res.iters[pb]) + 1):
        r = T[it]
        print(f"it {it:3d} f {r[14]:+.8e} dinf {r[0]:.2e} pinf {r[1]:.2e} compl {r[2]:.2e} mu {r[3]:.1e}->{r[4]:.1e} "
              f"dF {r[5]:.2e} dw {r[6]:.2e} dc {r[7]:.2e} tries {int(r[8])} ap {r[9]:.3e} az {r[10]:.3e} "
              f"alpha {r[11]:.3e} acc {int(r[12])} nu {r[13]:.2e} ls {int(r[15])}")
    sys.stdout.flush()
    spec = PR.pilz6_bench(N=N, q0=Q0[pb], line_ref=LR[pb])
    with tempfile.TemporaryFile(mode="w+") as tf:
        saved = os.dup(2)
        os.dup2(tf.fileno(), 2)
        try:
            _, r = O.solve(ref, spec, F_init=PR.BENCH_F_INIT, verbose=2, **opts)
        finally:
            os.dup2(saved, 2)
            os.close(saved)
        tf.seek(0)
        print(f"ORACLE: status {r.status} iters {r.iter} obj {r.obj:.10g}")
        print(tf.read())


if __name__ == "__main__":
    main()
