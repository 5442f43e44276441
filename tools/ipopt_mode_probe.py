"""Diagnostic: IPOPT-mode (filter line search + restoration) cold solves of the reference's dual-arm box task
(Box_Pilz_6DOF.py, x0 = 0 as L455-456 pass no x0) on the device; writes the solutions to gpurun_out/."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mpc_fatigue_amd import problems as PR  # noqa: E402
from mpc_fatigue_amd.gocp import GOCP  # noqa: E402
from mpc_fatigue_amd.solution_io import read_solution_csv  # noqa: E402

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASES = {"G1": ("G1_box_N50", dict(N=50)), "G2": ("G2_box_N80", dict(N=80)),
         "G3": ("G3_box_N80", dict(N=80, left_const=True)), "G4": ("G4_box_N80", dict(N=80, right_const=False))}

out = {}
for c in (sys.argv[1:] or list(CASES)):
    name, kw = CASES[c]
    g = read_solution_csv(os.path.join(HERE, "tests", "golden", name + "_solution.csv"))
    spec = PR.box_dual(q0=g[:12], **kw)
    ocp = GOCP(spec)
    t = time.time()
    r = ocp.solve(init_zero=True, bound_relax=1e-8, filter=True, max_iter=1500, max_soc=4)
    dt = time.time() - t
    dq = np.abs(ocp.q_traj(r.w[0]) - ocp.q_traj(g)).max()
    print(f"{c} status {int(r.status[0])} iter {int(r.iters[0])} obj {float(r.obj[0]):.6f} dq {dq:.3e} {dt:.1f}s",
          flush=True)
    out[c] = r.w[0]
os.makedirs(os.path.join(HERE, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(HERE, "gpurun_out", "ipopt_mode_probe.npz"), **out)

if os.environ.get("MF_TRACE_CASE"):  # per-iteration device trace of one case (verbose >= 2)
    import ctypes as C
    from mpc_fatigue_amd import _lib
    c = os.environ["MF_TRACE_CASE"]
    name, kw = CASES[c]
    g = read_solution_csv(os.path.join(HERE, "tests", "golden", name + "_solution.csv"))
    ocp = GOCP(PR.box_dual(q0=g[:12], **kw))
    _lib.lib().mf_gdebug_trace_reset()
    r = ocp.solve(init_zero=True, bound_relax=1e-8, filter=True, max_iter=int(os.environ.get("MF_TRACE_ITERS", "1500")),
                  max_soc=4, verbose=2)
    buf = np.zeros(2 * 4096 * 16)
    _lib.lib().mf_gdebug_trace(buf.ctypes.data_as(C.POINTER(C.c_double)))
    np.save(os.path.join(HERE, "gpurun_out", f"trace_{c}.npy"), buf.reshape(2, 4096, 16))
    print("trace", c, int(r.status[0]), int(r.iters[0]))
