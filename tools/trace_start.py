"""Diagnostic: one start of an IPOPT-mode generic bench batch (the draws of tools/ipopt_failures.py) solved alone on the device with the per-iteration trace (verbose >= 2, horizon 0), saved to
gpurun_out/trace_<case>_<i>.npy for comparison with the host IPM's verbose log.

    python tools/trace_start.py c3 119
"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

if __name__ == "__main__":
    case, i = sys.argv[1], int(sys.argv[2])
    from generic_bench import IPOPT_KW
    from mpc_fatigue_amd import _lib, problems as PR
    from mpc_fatigue_amd.gocp import GOCP
    from generic_bench import _golden_q0
    batch = int(os.environ.get("MF_BATCH", "512"))  # the draws of tools/ipopt_failures.py --batch
    rng = np.random.default_rng(0)
    q0b = _golden_q0()
    sp3 = PR.box_shared_fatigue(N=100, q0=q0b)
    X3 = np.hstack([q0b[None] + rng.uniform(-0.01, 0.01, (batch, 12)), np.tile(sp3["T0"], (batch, 1))])
    sp4 = PR.centauro(N=50, T=2.0)
    X4 = np.hstack([np.asarray(sp4["q0"])[None] + rng.uniform(-0.02, 0.02, (batch, 14)), np.tile(sp4["T0"], (batch, 1))])
    X, spec = (X3, sp3) if case == "c3" else (X4, sp4)
    X = X[i:i + 1]
    g = GOCP(spec)
    _lib.lib().mf_gdebug_trace_reset()
    r = g.solve(x0=np.ascontiguousarray(X), verbose=2, **IPOPT_KW)
    buf = np.zeros(2 * 4096 * 16)
    _lib.lib().mf_gdebug_trace(buf.ctypes.data_as(C.POINTER(C.c_double)))
    np.save(os.path.join(ROOT, "gpurun_out", f"trace_{case}_{i}.npy"), buf.reshape(2, 4096, 16))
    np.save(os.path.join(ROOT, "gpurun_out", f"w_{case}_{i}.npy"), r.w[0])
    print("trace", case, i, int(r.status[0]), int(r.iters[0]), float(r.obj[0]))
