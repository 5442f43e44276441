"""Op-counted FP64 work of one node evaluation of the headline path: the device's own sweep
templates (csrc/adj.hpp) run on the host with counting scalars (tests/native/flopcount.cpp) for exactly the lanes
k_eval_q (q directions, split sweep) and k_eval_node<..,1> (qd directions) run per node, plus k_eval_asm's
assembly counted from its loops.  Writes profiles/fp64_opcount.json, which bench.py's roofline.fp64 uses.

    python tools/flopcount.py [--check]     (--check: compare with the committed JSON, exit 1 on a mismatch)
"""
import ctypes as C
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
NATIVE = os.path.join(ROOT, "tests", "native")
LIB = os.path.join(NATIVE, "libflopcount.so")
OUT = os.path.join(ROOT, "profiles", "fp64_opcount.json")


def build():
    src = [os.path.join(NATIVE, "flopcount.cpp"), os.path.join(ROOT, "mpc_fatigue_amd", "csrc", "urdf.cpp")]
    deps = src + [os.path.join(ROOT, "mpc_fatigue_amd", "csrc", h) for h in ("adj.hpp", "dyn.hpp", "model.hpp")]
    if os.path.exists(LIB) and os.path.getmtime(LIB) >= max(os.path.getmtime(d) for d in deps):
        return
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    subprocess.check_call([hipcc, "-O2", "-std=c++17", "-fPIC", "-shared", "--offload-arch=gfx950",
                           "-x", "hip", src[0], "-x", "hip", src[1], "-o", LIB])


def count():
    from mpc_fatigue_amd import problems as PR
    build()
    L = C.CDLL(LIB)
    spec = PR.pilz6_bench(N=100)
    rng = np.random.default_rng(0)  # the counts do not depend on the values (no data-dependent branch but i == fp)
    q, qd = rng.uniform(-1, 1, 6), rng.uniform(-0.3, 0.3, 6)
    Fw, c, yl = np.array([20.0, 0.0, 0.0]), rng.normal(size=6), np.array([0.3, -0.2, 0.0])
    ops = np.zeros(12, dtype=np.int64)
    p = lambda a: a.ctypes.data_as(C.POINTER(C.c_double))
    n = L.flop_node(PR.read_urdf(spec["urdf"]).encode(), spec["frame"].encode(), p(q), p(qd), p(Fw), p(c), p(yl),
                    ops.ctypes.data_as(C.POINTER(C.c_longlong)))
    assert n == 6, n
    NJ, NF = 6, 1
    NV = 2 * NJ + NF
    # k_eval_asm per node: lower-triangle Hessian entries (NJ x (2 mul + add) Gauss-Newton / barrier term + the raw
    # entry), the diagonal, the cost gradient (NJ x (3 mul + add) + the qd / F terms), the per-joint weights
    tri = NV * (NV + 1) // 2
    asm = tri * (3 * NJ + 1) + NV + NV * NJ * 4 + 3 * (NJ + NF) + NJ * 8
    # the force columns / force Hessian row emitted by the q lanes (fdir . dp / d tan: 3 mul + 2 add per lane)
    emit = NJ * 5
    rec = {"kernel": "k_eval_node (k_eval_q + k_eval_node<..,1>) + k_eval_asm, Pilz 6DOF, NF = 1, NL = 2",
           "q_lanes": [int(x) for x in ops[:6]], "qd_lanes": [int(x) for x in ops[6:]],
           "sweeps": int(ops.sum()), "assembly": asm, "emit": emit,
           "fp64_ops_per_node_eval": int(ops.sum()) + asm + emit,
           "eval_phase_ops_per_node_eval": int(ops.sum()) + emit,
           "note": "one op = one FP64 add / sub / mul (an FMA = 2), counted on the device templates with counting "
                   "scalars (tests/native/flopcount.cpp); sin / cos (12 per node, once per node in LDS) not counted; "
                   "model-constant products inside the reverse sweep (plain double in adj.hpp) not counted"}
    return rec


if __name__ == "__main__":
    rec = count()
    if "--check" in sys.argv:
        with open(OUT) as f:
            old = json.load(f)
        ok = old["fp64_ops_per_node_eval"] == rec["fp64_ops_per_node_eval"]
        print("fp64_opcount", rec["fp64_ops_per_node_eval"], "committed", old["fp64_ops_per_node_eval"])
        sys.exit(0 if ok else 1)
    with open(OUT, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec))
