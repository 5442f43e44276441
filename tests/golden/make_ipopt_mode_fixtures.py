"""Generates tests/golden/ipopt_mode_*.csv: the oracle's (oracle/mf_ocp.c) IPOPT-mode solutions, solved as the
reference solves -- IPOPT from x0 = 0, no homotopy -- with IPOPT's globalisation (filter line search, watchdog, soft
restoration, and IPOPT's restoration phase: elastic p, n on every constraint row, the dynamics rows included) and
bound_relax_factor 1e-8, the KKT factored by the device's Riccati elimination (riccati = 2: ric_relax in the
restoration phase).

  ipopt_mode_G{1,2,3,4}   the dual-arm box task Box_Pilz_6DOF.py (L455-456) from each reference solution's own q_0;
                          G1, G2, G4 equal the reference's own IPOPT solutions (plotter/solution.csv, Result_2,
                          Result_1) to <= 3e-8 rad; G3 is a neighbouring local minimum of Result_4's problem
  ipopt_mode_C2_{41,45,48} C2 (force_optimization_pilz_6DOF.py:195-197) on horizons 41, 45, 48 of the bench batch
                          (pilz6_batch_q0(64, seed=0), line reference fk(q0)): the starts whose restoration fails when
                          the dynamics rows are kept exact (the build's variant before round 5)

The device solver (csrc/gipm.hip, filter mode) is checked against these in tests/test_gpu_generic.py, so the GPU
tests need not run the slow hyper-dual checker.  tests/test_oracle_generic.py re-derives G1 and G4 on every CPU run.

Run:  python tests/golden/make_ipopt_mode_fixtures.py [case ...]   (a few minutes per case, 7 processes)
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from mpc_fatigue_amd import problems as PR  # noqa: E402
from oracle import generic as G  # noqa: E402

IPOPT_MODE = dict(init_zero=True, bound_relax=1e-8, max_iter=3000, max_soc=4, filter=True, resto_hard_dyn=False,
                  riccati=2)
CASES = {"G1": ("G1_box_N50", dict(N=50)), "G2": ("G2_box_N80", dict(N=80)),
         "G3": ("G3_box_N80", dict(N=80, left_const=True)), "G4": ("G4_box_N80", dict(N=80, right_const=False)),
         "C2_41": (41, None), "C2_45": (45, None), "C2_48": (48, None)}


def c2_spec(i):
    from oracle import pin_np as P
    from oracle.urdf_np import load_urdf_file
    base = PR.pilz6_bench(N=100)
    q0 = PR.pilz6_batch_q0(64, seed=0)[i]
    lr = P.forward_kinematics(load_urdf_file(PR.urdf_path(base["urdf"])), q0, "prbt_link_5")[0][:2]
    return PR.pilz6_bench(N=100, q0=q0, line_ref=lr)


def run(c):
    from oracle import generic as G
    name, kw = CASES[c]
    if kw is None:
        spec = c2_spec(name)
    else:
        g = np.loadtxt(os.path.join(HERE, f"{name}_solution.csv"), delimiter=",")
        spec = PR.box_dual(q0=g[:12], **kw)
    w, r = G.solve(spec, **IPOPT_MODE)
    assert r.status == 0, (c, r.status, r.iter)
    np.savetxt(os.path.join(HERE, f"ipopt_mode_{c}.csv"), w[None], delimiter=",", fmt="%.17g")
    return c, r.iter, r.obj


if __name__ == "__main__":
    from multiprocessing import Pool
    os.environ.setdefault("OMP_NUM_THREADS", "1")
    import json
    jf = os.path.join(HERE, "ipopt_mode_fixtures.json")  # the oracle's iteration counts and objectives
    meta = json.load(open(jf)) if os.path.exists(jf) else {}
    with Pool(7) as p:
        for c, it, obj in p.imap_unordered(run, sys.argv[1:] or list(CASES)):
            print(c, it, obj, flush=True)
            meta[c] = {"iter": it, "obj": obj}
    json.dump(dict(sorted(meta.items())), open(jf, "w"), indent=1)
