"""Generates tests/golden/ipopt_mode_G{1,2,3,4}.csv: the oracle's (oracle/mf_ocp.c) IPOPT-mode solutions of the
reference's dual-arm box task Box_Pilz_6DOF.py, solved as L455-456 solve it -- IPOPT from x0 = 0, no homotopy --
with IPOPT's globalisation (filter line search, watchdog, soft restoration, restoration phase with the dynamics
rows exact: the device's variant) and bound_relax_factor 1e-8, from each reference solution's own q_0.

The device solver (csrc/gipm.hip, filter mode) is checked against these in tests/test_gpu_generic.py, so the GPU
tests need not run the slow hyper-dual checker.  G1, G2, G4 equal the reference's own IPOPT solutions
(plotter/solution.csv, Result_2, Result_1) to <= 3e-8 rad; G3 is a neighbouring local minimum of Result_4's problem
(objective 1505.98 against 1506.78).  tests/test_oracle_generic.py re-derives G1 and G4 on every CPU run.

Run:  python tests/golden/make_ipopt_mode_fixtures.py   (about 1 min per case on 8 threads)
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from mpc_fatigue_amd import problems as PR  # noqa: E402
from oracle import generic as G  # noqa: E402

IPOPT_MODE = dict(init_zero=True, bound_relax=1e-8, max_iter=1500, max_soc=4, filter=True, resto_hard_dyn=True)
CASES = {"G1": ("G1_box_N50", dict(N=50)), "G2": ("G2_box_N80", dict(N=80)),
         "G3": ("G3_box_N80", dict(N=80, left_const=True)), "G4": ("G4_box_N80", dict(N=80, right_const=False))}

if __name__ == "__main__":
    for c in (sys.argv[1:] or list(CASES)):
        name, kw = CASES[c]
        g = np.loadtxt(os.path.join(HERE, f"{name}_solution.csv"), delimiter=",")
        w, r = G.solve(PR.box_dual(q0=g[:12], **kw), **IPOPT_MODE)
        assert r.status == 0, (c, r.status, r.iter)
        np.savetxt(os.path.join(HERE, f"ipopt_mode_{c}.csv"), w[None], delimiter=",", fmt="%.17g")
        print(c, r.iter, r.obj)
