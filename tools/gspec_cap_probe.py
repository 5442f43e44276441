"""Diagnostic: the generic solver's launch policy per family (verbose lines of mf_gsolve: the running count from
which k_gspec's concurrent inertia tries start, the k_gkkt occupancy-variant threshold).  One IPOPT-mode iteration
on two starts of C3 (box), C4 (Centauro) and C2 (chain)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mpc_fatigue_amd import pin  # noqa: E402
from mpc_fatigue_amd import problems as PR  # noqa: E402
from mpc_fatigue_amd.gocp import GOCP  # noqa: E402

IP = dict(init_zero=True, bound_relax=1e-8, filter=True, max_soc=4, max_iter=1, verbose=True)
g1 = np.loadtxt(os.path.join(ROOT, "tests", "golden", "G1_box_N50_solution.csv"), delimiter=",")[:12]
sp3 = PR.box_shared_fatigue(N=100, q0=g1)
X3 = np.hstack([np.tile(g1, (2, 1)), np.tile(sp3["T0"], (2, 1))])
sp4 = PR.centauro(N=50, T=2.0)
X4 = np.hstack([np.tile(sp4["q0"], (2, 1)), np.tile(sp4["T0"], (2, 1))])
sp2 = PR.pilz6_bench(N=100)
X2 = PR.pilz6_batch_q0(2, seed=0)
L2 = pin.generate_forward_kin(PR.read_urdf(sp2["urdf"]), sp2["frame"]).batch(X2)[0][:, :2]
for name, sp, X, lr in (("C3", sp3, X3, None), ("C4", sp4, X4, None), ("C2", sp2, X2, np.ascontiguousarray(L2))):
    print(name, flush=True)
    GOCP(sp).solve(x0=np.ascontiguousarray(X), line_ref=lr, **IP)
