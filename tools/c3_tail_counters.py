"""Diagnostic: solver counters (mf_gdebug_counters) of the C3 shared-budget bench starts that run to the iteration cap
in IPOPT mode -- inertia corrections (extra Riccati factorisations) and restoration iterations per iteration, the
work that sets the C3 leg's tail.  Usage: python tools/c3_tail_counters.py [starts] [cap]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mpc_fatigue_amd import problems as PR  # noqa: E402
from mpc_fatigue_amd.gocp import GOCP  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
CAP = int(sys.argv[2]) if len(sys.argv) > 2 else 1500
g1 = np.loadtxt(os.path.join(ROOT, "tests", "golden", "G1_box_N50_solution.csv"), delimiter=",")[:12]
sp = PR.box_shared_fatigue(N=100, q0=g1)
rng = np.random.default_rng(0)  # tools/generic_bench.py's draw
X = np.hstack([g1[None] + rng.uniform(-0.01, 0.01, (4096, 12)), np.tile(sp["T0"], (4096, 1))])[:B]
g = GOCP(sp)
r = g.solve(x0=np.ascontiguousarray(X), init_zero=True, bound_relax=1e-8, filter=True, max_soc=4, max_iter=CAP)
print("status", {int(s): int((r.status == s).sum()) for s in np.unique(r.status)}, flush=True)
for st in (0, 1):
    idx = np.flatnonzero(r.status == st)
    if len(idx) == 0:
        continue
    C = np.array([[g.counters(int(b))[k] for k in GOCP.COUNTERS] for b in idx[:64]], float)
    it = np.maximum(C[:, 0], 1)
    print(f"status {st}: {len(idx)} starts (counters of {len(C)}): iterations {it.mean():.0f}, inertia corrections "
          f"per iteration {np.mean(C[:, 2] / it):.2f}, restoration iterations share {np.mean(C[:, 9] / it):.2f}, "
          f"restoration phases {C[:, 5].mean():.1f}, line-search failures {C[:, 3].mean():.1f}, SOC steps per "
          f"iteration {np.mean(C[:, 4] / it):.2f}", flush=True)
