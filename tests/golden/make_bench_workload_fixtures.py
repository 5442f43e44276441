"""Generates tests/golden/bench_{c3,c4}_{i}.csv and tests/golden/ipopt_mode_C3sf.csv: the hyper-dual oracle's
(oracle/mf_ocp.c, its own dual-number node derivatives) IPOPT-mode solutions of the generic bench workloads
(tools/generic_bench.py, BASELINE configs 3 and 4):

  bench_c3_{0,1}     C3 shared fatigue budget, N = 100, q0 = the reference's IK start (tests/golden G1) + U(-0.01, 0.01)
  bench_c4_{0,1,2}   C4 Centauro, N = 50, T = 2 s, q0 = the IK start + U(-0.02, 0.02)
  ipopt_mode_C3sf    C3 shared fatigue budget, N = 100, from the unperturbed G1 start

each solved as the reference solves (Box_Pilz_6DOF.py:455-456, RepeatedMPCwithThermal.py:464-466): IPOPT from
x0 = 0 with the filter globalisation (IPOPT's restoration phase: elastic variables on every row, the dynamics rows
included) and bound_relax_factor 1e-8, the KKT factored by the device's Riccati elimination (riccati = 2).  The perturbations are numpy default_rng(0) draws; each file holds the full decision
vector w, whose first nx entries are the start x_0, so the GPU tests read the starts back from the fixtures.
tests/test_gpu_generic.py compares the device against these (the hyper-dual oracle takes minutes per C3 horizon,
too slow for the GPU box).

Run:  python tests/golden/make_bench_workload_fixtures.py   (about 10 min on 6 processes)
"""
import os
import sys
from multiprocessing import Pool

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from mpc_fatigue_amd import problems as PR  # noqa: E402

IPOPT_MODE = dict(init_zero=True, bound_relax=1e-8, max_iter=3000, max_soc=4, filter=True, resto_hard_dyn=False,
                  riccati=2)


def jobs():
    rng = np.random.default_rng(0)
    q0b = np.loadtxt(os.path.join(HERE, "G1_box_N50_solution.csv"), delimiter=",")[:12]
    sp3 = PR.box_shared_fatigue(N=100, q0=q0b)
    out = [("ipopt_mode_C3sf", sp3)]
    for i, d in enumerate(rng.uniform(-0.01, 0.01, (2, 12))):
        out.append((f"bench_c3_{i}", dict(sp3, q0=list(q0b + d))))
    sp4 = PR.centauro(N=50, T=2.0)
    q0c = np.asarray(sp4["q0"])
    for i, d in enumerate(rng.uniform(-0.02, 0.02, (3, 14))):
        out.append((f"bench_c4_{i}", dict(sp4, q0=list(q0c + d))))
    return out


def run(job):
    from oracle import generic as G
    name, spec = job
    w, r = G.solve(spec, **IPOPT_MODE)
    assert r.status == 0, (name, r.status, r.iter)
    np.savetxt(os.path.join(HERE, f"{name}.csv"), w[None], delimiter=",", fmt="%.17g")
    return name, r.iter, r.obj


if __name__ == "__main__":
    os.environ.setdefault("OMP_NUM_THREADS", "1")
    with Pool(6) as p:
        for name, it, obj in p.imap_unordered(run, jobs()):
            print(name, it, obj, flush=True)
