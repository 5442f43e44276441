"""The CPU baseline's solver (oracle/cpu_fast.py: the product's node functions compiled for the host,
plugged into the generic oracle IPM) is the same algorithm as the hyper-dual checker: same iterates to
rounding, same iteration counts, and on the dual-arm box the same reference trajectory (G1)."""
import time

import numpy as np
import pytest

from mpc_fatigue_amd import problems as PR
from oracle import cpu_fast as CF
from oracle import generic as G
from tests.test_oracle_generic import box_homotopy, q_traj

KW = dict(tol=1e-8, constr_viol_tol=1e-8, max_iter=300, mu_init=0.1)


@pytest.mark.parametrize("make", [lambda: PR.pilz6_bench(N=20), lambda: PR.pilz6_thermal(N=20)])
def test_fast_nodes_reproduce_hyperdual_solve(make):
    spec = make()
    kw = dict(KW, F_init=PR.BENCH_F_INIT) if not spec.get("thermal") else KW
    w0, r0 = G.solve(spec, **kw)
    w1, r1 = G.solve(spec, **kw, **CF.FastNodes(spec).opts_kw())
    assert (r0.status, r0.iter) == (r1.status, r1.iter)
    assert r0.status == 0
    assert np.abs(w0 - w1).max() < 1e-7


def test_fast_nodes_box_resolve_matches_reference(golden):
    g, N = golden["G1_box_N50"]
    spec = PR.box_dual(q0=g[:12], N=N)
    w, res = box_homotopy(spec, **CF.FastNodes(spec).opts_kw())
    assert all(r.status == 0 for r in res)
    assert np.abs(q_traj(w, N) - q_traj(g, N)).max() < 1e-6


def test_fast_nodes_batch_threads_agree():
    """OpenMP over horizons: the shared read-only node context gives the same answers per thread count."""
    Q = PR.pilz6_batch_q0(8, seed=3)
    specs = [PR.pilz6_bench(N=12, q0=q) for q in Q]
    fn = CF.FastNodes(specs[0])
    w1, R1 = CF.solve_batch(specs, nthreads=1, F_init=PR.BENCH_F_INIT, **KW, **fn.opts_kw())
    w4, R4 = CF.solve_batch(specs, nthreads=4, F_init=PR.BENCH_F_INIT, **KW, **fn.opts_kw())
    w0, R0 = G.solve_batch(specs, nthreads=4, F_init=PR.BENCH_F_INIT, **KW)  # the checker (hyper-dual, -O2)
    assert [r.iter for r in R0] == [r.iter for r in R4]
    assert np.abs(w0 - w4).max() < 1e-7
    assert np.array_equal(w1, w4)
    assert [r.iter for r in R1] == [r.iter for r in R4]
