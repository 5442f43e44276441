"""The oracle's Riccati elimination in IPOPT's restoration phase (oracle/mf_ocp.c ric_relax):
the elastic p, n on the dynamics rows relax dx_{k+1} = A dx_k + B du_k + r into ... - D_r dlam_k, which the
stage recursion absorbs through L = I + P D_r.  riccati = 3 factors and solves every restoration step both
ways (block-tridiagonal Bunch-Kaufman and the Riccati recursion) and records the largest difference of the
primal-dual steps relative to their size; the restoration problem follows IpRestoIpoptNLP.cpp (elastic
variables on every row) or, with resto_hard_dyn, keeps the dynamics rows exact (the device's variant).
Horizon 2 of the C2 bench batch (force_optimization_pilz_6DOF.py, N = 100, IPOPT mode from x0 = 0) enters
the restoration phase.  CPU only."""
import numpy as np
import pytest

from mpc_fatigue_amd import problems as PR
from oracle import generic as G

IPOPT_KW = dict(init_zero=True, bound_relax=1e-8, filter=True, max_iter=3000, max_soc=4)


@pytest.fixture(scope="module")
def c2_spec():
    from oracle import pin_np as P
    from oracle.urdf_np import load_urdf_file
    base = PR.pilz6_bench(N=100)
    ref = load_urdf_file(PR.urdf_path(base["urdf"]))
    q0 = PR.pilz6_batch_q0(3, seed=0)[2]
    lr = P.forward_kinematics(ref, q0, "prbt_link_5")[0][:2]
    return PR.pilz6_bench(N=100, q0=q0, line_ref=lr)


@pytest.mark.parametrize("hard_dyn", [False, True], ids=["elastic_dynamics", "hard_dynamics"])
def test_restoration_riccati_steps_equal_banded(c2_spec, hard_dyn):
    L = G.lib()
    L.mfg_ric_check_max(1)
    _, R = G.solve_batch([c2_spec], nthreads=1, riccati=3, resto_hard_dyn=hard_dyn, **IPOPT_KW)
    diff = L.mfg_ric_check_max(1)
    assert R[0].status == 0, R[0].status
    assert 0.0 < diff < 1e-8, diff   # > 0: the restoration phase ran and was checked
