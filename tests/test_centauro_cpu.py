"""Centauro thermal box lift (C4, python/Centauro_script/RepeatedMPCwithThermal.py) on the CPU: the
reference's committed Centauro solutions pin the invariant checks, the oracle's node derivatives are
checked by finite differences, and the oracle solves on the substitute arms satisfy the same invariants
plus the relative-pose and equilibrium rows.  The URDF is absent from the reference, so trajectories
themselves are parity-unpinned."""
import os

import numpy as np

from mpc_fatigue_amd import problems as PR
from mpc_fatigue_amd.solution_io import centauro_invariants, centauro_split, read_solution_csv
from oracle import cpu_fast as CF
from oracle import generic as G
from oracle import pin_np as P
from oracle.urdf_np import load_urdf_file
from tests.conftest import GOLDEN
from tests.test_oracle_generic import _fd_check


def test_reference_centauro_solution_invariants():
    """Centauro_solutions/FullPosition/Both/solution.csv (N = 50, T = 2, m = 10, equilibrium rows
    within +-0.001): continuity at the solver tolerance and the box's force balance."""
    w = read_solution_csv(os.path.join(GOLDEN, "centauro_fullposition_both_N50_solution.csv"))
    assert w.size == 50 * 34 + 14
    inv = centauro_invariants(w, 50, 2.0 / 50, 98.1, thermal=False)
    assert inv["continuity"] < 2.5e-8
    assert inv["force_z"] < 1e-3 + 1e-8 and inv["force_xy"] < 1e-3 + 1e-8


def test_centauro_node_derivatives_fd():
    spec = PR.centauro(N=1)
    rng = np.random.default_rng(0)
    q0 = np.asarray(spec["q0"])
    xu = np.r_[q0 + 0.1 * rng.normal(size=14), 20 + 5 * rng.normal(size=14), 0.5 * rng.normal(size=14),
               [1.0, 2.0, 49.0], [-1.0, 0.5, 48.0]]
    _fd_check(spec, xu, 14, 12, 28)


def _models():
    u = os.path.join(os.path.dirname(PR.urdf_path("x")))
    return [load_urdf_file(os.path.join(u, f"centauro_substitute_arm{k}.urdf")) for k in (1, 2)]


def relpose(ms, q):
    pL, RL = P.forward_kinematics(ms[0], q[:7], "mass1_ee")
    pR, RR = P.forward_kinematics(ms[1], q[7:], "mass2_ee")
    Ro = RL @ RR.T
    return np.r_[RL.T @ (pR - pL), 0.5 * (Ro[2, 1] - Ro[1, 2]), 0.5 * (Ro[2, 0] - Ro[0, 2]), 0.5 * (Ro[1, 0] - Ro[0, 1])], pL, pR


def check_solution(spec, w, tol=1e-7):
    N, ms = spec["N"], _models()
    inv = centauro_invariants(w, N, spec["h"], spec["box_mg"])
    assert inv["continuity"] < 1e-9 and inv["force_z"] < tol and inv["force_xy"] < tol, inv
    b = centauro_split(w, N)
    r0, _, _ = relpose(ms, b["q"][0])
    for k in range(1, N):
        rk, pL, pR = relpose(ms, b["q"][k])
        assert np.abs(rk - r0).max() < tol, k
        m = np.cross(pL - pR, b["F"][k, :3] - b["F"][k, 3:])
        assert np.abs(m).max() < tol
    assert (b["T"][1:] <= 80 + 1e-6).all() and (b["T"][1:] >= -1e-6).all()
    return b


def test_centauro_oracle_solve_invariants():
    spec = PR.centauro(N=10)
    w, r = G.solve(spec, u_init=PR.centauro_u_init(spec), max_iter=500, max_soc=4)
    assert r.status == 0, (r.status, r.iter)
    b = check_solution(spec, w)
    assert b["T"][-1].max() > 20.0  # the windings heat up


def test_centauro_fast_nodes_reproduce_hyperdual():
    spec = PR.centauro(N=10)
    kw = dict(u_init=PR.centauro_u_init(spec), max_iter=500, max_soc=4)
    w0, r0 = G.solve(spec, **kw)
    w1, r1 = G.solve(spec, **kw, **CF.FastNodes(spec).opts_kw())
    assert (r0.status, r0.iter) == (r1.status, r1.iter)
    assert np.abs(w0 - w1).max() < 1e-7
