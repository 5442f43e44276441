"""Pins the oracle (oracle/) against the reference's own committed IPOPT solutions.

The reference has no tests; its only numeric pins are the
dual-arm Box_Pilz_6DOF solutions (plotter/solution.csv, plotter/Result_{2,4,1}/
solution.csv, copied to tests/golden/).  Layout per node k:
[q(12), qd(12), F_L(3), F_R(3)] x N + q_N(12)   (Box_Pilz_6DOF.py:213-436).
Constraints they satisfy at IPOPT tolerance, re-evaluated here with the oracle's
FK / Jacobian / RNEA (so a wrong model fails these tests):
  * distance |E1 - E2|^2 = 0.04 at every node        (Box_Pilz_6DOF.py:279-282)
  * moment equilibrium within +-1e-4                 (Box_Pilz_6DOF.py:273-277)
  * IK start at (0.2,0.6,0.4) / (0.4,0.6,0.4) with the reference orientations (L96-156)
  * phase-scheduled torque limits of the right arm are ACTIVE in the last third:
    tau = ID - J^T [F;0] sits on a bound to IPOPT precision   (Box_Pilz_6DOF.py:287-349)
"""
import os

import numpy as np
import pytest

from oracle import oracle as O
from oracle import pin_np as P
from oracle.urdf_np import load_urdf_file
from tests.conftest import ROOT

URDF = os.path.join(ROOT, "mpc_fatigue_amd", "urdf")


@pytest.fixture(scope="module")
def arms():
    return (load_urdf_file(os.path.join(URDF, "pilz_robot_6DOF_first.urdf")),
            load_urdf_file(os.path.join(URDF, "pilz_robot_6DOF_second.urdf")))


def nodes(sol, N):
    n = 30
    for k in range(N):
        yield k, sol[k * n:k * n + 12], sol[k * n + 12:k * n + 24], sol[k * n + 24:k * n + 30]


@pytest.mark.parametrize("name", ["G1_box_N50", "G2_box_N80", "G3_box_N80", "G4_box_N80"])
@pytest.mark.parametrize("impl", ["numpy", "c"])
def test_distance_and_moment_pins(golden, arms, name, impl):
    sol, N = golden[name]
    mf, ms = arms
    fk = P.forward_kinematics if impl == "numpy" else O.forward_kinematics
    for k, q, qd, F in nodes(sol, N):
        E1, _ = fk(mf, q[:6], "end_effector")
        E2, _ = fk(ms, q[6:], "end_effector")
        d = E1 - E2
        # k = 0, 1 carry the fixed IK start (q_1 = q_0 + h*0); later nodes are IPOPT-tight
        assert abs(d @ d - 0.04) < (1e-10 if k <= 1 else 1e-11)
        mom = np.cross(d, F[:3] - F[3:])
        assert np.all(np.abs(mom) <= 1e-4 + 1e-7)  # IPOPT relaxes bounds by ~1e-8 relative


def test_ik_start_pin(golden, arms):
    sol, _ = golden["G1_box_N50"]
    mf, ms = arms
    p1, R1 = P.forward_kinematics(mf, sol[:6], "end_effector")
    p2, R2 = P.forward_kinematics(ms, sol[6:12], "end_effector")
    np.testing.assert_allclose(p1, [0.2, 0.6, 0.4], atol=1e-8)
    np.testing.assert_allclose(p2, [0.4, 0.6, 0.4], atol=1e-8)
    np.testing.assert_allclose(R1, [[0, 0, 1], [0, 1, 0], [-1, 0, 0]], atol=1e-8)
    np.testing.assert_allclose(R2, [[0, 0, -1], [0, 1, 0], [1, 0, 0]], atol=1e-8)


# final-third bounds of the right arm, joints 0..2 (Box_Pilz_6DOF.py:311-349)
RR_LAST = np.array([[-5.0, 5.0], [-5.0, 5.0], [-10.0, 5.0]])


@pytest.mark.parametrize("name,active", [("G1_box_N50", True), ("G2_box_N80", True), ("G3_box_N80", True),
                                         ("G4_box_N80", False)])
def test_active_torque_bounds_pin_rnea_and_jacobian(golden, arms, name, active):
    sol, N = golden[name]
    _, ms = arms
    worst = 0.0
    for k, q, qd, F in nodes(sol, N):
        W = np.r_[F[3:], 0, 0, 0]
        tau = O.inverse_dynamics(ms, q[6:], qd[6:], np.zeros(6)) - O.jacobian(ms, q[6:], "end_effector").T @ W
        tau_np = P.inverse_dynamics(ms, q[6:], qd[6:], np.zeros(6)) - P.jacobian(ms, q[6:], "end_effector").T @ W
        np.testing.assert_allclose(tau, tau_np, atol=1e-10)
        if active and k >= int(0.75 * N):
            # last phase (k >= 2N/3): after a few transition nodes all three joints sit on a bound
            dist = np.abs(tau[:3, None] - RR_LAST).min(1)  # distance to the nearest bound
            worst = max(worst, dist.max())
            assert np.all(tau[:3] >= RR_LAST[:, 0] - 1e-6) and np.all(tau[:3] <= RR_LAST[:, 1] + 1e-6)
        if not active:
            assert np.all(np.abs(tau) <= 500 + 1e-6)
    if active:
        assert worst < 1e-6, worst


def test_c_oracle_matches_numpy_restatement():
    rng = np.random.default_rng(3)
    for f in ["pilz_robot_6DOF.urdf", "pilz_robot_3DOF.urdf", "pilz_robot_6DOF_second.urdf"]:
        m = load_urdf_file(os.path.join(URDF, f))
        frame = "end_effector" if "second" in f else "prbt_link_5"
        for _ in range(5):
            q, qd, qdd = rng.normal(size=(3, m.nq))
            np.testing.assert_allclose(O.inverse_dynamics(m, q, qd, qdd), P.inverse_dynamics(m, q, qd, qdd), atol=1e-12)
            p1, R1 = O.forward_kinematics(m, q, frame)
            p2, R2 = P.forward_kinematics(m, q, frame)
            np.testing.assert_allclose(p1, p2, atol=1e-14)
            np.testing.assert_allclose(R1, R2, atol=1e-14)
            np.testing.assert_allclose(O.jacobian(m, q, frame), P.jacobian(m, q, frame), atol=1e-14)


def test_fixed_joint_merging_3dof():
    """pilz_robot_3DOF.urdf: joints 4-6 fixed -> 3 DoF, links 4/5/flange merged into joint 3's body."""
    m3 = load_urdf_file(os.path.join(URDF, "pilz_robot_3DOF.urdf"))
    m6 = load_urdf_file(os.path.join(URDF, "pilz_robot_6DOF.urdf"))
    assert m3.nq == 3
    q3 = np.array([0.3, -0.7, 1.1])
    # gravity torque of the merged model equals the 6-DOF model with joints 4-6 at 0
    t3 = P.inverse_dynamics(m3, q3, np.zeros(3), np.zeros(3))
    t6 = P.inverse_dynamics(m6, np.r_[q3, 0, 0, 0], np.zeros(6), np.zeros(6))
    np.testing.assert_allclose(t3, t6[:3], atol=1e-12)
    np.testing.assert_allclose(P.forward_kinematics(m3, q3, "prbt_link_5")[0],
                               P.forward_kinematics(m6, np.r_[q3, 0, 0, 0], "prbt_link_5")[0], atol=1e-14)


def test_node_derivatives_finite_differences():
    from mpc_fatigue_amd import problems as PR
    m = load_urdf_file(os.path.join(URDF, "pilz_robot_6DOF.urdf"))
    spec = PR.pilz6_force(N=1)
    rng = np.random.default_rng(1)
    q, qd = rng.normal(size=(2, 6))
    F = np.array([3.0])
    cw, yl = rng.normal(size=6), rng.normal(size=2)
    _, Jt, _, Jp, H = O.node_derivs(m, spec, q, qd, F, cw, yl)
    x = np.r_[q, qd, F]

    def grad(x):
        _, J, _, Jp_, _ = O.node_derivs(m, spec, x[:6], x[6:12], x[12:], cw, yl)
        return cw @ J + np.r_[yl @ Jp_[:2], np.zeros(7)]

    def tau(x):
        return O.node_derivs(m, spec, x[:6], x[6:12], x[12:], cw, yl)[0]

    eps = 1e-6
    Jfd = np.array([(tau(x + eps * e) - tau(x - eps * e)) / (2 * eps) for e in np.eye(13)]).T
    Hfd = np.array([(grad(x + eps * e) - grad(x - eps * e)) / (2 * eps) for e in np.eye(13)])
    np.testing.assert_allclose(Jt, Jfd, atol=1e-7)
    np.testing.assert_allclose(H, Hfd, atol=1e-6)
    np.testing.assert_allclose(H, H.T, atol=1e-12)
