"""Phase-scheduled torque limits: the builders reproduce the reference's
tables (both_robots_torque_limited_2_pilz.py:120-147, Box_Pilz_6DOF.py:287-383), and the
oracle solves the single-arm C2 task under them (CPU)."""
import numpy as np

from mpc_fatigue_amd import problems as PR
from oracle import oracle as O
from oracle import pin_np as P
from oracle.urdf_np import load_urdf_file


def test_time_phase_table():
    N, T = 100, 2.0
    lo, hi = PR.time_phase_limits(N, T)
    n1, n2 = int(0.75 / (T / N)), int(1.5 / (T / N))
    assert (n1, n2) == (37, 75)
    np.testing.assert_array_equal(hi[0], [60, 30, 1000, 300, 300, 50])
    np.testing.assert_array_equal(hi[n1 - 1], [60, 30, 1000, 300, 300, 50])
    np.testing.assert_array_equal(hi[n1], [10, 100, 50, 500, 1500, 50])
    np.testing.assert_array_equal(hi[n2 - 1], [10, 100, 50, 500, 1500, 50])
    np.testing.assert_array_equal(hi[n2], [50, 110, 400, 300, 500, 50])
    np.testing.assert_array_equal(lo, -hi)


def test_box_phase_tables():
    N = 50
    lo, hi = PR.box_phase_limits(N, "right")
    k1, k2 = int(N / 3), int(2 * N / 3)
    np.testing.assert_array_equal(np.c_[lo[0, :3], hi[0, :3]], [[-200, 100], [-60, 60], [-30, 40]])
    np.testing.assert_array_equal(np.c_[lo[k1, :3], hi[k1, :3]], [[-50, 50], [-30, 10], [-20, 20]])
    np.testing.assert_array_equal(np.c_[lo[k2, :3], hi[k2, :3]], [[-5, 5], [-5, 5], [-10, 5]])
    assert np.all(hi[:, 3:] == 500) and np.all(lo[:, 3:] == -500)
    lo, hi = PR.box_phase_limits(N, "left")
    np.testing.assert_array_equal(np.c_[lo[0, :2], hi[0, :2]], [[-600, 400], [-60, 60]])
    np.testing.assert_array_equal(np.c_[lo[k1, :2], hi[k1, :2]], [[-50, 50], [-30, 40]])
    np.testing.assert_array_equal(np.c_[lo[k2, :2], hi[k2, :2]], [[-5, 5], [-5, 5]])
    assert np.all(hi[:, 2:] == 500)
    lo, hi = PR.box_phase_limits(N, "right", constrained=False)
    assert np.all(hi == 500) and np.all(lo == -500)


def test_oracle_solves_phase_scheduled_c2():
    N = 40
    ref = load_urdf_file(PR.urdf_path("pilz_robot_6DOF.urdf"))
    q0 = PR.pilz6_batch_q0(1, seed=1)[0]
    sp = PR.pilz6_phase(N=N, q0=q0, line_ref=P.forward_kinematics(ref, q0, "prbt_link_5")[0][:2])
    w, r = O.solve(ref, sp, tol=1e-8, constr_viol_tol=1e-8, max_iter=300, mu_init=0.1, F_init=PR.BENCH_F_INIT)
    assert r.status == 0
    # torques at the solution respect the per-node table (tau = ID - J^T [F;0])
    n, st = 6, 13
    for k in range(N):
        qk = w[:n] if k == 0 else w[n + (k - 1) * st + 7:n + (k - 1) * st + 13]
        qdk, Fk = w[n + k * st:n + k * st + 6], w[n + k * st + 6]
        tau = O.inverse_dynamics(ref, qk, qdk, np.zeros(n)) - O.jacobian(ref, qk, "prbt_link_5").T @ np.r_[Fk, 0, 0, 0, 0, 0]
        assert np.all(tau <= sp["tau_hi"][k] + 1e-6) and np.all(tau >= sp["tau_lo"][k] - 1e-6)
