"""Host side of the receding-horizon loop: the w-layout split and the
restart state of mpc_principal.py:357-377, and the oracle's warm start (CPU only)."""
import numpy as np

from mpc_fatigue_amd import problems as PR
from mpc_fatigue_amd.mpc import next_initial_state, split_w
from oracle import oracle as O
from oracle import pin_np as P
from oracle.urdf_np import load_urdf_file


def test_split_w_layout():
    n, nf, N = 6, 1, 3
    w = np.arange(n + N * (2 * n + nf), dtype=float)[None]
    q, qd, F = split_w(w, n, nf, N)
    assert q.shape == (1, N + 1, n) and qd.shape == (1, N, n) and F.shape == (1, N, nf)
    assert q[0, 0, 0] == 0 and qd[0, 0, 0] == n and F[0, 0, 0] == 2 * n and q[0, 1, 0] == 2 * n + nf
    qN, qdl = next_initial_state(w, n, nf, N)
    np.testing.assert_array_equal(qN[0], q[0, N])
    np.testing.assert_array_equal(qdl[0], qd[0, N - 1])



def test_oracle_warm_start_from_solution():
    """Warm-starting from a converged solution (multipliers cold) converges to the same point."""
    N = 10
    spec = PR.pilz6_bench(N=N)
    ref = load_urdf_file(PR.urdf_path(spec["urdf"]))
    q0 = PR.pilz6_batch_q0(1, seed=2)[0]
    sp = PR.pilz6_bench(N=N, q0=q0, line_ref=P.forward_kinematics(ref, q0, "prbt_link_5")[0][:2])
    opts = dict(tol=1e-8, constr_viol_tol=1e-8, max_iter=300, mu_init=0.1, F_init=PR.BENCH_F_INIT)
    w1, r1 = O.solve(ref, sp, **opts)
    w2, r2 = O.solve(ref, sp, w0=w1, **opts)
    assert r1.status == 0 and r2.status == 0
    np.testing.assert_allclose(w2, w1, atol=1e-6)


def test_oracle_warm_start_constants_from_solution():
    """IPOPT warm_start_init_point (push 1e-3, bound multipliers 1e-3) from a converged solution: converges in
    fewer iterations than the cold constants and to the same point."""
    N = 10
    spec = PR.pilz6_bench(N=N)
    ref = load_urdf_file(PR.urdf_path(spec["urdf"]))
    q0 = PR.pilz6_batch_q0(1, seed=2)[0]
    sp = PR.pilz6_bench(N=N, q0=q0, line_ref=P.forward_kinematics(ref, q0, "prbt_link_5")[0][:2])
    opts = dict(tol=1e-8, constr_viol_tol=1e-8, max_iter=300, mu_init=0.1, F_init=PR.BENCH_F_INIT)
    w1, r1 = O.solve(ref, sp, **opts)
    w2, r2 = O.solve(ref, sp, w0=w1, warm_start=True, **opts)
    assert r1.status == 0 and r2.status == 0
    np.testing.assert_allclose(w2, w1, atol=1e-6)


def test_oracle_receding_horizon_converges_every_step():
    """The C2 loop of mpc.RecedingHorizon on the oracle (line re-anchored at each q_0, restart at rest, IPOPT
    warm-start constants): every horizon of every restart converges."""
    N, B, steps = 20, 4, 3
    spec = PR.pilz6_bench(N=N)
    ref = load_urdf_file(PR.urdf_path(spec["urdf"]))
    opts = dict(tol=1e-8, constr_viol_tol=1e-8, max_iter=300, mu_init=0.1, F_init=PR.BENCH_F_INIT)
    for q0 in PR.pilz6_batch_q0(B, seed=5):
        w0 = None
        for s in range(steps):
            sp = PR.pilz6_bench(N=N, q0=q0, line_ref=P.forward_kinematics(ref, q0, "prbt_link_5")[0][:2])
            w, r = O.solve(ref, sp, w0=w0, warm_start=w0 is not None, **opts)
            assert r.status == 0, (s, r.status, r.iter)
            qN, _ = next_initial_state(w, 6, 1, N)
            q0, w0 = qN[0], w


def test_generic_restart_state_rules():
    """restart_state: x_0 <- x_N with T - 0.05, qd_0 <- qd_{N-1}, 4-decimal rounding
    (mpc_principal.py:365-373), numpy path (GRecedingHorizon.next_initial on the device)."""
    from mpc_fatigue_amd.mpc import restart_state

    n, nx, nu, N = 3, 6, 3, 3
    w = np.random.default_rng(0).normal(size=(2, nx + N * (nu + nx)))
    x0, u0 = restart_state(w, nx, nu, N, n, True)
    off = nx + (N - 1) * (nu + nx)
    xN = w[:, off + nu:off + nu + nx]
    np.testing.assert_array_equal(x0[:, :3], np.round(xN[:, :3], 4))
    np.testing.assert_array_equal(x0[:, 3:], np.round(xN[:, 3:] - 0.05, 4))
    np.testing.assert_array_equal(u0, np.round(w[:, off:off + nu], 4))
    x0, u0 = restart_state(w, nx, nu, N, n, True, carry_velocity=False, decimals=None)
    np.testing.assert_array_equal(u0, 0.0 * w[:, off:off + nu])
    np.testing.assert_array_equal(x0[:, 3:], xN[:, 3:] - 0.05)
    import torch
    xt, ut = restart_state(torch.from_numpy(w), nx, nu, N, n, True)
    np.testing.assert_array_equal(xt.numpy(), restart_state(w, nx, nu, N, n, True)[0])
