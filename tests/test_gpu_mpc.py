"""GPU parity of the warm-started solve and the receding-horizon loop (SURVEY.md s.8 a14,
mpc_principal.py:357-377, RepeatedMPCwithThermal.py:445-487) against the oracle run through
the same loop (oracle/mf_oracle.c warm start: q_k, qd_k (k >= 1), F_k from x0, pushed into
their bounds with IPOPT's warm_start_init_point constants: push 1e-3, bound multipliers 1e-3,
constraint multipliers 0).

Each oracle step starts from the GPU's previous solution (q_N and the warm start), so every
step compares one solve on identical inputs.  Tolerance 1e-6 on the cold step and the single
warm-started solve, 1e-5 on warm steps of the loop; the reference's own target is 1e-4 rad.
"""
import numpy as np
import pytest

from mpc_fatigue_amd import problems as PR
from mpc_fatigue_amd.mpc import RecedingHorizon, next_initial_state
from oracle import oracle as O
from oracle import pin_np as P
from oracle.urdf_np import load_urdf_file

pytestmark = pytest.mark.gpu
OPTS = dict(tol=1e-8, constr_viol_tol=1e-8, max_iter=300, mu_init=0.1, F_init=PR.BENCH_F_INIT)


@pytest.mark.parametrize("warm", [False, True])
def test_warm_start_per_problem_qd0_matches_oracle(warm):
    """mf_solve_batch_ws with a per-problem qd_0 and a warm start, one solve (cold constants or IPOPT's
    warm_start_init_point constants)."""
    N, B = 16, 3
    spec = PR.pilz6_bench(N=N)
    ref = load_urdf_file(PR.urdf_path(spec["urdf"]))
    Q0 = PR.pilz6_batch_q0(B, seed=9)
    LR = np.array([P.forward_kinematics(ref, q, "prbt_link_5")[0][:2] for q in Q0])
    rng = np.random.default_rng(1)
    QD0 = rng.uniform(-0.05, 0.05, size=(B, 6))
    cold = [O.solve(ref, PR.pilz6_bench(N=N, q0=Q0[b], line_ref=LR[b]), **OPTS)[0] for b in range(B)]
    W0 = np.array(cold) + rng.uniform(-1e-3, 1e-3, size=(B, len(cold[0])))
    from mpc_fatigue_amd.ocp import OCP
    res = OCP(spec).solve_ws(Q0, qd0=QD0, w0=W0, line_ref=LR, warm_start=warm, **OPTS)
    for b in range(B):
        sp = PR.pilz6_bench(N=N, q0=Q0[b], line_ref=LR[b])
        sp["qd0"] = QD0[b]
        w, r = O.solve(ref, sp, w0=W0[b], warm_start=warm, **OPTS)
        assert r.status == res.status[b], (b, r.status, res.status[b])
        if r.status == 0:
            np.testing.assert_allclose(res.w[b], w, atol=1e-6)


def test_receding_horizon_matches_oracle():
    """C2 restarted as mpc_principal.py:357-377 (q_0 <- q_N, warm start = the previous solution with IPOPT's
    warm_start_init_point constants), each horizon's line anchored at its own q_0 (mpc.RecedingHorizon
    reanchor_line) and restarted at rest: every step of every horizon converges, GPU = oracle."""
    N, B, steps = 20, 4, 3
    spec = PR.pilz6_bench(N=N)
    ref = load_urdf_file(PR.urdf_path(spec["urdf"]))
    Q0 = PR.pilz6_batch_q0(B, seed=5)
    gpu = RecedingHorizon(spec, carry_velocity=False, reanchor_line=True, **OPTS).run(Q0, steps)
    n, nf = 6, 1
    for b in range(B):
        q0, w0 = Q0[b], None
        for s in range(steps):
            lr = P.forward_kinematics(ref, q0, "prbt_link_5")[0][:2]
            sp = PR.pilz6_bench(N=N, q0=q0, line_ref=lr)
            w, r = O.solve(ref, sp, w0=w0, warm_start=w0 is not None, **OPTS)
            assert r.status == 0 and gpu[s].status[b] == 0, (b, s, r.status, gpu[s].status[b])
            assert abs(int(gpu[s].iters[b]) - r.iter) <= (2 if s == 0 else 5), (b, s, gpu[s].iters[b], r.iter)
            np.testing.assert_allclose(gpu[s].w[b], w, atol=1e-6 if s == 0 else 1e-5)
            # the next oracle horizon starts from the GPU's solution, so each step compares one
            # solve on identical inputs
            qN, _ = next_initial_state(gpu[s].w[b], n, nf, N)
            q0, w0 = qN[0], gpu[s].w[b].copy()
