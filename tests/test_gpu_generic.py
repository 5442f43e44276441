"""GPU parity of the generic solver (csrc/gipm.hip, C ABI mf_gproblem_* / mf_gsolve_batch) against the
generic oracle (oracle/mf_ocp.c) and against the reference's own IPOPT trajectories.

* node records of the device kernel = the oracle's hyper-dual records (box, chain, thermal)
* C2 through the generic path = the generic oracle (same iteration, same options)
* IPOPT mode (filter line search + restoration, x0 = 0, no homotopy, as Box_Pilz_6DOF.py:455-456 solve): G1, G2,
  G4 reproduced on the GPU to 1e-6 rad, every case = the oracle in the same mode
* C3 Box_Pilz_6DOF.py re-solved on the GPU from the reference's IK start matches plotter/solution.csv
  (G1, N=50), Result_2 (G2, N=80) and Result_1 (G4) to 1e-6 rad on every joint angle (SURVEY.md
  s.8c (vi)), and equals the oracle's solve
* Result_4 (G3, LeftConst) is a KKT point of the build's transcription: started there with IPOPT's
  warm_start_init_point constants the GPU converges back to it (<= 1e-6 rad, equal objective)
* the thermal C2 variant (a8) = the oracle; C4 at the committed fixture's horizon (N = 50, T = 2) and
  with the 80 C winding bound active = the oracle
"""
import numpy as np
import pytest

from mpc_fatigue_amd import problems as PR
from oracle import generic as G
from tests.conftest import has_gpu

pytestmark = pytest.mark.gpu

if has_gpu():
    from mpc_fatigue_amd.gocp import GOCP


def rec_split(rec, nx, nu, ni, ne):
    nv = nx + nu
    o = [0]

    def take(n, shape=None):
        a = rec[o[0]:o[0] + n]
        o[0] += n
        return a.reshape(shape) if shape else a
    l = take(1)[0]
    gl = take(nv)
    ci = take(ni)
    Ji = take(ni * nv, (ni, nv))
    ce = take(ne)
    Je = take(ne * nx, (ne, nx))
    f = take(nx)
    A = take(nx * nx, (nx, nx))
    B = take(nx * nu, (nx, nu))
    W = take(nv * nv, (nv, nv))
    return l, gl, ci, Ji, ce, Je, f, A, B, W


@pytest.mark.parametrize("case", ["chain", "thermal", "box"])
def test_device_node_record_matches_oracle(golden, case):
    rng = np.random.default_rng(7)
    if case == "box":
        g, _ = golden["G1_box_N50"]
        spec = PR.box_dual(N=2)
        xu = g[20 * 30:21 * 30].copy()
    elif case == "chain":
        spec = dict(PR.pilz6_bench(N=2), wtau=0.2)
        xu = np.r_[rng.normal(size=6), 0.3 * rng.normal(size=6), [15.0]]
    else:
        spec = PR.pilz6_thermal(N=2)
        xu = np.r_[rng.normal(size=6), 60 + rng.normal(size=6), 0.3 * rng.normal(size=6), [25.0]]
    ocp = GOCP(spec)
    nx, nu, ni, ne = ocp.nx, ocp.nu, ocp.ni, ocp.ne
    yi, ye, lam = 10 * rng.normal(size=ni), rng.normal(size=max(ne, 1)), rng.normal(size=nx)
    rec = ocp.node_record(xu, yi, ye, lam, line_ref=spec.get("line_ref"))
    l, gl, ci, Ji, ce, Je, f, A, B, W = rec_split(rec, nx, nu, ni, ne)
    vals, jac, H = G.node_derivs(spec, xu, yi, ye, lam)
    sc = lambda a: max(1.0, np.abs(a).max())
    assert abs(l - vals[0]) <= 1e-12 * sc(vals[0])
    np.testing.assert_allclose(ci, vals[1:1 + ni], atol=1e-11 * sc(ci))
    np.testing.assert_allclose(f, vals[1 + ni + ne:], atol=1e-12 * sc(f))
    np.testing.assert_allclose(gl, jac[0], atol=1e-11 * sc(gl))
    np.testing.assert_allclose(Ji, jac[1:1 + ni], atol=1e-11 * sc(Ji))
    np.testing.assert_allclose(Je, jac[1 + ni:1 + ni + ne, :nx], atol=1e-12 * sc(Je))
    np.testing.assert_allclose(A, jac[1 + ni + ne:, :nx], atol=1e-12 * sc(A))
    np.testing.assert_allclose(B, jac[1 + ni + ne:, nx:], atol=1e-12 * sc(B))
    np.testing.assert_allclose(W, H, atol=1e-10 * sc(H))


def test_c2_generic_path_matches_oracle():
    spec = PR.pilz6_bench(N=20)
    ocp = GOCP(spec)
    r = ocp.solve(F_init=PR.BENCH_F_INIT, max_soc=4)
    w_ref, r_ref = G.solve(spec, F_init=PR.BENCH_F_INIT, max_iter=300, max_soc=4)
    assert r.status[0] == 0 and r_ref.status == 0
    assert abs(int(r.iters[0]) - r_ref.iter) <= 2
    np.testing.assert_allclose(r.w[0], w_ref, atol=1e-6)


@pytest.mark.parametrize("name,kw", [("G1_box_N50", dict(N=50)), ("G2_box_N80", dict(N=80)),
                                     ("G4_box_N80", dict(N=80, right_const=False))])
def test_box_gpu_resolve_matches_reference(golden, name, kw):
    g, N = golden[name]
    spec = PR.box_dual(q0=g[:12], **kw)
    ocp = GOCP(spec)
    r, stages = ocp.solve_box()
    assert all(int(s.status[0]) == 0 for s in stages), [(int(s.status[0]), int(s.iters[0])) for s in stages]
    dq = np.abs(ocp.q_traj(r.w[0]) - ocp.q_traj(g)).max()
    assert dq < 1e-6, dq
    # and the device solve equals the oracle's solve of the same homotopy
    w_or = None
    for tol in PR.box_homotopy_tolerances():
        w_or, ro = G.solve(dict(spec, pos_toll=tol), w0=w_or, u_init=PR.box_u_init(spec), max_iter=1000, max_soc=4)
    assert np.abs(ocp.q_traj(r.w[0]) - ocp.q_traj(w_or)).max() < 1e-7


IPOPT_MODE = dict(init_zero=True, bound_relax=1e-8, filter=True, max_iter=1500, max_soc=4)


@pytest.mark.parametrize("case,name,kw", [("G1", "G1_box_N50", dict(N=50)), ("G2", "G2_box_N80", dict(N=80)),
                                          ("G3", "G3_box_N80", dict(N=80, left_const=True)),
                                          ("G4", "G4_box_N80", dict(N=80, right_const=False))])
def test_box_gpu_ipopt_mode_cold_solve(golden, case, name, kw):
    """Box_Pilz_6DOF.py solved on the GPU as the reference solves it (L455-456): IPOPT from x0 = 0, no homotopy,
    with IPOPT's globalisation (mf_gopts.filter: filter line search, watchdog, soft restoration, restoration phase)
    and bound_relax_factor 1e-8.  All four of the reference's own IPOPT trajectories -- G1 = plotter/solution.csv, G2 =
    Result_2, G3 = Result_4 (LeftConst), G4 = Result_1 -- are reproduced to 1e-6 rad (measured r06h: 3.2e-10, 2.5e-8,
    8.1e-12, 1.5e-9; G3 at objective 1506.778154 against the CSV's 1506.778151).  Against the oracle's solve in the same
    mode (tests/golden/ipopt_mode_G*.csv): G1, G2, G4 to 1e-6 rad; on G3 the oracle's path ends at a neighbouring minimum
    (1506.826, 0.0101 rad away: DESIGN.md s.2's table), so there the device point is checked by the oracle's own KKT
    test instead (E_0 <= 1e-8 at the device's primal-dual point)."""
    import os
    g, N = golden[name]
    spec = PR.box_dual(q0=g[:12], **kw)
    ocp = GOCP(spec)
    r = ocp.solve(**IPOPT_MODE)
    assert int(r.status[0]) == 0, (int(r.status[0]), int(r.iters[0]))
    q = ocp.q_traj(r.w[0])
    dq_ref = np.abs(q - ocp.q_traj(g)).max()
    w_or = np.loadtxt(os.path.join(os.path.dirname(__file__), "golden", f"ipopt_mode_{case}.csv"), delimiter=",")
    dq_or = np.abs(q - ocp.q_traj(w_or)).max()
    print(f"{case}: {int(r.iters[0])} iterations, objective {float(r.obj[0]):.9f}, dq vs the reference's CSV {dq_ref:.2e}, "
          f"vs the oracle's solve {dq_or:.2e}")
    assert dq_ref < 1e-6
    if case != "G3":
        assert dq_or < 1e-6
    else:
        s, d = ocp.point(0)
        k = G.kkt_at(spec, r.w[0], s, d, bound_relax=1e-8)
        assert k["E0"] <= 1e-8 and k["pinf"] <= 1e-8, k
        assert abs(float(r.obj[0]) - 1506.778151) <= 1e-5


def test_box_gpu_g3_is_a_kkt_point(golden):
    """G3 = plotter/Result_4/solution.csv (Box_Pilz_6DOF.py with LeftConst = True, N = 80).  The cold homotopy
    reaches another local minimum (objective 1535.4 against G3's 1506.78): the problem has
    several.  Started at G3 itself with IPOPT's warm_start_init_point constants and mu_0 = 1e-3, the GPU
    solver converges back to G3: G3 is a KKT point of the build's transcription (E_0 <= 1e-8 within 1e-6
    rad of it) with the same objective, and the device equals the oracle."""
    g, N = golden["G3_box_N80"]
    spec = PR.box_dual(q0=g[:12], N=N, left_const=True)
    ocp = GOCP(spec)
    kw = dict(w0=g, warm_start=True, mu_init=1e-3, max_iter=300, max_soc=4)
    r = ocp.solve(**kw)
    assert int(r.status[0]) == 0, (int(r.status[0]), int(r.iters[0]))
    assert float(r.kkt[0]) <= 1e-8
    dq = np.abs(ocp.q_traj(r.w[0]) - ocp.q_traj(g)).max()
    assert dq < 1e-6, dq
    one = PR.box_dual(N=1, q0=g[:12], left_const=True)
    f_g3 = sum(G.node_derivs(one, g[k * 30:k * 30 + 30], np.zeros(18), np.zeros(1), np.zeros(12))[0][0]
               for k in range(N))
    assert abs(float(r.obj[0]) - f_g3) <= 1e-7 * abs(f_g3), (float(r.obj[0]), f_g3)
    w_or, r_or = G.solve(spec, **kw)
    assert r_or.status == 0 and abs(int(r.iters[0]) - r_or.iter) <= 2
    np.testing.assert_allclose(r.w[0], w_or, atol=1e-7)


def test_thermal_gpu_matches_oracle():
    spec = PR.pilz6_thermal(N=40, T0=79.0)
    ocp = GOCP(spec)
    r = ocp.solve(F_init=PR.BENCH_F_INIT, max_soc=4)
    w_ref, r_ref = G.solve(spec, F_init=PR.BENCH_F_INIT, max_iter=300, max_soc=4)
    assert r.status[0] == 0 and r_ref.status == 0
    np.testing.assert_allclose(r.w[0], w_ref, atol=1e-6)


def _oracle_receding(spec, x0, steps, decimals, **kw):
    """The restart of mpc_principal.py:357-377 on the oracle: x_0 <- x_N (T - 0.05), qd_0 <- qd_{N-1},
    rounded to `decimals`, warm start = the previous solution."""
    n, N = len(spec["q0"]), spec["N"]
    g, _ = G.make(spec)
    nx, nu = g.nx, g.nu
    x, u, prev, out = np.asarray(x0, float), np.zeros(nu), None, []
    rnd = (lambda a: np.round(a, decimals)) if decimals is not None else (lambda a: a)
    for _ in range(steps):
        sp = dict(spec, q0=list(x[:n]), T0=list(x[n:]), qd0=list(u[:n]))
        w, r = G.solve(sp, w0=prev, warm_start=prev is not None, **kw)
        out.append((w, r))
        off = nx + (N - 1) * (nu + nx)
        xN = w[off + nu:off + nu + nx].copy()
        xN[n:] -= 0.05
        x, u, prev = rnd(xN), rnd(w[off:off + nu]), w
    return out


@pytest.mark.parametrize("decimals,steps", [(None, 4), (4, 2)])
def test_thermal_receding_horizon_matches_oracle(decimals, steps):
    """Thermal receding horizon (rows a8 + a14): T_0 <- T_N - 0.05, qd_0 <- qd_{N-1} carried, the
    device-resident warm start, GPU = oracle at every step.  With the reference's 4-decimal rounding
    the restart can land q_0 on a joint limit (here joint 3 at -2.35) and the next horizon is then
    infeasible for both solvers -- the same status on both."""
    from mpc_fatigue_amd.mpc import GRecedingHorizon

    spec = PR.with_thermal(PR.pilz3_working(N=20), T0=20.0)
    kw = dict(max_iter=300, max_soc=4)
    x0 = np.r_[spec["q0"], spec["T0"]]
    ref = _oracle_receding(spec, x0, steps, decimals, **kw)
    loop = GRecedingHorizon(spec, carry_velocity=True, decimals=decimals, **kw)
    res = loop.run(x0[None], steps)
    for s, (r, (w_or, r_or)) in enumerate(zip(res, ref)):
        assert r.status[0] == r_or.status, (s, r.status[0], r_or.status)
        if r_or.status == 0:
            np.testing.assert_allclose(r.w[0], w_or, atol=1e-6, err_msg=f"step {s}")
    if decimals is None:
        assert all(r_or.status == 0 for _, r_or in ref)
        # the temperatures carried across restarts drop by T_drop at each restart
        w1 = res[1].w[0]
        np.testing.assert_allclose(w1[3:6], np.asarray(ref[0][0][-3:]) - 0.05, atol=1e-9)


def test_centauro_device_record_matches_oracle():
    """C4 node record from the device kernel (k_grec<CentauroFam>) = the oracle's hyper-dual record:
    tau = ID + J^T F of both 7-DOF arms, relative pose rows, equilibrium (mixed) rows, thermal dynamics,
    the full Lagrangian Hessian."""
    rng = np.random.default_rng(5)
    spec = PR.centauro(N=2)
    ocp = GOCP(spec)
    nx, nu, ni, ne, nm = ocp.nx, ocp.nu, ocp.ni, ocp.ne, ocp.nem
    assert (nx, nu, ni, ne, nm) == (28, 20, 14, 6, 6)
    q0 = np.asarray(spec["q0"])
    xu = np.r_[q0 + 0.2 * rng.normal(size=14), 20 + 30 * rng.uniform(size=14), 0.5 * rng.normal(size=14),
               rng.normal(size=3) * 5 + [0, 0, 49], rng.normal(size=3) * 5 + [0, 0, 49]]
    yi, ye, lam = 10 * rng.normal(size=ni), rng.normal(size=ne + nm), rng.normal(size=nx)
    rec = ocp.node_record(xu, yi, ye, lam, line_ref=np.zeros(6))
    nv = nx + nu
    vals, jac, H = G.node_derivs(spec, xu, yi, ye, lam)
    o = 1 + nv + ni + ni * nv
    ce, Je = rec[o:o + ne], rec[o + ne:o + ne + ne * nx].reshape(ne, nx)
    o += ne + ne * nx
    cm, Jm = rec[o:o + nm], rec[o + nm:o + nm + nm * nv].reshape(nm, nv)
    o += nm + nm * nv
    W = rec[-nv * nv:].reshape(nv, nv)
    sc = lambda a: max(1.0, np.abs(a).max())
    np.testing.assert_allclose(rec[0], vals[0], rtol=1e-12)
    np.testing.assert_allclose(rec[1:1 + nv], jac[0], atol=1e-11 * sc(jac[0]))
    np.testing.assert_allclose(rec[1 + nv:1 + nv + ni], vals[1:1 + ni], atol=1e-11 * sc(vals[1:1 + ni]))
    np.testing.assert_allclose(ce, vals[1 + ni:1 + ni + ne], atol=1e-12)
    np.testing.assert_allclose(Je, jac[1 + ni:1 + ni + ne, :nx], atol=1e-12)
    np.testing.assert_allclose(cm, vals[1 + ni + ne:1 + ni + ne + nm], atol=1e-11 * sc(cm))
    np.testing.assert_allclose(Jm, jac[1 + ni + ne:1 + ni + ne + nm], atol=1e-11 * sc(Jm))
    np.testing.assert_allclose(rec[o:o + nx], vals[1 + ni + ne + nm:], atol=1e-12 * sc(vals[1 + ni + ne + nm:]))
    np.testing.assert_allclose(W, H, atol=1e-10 * sc(H))


def test_centauro_gpu_matches_oracle_c4():
    """C4 at the reference's horizon (N = 40, T = 30 s, RepeatedMPCwithThermal.py:86-90) from the IK start:
    GPU = oracle, and the solution keeps the box balanced and the hands' relative pose."""
    from tests.test_centauro_cpu import check_solution

    spec = PR.centauro(N=40)
    ocp = GOCP(spec)
    kw = dict(u_init=PR.centauro_u_init(spec), max_iter=500, max_soc=4)
    r = ocp.solve(**kw)
    w_ref, r_ref = G.solve(spec, **kw)
    assert int(r.status[0]) == 0 and r_ref.status == 0, (int(r.status[0]), int(r.iters[0]), r_ref.status)
    assert abs(int(r.iters[0]) - r_ref.iter) <= 2
    np.testing.assert_allclose(r.w[0], w_ref, atol=1e-6)
    check_solution(spec, r.w[0])


def test_centauro_receding_horizon_gpu_matches_oracle():
    """The thermal MPC loop of RepeatedMPCwithThermal.py:154-487 (restart x_0 <- x_N with T - 0.05,
    qd_0 <- qd_{N-1}, 4-decimal rounding, targets rounded to 3 decimals after the first solve, previous
    solution as warm start) on the GPU, step by step equal to the oracle; the windings heat up."""
    from mpc_fatigue_amd.mpc import GRecedingHorizon

    N, steps = 20, 3
    spec = PR.centauro(N=N)
    # the reference's loop tolerances (tol = constr_viol_tol = 1e-3, RepeatedMPCwithThermal.py:441-445): the
    # rounded orientation target cannot be met exactly at node 1 (q_1 is fixed by q_0 and qd_0)
    kw = dict(u_init=PR.centauro_u_init(spec), tol=1e-3, constr_viol_tol=1e-3, max_iter=500, max_soc=4)
    loop = GRecedingHorizon(spec, restart_spec=dict(spec, target_decimals=3), **kw)
    x0 = np.r_[spec["q0"], spec["T0"]]
    res = loop.run(x0[None], steps)
    g, _ = G.make(spec)
    nx, nu = g.nx, g.nu
    x, u, prev = x0, np.zeros(nu), None
    for s in range(steps):
        sp = PR.centauro(N=N, q0=x[:14], T0=x[14:], qd0=u[:14], target_decimals=(3 if s else -1))
        w, r = G.solve(sp, w0=prev, warm_start=prev is not None, **kw)
        assert int(res[s].status[0]) == r.status == 0, (s, int(res[s].status[0]), r.status)
        if r.status == 0:
            np.testing.assert_allclose(res[s].w[0], w, atol=1e-6, err_msg=f"step {s}")
        off = nx + (N - 1) * (nu + nx)
        xN = w[off + nu:off + nu + nx].copy()
        xN[14:] -= 0.05
        x, u, prev = np.round(xN, 4), np.round(w[off:off + nu], 4), w
    assert x[14:].max() > 20.5


def test_centauro_mpc_principal_warm_first_solve_matches_oracle():
    """mpc_principal.py:348-360 starts its loop with warm_start_init_point already at s = 0, from x0 = sol0
    (RepeatedMPCwithThermal.py runs that solve cold): GRecedingHorizon.run(w0=sol0, warm_first=True) on the
    GPU equals the oracle's warm-started solve from the same sol0 (the reference's held state, each hand
    carrying half the box), step 0 and the first restart."""
    from mpc_fatigue_amd.mpc import GRecedingHorizon

    N = 20
    spec = PR.centauro(N=N)
    kw = dict(tol=1e-3, constr_viol_tol=1e-3, max_iter=500, max_soc=4)
    g, _ = G.make(spec)
    nx, nu = g.nx, g.nu
    x0 = np.r_[spec["q0"], spec["T0"]]
    sol0 = np.r_[x0, np.tile(np.r_[PR.centauro_u_init(spec), x0], N)]  # sol0: held state, F = (0, 0, mg/2)
    loop = GRecedingHorizon(spec, restart_spec=dict(spec, target_decimals=3), **kw)
    res = loop.run(x0[None], 2, w0=sol0, warm_first=True)
    w, r = G.solve(spec, w0=sol0, warm_start=True, **kw)
    assert int(res[0].status[0]) == r.status == 0, (int(res[0].status[0]), r.status)
    np.testing.assert_allclose(res[0].w[0], w, atol=1e-6)
    assert abs(int(res[0].iters[0]) - r.iter) <= 2
    assert int(res[1].status[0]) == 0


def test_box_shared_fatigue_gpu_matches_oracle(golden):
    """C3 at N = 100 with the shared fatigue budget (BASELINE config 3; build-defined, parity against the
    oracle only): the winding temperatures of all 12 joints as state, one budget row per node.  IPOPT mode (the
    bench's path: one cold solve from x0 = 0, filter globalisation, bound_relax 1e-8) equals the hyper-dual
    oracle's solution (tests/golden/ipopt_mode_C3sf.csv) on every state to 1e-6, and the budget and the
    temperature bounds hold.  The merit-mode homotopy (pos_toll 1 -> 1e-2 -> 1e-4) is checked stage by stage
    against the oracle with the device's Riccati elimination, each oracle stage started from the device's previous
    stage: the first two stages equal it on every state to 1e-6.  The last stage (pos_toll 1e-4, the reference's
    +-1e-4 equilibrium windows) ends on a round-off-sensitive path -- 78, 108 and 140 iterations for the oracle's
    Riccati, the device and the oracle's banded KKT from the same start since round 4's codegen change (DESIGN.md
    s.9) -- so there the objective is compared at 1e-8, the states at 1e-3, and the budget / bounds asserted."""
    import os
    g, _ = golden["G1_box_N50"]
    spec = PR.box_shared_fatigue(N=100, q0=g[:12])
    ocp = GOCP(spec)
    assert (ocp.nx, ocp.nu, ocp.ni, ocp.ne) == (24, 18, 19, 1)
    wf = np.loadtxt(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ipopt_mode_C3sf.csv"),
                    delimiter=",")
    ri = ocp.solve(**IPOPT_MODE)
    assert int(ri.status[0]) == 0, (int(ri.status[0]), int(ri.iters[0]))
    assert np.abs(ocp.q_traj(ri.w[0]) - ocp.q_traj(wf)).max() < 1e-6
    relax = 1e-8 * np.maximum(1.0, np.abs(spec["T_budget"]))

    def bounds_hold(X):
        return (X[:, 12:].sum(1) <= spec["T_budget"] + relax + 1e-6).all() and (X[:, 12:] <= spec["T_hi"] + 1e-6).all()
    assert bounds_hold(ocp.q_traj(ri.w[0]))
    r, stages = ocp.solve_box()
    assert all(int(s.status[0]) == 0 for s in stages), [(int(s.status[0]), int(s.iters[0])) for s in stages]
    w_prev = None
    for i, (tol, st) in enumerate(zip(PR.box_homotopy_tolerances(), stages)):
        w_or, ro = G.solve(dict(spec, pos_toll=tol), w0=w_prev, u_init=PR.box_u_init(spec), max_iter=1000, max_soc=4,
                           riccati=True)
        assert ro.status == 0, (i, ro.status, ro.iter)
        dq = np.abs(ocp.q_traj(st.w[0]) - ocp.q_traj(w_or)).max()
        if i < 2:
            assert dq < 1e-6, (i, dq, int(st.iters[0]), ro.iter)
        else:
            assert dq < 1e-3, dq
            assert abs(float(st.obj[0]) - ro.obj) <= 1e-8 * abs(ro.obj)
        w_prev = st.w[0]
    assert bounds_hold(ocp.q_traj(r.w[0]))


def test_centauro_gpu_n50_fixture_horizon():
    """C4 at BASELINE's N = 50 over the horizon of the committed Centauro fixture (Centauro_dynamics.py:90-91:
    T = 2 s, N = 50; Const1 relative pose), thermal state included: GPU = oracle and the solution passes the
    fixture's invariants (Euler continuity, force and moment balance, relative pose held)."""
    from tests.test_centauro_cpu import check_solution

    spec = PR.centauro(N=50, T=2.0)
    ocp = GOCP(spec)
    kw = dict(u_init=PR.centauro_u_init(spec), max_iter=500, max_soc=4)
    r = ocp.solve(**kw)
    w_ref, r_ref = G.solve(spec, **kw)
    assert int(r.status[0]) == 0 and r_ref.status == 0, (int(r.status[0]), int(r.iters[0]), r_ref.status)
    assert abs(int(r.iters[0]) - r_ref.iter) <= 2
    np.testing.assert_allclose(r.w[0], w_ref, atol=1e-6)
    check_solution(spec, r.w[0])


def test_centauro_gpu_winding_bound_active():
    """The 80 C winding bound (T in [0, 80], RepeatedMPCwithThermal.py:122-123, MPC_parameters.py:49) active:
    C4 (N = 20, T = 30 s) with the windings starting at 79 C.  The bound holds at >= 10 (node, joint) pairs
    and costs objective against the cold-winding solve (the solver re-poses the arms to shed load); GPU =
    oracle, same active set."""
    N = 20
    cold = PR.centauro(N=N)
    spec = PR.centauro(N=N, T0=79.0)
    ocp = GOCP(spec)
    kw = dict(u_init=PR.centauro_u_init(spec), max_iter=500, max_soc=4)
    r = ocp.solve(**kw)
    w_ref, r_ref = G.solve(spec, **kw)
    assert int(r.status[0]) == 0 and r_ref.status == 0, (int(r.status[0]), int(r.iters[0]), r_ref.status)
    np.testing.assert_allclose(r.w[0], w_ref, atol=1e-6)
    T_gpu, T_or = ocp.q_traj(r.w[0])[:, 14:], ocp.q_traj(w_ref)[:, 14:]
    act_gpu, act_or = T_gpu > 80.0 - 1e-5, T_or > 80.0 - 1e-5
    assert act_gpu.sum() >= 10 and (act_gpu == act_or).all()
    assert T_gpu.max() <= 80.0 + 1e-8
    _, r_cold = G.solve(cold, **kw)
    assert float(r.obj[0]) > r_cold.obj + 0.1


def _golden_q0_g1():
    import os
    return np.loadtxt(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "G1_box_N50_solution.csv"),
                      delimiter=",")[:12]


def test_generic_bench_workloads_match_hyperdual_oracle():
    """The bench's generic figures (tools/generic_bench.py, BASELINE configs 3 and 4, IPOPT mode): perturbed starts
    drawn as the bench draws them (C3 shared budget N=100, q0 + U(-0.01, 0.01); C4 Centauro N=50, q0 +
    U(-0.02, 0.02)), solved on the device as the bench solves them -- one cold solve from x0 = 0 with the filter
    globalisation and bound_relax 1e-8 (Box_Pilz_6DOF.py:455-456, RepeatedMPCwithThermal.py:464-466) -- equal the
    independent hyper-dual oracle (oracle/mf_ocp.c with its own dual-number node derivatives, not the product's
    node functions; fixtures tests/golden/bench_c{3,4}_*.csv, make_bench_workload_fixtures.py) on every state to
    1e-6; the batched device solve equals the single solve."""
    import sys
    import os
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    from generic_bench import IPOPT_KW

    gdir = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    sp3 = PR.box_shared_fatigue(N=100, q0=_golden_q0_g1())
    sp4 = PR.centauro(N=50, T=2.0)
    for spec, names in ((sp3, ["bench_c3_0", "bench_c3_1"]), (sp4, ["bench_c4_0", "bench_c4_1", "bench_c4_2"])):
        g = GOCP(spec)
        W = np.vstack([np.loadtxt(os.path.join(gdir, f"{n}.csv"), delimiter=",")[None] for n in names])
        X = np.ascontiguousarray(W[:, :g.nx])
        r = g.solve(x0=X, **IPOPT_KW)
        assert (r.status == 0).all(), r.status
        for i, n in enumerate(names):
            assert np.abs(g.q_traj(r.w[i]) - g.q_traj(W[i])).max() < 1e-6, n
        r1 = g.solve(x0=X[:1], **IPOPT_KW)
        assert np.abs(r1.w[0] - r.w[0]).max() < 1e-9


@pytest.mark.parametrize("case", ["chain_merit", "centauro_ipopt"])
def test_stream_solve_equals_batch_solve(case):
    """Continuous batching (mf_gsolve_stream_dev): a few slots working through many problems -- each slot
    handed the next problem when its own finishes (x_0, line reference and warm-start rows re-staged,
    k_gharvest) -- give every problem exactly the batch solve's result (same arithmetic per horizon)."""
    from mpc_fatigue_amd import pin
    rng = np.random.default_rng(3)
    if case == "chain_merit":
        spec = PR.pilz6_bench(N=20)
        T, slots = 40, 7
        Q0 = PR.pilz6_batch_q0(T, seed=5)
        fk = pin.generate_forward_kin(PR.read_urdf(spec["urdf"]), spec["frame"])
        LR = fk.batch(Q0)[0][:, :2]
        X, kw = Q0, dict(F_init=PR.BENCH_F_INIT, max_soc=4, line_ref=LR)
    else:
        spec = PR.centauro(N=20, T=2.0)
        T, slots = 12, 5
        q0 = np.asarray(spec["q0"])
        X = np.hstack([q0[None] + rng.uniform(-0.02, 0.02, (T, 14)), np.tile(spec["T0"], (T, 1))])
        kw = dict(IPOPT_MODE)
    g = GOCP(spec)
    rb = g.solve(x0=X, **kw)
    rs = g.solve_stream(X, slots, **kw)
    np.testing.assert_array_equal(rs.status, rb.status)
    np.testing.assert_array_equal(rs.iters, rb.iters)
    np.testing.assert_array_equal(rs.w, rb.w)
    assert (rb.status == 0).mean() >= 0.5


def test_c2_ipopt_mode_sixteen_horizons_match_oracle():
    """C2 as the reference solves it (IPOPT mode from x0 = 0, the generic solver's chain family) on 16 horizons spread
    over the 4096-start draw (every 256th) against the oracle's IPOPT-mode solves with the device's elimination
    (riccati = 2): the same status everywhere, every device point a KKT point by the oracle's own check (E_0 <= 1e-8 at
    the device's primal-dual point), and either the oracle's optimum (q, qd, F to 1e-5, objective to 1e-12) or -- where
    the two paths part at round-off inside a restoration phase -- a neighbouring optimum of C2's flat valley (a joint
    velocity bound-to-bound at one node, objective within 5e-5; tests/c2check.py), the oracle's on at least half."""
    from oracle import pin_np as P
    from oracle.urdf_np import load_urdf_file
    from tests import c2check
    N = 100
    base = PR.pilz6_bench(N=N)
    ref = load_urdf_file(PR.urdf_path(base["urdf"]))
    idx = np.arange(0, 4096, 256)
    Q0 = PR.pilz6_batch_q0(4096, seed=0)[idx]
    LR = np.array([P.forward_kinematics(ref, q, "prbt_link_5")[0][:2] for q in Q0])
    kw = dict(IPOPT_MODE, max_iter=3000)
    g = GOCP(base)
    r = g.solve(x0=Q0, line_ref=LR, **kw)
    specs = [PR.pilz6_bench(N=N, q0=Q0[b], line_ref=LR[b]) for b in range(len(idx))]
    W, R = G.solve_batch(specs, nthreads=16, riccati=2, **kw)
    same = 0
    for b in range(len(idx)):
        assert int(r.status[b]) == R[b].status == 0, (idx[b], int(r.status[b]), R[b].status)
        c = c2check.compare(g, b, specs[b], r.w[b], float(r.obj[b]), W[b], R[b].obj, q_tol=1e-5)
        print(f"start {idx[b]}: device {int(r.iters[b])} it, oracle {R[b].iter} it, E0 {c['E0']:.1e}, dobj {c['dobj']:.1e}, "
              f"dq(0..N-1) {c['inner_dq']:.1e}, dq {c['dq']:.1e}, {c['kind']}")
        assert c["E0"] <= 1e-8 and c["pinf"] <= 1e-8, (idx[b], c)
        assert c["dobj"] <= (1e-12 if c["kind"] != "neighbour" else 5e-5), (idx[b], c)
        same += c["kind"] != "neighbour"
    print("the oracle's optimum:", same, "of", len(idx))
    assert same >= len(idx) // 2


def test_c2_ipopt_restoration_with_elastic_dynamics_rows():
    """IPOPT's restoration problem (IpRestoIpoptNLP: elastic p, n on every constraint row, the dynamics rows
    x_{k+1} = f(x_k, u_k) included) on the device: the Riccati recursion through the relaxed rows
    dx_{k+1} = A dx_k + B du_k + r - D_r dlam_k (csrc/gipm.hip relax_stage, oracle ric_relax).  Horizons 41, 45, 48 of
    the C2 bench batch are the starts whose restoration fails when the dynamics rows are kept exact (the build's
    variant before round 5, resto_hard_dyn: status 4 on the device); with IPOPT's restoration the device converges on
    all three to the oracle's solution (riccati = 2, tests/golden/ipopt_mode_C2_*.csv) by tests/c2check.py's check: the
    device point passes the oracle's KKT check, the objective to 1e-8, nodes 0..N-1 to 1e-6 rad, the last node the
    oracle's or its mirror image."""
    import json
    import os
    from oracle import pin_np as P
    from oracle.urdf_np import load_urdf_file
    from tests import c2check
    gdir = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    meta = json.load(open(os.path.join(gdir, "ipopt_mode_fixtures.json")))
    idx = [41, 45, 48]
    base = PR.pilz6_bench(N=100)
    ref = load_urdf_file(PR.urdf_path(base["urdf"]))
    Q0 = PR.pilz6_batch_q0(64, seed=0)[idx]
    LR = np.array([P.forward_kinematics(ref, q, "prbt_link_5")[0][:2] for q in Q0])
    g = GOCP(base)
    kw = dict(IPOPT_MODE, max_iter=3000)
    rh = g.solve(x0=Q0, line_ref=LR, resto_hard_dyn=True, **kw)
    print("exact dynamics rows: status", rh.status.tolist(), "iters", rh.iters.tolist())
    assert (rh.status == 4).all(), rh.status
    r = g.solve(x0=Q0, line_ref=LR, **kw)
    print("elastic dynamics rows: status", r.status.tolist(), "iters", r.iters.tolist())
    for b, i in enumerate(idx):
        w_or = np.loadtxt(os.path.join(gdir, f"ipopt_mode_C2_{i}.csv"), delimiter=",")
        m = meta[f"C2_{i}"]
        assert int(r.status[b]) == 0, (i, int(r.status[b]), int(r.iters[b]))
        spec = PR.pilz6_bench(N=100, q0=Q0[b], line_ref=LR[b])
        c = c2check.compare(g, b, spec, r.w[b], float(r.obj[b]), w_or, m["obj"], q_tol=1e-5)
        print(f"horizon {i}: device {int(r.iters[b])} it, oracle {m['iter']} it, {c}")
        assert c["E0"] <= 1e-8 and c["pinf"] <= 1e-8, (i, c)
        if i == 45:  # the oracle's optimum (r05, r06d, r06i: 306 / 307 iterations against the oracle's 307)
            assert c["kind"] == "same" and c["dobj"] <= 1e-12 and abs(int(r.iters[b]) - m["iter"]) <= 2, (i, c)
        else:  # 41, 48: the paths part inside a restoration phase; neighbouring optima (r06d: dobj 2.2e-6, 5.0e-6)
            assert c["dobj"] <= 5e-5, (i, c)


@pytest.mark.parametrize("case", ["c3", "c4", "c2"])
def test_concurrent_inertia_tries_equal_sequential_search(case):
    """The tail mode of the IPOPT-mode solver (csrc/gipm.hip k_gspec): while at most 64 horizons run, the first four
    delta_w candidates of IPOPT's inertia-correction search are factored concurrently, and k_gkkt replays the
    sequential search over their results.  Every horizon's solve -- status, iteration count and solution -- is the
    sequential search's bit for bit (bench starts of C3 shared budget / C4 Centauro / C2, restoration included)."""
    import os
    gdir = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    kw = dict(IPOPT_MODE, max_iter=3000)
    lr = None
    if case == "c3":
        spec = PR.box_shared_fatigue(N=100, q0=_golden_q0_g1())
        X = np.vstack([np.loadtxt(os.path.join(gdir, f"bench_c3_{i}.csv"), delimiter=",")[None, :24] for i in (0, 1)])
    elif case == "c4":
        spec = PR.centauro(N=50, T=2.0)
        X = np.vstack([np.loadtxt(os.path.join(gdir, f"bench_c4_{i}.csv"), delimiter=",")[None, :28] for i in (0, 1)])
    else:
        from oracle import pin_np as P
        from oracle.urdf_np import load_urdf_file
        spec = PR.pilz6_bench(N=100)
        ref = load_urdf_file(PR.urdf_path(spec["urdf"]))
        X = PR.pilz6_batch_q0(64, seed=0)[[41, 45, 2]]
        lr = np.array([P.forward_kinematics(ref, q, "prbt_link_5")[0][:2] for q in X])
    g = GOCP(spec)
    X = np.ascontiguousarray(X)
    r1 = g.solve(x0=X, line_ref=lr, inertia_spec=-1, **kw)
    r2 = g.solve(x0=X, line_ref=lr, **kw)
    print(case, "sequential", r1.status.tolist(), r1.iters.tolist(), "concurrent", r2.status.tolist(), r2.iters.tolist())
    np.testing.assert_array_equal(r2.status, r1.status)
    np.testing.assert_array_equal(r2.iters, r1.iters)
    np.testing.assert_array_equal(r2.w, r1.w)


def test_chain_occupancy_variant_equals_default():
    """The chain families' k_gkkt has a register-capped variant (csrc/gipm.hip GOcc: 128 VGPRs, 4 waves per SIMD) that
    the host launches while more than four horizons per CU run.  Register allocation does not change the arithmetic:
    the first 16 horizons of a 2048-start C2 batch (IPOPT mode, every launch above the threshold on a 256-CU device)
    end bit-identical to the same 16 solved alone (default variant)."""
    from oracle import pin_np as P
    from oracle.urdf_np import load_urdf_file
    spec = PR.pilz6_bench(N=100)
    ref = load_urdf_file(PR.urdf_path(spec["urdf"]))
    X = np.ascontiguousarray(PR.pilz6_batch_q0(2048, seed=0))
    lr = np.ascontiguousarray(np.array([P.forward_kinematics(ref, q, "prbt_link_5")[0][:2] for q in X]))
    g = GOCP(spec)
    kw = dict(IPOPT_MODE, max_iter=40, inertia_spec=-1)
    rb = g.solve(x0=X, line_ref=lr, **kw)
    rs = g.solve(x0=X[:16], line_ref=lr[:16], **kw)
    print("2048-start batch: status", np.unique(rb.status, return_counts=True), "| first 16 iterations", rs.iters.tolist())
    np.testing.assert_array_equal(rb.status[:16], rs.status)
    np.testing.assert_array_equal(rb.iters[:16], rs.iters)
    np.testing.assert_array_equal(rb.w[:16], rs.w)


def test_watchdog_stop_with_failed_search():
    """A failed backtracking search after StopWatchDog (IPOPT's watchdog: the stored point and direction restored, the
    search from alpha_max / 2 fails): the oracle re-evaluates the stored point before it augments the filter and
    starts the soft restoration (oracle/mf_ocp.c ipm_filter), the device spends a GP_WDSOFT round on the same
    re-evaluation (csrc/gipm.hip).  The oracle's IPM takes that path on starts 8, 12 and 13 of the C3
    shared-budget bench draw (tools/watchdog_scan.py); device and oracle part at round-off inside the long restoration
    sequences before it (tools/ipopt_trace_cmp.py: the same iterates to 3 digits for ~140 iterations on start 0), so
    the device's own path is checked: on the first 64 starts of the draw some horizons take it (mf_gdebug_counters;
    measured: starts 25, 44, 50, 52, each then stopping at the 1,500 cap) and every one of them continues to a KKT
    point (status 0, E_0 <= 1e-8) or to one of IPOPT's own outcomes.  The oracle on the same four starts: the path on
    25, 44 and 52 as well, the cap on 25, 50 and 52, convergence on 44 after 1,456 iterations.  Each device outcome is
    then judged by the oracle's own optimality measures at the device's final primal-dual point (mfg_opts.kkt_at):
    converged horizons are KKT points of the oracle's problem, capped ones are not."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    from watchdog_scan import spec_of
    specs = [spec_of("c3", i) for i in range(64)]
    X = np.vstack([np.r_[sp["q0"], sp["T0"]][None] for sp in specs])
    g = GOCP(specs[0])
    r = g.solve(x0=X, **dict(IPOPT_MODE, max_iter=1500))
    cnt = [g.counters(b) for b in range(64)]
    hit = [b for b in range(64) if cnt[b]["wd_failed_searches"] > 0]
    print("starts with a failed search after StopWatchDog:", [(b, cnt[b]["wd_failed_searches"], int(r.status[b]),
                                                                int(r.iters[b])) for b in hit])
    assert hit, "no horizon took the path"
    assert all(int(r.status[b]) in (0, 1, 4, 5) for b in hit)
    # the device's outcome judged by the oracle's own functions at the device's final primal-dual point
    # (mfg_opts.kkt_at): a converged horizon is a KKT point of the oracle's problem (E_0 <= 1e-8, its objective
    # the device's), a horizon stopped at the cap is not (E_0 > 1e-8 by the oracle's measure as well)
    for b in hit:
        s_b, d_b = g.point(b)
        k = G.kkt_at(specs[b], r.w[b], s_b, d_b, bound_relax=1e-8)
        print(f"start {b}: status {int(r.status[b])}, device E0 {float(r.kkt[b]):.3e}, oracle E0 at the device point "
              f"{k['E0']:.3e} (pinf {k['pinf']:.1e}), obj {float(r.obj[b]):.10g} / {k['obj']:.10g}")
        assert abs(k["obj"] - float(r.obj[b])) <= 1e-9 * max(1.0, abs(k["obj"]))
        if int(r.status[b]) == 0:
            assert float(r.kkt[b]) <= 1e-8
            assert k["E0"] <= 1e-8 and k["pinf"] <= 1e-8
        elif int(r.status[b]) == 1:
            assert k["E0"] > 1e-8
