"""The oracle's KKT check (oracle/mf_ocp.c mfg_opts.kkt_at) that the GPU parity tests apply to device solutions, and
C2's last-node symmetry that tests/c2check.py accepts (CPU only)."""
import numpy as np
import pytest

from mpc_fatigue_amd import problems as PR
from oracle import generic as G
from oracle import pin_np as P
from oracle.urdf_np import load_urdf_file
from tests import c2check

IPOPT_MODE = dict(init_zero=True, filter=True, bound_relax=1e-8, max_iter=3000, max_soc=4)


@pytest.fixture(scope="module")
def c2_small():
    N = 12
    base = PR.pilz6_bench(N=N)
    ref = load_urdf_file(PR.urdf_path(base["urdf"]))
    q0 = PR.pilz6_batch_q0(2, seed=1)[0]
    spec = PR.pilz6_bench(N=N, q0=q0, line_ref=P.forward_kinematics(ref, q0, "prbt_link_5")[0][:2])
    g, _ = G.make(spec)
    dual = np.zeros(N * g.nx + 3 * N * g.ni + N * g.ne + 2 * (N + 1) * g.nx + 2 * N * g.nu + 1)
    s = np.zeros(N * g.ni)
    w, r = G.solve(spec, dual_out=dual, s_out=s, riccati=2, **IPOPT_MODE)
    assert r.status == 0
    return spec, w, s, dual[:-1], r


def test_kkt_at_reproduces_the_solvers_optimality_error(c2_small):
    spec, w, s, d, r = c2_small
    k = G.kkt_at(spec, w, s, d, bound_relax=1e-8)
    assert k["E0"] == pytest.approx(r.kkt, rel=1e-12, abs=1e-15)
    assert k["E0"] <= 1e-8 and k["pinf"] <= 1e-8
    assert k["obj"] == pytest.approx(r.obj, rel=1e-14)
    w2 = w.copy()
    w2[6 + 5 * 13 + 2] += 1e-6  # one joint velocity: the point is no longer stationary
    assert G.kkt_at(spec, w2, s, d, bound_relax=1e-8)["E0"] > 1e-6


def test_c2_last_node_mirror_is_feasible_with_the_same_objective(c2_small):
    """(qd_{N-1}, q_N) -> (-qd_{N-1}, 2 q_{N-1} - q_N) keeps every row and the objective of C2 (tau even in qd at
    qdd = 0, q_N in no other row): the primal residual and the objective of the mirrored point equal the original's."""
    spec, w, s, d, r = c2_small
    N = spec["N"]
    st = 13
    wm = w.copy()
    o = 6 + (N - 1) * st
    qd = w[o:o + 6]
    qprev = w[o - 6:o] if N > 1 else w[:6]
    wm[o:o + 6] = -qd
    wm[o + 7:o + 13] = 2.0 * qprev - w[o + 7:o + 13]
    assert np.abs(qd).max() > 1e-3  # the last velocity is not zero: the mirror is another point
    k0 = G.kkt_at(spec, w, s, np.zeros_like(d), bound_relax=1e-8)
    k1 = G.kkt_at(spec, wm, s, np.zeros_like(d), bound_relax=1e-8)
    assert k1["pinf"] <= 1e-9 and abs(k1["pinf"] - k0["pinf"]) <= 1e-9
    assert k1["obj"] == pytest.approx(k0["obj"], rel=1e-14)
    q, v, F = c2check.split(wm, N)
    np.testing.assert_allclose(v[N - 1], -qd)
