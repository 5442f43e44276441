"""Shared parity check of a device C2 solution (IPOPT mode) against the oracle (test helper, no test here).

C2 (force_optimization_pilz_6DOF.py) has an exact symmetry: q_N appears in no row but the last dynamics row (the line
rows stop at k < N, L150-156, and the joint angles are unbounded), and tau = ID(q, qd, 0) - J^T F is even in qd (at
qdd = 0 the velocity terms are quadratic), so (qd_{N-1}, q_N) -> (-qd_{N-1}, 2 q_{N-1} - q_N) maps every feasible point,
with its objective, its barrier terms (the qd bounds are symmetric) and its multipliers' KKT system, onto another.  Two
solves that part at round-off can therefore end at the two mirror images; they then agree on nodes 0..N-1 and on the
objective, and their last velocities are negatives of each other.

check_solution: (1) the oracle's own optimality error at the device's primal-dual point (mfg_opts.kkt_at: E_0 at mu = 0
and the constraint violation, the problem as solved: bound_relax 1e-8) <= 1e-8; (2) the oracle's objective at that
point = the device's; (3) against the oracle's solve: the objective to `obj_tol` relative, q_0..q_{N-1} to `q_tol`, and
either the same q_N (same path) or the mirror image of the oracle's (qd_{N-1}, q_N)."""
from __future__ import annotations

import numpy as np

from oracle import generic as G

N_J, N_F = 6, 1


def split(w: np.ndarray, N: int):
    """(q (N+1, 6), qd (N, 6), F (N,)) of a C2 solution vector [q_0 | (qd_k, F_k, q_{k+1})]."""
    st = 2 * N_J + N_F
    blk = w[N_J:].reshape(N, st)
    q = np.vstack([w[:N_J][None], blk[:, N_J + N_F:]])
    return q, blk[:, :N_J], blk[:, N_J]


def kkt_of_device_point(g, b: int, spec: dict, w: np.ndarray) -> dict:
    """The oracle's optimality measures at problem b's final primal-dual point of the handle's last solve."""
    s, d = g.point(b)
    return G.kkt_at(spec, w, s, d, bound_relax=1e-8)


def check_solution(g, b: int, spec: dict, w_dev: np.ndarray, obj_dev: float, w_or: np.ndarray, obj_or: float,
                   obj_tol: float = 1e-8, q_tol: float = 1e-6) -> dict:
    N = spec["N"]
    k = kkt_of_device_point(g, b, spec, w_dev)
    assert k["E0"] <= 1e-8 and k["pinf"] <= 1e-8, (b, k)
    assert abs(k["obj"] - obj_dev) <= 1e-12 * abs(obj_dev), (b, k["obj"], obj_dev)
    dobj = abs(obj_dev - obj_or) / abs(obj_or)
    assert dobj <= obj_tol, (b, obj_dev, obj_or, dobj)
    qg, vg, Fg = split(w_dev, N)
    qo, vo, Fo = split(w_or, N)
    inner = max(np.abs(qg[:N] - qo[:N]).max(), np.abs(vg[:N - 1] - vo[:N - 1]).max())
    assert inner <= q_tol, (b, inner)
    dF = np.abs(Fg - Fo).max() / max(1.0, np.abs(Fo).max())
    assert dF <= q_tol, (b, dF)
    same = np.abs(qg[N] - qo[N]).max() <= q_tol and np.abs(vg[N - 1] - vo[N - 1]).max() <= q_tol
    mirror = (np.abs(vg[N - 1] + vo[N - 1]).max() <= q_tol
              and np.abs(qg[N] - (2.0 * qo[N - 1] - qo[N])).max() <= q_tol)
    assert same or mirror, (b, vg[N - 1], vo[N - 1])
    return {"E0": k["E0"], "pinf": k["pinf"], "dobj": dobj, "inner_dq": float(inner), "same": bool(same),
            "mirror": bool(mirror and not same), "dq": float(np.abs(qg - qo).max())}
