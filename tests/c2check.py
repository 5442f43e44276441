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


def compare(g, b: int, spec: dict, w_dev: np.ndarray, obj_dev: float, w_or: np.ndarray, obj_or: float,
            q_tol: float = 1e-6) -> dict:
    """Measures of a device solution against the oracle's (no assertion): the oracle's KKT check at the device point,
    the relative objective difference, the largest difference over nodes 0..N-1 (q, qd, F) and at the last node, and
    the relation of the last node: "same", "mirror" (the exact image under C2's last-node symmetry) or "neighbour" (a
    different KKT point: the paths parted)."""
    N = spec["N"]
    k = kkt_of_device_point(g, b, spec, w_dev)
    dobj = abs(obj_dev - obj_or) / abs(obj_or)
    qg, vg, Fg = split(w_dev, N)
    qo, vo, Fo = split(w_or, N)
    dF = np.abs(Fg - Fo).max() / max(1.0, np.abs(Fo).max())
    inner = max(np.abs(qg[:N] - qo[:N]).max(), np.abs(vg[:N - 1] - vo[:N - 1]).max(), dF)
    same_last = np.abs(qg[N] - qo[N]).max() <= q_tol and np.abs(vg[N - 1] - vo[N - 1]).max() <= q_tol
    mirror_last = (np.abs(vg[N - 1] + vo[N - 1]).max() <= q_tol
                   and np.abs(qg[N] - (2.0 * qo[N - 1] - qo[N])).max() <= q_tol)
    kind = "neighbour"
    if inner <= q_tol:
        kind = "same" if same_last else ("mirror" if mirror_last else "neighbour")
    return {"E0": k["E0"], "pinf": k["pinf"], "obj_at_point": k["obj"], "dobj": dobj, "inner_dq": float(inner),
            "dq": float(np.abs(qg - qo).max()), "kind": kind}


def check_solution(g, b: int, spec: dict, w_dev: np.ndarray, obj_dev: float, w_or: np.ndarray, obj_or: float,
                   obj_tol: float = 1e-8, q_tol: float = 1e-6) -> dict:
    """compare() with assertions: a KKT point by the oracle's check, the device's objective at it, and the oracle's
    solution or its mirror image (objective to obj_tol, nodes 0..N-1 to q_tol)."""
    c = compare(g, b, spec, w_dev, obj_dev, w_or, obj_or, q_tol)
    assert c["E0"] <= 1e-8 and c["pinf"] <= 1e-8, (b, c)
    assert abs(c["obj_at_point"] - obj_dev) <= 1e-12 * abs(obj_dev), (b, c["obj_at_point"], obj_dev)
    assert c["dobj"] <= obj_tol, (b, c)
    assert c["kind"] in ("same", "mirror"), (b, c)
    return c
