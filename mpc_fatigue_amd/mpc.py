"""Receding-horizon loop over batches of horizons.

The reference restarts every OCP from the end of the previous one and warm-starts it with
the previous solution (``python/Centauro_script/mpc_principal.py:357-377``,
``RepeatedMPCwithThermal.py:445-448, 462-487``):

* ``q0 <- sol[N*n : N*n + nq]``   -- the joint angles at the last node (q_N),
* ``qc_dot0 <- sol[k*n + 2nq : ...]`` with the loop variable left at k = N-1 -- the last
  joint velocity (qd_{N-1}),
* ``Solver(x0 = sol, ...)`` with IPOPT ``warm_start_init_point``: the previous primal point,
  multipliers cold.

``RecedingHorizon`` runs that loop for a batch of horizons through ``mf_solve_batch_ws``
(the GPU init kernel pushes the warm start into the bounds exactly as the oracle does).
The thermal restart ``T0 <- T_N - 0.05`` belongs to the thermal state (row a8) that the
Pilz transcriptions do not carry.
"""
from __future__ import annotations

import numpy as np

from .ocp import OCP


def split_w(w: np.ndarray, n: int, nf: int, N: int):
    """w (B, wsize) in the reference layout [q_0 | (qd_k, F_k, q_{k+1}) for k < N] ->
    q (B, N+1, n), qd (B, N, n), F (B, N, nf)."""
    w = np.atleast_2d(w)
    B, st = w.shape[0], 2 * n + nf
    blk = w[:, n:].reshape(B, N, st)
    q = np.concatenate([w[:, None, :n], blk[:, :, n + nf:]], axis=1)
    return q, blk[:, :, :n], blk[:, :, n:n + nf]


def next_initial_state(w: np.ndarray, n: int, nf: int, N: int):
    """(q_N, qd_{N-1}) of each solution: the next horizon's fixed initial state."""
    q, qd, _ = split_w(w, n, nf, N)
    return q[:, N, :].copy(), qd[:, N - 1, :].copy()


class RecedingHorizon:
    """Repeated OCP solves of the spec's problem for a batch of initial states."""

    def __init__(self, spec: dict, carry_velocity: bool = True, **opts):
        """carry_velocity: restart with qd_0 = qd_{N-1} as the reference does.  For the C2 line
        task that velocity sits on its +-0.4 bounds at the end of a horizon, and the next
        horizon is then infeasible (the frame cannot return to the line by node 2; the oracle
        and the GPU both stop at max_iter with the same violation), so the C2 loop restarts
        at rest (carry_velocity=False)."""
        self.spec = spec
        self.ocp = OCP(spec)
        self.carry_velocity = carry_velocity
        self.opts = opts

    def run(self, q0, steps: int, line_ref=None, qd0=None):
        """Returns the list of per-step SolveResults (host arrays)."""
        o = self.ocp
        q0 = np.ascontiguousarray(np.atleast_2d(np.asarray(q0, float)))
        qd = None if qd0 is None else np.atleast_2d(np.asarray(qd0, float))
        w0, out = None, []
        for _ in range(steps):
            r = o.solve_ws(q0, qd0=qd, w0=w0, line_ref=line_ref, **self.opts)
            out.append(r)
            q0, qdl = next_initial_state(r.w, o.n, o.nf, o.N)
            qd = qdl if self.carry_velocity else None
            w0 = r.w
        return out
