"""Receding-horizon loop over batches of horizons.

The reference restarts every OCP from the end of the previous one and warm-starts it with
the previous solution (``python/Centauro_script/mpc_principal.py:357-377``,
``RepeatedMPCwithThermal.py:445-448, 462-487``):

* ``q0 <- sol[N*n : N*n + nq]``   -- the joint angles at the last node (q_N),
* ``qc_dot0 <- sol[k*n + 2nq : ...]`` with the loop variable left at k = N-1 -- the last
  joint velocity (qd_{N-1}),
* ``Solver(x0 = sol, ...)`` with IPOPT ``warm_start_init_point = yes`` (``RepeatedMPCwithThermal.py:445-446``
  from the second solve on): the previous primal point pushed into its bounds by
  warm_start_bound_push = _frac = 1e-3, bound multipliers warm_start_mult_bound_push = 1e-3 (CasADi
  passes lam_x0 = 0), constraint multipliers 0 (lam_g0 = 0); mu_init stays IPOPT's 0.1.

``RecedingHorizon`` runs that loop for a batch of horizons through ``mf_solve_batch_ws``
(the GPU init kernel pushes the warm start into the bounds exactly as the oracle does).

``GRecedingHorizon`` runs it for the generic problems (gocp.GOCP: thermal state, dual arm)
with the whole restart of ``mpc_principal.py:365-374``:

* ``T_0 <- T_N - 0.05`` for the winding temperatures,
* every restart value rounded to 4 decimals (``np.round(., 4)``, L371-373),
* the warm start and the next initial state kept on the device: the previous solution
  vector is the next solve's ``w0`` (ping-pong buffers, mf_gsolve_batch_dev) and the next
  (x_0, qd_0) are sliced from it without a host round trip.
"""
from __future__ import annotations

import numpy as np

from .gocp import GOCP
from .ocp import OCP, SolveResult


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

    def __init__(self, spec: dict, carry_velocity: bool = True, warm_start: bool = True,
                 reanchor_line: bool = False, **opts):
        """carry_velocity: restart with qd_0 = qd_{N-1} as the reference does.  For the C2 line
        task that velocity sits on its +-0.4 bounds at the end of a horizon, and the next
        horizon is then often infeasible (the frame cannot return to the line by node 2: 18 of
        96 restarts fail even from a cold start), so the C2 loop restarts at rest
        (carry_velocity=False).
        warm_start: IPOPT warm_start_init_point constants for the solves after the first.
        reanchor_line: each horizon's line reference is the frame position of its own q_0 (as
        the C5 batch anchors every horizon, problems.pilz6_batch_q0).  The transcription puts the
        line on nodes k < N only (force_optimization_pilz_6DOF.py:150-156 inside ``for k in
        range(N)``), so q_N may end off a fixed line and the restarted horizon then has to reach it
        by node 2 with |qd| <= 0.4: at the edge of that reach the line rows and the active velocity
        bounds are linearly dependent and the multipliers diverge (measured: DESIGN.md s.3)."""
        self.spec = spec
        self.ocp = OCP(spec)
        self.carry_velocity = carry_velocity
        self.warm_start = warm_start
        self.reanchor_line = reanchor_line
        self.opts = opts
        if reanchor_line:
            from .pin import ForwardKinematics
            self._fk = ForwardKinematics(self.ocp.model, spec["frame"])

    def run(self, q0, steps: int, line_ref=None, qd0=None):
        """Returns the list of per-step SolveResults (host arrays)."""
        o = self.ocp
        q0 = np.ascontiguousarray(np.atleast_2d(np.asarray(q0, float)))
        qd = None if qd0 is None else np.atleast_2d(np.asarray(qd0, float))
        w0, out = None, []
        for _ in range(steps):
            if self.reanchor_line:
                line_ref = self._fk.batch(q0)[0][:, :2]
            r = o.solve_ws(q0, qd0=qd, w0=w0, line_ref=line_ref,
                           warm_start=self.warm_start and w0 is not None, **self.opts)
            out.append(r)
            q0, qdl = next_initial_state(r.w, o.n, o.nf, o.N)
            qd = qdl if self.carry_velocity else None
            w0 = r.w
        return out


def _round(x, decimals: int):
    """np.round(x, decimals) (round half to even on x * 10^decimals) for numpy or torch arrays."""
    if decimals is None:
        return x
    if isinstance(x, np.ndarray):
        return np.round(x, decimals)
    return x.round(decimals=decimals)


def restart_state(w, nx: int, nu: int, N: int, n: int, thermal: bool, T_drop: float = 0.05,
                  carry_velocity: bool = True, decimals: int | None = 4):
    """(x_0, u_0) of the next horizon from solutions w (batch, wsize), numpy or torch:
    x_0 = x_N (temperatures - T_drop), u_0 = u_{N-1} (its fixed part, the joint velocities, is
    what the next horizon holds; zero without carry_velocity), both rounded (mpc_principal.py:365-373)."""
    off = nx + (N - 1) * (nu + nx)
    xN = w[:, off + nu:off + nu + nx]
    x0 = xN.clone() if hasattr(xN, "clone") else xN.copy()
    if thermal:
        x0[:, n:2 * n] = x0[:, n:2 * n] - T_drop
    u0 = w[:, off:off + nu] * (1.0 if carry_velocity else 0.0)
    return _round(x0, decimals), _round(u0, decimals)


class GRecedingHorizon:
    """Repeated solves of a generic problem (gocp.GOCP) for a batch of initial states, restarted
    as mpc_principal.py:357-377 restarts the Centauro MPC.

    The first solve differs between the reference's two Centauro loops:
      * RepeatedMPCwithThermal.py:445-448, 464-466: cold -- no x0 (IPOPT from 0, the `x0=sol0` call is
        commented out at L465) and no warm_start_init_point; run(x0, ...) with w0=None.
      * mpc_principal.py:348-351, 357-360: warm_start_init_point = yes already at s = 0, from x0 = sol0;
        run(x0, ..., w0=sol0, warm_first=True).
    From the second solve on both warm-start from the previous solution (L446 / L349)."""

    def __init__(self, spec: dict, carry_velocity: bool = True, T_drop: float = 0.05, decimals: int | None = 4,
                 models=None, restart_spec: dict | None = None, warm_start: bool = True, **opts):
        """restart_spec: the problem solved from the second step on (the Centauro loop rounds its
        relative-pose targets after the first solve, RepeatedMPCwithThermal.py:485-486); default spec.
        warm_start: IPOPT warm_start_init_point constants from the second solve on (L445-446)."""
        self.spec = spec
        self.g = GOCP(spec, models=models)
        self.g_restart = GOCP(restart_spec, models=self.g.models) if restart_spec is not None else self.g
        self.n = len(spec["q0"])
        self.thermal = bool(spec.get("thermal", False))
        self.carry_velocity = carry_velocity
        self.T_drop = T_drop
        self.decimals = decimals
        self.warm_start = warm_start
        self.opts = opts

    def next_initial(self, w):
        g = self.g
        return restart_state(w, g.nx, g.nu, g.N, self.n, self.thermal, self.T_drop, self.carry_velocity,
                             self.decimals)

    def run(self, x0, steps: int, u0=None, line_ref=None, device: int = 0, w0=None, warm_first: bool = False) -> list:
        """Device-resident loop; returns the per-step SolveResults (host copies).  w0: the first solve's start
        (the reference's sol0, B x wsize or one row for every problem); warm_first: that solve with IPOPT's
        warm_start_init_point constants (mpc_principal.py:349-351) instead of the cold initial point."""
        import torch

        g = self.g
        dev = torch.device("cuda", device)
        x = torch.as_tensor(np.atleast_2d(np.asarray(x0, float)), dtype=torch.float64, device=dev).contiguous()
        B = x.shape[0]
        u = None if u0 is None else torch.as_tensor(np.broadcast_to(np.asarray(u0, float), (B, g.nu)).copy(),
                                                      dtype=torch.float64, device=dev)
        lr = None if line_ref is None else torch.as_tensor(np.asarray(line_ref, float).reshape(B, 2),
                                                           dtype=torch.float64, device=dev).contiguous()
        wbuf = [torch.empty((B, g.wsize), dtype=torch.float64, device=dev) for _ in range(2)]
        out = {"status": torch.empty(B, dtype=torch.int32, device=dev),
               "iters": torch.empty(B, dtype=torch.int32, device=dev),
               "kkt": torch.empty(B, dtype=torch.float64, device=dev),
               "obj": torch.empty(B, dtype=torch.float64, device=dev)}
        stream = torch.cuda.current_stream(dev).cuda_stream
        res, prev = [], None
        if w0 is not None:
            prev = torch.as_tensor(np.broadcast_to(np.asarray(w0, float), (B, g.wsize)).copy(), dtype=torch.float64,
                                   device=dev).contiguous()
        for s in range(steps):
            w = wbuf[s % 2]
            ptr = {k: v.data_ptr() for k, v in out.items()}
            ptr["w"] = w.data_ptr()
            (g if s == 0 else self.g_restart).solve_dev(
                x.data_ptr(), None if u is None else u.data_ptr(), None if prev is None else prev.data_ptr(),
                None if lr is None else lr.data_ptr(), B, ptr, stream=stream,
                warm_start=(self.warm_start and s > 0) or (warm_first and s == 0 and prev is not None), **self.opts)
            res.append(SolveResult(w.cpu().numpy(), out["status"].cpu().numpy(), out["iters"].cpu().numpy(),
                                   out["kkt"].cpu().numpy(), out["obj"].cpu().numpy()))
            x, u = self.next_initial(w)
            x, u = x.contiguous(), u.contiguous()
            prev = w
        return res
