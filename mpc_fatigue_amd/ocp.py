"""Fatigue-aware OCP: problem spec -> batched MI355X interior-point solve.

Replaces the per-node symbolic transcription loop + ``nlpsol('ipopt')`` of the
reference scripts (e.g. python/Pilz_6_DOF/force_optimization_pilz_6DOF.py:103-197)
with one ``mf_problem`` built from a spec dict (``mpc_fatigue_amd.problems``)
and solved for a batch of initial states on the GPU.

    ocp = OCP(problems.pilz6_force(N=100))
    res = ocp.solve(q0_batch, line_ref=refs)      # res.w in the reference layout
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib
from .problems import read_urdf

STATUS = {0: "converged", 1: "max_iter", 2: "line_search_failure", 3: "inertia_failure"}


@dataclass
class SolveResult:
    w: np.ndarray          # (batch, wsize) reference layout [q0 | (qd_k, F_k, q_{k+1})]
    status: np.ndarray     # (batch,) int
    iters: np.ndarray      # (batch,) int
    kkt: np.ndarray        # (batch,) final scaled KKT error E_0
    obj: np.ndarray        # (batch,) objective

    @property
    def converged(self) -> np.ndarray:
        return self.status == 0


def default_opts(tol=1e-8, constr_viol_tol=1e-8, max_iter=200, mu_init=0.1, F_init=0.0, verbose=False,
                 warm_start=False):
    """mf_solver_opts; warm_start: IPOPT warm_start_init_point constants for a w0 start."""
    return _lib.SolverOpts(tol, constr_viol_tol, max_iter, mu_init, F_init, int(verbose), int(warm_start))


class OCP:
    def __init__(self, spec: dict, model: _lib.Model | None = None):
        self.spec = spec
        self.model = model if model is not None else _lib.Model(read_urdf(spec["urdf"]))
        n = self.model.nq
        self.n, self.N, self.nf = n, spec["N"], spec["nf"]
        self.nl = 2 if spec["use_line"] else 0
        ps = _lib.ProblemSpec()
        ps.N = spec["N"]
        ps.h = spec["h"]
        ps.frame = self.model.frame_id(spec["frame"])
        ps.nf = spec["nf"]
        fd = np.zeros(9)
        fd[:3 * spec["nf"]] = np.asarray(spec["fdir"], float).reshape(-1)
        ps.fdir[:] = list(fd)
        ps.use_line = int(spec["use_line"])
        ps.line_ref[:] = list(spec.get("line_ref", [0.0, 0.0]))
        ps.wF, ps.wqd, ps.wtau = spec["wF"], spec["wqd"], spec["wtau"]

        def arr(v, fill):
            a = np.full(_lib.MF_MAX_JOINTS, fill, float)
            a[:n] = np.broadcast_to(np.asarray(v, float), (n,))
            return list(a)

        ps.qd0[:] = arr(spec.get("qd0", 0.0), 0.0)
        ps.qd_lo[:] = arr(spec["qd_lo"], -np.inf)
        ps.qd_hi[:] = arr(spec["qd_hi"], np.inf)
        ps.q_lo[:] = arr(spec["q_lo"], -np.inf)
        ps.q_hi[:] = arr(spec["q_hi"], np.inf)
        self._tlo = np.ascontiguousarray(np.broadcast_to(np.asarray(spec["tau_lo"], float), (self.N, n)))
        self._thi = np.ascontiguousarray(np.broadcast_to(np.asarray(spec["tau_hi"], float), (self.N, n)))
        ps.tau_lo = _lib.dptr(self._tlo)
        ps.tau_hi = _lib.dptr(self._thi)
        h = C.c_void_p()
        _lib.check(_lib.lib().mf_problem_create(self.model.handle, C.byref(ps), C.byref(h)))
        self._h = h
        self.wsize = _lib.lib().mf_problem_wsize(h)

    @property
    def handle(self):
        return self._h

    def solve(self, q0, line_ref=None, device: int = 0, **opts) -> SolveResult:
        q0 = np.ascontiguousarray(np.atleast_2d(np.asarray(q0, float)))
        B = q0.shape[0]
        lr = None if line_ref is None else np.ascontiguousarray(np.asarray(line_ref, float).reshape(B, 2))
        o = default_opts(**opts)
        w = np.zeros((B, self.wsize))
        st = np.zeros(B, np.int32)
        it = np.zeros(B, np.int32)
        kkt = np.zeros(B)
        obj = np.zeros(B)
        _lib.check(_lib.lib().mf_solve_batch(self._h, B, _lib.dptr(q0), None if lr is None else _lib.dptr(lr),
                                             C.byref(o), _lib.dptr(w), _lib.iptr(st), _lib.iptr(it),
                                             _lib.dptr(kkt), _lib.dptr(obj), device))
        return SolveResult(w, st, it, kkt, obj)

    def solve_ws(self, q0, qd0=None, w0=None, line_ref=None, device: int = 0, **opts) -> SolveResult:
        """Warm-started solve (mf_solve_batch_ws): per-problem fixed qd_0 and a warm start w0 in
        the w layout, as the receding-horizon scripts call Solver(x0 = sol, ...)."""
        q0 = np.ascontiguousarray(np.atleast_2d(np.asarray(q0, float)))
        B = q0.shape[0]
        qd = None if qd0 is None else np.ascontiguousarray(np.broadcast_to(np.asarray(qd0, float), (B, self.n)))
        w0a = None if w0 is None else np.ascontiguousarray(np.broadcast_to(np.asarray(w0, float), (B, self.wsize)))
        lr = None if line_ref is None else np.ascontiguousarray(np.asarray(line_ref, float).reshape(B, 2))
        o = default_opts(**opts)
        w = np.zeros((B, self.wsize))
        st = np.zeros(B, np.int32)
        it = np.zeros(B, np.int32)
        kkt = np.zeros(B)
        obj = np.zeros(B)
        _lib.check(_lib.lib().mf_solve_batch_ws(self._h, B, _lib.dptr(q0), None if qd is None else _lib.dptr(qd),
                                                None if w0a is None else _lib.dptr(w0a),
                                                None if lr is None else _lib.dptr(lr), C.byref(o), _lib.dptr(w),
                                                _lib.iptr(st), _lib.iptr(it), _lib.dptr(kkt), _lib.dptr(obj), device))
        return SolveResult(w, st, it, kkt, obj)

    def solve_ws_dev(self, q0_ptr: int, qd0_ptr, w0_ptr, lref_ptr, batch: int, out: dict, stream: int = 0,
                     **opts) -> None:
        """Device-pointer form of solve_ws (qd0_ptr / w0_ptr / lref_ptr may be None)."""
        o = default_opts(**opts)
        _lib.check(_lib.lib().mf_solve_batch_ws_dev(self._h, batch, q0_ptr, qd0_ptr, w0_ptr, lref_ptr, C.byref(o),
                                                    out["w"], out["status"], out["iters"], out["kkt"], out["obj"],
                                                    stream))

    def solve_dev(self, q0_ptr: int, lref_ptr: int | None, batch: int, out: dict, stream: int = 0, **opts) -> None:
        """All pointers are device addresses (e.g. torch tensors' data_ptr())."""
        o = default_opts(**opts)
        _lib.check(_lib.lib().mf_solve_batch_dev(self._h, batch, q0_ptr, lref_ptr, C.byref(o), out["w"],
                                                 out["status"], out["iters"], out["kkt"], out["obj"], stream))

    def timing(self, enable: bool = True) -> None:
        _lib.check(_lib.lib().mf_problem_timing(self._h, int(enable)))

    def kernel_stats(self) -> dict:
        """{kernel name: (total ms, launches)} of the solver's launches since timing(True)."""
        K = _lib.MF_NKERNELS
        ms = np.zeros(K)
        n = (C.c_long * K)()
        _lib.check(_lib.lib().mf_problem_kernel_stats(self._h, _lib.dptr(ms), n))
        out = {}
        for i in range(K):
            name = _lib.lib().mf_kernel_name(i).decode()
            if name:
                out[name] = (float(ms[i]), int(n[i]))
        return out

    def trace(self) -> dict:
        """Per-chunk trace of the last timed solve (mf_problem_trace): iteration at the chunk start,
        problems running at its start, GPU ms of the chunk's launches."""
        L = _lib.lib()
        n = _lib.check(L.mf_problem_trace(self._h, None, None, None, 0))
        it, run, ms = np.zeros(n, np.int32), np.zeros(n, np.int32), np.zeros(n)
        L.mf_problem_trace(self._h, _lib.iptr(it), _lib.iptr(run), _lib.dptr(ms), n)
        return {"iter": it, "running": run, "ms": ms}

    def node_eval(self, x, u, line_ref=None):
        """(x, u) -> (xnext, g, cost, jac) for a batch of shooting nodes (mf_node_eval)."""
        n, nf, nl = self.n, self.nf, self.nl
        x = np.ascontiguousarray(np.asarray(x, float).reshape(-1, n))
        u = np.ascontiguousarray(np.asarray(u, float).reshape(-1, n + nf))
        K = x.shape[0]
        lr = None if line_ref is None else np.ascontiguousarray(np.asarray(line_ref, float).reshape(K, 2))
        xn, g, c = np.zeros((K, n)), np.zeros((K, n + nl)), np.zeros(K)
        nrow, ncol = 2 * n + nl + 1, 2 * n + nf
        jac = np.zeros((K, ncol, nrow))
        _lib.check(_lib.lib().mf_node_eval(self._h, _lib.dptr(x), _lib.dptr(u), None if lr is None else _lib.dptr(lr),
                                           _lib.dptr(xn), _lib.dptr(g), _lib.dptr(c), _lib.dptr(jac), K))
        return xn, g, c, jac.transpose(0, 2, 1)

    def unpack(self, w: np.ndarray):
        """Reference layout -> (q (N+1,n), qd (N,n), F (N,nf))."""
        n, N, nf = self.n, self.N, self.nf
        q0 = w[:n]
        blk = w[n:].reshape(N, 2 * n + nf)
        q = np.vstack([q0[None], blk[:, n + nf:]])
        return q, blk[:, :n], blk[:, n:n + nf]

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and _lib._lib is not None:
            _lib._lib.mf_problem_free(h)
            self._h = None
