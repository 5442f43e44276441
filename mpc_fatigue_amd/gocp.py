"""Generic stage-structured OCPs on the MI355X: the dual-arm box (C3), thermal fatigue (a8) and the
Centauro thermal box lift (C4).

Replaces the per-node transcription loops + ``nlpsol('ipopt')`` of
``python/2_pilz_6_DOF/Box_Pilz_6DOF.py:219-456`` and of the thermal MPC
(``python/Centauro_script/RepeatedMPCwithThermal.py:183-402`` with
``python/Libraries/Tmodel_library.py:9-41``) by one ``mf_gproblem`` (``mf_gspec``, C ABI in
include/mpcfatigue.h) solved for a batch of initial states by the generic device solver
(csrc/gipm.hip).  The decision vector keeps the reference layout ``[x_0 | (u_k, x_{k+1})]``,
which for the box is exactly the CSV row ``Box_Pilz_6DOF.py:464-466`` writes.

    ocp = GOCP(problems.box_dual(N=50))
    res = ocp.solve_box(q0[None])          # equilibrium-tolerance homotopy, then the reference problem
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib
from .ocp import SolveResult
from .problems import box_homotopy_tolerances, box_u_init, read_urdf

INF = float("inf")
FAM_CHAIN, FAM_BOX, FAM_CENTAURO = 0, 1, 2


@dataclass
class GBounds:
    x_lo: np.ndarray
    x_hi: np.ndarray
    u_lo: np.ndarray
    u_hi: np.ndarray
    c_lo: np.ndarray
    c_hi: np.ndarray
    x0: np.ndarray


def bounds(spec: dict, n: int) -> GBounds:
    """Per-node bounds of a problem spec in the generic NLP form."""
    N = spec["N"]
    if spec.get("family") == "centauro":
        nq = 14
        u_lo = np.hstack([np.tile(np.asarray(spec["qd_lo"], float), (N, 1)), np.full((N, 6), -INF)])
        u_hi = np.hstack([np.tile(np.asarray(spec["qd_hi"], float), (N, 1)), np.full((N, 6), INF)])
        u_lo[0, :nq] = u_hi[0, :nq] = np.asarray(spec["qd0"], float)
        return GBounds(np.r_[spec["q_lo"], np.full(nq, spec["T_lo"])], np.r_[spec["q_hi"], np.full(nq, spec["T_hi"])],
                       u_lo, u_hi, np.asarray(spec["tau_lo"], float), np.asarray(spec["tau_hi"], float),
                       np.r_[spec["q0"], spec["T0"]])
    if spec.get("family") == "box":
        tol = spec["pos_toll"]
        c_lo = np.hstack([np.full((N, 6), -tol), np.asarray(spec["tau_lo"], float)])
        c_hi = np.hstack([np.full((N, 6), tol), np.asarray(spec["tau_hi"], float)])
        u_lo = np.hstack([np.tile(np.asarray(spec["qd_lo"], float), (N, 1)), np.full((N, 6), -INF)])
        u_hi = np.hstack([np.tile(np.asarray(spec["qd_hi"], float), (N, 1)), np.full((N, 6), INF)])
        u_lo[0, :12] = u_hi[0, :12] = np.asarray(spec["qd0"], float)
        x_lo, x_hi = np.asarray(spec["q_lo"], float), np.asarray(spec["q_hi"], float)
        x0 = np.asarray(spec["q0"], float)
        if spec.get("thermal", False):  # shared fatigue budget (problems.box_shared_fatigue)
            x_lo, x_hi = np.r_[x_lo, np.full(12, spec["T_lo"])], np.r_[x_hi, np.full(12, spec["T_hi"])]
            x0 = np.r_[x0, np.broadcast_to(np.asarray(spec["T0"], float), (12,))]
            c_lo = np.hstack([c_lo, np.full((N, 1), -INF)])
            c_hi = np.hstack([c_hi, np.full((N, 1), spec["T_budget"])])
        return GBounds(x_lo, x_hi, u_lo, u_hi, c_lo, c_hi, x0)
    nf = spec["nf"]
    x_lo = np.broadcast_to(np.asarray(spec["q_lo"], float), (n,))
    x_hi = np.broadcast_to(np.asarray(spec["q_hi"], float), (n,))
    x0 = np.asarray(spec["q0"], float)
    if spec.get("thermal", False):
        x_lo = np.r_[x_lo, np.full(n, spec["T_lo"])]
        x_hi = np.r_[x_hi, np.full(n, spec["T_hi"])]
        x0 = np.r_[x0, np.broadcast_to(np.asarray(spec["T0"], float), (n,))]
    c_lo = np.broadcast_to(np.asarray(spec["tau_lo"], float), (N, n))
    c_hi = np.broadcast_to(np.asarray(spec["tau_hi"], float), (N, n))
    u_lo = np.hstack([np.tile(np.broadcast_to(np.asarray(spec["qd_lo"], float), (n,)), (N, 1)), np.full((N, nf), -INF)])
    u_hi = np.hstack([np.tile(np.broadcast_to(np.asarray(spec["qd_hi"], float), (n,)), (N, 1)), np.full((N, nf), INF)])
    u_lo[0, :n] = u_hi[0, :n] = np.broadcast_to(np.asarray(spec.get("qd0", 0.0), float), (n,))
    return GBounds(np.asarray(x_lo, float), np.asarray(x_hi, float), u_lo, u_hi, c_lo, c_hi, x0)


class GOCP:
    """Owning handle of an ``mf_gproblem`` built from a spec of ``mpc_fatigue_amd.problems``."""

    def __init__(self, spec: dict, models=None):
        self.spec = spec
        urdfs = spec["urdf"] if isinstance(spec["urdf"], (list, tuple)) else [spec["urdf"]]
        self.models = models if models is not None else [_lib.Model(read_urdf(u)) for u in urdfs]
        n = self.models[0].nq
        cent = spec.get("family") == "centauro"
        box = spec.get("family") == "box"
        two = box or cent
        g = _lib.GSpec()
        g.family = FAM_CENTAURO if cent else (FAM_BOX if box else FAM_CHAIN)
        g.N, g.h, g.eq_from = spec["N"], spec["h"], (1 if cent else 2)
        frames = spec.get("frames", [spec["frame"], spec["frame"]])
        g.frame0 = self.models[0].frame_id(frames[0])
        g.frame1 = self.models[1].frame_id(frames[1]) if two else 0
        g.target_decimals = int(spec.get("target_decimals", -1))
        self.nem = 6 if cent else 0
        if cent:
            g.box_mg, g.w_box, g.w_qd, g.wF = spec["box_mg"], spec["w_box"], spec["w_qd"], spec["wF"]
            g.box_pdes[:] = list(spec["p_des"])
            g.thermal, g.wT = 1, spec.get("wT", 0.0)
            g.th_a, g.th_b, g.Ra, g.Rh = spec["th_a"], spec["th_b"], spec["Ra"], spec["Rh"]
            kt = np.zeros(_lib.MF_MAX_JOINTS)
            kt[:14] = spec["ktau"]
            g.ktau[:] = list(kt)
        elif box:
            g.box_mg, g.box_L, g.w_box, g.w_qd = spec["box_mg"], spec["box_L"], spec["w_box"], spec["w_qd"]
            g.box_pdes[:] = list(spec["p_des"])
            if spec.get("thermal", False):
                g.thermal, g.wT = 1, spec.get("wT", 0.0)
                g.th_a, g.th_b, g.Ra, g.Rh = spec["th_a"], spec["th_b"], spec["Ra"], spec["Rh"]
                kt = np.zeros(_lib.MF_MAX_JOINTS)
                kt[:12] = spec["ktau"]
                g.ktau[:] = list(kt)
        else:
            g.nf, g.use_line = spec["nf"], int(spec["use_line"])
            fd = np.zeros(9)
            fd[:3 * spec["nf"]] = np.asarray(spec["fdir"], float).reshape(-1)
            g.fdir[:] = list(fd)
            g.line_ref[:] = list(spec.get("line_ref", [0.0, 0.0]))
            g.wF, g.wqd, g.wtau, g.wT = spec["wF"], spec["wqd"], spec["wtau"], spec.get("wT", 0.0)
            if spec.get("thermal", False):
                g.thermal = 1
                g.th_a, g.th_b, g.Ra, g.Rh = spec["th_a"], spec["th_b"], spec["Ra"], spec["Rh"]
                kt = np.zeros(_lib.MF_MAX_JOINTS)
                kt[:n] = spec["ktau"]
                g.ktau[:] = list(kt)
        bd = bounds(spec, n)
        lo = np.full(_lib.MF_GX_MAX, -INF)
        hi = np.full(_lib.MF_GX_MAX, INF)
        lo[:len(bd.x_lo)] = bd.x_lo
        hi[:len(bd.x_hi)] = bd.x_hi
        g.x_lo[:] = list(lo)
        g.x_hi[:] = list(hi)
        self._keep = [np.ascontiguousarray(a, dtype=np.float64) for a in (bd.u_lo, bd.u_hi, bd.c_lo, bd.c_hi)]
        g.u_lo, g.u_hi, g.c_lo, g.c_hi = (_lib.dptr(a) for a in self._keep)
        self.bounds = bd
        h = C.c_void_p()
        _lib.check(_lib.lib().mf_gproblem_create(self.models[0].handle, self.models[1].handle if two else None,
                                                 C.byref(g), C.byref(h)))
        self._h = h
        d = (C.c_int * 5)()
        _lib.check(_lib.lib().mf_gproblem_dims(h, d))
        self.nx, self.nu, self.ni, self.ne, self.wsize = list(d)
        self.N = spec["N"]
        self.gspec = g

    @property
    def handle(self):
        return self._h

    def opts(self, tol=1e-8, constr_viol_tol=1e-8, max_iter=300, mu_init=0.1, init_zero=False, F_init=0.0,
             u_init=None, max_soc=4, verbose=False, warm_start=False, filter=False, bound_relax=0.0,
             resto_hard_dyn=False, inertia_spec=0):
        """mf_gopts; warm_start: IPOPT warm_start_init_point constants for a w0 start; filter: IPOPT's
        globalisation (filter line search, watchdog, soft restoration, restoration phase) instead of the
        l1-merit search; bound_relax: IPOPT's bound_relax_factor; resto_hard_dyn: the restoration problem without
        elastic variables on the dynamics rows (the pre-round-5 variant; IPOPT's own restoration by default);
        inertia_spec: -1 turns off the concurrent inertia tries of the few-horizons tail (results are the same)."""
        o = _lib.GOpts(tol, constr_viol_tol, max_iter, mu_init, int(init_zero), F_init, None, max_soc, int(verbose),
                       int(warm_start), int(filter), float(bound_relax), int(resto_hard_dyn), int(inertia_spec))
        if u_init is not None:
            o._u = np.ascontiguousarray(u_init, dtype=np.float64)
            o.u_init = _lib.dptr(o._u)
        return o

    def solve(self, x0=None, u0=None, w0=None, line_ref=None, device: int = 0, **opts) -> SolveResult:
        """Batched solve from initial states x0 (batch x nx; default the spec's)."""
        x0 = self.bounds.x0[None] if x0 is None else x0
        x0 = np.ascontiguousarray(np.atleast_2d(np.asarray(x0, float)))
        B = x0.shape[0]
        u0a = None if u0 is None else np.ascontiguousarray(np.broadcast_to(np.asarray(u0, float), (B, self.nu)))
        w0a = None if w0 is None else np.ascontiguousarray(np.broadcast_to(np.asarray(w0, float), (B, self.wsize)))
        lr = None if line_ref is None else np.ascontiguousarray(np.asarray(line_ref, float).reshape(B, 2))
        o = self.opts(**opts)
        w = np.zeros((B, self.wsize))
        st, it = np.zeros(B, np.int32), np.zeros(B, np.int32)
        kkt, obj = np.zeros(B), np.zeros(B)
        _lib.check(_lib.lib().mf_gsolve_batch(self._h, B, _lib.dptr(x0), None if u0a is None else _lib.dptr(u0a),
                                              None if w0a is None else _lib.dptr(w0a),
                                              None if lr is None else _lib.dptr(lr), C.byref(o), _lib.dptr(w),
                                              _lib.iptr(st), _lib.iptr(it), _lib.dptr(kkt), _lib.dptr(obj), device))
        return SolveResult(w, st, it, kkt, obj)

    def solve_dev(self, x0_ptr, u0_ptr, w0_ptr, lref_ptr, batch: int, out: dict, stream: int = 0, **opts) -> None:
        """Device-pointer form (torch tensors' data_ptr(); u0 / w0 / lref may be None)."""
        o = self.opts(**opts)
        _lib.check(_lib.lib().mf_gsolve_batch_dev(self._h, batch, x0_ptr, u0_ptr, w0_ptr, lref_ptr, C.byref(o),
                                                  out["w"], out["status"], out["iters"], out["kkt"], out["obj"],
                                                  stream))

    def solve_stream_dev(self, x0_ptr, u0_ptr, w0_ptr, lref_ptr, total: int, slots: int, out: dict, stream: int = 0,
                         **opts) -> None:
        """Continuous batching (mf_gsolve_stream_dev): `slots` concurrent solves work through `total` problems
        (inputs / outputs with `total` rows, device pointers); each problem's result equals solve_dev's."""
        o = self.opts(**opts)
        _lib.check(_lib.lib().mf_gsolve_stream_dev(self._h, total, slots, x0_ptr, u0_ptr, w0_ptr, lref_ptr, C.byref(o),
                                                   out["w"], out["status"], out["iters"], out["kkt"], out["obj"],
                                                   stream))

    def solve_stream(self, x0, slots: int, u0=None, w0=None, line_ref=None, **opts) -> SolveResult:
        """Host-array convenience over solve_stream_dev (torch device buffers)."""
        import torch
        dev = torch.device("cuda", torch.cuda.current_device())
        x0 = np.ascontiguousarray(np.atleast_2d(x0), dtype=np.float64)
        T = x0.shape[0]
        t = lambda a, n: None if a is None else torch.as_tensor(
            np.broadcast_to(np.asarray(a, float), (T, n)).copy(), device=dev)
        xd, ud, wd, ld = t(x0, self.nx), t(u0, self.nu), t(w0, self.wsize), t(line_ref, 2)
        out = {"w": torch.empty((T, self.wsize), dtype=torch.float64, device=dev),
               "status": torch.empty(T, dtype=torch.int32, device=dev), "iters": torch.empty(T, dtype=torch.int32, device=dev),
               "kkt": torch.empty(T, dtype=torch.float64, device=dev), "obj": torch.empty(T, dtype=torch.float64, device=dev)}
        p = lambda a: None if a is None else a.data_ptr()
        self.solve_stream_dev(p(xd), p(ud), p(wd), p(ld), T, slots, {k: v.data_ptr() for k, v in out.items()},
                              stream=torch.cuda.current_stream(dev).cuda_stream, **opts)
        torch.cuda.synchronize(dev)
        return SolveResult(*(out[k].cpu().numpy() for k in ("w", "status", "iters", "kkt", "obj")))

    def node_record(self, xu, yi, ye, lam, line_ref=None, device: int = 0) -> np.ndarray:
        """One node record from the device kernel (layout: mf_gnode_record).  ye = [state rows | mixed rows];
        line_ref: the line reference (chain) or the 6 pose targets (Centauro)."""
        ne = self.ne + self.nem
        arr = [np.ascontiguousarray(a, dtype=np.float64) for a in (xu, yi, ye if ne else np.zeros(1), lam)]
        lr = None if line_ref is None else np.ascontiguousarray(line_ref, dtype=np.float64)
        rec = np.zeros(8192)
        n = _lib.check(_lib.lib().mf_gnode_record(self._h, *[_lib.dptr(a) for a in arr],
                                                  None if lr is None else _lib.dptr(lr), _lib.dptr(rec), device))
        return rec[:n]

    def solve_box(self, q0=None, device: int = 0, tolerances=None, **opts) -> tuple[SolveResult, list]:
        """C3 solve: the equilibrium-tolerance homotopy of problems.box_homotopy_tolerances, each
        stage a solve warm-started from the previous stage's primal point; the last stage is the
        reference problem itself (pos_toll = 1e-4).  Returns (last result, per-stage results)."""
        assert self.spec.get("family") == "box"
        stages = []
        w = None
        opts.setdefault("max_iter", 1000)
        for tol in (tolerances or box_homotopy_tolerances()):
            g = GOCP(dict(self.spec, pos_toll=tol), models=self.models)
            r = g.solve(x0=q0, w0=w, device=device, u_init=box_u_init(self.spec), **opts)
            stages.append(r)
            w = r.w
        return stages[-1], stages

    COUNTERS = ("iterations", "status", "inertia_corrections", "ls_failures", "soc_steps", "resto_phases",
                "watchdog_starts", "soft_resto_steps", "wd_failed_searches", "resto_iterations")

    def counters(self, b: int = 0) -> dict:
        """Solver counters of problem b after the last solve (mf_gdebug_counters)."""
        out = np.zeros(10, np.int32)
        _lib.check(_lib.lib().mf_gdebug_counters(self._h, int(b), _lib.iptr(out)))
        return dict(zip(self.COUNTERS, (int(v) for v in out)))

    KERNELS = ("k_geval", "k_gasm", "k_gpre", "k_gkkt", "k_gls")

    def timing(self, enable: bool = True) -> None:
        """Per-phase HIP-event timing of the next solves on this handle (mf_gproblem_timing; resets the totals)."""
        _lib.check(_lib.lib().mf_gproblem_timing(self._h, int(enable)))

    def kernel_stats(self) -> dict:
        """{phase: (total ms, launches)} since timing(True)."""
        ms, n, ne = (C.c_double * 5)(), (C.c_long * 5)(), C.c_longlong(0)
        _lib.check(_lib.lib().mf_gproblem_kernel_stats(self._h, ms, n, C.byref(ne)))
        return {k: (float(ms[i]), int(n[i])) for i, k in enumerate(self.KERNELS)}

    def node_evals(self) -> int:
        """Node evaluations k_geval made since timing(True) (device-counted)."""
        ms, n, ne = (C.c_double * 5)(), (C.c_long * 5)(), C.c_longlong(0)
        _lib.check(_lib.lib().mf_gproblem_kernel_stats(self._h, ms, n, C.byref(ne)))
        return int(ne.value)

    def point(self, b: int = 0) -> tuple[np.ndarray, np.ndarray]:
        """(slacks (N x ni), duals [lam | yi | ye | zxL | zxU | zuL | zuU | vL | vU]) of problem b after the last solve
        (mf_gdebug_slacks / mf_gdebug_duals): with the solution vector, the primal-dual point an oracle-side KKT check
        takes."""
        N = self.N
        s = np.zeros(N * max(1, self.ni))
        _lib.check(_lib.lib().mf_gdebug_slacks(self._h, int(b), _lib.dptr(s)))
        nd = N * self.nx + 3 * N * max(1, self.ni) + N * max(1, self.ne + self.nem) + 2 * (N + 1) * self.nx \
            + 2 * N * self.nu + 1
        d = np.zeros(nd + 64)
        n = _lib.check(_lib.lib().mf_gdebug_duals(self._h, int(b), _lib.dptr(d)))
        return s[:N * self.ni], d[:n - 1]

    def q_traj(self, w: np.ndarray) -> np.ndarray:
        """State trajectory x_0..x_N (N+1, nx) of a solution vector."""
        nx, nu, N = self.nx, self.nu, self.N
        return np.vstack([w[:nx][None], w[nx:].reshape(N, nu + nx)[:, nu:]])

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and _lib._lib is not None:
            _lib._lib.mf_gproblem_free(h)
            self._h = None
