"""CPU-baseline helper (test/bench infrastructure only): the product's node functions
(``mpc_fatigue_amd/csrc/gfam.hpp``, forward-over-reverse lanes + closed-form assembly) compiled for the
host into ``oracle/libmfcpu.so`` and plugged into the generic oracle IPM (``oracle/mf_ocp.c``) as its
node-record / node-value provider.  The result is the same interior-point algorithm as the device
solver with efficient derivatives on the host -- the honest CPU baseline bench.py reports -- while
the hyper-dual restatement stays the parity checker.  Nothing in ``mpc_fatigue_amd`` imports this.

    fn = FastNodes(spec)                       # one per spec family / model
    w, R = solve_batch(specs, nthreads=16, **fn.opts_kw())   # this library's -O3 build of the IPM
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import generic as G
from . import oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "libmfcpu.so")
URDF_DIR = os.path.join(os.path.dirname(HERE), "mpc_fatigue_amd", "urdf")
GX = 32

NODE_CB = C.CFUNCTYPE(C.c_int, C.c_void_p, *([C.c_void_p] * 5), C.c_int, C.c_void_p)


class GParams(C.Structure):
    """Mirror of mf::GParams (mpc_fatigue_amd/csrc/gfam.hpp)."""
    _fields_ = [("N", C.c_int), ("h", C.c_double), ("eq_from", C.c_int),
                ("nf", C.c_int), ("use_line", C.c_int), ("thermal", C.c_int), ("fdir", C.c_double * 9),
                ("wF", C.c_double), ("wqd", C.c_double), ("wtau", C.c_double), ("wT", C.c_double),
                ("th_a", C.c_double), ("th_b", C.c_double), ("Ra", C.c_double), ("Rh", C.c_double),
                ("ktau", C.c_double * 16),
                ("box_mg", C.c_double), ("box_L", C.c_double), ("box_pdes", C.c_double * 3), ("w_box", C.c_double),
                ("w_qdb", C.c_double),
                ("x_lo", C.c_double * GX), ("x_hi", C.c_double * GX),
                ("tol", C.c_double), ("constr_viol_tol", C.c_double), ("mu_init", C.c_double), ("F_init", C.c_double),
                ("max_iter", C.c_int), ("max_soc", C.c_int), ("init_zero", C.c_int), ("has_u_init", C.c_int),
                ("warm_start", C.c_int), ("pad_ws", C.c_int), ("u_init", C.c_double * GX), ("force_from", C.c_int), ("tier1_from", C.c_int),
                ("tier1_to", C.c_int), ("target_decimals", C.c_int), ("dc_always", C.c_int),
                ("filter", C.c_int), ("dbg", C.c_int)]


def gparams(spec: dict) -> GParams:
    """Family parameters of a spec (the node functions read only these; bounds stay in the IPM)."""
    g = GParams()
    g.N, g.h, g.eq_from = spec["N"], spec["h"], 2
    if spec.get("family") == "box":
        g.box_mg, g.box_L, g.w_box, g.w_qdb = spec["box_mg"], spec["box_L"], spec["w_box"], spec["w_qd"]
        g.box_pdes[:] = list(spec["p_des"])
        if spec.get("thermal", False):
            g.thermal, g.th_a, g.th_b, g.Ra, g.Rh = 1, spec["th_a"], spec["th_b"], spec["Ra"], spec["Rh"]
            g.wT = spec.get("wT", 0.0)
            kt = np.zeros(16)
            kt[:12] = spec["ktau"]
            g.ktau[:] = list(kt)
    elif spec.get("family") == "centauro":
        g.box_mg, g.w_box, g.w_qdb, g.wF = spec["box_mg"], spec["w_box"], spec["w_qd"], spec["wF"]
        g.box_pdes[:] = list(spec["p_des"])
        g.thermal, g.th_a, g.th_b, g.Ra, g.Rh = 1, spec["th_a"], spec["th_b"], spec["Ra"], spec["Rh"]
        g.wT = spec.get("wT", 0.0)
        kt = np.zeros(16)
        kt[:14] = spec["ktau"]
        g.ktau[:] = list(kt)
        g.target_decimals, g.dc_always, g.eq_from = int(spec.get("target_decimals", -1)), 1, 1
    else:
        g.nf, g.use_line, g.thermal = spec["nf"], int(spec["use_line"]), int(spec.get("thermal", False))
        fd = np.zeros(9)
        fd[:3 * spec["nf"]] = np.asarray(spec["fdir"], float).reshape(-1)
        g.fdir[:] = list(fd)
        g.wF, g.wqd, g.wtau, g.wT = spec["wF"], spec["wqd"], spec["wtau"], spec.get("wT", 0.0)
        if g.thermal:
            g.th_a, g.th_b, g.Ra, g.Rh = spec["th_a"], spec["th_b"], spec["Ra"], spec["Rh"]
            kt = np.zeros(16)
            kt[:len(spec["ktau"])] = spec["ktau"]
            g.ktau[:] = list(kt)
    return g


_lib = None


def lib():
    global _lib
    if _lib is None:
        O.build()
        L = C.CDLL(LIB)
        L.mfc_create.restype = C.c_void_p
        L.mfc_create.argtypes = [C.c_int, C.c_char_p, C.c_char_p, C.c_char_p, C.c_char_p, C.POINTER(GParams)]
        L.mfc_free.argtypes = [C.c_void_p]
        assert L.mfc_gparams_size() == C.sizeof(GParams), "GParams mirror out of date"
        _lib = G.bind(L)
    return _lib


def family_code(spec: dict) -> int:
    if spec.get("family") == "box":
        return 4 if spec.get("thermal", False) else 0
    if spec.get("family") == "centauro":
        return 3
    if spec["nf"] != 1 or not spec["use_line"]:
        raise ValueError("cpu_fast instantiates the box, Centauro and the 6-DOF force+line chains only")
    return 2 if spec.get("thermal", False) else 1


_alive = []  # contexts stay alive for the process: opts_kw() hands out raw pointers into them


class FastNodes:
    """Host node functions for one spec (family, model, weights); thread-safe (read-only context)."""

    def __init__(self, spec: dict):
        L = lib()
        names = spec["urdf"] if isinstance(spec["urdf"], (list, tuple)) else [spec["urdf"], spec["urdf"]]
        txt = [open(os.path.join(URDF_DIR, u), "rb").read() for u in names]
        frames = spec.get("frames", [spec["frame"], spec["frame"]])
        self._g = gparams(spec)
        self._ctx = L.mfc_create(family_code(spec), txt[0], txt[1], frames[0].encode(), frames[1].encode(),
                                 C.byref(self._g))
        if not self._ctx:
            raise RuntimeError("mfc_create failed")
        self._L = L
        _alive.append(self)

    def opts_kw(self) -> dict:
        """Keyword arguments for oracle.generic.opts / solve / solve_batch."""
        return dict(node_cb=C.cast(self._L.mfc_node, C.c_void_p).value, node_ctx=self._ctx,
                    val_cb=C.cast(self._L.mfc_values, C.c_void_p).value)


def solve_batch(specs: list, nthreads: int = 0, **kw):
    """oracle.generic.solve_batch on this library's -O3 build of the generic IPM."""
    return G.solve_batch(specs, nthreads=nthreads, L=lib(), **kw)
