"""ctypes binding of libmpcfatigue.so (C ABI: include/mpcfatigue.h).

The library is built in-tree (``mpc_fatigue_amd/libmpcfatigue.so``) by
``build()`` / ``make -C mpc_fatigue_amd``.  There is deliberately no CPU
fallback: if the shared object is missing, or the process has no HIP device,
every compute call raises ``MFError``.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# MF_LIB selects a diagnostic build of the same library (e.g. libmpcfatigue_stamps.so)
LIB_PATH = os.path.join(HERE, os.environ.get("MF_LIB", "libmpcfatigue.so"))
MF_MAX_JOINTS = 16
MF_NKERNELS = 5

MF_ERR = {0: "OK", -1: "ARG", -2: "URDF", -3: "FRAME", -4: "DEVICE", -5: "UNSUPPORTED", -6: "NOMEM"}


class MFError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"libmpcfatigue error {code} ({MF_ERR.get(code, '?')}): {msg}")
        self.code = code


def build(force: bool = False) -> str:
    """Compile libmpcfatigue.so for gfx950 with hipcc (in-tree)."""
    args = ["make", "-s", "-C", HERE, "-j4"]
    if force:
        subprocess.check_call(["make", "-s", "-C", HERE, "clean"])
    subprocess.check_call(args)
    return LIB_PATH


class ProblemSpec(C.Structure):
    _fields_ = [
        ("N", C.c_int), ("h", C.c_double), ("frame", C.c_int), ("nf", C.c_int),
        ("fdir", C.c_double * 9), ("use_line", C.c_int), ("line_ref", C.c_double * 2),
        ("wF", C.c_double), ("wqd", C.c_double), ("wtau", C.c_double),
        ("qd0", C.c_double * MF_MAX_JOINTS),
        ("qd_lo", C.c_double * MF_MAX_JOINTS), ("qd_hi", C.c_double * MF_MAX_JOINTS),
        ("q_lo", C.c_double * MF_MAX_JOINTS), ("q_hi", C.c_double * MF_MAX_JOINTS),
        ("tau_lo", C.POINTER(C.c_double)), ("tau_hi", C.POINTER(C.c_double)),
    ]


MF_GX_MAX = 32


class GSpec(C.Structure):
    """mf_gspec (include/mpcfatigue.h): generic stage-structured OCP (box C3, thermal a8, Centauro C4)."""
    _fields_ = [
        ("family", C.c_int), ("N", C.c_int), ("h", C.c_double), ("frame0", C.c_int), ("frame1", C.c_int),
        ("eq_from", C.c_int), ("nf", C.c_int), ("fdir", C.c_double * 9), ("use_line", C.c_int),
        ("line_ref", C.c_double * 2), ("wF", C.c_double), ("wqd", C.c_double), ("wtau", C.c_double),
        ("wT", C.c_double), ("thermal", C.c_int), ("th_a", C.c_double), ("th_b", C.c_double), ("Ra", C.c_double),
        ("Rh", C.c_double), ("ktau", C.c_double * MF_MAX_JOINTS),
        ("box_mg", C.c_double), ("box_L", C.c_double), ("box_pdes", C.c_double * 3), ("w_box", C.c_double),
        ("w_qd", C.c_double),
        ("x_lo", C.c_double * MF_GX_MAX), ("x_hi", C.c_double * MF_GX_MAX),
        ("u_lo", C.POINTER(C.c_double)), ("u_hi", C.POINTER(C.c_double)),
        ("c_lo", C.POINTER(C.c_double)), ("c_hi", C.POINTER(C.c_double)),
        ("target_decimals", C.c_int),
    ]


class GOpts(C.Structure):
    """mf_gopts (include/mpcfatigue.h)."""
    _fields_ = [("tol", C.c_double), ("constr_viol_tol", C.c_double), ("max_iter", C.c_int),
                ("mu_init", C.c_double), ("init_zero", C.c_int), ("F_init", C.c_double),
                ("u_init", C.POINTER(C.c_double)), ("max_soc", C.c_int), ("verbose", C.c_int),
                ("warm_start", C.c_int), ("filter", C.c_int), ("bound_relax", C.c_double),
                ("resto_hard_dyn", C.c_int), ("inertia_spec", C.c_int)]


class SolverOpts(C.Structure):
    _fields_ = [("tol", C.c_double), ("constr_viol_tol", C.c_double), ("max_iter", C.c_int),
                ("mu_init", C.c_double), ("F_init", C.c_double), ("verbose", C.c_int), ("warm_start", C.c_int)]


_lib = None


def _hip_runtimes() -> list[str]:
    """Distinct libamdhip64 files mapped into this process (/proc/self/maps)."""
    seen = set()
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                p = line.split()[-1] if line.strip() else ""
                if "libamdhip64" in os.path.basename(p):
                    seen.add(os.path.realpath(p))
    except OSError:
        pass
    return sorted(seen)


def _torch_runtime_first() -> None:
    """One HIP runtime per process.  torch bundles its own libamdhip64 under the same soname (libamdhip64.so.7) as
    the ROCm one this library links; its libc10_hip asks for it by the unversioned name, so if ROCm's copy were
    mapped first torch would map a second runtime next to it and report "No HIP GPUs are available".  Importing
    torch first (when it is installed) maps torch's runtime, and the dynamic linker then satisfies this library's
    libamdhip64.so.7 with that same object."""
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


def lib() -> C.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise MFError(-4, f"{LIB_PATH} not built (run __graft_entry__.build() or make -C mpc_fatigue_amd)")
    _torch_runtime_first()
    L = C.CDLL(LIB_PATH)
    rt = _hip_runtimes()
    if len(rt) > 1:
        raise MFError(-4, "two HIP runtimes mapped in one process (" + ", ".join(rt) + "): import torch before "
                          "anything that loads ROCm's libamdhip64 directly")
    vp, dp, ip, cp = C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_int), C.c_char_p
    sig = {
        "mf_model_from_urdf": ([cp, C.POINTER(vp)], C.c_int),
        "mf_model_free": ([vp], None),
        "mf_model_nq": ([vp], C.c_int),
        "mf_model_export": ([vp, dp, C.c_int], C.c_int),
        "mf_frame_id": ([vp, cp], C.c_int),
        "mf_frame_export": ([vp, C.c_int, dp], C.c_int),
        "mf_id": ([vp, dp, dp, dp, dp, C.c_int], C.c_int),
        "mf_fk": ([vp, C.c_int, dp, dp, dp, C.c_int], C.c_int),
        "mf_jac": ([vp, C.c_int, dp, dp, C.c_int], C.c_int),
        "mf_id_dev": ([vp, vp, vp, vp, vp, C.c_int, vp], C.c_int),
        "mf_fk_dev": ([vp, C.c_int, vp, vp, vp, C.c_int, vp], C.c_int),
        "mf_jac_dev": ([vp, C.c_int, vp, vp, C.c_int, vp], C.c_int),
        "mf_problem_create": ([vp, C.POINTER(ProblemSpec), C.POINTER(vp)], C.c_int),
        "mf_problem_free": ([vp], None),
        "mf_problem_wsize": ([vp], C.c_int),
        "mf_node_eval": ([vp, dp, dp, dp, dp, dp, dp, dp, C.c_int], C.c_int),
        "mf_solve_batch": ([vp, C.c_int, dp, dp, C.POINTER(SolverOpts), dp, ip, ip, dp, dp, C.c_int], C.c_int),
        "mf_solve_batch_dev": ([vp, C.c_int, vp, vp, C.POINTER(SolverOpts), vp, vp, vp, vp, vp, vp], C.c_int),
        "mf_solve_batch_ws": ([vp, C.c_int, dp, dp, dp, dp, C.POINTER(SolverOpts), dp, ip, ip, dp, dp, C.c_int], C.c_int),
        "mf_solve_batch_ws_dev": ([vp, C.c_int, vp, vp, vp, vp, C.POINTER(SolverOpts), vp, vp, vp, vp, vp, vp], C.c_int),
        "mf_problem_timing": ([vp, C.c_int], C.c_int),
        "mf_problem_kernel_stats": ([vp, dp, C.POINTER(C.c_long)], C.c_int),
        "mf_problem_trace": ([vp, ip, ip, dp, C.c_int], C.c_int),
        "mf_kernel_name": ([C.c_int], cp),
        "mf_ik_batch": ([vp, C.c_int, dp, dp, dp, dp, C.c_int, C.c_int, C.c_double, C.c_double, C.c_double], C.c_int),
        "mf_ik_batch_dev": ([vp, C.c_int, vp, vp, vp, vp, C.c_int, C.c_int, C.c_double, C.c_double, C.c_double, vp],
                            C.c_int),
        "mf_gopts_init": ([C.POINTER(GOpts)], C.c_int),
        "mf_gproblem_create": ([vp, vp, C.POINTER(GSpec), C.POINTER(vp)], C.c_int),
        "mf_gproblem_free": ([vp], None),
        "mf_gproblem_dims": ([vp, ip], C.c_int),
        "mf_gsolve_batch": ([vp, C.c_int, dp, dp, dp, dp, C.POINTER(GOpts), dp, ip, ip, dp, dp, C.c_int], C.c_int),
        "mf_gsolve_batch_dev": ([vp, C.c_int, vp, vp, vp, vp, C.POINTER(GOpts), vp, vp, vp, vp, vp, vp], C.c_int),
        "mf_gsolve_stream_dev": ([vp, C.c_int, C.c_int, vp, vp, vp, vp, C.POINTER(GOpts), vp, vp, vp, vp, vp, vp],
                                 C.c_int),
        "mf_gnode_record": ([vp, dp, dp, dp, dp, dp, dp, C.c_int], C.c_int),
        "mf_gdebug_duals": ([vp, C.c_int, dp], C.c_int),
        "mf_gdebug_slacks": ([vp, C.c_int, dp], C.c_int),
        "mf_debug_bk_compare": ([dp, C.c_int, C.c_int, dp, dp, ip], C.c_int),
        "mf_gproblem_timing": ([vp, C.c_int], C.c_int),
        "mf_gproblem_kernel_stats": ([vp, dp, C.POINTER(C.c_long), C.POINTER(C.c_longlong)], C.c_int),
        "mf_gdebug_counters": ([vp, C.c_int, ip], C.c_int),
        "mf_gdebug_trace": ([dp], C.c_int),
        "mf_gdebug_trace_reset": ([], C.c_int),
        "mf_last_error": ([], cp),
    }
    for name, (argt, rest) in sig.items():
        fn = getattr(L, name)
        fn.argtypes = argt
        fn.restype = rest
    _lib = L
    return L


EXPORTED_SYMBOLS = [
    "mf_model_from_urdf", "mf_model_free", "mf_model_nq", "mf_model_export", "mf_frame_id", "mf_frame_export",
    "mf_id", "mf_fk", "mf_jac", "mf_id_dev", "mf_fk_dev", "mf_jac_dev", "mf_problem_create", "mf_problem_free",
    "mf_problem_wsize", "mf_node_eval", "mf_solve_batch", "mf_solve_batch_dev", "mf_solve_batch_ws",
    "mf_solve_batch_ws_dev", "mf_problem_timing",
    "mf_problem_kernel_stats", "mf_problem_trace", "mf_kernel_name", "mf_ik_batch", "mf_ik_batch_dev", "mf_last_error",
    "mf_gopts_init", "mf_gproblem_create", "mf_gproblem_free", "mf_gproblem_dims", "mf_gsolve_batch", "mf_gsolve_batch_dev",
    "mf_gsolve_stream_dev",
    "mf_gnode_record", "mf_gdebug_duals", "mf_gdebug_slacks", "mf_debug_bk_compare", "mf_gproblem_timing", "mf_gproblem_kernel_stats",
    "mf_gdebug_counters", "mf_gdebug_trace", "mf_gdebug_trace_reset",
]


def check(code: int) -> int:
    if code < 0:
        msg = lib().mf_last_error()
        raise MFError(code, msg.decode() if msg else "")
    return code


def dptr(a: np.ndarray):
    assert a.dtype == np.float64 and a.flags.c_contiguous
    return a.ctypes.data_as(C.POINTER(C.c_double))


def iptr(a: np.ndarray):
    assert a.dtype == np.int32 and a.flags.c_contiguous
    return a.ctypes.data_as(C.POINTER(C.c_int))


class Model:
    """Owning handle of an ``mf_model`` (URDF → kinematic tree, Pinocchio semantics)."""

    def __init__(self, urdf_xml: str):
        h = C.c_void_p()
        check(lib().mf_model_from_urdf(urdf_xml.encode(), C.byref(h)))
        self._h = h
        self.nq = lib().mf_model_nq(h)
        self.nv = self.nq

    @property
    def handle(self):
        return self._h

    def frame_id(self, name: str) -> int:
        return check(lib().mf_frame_id(self._h, name.encode()))

    def export(self) -> np.ndarray:
        need = check(lib().mf_model_export(self._h, None, 0))
        b = np.zeros(need)
        lib().mf_model_export(self._h, dptr(b), need)
        return b

    def frame_record(self, frame: int) -> np.ndarray:
        r = np.zeros(13)
        check(lib().mf_frame_export(self._h, frame, dptr(r)))
        return r

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and _lib is not None:
            _lib.mf_model_free(h)
            self._h = None
