"""Forward-over-reverse node derivatives (csrc/adj.hpp) vs the oracle, on the CPU.

The GPU eval kernel runs the template ``node_fwd_rev<Dual, n>`` with one tangent
direction per lane.  tests/native/adjcheck.cpp instantiates the same template
for the host, so its tau, d tau/dw, frame point, d p/dq and the exact Hessian
of phi = c.tau + yl.p can be checked here against the oracle's hyper-dual
restatement (oracle/mf_oracle.c mfo_node_derivs) without a GPU.
"""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

from mpc_fatigue_amd import problems as PR
from oracle import oracle as O
from oracle.urdf_np import load_urdf_file
from tests.conftest import ROOT

NATIVE = os.path.join(ROOT, "tests", "native")
LIB = os.environ.get("MF_ADJCHECK_LIB") or os.path.join(NATIVE, "libadjcheck.so")  # sanitizer build: tests/test_sanitizers.py


def _build():
    if os.environ.get("MF_ADJCHECK_LIB"):
        return
    src = [os.path.join(NATIVE, "adjcheck.cpp"), os.path.join(ROOT, "mpc_fatigue_amd", "csrc", "urdf.cpp")]
    deps = src + [os.path.join(ROOT, "mpc_fatigue_amd", "csrc", h) for h in ("adj.hpp", "dyn.hpp", "model.hpp")]
    if os.path.exists(LIB) and os.path.getmtime(LIB) >= max(os.path.getmtime(d) for d in deps):
        return
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    subprocess.check_call([hipcc, "-O2", "-std=c++17", "-fPIC", "-shared", "--offload-arch=gfx950",
                           "-x", "hip", src[0], "-x", "hip", src[1], "-o", LIB])


@pytest.fixture(scope="module")
def adj():
    _build()
    L = C.CDLL(LIB)
    L.adj_node.restype = C.c_int
    return L


def _p(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


CASES = [("pilz_robot_6DOF.urdf", "prbt_link_5", 1), ("pilz_robot_6DOF.urdf", "prbt_link_5", 0),
         ("pilz_robot_3DOF.urdf", "prbt_link_5", 0), ("pilz_robot_6DOF_first.urdf", "end_effector", 3),
         ("pilz_robot_6DOF_second.urdf", "end_effector", 2)]


@pytest.mark.parametrize("split", [0, 1])
@pytest.mark.parametrize("urdf,frame,nf", CASES)
def test_fwd_rev_matches_hyperdual_oracle(adj, urdf, frame, nf, split):
    """split = 1: the q directions run node_fwd_rev_split (plain FP64 below joint v, k_eval_node's q class)."""
    adj.adj_set_split(split)
    xml = open(PR.urdf_path(urdf)).read()
    m = load_urdf_file(PR.urdf_path(urdf))
    n = m.nq
    nv = 2 * n + nf
    rng = np.random.default_rng(11)
    fdir = rng.normal(size=(3, 3))
    fdir /= np.linalg.norm(fdir, axis=1, keepdims=True)
    spec = dict(PR.pilz6_force(N=4) if n == 6 else PR.pilz3_working(N=4))
    spec.update(frame=frame, nf=nf, fdir=fdir[:nf].tolist(), use_line=True)
    for _ in range(4):
        q, qd = rng.uniform(-2.5, 2.5, (2, n))
        F = rng.uniform(-80, 80, max(nf, 1))
        cw, yl = rng.normal(size=n), rng.normal(size=2)
        tau, Jt, pf, Jp, H = O.node_derivs(m, spec, q, qd, F, cw, yl)
        out = [np.zeros(n), np.zeros(n * nv), np.zeros(3), np.zeros(3 * n), np.zeros(nv * nv)]
        fd = np.ascontiguousarray(fdir.reshape(-1))
        rc = adj.adj_node(xml.encode(), frame.encode(), nf, _p(fd), 2, _p(q), _p(qd), _p(np.ascontiguousarray(F)),
                          _p(cw), _p(yl), *[_p(a) for a in out])
        assert rc == 0
        scale = max(1.0, np.abs(H).max())
        np.testing.assert_allclose(out[0], tau, rtol=0, atol=1e-12)
        np.testing.assert_allclose(out[1].reshape(n, nv), Jt, rtol=0, atol=1e-12)
        np.testing.assert_allclose(out[2], pf, rtol=0, atol=1e-14)
        np.testing.assert_allclose(out[3].reshape(3, n), Jp, rtol=0, atol=1e-14)
        np.testing.assert_allclose(out[4].reshape(nv, nv), H, rtol=0, atol=1e-12 * scale)
