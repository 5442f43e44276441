"""Node records of the generic families (csrc/gfam.hpp) vs the oracle, on the CPU.

tests/native/famcheck.cpp instantiates, for the host, exactly the functions the device kernel
k_geval runs (pre-pass, seeds, one forward-over-reverse lane per tangent direction, record
entries), so the record -- values, cost gradient, constraint Jacobians, dynamics Jacobians and the
exact Lagrangian Hessian assembled from lane columns plus closed-form algebraic terms -- can be
compared with the oracle's hyper-dual restatement (oracle/mf_ocp.c mfg_node_derivs) without a GPU.
"""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

from mpc_fatigue_amd import problems as PR
from oracle import generic as G
from oracle.cpu_fast import GParams, gparams
from tests.conftest import ROOT

NATIVE = os.path.join(ROOT, "tests", "native")
LIB = os.environ.get("MF_FAMCHECK_LIB") or os.path.join(NATIVE, "libfamcheck.so")  # sanitizer build: tests/test_sanitizers.py
CSRC = os.path.join(ROOT, "mpc_fatigue_amd", "csrc")


def _build():
    if os.environ.get("MF_FAMCHECK_LIB"):
        return
    src = [os.path.join(NATIVE, "famcheck.cpp"), os.path.join(CSRC, "urdf.cpp")]
    deps = src + [os.path.join(CSRC, h) for h in ("gfam.hpp", "adj.hpp", "dyn.hpp", "model.hpp")]
    if os.path.exists(LIB) and os.path.getmtime(LIB) >= max(os.path.getmtime(d) for d in deps):
        return
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    subprocess.check_call([hipcc, "-O2", "-std=c++17", "-fPIC", "-shared", "--offload-arch=gfx950",
                           "-x", "hip", src[0], "-x", "hip", src[1], "-o", LIB])


@pytest.fixture(scope="module")
def fam():
    _build()
    L = C.CDLL(LIB)
    L.fam_node_record.restype = C.c_int
    assert L.fam_gparams_size() == C.sizeof(GParams)
    return L


def _p(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def compare(fam, family, spec, xu, nx, nu, ni, ne, seed=0, nm=0):
    rng = np.random.default_rng(seed)
    yi, ye, lam = rng.normal(size=ni) * 10, rng.normal(size=max(ne + nm, 1)), rng.normal(size=nx)
    urdfs = spec["urdf"] if isinstance(spec["urdf"], list) else [spec["urdf"], spec["urdf"]]
    x0 = open(PR.urdf_path(urdfs[0])).read().encode()
    x1 = open(PR.urdf_path(urdfs[1])).read().encode()
    nv = nx + nu
    rec = np.zeros(8192)
    lref = np.zeros(6)
    lref[:2] = spec.get("line_ref", [0.0, 0.0]) if family != 3 else [0.0, 0.0]
    g = gparams(spec)
    n = fam.fam_node_record(family, x0, x1, spec["frame"].encode(), C.byref(g), _p(np.ascontiguousarray(xu)),
                            _p(yi), _p(ye), _p(lam), _p(lref), _p(rec))
    assert n > 0
    vals, jac, H = G.node_derivs(spec, xu, yi, ye, lam)
    o = 0
    l = rec[o]; o += 1
    gl = rec[o:o + nv]; o += nv
    ci = rec[o:o + ni]; o += ni
    Ji = rec[o:o + ni * nv].reshape(ni, nv); o += ni * nv
    ce = rec[o:o + ne]; o += ne
    Je = rec[o:o + ne * nx].reshape(ne, nx); o += ne * nx
    cm = rec[o:o + nm]; o += nm
    Jm = rec[o:o + nm * nv].reshape(nm, nv); o += nm * nv
    f = rec[o:o + nx]; o += nx
    A = rec[o:o + nx * nx].reshape(nx, nx); o += nx * nx
    B = rec[o:o + nx * nu].reshape(nx, nu); o += nx * nu
    W = rec[o:o + nv * nv].reshape(nv, nv); o += nv * nv
    assert o == n
    sc = lambda a: max(1.0, np.abs(a).max(initial=0.0))
    ie, im, iF = 1 + ni, 1 + ni + ne, 1 + ni + ne + nm
    np.testing.assert_allclose(l, vals[0], rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(ci, vals[1:ie], atol=1e-11 * sc(ci))
    np.testing.assert_allclose(ce, vals[ie:im], atol=1e-12)
    np.testing.assert_allclose(cm, vals[im:iF], atol=1e-11 * sc(cm))
    np.testing.assert_allclose(f, vals[iF:], atol=1e-12 * sc(f))
    np.testing.assert_allclose(gl, jac[0], atol=1e-11 * sc(jac[0]))
    np.testing.assert_allclose(Ji, jac[1:ie], atol=1e-11 * sc(Ji))
    np.testing.assert_allclose(Je, jac[ie:im, :nx], atol=1e-12 * sc(Je))
    assert np.abs(jac[ie:im, nx:]).max(initial=0.0) == 0.0  # state rows: no u dependence
    np.testing.assert_allclose(Jm, jac[im:iF], atol=1e-11 * sc(Jm))
    np.testing.assert_allclose(A, jac[iF:, :nx], atol=1e-12 * sc(A))
    np.testing.assert_allclose(B, jac[iF:, nx:], atol=1e-12 * sc(B))
    np.testing.assert_allclose(W, H, atol=1e-10 * sc(H))
    np.testing.assert_allclose(W, W.T, atol=1e-11 * sc(W))


@pytest.mark.parametrize("k", [0, 17, 40])
def test_box_record_matches_oracle(fam, golden, k):
    g, _ = golden["G1_box_N50"]
    xu = g[k * 30:k * 30 + 30].copy()
    if k == 0:
        xu[12:24] = np.random.default_rng(2).uniform(-1, 0.5, 12)  # non-zero velocities
    compare(fam, 0, PR.box_dual(N=1), xu, 12, 18, 18, 1, seed=k)


@pytest.mark.parametrize("seed", [0, 1])
def test_chain_record_matches_oracle(fam, seed):
    rng = np.random.default_rng(seed)
    spec = dict(PR.pilz6_bench(N=1), wtau=0.3, wqd=2.0)
    xu = np.r_[rng.normal(size=6), 0.3 * rng.normal(size=6), [20.0]]
    compare(fam, 1, spec, xu, 6, 7, 6, 2, seed=seed)


@pytest.mark.parametrize("seed", [0, 1])
def test_thermal_record_matches_oracle(fam, seed):
    rng = np.random.default_rng(10 + seed)
    spec = dict(PR.pilz6_thermal(N=1), wtau=0.1)
    xu = np.r_[rng.normal(size=6), 60 + rng.normal(size=6), 0.3 * rng.normal(size=6), [40.0]]
    compare(fam, 2, spec, xu, 12, 7, 6, 2, seed=seed)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_centauro_record_matches_oracle(fam, seed):
    """C4 node (two 7-DOF substitute arms, thermal state, relative pose + equilibrium rows) vs the hyper-dual
    restatement: tau = ID + J^T F, the closed-form pose derivatives and the full Lagrangian Hessian."""
    rng = np.random.default_rng(20 + seed)
    spec = PR.centauro(N=1)
    q0 = np.asarray(spec["q0"])
    xu = np.r_[q0 + 0.2 * rng.normal(size=14), 20 + 30 * rng.uniform(size=14), 0.5 * rng.normal(size=14),
               rng.normal(size=3) * 5 + [0, 0, 49], rng.normal(size=3) * 5 + [0, 0, 49]]
    compare(fam, 3, spec, xu, 28, 20, 14, 6, seed=seed, nm=6)


@pytest.mark.parametrize("k", [0, 30])
def test_box_shared_fatigue_record_matches_oracle(fam, golden, k):
    """N2 node (dual-arm box + winding temperatures of the 12 joints + the shared budget row)."""
    g, _ = golden["G1_box_N50"]
    xu = np.r_[g[k * 30:k * 30 + 12], 60.0 + np.arange(12.0), g[k * 30 + 12:k * 30 + 30]]
    compare(fam, 4, PR.box_shared_fatigue(N=1), xu, 24, 18, 19, 1, seed=k)
