"""AddressSanitizer + UndefinedBehaviorSanitizer runs of the host code:

* the C checker (oracle/mf_oracle.c, oracle/mf_ocp.c) built with gcc -fsanitize=address,undefined
  (``make -C oracle asan``) and exercised by the oracle's own tests in a child Python process with
  gcc's libasan preloaded;
* the product's host-compiled code -- the URDF parser (csrc/urdf.cpp), the forward-over-reverse node
  derivatives (csrc/adj.hpp) and the generic family record functions (csrc/gfam.hpp) -- built with
  hipcc, the sanitizer flags on the host side only (-Xarch_host), exercised by tests/test_adjoint_cpu.py
  and tests/test_gfam_cpu.py in a child process with clang's ASan runtime preloaded.

Any report aborts the child (halt_on_error, -fno-sanitize-recover), failing the test.  GPU code is not
sanitized (device ASan is not available on the MI355X pool).
"""
import glob
import os
import subprocess
import sys

import pytest

from tests.conftest import ROOT

SAN_ENV = {"ASAN_OPTIONS": "detect_leaks=0:halt_on_error=1:abort_on_error=0",
           "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1", "OMP_NUM_THREADS": "2"}
NATIVE = os.path.join(ROOT, "tests", "native")
CSRC = os.path.join(ROOT, "mpc_fatigue_amd", "csrc")


def _child(args, env_extra, timeout=900):
    env = dict(os.environ, **SAN_ENV, **env_extra)
    r = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider", *args], cwd=ROOT,
                       env=env, capture_output=True, text=True, timeout=timeout)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "ERROR: AddressSanitizer" not in out and "runtime error:" not in out, out[-4000:]
    return out


def test_oracle_c_asan_ubsan():
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "asan"], stdout=subprocess.DEVNULL)
    libasan = subprocess.check_output(["gcc", "-print-file-name=libasan.so"], text=True).strip()
    assert os.path.exists(libasan)
    # the IPOPT-mode code (filter, watchdog, soft restoration, IPOPT's restoration phase with elastic dynamics rows,
    # the Riccati recursion through them and the banded factorisation of the same system) runs under the sanitizers
    # through the C2 restoration check (test_oracle_resto_riccati, riccati = 3); the box cold solves repeat the same
    # code at 400-550 iterations and would take the child past its time limit at ASan speed
    _child(["tests/test_oracle_golden.py", "tests/test_oracle_generic.py", "tests/test_oracle_resto_riccati.py", "-k",
            "not resolve_matches_reference_trajectory and not ipopt_mode and not hard_dynamics"],
           {"LD_PRELOAD": libasan, "MF_ORACLE_LIB": os.path.join(ROOT, "oracle", "_asan", "libmforacle.so")})


def _clang_asan_rt():
    c = sorted(glob.glob("/opt/rocm/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so"))
    if not c:
        pytest.skip("clang ASan runtime not found")
    return c[-1]


def _hipcc_san(src, out):
    deps = src + [os.path.join(CSRC, h) for h in ("gfam.hpp", "adj.hpp", "dyn.hpp", "model.hpp")]
    if os.path.exists(out) and os.path.getmtime(out) >= max(os.path.getmtime(d) for d in deps):
        return
    os.makedirs(os.path.dirname(out), exist_ok=True)
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    san = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
           "-Xarch_host", "-fno-sanitize-recover=undefined", "-Xarch_host", "-fno-omit-frame-pointer"]
    subprocess.check_call([hipcc, "-O1", "-g", "-std=c++17", "-fPIC", "-shared", "--offload-arch=gfx950", *san,
                           "-x", "hip", src[0], "-x", "hip", src[1], "-o", out])


def test_host_product_code_asan_ubsan():
    rt = _clang_asan_rt()
    urdf = os.path.join(CSRC, "urdf.cpp")
    fam = os.path.join(NATIVE, "_asan", "libfamcheck.so")
    adj = os.path.join(NATIVE, "_asan", "libadjcheck.so")
    _hipcc_san([os.path.join(NATIVE, "famcheck.cpp"), urdf], fam)
    _hipcc_san([os.path.join(NATIVE, "adjcheck.cpp"), urdf], adj)
    _child(["tests/test_gfam_cpu.py", "tests/test_adjoint_cpu.py"],
           {"LD_PRELOAD": rt, "MF_FAMCHECK_LIB": fam, "MF_ADJCHECK_LIB": adj})
