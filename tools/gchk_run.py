"""Diagnostic: run one generic solve on the check-instrumented library (libmpcfatigue_gchk.so, -DMF_GCHK) with its
progress checkpoints and stored-factorisation index checks mapped to host memory; the words are written to
gpurun_out/gchk_<case>.bin at the end of the solve, or by the library's SIGABRT handler if the runtime aborts on a
GPU fault.  `decode` prints the last checkpoint per problem (run on the CPU afterwards).

    python tools/gchk_run.py run chain_merit|box_merit|chain_filter
    python tools/gchk_run.py suite tests/test_gpu_generic.py   (the generic GPU tests on the check build; the
                                                               index-check violations of every solve are ORed)
    python tools/gchk_run.py decode gpurun_out/gchk_<case>.bin
"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(case):
    os.environ["MF_LIB"] = "libmpcfatigue_gchk.so"
    from mpc_fatigue_amd import _lib, problems as PR
    from mpc_fatigue_amd.gocp import GOCP
    L = _lib.lib()
    L.mf_gdebug_chk_attach.argtypes = [C.c_char_p]
    L.mf_gdebug_chk_dump.argtypes = []
    out = os.path.join(ROOT, "gpurun_out", f"gchk_{case}.bin")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    _lib.check(L.mf_gdebug_chk_attach(out.encode()))
    try:
        if case == "chain_merit":
            spec = PR.pilz6_bench(N=20)
            r = GOCP(spec).solve(F_init=PR.BENCH_F_INIT, max_soc=4)
        elif case == "chain_filter":
            spec = PR.pilz6_bench(N=20)
            r = GOCP(spec).solve(F_init=PR.BENCH_F_INIT, max_soc=4, filter=True, bound_relax=1e-8)
        elif case == "box_merit":
            g = np.loadtxt(os.path.join(ROOT, "tests", "golden", "G1_box_N50_solution.csv"), delimiter=",")
            spec = PR.box_dual(q0=g[:12], N=50)
            r, _ = GOCP(spec).solve_box()
        else:
            raise SystemExit(f"unknown case {case}")
    finally:
        L.mf_gdebug_chk_dump()  # (host memory: readable after a device fault)
        decode(out)
    print(case, "status", r.status.tolist(), "iters", r.iters.tolist(), flush=True)


def suite(target):
    """Run pytest on `target` in this process with the check build attached; after every solve the violation
    words are collected (the library clears them at each attach), and any violation fails the run."""
    os.environ["MF_LIB"] = "libmpcfatigue_gchk.so"
    import pytest
    import torch
    assert torch.cuda.is_available()  # (the runtime initialised by torch first, as in a plain pytest run)
    from mpc_fatigue_amd import _lib
    from mpc_fatigue_amd import gocp
    L = _lib.lib()
    L.mf_gdebug_chk_attach.argtypes = [C.c_char_p]
    out = os.path.join(ROOT, "gpurun_out", "gchk_suite.bin")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    _lib.check(L.mf_gdebug_chk_attach(out.encode()))
    seen = {"solves": 0, "violations": 0}
    orig = gocp.GOCP.solve

    def solve(self, *a, **kw):
        r = orig(self, *a, **kw)
        L.mf_gdebug_chk_dump()
        w = np.fromfile(out, dtype=np.uint32).reshape(-1, 68)
        bad = int((w[:, 1] != 0).sum())
        seen["solves"] += 1
        seen["violations"] += bad
        if bad:
            print(f"[gchk] {bad} problems with index violations", flush=True)
            decode(out)
        _lib.check(L.mf_gdebug_chk_attach(out.encode()))
        return r

    gocp.GOCP.solve = solve
    rc = pytest.main(["-x", "-q", "-m", "gpu", "-p", "no:cacheprovider", target])
    print(f"[gchk] {seen['solves']} solves checked, {seen['violations']} problems with violations", flush=True)
    raise SystemExit(rc if rc else (1 if seen["violations"] else 0))


def decode(path):
    w = np.fromfile(path, dtype=np.uint32).reshape(-1, 68)
    live = np.flatnonzero(w[:, 0] | w[:, 1])
    for b in live[:16]:
        c, bad, aux, val = (int(v) for v in w[b, :4])
        print(f"problem {b}: iter {c >> 12} phase {(c >> 8) & 15} checkpoint {c & 255} aux {aux} "
              f"violations {bad:#x} value {val}")
        ln = w[b, 4:]
        print("  lanes (node, step):", [(int(v) >> 8, int(v) & 255) for v in ln if v])
    print(f"{len(live)} problems recorded; violations on {int((w[:, 1] != 0).sum())}")


if __name__ == "__main__":
    {"run": run, "decode": decode, "suite": suite}[sys.argv[1]](sys.argv[2])
