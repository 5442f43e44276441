"""Generates tests/golden/ipopt_mode_C3_wd13.csv (+ .json): start 13 of the C3 shared-budget bench draw
(tools/generic_bench.py: the G1 start + U(-0.01, 0.01), default_rng(0)) solved in IPOPT mode by the oracle's IPM
(oracle/mf_ocp.c, the device's Riccati elimination, IPOPT's restoration) with the product's node functions built for
the host (oracle/libmfcpu.so).  Its path contains a backtracking search after StopWatchDog that fails
(tools/watchdog_scan.py; the oracle then re-evaluates the stored point before the soft restoration -- the device's
GP_WDSOFT round).  The json holds the oracle's iteration count, objective and the number of such failed searches.

Run:  python tests/golden/make_watchdog_fixture.py   (about a minute)
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

from watchdog_scan import spec_of  # noqa: E402

if __name__ == "__main__":
    from oracle import cpu_fast as CF
    from oracle import generic as G
    spec = spec_of("c3", 13)
    fk = CF.FastNodes(spec)
    L = G.bind(CF.lib())
    L.mfg_wdfail_count.argtypes = [G.C.c_int]
    L.mfg_wdfail_count(1)
    w, R = G.solve_batch([spec], nthreads=1, L=L, init_zero=True, filter=True, bound_relax=1e-8, max_iter=3000,
                         max_soc=4, riccati=2, **fk.opts_kw())
    r = R[0]
    assert r.status == 0, (r.status, r.iter)
    np.savetxt(os.path.join(HERE, "ipopt_mode_C3_wd13.csv"), w[0][None], delimiter=",", fmt="%.17g")
    meta = {"iter": r.iter, "obj": r.obj, "wd_failed_searches": L.mfg_wdfail_count(1)}
    json.dump(meta, open(os.path.join(HERE, "ipopt_mode_C3_wd13.json"), "w"), indent=1)
    print(meta)
