"""Device vs oracle IPOPT-mode paths, iteration by iteration: the device's trace of horizon 0 (mf_gdebug_trace rows
of k_gpre: iteration, mode, mu, E_0, primal and dual infeasibility) against the oracle's verbose trace of the same solve
(oracle/mf_ocp.c, riccati = 2, hyper-dual node functions, or the product's with --fast).  Prints the first
iterations where they part.

    python tools/ipopt_trace_cmp.py device c3 0 > trace.npy   (GPU: writes the device rows)
    python tools/ipopt_trace_cmp.py compare c3 0 trace.npy [--fast]
"""
import os
import re
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from watchdog_scan import spec_of  # noqa: E402

KW = dict(init_zero=True, filter=True, bound_relax=1e-8, max_iter=3000, max_soc=4)


def x0_of(case, spec):
    return np.r_[spec["q0"], spec["T0"]] if case != "c2" else np.asarray(spec["q0"])


def device(case, i, out):
    import ctypes as C
    from mpc_fatigue_amd import _lib
    from mpc_fatigue_amd.gocp import GOCP
    spec = spec_of(case, i)
    g = GOCP(spec)
    L = _lib.lib()
    L.mf_gdebug_trace_reset()
    lr = np.asarray(spec["line_ref"])[None] if case == "c2" else None
    r = g.solve(x0=x0_of(case, spec)[None], line_ref=lr, verbose=2, **KW)
    buf = np.zeros(2 * 4096 * 16)
    L.mf_gdebug_trace(_lib.dptr(buf))
    np.save(out, buf.reshape(2, 4096, 16))
    print("device", int(r.status[0]), int(r.iters[0]), float(r.obj[0]), g.counters(0), file=sys.stderr)


def oracle_trace(case, i, fast):
    code = f"""
import sys
sys.path.insert(0, {ROOT!r}); sys.path.insert(0, {os.path.join(ROOT, 'tools')!r})
from watchdog_scan import spec_of
from oracle import generic as G
spec = spec_of({case!r}, {i})
kw = dict({KW!r}, riccati=2, verbose=1)
if {fast}:
    from oracle import cpu_fast as CF
    w, R = G.solve_batch([spec], nthreads=1, L=G.bind(CF.lib()), **kw, **CF.FastNodes(spec).opts_kw())
    r = R[0]
else:
    w, r = G.solve(spec, **kw)
print("oracle", r.status, r.iter, r.obj, file=sys.stderr)
"""
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=dict(os.environ, OMP_NUM_THREADS="1"))
    rows = []
    for line in p.stderr.splitlines():
        m = re.match(r"(r?)it\s+(\d+) f (\S+) dinf (\S+) pinf (\S+) compl (\S+) mu (\S+)", line)
        if m:
            rows.append((m.group(1) == "r", int(m.group(2)), float(m.group(4)), float(m.group(5)), float(m.group(7))))
        elif line.startswith("oracle"):
            print(line)
    return rows


if __name__ == "__main__":
    what, case, i = sys.argv[1], sys.argv[2], int(sys.argv[3])
    if what == "device":
        device(case, i, sys.argv[4])
    else:
        dev = np.load(sys.argv[4])[0]
        orc = oracle_trace(case, i, "--fast" in sys.argv)
        shown = 0
        for resto, it, dinf, pinf, mu in orc:
            d = dev[it]
            if d[0] != it:
                continue
            dm, dmu, dpinf, ddinf = int(d[1]), d[2], d[4], d[5]
            rel = max(abs(dpinf - pinf) / max(pinf, 1e-300), abs(ddinf - dinf) / max(dinf, 1e-300))
            if dm != int(resto) and not resto:
                continue  # a restoration phase starts within this iteration: its first row took the number
            flag = (dm != int(resto)) or rel > 2e-2 or abs(dmu - mu) > 2e-2 * mu
            if flag or it < 3:
                print(f"it {it:4d} oracle {'r' if resto else ' '} mu {mu:.1e} pinf {pinf:.3e} dinf {dinf:.3e} | device mode {dm} "
                      f"mu {dmu:.1e} pinf {dpinf:.3e} dinf {ddinf:.3e}  rel {rel:.1e}")
                shown += flag
                if shown >= 12:
                    break
