"""Diagnostic (GPU): running-horizon count and wall time per 4-iteration chunk of one batched C2 solve
(bench instance), to measure the iteration tail (share of the solve spent with < 10 % running)."""
import os
import re
import subprocess
import sys

if len(sys.argv) > 1 and sys.argv[1] == "child":
    sys.path.insert(0, ".")
    import numpy as np
    import torch
    from mpc_fatigue_amd import _lib, problems as PR
    from mpc_fatigue_amd.ocp import OCP
    B = int(sys.argv[2])
    spec = PR.pilz6_bench(N=100)
    ocp = OCP(spec)
    from oracle import pin_np as P
    from oracle.urdf_np import load_urdf_file
    ref = load_urdf_file(PR.urdf_path(spec["urdf"]))
    Q0 = PR.pilz6_batch_q0(B, seed=0)
    LR = np.array([P.forward_kinematics(ref, q, "prbt_link_5")[0][:2] for q in Q0])
    ocp.solve(Q0, line_ref=LR, F_init=PR.BENCH_F_INIT, max_iter=300)  # warm-up
    r = ocp.solve(Q0, line_ref=LR, F_init=PR.BENCH_F_INIT, max_iter=300, verbose=True)
    print("iters mean", r.iters.mean(), "max", r.iters.max(), file=sys.stderr)
    sys.exit(0)

B = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
p = subprocess.run([sys.executable, __file__, "child", str(B)], capture_output=True, text=True)
rows = []
for line in p.stderr.splitlines():
    m = re.search(r"after (\d+) iterations: (\d+) running  t=([\d.]+)", line)
    if m:
        rows.append((int(m.group(1)), int(m.group(2)), float(m.group(3))))
    elif "iters" in line:
        print(line)
# the verbose solve is the second one: keep rows after the last reset of t
cut = max(i for i, r in enumerate(rows) if r[0] == 4)
rows = rows[cut:]
prev_t, prev_a = 0.0, B
tail = 0.0
for it, act, t in rows:
    dt = t - prev_t
    if prev_a < 0.1 * B:
        tail += dt
    print(f"it {it:4d} running {act:6d} chunk {dt:7.2f} ms  cum {t:8.1f} ms")
    prev_t, prev_a = t, act
print(f"total {prev_t:.1f} ms, spent with < 10% running: {tail:.1f} ms ({100 * tail / prev_t:.1f} %)")
