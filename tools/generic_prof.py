"""Per-iteration probe of the generic device solver (csrc/gipm.hip) for rocprofv3: C3 shared budget N=100
(first homotopy stage, pos_toll = 1) and C4 Centauro N=50, `batch` perturbed starts, a fixed iteration cap so
that every horizon runs the same number of iterations (k_geval + k_giter per iteration).

    python tools/generic_prof.py [--batch 1024] [--iters 12] [--cases c3,c4] [--full]

--full: also the whole first homotopy stage (max_iter 1000) with the status / iteration histogram.
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=12)
    ap.add_argument("--cases", default="c3,c4")
    ap.add_argument("--full", action="store_true")
    a = ap.parse_args()
    import torch

    from mpc_fatigue_amd import problems as PR
    from mpc_fatigue_amd.gocp import GOCP
    from tools.generic_bench import _golden_q0

    torch.cuda.init()
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    rng = np.random.default_rng(0)
    B = a.batch
    cases = []
    if "c3" in a.cases:
        q0b = _golden_q0()
        sp = PR.box_shared_fatigue(N=100, q0=q0b)
        X = np.hstack([q0b[None] + rng.uniform(-0.01, 0.01, (B, 12)), np.tile(sp["T0"], (B, 1))])
        cases.append(("c3_shared_stage0", dict(sp, pos_toll=1.0), X, dict(u_init=PR.box_u_init(sp), max_soc=4)))
    if "c4" in a.cases:
        sp = PR.centauro(N=50, T=2.0)
        q0c = np.asarray(sp["q0"])
        X = np.hstack([q0c[None] + rng.uniform(-0.02, 0.02, (B, 14)), np.tile(sp["T0"], (B, 1))])
        cases.append(("c4_centauro_n50", sp, X, dict(u_init=PR.centauro_u_init(sp), max_soc=4)))
    for name, spec, X, kw in cases:
        g = GOCP(spec)
        x = torch.as_tensor(X, dtype=torch.float64, device=dev).contiguous()
        ob = {"w": torch.empty((B, g.wsize), dtype=torch.float64, device=dev),
              "status": torch.empty(B, dtype=torch.int32, device=dev),
              "iters": torch.empty(B, dtype=torch.int32, device=dev),
              "kkt": torch.empty(B, dtype=torch.float64, device=dev),
              "obj": torch.empty(B, dtype=torch.float64, device=dev)}
        ptr = {k: v.data_ptr() for k, v in ob.items()}
        runs = [("warm-up", 1), (f"{a.iters} iterations", a.iters)] + ([("full", 1000)] if a.full else [])
        for label, mi in runs:
            torch.cuda.synchronize(dev)
            t = time.perf_counter()
            g.solve_dev(x.data_ptr(), None, None, None, B, ptr, stream=stream.cuda_stream, max_iter=mi, **kw)
            torch.cuda.synchronize(dev)
            dt = time.perf_counter() - t
            st = ob["status"].cpu().numpy()
            it = ob["iters"].cpu().numpy()
            hist = {int(s): int((st == s).sum()) for s in np.unique(st)}
            pct = np.percentile(it, [50, 90, 99, 100]).tolist()
            print(f"[generic_prof] {name} {label}: {dt:.3f} s, {dt / max(1, it.max()) * 1e3:.2f} ms per iteration "
                  f"(max), status {hist}, iterations p50/p90/p99/max {pct}", flush=True)


if __name__ == "__main__":
    main()
