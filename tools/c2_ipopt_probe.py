"""C2 solved as the reference solves it (IPOPT mode from x0 = 0, force_optimization_pilz_6DOF.py:195-197) on the
first B horizons of the C5 batch: time, status counts, iteration distribution, per-horizon solver counters and the
running-count trajectory (verbose host log with timestamps on stderr).

    python tools/c2_ipopt_probe.py [B] [--max-iter 3000] [--reps 1] [--counters] [--timing] [--cstamps]

--cstamps runs the diagnostic build libmpcfatigue_cstamps.so (make -C mpc_fatigue_amd libmpcfatigue_cstamps.so) and
reports k_gkkt_chain's per-phase cycle counts over the timed solve.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("batch", type=int, nargs="?", default=8192)
    ap.add_argument("--max-iter", type=int, default=3000)
    ap.add_argument("--reps", type=int, default=1)
    ap.add_argument("--counters", action="store_true")
    ap.add_argument("--verbose", type=int, default=1)
    ap.add_argument("--timing", action="store_true", help="per-phase HIP-event timing of the (first) timed solve")
    ap.add_argument("--cstamps", action="store_true", help="k_gkkt_chain phase cycles (diagnostic build)")
    ap.add_argument("--no-spec", action="store_true", help="no concurrent inertia tries in the tail (inertia_spec -1)")
    a = ap.parse_args()
    if a.cstamps:
        os.environ["MF_LIB"] = "libmpcfatigue_cstamps.so"
    import torch
    torch.cuda.init()
    from mpc_fatigue_amd import pin, problems as PR
    from mpc_fatigue_amd.gocp import GOCP
    dev = torch.device("cuda", 0)
    B = a.batch
    sp = PR.pilz6_bench(N=100)
    Q = PR.pilz6_batch_q0(B, seed=0)
    lr = pin.generate_forward_kin(PR.read_urdf(sp["urdf"]), sp["frame"]).batch(Q)[0][:, :2]
    g = GOCP(sp)
    x = torch.as_tensor(Q, dtype=torch.float64, device=dev).contiguous()
    l = torch.as_tensor(np.ascontiguousarray(lr), dtype=torch.float64, device=dev).contiguous()
    out = {"w": torch.empty((B, g.wsize), dtype=torch.float64, device=dev),
           "status": torch.empty(B, dtype=torch.int32, device=dev), "iters": torch.empty(B, dtype=torch.int32, device=dev),
           "kkt": torch.empty(B, dtype=torch.float64, device=dev), "obj": torch.empty(B, dtype=torch.float64, device=dev)}
    ptr = {k: v.data_ptr() for k, v in out.items()}
    kw = dict(init_zero=True, filter=True, bound_relax=1e-8, max_iter=a.max_iter, max_soc=4)
    if a.no_spec:
        kw["inertia_spec"] = -1
    s = torch.cuda.current_stream(dev).cuda_stream
    g.solve_dev(x.data_ptr(), None, None, l.data_ptr(), B, ptr, stream=s, **dict(kw, max_iter=1))
    torch.cuda.synchronize()
    ts = []
    if a.timing:
        g.timing(True)
    if a.cstamps:
        import ctypes
        from mpc_fatigue_amd import _lib
        L = _lib.lib()
        assert L.mf_debug_cstamps_reset() == 0
    for r in range(a.reps):
        t0 = time.perf_counter()
        g.solve_dev(x.data_ptr(), None, None, l.data_ptr(), B, ptr, stream=s, verbose=a.verbose if r == 0 else 0, **kw)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    st = out["status"].cpu().numpy()
    it = out["iters"].cpu().numpy()
    sv, sc = np.unique(st, return_counts=True)
    rec = {"batch": B, "seconds": ts, "horizons_per_s": float((st == 0).sum() / np.median(ts)),
           "status_counts": {int(k): int(v) for k, v in zip(sv, sc)},
           "iters_mean": float(it.mean()), "iters_pct": {p: float(np.percentile(it, p)) for p in (50, 90, 99, 99.9, 100)}}
    if a.timing:
        rec["kernel_ms"] = {k: round(v[0], 1) for k, v in g.kernel_stats().items()}
        rec["node_evals"] = g.node_evals()
        g.timing(False)
    if a.cstamps:
        cs = (ctypes.c_ulonglong * 16)()
        assert L.mf_debug_cstamps(cs) == 0
        cs = list(cs)
        names = ["setup", "stage_loads", "slack_w_tv", "block_rows_vec", "bk_factor", "stores_solve", "p_update",
                 "forward", "slack_mult"]
        tot = sum(cs[:9]) + cs[12]
        rec["cstamps"] = {"cycles_share": {n: round(cs[i] / max(1, tot), 4) for i, n in enumerate(names)},
                          "sweeps": cs[9], "stages": cs[10], "launches": cs[11],
                          "cycles_per_stage": {n: round(cs[i] / max(1, cs[10]), 1) for i, n in enumerate(names[1:7], 1)},
                          "cycles_per_launch": round(tot / max(1, cs[11]), 1),
                          "pivoted_factor": {"cycles_share": round(cs[12] / max(1, tot), 4), "count": cs[13]},
                          "sweeps_wrong_inertia": cs[14], "sweeps_singular": cs[15]}
    if a.counters:
        C = np.array([list(g.counters(b).values()) for b in range(B)])
        rec["counters_mean"] = dict(zip(GOCP.COUNTERS, (float(v) for v in C.mean(0))))
        rec["resto_iter_share"] = float(C[:, 9].sum() / max(1, C[:, 0].sum()))
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
