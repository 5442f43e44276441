"""Throughput of the generic device solver (csrc/gipm.hip) on BASELINE configs 3 and 4, batched over
perturbed initial states (bench.py imports generic_extra for its `generic` keys; run alone for a probe):

    python tools/generic_bench.py [--batch 1024] [--sample 2]

C3-shared: problems.box_shared_fatigue(N=100) from the reference's IK start q0 (tests/golden G1) with
  q0_i = q0 + U(-0.01, 0.01) per joint.
C4: problems.centauro(N=50, T=2) (the committed Centauro fixture's horizon, Centauro_dynamics.py:90-91)
  from the IK start with q0_i = q0 + U(-0.02, 0.02).
mode "ipopt" (default): one solve per horizon as the reference makes it -- IPOPT from x0 = 0 (Box_Pilz_6DOF.py:
  455-456 and the first solve of RepeatedMPCwithThermal.py:464-466 pass no x0), with IPOPT's globalisation
  (mf_gopts.filter: filter line search, watchdog, soft restoration, restoration phase) and bound_relax_factor 1e-8.
mode "merit": round 3's figure -- the l1-merit search, C3 through the pos_toll homotopy 1 -> 1e-2 -> 1e-4 from
  F = (0, 0, m g / 2), C4 from the reference's sol0 controls.
A horizon counts when its last stage converged (E_0 <= 1e-8).  GPU-vs-CPU: the first `sample` horizons
solved by the host IPM (oracle/libmfcpu.so, the same algorithm) and compared on the state trajectories.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


# iteration caps of the C3 homotopy stages in the bench figure (pos_toll 1, 1e-2, 1e-4): the intermediate stages only
# carry the iterate along the homotopy (their end points warm-start the next stage); the last stage is the reference
# problem with the full 1000-iteration cap
GENERIC_STAGE_CAPS = [150, 300, 1000]


def _golden_q0():
    g = np.loadtxt(os.path.join(ROOT, "tests", "golden", "G1_box_N50_solution.csv"), delimiter=",")
    return g[:12]


def _x_traj(w, nx, nu, N):
    w = np.atleast_2d(w)
    return np.concatenate([w[:, None, :nx], w[:, nx:].reshape(w.shape[0], N, nu + nx)[:, :, nu:]], axis=1)


# IPOPT at the reference's settings: no option is set in Box_Pilz_6DOF.py:455 / RepeatedMPCwithThermal.py:466, so
# max_iter is IPOPT's default 3000 (the filter path of a few starts is long: r04, 2 of 512 C3 starts need more than
# 1500 iterations on the device, 5 others on the host IPM -- round-off-sensitive restoration exits)
IPOPT_KW = dict(init_zero=True, filter=True, bound_relax=1e-8, max_iter=3000, max_soc=4)


def generic_extra(batch: int = 1024, sample: int = 2, cpu: bool = True, seed: int = 0, cases=("c3", "c4"),
                  stage_caps=None, batch_c4: int | None = None, mode: str = "ipopt", slots: int = 0,
                  max_iter: int = 0) -> dict:
    """slots > 0 (single-stage IPOPT mode): continuous batching -- `slots` concurrent solves work through the
    `batch` starts (mf_gsolve_stream_dev), so the few long solves no longer hold the device at one-horizon latency."""
    """stage_caps: iteration caps of the C3 homotopy stages (merit mode; default: 1000 each, GOCP.solve_box's)."""
    import torch

    from mpc_fatigue_amd import problems as PR
    from mpc_fatigue_amd.gocp import GOCP

    dev = torch.device("cuda", torch.cuda.current_device())
    stream = torch.cuda.current_stream(dev)
    rng = np.random.default_rng(seed)
    cap = {"max_iter": max_iter} if max_iter else {}
    out = {}
    todo = cases
    cases = []
    q0b = _golden_q0()
    sp3 = PR.box_shared_fatigue(N=100, q0=q0b)
    X3 = np.hstack([q0b[None] + rng.uniform(-0.01, 0.01, (batch, 12)), np.tile(sp3["T0"], (batch, 1))])
    if mode == "ipopt":
        cases.append(("c3_shared_budget_n100", sp3, X3, [sp3], dict(IPOPT_KW, **cap)))
    else:
        cases.append(("c3_shared_budget_n100", sp3, X3, [dict(sp3, pos_toll=t) for t in PR.box_homotopy_tolerances()],
                      dict(u_init=PR.box_u_init(sp3), max_iter=1000, max_soc=4)))
    sp4 = PR.centauro(N=50, T=2.0)
    q0c = np.asarray(sp4["q0"])
    b4 = batch_c4 or batch
    X4 = np.hstack([q0c[None] + rng.uniform(-0.02, 0.02, (b4, 14)), np.tile(sp4["T0"], (b4, 1))])
    if mode == "ipopt":
        cases.append(("c4_centauro_n50", sp4, X4, [sp4], dict(IPOPT_KW, **cap)))
    else:
        cases.append(("c4_centauro_n50", sp4, X4, [sp4], dict(u_init=PR.centauro_u_init(sp4), max_iter=500, max_soc=4)))
    lrefs = {}
    if "c2" in todo:  # C2 as the reference solves it (IPOPT from x0 = 0) on the C5 batch's horizons
        from mpc_fatigue_amd import pin
        sp2 = PR.pilz6_bench(N=100)
        Q2 = PR.pilz6_batch_q0(batch, seed=0)
        lrefs["c2_pilz6_n100_ipopt"] = pin.generate_forward_kin(PR.read_urdf(sp2["urdf"]), sp2["frame"]).batch(Q2)[0][:, :2]
        cases.append(("c2_pilz6_n100_ipopt", sp2, Q2, [sp2], dict(IPOPT_KW, **cap)))
    cases = [c for c in cases if c[0][:2] in todo]
    for name, spec, X, stages, kw in cases:
        batch = X.shape[0]
        caps = list(stage_caps) if (stage_caps and len(stages) > 1) else [kw["max_iter"]] * len(stages)
        gs = [GOCP(st) for st in stages]
        nx, nu, N = gs[0].nx, gs[0].nu, spec["N"]
        x = torch.as_tensor(X, dtype=torch.float64, device=dev).contiguous()
        lr = (torch.as_tensor(np.ascontiguousarray(lrefs[name]), dtype=torch.float64, device=dev)
              if name in lrefs else None)
        lrp = None if lr is None else lr.data_ptr()
        bufs = [{"w": torch.empty((batch, gs[0].wsize), dtype=torch.float64, device=dev),
                 "status": torch.empty(batch, dtype=torch.int32, device=dev),
                 "iters": torch.empty(batch, dtype=torch.int32, device=dev),
                 "kkt": torch.empty(batch, dtype=torch.float64, device=dev),
                 "obj": torch.empty(batch, dtype=torch.float64, device=dev)} for _ in stages]

        def run(label, max_iter=None):
            import threading
            done = threading.Event()

            def heartbeat():  # a long batch solve prints nothing for minutes (gpurun's silence guard)
                t_hb = time.perf_counter()
                while not done.wait(30.0):
                    print(f"[generic_bench] {name} {label}: running {time.perf_counter() - t_hb:.0f}s", file=sys.stderr,
                          flush=True)
            threading.Thread(target=heartbeat, daemon=True).start()
            try:
                _run(label, max_iter)
            finally:
                done.set()

        def _run(label, max_iter=None):
            prev = None
            for i, (g, ob) in enumerate(zip(gs, bufs)):
                ptr = {k: v.data_ptr() for k, v in ob.items()}
                kw2 = dict(kw, max_iter=caps[i] if max_iter is None else max_iter)
                t = time.perf_counter()
                if slots and len(gs) == 1 and slots < batch:
                    g.solve_stream_dev(x.data_ptr(), None, None, lrp, batch, slots, ptr, stream=stream.cuda_stream,
                                       **kw2)
                else:
                    g.solve_dev(x.data_ptr(), None, None if prev is None else prev.data_ptr(), lrp, batch, ptr,
                                stream=stream.cuda_stream, **kw2)
                torch.cuda.synchronize(dev)
                print(f"[generic_bench] {name} {label} stage {i}: {time.perf_counter() - t:.2f}s "
                      f"converged {int((ob['status'] == 0).sum().item())}/{batch}", file=sys.stderr, flush=True)
                prev = ob["w"]

        run("warm-up", max_iter=1)  # workspaces allocated, code loaded
        t0 = time.perf_counter()
        run("timed")
        dt = time.perf_counter() - t0
        st = bufs[-1]["status"].cpu().numpy()
        its = [int(b["iters"].sum().item()) for b in bufs]
        conv = int((st == 0).sum())
        sv, sc = np.unique(st, return_counts=True)
        rec = {"mode": mode, "value": conv / dt, "unit": "horizons/s", "batch": batch, "converged": conv,
               "status_counts": {int(a): int(c) for a, c in zip(sv, sc)},
               "slots": (slots if (slots and len(stages) == 1 and slots < batch) else batch),
               "converged_frac": conv / batch, "seconds": dt, "stages": len(stages),
               "mean_iters_per_stage": [i / batch for i in its], "stage_max_iter": caps,
               "N": N, "nx": nx, "nu": nu, "ni": gs[0].ni}
        if cpu and sample > 0:
            from oracle import cpu_fast as CF
            from oracle import generic as G
            fk = CF.FastNodes(spec)
            w = None
            t1 = time.perf_counter()
            # the same stages and caps on one host thread per horizon, with the GPU's KKT algorithm (the Riccati
            # recursion, mfg_opts.riccati) and the product's node functions built for the host
            for st_spec, cap in zip(stages, caps):
                if name in lrefs:  # chain family: the start and its own line reference
                    specs = [dict(st_spec, q0=list(X[i]), line_ref=list(lrefs[name][i])) for i in range(sample)]
                else:
                    specs = [dict(st_spec, q0=list(X[i, :len(spec["q0"])]), T0=list(X[i, len(spec["q0"]):]))
                             for i in range(sample)]
                kwc = dict(kw, max_iter=cap, riccati=True, **fk.opts_kw())
                if kw.get("filter"):
                    kwc["riccati"] = 2  # the device's elimination in IPOPT's restoration phase too (ric_relax)
                res = [G.solve_batch([sp_], nthreads=1, L=CF.lib(), w0=(None if w is None else w[i]), **kwc)
                       for i, sp_ in enumerate(specs)]
                w = np.vstack([r[0] for r in res])
                R = [r[1][0] for r in res]
            tc = time.perf_counter() - t1
            wg = bufs[-1]["w"][:sample].cpu().numpy()
            both = np.array([r.status == 0 for r in R]) & (st[:sample] == 0)
            rec["gpu_vs_cpu"] = {"horizons": sample, "both_converged": int(both.sum()),
                                 "max_dx": (float(np.abs(_x_traj(wg[both], nx, nu, N) - _x_traj(w[both], nx, nu, N)).max())
                                            if both.any() else None),
                                 "cpu_seconds": tc, "cpu_one_thread_horizons_per_s": sample / tc,
                                 "cpu_note": "the same stages on one host thread per horizon (Riccati KKT, -O3 host "
                                             "build of the product's node functions, oracle/libmfcpu.so)"}
        out[name] = rec
        print(f"[generic_bench] {name}: {json.dumps(rec)}", file=sys.stderr, flush=True)
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--cases", default="c3,c4", help="comma list of c3 (shared budget N=100) and c4 (Centauro N=50)")
    ap.add_argument("--sample", type=int, default=2)
    ap.add_argument("--caps", default="", help="comma list of C3 homotopy stage iteration caps (default 1000 each)")
    ap.add_argument("--mode", default="ipopt", choices=["ipopt", "merit"])
    ap.add_argument("--slots", type=int, default=0, help="continuous batching: concurrent solves (0: the whole batch)")
    ap.add_argument("--max-iter", type=int, default=0, help="iteration cap (0: IPOPT's default 3000)")
    ap.add_argument("--no-spec", action="store_true", help="sequential inertia tries only (mf_gopts.inertia_spec = -1)")
    a = ap.parse_args()
    import torch
    torch.cuda.init()
    caps = [int(c) for c in a.caps.split(",")] if a.caps else None
    if a.no_spec:
        IPOPT_KW["inertia_spec"] = -1
    print(json.dumps(generic_extra(a.batch, a.sample, cases=tuple(a.cases.split(",")), stage_caps=caps, mode=a.mode,
                                   max_iter=a.max_iter,
                                   slots=a.slots)))
