"""Benchmark: MPC horizons solved / s, Pilz-6DOF N=100, batched on MI355X.

A step = one complete solve, as the reference solves C2 (force_optimization_pilz_6DOF.py:195-197: nlpsol('ipopt')
at IPOPT's defaults, no x0), of this rank's shard of horizons: IPOPT from x0 = 0 with IPOPT's globalisation (filter
line search, watchdog, soft restoration, the restoration phase with elastic variables on every row), bound_relax_factor
1e-8 and max_iter 3000, on the device (csrc/gipm.hip, chain family) -- followed (N > 1) by the RCCL gather of every
shard's solutions to rank 0.  The batched configuration of BASELINE.json (C5: 8192 independent horizons, q0_i = q0_IK +
U(-0.05, 0.05) per joint, line reference = fk(q0_i)[0:2]); every GPU solves a C5-sized batch of 8192 horizons (weak
scaling; --batch 1024 gives C5's 8-GPU shard size, --c5 the 8192 in total).  value = horizons that reached IPOPT's
tolerance (E_0 <= 1e-8) on all ranks / max-over-ranks wall time (inputs resident in HBM).

    python bench.py [--gpus N --steps K --warmup W --batch B --nodes 100]
    python bench.py --c5 ...   (C5 as SURVEY.md s.8(e): --batch horizons in total, sharded; strong scaling)
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

Also reported: the node-evaluation phase's achieved rate against its HBM roofline (per-phase HIP-event timing,
SURVEY.md s.8(d)'s 952 algorithmic bytes per device-counted node evaluation), every phase's share, C5's 1024-horizon
shard, the single-problem latency, the specialised l1-merit solver of rounds 1-5 as a labelled non-reference figure
(merit_mode), BASELINE configs 3 and 4 (generic), and the CPU baseline = the same IPOPT-mode algorithm on the host
with the product's node functions compiled for the CPU, on all cores and on one core (rank 0, N = 1 only, bounded
sample), whose solutions are compared with the GPU's for the same horizons.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "MPC horizons solved/sec, Pilz 6DOF N=100 shooting nodes, 1 MI355X"
HBM_PEAK_GBS = 8000.0         # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
FP64_PEAK_TFS = 78.6          # MI355X FP64 vector peak (spec)


# algorithmic bytes of the C2 node evaluation, per shooting node.  Read q_k(6),
# qd_k(6), F_k(1) = 104 B; write x_next(6) + cost(1) + tau(6) + line(2) + d tau/d(q,qd,F) (78)
# + d line/dq (12) + d cost/dF (1) = 106 doubles = 848 B.
NODE_BYTES = 952


def cpu_threads() -> tuple[int, str]:
    """Threads for the all-cores CPU leg: the CPUs this process may run on (sched_getaffinity), capped by
    OMP_NUM_THREADS when the environment sets it (the GPU box allots 16 host CPUs per GPU and exports
    OMP_NUM_THREADS=16; os.cpu_count() there reports the whole host)."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and 0 < int(env) < aff:
        return int(env), f"OMP_NUM_THREADS={env} (the host share of this GPU); affinity allows {aff}, nproc {os.cpu_count()}"
    return aff, f"every CPU of the process affinity ({aff}; nproc {os.cpu_count()})"


def cpu_baseline(spec_of, Q0, lrefs, opts, threads: int, sample_mt: int, sample_1t: int, reps: int):
    """The CPU baseline (rank 0, N = 1): the same interior-point algorithm on the host -- the generic
    oracle IPM (oracle/mf_ocp.c) with the product's forward-over-reverse node functions compiled for
    the host (oracle/cpu_fast.cpp, -O3 AVX2/FMA) and the device's Riccati KKT recursion -- OpenMP over
    horizons on `threads` cores and on one core; median of `reps` timed runs after one warm-up run.  Also the phase split of the host solve
    (node derivatives / KKT factorisation / directions / line search, mfg_time_get).
    Returns (record, CPU solutions)."""
    import ctypes as C

    from oracle import cpu_fast as CF

    specs = [spec_of(Q0[i], lrefs[i]) for i in range(max(sample_mt, sample_1t))]
    kw = dict(opts, **CF.FastNodes(specs[0]).opts_kw())
    kw.setdefault("riccati", True)
    L = C.CDLL(CF.LIB)
    L.mfg_time_get.argtypes = [C.POINTER(C.c_double)]

    def run(sp, nt):
        t0 = time.perf_counter()
        w, R = CF.solve_batch(sp, nthreads=nt, **kw)
        return time.perf_counter() - t0, w, R

    out = {}
    for label, S, nt in (("all_cores", sample_mt, threads), ("one_core", sample_1t, 1)):
        run(specs[:min(S, nt)], nt)  # warm-up
        ts = []
        L.mfg_time_reset()
        for _ in range(reps):
            dt, w, R = run(specs[:S], nt)
            ts.append(dt)
        conv = sum(1 for r in R if r.status == 0)
        out[label] = {"value": conv / float(np.median(ts)), "threads": nt, "horizons": S, "converged": conv,
                      "median_s": float(np.median(ts)), "runs_s": [round(t, 3) for t in ts]}
        if label == "one_core":
            a = (C.c_double * 5)()
            L.mfg_time_get(a)
            tot = max(a[4], 1e-12)
            split = {"node_derivatives": a[0] / tot, "kkt_factorisation": a[1] / tot, "kkt_directions": a[2] / tot,
                     "line_search": a[3] / tot, "other": (a[4] - a[0] - a[1] - a[2] - a[3]) / tot}
        if label == "all_cores":
            w_mt, st_mt, ob_mt = w, np.array([r.status for r in R]), np.array([r.obj for r in R])
    rec = {"value": out["all_cores"]["value"], "unit": "horizons/s", "cores": threads, "kind": "port",
           "single_core": out["one_core"]["value"], "nproc": os.cpu_count(), "detail": out,
           "time_split_one_core": split,
           "sample": (f"first {sample_mt} horizons of the same batch on {threads} threads and the first {sample_1t} "
                      f"on 1 thread (median of {reps} runs after a warm-up); generic IPM oracle/mf_ocp.c with the "
                      "product's node functions, both built for the host at -O3 -march=x86-64-v3 (oracle/libmfcpu.so); "
                      "the GPU's algorithm: IPOPT mode from x0 = 0 (filter, watchdog, restoration with elastic rows) "
                      "and the device's Riccati recursion (mfg_opts.riccati = 2, stage blocks factored by "
                      "Bunch-Kaufman), not the checker's block-tridiagonal factorisation")}
    return rec, w_mt, st_mt, ob_mt


def workload_plan(batch: int, c5: bool, world: int) -> tuple[int, str, str]:
    """(horizons over all ranks, scaling label, workload prefix): by default every GPU solves its own `batch`
    horizons (weak scaling); with --c5 `batch` is C5's total, sharded over the ranks."""
    gB = batch if c5 else batch * world
    return gB, ("strong" if c5 else "weak"), (f"C5: {gB} horizons in total over {world} GPU(s), " if c5 else "")


class StepLoop:
    """Steps in flight.  Consecutive steps are independent batched solves, each on its own slot (solver workspace,
    stream, host thread), so the iteration tail of one step overlaps the bulk of the next; every step still solves
    the whole shard.  solve(step, slot, nb, ev) runs one step on `slot` and returns when it is done, after waiting
    for `ev` (the event of that slot's last gather, or None); gather(step, slot) collects a finished step's
    solutions from the slot's buffers (N > 1: the RCCL gather to rank 0) and returns the event the slot's next solve
    waits for, so a slot's outputs are not overwritten before their gather has read them and no slot waits for
    another's work.  Steps finish, and are gathered, in order."""

    def __init__(self, inflight: int, solve, gather=None):
        self.inflight = max(1, inflight)
        self.solve, self.gather = solve, gather
        self.gathered = [None] * self.inflight

    def run(self, K: int, nb: int, gather: bool = True, first: int = 0) -> None:
        from concurrent.futures import ThreadPoolExecutor
        n = self.inflight
        with ThreadPoolExecutor(n) as ex:
            futs = []
            for s_ in range(K + n):
                if s_ >= n:  # step s_ - n done: its slot is free (gather its solutions)
                    futs[s_ - n].result()
                    if gather and self.gather is not None:
                        i = (s_ - n) % n
                        self.gathered[i] = self.gather(first + s_ - n, i)
                if s_ < K:
                    i = s_ % n
                    futs.append(ex.submit(self.solve, first + s_, i, nb, self.gathered[i]))


# C2 exactly as the reference solves it (force_optimization_pilz_6DOF.py:195-197: nlpsol('ipopt') at its defaults, no
# x0): IPOPT from x0 = 0 with IPOPT's globalisation -- filter line search, watchdog, soft restoration, the restoration
# phase with elastic variables on every row -- bound_relax_factor 1e-8, IPOPT's default max_iter 3000 (csrc/gipm.hip,
# the chain family)
IPOPT_MODE = dict(init_zero=True, filter=True, bound_relax=1e-8, max_soc=4, tol=1e-8, constr_viol_tol=1e-8,
                  mu_init=0.1)


def wq_traj(w: np.ndarray, n: int, nf: int, N: int) -> np.ndarray:
    """(B, N+1, n) joint trajectories of solution vectors in the reference layout [q_0 | (qd_k, F_k, q_{k+1})]."""
    w = np.atleast_2d(w)
    return np.concatenate([w[:, None, :n], w[:, n:].reshape(w.shape[0], N, 2 * n + nf)[:, :, n + nf:]], axis=1)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=8192,
                    help="horizons per GPU (default: the C5 batch of 8192 on every GPU, weak scaling)")
    ap.add_argument("--c5", action="store_true",
                    help="BASELINE config C5 as SURVEY.md s.8(e) defines it: --batch horizons IN TOTAL (default 8192), "
                         "sharded over the ranks by shard_range (1024 per GPU at N = 8; strong scaling)")
    ap.add_argument("--nodes", type=int, default=100)
    ap.add_argument("--max-iter", type=int, default=3000, help="IPOPT's default max_iter")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=0, help="horizons in the CPU sample (0: 4 per thread)")
    ap.add_argument("--cpu-reps", type=int, default=3, help="timed CPU runs (median reported)")
    ap.add_argument("--no-extra", action="store_true",
                    help="skip the 1024-shard, single-problem and merit-mode figures")
    ap.add_argument("--no-generic", action="store_true",
                    help="skip the generic-solver figures (BASELINE configs 3 and 4, tools/generic_bench.py)")
    ap.add_argument("--generic-batch", type=int, default=4096,
                    help="starts per generic-solver figure (the C3 figure is set by a few starts that run to the "
                         "cap at single-horizon latency, so a larger batch amortises that tail)")
    ap.add_argument("--inflight", type=int, default=3,
                    help="independent steps in flight (own workspace, stream and host thread each; measured r06zb: "
                         "2 -> 1,291, 3 -> 1,496, 4 -> 1,491 horizons/s)")
    ap.add_argument("--hw-queues", type=int, default=8,
                    help="HIP hardware queues of this process (GPU_MAX_HW_QUEUES, set before the runtime starts, "
                         "over any exported value; 0 = keep the exported value)")
    args = ap.parse_args()
    if args.hw_queues > 0:
        os.environ["GPU_MAX_HW_QUEUES"] = str(min(args.hw_queues, 32))

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", rank=rank, world_size=world)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    from mpc_fatigue_amd import _lib, problems as PR
    from mpc_fatigue_amd.gocp import GOCP
    from mpc_fatigue_amd.ocp import OCP
    from mpc_fatigue_amd.shard import shard_range, gather_solutions

    N = args.nodes
    spec = PR.pilz6_bench(N=N)
    g0 = GOCP(spec)
    n, nf = 6, 1
    gB, scaling, wl_prefix = workload_plan(args.batch, args.c5, world)  # C5: a fixed total; default: --batch per GPU
    lo, hi = shard_range(gB, world, rank)
    B = hi - lo
    Q0_all = PR.pilz6_batch_q0(gB, seed=0)
    q0 = torch.tensor(Q0_all[lo:hi], dtype=torch.float64, device=dev).contiguous()
    lref = torch.empty((B, 2), dtype=torch.float64, device=dev)
    pos = torch.empty((B, 3), dtype=torch.float64, device=dev)
    stream = torch.cuda.current_stream(dev)
    model = g0.models[0]
    _lib.check(_lib.lib().mf_fk_dev(model.handle, model.frame_id(spec["frame"]), q0.data_ptr(), pos.data_ptr(), None,
                                    B, stream.cuda_stream))
    lref.copy_(pos[:, :2])

    def outputs(nb):
        return {"w": torch.empty((nb, g0.wsize), dtype=torch.float64, device=dev),
                "status": torch.empty(nb, dtype=torch.int32, device=dev),
                "iters": torch.empty(nb, dtype=torch.int32, device=dev),
                "kkt": torch.empty(nb, dtype=torch.float64, device=dev),
                "obj": torch.empty(nb, dtype=torch.float64, device=dev)}
    out = outputs(B)
    ptrs = {k: v.data_ptr() for k, v in out.items()}
    opts = dict(IPOPT_MODE, max_iter=args.max_iter)

    # Steps in flight (StepLoop): each slot is its own solver handle (workspace), HIP stream and host thread (the
    # solve's host loop polls its stream); every slot solves on a stream of its own (none on the default stream,
    # where the N > 1 gathers run)
    inflight = max(1, args.inflight)
    slots = [(g0, torch.cuda.Stream(dev), out, ptrs)]
    for _ in range(inflight - 1):
        ob = {k: torch.empty_like(v) for k, v in out.items()}
        slots.append((GOCP(spec, models=g0.models), torch.cuda.Stream(dev), ob, {k: v.data_ptr() for k, v in ob.items()}))
    torch.cuda.synchronize(dev)

    def solve_on(step, i, nb=B, ev=None, **kw):
        torch.cuda.set_device(dev)  # the HIP device is per host thread
        g, st, ob, pt = slots[i]
        if ev is not None:  # this slot's previous solutions gathered (N > 1)
            st.wait_event(ev)
        g.solve_dev(q0.data_ptr(), None, None, lref.data_ptr(), nb, pt, stream=st.cuda_stream, **dict(opts, **kw))
        st.synchronize()

    def gather_slot(step, i):
        _, _, ob, _ = slots[i]
        gather_solutions(ob["w"], ob["status"], rank, world, total=gB)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(dev))  # the stream the gather ran on
        return ev

    loop = StepLoop(inflight, solve_on, gather_slot if world > 1 else None)

    def run_steps(K, nb=B, first=0):
        loop.run(K, nb, gather=(nb == B), first=first)

    run_steps(max(args.warmup, 1))              # untimed warm-up step(s)
    for i in range(1, inflight):                # every other slot's workspace allocated, code loaded
        solve_on(0, i, max_iter=1)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    run_steps(args.steps)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = torch.tensor([t1 - t0], dtype=torch.float64, device=dev)
    # every slot solved the same shard: the converged count of one step is that of any slot's last solve
    status = out["status"].cpu().numpy()
    iters = out["iters"].cpu().numpy()
    conv = torch.tensor([int((status == 0).sum())], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
        dist.all_reduce(conv, op=dist.ReduceOp.SUM)
    elapsed = float(elapsed.item())
    converged = float(conv.item())
    value = converged * args.steps / elapsed
    sv, sc = np.unique(status, return_counts=True)

    # ---- the node-evaluation phase vs its HBM roofline; HIP events on the solve stream, one more
    # step of the same batch solved alone after the timed region (steps in flight would share the GPU)
    g0.timing(True)
    solve_on(0, 0)
    torch.cuda.synchronize(dev)
    stats = g0.kernel_stats()
    nevals = g0.node_evals()
    g0.timing(False)
    ev_ms = stats["k_geval"][0] + stats["k_gasm"][0]
    ev_launches = stats["k_geval"][1]
    per_launch_ms = ev_ms / max(1, ev_launches)
    total_bytes = NODE_BYTES * float(nevals)
    bytes_per_launch = total_bytes / max(1, ev_launches)
    achieved = total_bytes / (ev_ms / 1e3) / 1e9
    traffic, iter_traffic = None, None
    pmc_path = os.path.join(ROOT, "profiles", "pmc_traffic_ipopt.json")
    if os.path.exists(pmc_path):
        with open(pmc_path) as f:
            pmc = json.load(f)
        if pmc.get("eval_hbm_bytes_per_node_eval"):
            traffic = pmc["eval_hbm_bytes_per_node_eval"] * total_bytes / NODE_BYTES / max(1, ev_launches)
        iter_traffic = pmc.get("iteration")
    total_ms = sum(v[0] for v in stats.values())
    roofline = {
        "kernel": "k_geval+k_gasm", "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
        "traffic_over_algorithmic": (traffic / bytes_per_launch) if traffic else None,
        "algorithmic_bytes_per_launch": bytes_per_launch, "bytes_per_node": NODE_BYTES,
        "node_evaluations": nevals, "avg_launch_ms": per_launch_ms, "launches": ev_launches,
        "kernel_ms": {k: v[0] for k, v in stats.items()},
        "kernel_share": {k: v[0] / total_ms for k, v in stats.items()},
        "iteration_traffic": iter_traffic,
        "launch_note": ("one node-evaluation launch = the generic solver's k_geval (sweeps) then k_gasm (records) on one "
                        "stream; rocprofv3 lists the two, their averages sum to avg_launch_ms.  Bytes: SURVEY.md s.8(d) "
                        "952 B per running node evaluation (device-counted).  The dominant phase is k_gkkt "
                        "(kernel_share), a serial 100-stage Riccati sweep per horizon: latency-bound, not HBM-bound"),
        "timing": "HIP events over one step of the same batch solved alone after the timed region",
    }

    result = {
        "metric": METRIC, "value": value, "unit": "horizons/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "scaling": scaling, "vs_baseline": None, "dtype": "f64", "data": "synthetic",
        "config": {"workload": wl_prefix +
                               f"pilz6_force N={N} (fatigue floor {PR.BENCH_FLOOR:g} Nm), {B} horizons per GPU, "
                               "q0 = IK + U(-0.05,0.05), line ref = fk(q0); solved as the reference solves it: IPOPT "
                               "from x0 = 0 (filter line search, watchdog, soft restoration, restoration phase with "
                               "elastic rows, bound_relax 1e-8, max_iter 3000)",
                   "solver": "ipopt_mode (csrc/gipm.hip, chain family)",
                   "horizon_nodes": N, "batch_per_gpu": B, "global_batch": gB,
                   "parallelism": f"dp{world} (independent horizons; RCCL gather of solutions)",
                   "converged_per_step": converged, "converged_frac": converged / gB,
                   "status_counts": {int(a): int(c) for a, c in zip(sv, sc)},
                   "mean_iters": float(iters.mean()), "max_iters": int(iters.max()),
                   "steps_in_flight": inflight, "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"),
                   "tol": opts["tol"], "max_iter": opts["max_iter"]},
        "roofline": roofline,
        "cpu_baseline": None,
    }

    if world == 1 and not args.no_extra:
        def timed(nb, reps):
            o = {k: v[:nb] for k, v in out.items()}
            pt = {k: v.data_ptr() for k, v in o.items()}
            s0 = slots[0][1]
            ts = []
            for _ in range(reps):
                torch.cuda.synchronize(dev)
                t = time.perf_counter()
                g0.solve_dev(q0.data_ptr(), None, None, lref.data_ptr(), nb, pt, stream=s0.cuda_stream, **opts)
                torch.cuda.synchronize(dev)
                ts.append(time.perf_counter() - t)
            return float(np.median(ts)), int((o["status"] == 0).sum().item()), o
        if B >= 1024:
            t1024, c1024, _ = timed(1024, 1)
            result["c5_shard_1024"] = {"value": c1024 / t1024, "unit": "horizons/s", "ms_per_step": t1024 * 1e3,
                                       "converged": c1024, "note": "first 1024 horizons of the batch, one step alone"}
            # the same shard as each rank of an 8-GPU C5 run solves it (--c5 at N = 8): steps in flight
            K1 = 4 * inflight
            torch.cuda.synchronize(dev)
            t = time.perf_counter()
            run_steps(K1, nb=1024)
            torch.cuda.synchronize(dev)
            tk = time.perf_counter() - t
            ck = int((out["status"][:1024] == 0).sum().item())
            result["c5_shard_1024"]["inflight"] = {
                "value": ck * K1 / tk, "steps": K1, "steps_in_flight": inflight, "ms_per_step": tk / K1 * 1e3,
                "note": "1024 horizons per step, the bench's steps in flight (the per-rank load of C5 on 8 GPUs)"}
        t1, c1, o1 = timed(1, 3)
        result["single_problem"] = {"ms_per_solve": t1 * 1e3, "converged": c1, "iters": int(o1["iters"][0].item()),
                                    "note": "horizon 0 of the batch alone, IPOPT mode, median of 3 (host-polled every "
                                            "4 launch rounds)"}
        # the specialised l1-merit solver of rounds 1-5 (csrc/ipm_kernels.hip): a build-defined globalisation from the
        # held state with F = 1 that ends at a neighbouring optimum of the reference's; labelled, not
        # the headline
        ocp = OCP(spec)
        mo = outputs(B)
        mopt = dict(tol=1e-8, constr_viol_tol=1e-8, max_iter=300, mu_init=0.1, F_init=PR.BENCH_F_INIT)
        s0 = slots[0][1]
        ocp.solve_dev(q0.data_ptr(), lref.data_ptr(), B, {k: v.data_ptr() for k, v in mo.items()},
                      stream=s0.cuda_stream, **mopt)
        torch.cuda.synchronize(dev)
        t = time.perf_counter()
        ocp.solve_dev(q0.data_ptr(), lref.data_ptr(), B, {k: v.data_ptr() for k, v in mo.items()},
                      stream=s0.cuda_stream, **mopt)
        torch.cuda.synchronize(dev)
        tm = time.perf_counter() - t
        cm = int((mo["status"] == 0).sum().item())
        wi = out["w"][:2].cpu().numpy()
        wm = mo["w"][:2].cpu().numpy()
        result["merit_mode"] = {
            "value": cm / tm, "unit": "horizons/s", "ms_per_step": tm * 1e3, "converged": cm,
            "mean_iters": float(mo["iters"].float().mean().item()),
            "max_dq_vs_ipopt_mode_h01": float(np.abs(wq_traj(wi, n, nf, N) - wq_traj(wm, n, nf, N)).max()),
            "note": ("NOT the reference's algorithm: the specialised l1-merit interior point (csrc/ipm_kernels.hip) "
                     "started from the held state with F = 1, one step of the same batch alone; it reaches a "
                     "neighbouring optimum of the IPOPT-mode answer (max_dq on horizons 0 and 1)")}

    if world == 1 and not args.no_extra and not args.no_generic:
        # BASELINE configs 3 (dual-arm shared fatigue budget, N = 100) and 4 (Centauro, N = 50) through the
        # generic stage-structured solver (csrc/gipm.hip): batches of perturbed starts, GPU vs the host IPM
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        from generic_bench import generic_extra
        torch.cuda.set_device(dev)
        result["generic"] = generic_extra(batch=args.generic_batch, sample=2, cpu=not args.no_cpu_baseline,
                                          mode="ipopt", cases=("c3", "c4"), max_iter=1500)

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import pin_np as P
        from oracle.urdf_np import load_urdf_file

        threads, why = cpu_threads()
        S = args.cpu_sample or 4 * threads
        ref = load_urdf_file(PR.urdf_path(spec["urdf"]))
        Qs = Q0_all[:S]
        lrs = [P.forward_kinematics(ref, Qs[i], "prbt_link_5")[0][:2] for i in range(S)]
        rec, w_cpu, st_cpu, obj_cpu = cpu_baseline(lambda q, lr: PR.pilz6_bench(N=N, q0=q, line_ref=lr), Qs, lrs,
                                                   dict(opts, riccati=2), threads, S, max(2, min(4, S)), args.cpu_reps)
        # the bench's own answers against the CPU solutions of the same horizons
        w_gpu = out["w"][:S].cpu().numpy()
        st_gpu = out["status"][:S].cpu().numpy()
        ob_gpu = out["obj"][:S].cpu().numpy()
        both = (st_gpu == 0) & (st_cpu == 0)
        dq = np.abs(wq_traj(w_gpu, n, nf, N) - wq_traj(w_cpu, n, nf, N)).max(axis=(1, 2))
        dq_in = np.abs(wq_traj(w_gpu, n, nf, N)[:, :N] - wq_traj(w_cpu, n, nf, N)[:, :N]).max(axis=(1, 2))
        dob = np.abs(ob_gpu - obj_cpu) / np.abs(obj_cpu)
        rec["cores_note"] = why
        rec["gpu_vs_cpu"] = {"horizons": S, "both_converged": int(both.sum()),
                             "same_status": int((st_gpu == st_cpu).sum()),
                             "max_dq": float(dq[both].max()) if both.any() else None,
                             "max_dq_nodes_0_to_N-1": float(dq_in[both].max()) if both.any() else None,
                             "same_path_1e-6": int((dq[both] < 1e-6).sum()),
                             "max_rel_dobj": float(dob[both].max()) if both.any() else None}
        result["cpu_baseline"] = rec
    if rank == 0:
        print(json.dumps(result))
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
