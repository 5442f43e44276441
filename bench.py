"""Benchmark: MPC horizons solved / s, Pilz-6DOF N=100, batched on MI355X.

A step = one complete interior-point solve (from the initial guess to
convergence) of this rank's shard of horizons, followed (N > 1) by the RCCL
gather of every shard's solutions to rank 0 -- the batched configuration of
BASELINE.json (C5: 8192 independent horizons, q0_i = q0_IK + U(-0.05, 0.05) per
joint, line reference = fk(q0_i)[0:2]).  Every GPU solves a C5-sized batch of
8192 horizons (weak scaling: N GPUs solve N x 8192 distinct horizons; --batch 1024
gives C5's 8-GPU shard size).  value = horizons that reached the KKT tolerance on
all ranks / max-over-ranks wall time (inputs resident in HBM).

    python bench.py [--gpus N --steps K --warmup W --batch B --nodes 100]
    python bench.py --c5 ...   (C5 as SURVEY.md s.8(e): --batch horizons in total, sharded; strong scaling)
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

Also reported: the node-evaluation kernel's achieved rate against its HBM
roofline (per-kernel HIP-event timing over the timed region, SURVEY.md s.8(d)'s
952 algorithmic bytes per node evaluation, PMC traffic per node evaluation from
profiles/pmc_traffic.json), the iteration tail (GPU time per 4-iteration chunk
and running count), C5's 1024-horizon shard and the single-problem latency, and
the CPU baseline = the same interior-point algorithm on the host with the
product's node functions compiled for the CPU, on all cores and on one core
(rank 0, N = 1 only, bounded sample), whose solutions are compared with the
GPU's for the same horizons (max_dq).
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
    kw = dict(opts, riccati=True, **CF.FastNodes(specs[0]).opts_kw())
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
            w_mt, st_mt = w, np.array([r.status for r in R])
    rec = {"value": out["all_cores"]["value"], "unit": "horizons/s", "cores": threads, "kind": "port",
           "single_core": out["one_core"]["value"], "nproc": os.cpu_count(), "detail": out,
           "time_split_one_core": split,
           "sample": (f"first {sample_mt} horizons of the same batch on {threads} threads and the first {sample_1t} "
                      f"on 1 thread (median of {reps} runs after a warm-up); generic IPM oracle/mf_ocp.c with the "
                      "product's node functions, both built for the host at -O3 -march=x86-64-v3 (oracle/libmfcpu.so); "
                      "KKT by the device's Riccati recursion (mfg_opts.riccati, stage blocks factored by Bunch-Kaufman, "
                      "the GPU's algorithm), not the checker's block-tridiagonal factorisation")}
    return rec, w_mt, st_mt


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
    ap.add_argument("--max-iter", type=int, default=300)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=0, help="horizons in the CPU sample (0: 4 per thread)")
    ap.add_argument("--cpu-reps", type=int, default=5, help="timed CPU runs (median reported)")
    ap.add_argument("--no-extra", action="store_true", help="skip the 1024-shard and single-problem figures")
    ap.add_argument("--no-generic", action="store_true",
                    help="skip the generic-solver figures (BASELINE configs 3 and 4, tools/generic_bench.py)")
    ap.add_argument("--generic-batch", type=int, default=4096,
                    help="starts per generic-solver figure (the C3 figure is set by a few starts that run to the "
                         "last stage's cap at single-horizon latency, so a larger batch amortises that tail: 1024 "
                         "starts 20 horizons/s, 4096 starts 52, r03af)")
    ap.add_argument("--inflight", type=int, default=4,
                    help="independent steps in flight (own workspace, stream and host thread each)")
    ap.add_argument("--hw-queues", type=int, default=8,
                    help="HIP hardware queues of this process (GPU_MAX_HW_QUEUES, set before the runtime starts, "
                         "over any exported value; 0 = keep the exported value): "
                         "with the runtime's default of 4, the steps' streams and the default stream share queues "
                         "and serialise (r03ab/r03ac: 4 in flight 11.3k horizons/s on 4 queues, 12.0k on 8)")
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
    from mpc_fatigue_amd.ocp import OCP
    from mpc_fatigue_amd.shard import shard_range, gather_solutions

    N = args.nodes
    spec = PR.pilz6_bench(N=N)
    ocp = OCP(spec)
    n = ocp.n
    gB, scaling, wl_prefix = workload_plan(args.batch, args.c5, world)  # C5: a fixed total; default: --batch per GPU
    lo, hi = shard_range(gB, world, rank)
    B = hi - lo
    Q0_all = PR.pilz6_batch_q0(gB, seed=0)
    q0 = torch.tensor(Q0_all[lo:hi], dtype=torch.float64, device=dev).contiguous()
    lref = torch.empty((hi - lo, 2), dtype=torch.float64, device=dev)
    pos = torch.empty((hi - lo, 3), dtype=torch.float64, device=dev)
    stream = torch.cuda.current_stream(dev)
    frame = ocp.model.frame_id(spec["frame"])
    _lib.check(_lib.lib().mf_fk_dev(ocp.model.handle, frame, q0.data_ptr(), pos.data_ptr(), None, hi - lo,
                                    stream.cuda_stream))
    lref.copy_(pos[:, :2])
    out = {
        "w": torch.empty((hi - lo, ocp.wsize), dtype=torch.float64, device=dev),
        "status": torch.empty(hi - lo, dtype=torch.int32, device=dev),
        "iters": torch.empty(hi - lo, dtype=torch.int32, device=dev),
        "kkt": torch.empty(hi - lo, dtype=torch.float64, device=dev),
        "obj": torch.empty(hi - lo, dtype=torch.float64, device=dev),
    }
    ptrs = {k: v.data_ptr() for k, v in out.items()}
    opts = dict(tol=1e-8, constr_viol_tol=1e-8, max_iter=args.max_iter, mu_init=0.1, F_init=PR.BENCH_F_INIT)

    # Steps in flight (StepLoop): each slot is its own solver workspace, HIP stream and host thread (the
    # solve's host loop polls its stream); every slot solves on a stream of its own (none on the default
    # stream, where the N > 1 gathers run)
    inflight = max(1, args.inflight)
    slots = [(ocp, torch.cuda.Stream(dev), out, ptrs)]
    for _ in range(inflight - 1):
        ob = {k: torch.empty_like(v) for k, v in out.items()}
        slots.append((OCP(spec), torch.cuda.Stream(dev), ob, {k: v.data_ptr() for k, v in ob.items()}))
    torch.cuda.synchronize(dev)

    def solve_on(step, i, nb=hi - lo, ev=None):
        torch.cuda.set_device(dev)  # the HIP device is per host thread
        o, st, ob, pt = slots[i]
        if ev is not None:  # this slot's previous solutions gathered (N > 1)
            st.wait_event(ev)
        o.solve_dev(q0.data_ptr(), lref.data_ptr(), nb, pt, stream=st.cuda_stream, **opts)
        st.synchronize()

    def gather_slot(step, i):
        _, _, ob, _ = slots[i]
        gather_solutions(ob["w"], ob["status"], rank, world, total=gB)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(dev))  # the stream the gather ran on
        return ev

    loop = StepLoop(inflight, solve_on, gather_slot if world > 1 else None)

    def run_steps(K, nb=hi - lo):
        loop.run(K, nb, gather=(nb == hi - lo))

    run_steps(max(args.warmup, inflight))  # every slot warm (workspace allocated)
    torch.cuda.synchronize(dev)
    if inflight == 1:
        ocp.timing(True)
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
    status = out["status"].cpu().numpy()
    iters = out["iters"].cpu().numpy()
    conv = torch.tensor([int((status == 0).sum())], dtype=torch.float64, device=dev)
    node_evals = torch.tensor([float(((iters + 1) * N).sum())], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
        dist.all_reduce(conv, op=dist.ReduceOp.SUM)
    elapsed = float(elapsed.item())
    converged = float(conv.item())
    value = converged * args.steps / elapsed

    # ---- node-evaluation kernel vs its HBM roofline; HIP events on the solve stream
    # With steps in flight the per-kernel HIP-event durations of the timed region include the other
    # step's kernels running beside them; the kernel figures then come from one more step of the same
    # batch solved alone right after the timed region (same solver, same iterations).
    timing_steps = args.steps
    if inflight > 1:
        ocp.timing(True)
        solve_on(0, 0)
        torch.cuda.synchronize(dev)
        timing_steps = 1
    stats = ocp.kernel_stats()
    trace = ocp.trace()
    ocp.timing(False)
    ev_ms, ev_launches = stats["k_eval_node"]
    per_launch_ms = ev_ms / max(1, ev_launches)
    total_bytes = NODE_BYTES * float(node_evals.item()) * timing_steps  # this rank's node evaluations
    bytes_per_launch = total_bytes / max(1, ev_launches)
    achieved = total_bytes / (ev_ms / 1e3) / 1e9
    traffic, fp64, iter_traffic = None, None, None
    pmc_path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(pmc_path):
        with open(pmc_path) as f:
            pmc = json.load(f)
        ev = pmc.get("k_eval_node", {})
        # whole-iteration HBM traffic (PMC FETCH_SIZE + WRITE_SIZE of every per-iteration kernel, per launch) at the
        # profiled workload, and per running horizon-iteration (running horizons per launch = node evaluations / N)
        it_k = ["k_eval_q", "k_eval_node[qd]", "k_eval_asm", "k_ipm_pre", "k_ipm_kkt", "k_kkt_recover", "k_ipm_post",
                "k_post_update", "k_compact"]
        it_k = [k for k in it_k if k in pmc]  # (k_post_update: folded into k_ipm_post in round 3)
        if "k_ipm_kkt" in it_k and ev.get("node_evals"):
            per_k = {k: pmc[k]["hbm_bytes_per_launch"] for k in it_k}
            tot = sum(per_k.values())
            running = ev["node_evals"] / ev["launches"] / N
            iter_traffic = {"hbm_bytes_per_iteration": tot, "running_horizons_per_iteration": running,
                            "hbm_bytes_per_horizon_iteration": tot / running,
                            "eval_algorithmic_bytes_per_horizon_iteration": NODE_BYTES * N,
                            "per_kernel_bytes_per_iteration": per_k,
                            "source": "profiles/pmc_traffic.json (PMC of tools/traffic_run.py: the C5 batch solved once)"}
        if ev.get("hbm_bytes_per_node_eval"):
            traffic = ev["hbm_bytes_per_node_eval"] * total_bytes / NODE_BYTES / max(1, ev_launches)
        if ev.get("fp64_flops_per_node_eval"):
            fl = ev["fp64_flops_per_node_eval"] * total_bytes / NODE_BYTES / max(1, ev_launches)
            tfs = fl / (per_launch_ms / 1e3) / 1e12
            fp64 = {"achieved": tfs, "peak": FP64_PEAK_TFS, "unit": "TFLOP/s", "frac": tfs / FP64_PEAK_TFS,
                    "flops_per_launch": fl,
                    "note": "executed FP64 VALU flops (PMC SQ_INSTS_VALU_{FMA,MUL,ADD}_F64 x 64, per node evaluation "
                            "of the same workload, profiles/pmc_traffic.json) over this run's launch time"}
    # algorithmic FP64 work: op-counted on the device templates (tools/flopcount.py, profiles/fp64_opcount.json)
    opc_path = os.path.join(ROOT, "profiles", "fp64_opcount.json")
    if os.path.exists(opc_path):
        with open(opc_path) as f:
            opc = json.load(f)
        fla = opc["eval_phase_ops_per_node_eval"] * total_bytes / NODE_BYTES / max(1, ev_launches)
        tfa = fla / (per_launch_ms / 1e3) / 1e12
        algo = {"achieved": tfa, "peak": FP64_PEAK_TFS, "unit": "TFLOP/s", "frac": tfa / FP64_PEAK_TFS,
                "flops_per_launch": fla, "ops_per_node_eval": opc["eval_phase_ops_per_node_eval"],
                "note": "op-counted algorithmic FP64 work of the eval phase's lanes per node evaluation "
                        "(profiles/fp64_opcount.json) over this run's launch time"}
        fp64 = dict(algo, executed=fp64)
    total_ms = sum(v[0] for v in stats.values())
    roofline = {
        "kernel": "k_eval_node", "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
        "traffic_over_algorithmic": (traffic / bytes_per_launch) if traffic else None,
        "algorithmic_bytes_per_launch": bytes_per_launch, "bytes_per_node": NODE_BYTES,
        "avg_launch_ms": per_launch_ms, "launches": ev_launches,
        "kernel_ms": {k: v[0] for k, v in stats.items()},
        "kernel_share": {k: v[0] / total_ms for k, v in stats.items()}, "fp64": fp64,
        "iteration_traffic": iter_traffic,
        "launch_note": ("one k_eval_node launch = the solver's phase 0: k_eval_node<..,0> (q directions) then "
                        "k_eval_node<..,1> (qd directions) on one stream; rocprofv3 lists the two, their averages "
                        "sum to avg_launch_ms. Bytes: SURVEY.md s.8(d) 952 B per running node evaluation"),
        "timing": ("HIP events over the timed region" if inflight == 1 else
                   f"HIP events over one step of the same batch solved alone after the timed region ({inflight} steps "
                   "in flight in the timed region share the GPU, which would inflate every kernel's duration)"),
    }
    # iteration tail: per 4-iteration chunk, problems running at its start and its GPU time (last step)
    tr_ms = trace["ms"]
    tail = trace["running"] < 0.1 * B
    tail_rec = {"chunks": len(tr_ms), "gpu_ms": float(tr_ms.sum()), "share_below_10pct_running":
                float(tr_ms[tail].sum() / max(tr_ms.sum(), 1e-12)),
                "running_at_chunk": [int(x) for x in trace["running"]],
                "ms_per_chunk": [round(float(x), 2) for x in tr_ms]}

    result = {
        "metric": METRIC, "value": value, "unit": "horizons/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "scaling": scaling, "vs_baseline": None, "dtype": "f64", "data": "synthetic",
        "config": {"workload": wl_prefix +
                               f"pilz6_force N={N} (fatigue floor {PR.BENCH_FLOOR:g} Nm), {B} horizons per GPU, "
                               "q0 = IK + U(-0.05,0.05), line ref = fk(q0)",
                   "horizon_nodes": N, "batch_per_gpu": B, "global_batch": gB,
                   "parallelism": f"dp{world} (independent horizons; RCCL gather of solutions)",
                   "converged_per_step": converged, "converged_frac": converged / gB,
                   "mean_iters": float(iters.mean()), "max_iters": int(iters.max()),
                   "steps_in_flight": inflight, "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"),
                   "tol": opts["tol"]},
        "roofline": roofline,
        "tail": tail_rec,
        "cpu_baseline": None,
    }

    if world == 1 and not args.no_extra:
        # C5's per-GPU shard (1024 horizons) and the single-problem latency (BASELINE config 2), same solver
        def timed(nb, reps):
            o = {k: v[:nb] for k, v in out.items()}
            pt = {k: v.data_ptr() for k, v in o.items()}
            s0 = slots[0][1]
            ocp.solve_dev(q0.data_ptr(), lref.data_ptr(), nb, pt, stream=s0.cuda_stream, **opts)
            ts = []
            for _ in range(reps):
                torch.cuda.synchronize(dev)
                t = time.perf_counter()
                ocp.solve_dev(q0.data_ptr(), lref.data_ptr(), nb, pt, stream=s0.cuda_stream, **opts)
                torch.cuda.synchronize(dev)
                ts.append(time.perf_counter() - t)
            return float(np.median(ts)), int((o["status"] == 0).sum().item())
        if B >= 1024:
            t1024, c1024 = timed(1024, 3)
            rec1024 = {"value": c1024 / t1024, "unit": "horizons/s", "ms_per_step": t1024 * 1e3,
                       "converged": c1024, "note": "first 1024 horizons of the batch, one step alone, median of 3"}
            if inflight > 1:
                # the same shard at the bench's steps-in-flight setting (what each rank of the 8-GPU C5 run
                # would do with --batch 1024): K consecutive 1024-horizon steps, `inflight` of them at a time
                K = 4 * inflight
                run_steps(inflight, 1024)
                torch.cuda.synchronize(dev)
                t = time.perf_counter()
                run_steps(K, 1024)
                torch.cuda.synchronize(dev)
                dt = time.perf_counter() - t
                cK = sum(int((sl[2]["status"][:1024] == 0).sum().item()) for sl in slots)
                rec1024["inflight"] = {"value": cK / len(slots) * K / dt, "steps": K, "steps_in_flight": inflight,
                                       "ms_per_step": dt / K * 1e3,
                                       "note": f"{K} steps of the first 1024 horizons, {inflight} in flight"}
            result["c5_shard_1024"] = rec1024
        t1, c1 = timed(1, 5)
        result["single_problem"] = {"ms_per_solve": t1 * 1e3, "converged": c1, "iters": int(out["iters"][0].item()),
                                    "note": "horizon 0 of the batch alone, median of 5 (host-polled every 4 iterations)"}

    if world == 1 and not args.no_extra and not args.no_generic:
        # BASELINE configs 3 (dual-arm shared fatigue budget, N = 100) and 4 (Centauro, N = 50) through the
        # generic stage-structured solver (csrc/gipm.hip): batches of perturbed starts, GPU vs the host IPM
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        from generic_bench import generic_extra
        torch.cuda.set_device(dev)
        # IPOPT mode (the reference's solve: x0 = 0, filter globalisation, bound_relax 1e-8; no homotopy)
        # (c2: the headline's own C2 horizons solved as the reference solves them, through the generic solver)
        # (cap 1500: IPOPT's default 3000 only adds the last few starts' single-horizon tail, ~45 s per case, to
        # the default run; the 3000-cap figures: profiles/r04f_bench_default.json)
        result["generic"] = generic_extra(batch=args.generic_batch, sample=2, cpu=not args.no_cpu_baseline,
                                          mode="ipopt", cases=("c3", "c4", "c2"), max_iter=1500)

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import pin_np as P
        from oracle.urdf_np import load_urdf_file

        threads, why = cpu_threads()
        S = args.cpu_sample or 4 * threads
        ref = load_urdf_file(PR.urdf_path(spec["urdf"]))
        Qs = Q0_all[:S]
        lrs = [P.forward_kinematics(ref, Qs[i], "prbt_link_5")[0][:2] for i in range(S)]
        rec, w_cpu, st_cpu = cpu_baseline(lambda q, lr: PR.pilz6_bench(N=N, q0=q, line_ref=lr), Qs, lrs, opts,
                                          threads, S, max(2, min(8, S)), args.cpu_reps)
        # the bench's own answers against the CPU solutions of the same horizons
        w_gpu = out["w"][:S].cpu().numpy()
        st_gpu = out["status"][:S].cpu().numpy()
        both = (st_gpu == 0) & (st_cpu == 0)
        wq = lambda w: np.concatenate([w[:, :n]] + [w[:, n + k * (2 * n + ocp.nf) + n + ocp.nf:
                                                       n + (k + 1) * (2 * n + ocp.nf)] for k in range(N)], axis=1)
        rec["cores_note"] = why
        rec["gpu_vs_cpu"] = {"horizons": S, "both_converged": int(both.sum()),
                             "same_status": int((st_gpu == st_cpu).sum()),
                             "max_dq": float(np.abs(wq(w_gpu[both]) - wq(w_cpu[both])).max()) if both.any() else None}
        result["cpu_baseline"] = rec
    if rank == 0:
        print(json.dumps(result))
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
