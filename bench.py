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
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

Also reported: the dominant kernel's achieved rate against its roofline
(per-kernel HIP-event timing over the timed region, algorithmic bytes from
DESIGN.md section 5), and the CPU baseline = the oracle's C restatement of the
same solver on the host cores (rank 0, N = 1 only, bounded sample).
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


def node_bytes(n: int, nf: int, nl: int) -> dict:
    """Algorithmic HBM bytes per shooting node of one running horizon per launch.

    k_eval_node: reads q, qd, F, y_tau, y_line of the node; writes d tau/dw (n x nv), the raw
                 Hessian columns of the 2n lane directions (nv x 2n), d line/dq, tau, line, cost
    k_eval_asm : reads the raw Hessian's lower triangle, d tau/dw, the torque-slack and bound
                 multiplier data of the node; writes the condensed stage Hessian H0 and grad f
    k_ipm_kkt  : reads H0, d tau/dw, grad f and the stage data once, writes and reads back the
                 Riccati slot (Ku, Kl, P_{k+1}, ku, kl, p_{k+1}) and the step
    """
    nv, nu, nla = 2 * n + nf, n + nf, max(nl, 1)
    ev = (2 * n + nf + n + nl) + (n * nv + nv * 2 * n + nl * n + n + nl + 1)
    asm = (nv * (nv + 1) // 2 + n * nv + 3 * n + 2 * n + 6 * n + n + nf) + (nv * nv + nv)
    slot = nu * n + nl * n + n * n + nu + nl + n
    kkt = (nv * nv + n * nv + nv + n + nla + nl * n) + 2 * slot + (2 * n + nf + n + nl + n) + (2 * n + nv + 2 * n + nla)
    return {"k_eval_node": 8 * ev, "k_eval_asm": 8 * asm, "k_ipm_kkt": 8 * kkt}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=8192,
                    help="horizons per GPU (default: the C5 batch of 8192 on every GPU, weak scaling)")
    ap.add_argument("--nodes", type=int, default=100)
    ap.add_argument("--max-iter", type=int, default=300)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=0, help="horizons in the CPU sample (0: 2 per thread)")
    args = ap.parse_args()

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

    N, B = args.nodes, args.batch
    spec = PR.pilz6_bench(N=N)
    ocp = OCP(spec)
    n = ocp.n
    gB = B * world
    lo, hi = shard_range(gB, world, rank)
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

    def step():
        ocp.solve_dev(q0.data_ptr(), lref.data_ptr(), hi - lo, ptrs, stream=stream.cuda_stream, **opts)
        if world > 1:
            gather_solutions(out["w"], out["status"], rank, world)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    ocp.timing(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
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

    # ---- dominant kernel vs roofline (this rank's HIP-event timing over the timed region)
    stats = ocp.kernel_stats()
    ocp.timing(False)
    nb = node_bytes(n, ocp.nf, ocp.nl)
    dom = max(stats, key=lambda k: stats[k][0])
    dom_ms, dom_launches = stats[dom]
    per_launch_ms = dom_ms / max(1, dom_launches)
    if dom in nb:
        total_bytes = nb[dom] * float(node_evals.item()) * args.steps
        achieved = total_bytes / (dom_ms / 1e3) / 1e9
        bytes_per_launch = total_bytes / max(1, dom_launches)
    else:
        achieved, bytes_per_launch = None, None
    traffic, fp64 = None, None
    pmc_path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(pmc_path):
        with open(pmc_path) as f:
            pmc = json.load(f).get(dom, {})
        traffic = pmc.get("hbm_bytes_per_launch")
        if pmc.get("fp64_flops_per_launch"):
            # executed FP64 flops per launch (PMC, same workload) over this run's launch time
            tfs = pmc["fp64_flops_per_launch"] / (per_launch_ms / 1e3) / 1e12
            fp64 = {"achieved": tfs, "peak": FP64_PEAK_TFS, "unit": "TFLOP/s", "frac": tfs / FP64_PEAK_TFS,
                    "flops_per_launch": pmc["fp64_flops_per_launch"],
                    "note": "FP64 VALU work (the bound of this kernel); flops from SQ_INSTS_VALU_{FMA,MUL,ADD}_F64 x 64 lanes"}
    roofline = {
        "kernel": dom, "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": (achieved / HBM_PEAK_GBS) if achieved else None, "traffic": traffic,
        "avg_launch_ms": per_launch_ms, "launches": dom_launches, "algorithmic_bytes_per_launch": bytes_per_launch,
        "kernel_ms": {k: v[0] for k, v in stats.items()}, "fp64": fp64,
    }
    if dom == "k_eval_node":
        roofline["launch_note"] = ("one k_eval_node launch = the solver's phase 0: k_eval_node<..,0> (q directions) "
                                   "then k_eval_node<..,1> (qd directions) on one stream; rocprofv3 lists the two, "
                                   "their averages sum to avg_launch_ms")

    result = {
        "metric": METRIC, "value": value, "unit": "horizons/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
        "config": {"workload": f"pilz6_force N={N} (fatigue floor {PR.BENCH_FLOOR:g} Nm), {B} horizons per GPU, "
                               "q0 = IK + U(-0.05,0.05), line ref = fk(q0)",
                   "horizon_nodes": N, "batch_per_gpu": B, "global_batch": gB,
                   "parallelism": f"dp{world} (independent horizons; RCCL gather of solutions)",
                   "converged_per_step": converged, "converged_frac": converged / gB,
                   "mean_iters": float(iters.mean()), "max_iters": int(iters.max()),
                   "tol": opts["tol"]},
        "roofline": roofline,
        "cpu_baseline": None,
    }

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import oracle as O
        from oracle import pin_np as P
        from oracle.urdf_np import load_urdf_file

        threads = min(16, os.cpu_count() or 1)
        S = args.cpu_sample or 2 * threads
        ref = load_urdf_file(PR.urdf_path(spec["urdf"]))
        Qs = Q0_all[:S]
        specs = [PR.pilz6_bench(N=N, q0=Qs[i], line_ref=P.forward_kinematics(ref, Qs[i], "prbt_link_5")[0][:2])
                 for i in range(S)]
        c0 = time.perf_counter()
        _, R = O.solve_batch(ref, specs, nthreads=threads, **opts)
        c1 = time.perf_counter()
        cconv = sum(1 for r in R if r.status == 0)
        result["cpu_baseline"] = {"value": cconv / (c1 - c0), "unit": "horizons/s", "cores": threads,
                                  "kind": "port",
                                  "sample": f"first {S} horizons of the same batch, oracle/mf_oracle.c IPM, "
                                            f"OpenMP over horizons, {cconv}/{S} converged, {c1 - c0:.1f} s"}
    if rank == 0:
        print(json.dumps(result))
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
