"""Multi-process (world size 2, gloo on CPU) coverage of the N > 1 path:
the shard layout and the final gather of solutions to rank 0."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from mpc_fatigue_amd.shard import gather_solutions, shard_range


def test_shard_range_partitions_exactly():
    for total in [1, 7, 8192, 8193]:
        for world in [1, 2, 3, 8]:
            spans = [shard_range(total, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [h - l for l, h in spans]
            assert max(sizes) - min(sizes) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q, total, pass_total=True, claim=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = shard_range(total, world, rank)
    w = torch.arange(lo * 5, hi * 5, dtype=torch.float64).reshape(hi - lo, 5)
    st = torch.full((hi - lo,), rank, dtype=torch.int32)
    try:
        W, S = gather_solutions(w, st, rank, world, total=(claim or total) if pass_total else None)
    except ValueError as e:
        q.put(("error", rank, str(e)))
    else:
        if rank == 0:
            q.put((W.numpy().tolist(), S.numpy().tolist()))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,total,pass_total", [(2, 16, True), (2, 17, True), (2, 17, False)])
def test_gather_solutions_gloo(world, total, pass_total):
    """Equal shards and unequal ones (17 horizons over 2 ranks: 9 + 8, padded for the gather), with the
    total given or left to the collective row-count agreement."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, total, pass_total)) for r in range(world)]
    for p in procs:
        p.start()
    W, S = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    import numpy as np
    W = np.array(W)
    assert W.shape == (total, 5)
    np.testing.assert_array_equal(W.reshape(-1), np.arange(total * 5))
    spans = [shard_range(total, world, r) for r in range(world)]
    assert S == [r for r in range(world) for _ in range(spans[r][1] - spans[r][0])]


def test_gather_solutions_mismatch_fails_on_every_rank():
    """A total that disagrees with the shards held raises on every rank (none is left in the gather)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, 17, True, 18)) for r in range(2)]
    for p in procs:
        p.start()
    got = sorted(q.get(timeout=120)[:2] for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got == [("error", 0), ("error", 1)]


def _solve_worker(rank, world, port, q):
    """shard -> solve (the oracle stands in for the device on this CPU test) -> gather, the bench's N > 1
    data flow (bench.py: rank r solves horizons [lo, hi) of the global batch, RCCL gather to rank 0)."""
    import numpy as np

    from mpc_fatigue_amd import problems as PR
    from oracle import oracle as O
    from oracle import pin_np as P
    from oracle.urdf_np import load_urdf_file

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), OMP_NUM_THREADS="1")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    N, total = 8, 2 * world
    spec = PR.pilz6_bench(N=N)
    ref = load_urdf_file(PR.urdf_path(spec["urdf"]))
    Q0 = PR.pilz6_batch_q0(total, seed=0)
    lo, hi = shard_range(total, world, rank)
    specs = [PR.pilz6_bench(N=N, q0=Q0[i], line_ref=P.forward_kinematics(ref, Q0[i], "prbt_link_5")[0][:2])
             for i in range(lo, hi)]
    w, R = O.solve_batch(ref, specs, nthreads=1, tol=1e-8, constr_viol_tol=1e-8, max_iter=300, mu_init=0.1,
                         F_init=PR.BENCH_F_INIT)
    W, S = gather_solutions(torch.from_numpy(np.ascontiguousarray(w)),
                            torch.tensor([r.status for r in R], dtype=torch.int32), rank, world)
    if rank == 0:
        q.put((W.numpy().tolist(), S.numpy().tolist()))
    dist.destroy_process_group()


def test_shard_solve_gather_equals_single_process():
    import numpy as np

    from mpc_fatigue_amd import problems as PR
    from oracle import oracle as O
    from oracle import pin_np as P
    from oracle.urdf_np import load_urdf_file

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_solve_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    W, S = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    N, total = 8, 2 * world
    spec = PR.pilz6_bench(N=N)
    ref = load_urdf_file(PR.urdf_path(spec["urdf"]))
    Q0 = PR.pilz6_batch_q0(total, seed=0)
    specs = [PR.pilz6_bench(N=N, q0=q0, line_ref=P.forward_kinematics(ref, q0, "prbt_link_5")[0][:2]) for q0 in Q0]
    w1, R1 = O.solve_batch(ref, specs, nthreads=1, tol=1e-8, constr_viol_tol=1e-8, max_iter=300, mu_init=0.1,
                           F_init=PR.BENCH_F_INIT)
    np.testing.assert_array_equal(np.array(W), w1)  # same horizons in the same order, bit for bit
    assert S == [r.status for r in R1]


def _steploop_worker(rank, world, port, q, K, inflight):
    """bench.py's own step loop (StepLoop: steps in flight on per-slot buffers, per-slot gather to rank 0 after each
    step, the next solve on a slot waiting for that slot's gather event) at world size 2 on gloo, C5 as --c5 runs it
    (8192 horizons in total, shard_range over the ranks).  A deterministic CPU stand-in replaces the device solve:
    row i of step s is a function of (q0_i, s), written into the slot's own buffer by the slot's host thread."""
    import threading

    import numpy as np

    import bench
    from mpc_fatigue_amd import problems as PR

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), OMP_NUM_THREADS="1")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    gB, scaling, prefix = bench.workload_plan(8192, True, world)
    lo, hi = shard_range(gB, world, rank)
    Q0 = torch.from_numpy(PR.pilz6_batch_q0(gB, seed=0)[lo:hi])
    bufs = [{"w": torch.zeros((hi - lo, 7), dtype=torch.float64), "status": torch.zeros(hi - lo, dtype=torch.int32)}
            for _ in range(inflight)]
    busy = [threading.Lock() for _ in range(inflight)]
    log = []

    def solve(step, slot, nb, ev):
        if ev is not None:
            assert ev.is_set()  # this slot's previous solutions were gathered before it is overwritten
        with busy[slot]:
            b = bufs[slot]
            b["w"][:, :6] = torch.sin(Q0 * (step + 1))
            b["w"][:, 6] = step
            b["status"][:] = step % 3

    def gather(step, slot):
        W, S = gather_solutions(bufs[slot]["w"], bufs[slot]["status"], rank, world, total=gB)
        if rank == 0:
            log.append((step, W.numpy().copy(), S.numpy().copy()))
        ev = threading.Event()
        ev.set()
        return ev

    loop = bench.StepLoop(inflight, solve, gather)
    loop.run(inflight, hi - lo)                      # warm-up steps, gathered as the bench does
    loop.run(K, hi - lo, first=inflight)             # the timed steps
    loop.run(2, 1024, gather=False, first=100)       # the 1024-horizon shard figure: solves only, no gather
    if rank == 0:
        q.put((gB, scaling, prefix, hi - lo, [(s, W.tolist(), S.tolist()) for s, W, S in log]))
    dist.destroy_process_group()


def test_bench_step_loop_gloo_equals_single_process():
    """bench.py's step loop at world size 2 (gloo): C5's 8192 horizons sharded 4096 + 4096, 4 steps in flight,
    each finished step's per-slot solutions gathered to rank 0 in step order.  Every gathered result has the 8192
    rows of a single-process run of that step, bit for bit, and the labels are C5's strong scaling."""
    import numpy as np

    from mpc_fatigue_amd import problems as PR

    world, K, inflight = 2, 6, 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_steploop_worker, args=(r, world, port, q, K, inflight)) for r in range(world)]
    for p in procs:
        p.start()
    gB, scaling, prefix, shard0, log = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert (gB, scaling, shard0) == (8192, "strong", 4096)
    assert prefix == "C5: 8192 horizons in total over 2 GPU(s), "
    assert [s for s, _, _ in log] == list(range(inflight + K))  # every step gathered once, in order
    Q0 = PR.pilz6_batch_q0(gB, seed=0)
    for s, W, S in log:
        W = np.array(W)
        assert W.shape == (8192, 7)
        np.testing.assert_array_equal(W[:, :6], torch.sin(torch.from_numpy(Q0) * (s + 1)).numpy())
        assert (W[:, 6] == s).all() and S == [s % 3] * 8192
    # the default (weak) workload: every GPU its own batch
    import bench
    assert bench.workload_plan(8192, False, 8) == (65536, "weak", "")
