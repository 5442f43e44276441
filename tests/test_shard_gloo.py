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


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = shard_range(8 * world, world, rank)
    w = torch.arange(lo * 5, hi * 5, dtype=torch.float64).reshape(hi - lo, 5)
    st = torch.full((hi - lo,), rank, dtype=torch.int32)
    W, S = gather_solutions(w, st, rank, world)
    if rank == 0:
        q.put((W.numpy().tolist(), S.numpy().tolist()))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_gather_solutions_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    W, S = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    import numpy as np
    W = np.array(W)
    assert W.shape == (8 * world, 5)
    np.testing.assert_array_equal(W.reshape(-1), np.arange(8 * world * 5))
    assert S == [r for r in range(world) for _ in range(8)]
