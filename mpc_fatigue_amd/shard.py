"""Multi-GPU sharding of a batch of independent horizons.

The batched configuration (BASELINE.json C5: 8192 Pilz-6DOF horizons over
8 x MI355X) has no coupling between problems, so each rank solves a contiguous
shard with no data-path communication; the only collective is the final
gather of solutions (and convergence flags) to rank 0 over RCCL/xGMI.
One process per GPU, launched by torch.distributed.run.
"""
from __future__ import annotations


def shard_range(total: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous [lo, hi) of `total` problems owned by `rank` (balanced to within one)."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError("bad world/rank")
    base, extra = divmod(total, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def gather_solutions(w, status, rank: int, world: int, dst: int = 0):
    """Gather every rank's solution block to `dst`; returns (W, S) on dst, (None, None) elsewhere.

    Shards must have equal size (the bench uses batch-per-GPU shards).
    """
    import torch
    import torch.distributed as dist

    if world == 1:
        return w, status
    ws = [torch.empty_like(w) for _ in range(world)] if rank == dst else None
    ss = [torch.empty_like(status) for _ in range(world)] if rank == dst else None
    dist.gather(w, ws, dst=dst)
    dist.gather(status, ss, dst=dst)
    if rank == dst:
        return torch.cat(ws), torch.cat(ss)
    return None, None
