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


def gather_solutions(w, status, rank: int, world: int, dst: int = 0, total: int | None = None):
    """Gather every rank's solution block to `dst`; returns (W, S) on dst, (None, None) elsewhere.

    Shards may differ in size (shard_range of a total not divisible by world): the ranks first
    all-gather their row counts, so every rank knows every block's size and the same total; each
    rank pads its block to the largest one, the gather moves equal blocks, and dst drops the
    padding.  If `total` is given and the gathered row counts do not match shard_range(total),
    EVERY rank raises the same ValueError (no rank is left blocked in the gather).
    """
    import torch
    import torch.distributed as dist

    if world == 1:
        return w, status
    rows = w.shape[0]
    cnt = torch.tensor([rows], dtype=torch.int64, device=w.device)
    got = [torch.empty_like(cnt) for _ in range(world)]
    dist.all_gather(got, cnt)
    sizes = [int(c.item()) for c in got]
    if total is not None:
        want = [shard_range(total, world, r)[1] - shard_range(total, world, r)[0] for r in range(world)]
        if sizes != want:
            raise ValueError(f"shard rows {sizes} do not match shard_range({total}, {world}) = {want}")
    m = max(sizes)
    if rows < m:
        w = torch.cat([w, w.new_zeros((m - rows,) + tuple(w.shape[1:]))])
        status = torch.cat([status, status.new_full((m - rows,), -1)])
    ws = [torch.empty_like(w) for _ in range(world)] if rank == dst else None
    ss = [torch.empty_like(status) for _ in range(world)] if rank == dst else None
    dist.gather(w.contiguous(), ws, dst=dst)
    dist.gather(status.contiguous(), ss, dst=dst)
    if rank == dst:
        return torch.cat([x[:n] for x, n in zip(ws, sizes)]), torch.cat([x[:n] for x, n in zip(ss, sizes)])
    return None, None
