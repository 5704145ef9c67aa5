"""Sharding of independent gates over ranks: no data-path collective.

Gates are independent, so each rank (one process per GPU) owns a contiguous slice of the
global batch and runs it on its own device context (keys replicated).  The only collective
is a timing reduction (max of the per-rank elapsed time) used by bench.py.
"""


def shard_range(total, rank, world):
    """Contiguous slice [lo, hi) of `total` independent gates owned by `rank`."""
    if world <= 0 or not (0 <= rank < world) or total < 0:
        raise ValueError("bad shard arguments")
    per, extra = divmod(total, world)
    lo = rank * per + min(rank, extra)
    return lo, lo + per + (1 if rank < extra else 0)


def max_over_ranks(value, device=None):
    """max of a float over all ranks (torch.distributed; identity when not initialised)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def weak_scaling_value(batch_per_rank, world, steps, elapsed_max):
    """whole-job gates/s: every rank processed batch_per_rank gates per step."""
    return batch_per_rank * world * steps / elapsed_max
