"""Stripe sharding across GPUs: stripes are independent, so a batch is split into contiguous
ranges, one per rank, with no data-path collective.  torch.distributed (RCCL on ROCm) only carries the
benchmark's barriers and the max-over-ranks elapsed time."""


def stripe_range(num_stripes, rank, world):
    """Contiguous range [lo, hi) of rank `rank`: g * ceil(S/G) .. min(S, (g+1) * ceil(S/G))."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    per = (num_stripes + world - 1) // world
    lo = min(num_stripes, rank * per)
    return lo, min(num_stripes, lo + per)


def max_over_ranks(value, dist=None, device="cpu"):
    """MAX all-reduce of a float (the slowest rank defines the job's time)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return float(value)
    import torch
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
