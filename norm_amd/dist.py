"""Block striping across GPUs: one process per GPU, no data-path collective.

FEC blocks are independent, so rank r of W owns the contiguous block range
[r*B/W, (r+1)*B/W) of a batch and encodes/repairs it on its own GPU.  The process group
(RCCL "nccl" on GPUs, "gloo" on CPU for tests) is only used for the barrier and the
max-over-ranks timing of the benchmark.
"""
import os


def block_range(total, world, rank):
    """Contiguous [lo, hi) share of `total` blocks for `rank` (sizes differ by at most 1)."""
    if world <= 0 or not (0 <= rank < world):
        raise ValueError("bad world/rank")
    lo = total * rank // world
    hi = total * (rank + 1) // world
    return lo, hi


def shard(blocks, world, rank, strong=False):
    """(first_block, nblocks) of `rank` for a benchmark run.

    weak (default): every rank owns `blocks` blocks of its own, [rank*blocks, (rank+1)*blocks):
    the per-GPU work stays fixed as the world grows.
    strong: `blocks` is the fixed total, split into contiguous ranges by block_range."""
    if strong:
        lo, hi = block_range(blocks, world, rank)
        return lo, hi - lo
    if world <= 0 or not (0 <= rank < world):
        raise ValueError("bad world/rank")
    return rank * blocks, blocks


def env_ranks():
    """(world, rank, local_rank) from the torchrun environment (defaults: single process)."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def max_over_ranks(value, device=None):
    """Max of a float over all ranks (identity without an initialised process group)."""
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()):
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device or "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
