"""Block striping across GPUs: one process per GPU, no data-path collective.

FEC blocks are independent, so rank r of W owns the contiguous block range
[r*B/W, (r+1)*B/W) of a batch and encodes/repairs it on its own GPU.  The process group
(RCCL "nccl" on GPUs, "gloo" on CPU for tests) is only used for the barrier and the
max-over-ranks timing of the benchmark.
"""
import os
import socket
import subprocess
import sys


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


def free_port():
    """A TCP port on 127.0.0.1 that was free a moment ago (rendezvous of self-launched ranks)."""
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def plan_launch(gpus):
    """How a benchmark started with `--gpus N` gets its ranks.

    Returns N when this process must start N rank processes itself (no launcher set
    WORLD_SIZE and N > 1), else 0: the process is one rank of an existing launch (torchrun)
    or a single-GPU run.  Under a launcher an explicit --gpus must equal WORLD_SIZE, so a
    driver never records a one-GPU number as an N-GPU one."""
    world = os.environ.get("WORLD_SIZE")
    if world is None:
        return gpus if gpus and gpus > 1 else 0
    if gpus is not None and int(world) != gpus:
        raise SystemExit(f"--gpus {gpus} but WORLD_SIZE={world}: one rank per GPU expected")
    return 0


def launch_local_ranks(n, script, argv, extra_env=None):
    """Start `n` ranks of `script` on this node (RANK = LOCAL_RANK = r, WORLD_SIZE = n,
    rendezvous on 127.0.0.1), wait for all of them and return the worst exit status.  The
    caller must not have touched the GPU: the ranks are child processes, never an exec."""
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        env.update(extra_env or {})
        procs.append(subprocess.Popen([sys.executable, script] + list(argv), env=env))
    # a rank that fails would leave the others waiting at a barrier: stop them
    import time

    while True:
        codes = [p.poll() for p in procs]
        bad = [c for c in codes if c not in (None, 0)]
        if bad:
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            for p in procs:
                try:
                    p.wait(timeout=30)
                except subprocess.TimeoutExpired:
                    p.kill()
                    p.wait()
            return bad[0]
        if all(c == 0 for c in codes):
            return 0
        time.sleep(0.05)
