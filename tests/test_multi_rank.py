"""N>1 path on CPU: world_size-2 gloo process group, block striping and max-over-ranks.

The GPU kernels cannot run here, so each rank checks the striping contract with the oracle
as the per-shard computation: the concatenation of the shards' parity equals the parity of
the whole batch (checksum of checksums), shards are disjoint and cover the batch, and the
timing reduction returns the maximum."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from norm_amd.dist import block_range, shard


def test_block_range_partition():
    for total in (0, 1, 7, 65536, 1_000_003):
        for world in (1, 2, 3, 8):
            ranges = [block_range(total, world, r) for r in range(world)]
            assert ranges[0][0] == 0 and ranges[-1][1] == total
            for (a, b), (c, d) in zip(ranges, ranges[1:]):
                assert b == c and b >= a
            sizes = [b - a for a, b in ranges]
            assert max(sizes) - min(sizes) <= 1


def test_shard_weak_and_strong():
    # weak: every rank its own fixed share; strong: one fixed total split contiguously
    assert [shard(100, 4, r) for r in range(4)] == [(0, 100), (100, 100), (200, 100), (300, 100)]
    got = [shard(65536, 8, r, strong=True) for r in range(8)]
    assert sum(n for _, n in got) == 65536 and got[0][0] == 0
    assert all(a + n == b for (a, n), (b, _) in zip(got, got[1:]))
    with pytest.raises(ValueError):
        shard(10, 2, 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q, strong=True):
    import hashlib

    import torch.distributed as dist

    from norm_amd.dist import env_ranks, max_over_ranks
    from oracle import pyoracle as orc

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    k, m, vec, total = 16, 4, 48, 10
    # the partition bench.py --strong uses (total fixed) or its default weak one (total/world each)
    w, r, _ = env_ranks()
    lo, nb = shard(total if strong else total // world, w, r, strong)
    hi = lo + nb
    blocks = orc.make_blocks(k, m, vec, hi - lo, first_block=lo)
    orc.encode_blocks(orc.RS8, k, m, vec, blocks)
    digest = hashlib.sha256(blocks[:, k:].tobytes()).hexdigest()
    gathered = [None] * world
    dist.all_gather_object(gathered, (lo, hi, digest))
    mx = max_over_ranks(1.0 + rank)
    dist.barrier()
    dist.destroy_process_group()
    q.put((rank, gathered, mx))


@pytest.mark.parametrize("strong", [True, False])
def test_two_rank_gloo_striping(orc, strong):
    import hashlib

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, strong)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    k, m, vec, total = 16, 4, 48, 10
    whole = orc.encode_blocks(orc.RS8, k, m, vec, orc.make_blocks(k, m, vec, total))
    for rank, gathered, mx in results:
        assert mx == 2.0
        assert [g[:2] for g in gathered] == [block_range(total, world, r) for r in range(world)]
        for lo, hi, digest in gathered:
            assert digest == hashlib.sha256(whole[lo:hi, k:].tobytes()).hexdigest()
