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


# ---- bench.py --gpus N: the launch itself (--gpus must produce N ranks) ----
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(args, env_extra=None, timeout=300):
    import json
    import subprocess
    import sys

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                       timeout=timeout, env=env, cwd=ROOT)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    return r, [json.loads(ln) for ln in lines]


@pytest.mark.parametrize("n", [1, 2, 3])
def test_bench_gpus_flag_starts_n_ranks(n):
    """Without a launcher `bench.py --gpus N` starts N rank processes; rank 0 alone prints, and
    the line counts every rank that joined the group (the dry run's all-reduce of ones)."""
    r, out = _bench(["--gpus", str(n), "--dry-run", "--steps", "2", "--warmup", "1", "--blocks", "256"])
    assert r.returncode == 0, r.stderr[-2000:]
    assert len(out) == 1, r.stdout
    assert out[0]["n_gpus"] == n and out[0]["world_size"] == n and out[0]["steps"] == 2


def test_bench_gpus_must_match_launcher_world():
    r, out = _bench(["--gpus", "4", "--dry-run"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"}, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr and not out


def test_plan_launch():
    from norm_amd.dist import plan_launch

    old = {k: os.environ.pop(k, None) for k in ("WORLD_SIZE",)}
    try:
        assert plan_launch(None) == 0 and plan_launch(1) == 0 and plan_launch(8) == 8
        os.environ["WORLD_SIZE"] = "8"
        assert plan_launch(8) == 0 and plan_launch(None) == 0
        with pytest.raises(SystemExit):
            plan_launch(1)
    finally:
        os.environ.pop("WORLD_SIZE", None)
        if old["WORLD_SIZE"] is not None:
            os.environ["WORLD_SIZE"] = old["WORLD_SIZE"]


def test_bench_c5_dry_run_pinned_budget():
    """tools/bench_c5.py --gpus N --dry-run: N ranks on gloo, contiguous disjoint shares covering
    the stream, and a page-locked budget per rank (4 GB at N > 1) instead of the 26.8 GB share."""
    import json
    import subprocess
    import sys

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "bench_c5.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    out = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(out) == 1 and out[0]["n_gpus"] == 2
    ranks, pinned = out[0]["ranks"], out[0]["pinned"]
    assert [x["first"] for x in ranks] == [0, 131072]
    assert all(sum(x["blocks"].values()) == 131072 for x in ranks)
    assert all(0 < b <= 4_000_000_000 for b in pinned["per_rank_bytes"])
    assert pinned["total_bytes"] == sum(pinned["per_rank_bytes"]) < pinned["share_bytes_total"]
    for x in ranks:
        assert all(0 < x["pinned_blocks"][n] <= x["blocks"][n] for n in x["blocks"])
