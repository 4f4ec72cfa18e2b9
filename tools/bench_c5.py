"""BASELINE C5: mixed RS8/RS16 block stream striped over the GPUs of one node, segments in pinned
host memory (NORM's socket buffers), H2D / compute / D2H overlapped.

    python tools/bench_c5.py [--steps 2]                       # one GPU: 131,072 blocks (1M / 8)
    python tools/bench_c5.py --gpus 8                           # 8 rank processes, no launcher
    torchrun --nproc-per-node 8 tools/bench_c5.py               # weak: 131,072 blocks per GPU = C5
    torchrun --nproc-per-node N tools/bench_c5.py --strong      # strong: 1,048,576 blocks over N GPUs

Block b of the stream is RS16 (k=400, m=100, vec=1400: the fecTest shape) when
splitmix64(seed ^ b) % 8 == 0, otherwise RS8 (k=64, m=32, vec=1400).  Rank r owns the contiguous
block range [r*B/W, (r+1)*B/W) (FEC blocks are independent: no collective on the data path).
One step = encode every block, then repair 16 (RS8) / 50 (RS16) random source erasures per
block.  The RS8 and RS16 sub-streams run concurrently from two host threads, each through the
codec's pinned-staging pipeline (nfec_encode_host / nfec_decode_host).

Reported as one JSON line in bench.py's schema: value = host-resident GiB/s (source bytes
through encode + decode, all ranks / max-over-ranks time), plus the device-resident GiB/s of the
same mix with the blocks already in HBM (the two sub-streams on two HIP streams: 43.2 ms per
one-GPU step against 44.0 on one stream, profiles/r06/c5_streams/), and a device round trip
after the timing (erased source zeroed, repaired, compared).

Page-locked memory: a rank's whole share is 26.8 GB (114,726 RS8 x 96 x 1400 + 16,346 RS16 x
500 x 1400), 215 GB over 8 ranks.  At N = 1 the whole share is pinned; at N > 1 the host-resident
timing runs on the first blocks of each sub-stream within --pinned-gb per rank (default 4 GB,
32 GB over 8 ranks), the device-resident timing on the whole share.  The line reports the pinned
bytes per rank and in total.  --dry-run rehearses the launch, the per-rank plan and the pinned
budget on the CPU (gloo, no GPU, no FEC work).
"""
import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SEED = 0x4E4F524D
RS8 = (64, 32, 1400, 16)     # k, m, vec, source erasures
RS16 = (400, 100, 1400, 50)


def splitmix64(x):
    import numpy as np

    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=None,
                   help="GPUs = ranks; without a launcher N > 1 starts N rank processes (bench.py's rule)")
    p.add_argument("--blocks", type=int, default=0,
                   help="blocks per GPU (weak; default 1M / 8), or in total with --strong (default 1M)")
    p.add_argument("--strong", action="store_true", help="a fixed total split over the ranks")
    p.add_argument("--steps", type=int, default=2)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--serial", action="store_true", help="run the RS8 and RS16 sub-streams one after the other")
    p.add_argument("--pinned-gb", type=float, default=0.0,
                   help="page-locked bytes per rank for the host-resident timing (0: the whole share at N = 1, "
                        "4 GB at N > 1)")
    p.add_argument("--dry-run", action="store_true",
                   help="CPU rehearsal: launch, per-rank plan and pinned budget (gloo; no GPU, no FEC work)")
    p.add_argument("--share-gpu", action="store_true",
                   help="one-GPU rehearsal of the N-rank path (bench.py's): every rank on cuda:0, gloo collectives")
    a = p.parse_args()
    from norm_amd.dist import launch_local_ranks, plan_launch

    n = plan_launch(a.gpus)
    if n:
        sys.exit(launch_local_ranks(n, os.path.abspath(__file__), sys.argv[1:]))
    import numpy as np
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.dry_run:
        return dry_run(a, world, rank)
    share = a.share_gpu and world > 1
    if share:
        local = 0  # every rank on cuda:0; RCCL wants one rank per device, so gloo carries the reductions
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist

        if share:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    cdev = torch.device("cpu") if share else dev  # the collectives' tensors
    import norm_amd as na

    pl = plan(a, world, rank)
    total, lo, counts, pinned = pl["total"], pl["first"], pl["blocks"], pl["pinned_blocks"]

    jobs = []
    for name, (k, m, vec, er), n, enc_c, dec_c in (("RS8", RS8, counts["RS8"], na.NormEncoderRS8, na.NormDecoderRS8),
                                                  ("RS16", RS16, counts["RS16"], na.NormEncoderRS16, na.NormDecoderRS16)):
        if n == 0:
            continue
        enc, dec = enc_c(device=local), dec_c(device=local)
        assert enc.Init(k, m, vec) and dec.Init(k, m, vec)
        # synthetic source generated in HBM (the whole share: the device-resident timing); the
        # first `hn` blocks are also copied to pinned host memory (the host-resident timing)
        d = torch.zeros((n, k + m, vec), dtype=torch.uint8, device=dev)
        na.fill_blocks(d, k, vec, SEED ^ (0x16 if name == "RS16" else 0x8), first_block=lo)
        hn = pinned[name]
        host = torch.empty((hn, k + m, vec), dtype=torch.uint8, pin_memory=True)
        host.copy_(d[:hn])
        locs, cnts = na.make_erasures(n, k, er, SEED, m, first_block=lo)
        jobs.append(dict(name=name, k=k, m=m, vec=vec, er=er, n=n, hn=hn, enc=enc, dec=dec, host=host, dev=d,
                         hnp=host.numpy(), locs=locs[:hn].cpu().numpy().view(np.uint16),
                         cnts=cnts[:hn].cpu().numpy().view(np.uint16), dlocs=locs, dcnts=cnts))
    torch.cuda.synchronize()

    def host_job(j):
        t0 = time.perf_counter()
        j["enc"].encode_blocks_host(j["hnp"])
        t1 = time.perf_counter()
        st = j["dec"].decode_blocks_host(j["hnp"], j["locs"], j["cnts"])
        t2 = time.perf_counter()
        j["ok"] = bool((st == j["er"]).all())
        j["host_enc_s"], j["host_dec_s"] = t1 - t0, t2 - t1

    def host_step():
        if a.serial:
            for j in jobs:
                host_job(j)
            return
        th = [threading.Thread(target=host_job, args=(j,)) for j in jobs]
        for t in th:
            t.start()
        for t in th:
            t.join()

    def barrier():
        if dist is not None:
            dist.barrier()

    def max_time(t):
        if dist is None:
            return t
        x = torch.tensor([t], dtype=torch.float64, device=cdev)
        dist.all_reduce(x, op=dist.ReduceOp.MAX)
        return float(x.item())

    for _ in range(a.warmup):
        host_step()
    barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        host_step()
    barrier()
    host_s = max_time((time.perf_counter() - t0) / a.steps)
    host_ok = all(j["ok"] for j in jobs)

    # light round-trip check on a sample: erase, repair through the host path, compare
    sample_ok = True
    for j in jobs:
        n = min(64, j["hn"])
        keep = j["hnp"][:n].copy()
        rx = keep.copy()
        for b in range(n):
            for s in j["locs"][b, :j["cnts"][b]]:
                rx[b, s] = 0
        st = j["dec"].decode_blocks_host(rx, j["locs"][:n].copy(), j["cnts"][:n].copy())
        sample_ok &= bool(np.array_equal(rx, keep)) and bool((st == j["er"]).all())

    # device-resident rate of the same mix (blocks in HBM): the RS8 and RS16 sub-streams on two
    # HIP streams, as the host-resident step runs them from two threads (--serial: one stream,
    # one sub-stream after the other)
    dev_jobs = []
    main_s = torch.cuda.current_stream(dev)
    for i, j in enumerate(jobs):
        del j["host"], j["hnp"]  # the pinned copies are done with
        s = main_s if (i == 0 or a.serial) else torch.cuda.Stream(dev)
        dev_jobs.append((j, j["dev"], torch.empty(j["n"], dtype=torch.int32, device=dev), s))

    def dev_step():
        start = torch.cuda.Event()
        start.record(main_s)
        for j, d, st, s in dev_jobs:
            if s is not main_s:
                s.wait_event(start)
            j["enc"].encode_blocks(d, stream=s)
            j["dec"].decode_blocks(d, j["dlocs"], j["dcnts"], status=st, stream=s)
        for j, d, st, s in dev_jobs:
            if s is not main_s:
                done = torch.cuda.Event()
                done.record(s)
                main_s.wait_event(done)

    dev_step()
    torch.cuda.synchronize(dev)
    barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        dev_step()
    torch.cuda.synchronize(dev)
    barrier()
    dev_s = max_time((time.perf_counter() - t0) / a.steps)

    # device round trip after the timed steps: every sub-stream's erased source zeroed, repaired on
    # its own stream (concurrently, as timed), compared with the bytes before
    dev_ok = True
    for j, d, st, s in dev_jobs:
        j["keep"] = d[:, :j["k"]].clone()
        na.zero_erasures(d, j["dlocs"], j["dcnts"], j["vec"], stream=main_s)
    torch.cuda.synchronize(dev)
    for j, d, st, s in dev_jobs:
        j["dec"].decode_blocks(d, j["dlocs"], j["dcnts"], status=st, stream=s)
    torch.cuda.synchronize(dev)
    for j, d, st, s in dev_jobs:
        dev_ok &= bool(torch.equal(d[:, :j["k"]], j["keep"])) and bool((st == j["er"]).all())
        del j["keep"]

    def sum_ranks(v):
        t = torch.tensor([float(v)], dtype=torch.float64, device=cdev)
        if dist is not None:
            dist.all_reduce(t)
        return float(t.item())

    src_all = sum_ranks(sum(j["k"] * j["vec"] * j["n"] for j in jobs))        # device-resident step
    src_host = sum_ranks(sum(j["k"] * j["vec"] * j["hn"] for j in jobs))      # host-resident step
    pinned_all = sum_ranks(pl["pinned_bytes"])
    if rank == 0:
        print(json.dumps({
            "metric": "FEC encode+erasure-decode GiB/s (host-resident, pinned H2D/D2H), C5 mixed RS8/RS16 stream",
            "value": round(src_host / host_s / 2**30, 2), "unit": "GiB/s", "n_gpus": world,
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(host_s * 1e3, 1),
            "higher_is_better": True, "scaling": "strong" if a.strong else "weak", "vs_baseline": None,
            "dtype": "u8", "data": "synthetic (splitmix64 source segments, reference generators)",
            "config": {"workload": "C5 mixed RS8(64,32)/RS16(400,100) stream, vec=1400, pinned host segments",
                       "blocks_total": total, "rank0_blocks": counts,
                       "parallelism": f"block-striped x{world} (no collective)"},
            "pinned": {"rank0_blocks": pinned, "rank0_bytes": pl["pinned_bytes"], "total_bytes": int(pinned_all),
                       "budget_bytes_per_rank": pl["budget_bytes"],
                       "note": "host-resident timing on these first blocks of each sub-stream (page-locked); "
                               "device-resident timing on every block of the share"},
            "device_resident": {"value": round(src_all / dev_s / 2**30, 2), "unit": "GiB/s",
                                "ms_per_step": round(dev_s * 1e3, 2),
                                "streams": 1 if a.serial else len(dev_jobs)},
            "status_ok": host_ok, "sample_round_trip_ok": sample_ok, "device_round_trip_ok": dev_ok,
            "rank0_host_s": {j["name"]: [round(j["host_enc_s"], 3), round(j["host_dec_s"], 3)] for j in jobs},
            "note": "one step = encode + 16 (RS8) / 50 (RS16) source-erasure repair of every block; "
                    "GiB/s counts source bytes, all ranks / max-over-ranks time",
            **({"rehearsal": f"{world} ranks sharing cuda:0 over gloo (--share-gpu), not a scaling number"}
               if share else {}),
        }), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def plan(a, world, rank):
    """This rank's share of the stream (contiguous block range, split into its RS8 and RS16
    sub-streams) and how much of it is pinned for the host-resident timing."""
    import numpy as np

    from norm_amd.dist import shard

    per = a.blocks or ((1 << 20) if a.strong else (1 << 20) // 8)
    first, nmine = shard(per, world, rank, a.strong)
    ids = np.arange(first, first + nmine, dtype=np.uint64)
    is16 = (splitmix64(np.uint64(SEED) ^ ids) % np.uint64(8)) == 0
    blocks = {"RS8": int((~is16).sum()), "RS16": int(is16.sum())}
    bpb = {"RS8": (RS8[0] + RS8[1]) * RS8[2], "RS16": (RS16[0] + RS16[1]) * RS16[2]}
    share = sum(blocks[n] * bpb[n] for n in blocks)
    budget = int(a.pinned_gb * 1e9) if a.pinned_gb > 0 else (share if world == 1 else int(4e9))
    frac = min(1.0, budget / max(share, 1))
    pinned = {n: (blocks[n] if frac >= 1.0 else min(blocks[n], max(1, int(blocks[n] * frac)))) if blocks[n] else 0
              for n in blocks}
    return {"total": per if a.strong else per * world, "first": first, "blocks": blocks, "pinned_blocks": pinned,
            "pinned_bytes": sum(pinned[n] * bpb[n] for n in pinned), "share_bytes": share, "budget_bytes": budget}


def dry_run(a, world, rank):
    """The launch, the per-rank plans and the pinned budget on the CPU (gloo), one JSON line."""
    import torch
    import torch.distributed as dist

    if world > 1:
        dist.init_process_group("gloo")
    mine = plan(a, world, rank)
    plans = [mine]
    if world > 1:
        plans = [None] * world
        dist.all_gather_object(plans, mine)
    if rank == 0:
        print(json.dumps({
            "metric": "FEC encode+erasure-decode GiB/s (host-resident, pinned H2D/D2H), C5 mixed RS8/RS16 stream",
            "value": None, "n_gpus": len(plans), "dry_run": True, "world_size": world,
            "config": {"blocks_total": plans[0]["total"], "parallelism": f"block-striped x{world} (no collective)"},
            "pinned": {"per_rank_bytes": [p["pinned_bytes"] for p in plans],
                       "total_bytes": sum(p["pinned_bytes"] for p in plans),
                       "share_bytes_total": sum(p["share_bytes"] for p in plans),
                       "budget_bytes_per_rank": mine["budget_bytes"]},
            "ranks": [{"first": p["first"], "blocks": p["blocks"], "pinned_blocks": p["pinned_blocks"]} for p in plans],
        }), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
