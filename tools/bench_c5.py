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
same mix with the blocks already in HBM.
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
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    import norm_amd as na

    from norm_amd.dist import shard

    per = a.blocks or ((1 << 20) if a.strong else (1 << 20) // 8)
    first, nmine = shard(per, world, rank, a.strong)
    total = per if a.strong else per * world
    lo, hi = first, first + nmine
    ids = np.arange(lo, hi, dtype=np.uint64)
    is16 = (splitmix64(np.uint64(SEED) ^ ids) % np.uint64(8)) == 0
    counts = {"RS8": int((~is16).sum()), "RS16": int(is16.sum())}

    jobs = []
    for name, (k, m, vec, er), n, enc_c, dec_c in (("RS8", RS8, counts["RS8"], na.NormEncoderRS8, na.NormDecoderRS8),
                                                  ("RS16", RS16, counts["RS16"], na.NormEncoderRS16, na.NormDecoderRS16)):
        if n == 0:
            continue
        enc, dec = enc_c(device=local), dec_c(device=local)
        assert enc.Init(k, m, vec) and dec.Init(k, m, vec)
        host = torch.empty((n, k + m, vec), dtype=torch.uint8, pin_memory=True)
        # synthetic source generated on the GPU in chunks, then moved to pinned host memory
        chunk = max(1, (2 << 30) // ((k + m) * vec))
        for b0 in range(0, n, chunk):
            nb = min(chunk, n - b0)
            d = torch.zeros((nb, k + m, vec), dtype=torch.uint8, device=dev)
            na.fill_blocks(d, k, vec, SEED ^ (0x16 if name == "RS16" else 0x8), first_block=lo + b0)
            host[b0:b0 + nb].copy_(d)
            del d
        locs, cnts = na.make_erasures(n, k, er, SEED, m, first_block=lo)
        jobs.append(dict(name=name, k=k, m=m, vec=vec, er=er, n=n, enc=enc, dec=dec, host=host,
                         hnp=host.numpy(), locs=locs.cpu().numpy().view(np.uint16), cnts=cnts.cpu().numpy().view(np.uint16),
                         dlocs=locs, dcnts=cnts))
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
        x = torch.tensor([t], dtype=torch.float64, device=dev)
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
        n = min(64, j["n"])
        keep = j["hnp"][:n].copy()
        rx = keep.copy()
        for b in range(n):
            for s in j["locs"][b, :j["cnts"][b]]:
                rx[b, s] = 0
        st = j["dec"].decode_blocks_host(rx, j["locs"][:n].copy(), j["cnts"][:n].copy())
        sample_ok &= bool(np.array_equal(rx, keep)) and bool((st == j["er"]).all())

    # device-resident rate of the same mix (blocks in HBM)
    dev_jobs = []
    for j in jobs:
        d = j["host"].to(dev)
        dev_jobs.append((j, d, torch.empty(j["n"], dtype=torch.int32, device=dev)))
    stream = torch.cuda.current_stream(dev)

    def dev_step():
        for j, d, st in dev_jobs:
            j["enc"].encode_blocks(d, stream=stream)
            j["dec"].decode_blocks(d, j["dlocs"], j["dcnts"], status=st, stream=stream)

    dev_step()
    torch.cuda.synchronize(dev)
    barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        dev_step()
    torch.cuda.synchronize(dev)
    barrier()
    dev_s = max_time((time.perf_counter() - t0) / a.steps)

    src_rank = sum(j["k"] * j["vec"] * j["n"] for j in jobs)
    src_all = torch.tensor([float(src_rank)], dtype=torch.float64, device=dev)
    if dist is not None:
        dist.all_reduce(src_all)
    src_all = float(src_all.item())
    if rank == 0:
        print(json.dumps({
            "metric": "FEC encode+erasure-decode GiB/s (host-resident, pinned H2D/D2H), C5 mixed RS8/RS16 stream",
            "value": round(src_all / host_s / 2**30, 2), "unit": "GiB/s", "n_gpus": world,
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(host_s * 1e3, 1),
            "higher_is_better": True, "scaling": "strong" if a.strong else "weak", "vs_baseline": None,
            "dtype": "u8", "data": "synthetic (splitmix64 source segments, reference generators)",
            "config": {"workload": "C5 mixed RS8(64,32)/RS16(400,100) stream, vec=1400, pinned host segments",
                       "blocks_total": total, "rank0_blocks": counts,
                       "parallelism": f"block-striped x{world} (no collective)"},
            "device_resident": {"value": round(src_all / dev_s / 2**30, 2), "unit": "GiB/s",
                                "ms_per_step": round(dev_s * 1e3, 2)},
            "status_ok": host_ok, "sample_round_trip_ok": sample_ok,
            "rank0_host_s": {j["name"]: [round(j["host_enc_s"], 3), round(j["host_dec_s"], 3)] for j in jobs},
            "note": "one step = encode + 16 (RS8) / 50 (RS16) source-erasure repair of every block; "
                    "GiB/s counts source bytes, all ranks / max-over-ranks time",
        }), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
