"""Headline benchmark: RS8 k=64/m=32, 1400-byte segments, encode + 16-erasure decode, in HBM.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

`--gpus N` without a launcher starts N rank processes of this script itself (one per GPU,
before anything touches the GPU); under a launcher --gpus must equal WORLD_SIZE.  `--dry-run`
exercises the same launch, barrier, max-over-ranks timing and JSON line on the CPU (gloo, no
GPU, no FEC work) for the launcher's tests.

One step = one pass of the hot path over one batch resident in HBM: parity generation for
65,536 blocks (BASELINE C2) followed by erasure repair of 16 random source symbols in each of
them (C3).  Inputs are synthetic (splitmix64 segments generated on the GPU), the generator is
the reference's RS8(64,32) matrix.  For N > 1 (torchrun, one rank per GPU) every rank owns its
own 65,536 blocks (weak scaling: FEC blocks are independent, no data-path collective; the
process group only provides the barrier and the max-over-ranks timing).

value = k * vec * blocks_total / step_time  (source bytes through encode+decode, GiB/s),
the same formula as the CPU baseline; SURVEY.md 8d's "combined" figure,
2*k*vec*B / (t_enc + t_dec), counts each source byte twice and is exactly 2x this value.
--strong splits a fixed total of --blocks over the ranks instead (norm_amd/dist.py shard).  roofline = the encode kernel's
algorithmic HBM bytes per launch / its measured launch time vs 8 TB/s, for the step's dominant
kernel (the longer of the encode, (k+m)*vec per block, and the repair call, (k+e)*vec per block);
both halves are in the line.  After timing, one clean encode -> erase -> repair round trip from the
pristine source is compared byte for byte ("verified"; --no-verify skips it).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "FEC encode+erasure-decode GiB/s (device-resident), RS8 k=64/m=32 seg=1400B"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md); measured copy ~6300
VALU_PEAK = 7.86e13    # 256 CU x 4 SIMD x 32 lanes x 2.4 GHz, 32-bit bitwise ops (ubench: 76% reachable)


def encode_kernel_name(k, m, vec):
    """the kernel nfec_encode dispatches for this shape (nfec_api.cpp encode_device)"""
    if (k, m) not in ((64, 32), (64, 16), (64, 8)):
        return "gf8_matmul_kernel (RS8 encode, generic)"
    if vec % 8 == 0:
        return f"nfec::rs8_q4_enc_k{k}_m{m} (RS8 encode, 4 role waves sharing each column's transpose through LDS)"
    return f"nfec::rs8_enc_k{k}_m{m} (RS8 encode, compiler-allocated)"


def host_cores():
    """(cores this process can actually use, cores visible in its affinity mask).  A GPU box
    shows the whole machine's CPUs in the affinity mask while a cgroup quota (cpu.max) grants
    the job a share of them; threads beyond the share only time-slice."""
    visible = len(os.sched_getaffinity(0))
    usable = visible
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            quota, period = open(path).read().split()[:2]
            if quota != "max":
                usable = min(usable, max(1, int(int(quota) // int(period))))
        except (OSError, ValueError):
            pass
    return usable, visible


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=None,
                   help="GPUs = ranks (default 1, or WORLD_SIZE under a launcher)")
    p.add_argument("--dry-run", action="store_true",
                   help="CPU rehearsal of the multi-rank launch and reporting (gloo; no GPU, no FEC work)")
    p.add_argument("--share-gpu", action="store_true",
                   help="one-GPU rehearsal of the N-rank path: every rank runs the real workload on cuda:0 and "
                        "the collectives go over gloo (the line says so; never a scaling number)")
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--blocks", type=int, default=65536,
                   help="FEC blocks per GPU (weak scaling), or in total with --strong")
    p.add_argument("--strong", action="store_true",
                   help="strong scaling: --blocks is the fixed total, split over the ranks by block_range")
    p.add_argument("--k", type=int, default=64)
    p.add_argument("--m", type=int, default=32)
    p.add_argument("--vec", type=int, default=1400)
    p.add_argument("--erasures", type=int, default=16)
    p.add_argument("--cpu-blocks", type=int, default=4096)
    p.add_argument("--cpu-threads", type=int, default=0,
                   help="CPU-baseline threads (0 = every core this process may run on: the affinity mask, "
                        "capped by a cgroup CPU quota when one is set)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-verify", action="store_true",
                   help="skip the clean round trip after timing (by default the line carries 'verified': one "
                        "encode -> erase -> repair from the pristine source, every byte compared, as the "
                        "reference's fecTest does, fecTest.cpp:121-129)")
    p.add_argument("--host-steps", type=int, default=2,
                   help="also time K steps with blocks in pinned host memory (PCIe-inclusive, reported "
                        "under 'host_resident'; never the headline value; 0: skip)")
    p.add_argument("--host-blocks", type=int, default=0,
                   help="blocks per GPU in the pinned host batch of --host-steps (the first ones of the "
                        "device batch; 0: all of them at N = 1, a quarter per rank at N > 1)")
    return p.parse_args()


def dry_run(a, world, rank):
    """The multi-rank skeleton of main() on the CPU: gloo barrier, exactly K timed steps of a
    stand-in workload (a byte XOR-reduce of this rank's share, no FEC), max over ranks, one
    JSON line from rank 0 with n_gpus = the number of ranks that reported."""
    import numpy as np
    import torch
    import torch.distributed as dist

    if world > 1:
        dist.init_process_group("gloo")
    from norm_amd.dist import shard

    first, nb = shard(a.blocks, world, rank, a.strong)
    buf = np.random.default_rng(first).integers(0, 256, size=(min(nb, 64), a.k * a.vec), dtype=np.uint8)

    def barrier():
        if world > 1:
            dist.barrier()

    for _ in range(a.warmup):
        np.bitwise_xor.reduce(buf, axis=0)
    barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        np.bitwise_xor.reduce(buf, axis=0)
    elapsed = time.perf_counter() - t0
    barrier()
    ranks = 1
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        one = torch.ones(1)
        dist.all_reduce(one)
        ranks = int(one.item())
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "unit": "GiB/s", "n_gpus": ranks, "steps": a.steps,
                          "warmup": a.warmup, "ms_per_step": round(elapsed / a.steps * 1e3, 4),
                          "higher_is_better": True, "scaling": "strong" if a.strong else "weak",
                          "dry_run": True, "world_size": world,
                          "config": {"workload": "dry run: launch and reporting only, no FEC work",
                                     "blocks_total": a.blocks if a.strong else a.blocks * world}}))
    if world > 1:
        dist.destroy_process_group()


def main():
    a = parse()
    from norm_amd.dist import launch_local_ranks, plan_launch

    n = plan_launch(a.gpus)
    if n:
        # no launcher: one child process per GPU, started before this process touches the GPU
        sys.exit(launch_local_ranks(n, os.path.abspath(__file__), sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.dry_run:
        return dry_run(a, world, rank)
    import torch

    share = a.share_gpu and world > 1
    if world > torch.cuda.device_count() and not share:
        raise SystemExit(f"{world} ranks but {torch.cuda.device_count()} visible GPUs: one rank per GPU")
    dist = None
    if share:
        # rehearsal: the ranks share cuda:0, so RCCL (one rank per device) is out; gloo carries
        # the barrier and the max / min reductions on host tensors
        import torch.distributed as dist

        torch.cuda.set_device(0)
        dist.init_process_group("gloo")
    elif world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", local if world > 1 and not share else 0)
    cdev = torch.device("cpu") if share else dev  # where the collectives' tensors live

    from norm_amd import NormDecoderRS8, NormEncoderRS8, fill_blocks, make_erasures, stream_copy
    from norm_amd.dist import shard

    k, m, vec = a.k, a.m, a.vec
    seed = 0x4E4F524D
    enc, dec = NormEncoderRS8(device=dev.index), NormDecoderRS8(device=dev.index)
    assert enc.Init(k, m, vec) and dec.Init(k, m, vec)
    first, nb = shard(a.blocks, world, rank, a.strong)
    assert nb > 0, "every rank needs at least one block"
    blocks = torch.zeros((nb, k + m, vec), dtype=torch.uint8, device=dev)
    fill_blocks(blocks, k, vec, seed, first_block=first)
    locs, counts = make_erasures(nb, k, a.erasures, seed, m, first_block=first)
    status = torch.empty(nb, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)

    def step():
        enc.encode_blocks(blocks, stream=stream)
        dec.decode_blocks(blocks, locs, counts, status=status, stream=stream)

    def barrier():
        if dist is not None:
            dist.barrier()

    orig = None if a.no_verify else blocks[:, :k].clone()
    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize(dev)

    # ---- timed region: exactly K steps, barrier + sync on both sides ----
    # HIP events on the launch stream around each half of every step: the per-kernel durations
    # of the roofline come from the timed steps themselves, encode and repair interleaved as the
    # step runs them.  Recording one costs the stream ~5 us (a gap before the next kernel in the
    # kernel trace), so a step's end event is also the next step's start: 2K + 1 events, not 3K
    bounds = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps + 1)]
    mids = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps)]
    barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    bounds[0].record(stream)
    for i in range(a.steps):
        enc.encode_blocks(blocks, stream=stream)
        mids[i].record(stream)
        dec.decode_blocks(blocks, locs, counts, status=status, stream=stream)
        bounds[i + 1].record(stream)
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    barrier()
    elapsed = t1 - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # ---- per-kernel durations with HIP events on the launch stream ----
    def timed(fn, n):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(n):
            fn()
        e1.record(stream)
        e1.synchronize()
        return e0.elapsed_time(e1) / n  # ms per launch

    enc_ms = sum(bounds[i].elapsed_time(mids[i]) for i in range(a.steps)) / a.steps  # ms per launch
    dec_ms = sum(mids[i].elapsed_time(bounds[i + 1]) for i in range(a.steps)) / a.steps

    # achievable HBM rate on this box (report it beside the 8 TB/s spec): a 4 GiB
    # device-to-device copy by the library's streaming kernel (16 B per lane, non-temporal),
    # read + write bytes over its time; torch's copy_ (the runtime's blit kernel) beside it
    with torch.cuda.stream(stream):
        csrc = torch.empty(1 << 32, dtype=torch.uint8, device=dev)
        cdst = torch.empty_like(csrc)
        cdst.copy_(csrc)
    stream_copy(cdst, csrc, stream=stream)
    copy_ms = timed(lambda: stream_copy(cdst, csrc, stream=stream), 5)
    def blit():
        with torch.cuda.stream(stream):  # timed() brackets `stream`: the copy must run on it
            cdst.copy_(csrc)

    blit_ms = timed(blit, 5)
    copy_gbs = 2 * csrc.numel() / (copy_ms * 1e-3) / 1e9
    blit_gbs = 2 * csrc.numel() / (blit_ms * 1e-3) / 1e9
    del csrc, cdst

    host = None
    if a.host_steps > 0:
        import numpy as np

        # default: the whole batch on one GPU; a quarter per rank when several ranks pin host
        # memory at once (8 ranks x 8.8 GB of page-locked buffers is more than a node may grant)
        default_hb = nb if world == 1 else max(1, nb // 4)
        hb = min(nb, a.host_blocks) if a.host_blocks > 0 else default_hb
        hblocks = torch.empty((hb,) + tuple(blocks.shape[1:]), dtype=torch.uint8, pin_memory=True)
        hblocks.copy_(blocks[:hb])
        hnp = hblocks.numpy()
        hlocs = locs[:hb].cpu().numpy().view(np.uint16)
        hcounts = counts[:hb].cpu().numpy().view(np.uint16)

        def hstep():
            enc.encode_blocks_host(hnp)
            dec.decode_blocks_host(hnp, hlocs, hcounts)

        hstep()
        barrier()
        h0 = time.perf_counter()
        for _ in range(a.host_steps):
            hstep()
        h1 = time.perf_counter()
        barrier()
        he = h1 - h0
        if dist is not None:
            t = torch.tensor([he], dtype=torch.float64, device=cdev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            he = float(t.item())
        # the link's own rate on this box: pinned -> device DMA of 1 GiB (and back), the
        # ceiling of a path that must move every byte it codes over PCIe.  Per step the pipelines
        # move up 2 bytes per source byte (encode: the k source segments; decode: the k received
        # ones, nd surviving source + e substitute parity) and down (m + e) / k, so the
        # host-resident rate is bounded by h2d / 2 whatever the GPU does.
        lk_h = torch.empty(1 << 30, dtype=torch.uint8, pin_memory=True)
        lk_d = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
        with torch.cuda.stream(stream):
            lk_d.copy_(lk_h, non_blocking=True)
        def on_stream(dst, src):
            with torch.cuda.stream(stream):
                dst.copy_(src, non_blocking=True)

        h2d_ms = timed(lambda: on_stream(lk_d, lk_h), 3)
        d2h_ms = timed(lambda: on_stream(lk_h, lk_d), 3)
        # both directions at once, as the pipelines run them (parity and repaired segments come
        # down while the next chunk goes up): 512 MiB each way on two streams
        half = 1 << 29
        s2 = torch.cuda.Stream(device=dev)
        b0, b1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(dev)
        b0.record(stream)
        s2.wait_event(b0)
        for _ in range(3):
            with torch.cuda.stream(stream):
                lk_d[:half].copy_(lk_h[:half], non_blocking=True)
            with torch.cuda.stream(s2):
                lk_h[half:].copy_(lk_d[half:], non_blocking=True)
        stream.wait_stream(s2)
        b1.record(stream)
        b1.synchronize()
        bidir_gbs = 3 * half / (b0.elapsed_time(b1) * 1e-3) / 1e9  # per direction
        del lk_h, lk_d
        h2d_gbs = (1 << 30) / (h2d_ms * 1e-3) / 1e9
        up_per_src = 2.0
        down_per_src = (m + a.erasures) / k
        host = {
            "value": round(k * vec * hb * world / (he / a.host_steps) / 2**30, 2),
            "link_h2d_GBps": round(h2d_gbs, 1),
            "link_d2h_GBps": round((1 << 30) / (d2h_ms * 1e-3) / 1e9, 1),
            "link_bound_GiBps": round(h2d_gbs * 1e9 / up_per_src * world / 2**30, 2),
            "link_bidir_GBps_each_way": round(bidir_gbs, 1),
            # the step's own mix: (m + e) / k bytes per source byte come down (parity, repaired
            # segments) while 2 go up; while both directions run each gets the bidirectional
            # rate, the rest of the upload the one-way rate
            "link_mixed_bound_GiBps": round(world / ((down_per_src / bidir_gbs + (up_per_src - down_per_src) / h2d_gbs)
                                                     * 1e-9) / 2**30, 2),
            "blocks_per_gpu": hb,
            "unit": "GiB/s",
            "steps": a.host_steps,
            "ms_per_step": round(he / a.host_steps * 1e3, 2),
            "note": "same workload with the blocks in pinned host memory: nfec_encode_host (DMA: source up, "
                    "parity down) + nfec_decode_host (zero-copy slot moves: the 48 surviving source and 16 "
                    "substitute parity segments up, the 16 repaired segments down), overlapped with the kernels",
        }
        host["frac_of_link_bound"] = round(host["value"] / host["link_bound_GiBps"], 3)
        host["frac_of_mixed_bound"] = round(host["value"] / host["link_mixed_bound_GiBps"], 3)
        del hblocks, hnp

    ok = None
    if not a.no_verify:
        from norm_amd import zero_erasures

        # One clean round trip from the pristine source: encode once, erase, repair once, and
        # every byte must come back.  (Checking the state after the timed loop is not enough: a
        # decode that is off by a fixed linear offset cancels itself over an even number of
        # encode + decode steps.)
        blocks[:, :k].copy_(orig)
        enc.encode_blocks(blocks, stream=stream)
        keep = blocks.clone()
        zero_erasures(blocks, locs, counts, vec, stream=stream)
        dec.decode_blocks(blocks, locs, counts, status=status, stream=stream)
        torch.cuda.synchronize(dev)
        ok = bool(torch.equal(blocks, keep)) and bool((status == a.erasures).all())
        del keep
        if dist is not None:  # every rank's blocks: the line says true only if all came back
            t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=cdev)
            dist.all_reduce(t, op=dist.ReduceOp.MIN)
            ok = bool(t.item())

    if orig is not None:
        del orig
    total_blocks = a.blocks if a.strong else nb * world
    src_bytes = k * vec * total_blocks
    ms_per_step = elapsed / a.steps * 1e3
    value = src_bytes / (elapsed / a.steps) / 2**30
    enc_bytes = (k + m) * vec * nb  # algorithmic HBM bytes of one encode launch (per GPU)
    achieved = enc_bytes / (enc_ms * 1e-3) / 1e9
    # the repair reads the k - e surviving source and e substitute parity segments and writes the
    # e repaired ones: (k + e) * vec per block
    dec_bytes = (k + a.erasures) * vec * nb
    dec_achieved = dec_bytes / (dec_ms * 1e-3) / 1e9

    traffic = None
    dec_traffic = None
    valu = None
    pmc_path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(pmc_path):
        try:
            pmc = json.load(open(pmc_path))
            if pmc.get("blocks") == nb and pmc.get("k") == k and pmc.get("m") == m and pmc.get("vec") == vec:
                traffic = pmc.get("encode_hbm_bytes_per_launch")
                if a.erasures == 16:
                    dec_traffic = pmc.get("decode_hbm_bytes_per_launch")
                if pmc.get("valu_insts_per_launch"):
                    # the kernel is VALU-bound as much as HBM-bound: its
                    # wave64 VALU instructions (PMC SQ_INSTS_VALU) over the measured launch time
                    lane_ops = pmc["valu_insts_per_launch"] * 64 / (enc_ms * 1e-3)
                    valu = {"achieved": float("%.4g" % lane_ops), "peak": VALU_PEAK, "unit": "lane-ops/s",
                            "frac": round(lane_ops / VALU_PEAK, 4),
                            "insts_per_launch": pmc["valu_insts_per_launch"]}
        except Exception:
            traffic = None

    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return

    cpu = None
    if world == 1 and not a.no_cpu_baseline:
        from oracle import pyoracle as orc

        usable, visible = host_cores()
        threads = a.cpu_threads if a.cpu_threads > 0 else usable
        te, td, bad = orc.bench_rs8(k, m, vec, a.cpu_blocks, a.erasures, threads)
        te1, td1, bad1 = orc.bench_rs8(k, m, vec, 256, a.erasures, 1)
        cpu = {
            "value": round(k * vec * a.cpu_blocks / (te + td) / 2**30, 4),
            "unit": "GiB/s",
            "cores": threads,
            "kind": "port",
            "sample": (f"oracle C restatement (per-segment Encode + Gauss-Jordan Decode, -O2) on {a.cpu_blocks} "
                       f"blocks RS8({k},{m}) x {vec} B, {a.erasures} source erasures/block, one codec per thread on "
                       f"{threads} threads ({visible} CPUs in the affinity mask, {usable} usable under the cgroup "
                       f"quota); encode {te:.2f}s decode {td:.2f}s wall, bad blocks {bad}"),
            "host_cpus_visible": visible,
            "single_thread_value": round(k * vec * 256 / (te1 + td1) / 2**30, 4),
        }

    out = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "strong" if a.strong else "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (splitmix64 source segments generated in HBM; reference RS8 generator)",
        "config": {
            "workload": (f"RS8 k={k} m={m} seg={vec}B: encode + {a.erasures}-source-erasure decode of "
                         + (f"{a.blocks} blocks in total over {world} GPU(s)" if a.strong else f"{nb} blocks per GPU")
                         + " in HBM"),
            "k": k, "m": m, "vec": vec, "blocks_per_gpu": nb, "blocks_total": total_blocks, "erasures": a.erasures,
            "parallelism": f"block-striped x{world} (no collective)",
        },
        "roofline_encode": {
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "kernel": encode_kernel_name(k, m, vec),
            "algorithmic_bytes_per_launch": enc_bytes,
            "read_only_frac": round(k * vec * nb / (enc_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "achievable_copy": {"GBps": round(copy_gbs, 1), "frac": round(achieved / copy_gbs, 4),
                                "blit_GBps": round(blit_gbs, 1),
                                "note": "4 GiB device-to-device copy on this GPU by a streaming kernel "
                                        "(nfec_util_stream_copy), read + write bytes; blit_GBps: torch copy_"},
            "valu": valu,
        },
        # the other half of the step: the repair (plan + fused repair kernel, one decode call)
        "roofline_decode": {
            "bound": "hbm",
            "achieved": round(dec_achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(dec_achieved / HBM_PEAK_GBS, 4),
            "traffic": dec_traffic,
            "kernel": f"nfec::rs8_fdec_k{k}_m{m} + rs_plan2_kernel (one decode call)",
            "algorithmic_bytes_per_launch": dec_bytes,
        },
        "kernels_ms": {"encode": round(enc_ms, 4), "decode": round(dec_ms, 4)},
        "cpu_baseline": cpu,
    }
    # `roofline` is the step's dominant kernel: the one with the longer measured launch (the
    # repair call, plan included, on most boxes); both halves stay under roofline_encode /
    # roofline_decode
    dom = "roofline_decode" if dec_ms > enc_ms else "roofline_encode"
    out["roofline"] = dict(out[dom], dominant_of_step=dom.split("_")[1],
                           share_of_step=round(max(enc_ms, dec_ms) / (enc_ms + dec_ms), 4))
    out = {key: out[key] for key in ["metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                                     "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config",
                                     "roofline", "roofline_encode", "roofline_decode", "kernels_ms", "cpu_baseline"]}
    if host is not None:
        out["host_resident"] = host
    if ok is not None:
        out["verified"] = ok
    if share:
        out["rehearsal"] = (f"{world} ranks sharing cuda:0 over gloo (--share-gpu): the N-rank code path on one "
                            "GPU, not a scaling number")
    print(json.dumps(out))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
