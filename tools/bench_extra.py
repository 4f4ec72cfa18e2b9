"""Secondary workloads (not the headline bench line): one JSON line per workload.

    python tools/bench_extra.py [--workload c4|rs16|mdp|rs8] [--blocks N] [--steps K]

c4    RS16 k=4096 m=256 vec=1400 encode (BASELINE C4), default 4096 blocks in HBM
rs16  RS16 k=400 m=100 vec=1400 encode + 50-erasure decode (the C5 RS16 block type)
mdp   MDP k=64 m=32 vec=1400 encode + 16-erasure decode
rs8   RS8 with --k/--m/--erasures (other shapes than the headline)
rs8sweep  RS8 encode + decode over NORM-plausible shapes, one line per shape, with the time per
      source byte relative to (64, 32): (64,32), (16,4), (32,16), (64,16) shortened (numData
      drawn per block from [32, 64]), (128,32), (200,55), (64,8), (8,2) -- the generic-shape cliff

Inputs are synthetic (splitmix64 segments generated on the GPU); GiB/s counts source bytes
(k * vec per block) per pass, like the headline metric.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--workload", default="c4")
    p.add_argument("--blocks", type=int, default=0)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--k", type=int, default=0)
    p.add_argument("--m", type=int, default=0)
    p.add_argument("--vec", type=int, default=1400)
    p.add_argument("--erasures", type=int, default=-1)
    p.add_argument("--shortened", action="store_true",
                   help="numData drawn per block (--nd-dist; every NORM object's last block is shortened)")
    p.add_argument("--nd-dist", default="half", choices=["half", "rfc"],
                   help="half: numData uniform over [k/2, k]; rfc: k or k - 1 (RFC 5052 large and small "
                        "blocks, NORM's block partition, normObject.cpp:203-231)")
    p.add_argument("--accumulate", action="store_true", help="decode with NFEC_ACCUMULATE (erased source zeroed)")
    p.add_argument("--loss", default="source", choices=["source", "uniform"],
                   help="source: erasures among the source segments (the headline pattern); uniform: "
                        "drawn over all k + m segments, as NORM loses source and parity alike")
    p.add_argument("--options", type=int, default=0, help="encoder options (NFEC_OPT_*, e.g. the Toeplitz split's levels)")
    a = p.parse_args()
    import torch
    import norm_amd as na

    if a.workload == "rs8sweep":
        return rs8_sweep(a)

    shapes = {  # kind, k, m, blocks, erasures (0: encode only)
        "c4": (na.NFEC_RS16, 4096, 256, 4096, 0),
        "rs16": (na.NFEC_RS16, 400, 100, 16384, 50),
        "mdp": (na.NFEC_MDP, 64, 32, 65536, 16),
        "rs8": (na.NFEC_RS8, 64, 32, 65536, 16),
    }
    kind, k, m, nb, er = shapes[a.workload]
    k = a.k or k
    m = a.m or m
    nb = a.blocks or nb
    er = er if a.erasures < 0 else a.erasures
    vec = a.vec
    enc_cls = {na.NFEC_RS8: na.NormEncoderRS8, na.NFEC_RS16: na.NormEncoderRS16, na.NFEC_MDP: na.NormEncoderMDP}[kind]
    dec_cls = {na.NFEC_RS8: na.NormDecoderRS8, na.NFEC_RS16: na.NormDecoderRS16, na.NFEC_MDP: na.NormDecoderMDP}[kind]
    torch.cuda.set_device(0)
    t0 = time.perf_counter()
    enc = enc_cls(options=a.options) if a.options else enc_cls()
    assert enc.Init(k, m, vec)
    init_s = time.perf_counter() - t0
    dec = None
    if er:
        dec = dec_cls()
        assert dec.Init(k, m, vec)
    import numpy as np

    # segment stride: the batch layout keeps segments 8-byte aligned (vec 1460 -> 1464)
    blocks = torch.zeros((nb, k + m, (vec + 7) & ~7), dtype=torch.uint8, device="cuda")
    rng = np.random.default_rng(0x4E4F524D)
    nd = None
    ndh = np.full(nb, k, np.int64)
    if a.shortened:
        ndh = rng.integers(k // 2, k + 1, nb) if a.nd_dist == "half" else k - rng.integers(0, 2, nb)
        nd = torch.from_numpy(ndh.astype(np.uint16).view(np.int16)).cuda()
        na.fill_blocks(blocks, k, vec, 0x4E4F524D, per_block_num_data=nd)
    else:
        na.fill_blocks(blocks, k, vec, 0x4E4F524D)
    orig = blocks.clone() if er else None  # the pristine batch, for the round trip below
    if er and (a.loss == "uniform" or a.shortened):
        # per block: er distinct locations among the numData source (source loss) or among all
        # numData + m segments (uniform loss), ascending
        span = ndh + (m if a.loss == "uniform" else 0)
        keys = rng.random((nb, k + m))
        keys[np.arange(k + m)[None, :] >= span[:, None]] = 2.0
        pick = np.sort(np.argsort(keys, axis=1)[:, :er], axis=1)
        hl = np.zeros((nb, m), np.int16)
        hl[:, :er] = pick
        locs = torch.from_numpy(hl).cuda()
        counts = torch.full((nb,), er, dtype=torch.int16, device="cuda")
        status = torch.empty(nb, dtype=torch.int32, device="cuda")
    elif er:
        locs, counts = na.make_erasures(nb, k, er, 0x4E4F524D, m)
        status = torch.empty(nb, dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream()

    def timed(fn, n):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(n):
            fn()
        e1.record(stream)
        e1.synchronize()
        return e0.elapsed_time(e1) / n

    for _ in range(a.warmup):
        enc.encode_blocks(blocks, num_data=nd, stream=stream)
        if er:
            dec.decode_blocks(blocks, locs, counts, num_data=nd, status=status, accumulate=a.accumulate, stream=stream)
    torch.cuda.synchronize()
    enc_ms = timed(lambda: enc.encode_blocks(blocks, num_data=nd, stream=stream), a.steps)
    out = {
        "workload": a.workload,
        "codec": {na.NFEC_RS8: "RS8", na.NFEC_RS16: "RS16", na.NFEC_MDP: "MDP"}[kind],
        "k": k, "m": m, "vec": vec, "blocks": nb, "erasures": er, "loss": a.loss,
        "shortened": a.shortened, "accumulate": a.accumulate,
        "nd_dist": a.nd_dist if a.shortened else None,
        "source_GB": round(float(ndh.sum()) * vec / 1e9, 3),
        "init_s": round(init_s, 3),
        "encode_ms": round(enc_ms, 3),
        "encode_GiBps": round(float(ndh.sum()) * vec / (enc_ms * 1e-3) / 2**30, 2),
    }
    if kind == na.NFEC_RS16:
        from norm_amd import _native as N
        f = enc.features()
        out["toeplitz_levels"] = (2 if f & N.NFEC_FEATURE_RS16_TOEPLITZ2 else 1 if f & N.NFEC_FEATURE_RS16_TOEPLITZ else 0)
    out["encode_paths"] = {n: c for n, c in enc.encode_paths().items() if c}
    if kind == na.NFEC_RS16 and vec % 8 == 0 and not a.shortened:
        out["op_roofline"] = rs16_op_roofline(enc, k, m, nb, vec, enc_ms)
    if er:
        dec_ms = timed(lambda: dec.decode_blocks(blocks, locs, counts, num_data=nd, status=status, accumulate=a.accumulate,
                                                 stream=stream), a.steps)
        # one clean round trip from the pristine source: encode, erase, repair, every source
        # byte back (the timed loops repair in place, which alone would not catch a wrong map)
        blocks.copy_(orig)
        enc.encode_blocks(blocks, num_data=nd, stream=stream)
        keep = blocks.clone()
        na.zero_erasures(blocks, locs, counts, vec, stream=stream)
        dec.decode_blocks(blocks, locs, counts, num_data=nd, status=status, accumulate=a.accumulate, stream=stream)
        torch.cuda.synchronize()
        # parity erasures are zeroed and stay so (Decode fills source erasures only)
        src_ok = True
        for b0 in range(0, nb, 4096):
            sl = slice(b0, min(nb, b0 + 4096))
            mask = torch.arange(k + m, device="cuda")[None, :] < torch.from_numpy(ndh[sl]).cuda()[:, None]
            src_ok &= bool(((blocks[sl, :, :vec] == keep[sl, :, :vec]) | ~mask[:, :, None]).all())
        sdec = float(ndh.sum()) * vec
        out.update({
            "decode_ms": round(dec_ms, 3),
            "decode_GiBps": round(sdec / (dec_ms * 1e-3) / 2**30, 2),
            "combined_GiBps": round(sdec / ((enc_ms + dec_ms) * 1e-3) / 2**30, 2),
            "verified": src_ok and bool((status == er).all()),
        })
    print(json.dumps(out), flush=True)


VALU_PEAK = 7.86e13   # 256 CU x 4 SIMD x 32 lanes x 2.4 GHz (a wave64 VALU instruction: 2 cycles)


def rs16_op_roofline(enc, k, m, nb, vec, enc_ms):
    """Op roofline of the RS16 products from the tower kernel's own PMC counters (committed
    under profiles/, tools/pmc_r03.sh on this workload): per launch SQ_INSTS_VALU / SALU / BRANCH
    / LDS and the kernel's cycles (GRBM_GUI_ACTIVE / 8 XCDs).  Issue fractions: VALU x 2 cycles
    over 1,024 SIMDs, SALU and branches one per cycle per CU (256), against those cycles."""
    import glob
    import norm_amd as na

    from norm_amd import _native as N

    f = enc.features()
    split = bool(f & N.NFEC_FEATURE_RS16_TOEPLITZ)
    two = bool(f & N.NFEC_FEATURE_RS16_TOEPLITZ2)
    name = "gf16_tw_multi_kernel" if split else "gf16_tw_encode_kernel"
    form = (" (Toeplitz split, two Karatsuba levels: 9 tower-field products of m/4 rows over k/4 columns)" if two
            else " (Toeplitz split: 3 tower-field products of m/2 rows over k/2 columns)" if split
            else " (tower-field products, snippet calls)")
    out = {"kernel": name + form,
           "gf16_macs_per_s": float("%.4g" % (k * m * (vec // 2) * nb / (enc_ms * 1e-3))),
           "macs_note": "k*m*symbols of the generator product per second"
                        + (" (the split computes 9/16 of them)" if two
                           else " (the split computes 3/4 of them)" if split else "")}
    src = None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r0*", "pmc_tw_*summary.json")), reverse=True):
        d = json.load(open(path))
        meta = d.get("_workload", {})
        if meta.get("k") == k and meta.get("m") == m and meta.get("blocks") == nb and meta.get("vec") == vec:
            src = (path, d)
            break
    if src is None:
        out["pmc"] = None
        out["note"] = "no committed tower-kernel PMC summary for this shape (tools/pmc_r03.sh, PMC_SCRIPT=tools/bench_extra.py)"
        return out
    path, d = src
    meta = d.get("_workload", {})
    kern = [v for kk, v in d.items() if kk != "_workload" and name in kk]
    if not kern:
        out["pmc"] = None
        return out
    c = kern[0]
    cycles = c["GRBM_GUI_ACTIVE"] / 8.0
    # a large batch runs as several sub-batches (C4: two, each ~12.5 GB of split scratch), each
    # with its own product launch: the PMC summary holds per-launch averages over `dispatches`
    # launches of a run of `encodes` encodes (the pmc scripts run --warmup 1 --steps 1)
    encodes = meta.get("encodes", 2)
    launches = max(1, round(c.get("dispatches", encodes) / encodes))
    out.update({
        "pmc": os.path.relpath(path, ROOT),
        "cycles_per_launch": round(cycles),
        "insts_per_launch": {n: round(c[f"SQ_INSTS_{n.upper()}"]) for n in ("valu", "salu", "branch", "lds", "smem")
                             if f"SQ_INSTS_{n.upper()}" in c},
        "valu_issue_frac": round(c["SQ_INSTS_VALU"] * 2 / (1024 * cycles), 4),
        "salu_issue_frac": round(c["SQ_INSTS_SALU"] / (256 * cycles), 4),
        "branch_issue_frac": round(c.get("SQ_INSTS_BRANCH", 0) / (256 * cycles), 4),
        "launches_per_encode": launches,
        "valu_lane_ops_frac_of_peak": round(c["SQ_INSTS_VALU"] * launches * 64 / (enc_ms * 1e-3) / VALU_PEAK, 4),
        "note": "counters per launch of the product kernel; issue fractions against its own cycles "
                "(VALU 2 cycles per wave64 instruction per SIMD, SALU / branch 1 per cycle per CU); "
                "lane-op fraction: all product launches of one encode over the whole encode time",
    })
    return out


SWEEP = [  # k, m, shortened, source erasures
    (64, 32, False, 16), (16, 4, False, 4), (32, 16, False, 16), (64, 16, True, 8), (128, 32, False, 16),
    (200, 55, False, 16), (64, 8, False, 8), (8, 2, False, 2),
]


def rs8_sweep(a):
    """encode + source-erasure repair per shape; ns per source byte against the (64, 32) line"""
    import numpy as np
    import torch
    import norm_amd as na

    torch.cuda.set_device(0)
    stream = torch.cuda.current_stream()
    vec = a.vec
    base = None

    def timed(fn, n):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(n):
            fn()
        e1.record(stream)
        e1.synchronize()
        return e0.elapsed_time(e1) / n

    for k, m, short, er in SWEEP:
        # about 5.9 GB of source per shape (the headline's 65,536 x 64 x 1400), at most 1M blocks
        nb = a.blocks or min(1 << 20, (65536 * 64) // k)
        enc, dec = na.NormEncoderRS8(), na.NormDecoderRS8()
        assert enc.Init(k, m, vec) and dec.Init(k, m, vec)
        blocks = torch.zeros((nb, k + m, vec), dtype=torch.uint8, device="cuda")
        rng = np.random.default_rng(k * 1000 + m)
        nd = None
        if short:
            ndh = rng.integers(k // 2, k + 1, nb).astype(np.uint16)
            nd = torch.from_numpy(ndh.view(np.int16)).cuda()
            na.fill_blocks(blocks, k, vec, 0x4E4F524D, per_block_num_data=nd)
            hl = np.zeros((nb, m), np.int16)
            for b in range(nb):
                hl[b, :er] = np.sort(rng.choice(int(ndh[b]), er, replace=False))
            locs = torch.from_numpy(hl).cuda()
            counts = torch.full((nb,), er, dtype=torch.int16, device="cuda")
            src = float(ndh.astype(np.float64).sum()) * vec
        else:
            na.fill_blocks(blocks, k, vec, 0x4E4F524D)
            locs, counts = na.make_erasures(nb, k, er, 0x4E4F524D, m)
            src = float(k) * vec * nb
        status = torch.empty(nb, dtype=torch.int32, device="cuda")
        enc.encode_blocks(blocks, num_data=nd, stream=stream)
        dec.decode_blocks(blocks, locs, counts, num_data=nd, status=status, stream=stream)
        torch.cuda.synchronize()
        enc_ms = timed(lambda: enc.encode_blocks(blocks, num_data=nd, stream=stream), a.steps)
        dec_ms = timed(lambda: dec.decode_blocks(blocks, locs, counts, num_data=nd, status=status, stream=stream),
                       a.steps)
        # one clean round trip: encode, erase, repair, compare
        enc.encode_blocks(blocks, num_data=nd, stream=stream)
        keep = blocks.clone()
        na.zero_erasures(blocks, locs, counts, vec, stream=stream)
        dec.decode_blocks(blocks, locs, counts, num_data=nd, status=status, stream=stream)
        torch.cuda.synchronize()
        ok = bool(torch.equal(blocks, keep)) and bool((status == er).all())
        enc_ns, dec_ns = enc_ms * 1e6 / src, dec_ms * 1e6 / src
        if base is None:
            base = (enc_ns, dec_ns)
        print(json.dumps({
            "workload": "rs8sweep", "k": k, "m": m, "shortened": short, "vec": vec, "blocks": nb, "erasures": er,
            "source_GB": round(src / 1e9, 3),
            "encode_ms": round(enc_ms, 3), "decode_ms": round(dec_ms, 3),
            "encode_ns_per_source_byte": round(enc_ns, 5), "decode_ns_per_source_byte": round(dec_ns, 5),
            "encode_vs_64_32": round(enc_ns / base[0], 3), "decode_vs_64_32": round(dec_ns / base[1], 3),
            "encode_hbm_GBps": round((src / vec) * (k + m) / k * vec / (enc_ms * 1e-3) / 1e9, 1),
            "verified": ok,
        }), flush=True)
        del blocks, keep, status, locs, counts
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
