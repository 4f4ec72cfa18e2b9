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
    p.add_argument("--loss", default="source", choices=["source", "uniform"],
                   help="source: erasures among the source segments (the headline pattern); uniform: "
                        "drawn over all k + m segments, as NORM loses source and parity alike")
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
    enc = enc_cls()
    assert enc.Init(k, m, vec)
    init_s = time.perf_counter() - t0
    dec = None
    if er:
        dec = dec_cls()
        assert dec.Init(k, m, vec)
    blocks = torch.zeros((nb, k + m, vec), dtype=torch.uint8, device="cuda")
    na.fill_blocks(blocks, k, vec, 0x4E4F524D)
    if er and a.loss == "uniform":
        import numpy as np

        rng = np.random.default_rng(0x4E4F524D)
        pick = np.sort(np.argsort(rng.random((nb, k + m)), axis=1)[:, :er], axis=1)
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
        enc.encode_blocks(blocks, stream=stream)
        if er:
            dec.decode_blocks(blocks, locs, counts, status=status, stream=stream)
    torch.cuda.synchronize()
    enc_ms = timed(lambda: enc.encode_blocks(blocks, stream=stream), a.steps)
    out = {
        "workload": a.workload,
        "codec": {na.NFEC_RS8: "RS8", na.NFEC_RS16: "RS16", na.NFEC_MDP: "MDP"}[kind],
        "k": k, "m": m, "vec": vec, "blocks": nb, "erasures": er, "loss": a.loss,
        "init_s": round(init_s, 3),
        "encode_ms": round(enc_ms, 3),
        "encode_GiBps": round(k * vec * nb / (enc_ms * 1e-3) / 2**30, 2),
    }
    if kind == na.NFEC_RS16 and os.environ.get("NFEC_GF16_T3", "1") != "0" and vec % 8 == 0:
        # op roofline of the shared-table RS16 encode (gen_gf16_t3.hip), counted from its code:
        # per (item group of 64 lanes x 64 symbols, source column) every live parity row issues
        # 16 planes x 3 ds_read_b64 (512 B each) and 7 VALU per plane, and per pass of up to RP
        # rows the builder issues 506 VALU and 125 ds_write_b64 (RP = 44: 11 row waves x 4 rows;
        # row waves past the last row leave).  With the Toeplitz split (features bit 0) the
        # products are three of m/2 rows over k/2 columns instead of one of m rows over k.
        groups = -(-nb * vec // 8192)
        RP = 44
        split = bool(enc.features() & na.NFEC_FEATURE_RS16_TOEPLITZ)
        nprod, ncols, rows = (3, k // 2, m // 2) if split else (1, k, m)
        passes = -(-rows // RP)
        rows4 = -(-rows // 4) * 4
        units = groups * ncols * nprod
        lds_bytes = units * rows4 * 16 * 3 * 512
        valu = units * (rows4 * 16 * 7 + passes * 506)
        t = enc_ms * 1e-3
        out["op_roofline"] = {
            "kernel": "gf16_t3_multi_kernel (Toeplitz split: 3 products of m/2 rows over k/2 columns)"
                      if split else "gf16_t3_encode_kernel",
            "gf16_macs_per_s": float("%.4g" % (k * m * (vec // 2) * nb / t)),
            "macs_note": "k*m*symbols of the generator product per second (the split computes 3/4 of them)"
                         if split else "k*m*symbols per second",
            "lds": {"achieved": float("%.4g" % (lds_bytes / t)), "peak": 256 * 256 * 2.4e9, "unit": "B/s",
                    "frac": round(lds_bytes / t / (256 * 256 * 2.4e9), 4),
                    "note": "table reads only (ds_read_b64, counted at 256 B/clk/CU), over the whole encode time"},
            "valu": {"achieved": float("%.4g" % (valu * 64 / t)), "peak": 7.86e13, "unit": "lane-ops/s",
                     "frac": round(valu * 64 / t / 7.86e13, 4), "insts_per_launch": valu},
            "lds_insts_per_launch": units * rows4 * 16 * 3 + groups * nprod * passes * ncols * 125,
        }
    if er:
        dec_ms = timed(lambda: dec.decode_blocks(blocks, locs, counts, status=status, stream=stream), a.steps)
        keep = blocks.clone()
        na.zero_erasures(blocks, locs, counts, vec, stream=stream)
        dec.decode_blocks(blocks, locs, counts, status=status, stream=stream)
        torch.cuda.synchronize()
        out.update({
            "decode_ms": round(dec_ms, 3),
            "decode_GiBps": round(k * vec * nb / (dec_ms * 1e-3) / 2**30, 2),
            "combined_GiBps": round(k * vec * nb / ((enc_ms + dec_ms) * 1e-3) / 2**30, 2),
            # parity erasures are zeroed and stay so (Decode fills source erasures only)
            "verified": bool(torch.equal(blocks[:, :k], keep[:, :k])) and bool((status == er).all()),
        })
    print(json.dumps(out), flush=True)


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
