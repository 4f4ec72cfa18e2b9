"""Host-resident encode / decode timing (bench.py's host_resident leg, split by operation).

    python tools/host_rate.py [--blocks 16384] [--steps 3] [--chunk 0]

Blocks of RS8(64,32) x 1400 B live in pinned host memory; nfec_encode_host and nfec_decode_host
(16 source erasures per block) are timed separately, with the PCIe bytes each one moves
(encode: 64 segments up, 32 down; decode: 48 + 16 up, 16 down with the zero-copy slot moves) and
the rate those bytes imply.  --chunk sets NFEC_HOST_CHUNK_BLOCKS (pipeline chunk size).
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
    p.add_argument("--blocks", type=int, default=16384)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--chunk", type=int, default=0)
    p.add_argument("--k", type=int, default=64)
    p.add_argument("--m", type=int, default=32)
    p.add_argument("--vec", type=int, default=1400)
    p.add_argument("--erasures", type=int, default=16)
    a = p.parse_args()
    if a.chunk:
        os.environ["NFEC_HOST_CHUNK_BLOCKS"] = str(a.chunk)
    import numpy as np
    import torch

    from norm_amd import NormDecoderRS8, NormEncoderRS8, fill_blocks, make_erasures

    k, m, vec, nb = a.k, a.m, a.vec, a.blocks
    enc, dec = NormEncoderRS8(), NormDecoderRS8()
    assert enc.Init(k, m, vec) and dec.Init(k, m, vec)
    d = torch.zeros((nb, k + m, vec), dtype=torch.uint8, device="cuda")
    fill_blocks(d, k, vec, 0x4E4F524D)
    locs, counts = make_erasures(nb, k, a.erasures, 0x4E4F524D, m)
    h = torch.empty(d.shape, dtype=torch.uint8, pin_memory=True)
    h.copy_(d)
    hn = h.numpy()
    hl = locs.cpu().numpy().view(np.uint16)
    hc = counts.cpu().numpy().view(np.uint16)
    enc.encode_blocks_host(hn)
    dec.decode_blocks_host(hn, hl, hc)
    te = td = 0.0
    for _ in range(a.steps):
        t0 = time.perf_counter()
        enc.encode_blocks_host(hn)
        t1 = time.perf_counter()
        st = dec.decode_blocks_host(hn, hl, hc)
        t2 = time.perf_counter()
        te += t1 - t0
        td += t2 - t1
    te /= a.steps
    td /= a.steps
    seg = vec * nb
    out = {"blocks": nb, "chunk": a.chunk or "default", "encode_ms": round(te * 1e3, 2), "decode_ms": round(td * 1e3, 2),
           "encode_GBps_h2d": round(k * seg / te / 1e9, 1), "encode_GBps_d2h": round(m * seg / te / 1e9, 1),
           "decode_GBps_h2d": round((k - a.erasures + a.erasures) * seg / td / 1e9, 1),
           "decode_GBps_d2h": round(a.erasures * seg / td / 1e9, 1),
           "step_GiBps": round(k * seg / (te + td) / 2**30, 2), "ok": bool((st == a.erasures).all())}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
