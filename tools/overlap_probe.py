"""Probe: does running the repair of one sub-batch beside the encode of the next (two HIP
streams) beat running the two kernels back to back?  Same bytes either way.

    python tools/overlap_probe.py [--blocks 65536] [--parts 2 4 8]
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
    p.add_argument("--blocks", type=int, default=65536)
    p.add_argument("--parts", type=int, nargs="+", default=[1, 2, 4, 8])
    p.add_argument("--steps", type=int, default=10)
    a = p.parse_args()
    import torch

    from norm_amd import NormDecoderRS8, NormEncoderRS8, fill_blocks, make_erasures

    k, m, vec, nb = 64, 32, 1400, a.blocks
    enc, dec = NormEncoderRS8(), NormDecoderRS8()
    assert enc.Init(k, m, vec) and dec.Init(k, m, vec)
    blocks = torch.zeros((nb, k + m, vec), dtype=torch.uint8, device="cuda")
    fill_blocks(blocks, k, vec, 0x4E4F524D)
    locs, counts = make_erasures(nb, k, 16, 0x4E4F524D, m)
    status = torch.empty(nb, dtype=torch.int32, device="cuda")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    dec2 = NormDecoderRS8()
    assert dec2.Init(k, m, vec)

    def step(parts):
        if parts == 1:
            enc.encode_blocks(blocks, stream=s1)
            dec.decode_blocks(blocks, locs, counts, status=status, stream=s1)
            return
        sz = nb // parts
        evs = []
        for i in range(parts):
            sl = slice(i * sz, (i + 1) * sz)
            enc.encode_blocks(blocks[sl], stream=s1)
            e = torch.cuda.Event()
            e.record(s1)
            evs.append(e)
        for i in range(parts):
            sl = slice(i * sz, (i + 1) * sz)
            s2.wait_event(evs[i])
            dec.decode_blocks(blocks[sl], locs[sl], counts[sl], status=status[sl], stream=s2)
        s1.wait_stream(s2)

    out = {}
    for parts in a.parts:
        for _ in range(2):
            step(parts)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step(parts)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / a.steps * 1e3
        out[parts] = round(ms, 4)
        print(json.dumps({"parts": parts, "ms_per_step": round(ms, 4),
                          "GiBps": round(k * vec * nb / (ms * 1e-3) / 2**30, 1)}), flush=True)


if __name__ == "__main__":
    main()
