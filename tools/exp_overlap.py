"""Experiment: the headline step (RS8(64,32) encode + 16-erasure repair of 65,536 blocks in HBM)
with the batch split into P parts on S streams, so one part's repair runs beside another part's
encode (the two kernels leave both HBM and VALU about half idle when alone).

    python tools/exp_overlap.py [--parts 2] [--streams 2] [--steps 20]

Each part has its own encoder / decoder (a decode's plan scratch is per codec).  Stream j runs the
parts j, j + S, ... in order: encode then repair of each.  Stream j > 0 starts after the first
encode of stream j - 1 (offset), so encodes and repairs interleave.  Prints one JSON line per mode
and checks every repaired byte afterwards.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--blocks", type=int, default=65536)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--modes", default="seq,2x2,2x2o,4x2o,4x4o,8x2o")
    a = p.parse_args()
    import torch

    import norm_amd as na

    k, m, vec, er = 64, 32, 1400, 16
    seed = 0x4E4F524D
    dev = torch.device("cuda", 0)
    blocks = torch.zeros((a.blocks, k + m, vec), dtype=torch.uint8, device=dev)
    na.fill_blocks(blocks, k, vec, seed)
    locs, counts = na.make_erasures(a.blocks, k, er, seed, m)
    orig = blocks[:, :k].clone()
    src_bytes = k * vec * a.blocks
    for mode in a.modes.split(","):
        if mode == "seq":
            parts, nstreams, offset = 1, 1, False
        else:
            x, y = mode.rstrip("o").split("x")
            parts, nstreams, offset = int(x), int(y), mode.endswith("o")
        per = a.blocks // parts
        pieces = []
        for i in range(parts):
            lo, hi = i * per, (a.blocks if i == parts - 1 else (i + 1) * per)
            enc, dec = na.NormEncoderRS8(), na.NormDecoderRS8()
            assert enc.Init(k, m, vec) and dec.Init(k, m, vec)
            st = torch.empty(hi - lo, dtype=torch.int32, device=dev)
            pieces.append((enc, dec, blocks[lo:hi], locs[lo:hi], counts[lo:hi], st))
        streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(nstreams - 1)]

        def step():
            main_s = streams[0]
            start = torch.cuda.Event()
            start.record(main_s)
            firsts = []
            for j, s in enumerate(streams):
                s.wait_event(start)
                if offset and j:
                    s.wait_event(firsts[j - 1])
                for i in range(j, parts, nstreams):
                    enc, dec, b, lc, cn, st = pieces[i]
                    enc.encode_blocks(b, stream=s)
                    if i == j:
                        ev = torch.cuda.Event()
                        ev.record(s)
                        firsts.append(ev)
                    dec.decode_blocks(b, lc, cn, status=st, stream=s)
            for s in streams[1:]:
                done = torch.cuda.Event()
                done.record(s)
                main_s.wait_event(done)

        for _ in range(a.warmup):
            step()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step()
        torch.cuda.synchronize(dev)
        dt = (time.perf_counter() - t0) / a.steps
        # check: erased source zeroed after the timed steps (parity in place), then every part's
        # repair alone, so only the repair can bring the bytes back
        na.zero_erasures(blocks, locs, counts, vec)
        for enc, dec, b, lc, cn, st in pieces:
            dec.decode_blocks(b, lc, cn, status=st)
        torch.cuda.synchronize(dev)
        ok = bool(torch.equal(blocks[:, :k], orig)) and all(bool((pc[5] == er).all()) for pc in pieces)
        print(json.dumps({"mode": mode, "parts": parts, "streams": nstreams, "offset": offset,
                          "ms_per_step": round(dt * 1e3, 4), "GiBps": round(src_bytes / dt / 2**30, 2), "ok": ok}),
              flush=True)
        del pieces
        torch.cuda.synchronize(dev)


if __name__ == "__main__":
    main()
