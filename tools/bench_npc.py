"""npc file precoder throughput (not the headline bench line): one JSON line.

    python tools/bench_npc.py [--mb 1024] [--segment 1404] [--block 64] [--parity 32]
                              [--damage 16] [--dir /dev/shm]

Encodes a synthetic file with nfec_npc_encode_file, damages `--damage` segments of every
FEC block (a flipped byte breaks their CRC), decodes with nfec_npc_decode_file and checks
the output against the input.  Rates are input-file bytes per second, file to file (memory
mapped, page cache / tmpfs), including the PCIe transfers and the host gather/scatter.
With block/parity chosen so that (b * parity) % block == 0 the reference's segment-id
rotation leaves every repair exact (see norm_amd/csrc/npc.cpp).
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
    p.add_argument("--mb", type=int, default=1024)
    p.add_argument("--segment", type=int, default=1404)
    p.add_argument("--block", type=int, default=32)
    p.add_argument("--parity", type=int, default=32)
    p.add_argument("--damage", type=int, default=16)
    p.add_argument("--dir", default="/dev/shm")
    a = p.parse_args()
    import numpy as np

    from norm_amd import npc

    d = os.path.join(a.dir, f"nfec_npc_bench_{os.getpid()}")
    os.makedirs(d, exist_ok=True)
    src, enc, out = os.path.join(d, "input.bin"), os.path.join(d, "input.npc"), os.path.join(d, "output.bin")
    try:
        size = a.mb << 20
        rng = np.random.default_rng(7)
        with open(src, "wb") as f:
            for _ in range(a.mb):
                f.write(rng.integers(0, 256, 1 << 20, dtype=np.uint8).tobytes())
        params = npc.make_params(segment=a.segment, block=a.block, parity=a.parity)
        npc.encode_file(src, enc, params)  # warm: codec init, staging allocation
        t0 = time.perf_counter()
        npc.encode_file(src, enc, params)
        t_enc = time.perf_counter() - t0
        lay = npc.layout(params, os.path.getsize(enc), encode=False)
        pos = npc.positions(lay)
        k, m, ss = lay.num_data, lay.num_parity, lay.segment_size
        nd_last = lay.last_block_data
        with open(enc, "r+b") as f:  # damage `--damage` segments per block
            mm = np.memmap(f, dtype=np.uint8, mode="r+")
            for blk in range(lay.num_blocks):
                nd = nd_last if blk + 1 == lay.num_blocks else k
                for t in rng.choice(nd + m, min(a.damage, nd + m, m), replace=False):
                    mm[int(pos[blk * (k + m) + t]) * ss + 17] ^= 0x5A
            mm.flush()
            del mm
        t0 = time.perf_counter()
        _, nbytes = npc.decode_file(enc, out, params)
        t_dec = time.perf_counter() - t0
        ok = nbytes == size
        if ok:
            with open(src, "rb") as f1, open(out, "rb") as f2:
                while ok:
                    b1, b2 = f1.read(1 << 24), f2.read(1 << 24)
                    ok = b1 == b2
                    if not b1:
                        break
        print(json.dumps({
            "workload": "npc file precode", "file_MiB": a.mb, "segment": ss, "block": k, "parity": m,
            "fec_blocks": lay.num_blocks, "damaged_per_block": min(a.damage, m),
            "codec": "RS16" if lay.kind == 2 else "RS8",
            "encode_s": round(t_enc, 3), "encode_MiBps": round(a.mb / t_enc, 1),
            "decode_s": round(t_dec, 3), "decode_MiBps": round(a.mb / t_dec, 1),
            "round_trip_ok": bool(ok), "dir": a.dir,
        }), flush=True)
    finally:
        for f in (src, enc, out):
            if os.path.exists(f):
                os.unlink(f)
        os.rmdir(d)


if __name__ == "__main__":
    main()
