"""Host ceiling of an N-GPU NORM-form host-resident run: the segment-list gather rate at 1, 2, 4
and 8 stripes, on the host CPU only (no GPU).  A codec striped over N devices gathers N block
ranges at once through the process-wide host pool (host_pool.cpp); this times that code
(nfec_util_gather_probe) on a fixed batch of RS8(64,32) blocks whose 96 segments of 1400 bytes
sit scattered in one segment pool (NORM's block->SegmentList(), normSegment.cpp:14-86).

    python tools/host_gather_rate.py [--blocks 16384] [--reps 3]   -> one JSON line per stripe count
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--blocks", type=int, default=16384)
    p.add_argument("--slots", type=int, default=96)
    p.add_argument("--vec", type=int, default=1400)
    p.add_argument("--reps", type=int, default=3)
    p.add_argument("--stripes", default="1,2,4,8")
    a = p.parse_args()
    import numpy as np
    from norm_amd import _native as N
    import bench

    usable, visible = bench.host_cores()
    pool, pu, pv = N._U32(), N._U32(), N._U32()
    N.check(N.lib().nfec_host_threads(ctypes.byref(pool), ctypes.byref(pu), ctypes.byref(pv)), "host threads")
    stride = (a.vec + 7) & ~7
    nseg = a.blocks * a.slots
    t0 = time.perf_counter()
    seg = np.random.default_rng(1).integers(0, 256, (nseg, stride), dtype=np.uint8)
    order = np.random.default_rng(2).permutation(nseg)
    tab = (ctypes.c_void_p * nseg)(*(seg.ctypes.data + order.astype(np.int64) * stride).tolist())
    setup = time.perf_counter() - t0
    gb = a.blocks * a.slots * a.vec / 1e9
    for s in [int(x) for x in a.stripes.split(",")]:
        sec, mx = ctypes.c_double(), N._U32()
        N.check(N.lib().nfec_util_gather_probe(tab, a.blocks, a.slots, a.vec, s, a.reps, ctypes.byref(sec),
                                               ctypes.byref(mx)), "gather probe")
        print(json.dumps({
            "probe": "segment-list gather (host only)", "stripes": s, "blocks": a.blocks, "slots": a.slots,
            "vec": a.vec, "GB_per_pass": round(gb, 3), "seconds": round(sec.value, 4),
            "GBps": round(gb / sec.value, 2), "pool_workers": pool.value, "max_active_pieces": mx.value,
            "usable_cores": usable, "visible_cores": visible, "setup_s": round(setup, 1),
        }), flush=True)


if __name__ == "__main__":
    main()
