"""The host side of N-GPU striping: every host-batch copy of every codec and stripe
runs on one process-wide pool sized to the cores the job may use -- the affinity mask capped by
the cgroup cpu.max quota, as bench.py's host_cores reads it -- so a codec striped over 8 GPUs
(8 driver threads, one per device) never puts more copy threads on the cores than that.
The gathers are NORM's segment-list form (block->SegmentList(), scattered pool segments,
normSegment.cpp:14-86).  CPU only: nfec_util_gather_probe runs the real gather code without a
GPU."""
import ctypes
import os
import subprocess
import sys

import numpy as np
import pytest

from norm_amd import _native as N

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _cores():
    sys.path.insert(0, ROOT)
    import bench

    return bench.host_cores()  # (usable, visible)


def _pool():
    p, u, v = N._U32(), N._U32(), N._U32()
    N.check(N.lib().nfec_host_threads(ctypes.byref(p), ctypes.byref(u), ctypes.byref(v)), "host threads")
    return p.value, u.value, v.value


def _segment_table(nblocks, slots, vec, seed=5):
    """one pool of segments, handed out in a shuffled order (scattered, 8-byte aligned)"""
    stride = (vec + 7) & ~7
    pool = np.random.default_rng(seed).integers(0, 256, (nblocks * slots, stride), dtype=np.uint8)
    order = np.random.default_rng(seed + 1).permutation(nblocks * slots)
    base = pool.ctypes.data
    tab = (ctypes.c_void_p * (nblocks * slots))(*[base + int(i) * stride for i in order])
    return pool, tab


def test_pool_sized_to_usable_cores():
    pool, usable, visible = _pool()
    u, v = _cores()
    assert (usable, visible) == (u, v)
    if "NFEC_HOST_THREADS" not in os.environ:
        assert 1 <= pool <= min(usable, 64)


@pytest.mark.parametrize("stripes", [1, 2, 8])
def test_striped_gather_stays_within_the_pool(stripes):
    """8 stripes gather at once; the pool never runs more copy pieces than its workers (a
    thread per stripe and per call would have been 8 x 8 = 64)"""
    pool, usable, _ = _pool()
    nblocks, slots, vec = 8 * stripes * 24, 96, 1400   # >= 4 MiB per piece, several pieces per stripe
    keep, tab = _segment_table(nblocks, slots, vec)
    sec, mx = ctypes.c_double(), N._U32()
    N.check(N.lib().nfec_util_gather_probe(tab, nblocks, slots, vec, stripes, 1, ctypes.byref(sec), ctypes.byref(mx)),
            "gather probe")
    assert sec.value > 0
    assert 1 <= mx.value <= pool <= max(1, usable) if "NFEC_HOST_THREADS" not in os.environ else mx.value <= pool


def test_pool_respects_host_threads_override():
    """NFEC_HOST_THREADS=3: three workers whatever the cores (in a fresh process: the pool is
    sized once per process)"""
    code = ("import ctypes; from norm_amd import _native as N; p=N._U32(); "
            "N.lib().nfec_host_threads(ctypes.byref(p), None, None); print(p.value)")
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, NFEC_HOST_THREADS="3"))
    assert r.returncode == 0 and r.stdout.strip() == "3", r.stderr
