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


def test_throwing_piece_returns_an_error():
    """a piece that throws (std::bad_alloc in a gather's allocation, anything else) neither ends
    the process nor leaves the caller waiting: every piece runs and the call returns a status"""
    L = N.lib()
    assert L.nfec_util_pool_check(64, 0) == 64
    assert L.nfec_util_pool_check(64, 1) == N.NFEC_ENOMEM
    assert "out of memory" in N.last_error()
    assert L.nfec_util_pool_check(64, 2) == N.NFEC_EINVAL
    assert "pool check" in N.last_error()
    assert L.nfec_util_pool_check(2, 1) == N.NFEC_ENOMEM
    assert L.nfec_util_pool_check(64, 0) == 64  # the pool still works afterwards


def _wait_child(pid, seconds=60):
    import time

    t0 = time.time()
    while time.time() - t0 < seconds:
        done, status = os.waitpid(pid, os.WNOHANG)
        if done:
            return os.waitstatus_to_exitcode(status)
        time.sleep(0.05)
    os.kill(pid, 9)
    os.waitpid(pid, 0)
    return None


def test_pool_after_fork_runs_inline():
    """a child forked after the pool started inherits the pool object but not its workers: its
    pool calls (and a large host repair, which splits over the pool) run inline instead of
    queueing for threads that do not exist"""
    from norm_amd import NFEC_RS8, NormDecoderRS8, NormEncoderRS8

    L = N.lib()
    assert L.nfec_util_pool_check(32, 0) == 32  # the pool's workers run in this process
    k, m, vec, e = 128, 127, 16384, 100         # 200 MB of products: past the 8 MiB split
    enc, dec = NormEncoderRS8(options=N.NFEC_OPT_HOST_ONLY), NormDecoderRS8(options=N.NFEC_OPT_HOST_ONLY)
    assert enc.Init(k, m, vec) and dec.Init(k, m, vec)
    blk = np.random.default_rng(3).integers(0, 256, (k + m, vec), dtype=np.uint8)
    blk[k:] = 0
    for s in range(k):
        enc.Encode(s, blk[s], [blk[k + p] for p in range(m)])
    want = blk.copy()
    locs = list(range(1, k, k // e))[:e]  # source erasures only (parity is never filled)
    for s in locs:
        blk[s] = 0
    pid = os.fork()
    if pid == 0:  # child: no pytest machinery, exit code only
        code = 1
        try:
            if L.nfec_util_pool_check(32, 0) == 32 and L.nfec_util_pool_check(8, 1) == N.NFEC_ENOMEM:
                n = dec.Decode([blk[s] for s in range(k + m)], k, e, locs, host=True)
                code = 0 if n == e and np.array_equal(blk, want) else 2
        finally:
            os._exit(code)
    assert _wait_child(pid) == 0
