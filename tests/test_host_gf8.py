"""The host per-segment path (nfec_gf8_addmul_host, the body of nfec_encode_segment_host and of the
drop-in NormEncoderRS8::Encode / NormEncoderMDP::Encode): dst ^= c * src in the RS8 field, every form this CPU has (GFNI,
AVX2, scalar) against the oracle's product table -- the table the reference builds with
init_mul_table (src/common/normEncoderRS8.cpp:140-149), pinned to galois.cpp's field
(tests/test_oracle.py).  CPU only: no GPU is involved."""
import ctypes

import numpy as np
import pytest

from norm_amd import _native as N

FORMS = [N.NFEC_HOST_GF_SCALAR, N.NFEC_HOST_GF_AVX2, N.NFEC_HOST_GF_GFNI]


def _best():
    src = np.zeros(1, np.uint8)
    dst = np.zeros(1, np.uint8)
    return N.lib().nfec_gf8_addmul_host(dst.ctypes.data, src.ctypes.data, 1, 1, -1)


def _call(dst, src, c, n, form):
    return N.lib().nfec_gf8_addmul_host(dst.ctypes.data, src.ctypes.data, c, n, form)


@pytest.mark.parametrize("form", FORMS)
def test_every_coefficient_matches_oracle(orc, form):
    if form > _best():
        pytest.skip("this CPU lacks the instructions of that form")
    mul = orc.gf8_mul_table()
    rng = np.random.default_rng(form)
    src = np.arange(256, dtype=np.uint8).repeat(2)   # every byte value, 512 bytes
    for c in range(256):
        dst = rng.integers(0, 256, src.size, dtype=np.uint8)
        want = dst ^ mul[c][src]
        assert _call(dst, src, c, src.size, form) == form
        assert np.array_equal(dst, want), c


@pytest.mark.parametrize("form", FORMS)
@pytest.mark.parametrize("n", [0, 1, 31, 32, 33, 63, 1400, 1401, 1408])
def test_lengths_and_guard_bytes(orc, form, n):
    """unaligned buffers, tails: exactly n bytes change (the reference processes vector_size bytes)"""
    if form > _best():
        pytest.skip("this CPU lacks the instructions of that form")
    mul = orc.gf8_mul_table()
    rng = np.random.default_rng(n)
    src_buf = rng.integers(0, 256, n + 40, dtype=np.uint8)
    dst_buf = rng.integers(0, 256, n + 40, dtype=np.uint8)
    src, dst = src_buf[3:3 + n], dst_buf[5:5 + n]   # odd alignments
    before = dst_buf.copy()
    c = 0x8e
    _call(dst, src, c, n, form)
    want = before.copy()
    want[5:5 + n] ^= mul[c][src]
    assert np.array_equal(dst_buf, want)


def test_zero_coefficient_and_bad_form():
    src = np.full(64, 7, np.uint8)
    dst = np.arange(64, dtype=np.uint8)
    assert _call(dst, src, 0, 64, -1) >= 0
    assert np.array_equal(dst, np.arange(64, dtype=np.uint8))
    assert _call(dst, src, 3, 64, 7) == N.NFEC_EINVAL
    assert N.lib().nfec_gf8_addmul_host(None, None, 3, 0, -1) >= 0
    assert N.lib().nfec_gf8_addmul_host(ctypes.c_void_p(0), src.ctypes.data, 3, 8, -1) == N.NFEC_EINVAL


@pytest.mark.gpu
@pytest.mark.parametrize("k,m,vec", [(64, 16, 1408), (64, 32, 1400), (200, 55, 1401), (1, 1, 8)])
def test_encode_segment_host_matches_gpu_and_oracle(orc, k, m, vec):
    """nfec_encode_segment_host (the drop-in RS8 Encode's default) and nfec_encode_segment (the
    GPU round trip) give the oracle's per-segment parity, accumulated over a whole block"""
    import norm_amd as na

    enc = na.NormEncoderRS8()
    assert enc.Init(k, m, vec)
    host = orc.make_blocks(k, m, vec, 1)
    ref = orc.encode_blocks(N.NFEC_RS8, k, m, vec, host.copy())
    for fn in ("nfec_encode_segment_host", "nfec_encode_segment"):
        par = [np.zeros(vec, np.uint8) for _ in range(m)]
        arr = (ctypes.c_void_p * m)(*[p.ctypes.data for p in par])
        for s in range(k):
            d = np.ascontiguousarray(host[0, s, :vec])
            assert getattr(N.lib(), fn)(enc._h, s, d.ctypes.data, arr) == 0
        for p in range(m):
            assert np.array_equal(par[p], ref[0, k + p, :vec]), (fn, p)


@pytest.mark.gpu
@pytest.mark.parametrize("k,m,vec", [(64, 32, 1408), (20, 7, 1401), (5, 1, 64)])
def test_encode_segment_host_mdp_lfsr(orc, k, m, vec):
    """MDP on the host: the reference's LFSR step per in-order segment (normEncoderMDP.cpp:
    178-211) over zeroed parity gives the oracle's block parity, as the GPU per-call path does"""
    import norm_amd as na

    enc = na.NormEncoderMDP()
    assert enc.Init(k, m, vec)
    host = orc.make_blocks(k, m, vec, 1)
    ref = orc.encode_blocks(N.NFEC_MDP, k, m, vec, host.copy())
    for fn in ("nfec_encode_segment_host", "nfec_encode_segment"):
        par = [np.zeros(vec, np.uint8) for _ in range(m)]
        arr = (ctypes.c_void_p * m)(*[p.ctypes.data for p in par])
        for s in range(k):
            d = np.ascontiguousarray(host[0, s, :vec])
            assert getattr(N.lib(), fn)(enc._h, s, d.ctypes.data, arr) == 0
        for p in range(m):
            assert np.array_equal(par[p], ref[0, k + p, :vec]), (fn, p)


@pytest.mark.gpu
@pytest.mark.parametrize("k,m,vec", [(400, 100, 1400), (300, 20, 1401), (10, 4, 64)])
def test_encode_segment_host_rs16(orc, k, m, vec):
    """RS16 on the host: vec // 2 native-endian symbols per segment, an odd last byte untouched,
    block parity equal to the oracle's and to the GPU per-call path"""
    import norm_amd as na

    enc = na.NormEncoderRS16()
    assert enc.Init(k, m, vec)
    host = orc.make_blocks(k, m, vec, 1)
    ref = orc.encode_blocks(N.NFEC_RS16, k, m, vec, host.copy())
    for fn in ("nfec_encode_segment_host", "nfec_encode_segment"):
        par = [np.zeros(vec, np.uint8) for _ in range(m)]
        arr = (ctypes.c_void_p * m)(*[p.ctypes.data for p in par])
        for s in range(k):
            d = np.ascontiguousarray(host[0, s, :vec])
            assert getattr(N.lib(), fn)(enc._h, s, d.ctypes.data, arr) == 0
        for p in range(m):
            assert np.array_equal(par[p], ref[0, k + p, :vec]), (fn, p)


# ---- GF(2^16): the RS16 per-segment Encode's product (normEncoderRS16.cpp:472-482) ----

def _gf16_ref(orc, c, x):
    ex, lg, _ = orc.gf16_tables()
    x = x.astype(np.int64)
    out = np.zeros(x.shape, np.uint16)
    nz = x != 0
    if c:
        out[nz] = ex[(int(lg[c]) + lg[x[nz]]) % 65535]
    return out


@pytest.mark.parametrize("form", [N.NFEC_HOST_GF_SCALAR, N.NFEC_HOST_GF_GFNI])
@pytest.mark.parametrize("n", [0, 1, 15, 16, 17, 700, 701])
def test_gf16_addmul_matches_oracle(orc, form, n):
    if form > _best():
        pytest.skip("this CPU lacks the instructions of that form")
    rng = np.random.default_rng(n + 7 * form)
    for c in [0, 1, 2, 0x8000, 0xFFFF] + [int(v) for v in rng.integers(1, 65536, 12)]:
        buf = rng.integers(0, 65536, n + 3, dtype=np.uint16)
        src = buf[1:1 + n]                                   # 2-byte aligned, not 32
        dst_buf = rng.integers(0, 65536, n + 3, dtype=np.uint16)
        before = dst_buf.copy()
        rc = N.lib().nfec_gf16_addmul_host(dst_buf[1:].ctypes.data, src.ctypes.data, c, n, form)
        assert rc == form
        want = before.copy()
        want[1:1 + n] ^= _gf16_ref(orc, c, src)
        assert np.array_equal(dst_buf, want), c


def test_gf16_addmul_odd_byte_alignment(orc):
    """symbols starting at an odd byte address (a pointer the engine may be handed)"""
    rng = np.random.default_rng(5)
    raw = rng.integers(0, 256, 2 * 100 + 3, dtype=np.uint8)
    draw = rng.integers(0, 256, 2 * 100 + 3, dtype=np.uint8)
    src = raw[1:201]
    dst = draw[1:201]
    before = draw.copy()
    c = 0x1234
    N.lib().nfec_gf16_addmul_host(dst.ctypes.data, src.ctypes.data, c, 100, -1)
    want = before.copy()
    want[1:201] = (before[1:201].view(np.uint16) ^ _gf16_ref(orc, c, src.view(np.uint16))).view(np.uint8)
    assert np.array_equal(draw, want)


# ---- row dot products (nfec_gf_dot_host): the body of the host one-block repair ----

def _dot(bits, dst, srcs, coef, n, acc, form):
    arr = (ctypes.c_void_p * max(1, len(srcs)))(*[x.ctypes.data for x in srcs])
    co = np.ascontiguousarray(coef, np.uint16)
    return N.lib().nfec_gf_dot_host(bits, dst.ctypes.data, arr, co.ctypes.data, len(srcs), n, int(acc), form)


@pytest.mark.parametrize("form", FORMS)
@pytest.mark.parametrize("n", [0, 1, 31, 32, 127, 128, 129, 1400, 1408, 4100])
@pytest.mark.parametrize("acc", [False, True])
def test_gf8_dot_matches_oracle(orc, form, n, acc):
    if form > _best():
        pytest.skip("this CPU lacks the instructions of that form")
    mul = orc.gf8_mul_table()
    rng = np.random.default_rng(n * 3 + form + 17 * acc)
    for nc in (0, 1, 5, 64):
        srcs = [rng.integers(0, 256, n + 3, dtype=np.uint8)[1:1 + n] for _ in range(nc)]
        coef = rng.integers(0, 256, nc)
        if nc:
            coef[0] = 0
        dst_buf = rng.integers(0, 256, n + 6, dtype=np.uint8)
        before = dst_buf.copy()
        assert _dot(8, dst_buf[3:], srcs, coef, n, acc, form) == form
        want = before[3:3 + n].copy() if acc else np.zeros(n, np.uint8)
        for x, c in zip(srcs, coef):
            want ^= mul[int(c)][x]
        assert np.array_equal(dst_buf[3:3 + n], want), nc
        assert np.array_equal(dst_buf[:3], before[:3]) and np.array_equal(dst_buf[3 + n:], before[3 + n:])


@pytest.mark.parametrize("form", [N.NFEC_HOST_GF_SCALAR, N.NFEC_HOST_GF_GFNI])
@pytest.mark.parametrize("n", [0, 1, 15, 16, 31, 32, 33, 700, 701])
@pytest.mark.parametrize("acc", [False, True])
def test_gf16_dot_matches_oracle(orc, form, n, acc):
    if form > _best():
        pytest.skip("this CPU lacks the instructions of that form")
    rng = np.random.default_rng(n * 5 + form + 11 * acc)
    for nc in (0, 1, 3, 40):
        srcs = [rng.integers(0, 65536, n + 2, dtype=np.uint16)[1:1 + n] for _ in range(nc)]
        coef = rng.integers(0, 65536, nc)
        if nc > 2:
            coef[:3] = [0, 1, 0xFFFF]
        dst_buf = rng.integers(0, 65536, n + 4, dtype=np.uint16)
        before = dst_buf.copy()
        assert _dot(16, dst_buf[2:], srcs, coef, n, acc, form) == form
        want = before[2:2 + n].copy() if acc else np.zeros(n, np.uint16)
        for x, c in zip(srcs, coef):
            want ^= _gf16_ref(orc, int(c), x)
        assert np.array_equal(dst_buf[2:2 + n], want), nc
        assert np.array_equal(dst_buf[:2], before[:2]) and np.array_equal(dst_buf[2 + n:], before[2 + n:])


def test_gf16_matrices_every_byte_half(orc):
    """the GF(2^16) product's affine matrices come from two 256-entry tables (linear in c): every
    coefficient of the form c = b and c = b << 8, and sums of them, against log/exp"""
    if N.NFEC_HOST_GF_GFNI > _best():
        pytest.skip("no GFNI")
    rng = np.random.default_rng(9)
    x = rng.integers(0, 65536, 64, dtype=np.uint16)
    for c in list(range(256)) + [b << 8 for b in range(256)] + [int(v) for v in rng.integers(0, 65536, 64)]:
        dst = np.zeros(64, np.uint16)
        assert N.lib().nfec_gf16_addmul_host(dst.ctypes.data, x.ctypes.data, c, 64, N.NFEC_HOST_GF_GFNI) == N.NFEC_HOST_GF_GFNI
        assert np.array_equal(dst, _gf16_ref(orc, c, x)), c


def test_gf_dot_bad_arguments():
    src = np.zeros(8, np.uint8)
    dst = np.zeros(8, np.uint8)
    arr = (ctypes.c_void_p * 1)(src.ctypes.data)
    co = np.ones(1, np.uint16)
    assert N.lib().nfec_gf_dot_host(12, dst.ctypes.data, arr, co.ctypes.data, 1, 8, 0, -1) == N.NFEC_EINVAL
    assert N.lib().nfec_gf_dot_host(8, None, arr, co.ctypes.data, 1, 8, 0, -1) == N.NFEC_EINVAL
    nul = (ctypes.c_void_p * 1)(None)
    assert N.lib().nfec_gf_dot_host(8, dst.ctypes.data, nul, co.ctypes.data, 1, 8, 0, -1) == N.NFEC_EINVAL
    assert N.lib().nfec_gf_dot_host(8, dst.ctypes.data, arr, co.ctypes.data, 1, 8, 0, 7) == N.NFEC_EINVAL


def test_percall_table_regenerates():
    """tools/percall_table.py turns the committed per-call measurements into INTEGRATION.md's
    table: the rows it writes are the ones the document holds"""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, os.path.join(root, "tools", "percall_table.py")], capture_output=True,
                         text=True, timeout=60)
    assert out.returncode == 0, out.stderr
    doc = open(os.path.join(root, "INTEGRATION.md")).read()
    assert out.stdout.strip() in doc
