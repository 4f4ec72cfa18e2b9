"""Host-only codecs (NFEC_OPT_HOST_ONLY): a NORM node without a usable gfx950 still gets a
working NormEncoder / NormDecoder, since the drop-in's per-call defaults run on the CPU.  No GPU
is touched, so these run in the CPU suite.  Init's math (the generator: normEncoderRS8.cpp:400-462,
normEncoderRS16.cpp:399-461, normEncoderMDP.cpp:102-170), the per-segment Encode
(normEncoderRS8.cpp:473-483, RS16 :472-482, MDP LFSR :178-211) and the one-block Decode
(normEncoderRS8.cpp:652-757, RS16 :650-755, MDP :333-430) against the oracle byte for byte;
every GPU entry refuses a host-only codec with NFEC_EDEVICE."""
import ctypes

import numpy as np
import pytest

from norm_amd import (NFEC_MDP, NFEC_RS8, NFEC_RS16, NormDecoderMDP, NormDecoderRS8, NormDecoderRS16,
                      NormEncoderMDP, NormEncoderRS8, NormEncoderRS16)
from norm_amd import _native as N

ENC = {NFEC_RS8: NormEncoderRS8, NFEC_RS16: NormEncoderRS16, NFEC_MDP: NormEncoderMDP}
DEC = {NFEC_RS8: NormDecoderRS8, NFEC_RS16: NormDecoderRS16, NFEC_MDP: NormDecoderMDP}


def _pair(kind, k, m, vec):
    enc, dec = ENC[kind](options=N.NFEC_OPT_HOST_ONLY), DEC[kind](options=N.NFEC_OPT_HOST_ONLY)
    assert enc.Init(k, m, vec) and dec.Init(k, m, vec)
    return enc, dec


def test_host_only_codec_info_and_generator(orc):
    enc, _ = _pair(NFEC_RS8, 64, 32, 1400)
    info = N.CodecInfo()
    N.check(N.lib().nfec_codec_get_info(enc._h, ctypes.byref(info)), "info")
    assert info.device == -1 and info.num_data == 64 and info.num_parity == 32
    g = np.zeros((32, 64), np.uint8)
    N.check(N.lib().nfec_codec_get_generator(enc._h, g.ctypes.data, g.nbytes), "generator")
    assert np.array_equal(g, orc.generator(NFEC_RS8, 64, 32)[64:])  # (the oracle: the full n x k matrix)
    # Init's range checks hold without a device too
    assert not NormEncoderRS8(options=N.NFEC_OPT_HOST_ONLY).Init(200, 56, 64)
    assert not NormEncoderMDP(options=N.NFEC_OPT_HOST_ONLY).Init(200, 56, 64)


def test_host_only_refuses_gpu_entries():
    enc, dec = _pair(NFEC_RS8, 16, 4, 64)
    b = N.BlockBatch()
    blk = np.zeros((1, 20, 64), np.uint8)
    b.blocks, b.block_stride, b.seg_stride, b.nblocks = blk.ctypes.data, 20 * 64, 64, 1
    assert N.lib().nfec_encode(enc._h, ctypes.byref(b), None) == N.NFEC_EDEVICE
    assert N.lib().nfec_encode_host(enc._h, ctypes.byref(b)) == N.NFEC_EDEVICE
    vecs = (ctypes.c_void_p * 20)(*[blk[0, s].ctypes.data for s in range(20)])
    assert N.lib().nfec_encode_host_vectors(enc._h, vecs, 1, None, 0) == N.NFEC_EDEVICE
    par = (ctypes.c_void_p * 4)(*[blk[0, 16 + i].ctypes.data for i in range(4)])
    assert N.lib().nfec_encode_segment(enc._h, 0, blk[0, 0].ctypes.data, par) == N.NFEC_EDEVICE
    locs = (ctypes.c_uint32 * 1)(0)
    assert N.lib().nfec_decode_vectors(dec._h, vecs, 16, 1, locs) == N.NFEC_EDEVICE
    assert N.lib().nfec_decode_host_preferred(dec._h, 16, 1) == 1
    # a device list is refused with the option
    cfg = N.CodecConfig()
    cfg.kind, cfg.num_data, cfg.num_parity, cfg.vector_size = NFEC_RS8, 16, 4, 64
    devs = (ctypes.c_int32 * 2)(0, 0)
    cfg.devices = ctypes.cast(devs, ctypes.POINTER(ctypes.c_int32))
    cfg.num_devices = 2
    cfg.flags = N.NFEC_OPT_HOST_ONLY
    h = ctypes.c_void_p()
    assert N.lib().nfec_codec_create_ex(ctypes.byref(cfg), ctypes.byref(h)) == N.NFEC_EINVAL


CASES = [
    # kind, k, m, vec, numData, source erasures, parity erasures
    (NFEC_RS8, 64, 32, 1400, 64, 16, 0),
    (NFEC_RS8, 64, 32, 1408, 50, 10, 6),
    (NFEC_RS8, 200, 55, 1401, 150, 40, 10),
    (NFEC_RS16, 400, 100, 1400, 400, 40, 10),
    (NFEC_RS16, 60, 13, 1461, 45, 8, 5),
    (NFEC_MDP, 64, 32, 1408, 64, 16, 0),
    (NFEC_MDP, 40, 20, 1401, 30, 8, 6),
    # min(k, m) > 256: past the GPU plan's closed form (kPlanCfMaxE); the host repair takes any
    # size (the reference decodes any k + m <= 65535, normEncoderRS16.cpp:650-755)
    (NFEC_RS16, 600, 300, 1400, 600, 260, 20),
    (NFEC_RS16, 600, 300, 64, 550, 280, 0),
    (NFEC_RS16, 1000, 400, 32, 900, 400, 0),
]


@pytest.mark.parametrize("kind,k,m,vec,nd,es,ep", CASES)
def test_host_only_encode_decode_match_oracle(orc, kind, k, m, vec, nd, es, ep):
    rng = np.random.default_rng(k * 7 + m + vec)
    enc, dec = _pair(kind, k, m, vec)
    nda = np.array([nd], np.uint16) if nd < k else None
    host = orc.make_blocks(k, m, vec, 1, num_data=nda)
    ref = orc.encode_blocks(kind, k, m, vec, host.copy(), nda)
    # Encode: one call per source segment in order (MDP's LFSR requires it), zeroed parity
    par = [np.zeros(vec, np.uint8) for _ in range(m)]
    for s in range(nd):
        enc.Encode(s, host[0, s, :vec].copy(), par, host=True)
    for i in range(m):
        assert np.array_equal(par[i], ref[0, nd + i, :vec]), f"parity {i}"
    # Decode: erased source zero-filled, missing parity NULL
    e = np.sort(np.concatenate([rng.choice(nd, es, replace=False), nd + rng.choice(m, ep, replace=False)]))
    rx = [ref[0, s, :vec].copy() for s in range(nd + m)]
    for s in e:
        rx[s][:] = 0
    want = ref.copy()
    for s in e:
        want[0, s] = 0
    el = np.zeros((1, m), np.uint16)
    el[0, :len(e)] = e
    st_ref = orc.decode_blocks(kind, k, m, vec, want, el, np.array([len(e)], np.uint16), nda)
    vl = [None if (s in set(e.tolist()) and s >= nd) else rx[s] for s in range(nd + m)]
    st = dec.Decode(vl, nd, len(e), [int(x) for x in e])
    assert st == int(st_ref[0]) == len(e)
    for s in range(nd):
        assert np.array_equal(rx[s], want[0, s, :vec]), f"segment {s}"
