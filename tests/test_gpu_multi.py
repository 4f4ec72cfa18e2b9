"""One codec over several devices (nfec_codec_create_ex): host batches striped in contiguous block
ranges, one pipeline per device, bytes identical to the oracle.  The test box has one GPU, so
the device list is {0, 0} (and {0, 0, 0} for an uneven split): two or three full stripes with
their own staging, streams and host threads on one device -- the same code path an 8-GPU node
takes with {0..7}.  Reference callers this serves from one process: one NORM session's encoder
(normSession.cpp:834-889) and npc (normPrecode.cpp:588-880), SURVEY 8b/8e."""
import numpy as np
import pytest

from norm_amd import _native as N

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _codecs(kind, k, m, vec, devices):
    import norm_amd as na

    enc = {N.NFEC_RS8: na.NormEncoderRS8, N.NFEC_RS16: na.NormEncoderRS16, N.NFEC_MDP: na.NormEncoderMDP}[kind]
    dec = {N.NFEC_RS8: na.NormDecoderRS8, N.NFEC_RS16: na.NormDecoderRS16, N.NFEC_MDP: na.NormDecoderMDP}[kind]
    e, d = enc(devices=devices), dec(devices=devices)
    assert e.Init(k, m, vec) and d.Init(k, m, vec)
    return e, d


def _erase(orc, clean, k, m, es, seed):
    rng = np.random.default_rng(seed)
    nb = clean.shape[0]
    locs = np.zeros((nb, m), np.uint16)
    counts = np.full(nb, es, np.uint16)
    rx = clean.copy()
    for b in range(nb):
        e = np.sort(rng.choice(k, es, replace=False))
        locs[b, :es] = e
        rx[b, e] = 0
    return rx, locs, counts


@pytest.fixture(autouse=True)
def _small_chunks(monkeypatch):
    monkeypatch.setenv("NFEC_HOST_CHUNK_BLOCKS", "64")  # several pipeline chunks per stripe


@pytest.mark.parametrize("kind,k,m,vec,nb,es,devices", [
    (N.NFEC_RS8, 64, 32, 1400, 301, 16, [0, 0]),
    (N.NFEC_RS8, 64, 16, 1408, 200, 9, [0, 0, 0]),   # uneven split: 66/67/67
    (N.NFEC_RS16, 100, 20, 1400, 9, 12, [0, 0]),
    (N.NFEC_MDP, 64, 32, 1400, 40, 16, [0, 0]),
])
def test_striped_host_batch_matches_oracle(orc, kind, k, m, vec, nb, es, devices):
    enc, dec = _codecs(kind, k, m, vec, devices)
    assert enc.num_devices() == devices
    host = orc.make_blocks(k, m, vec, nb)
    host[:, k:] = 0x3C  # overwrite semantics: stale parity must not survive in any stripe
    ref = orc.encode_blocks(kind, k, m, vec, host.copy())
    pinned = torch.from_numpy(host.copy()).pin_memory().numpy()
    enc.encode_blocks_host(host)       # pageable
    enc.encode_blocks_host(pinned)     # page-locked
    assert np.array_equal(host, ref) and np.array_equal(pinned, ref)
    rx, locs, counts = _erase(orc, ref, k, m, es, 3)
    want = rx.copy()
    st_ref = orc.decode_blocks(kind, k, m, vec, want, locs, counts)
    st = dec.decode_blocks_host(rx, locs, counts)
    assert np.array_equal(st, st_ref) and np.array_equal(rx, want)


def test_striped_segment_lists_and_async(orc):
    """segment-list batches and their async form on a two-device codec, shortened blocks"""
    k, m, vec, nb = 64, 32, 1400, 150
    rng = np.random.default_rng(7)
    nd = rng.integers(1, k + 1, nb).astype(np.uint16)
    host = orc.make_blocks(k, m, vec, nb, num_data=nd)
    ref = orc.encode_blocks(N.NFEC_RS8, k, m, vec, host.copy(), nd)
    enc, dec = _codecs(N.NFEC_RS8, k, m, vec, [0, 0])
    segs = [[host[b, s].copy() for s in range(int(nd[b]) + m)] for b in range(nb)]
    enc.encode_vectors_host(segs, num_data=nd)
    for b in range(nb):
        for s in range(int(nd[b]) + m):
            assert np.array_equal(segs[b][s], ref[b, s]), (b, s)
    # async decode of full blocks, missing parity given as None
    clean = orc.encode_blocks(N.NFEC_RS8, k, m, vec, orc.make_blocks(k, m, vec, nb))
    rx, locs, counts = _erase(orc, clean, k, m, 12, 5)
    want = rx.copy()
    st_ref = orc.decode_blocks(N.NFEC_RS8, k, m, vec, want, locs, counts)
    segs = [[rx[b, s].copy() for s in range(k + m)] for b in range(nb)]
    req = dec.decode_vectors_host_async(segs, locs, counts)
    st = req.wait()
    assert np.array_equal(st, st_ref)
    for b in range(nb):
        for s in range(k):
            assert np.array_equal(segs[b][s], want[b, s]), (b, s)


@pytest.mark.parametrize("kind", [N.NFEC_RS8, N.NFEC_MDP])
@pytest.mark.parametrize("host_call", [False, True])
def test_multi_device_batch_and_per_call(orc, kind, host_call):
    """device batches run on the stripe of their device; per-call Encode/Decode on the first
    (GPU round trips, or the host paths, which read the first stripe's tables)"""
    k, m, vec, nb = 64, 32, 1400, 33
    enc, dec = _codecs(kind, k, m, vec, [0, 0])
    host = orc.make_blocks(k, m, vec, nb)
    ref = orc.encode_blocks(kind, k, m, vec, host.copy())
    dev = torch.from_numpy(host).cuda()
    enc.encode_blocks(dev)
    torch.cuda.synchronize()
    assert np.array_equal(dev.cpu().numpy(), ref)
    par = [np.zeros(vec, np.uint8) for _ in range(m)]
    for s in range(k):
        enc.Encode(s, host[0, s].copy(), par, host=host_call)
    for p in range(m):
        assert np.array_equal(par[p], ref[0, k + p])
    rx, locs, counts = _erase(orc, ref[:1], k, m, 16, 9)
    want = rx.copy()
    orc.decode_blocks(kind, k, m, vec, want, locs, counts)
    vl = [rx[0, s].copy() for s in range(k + m)]
    assert dec.Decode(vl, k, 16, [int(x) for x in locs[0, :16]], host=host_call) == 16
    for s in range(k):
        assert np.array_equal(vl[s], want[0, s])


def test_bad_device_list_fails():
    import ctypes

    cfg = N.CodecConfig()
    cfg.kind, cfg.num_data, cfg.num_parity, cfg.vector_size = N.NFEC_RS8, 64, 32, 1400
    devs = (ctypes.c_int32 * 2)(0, 99)
    cfg.devices = ctypes.cast(devs, ctypes.POINTER(ctypes.c_int32))
    cfg.num_devices = 2
    h = ctypes.c_void_p()
    assert N.lib().nfec_codec_create_ex(ctypes.byref(cfg), ctypes.byref(h)) == N.NFEC_EDEVICE and not h


def test_multi_device_codec_takes_host_mapped_batches(orc):
    """a device batch in pinned (host-mapped) host memory names no device: a {0, 0} codec runs it
    on its first stripe, as a one-device codec passes it through -- same bytes either way"""
    k, m, vec, nb = 16, 4, 64, 5
    host = orc.make_blocks(k, m, vec, nb)
    ref = orc.encode_blocks(N.NFEC_RS8, k, m, vec, host.copy())
    for devices in ([0], [0, 0]):
        enc, _ = _codecs(N.NFEC_RS8, k, m, vec, devices)
        pinned = torch.from_numpy(host.copy()).pin_memory()
        enc.encode_blocks(pinned)
        torch.cuda.synchronize()
        assert np.array_equal(pinned.numpy(), ref), devices


def test_multi_device_codec_refuses_pageable_batches():
    """plain pageable host memory (numpy) is no device batch: HIP does not know it, and a kernel
    dereferencing it would fault the GPU (no XNACK).  A striped codec refuses it with NFEC_EINVAL
    before any launch; pinned memory (above) and device memory run."""
    import ctypes

    k, m, vec, nb = 16, 4, 64, 3
    blk = np.zeros((nb, k + m, vec), np.uint8)
    enc, _ = _codecs(N.NFEC_RS8, k, m, vec, [0, 0])
    b = N.BlockBatch()
    b.blocks, b.block_stride, b.seg_stride, b.nblocks = blk.ctypes.data, (k + m) * vec, vec, nb
    assert N.lib().nfec_encode(enc._h, ctypes.byref(b), None) == N.NFEC_EINVAL
    assert "not on a device" in N.last_error()
