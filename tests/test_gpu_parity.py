"""Parity of the HIP path (through the C ABI) against the oracle, on the GPU.

Bar: bit-exact for every byte of every block (parity slots, repaired source slots, and
the untouched bytes), same per-block Decode return values as the reference algorithm.
Small cases are checked byte-for-byte against the oracle; the BASELINE full size is
checked by the encode -> erase -> decode round trip plus sampled blocks against the oracle.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from norm_amd import (NFEC_RS8, NFEC_RS16, NFEC_MDP, NormDecoderMDP, NormDecoderRS8, NormDecoderRS16,  # noqa: E402
                      NormEncoderMDP, NormEncoderRS8, NormEncoderRS16, fill_blocks, make_erasures, zero_erasures)

ENC = {NFEC_RS8: NormEncoderRS8, NFEC_RS16: NormEncoderRS16, NFEC_MDP: NormEncoderMDP}
DEC = {NFEC_RS8: NormDecoderRS8, NFEC_RS16: NormDecoderRS16, NFEC_MDP: NormDecoderMDP}


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    from norm_amd import device_count

    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    assert device_count() >= 1, "no gfx950 device visible to libnfec"


def _codecs(kind, k, m, vec):
    e, d = ENC[kind](), DEC[kind]()
    assert e.Init(k, m, vec) and d.Init(k, m, vec)
    return e, d


def _erasures(orc, kind, k, m, nblocks, n_src, n_par, num_data=None, seed_off=0):
    locs = np.zeros((nblocks, m), np.uint16)
    counts = np.zeros(nblocks, np.uint16)
    for b in range(nblocks):
        nd = k if num_data is None else int(num_data[b])
        src = orc.erasure_pattern(b + seed_off, nd, min(n_src, nd))
        par = (nd + orc.erasure_pattern(b + 9000 + seed_off, m, n_par)).astype(np.uint16)
        allp = np.concatenate([src, par])[:m]
        counts[b] = len(allp)
        locs[b, : len(allp)] = allp
    return locs, counts


def _erase(blocks, locs, counts):
    for b in range(blocks.shape[0]):
        for s in locs[b, : counts[b]]:
            blocks[b, s, :] = 0


ENC_CASES = [
    # kind, k, m, vec, seg_stride, nblocks
    (NFEC_RS8, 64, 32, 1400, 1400, 37),
    (NFEC_RS8, 64, 32, 1400, 1408, 5),
    (NFEC_RS8, 64, 16, 1408, 1408, 29),  # NORM's canonical code at its real vector size (segment + 8)
    (NFEC_RS8, 64, 8, 1408, 1408, 13),   # NORM's default parity count
    (NFEC_RS8, 64, 16, 1400, 1400, 9),
    (NFEC_RS8, 64, 8, 1400, 1400, 7),
    (NFEC_RS8, 64, 32, 1397, 1400, 6),   # segment tail (vec % 8 != 0)
    (NFEC_RS8, 64, 32, 1400, 1400, 700),  # many workgroups
    (NFEC_RS8, 64, 32, 1401, 1408, 5),
    (NFEC_RS8, 1, 1, 17, 24, 3),
    (NFEC_RS8, 16, 4, 64, 64, 11),
    (NFEC_RS8, 200, 55, 100, 104, 3),
    (NFEC_RS8, 128, 127, 64, 64, 2),
    (NFEC_RS8, 8, 40, 1401, 1408, 3),
    (NFEC_RS8, 64, 32, 8, 8, 300),
    (NFEC_RS16, 40, 10, 65, 72, 3),
    (NFEC_RS16, 400, 100, 64, 64, 2),
    (NFEC_RS16, 100, 20, 1400, 1400, 3),
    (NFEC_RS16, 700, 200, 64, 64, 2),     # offsets table > 16 MB: the exp-table encode kernel
    (NFEC_MDP, 64, 32, 1400, 1400, 4),
    (NFEC_MDP, 16, 4, 33, 40, 5),
]


@pytest.mark.parametrize("kind,k,m,vec,stride,nb", ENC_CASES)
def test_encode_matches_oracle(orc, kind, k, m, vec, stride, nb):
    enc, _ = _codecs(kind, k, m, vec)
    host = orc.make_blocks(k, m, vec, nb, seg_stride=stride)
    ref = orc.encode_blocks(kind, k, m, vec, host.copy())
    dev = torch.from_numpy(host).cuda()
    enc.encode_blocks(dev)
    torch.cuda.synchronize()
    assert np.array_equal(dev.cpu().numpy(), ref)


@pytest.mark.parametrize("kind", [NFEC_RS8, NFEC_RS16, NFEC_MDP])
def test_encode_shortened_blocks(orc, kind):
    k, m, vec, nb = 64, 16, 200, 7
    nd = np.array([64, 40, 1, 63, 17, 64, 2], np.uint16)
    enc, _ = _codecs(kind, k, m, vec)
    host = orc.make_blocks(k, m, vec, nb, num_data=nd)
    ref = orc.encode_blocks(kind, k, m, vec, host.copy(), nd)
    dev = torch.from_numpy(host).cuda()
    enc.encode_blocks(dev, num_data=torch.from_numpy(nd.astype(np.int16)).cuda())
    torch.cuda.synchronize()
    assert np.array_equal(dev.cpu().numpy(), ref)


@pytest.mark.parametrize("kind,k,m,vec,nb", [(NFEC_RS8, 32, 8, 96, 4), (NFEC_RS16, 32, 8, 96, 4),
                                              (NFEC_RS8, 64, 32, 1400, 9), (NFEC_RS8, 64, 16, 1397, 5)])
def test_encode_accumulates_like_reference(orc, kind, k, m, vec, nb):
    """Encode XORs into the parity buffers (reference contract: caller zeroes them)."""
    enc, _ = _codecs(kind, k, m, vec)
    host = orc.make_blocks(k, m, vec, nb)
    junk = np.random.default_rng(1).integers(0, 256, (nb, m, host.shape[2]), dtype=np.uint8)
    ref = orc.encode_blocks(kind, k, m, vec, host.copy())
    host[:, k:, :] = junk
    expect = ref.copy()
    nbytes = vec if kind == NFEC_RS8 else vec // 2 * 2
    expect[:, k:, :nbytes] ^= junk[:, :, :nbytes]
    expect[:, k:, nbytes:] = junk[:, :, nbytes:]
    dev = torch.from_numpy(host).cuda()
    enc.encode_blocks(dev, accumulate=True)
    torch.cuda.synchronize()
    assert np.array_equal(dev.cpu().numpy(), expect)


DEC_CASES = [
    # kind, k, m, vec, nblocks, source erasures, parity erasures
    (NFEC_RS8, 64, 32, 1400, 23, 16, 0),
    (NFEC_RS8, 64, 16, 1408, 19, 11, 5),   # NORM (64, 16), vector = segment + 8, source + parity lost
    (NFEC_RS8, 64, 8, 1408, 11, 6, 2),
    (NFEC_RS8, 64, 32, 1400, 9, 32, 0),
    (NFEC_RS8, 64, 32, 1400, 9, 20, 12),
    (NFEC_RS8, 64, 32, 1400, 5, 0, 7),
    (NFEC_RS8, 64, 32, 1400, 7, 1, 31),
    (NFEC_RS8, 64, 16, 1400, 7, 12, 4),
    (NFEC_RS8, 64, 8, 200, 9, 8, 0),
    (NFEC_RS8, 64, 8, 203, 9, 5, 3),
    (NFEC_RS8, 16, 4, 64, 13, 3, 1),
    (NFEC_RS8, 1, 1, 24, 4, 1, 0),
    (NFEC_RS8, 128, 127, 64, 2, 100, 27),
    (NFEC_RS8, 200, 55, 100, 3, 40, 10),
    (NFEC_RS16, 40, 10, 65, 3, 7, 3),
    (NFEC_RS16, 400, 100, 64, 2, 2, 0),
    (NFEC_RS16, 400, 100, 64, 1, 90, 10),
    (NFEC_RS16, 300, 400, 64, 2, 280, 10),   # > 256 source erasures: plan lists in global scratch
    (NFEC_RS16, 100, 300, 66, 2, 90, 5),     # m > k: decode rows sized by min(k, m)
    (NFEC_RS8, 16, 200, 64, 3, 16, 20),
    (NFEC_MDP, 64, 32, 1400, 4, 16, 0),
    (NFEC_MDP, 64, 32, 200, 4, 20, 12),
    (NFEC_MDP, 16, 4, 33, 6, 2, 2),
    (NFEC_MDP, 100, 100, 64, 3, 90, 10),    # m > 64: the locator prefix sums in dynamic LDS
    (NFEC_MDP, 50, 150, 40, 3, 50, 60),
]


@pytest.mark.parametrize("kind,k,m,vec,nb,es,ep", DEC_CASES)
def test_decode_matches_oracle(orc, kind, k, m, vec, nb, es, ep):
    enc, dec = _codecs(kind, k, m, vec)
    host = orc.encode_blocks(kind, k, m, vec, orc.make_blocks(k, m, vec, nb))
    locs, counts = _erasures(orc, kind, k, m, nb, es, ep)
    _erase(host, locs, counts)
    ref = host.copy()
    st_ref = orc.decode_blocks(kind, k, m, vec, ref, locs, counts)
    dev = torch.from_numpy(host).cuda()
    st = dec.decode_blocks(dev, torch.from_numpy(locs.astype(np.int16)).cuda(),
                           torch.from_numpy(counts.astype(np.int16)).cuda())
    torch.cuda.synchronize()
    assert np.array_equal(st.cpu().numpy(), st_ref)
    assert np.array_equal(dev.cpu().numpy(), ref)


def test_rs16_decode_layout_past_the_t3_offset_bound(orc):
    """RS16 decode stage 1 by the shared-table encode kernel needs every piece offset
    of an 8 KiB item group below 2^31 (t3_prepare).  A padded seg_stride past that bound must
    decode through the gather stage, not fail after the plan marked blocks for the encode path."""
    k, m, vec, nb, es = 40, 10, 64, 3, 6
    stride = 352 * 1024                       # 130 blocks x (50 x 352 KiB) > 2^31
    enc, dec = _codecs(NFEC_RS16, k, m, vec)
    host = orc.encode_blocks(NFEC_RS16, k, m, vec, orc.make_blocks(k, m, vec, nb, seg_stride=stride))
    locs, counts = _erasures(orc, NFEC_RS16, k, m, nb, es, 0)
    _erase(host, locs, counts)
    ref = host.copy()
    st_ref = orc.decode_blocks(NFEC_RS16, k, m, vec, ref, locs, counts)
    dev = torch.from_numpy(host).cuda()
    st = dec.decode_blocks(dev, torch.from_numpy(locs.astype(np.int16)).cuda(),
                           torch.from_numpy(counts.astype(np.int16)).cuda())
    torch.cuda.synchronize()
    assert np.array_equal(st.cpu().numpy(), st_ref) and (st_ref == es).all()
    assert np.array_equal(dev.cpu().numpy(), ref)


@pytest.mark.parametrize("kind", [NFEC_RS8, NFEC_RS16, NFEC_MDP])
def test_decode_shortened_blocks(orc, kind):
    k, m, vec, nb = 64, 16, 120, 6
    nd = np.array([40, 64, 1, 17, 63, 5], np.uint16)
    enc, dec = _codecs(kind, k, m, vec)
    host = orc.encode_blocks(kind, k, m, vec, orc.make_blocks(k, m, vec, nb, num_data=nd), nd)
    locs, counts = _erasures(orc, kind, k, m, nb, 12, 3, num_data=nd)
    _erase(host, locs, counts)
    ref = host.copy()
    st_ref = orc.decode_blocks(kind, k, m, vec, ref, locs, counts, nd)
    dev = torch.from_numpy(host).cuda()
    st = dec.decode_blocks(dev, torch.from_numpy(locs.astype(np.int16)).cuda(),
                           torch.from_numpy(counts.astype(np.int16)).cuda(),
                           num_data=torch.from_numpy(nd.astype(np.int16)).cuda())
    torch.cuda.synchronize()
    assert np.array_equal(st.cpu().numpy(), st_ref)
    assert np.array_equal(dev.cpu().numpy(), ref)


@pytest.mark.parametrize("kind", [NFEC_RS8, NFEC_RS16])
def test_decode_shortened_many_erasures_generic_plan(orc, kind):
    """RS8 and RS16 through the generic plan with 65..255 erasures per block and per-block
    numData: the log-domain elimination with its lists in the block's global scratch
    (min(k, m) > 64), shortened-block column offsets included."""
    k, m, vec, nb = 128, 127, 72, 4
    nd = np.array([128, 100, 90, 127], np.uint16)
    enc, dec = _codecs(kind, k, m, vec)
    host = orc.encode_blocks(kind, k, m, vec, orc.make_blocks(k, m, vec, nb, num_data=nd), nd)
    locs, counts = _erasures(orc, kind, k, m, nb, 90, 20, num_data=nd, seed_off=77)
    assert counts.min() >= 65 and counts.max() <= m
    _erase(host, locs, counts)
    ref = host.copy()
    st_ref = orc.decode_blocks(kind, k, m, vec, ref, locs, counts, nd)
    assert (st_ref == counts).all()
    dev = torch.from_numpy(host).cuda()
    st = dec.decode_blocks(dev, torch.from_numpy(locs.astype(np.int16)).cuda(),
                           torch.from_numpy(counts.astype(np.int16)).cuda(),
                           num_data=torch.from_numpy(nd.astype(np.int16)).cuda())
    torch.cuda.synchronize()
    assert np.array_equal(st.cpu().numpy(), st_ref)
    assert np.array_equal(dev.cpu().numpy(), ref)


@pytest.mark.parametrize("kind", [NFEC_RS8, NFEC_RS16])
def test_decode_accumulates_into_nonzero_erased_buffers(orc, kind):
    """Reference Decode XORs the repair into the erased buffer; with a non-zeroed buffer
    the output is junk ^ data, and the accumulate flag reproduces it byte for byte."""
    k, m, vec, nb = 32, 8, 96, 3
    enc, dec = _codecs(kind, k, m, vec)
    host = orc.encode_blocks(kind, k, m, vec, orc.make_blocks(k, m, vec, nb))
    locs, counts = _erasures(orc, kind, k, m, nb, 6, 1)
    rng = np.random.default_rng(7)
    for b in range(nb):
        for s in locs[b, : counts[b]]:
            host[b, s, :] = rng.integers(0, 256, vec, dtype=np.uint8)
    ref = host.copy()
    orc.decode_blocks(kind, k, m, vec, ref, locs, counts)
    dev = torch.from_numpy(host).cuda()
    dec.decode_blocks(dev, torch.from_numpy(locs.astype(np.int16)).cuda(),
                      torch.from_numpy(counts.astype(np.int16)).cuda(), accumulate=True)
    torch.cuda.synchronize()
    assert np.array_equal(dev.cpu().numpy(), ref)


def test_decode_rejects_undecodable_blocks(orc):
    """More erasures than parity, unsorted or out-of-range lists: status 0, block untouched."""
    k, m, vec = 16, 4, 64
    enc, dec = _codecs(NFEC_RS8, k, m, vec)
    host = orc.encode_blocks(NFEC_RS8, k, m, vec, orc.make_blocks(k, m, vec, 4))
    locs = np.zeros((4, 8), np.uint16)
    counts = np.array([5, 2, 2, 4], np.uint16)
    locs[0, :5] = [0, 1, 2, 3, 4]          # 5 erasures > 4 parity
    locs[1, :2] = [5, 3]                   # unsorted
    locs[2, :2] = [1, 30]                  # out of range slot
    locs[3, :4] = [0, 1, 16, 17]           # 2 source + 2 parity lost: decodable
    before = host.copy()
    dev = torch.from_numpy(host).cuda()
    st = dec.decode_blocks(dev, torch.from_numpy(locs.astype(np.int16)).cuda(),
                           torch.from_numpy(counts.astype(np.int16)).cuda())
    torch.cuda.synchronize()
    st = st.cpu().numpy()
    assert list(st[:3]) == [0, 0, 0] and st[3] == 4
    out = dev.cpu().numpy()
    assert np.array_equal(out[:3], before[:3])
    assert np.array_equal(out[3], before[3])  # nothing was erased, the repair rewrites the same bytes


@pytest.mark.parametrize("host", [False, True])
@pytest.mark.parametrize("kind", [NFEC_RS8, NFEC_RS16, NFEC_MDP])
def test_per_call_reference_surface(orc, kind, host):
    """Encode()/Decode() with scattered host vectors, exactly as fecTest drives them: the GPU
    round trip (host=False) and the host paths (the drop-in's defaults)."""
    k, m, vec = 20, 6, 64
    enc, dec = _codecs(kind, k, m, vec)
    blk = orc.make_blocks(k, m, vec, 1)[0]
    ref = orc.encode_blocks(kind, k, m, vec, blk[None].copy())[0]
    data = [bytearray(blk[s].tobytes()) for s in range(k)]
    parity = [bytearray(vec) for _ in range(m)]
    for s in range(k):
        enc.Encode(s, bytes(data[s]), parity, host=host)
    assert all(bytes(parity[i]) == ref[k + i].tobytes() for i in range(m))
    vecs = [bytearray(ref[s].tobytes()) for s in range(k + m)]
    erased = [1, 5, 6, k + 2]
    for s in erased:
        vecs[s] = bytearray(vec)
    vlist = list(vecs)
    vlist[k + 2] = None  # missing parity passed as NULL like NormObject
    assert dec.Decode(vlist, k, len(erased), erased, host=host) == len(erased)
    for s in range(k):
        assert bytes(vlist[s]) == ref[s].tobytes()


@pytest.mark.parametrize("host", [False, True])
@pytest.mark.parametrize("kind", [NFEC_RS8, NFEC_RS16])
@pytest.mark.parametrize("vec,nd,junk", [(64, 20, False), (64, 20, True), (66, 20, False), (64, 13, False),
                                          (1408, 20, True)])
def test_per_call_paths(orc, kind, vec, nd, junk, host):
    """The per-call Encode/Decode on the GPU (host=False) take the batch fast paths for a full
    block with zero-filled erased buffers (tower kernel / fused repair, overwrite) and the general
    ones otherwise: a shortened block (numData < k), non-zero erased buffers (the reference XORs
    the repair into them, normEncoderRS8.cpp:728-755), an odd-multiple vector size
    (vec % 8 != 0).  host=True: the same calls on the host paths."""
    k, m = 20, 6
    enc, dec = _codecs(kind, k, m, vec)
    blk = orc.make_blocks(k, m, vec, 1, num_data=np.array([nd], np.uint16))[0]
    ref = orc.encode_blocks(kind, k, m, vec, blk[None].copy(), np.array([nd], np.uint16))[0]
    parity = [bytearray(vec) for _ in range(m)]
    for s in range(nd):
        enc.Encode(s, blk[s, :vec].tobytes(), parity, host=host)
    assert all(bytes(parity[i]) == ref[nd + i, :vec].tobytes() for i in range(m))
    vecs = [bytearray(ref[s, :vec].tobytes()) for s in range(nd + m)]
    erased = [0, 3, nd - 1, nd + 1]
    rng = np.random.default_rng(7)
    noise = {}
    for s in erased:
        noise[s] = rng.integers(0, 256, vec, dtype=np.uint8).tobytes() if junk else bytes(vec)
        vecs[s] = bytearray(noise[s])
    assert dec.Decode(vecs, nd, len(erased), erased, host=host) == len(erased)
    nbytes = vec if kind == NFEC_RS8 else vec // 2 * 2
    for s in range(nd):
        want = bytearray(ref[s, :vec].tobytes())
        if s in noise:  # accumulate: repair XOR what the buffer held (odd RS16 last byte: untouched)
            n = np.frombuffer(noise[s], np.uint8)
            w = np.frombuffer(bytes(want), np.uint8).copy()
            w[:nbytes] ^= n[:nbytes]
            w[nbytes:] = n[nbytes:]
            want = bytearray(w.tobytes())
        assert bytes(vecs[s]) == bytes(want), s


def test_host_batch_paths_match_device(orc):
    k, m, vec, nb = 64, 32, 1400, 40
    enc, dec = _codecs(NFEC_RS8, k, m, vec)
    host = orc.make_blocks(k, m, vec, nb)
    ref = orc.encode_blocks(NFEC_RS8, k, m, vec, host.copy())
    enc.encode_blocks_host(host)
    assert np.array_equal(host, ref)
    locs, counts = _erasures(orc, NFEC_RS8, k, m, nb, 16, 2)
    _erase(host, locs, counts)
    st = dec.decode_blocks_host(host, locs, counts)
    assert np.all(st == counts)
    assert np.array_equal(host[:, :k], ref[:, :k])


@pytest.mark.parametrize("pinned", [False, True])
@pytest.mark.parametrize("kind,k,m,vec,stride,nb", [
    (NFEC_RS8, 64, 32, 1400, 1408, 1100),   # several pipeline chunks, padded slots
    (NFEC_RS8, 20, 12, 1000, 1000, 70),
    (NFEC_RS16, 30, 10, 998, 1000, 33),
    (NFEC_MDP, 24, 8, 600, 608, 50),
])
def test_host_batch_pipeline(orc, kind, k, m, vec, stride, nb, pinned, monkeypatch):
    """nfec_encode_host/nfec_decode_host over multi-chunk batches, pinned and pageable caller
    buffers: parity and repaired source match the oracle and slot padding is never written."""
    monkeypatch.setenv("NFEC_HOST_CHUNK_BLOCKS", str(max(1, nb // 4)))  # several pipeline chunks
    enc, dec = _codecs(kind, k, m, vec)
    base = orc.make_blocks(k, m, vec, nb, seg_stride=stride)
    base[:, :, vec:] = 0xA5
    ref = orc.encode_blocks(kind, k, m, vec, base.copy())
    if pinned:
        host = torch.empty(base.shape, dtype=torch.uint8).pin_memory().numpy()
        host[...] = base
    else:
        host = base.copy()
    host[:, k:, :vec] = 0x3C   # stale parity must be overwritten
    enc.encode_blocks_host(host)
    assert np.array_equal(host, ref)
    locs, counts = _erasures(orc, kind, k, m, nb, m - 3, 3)
    for b in range(nb):
        for s in locs[b, : counts[b]]:
            host[b, s, :vec] = 0
    st = dec.decode_blocks_host(host, locs, counts)
    assert np.all(st == counts)
    assert np.array_equal(host[:, :k], ref[:, :k])
    assert np.all(host[:, :, vec:] == 0xA5)


@pytest.mark.parametrize("pinned", [False, True])
@pytest.mark.parametrize("kind", [NFEC_RS8, NFEC_RS16, NFEC_MDP])
def test_host_decode_windows(orc, kind, pinned, monkeypatch):
    """RS host decode uploads only [0, the last parity slot a block of the chunk uses) and
    downloads [0, max numData).  Chunks with different windows (16 / 2 / 0 source erasures,
    parity erasures, shortened blocks, an undecodable block) take turns on the pipeline's device
    slots, so a window that is too short would decode from, or write back, another chunk's
    bytes.  Every byte the reference leaves alone must come back unchanged, including the
    unused parity slots, which hold garbage here (the decoder never reads them)."""
    k, m, vec, nb = 24, 16, 504, 48
    monkeypatch.setenv("NFEC_HOST_CHUNK_BLOCKS", "8")  # 6 chunks over the pipeline's slots
    _, dec = _codecs(kind, k, m, vec)
    nd = np.full(nb, k, np.uint16)
    nd[8:16] = [24, 5, 17, 24, 1, 9, 24, 12]
    host = orc.encode_blocks(kind, k, m, vec, orc.make_blocks(k, m, vec, nb, num_data=nd), nd)
    locs = np.zeros((nb, m), np.uint16)
    counts = np.zeros(nb, np.uint16)
    plan = [(16, 0), (3, 2), (2, 0), (0, 0), (5, 4), (15, 1)]  # (source, parity) erasures per chunk
    for b in range(nb):
        ns, npar = plan[b // 8]
        ns = min(ns, int(nd[b]))
        src = orc.erasure_pattern(b, int(nd[b]), ns) if ns else np.zeros(0, np.uint16)
        par = (int(nd[b]) + orc.erasure_pattern(b + 500, m, npar)).astype(np.uint16) if npar else np.zeros(0, np.uint16)
        allp = np.concatenate([src, par]).astype(np.uint16)
        counts[b] = len(allp)
        locs[b, :len(allp)] = allp
    counts[47] = m + 1  # undecodable (more erasures than parity): untouched, status 0
    _erase(host, locs, np.minimum(counts, m))
    ref = host.copy()
    st_ref = orc.decode_blocks(kind, k, m, vec, ref, locs, np.minimum(counts, m).astype(np.uint16), nd)
    st_ref[47] = 0
    ref[47] = host[47]
    if kind != NFEC_MDP:
        # garbage in the parity slots no decode reads (past the first e surviving parities)
        for b in range(nb):
            n = int(nd[b])
            es = int(np.sum(locs[b, :min(counts[b], m)] < n))
            er = set(int(x) for x in locs[b, :min(counts[b], m)])
            used = 0
            for v in range(n, n + m):
                if v in er:
                    continue
                if used >= es or b == 47:
                    host[b, v, :vec] = 0x77
                    ref[b, v, :vec] = 0x77
                used += 1
    if pinned:
        buf = torch.empty(host.shape, dtype=torch.uint8).pin_memory().numpy()
        buf[...] = host
        host = buf
    st = dec.decode_blocks_host(host, locs, counts, num_data=nd)
    assert np.array_equal(st, st_ref)
    assert np.array_equal(host, ref)


def test_device_workload_generators_match_oracle(orc):
    k, m, vec, nb = 64, 32, 1400, 9
    dev = torch.zeros((nb, k + m, 1400), dtype=torch.uint8, device="cuda")
    fill_blocks(dev, k, vec, orc.SEED, first_block=100)
    locs, counts = make_erasures(nb, k, 16, orc.SEED, m, first_block=100)
    torch.cuda.synchronize()
    host = orc.make_blocks(k, m, vec, nb, first_block=100)
    assert np.array_equal(dev.cpu().numpy(), host)
    for b in range(nb):
        assert counts[b].item() == 16
        assert np.array_equal(locs[b, :16].cpu().numpy().astype(np.uint16), orc.erasure_pattern(100 + b, k, 16))


def test_full_size_roundtrip_c2_c3(orc):
    """BASELINE C2/C3 at full size: 65,536 blocks of RS8(64,32) x 1400 B in HBM.
    Size-independent properties: erase 16 random source symbols per block, decode, and every
    byte of every block must equal the pre-erasure bytes; sampled blocks' parity must equal
    the oracle's."""
    k, m, vec, nb = 64, 32, 1400, 65536
    enc, dec = _codecs(NFEC_RS8, k, m, vec)
    blocks = torch.zeros((nb, k + m, vec), dtype=torch.uint8, device="cuda")
    fill_blocks(blocks, k, vec, orc.SEED)
    enc.encode_blocks(blocks)
    torch.cuda.synchronize()
    for b in (0, 1, 4097, 65535):
        ref = orc.encode_blocks(NFEC_RS8, k, m, vec, orc.make_blocks(k, m, vec, 1, first_block=b))
        assert np.array_equal(blocks[b].cpu().numpy(), ref[0])
    keep = blocks.clone()
    locs, counts = make_erasures(nb, k, 16, orc.SEED, m)
    zero_erasures(blocks, locs, counts, vec)
    assert not torch.equal(blocks, keep)
    st = dec.decode_blocks(blocks, locs, counts)
    torch.cuda.synchronize()
    assert bool((st == 16).all())
    assert torch.equal(blocks, keep)


@pytest.mark.parametrize("m", [32, 16, 8])
@pytest.mark.parametrize("accumulate", [False, True])
def test_fused_decode_mixed_batch(orc, m, accumulate):
    """The fused per-block repair (gen_fdec_asm.hip) takes blocks with e <= 16 repaired from
    parity rows 0..e-1; the unfused kernels take the rest of the same batch.  Mix both kinds:
    1..16 source erasures, every third block also losing parity rows among the first ones,
    and (accumulate) junk in the erased buffers XORed into the repair."""
    k, vec, nb = 64, 1400, 48
    enc, dec = _codecs(NFEC_RS8, k, m, vec)
    clean = orc.encode_blocks(NFEC_RS8, k, m, vec, orc.make_blocks(k, m, vec, nb))
    rng = np.random.default_rng(21)
    locs = np.zeros((nb, m), np.uint16)
    counts = np.zeros(nb, np.uint16)
    for b in range(nb):
        es = 1 + b % min(16, m)
        src = np.sort(rng.choice(k, es, replace=False))
        par = k + np.sort(rng.choice(4, 2, replace=False)) if b % 3 == 0 and es + 2 <= m else np.array([], int)
        e = np.concatenate([src, par]).astype(np.uint16)
        locs[b, :len(e)] = e
        counts[b] = len(e)
    rx = clean.copy()
    for b in range(nb):
        for s in locs[b, :counts[b]]:
            rx[b, s] = rng.integers(0, 256, vec, dtype=np.uint8) if (accumulate and s < k) else 0
    ref = rx.copy()
    st_ref = orc.decode_blocks(NFEC_RS8, k, m, vec, ref, locs, counts)
    if accumulate:  # reference contract: repair XORs into the erased buffers
        expect = rx.copy()
        for b in range(nb):
            for s in locs[b, :counts[b]]:
                if s < k:
                    expect[b, s] ^= clean[b, s]
    else:
        expect = ref
    dev = torch.from_numpy(rx).cuda()
    st = dec.decode_blocks(dev, torch.from_numpy(locs.astype(np.int16)).cuda(),
                           torch.from_numpy(counts.astype(np.int16)).cuda(), accumulate=accumulate)
    torch.cuda.synchronize()
    assert np.array_equal(st.cpu().numpy(), st_ref)
    assert np.array_equal(dev.cpu().numpy(), expect)


@pytest.mark.parametrize("m,ne", [(32, 16), (32, 24), (16, 16), (16, 9), (8, 8), (8, 5)])
def test_fused_decode_random_loss(orc, m, ne):
    """NORM loses source and parity segments alike: ne erasures drawn uniformly over all k + m
    slots.  The fused kernel takes every block whose substitute parities (the first e surviving
    rows, reference scan normEncoderRS8.cpp:660-718) lie below min(16, m) -- for m <= 16 all of
    them -- with the inverse written by parity row; the rest go unfused.  Bytes and statuses
    must match the reference decode."""
    k, vec, nb = 64, 1400, 96
    enc, dec = _codecs(NFEC_RS8, k, m, vec)
    clean = orc.encode_blocks(NFEC_RS8, k, m, vec, orc.make_blocks(k, m, vec, nb))
    rng = np.random.default_rng(1000 + 10 * m + ne)
    locs = np.zeros((nb, m), np.uint16)
    counts = np.full(nb, ne, np.uint16)
    for b in range(nb):
        locs[b, :ne] = np.sort(rng.choice(k + m, ne, replace=False))
    rx = clean.copy()
    _erase(rx, locs, counts)
    ref = rx.copy()
    st_ref = orc.decode_blocks(NFEC_RS8, k, m, vec, ref, locs, counts)
    dev = torch.from_numpy(rx).cuda()
    st = dec.decode_blocks(dev, torch.from_numpy(locs.astype(np.int16)).cuda(),
                           torch.from_numpy(counts.astype(np.int16)).cuda())
    torch.cuda.synchronize()
    assert np.array_equal(st.cpu().numpy(), st_ref)
    assert np.array_equal(dev.cpu().numpy(), ref)
    assert np.array_equal(ref[:, :k], clean[:, :k])


@pytest.mark.parametrize("m,codeword", [(32, True), (32, False), (16, True), (16, False)])
def test_mdp_snippet_solve(orc, m, codeword):
    """MDP decode through the bit-sliced snippet solve (gen_solve_asm.hip, blocks with <= 16
    erased source vectors and <= 96 survivors) and, for the rest of the batch, the generic
    kernel.  Erasures over source and parity, shortened blocks, and (codeword=False) survivors
    that are not a codeword: the reference's syndrome / Forney chain is a fixed linear map of
    all survivors, so the bytes must match it for any input."""
    k, vec, nb = 64, 1400, 40
    _, dec = _codecs(NFEC_MDP, k, m, vec)
    nd = np.full(nb, k, np.uint16)
    nd[5], nd[17], nd[30] = 40, 9, 63
    blocks = orc.make_blocks(k, m, vec, nb, num_data=nd)
    if codeword:
        blocks = orc.encode_blocks(NFEC_MDP, k, m, vec, blocks, nd)
    else:
        rng0 = np.random.default_rng(5)
        for b in range(nb):
            blocks[b, : int(nd[b]) + m] = rng0.integers(0, 256, (int(nd[b]) + m, vec), dtype=np.uint8)
    rng = np.random.default_rng(77 + m)
    locs = np.zeros((nb, m), np.uint16)
    counts = np.zeros(nb, np.uint16)
    for b in range(nb):
        n = int(nd[b]) + m
        ne = min(m, 1 + b % 20)  # 1..20 erasures: e > 16 source ones go to the generic kernel
        locs[b, :ne] = np.sort(rng.choice(n, ne, replace=False))
        counts[b] = ne
    _erase(blocks, locs, counts)
    ref = blocks.copy()
    st_ref = orc.decode_blocks(NFEC_MDP, k, m, vec, ref, locs, counts, nd)
    dev = torch.from_numpy(blocks).cuda()
    st = dec.decode_blocks(dev, torch.from_numpy(locs.astype(np.int16)).cuda(),
                           torch.from_numpy(counts.astype(np.int16)).cuda(),
                           num_data=torch.from_numpy(nd.astype(np.int16)).cuda())
    torch.cuda.synchronize()
    assert np.array_equal(st.cpu().numpy(), st_ref)
    assert np.array_equal(dev.cpu().numpy(), ref)


@pytest.mark.parametrize("m", [32, 8])
def test_unfused_gate_across_calls(orc, m):
    """The unfused stage 1 + solve run only when the plan opened this call's gate word (some
    block the fused kernel does not take).  One decoder, three calls in a row: a batch with
    unfused blocks, an all-fused batch (the word still holds the first call's generation),
    then a batch whose only unfused block is the last one."""
    k, vec, nb = 64, 1400, 40
    enc, dec = _codecs(NFEC_RS8, k, m, vec)
    clean = orc.encode_blocks(NFEC_RS8, k, m, vec, orc.make_blocks(k, m, vec, nb))
    rng = np.random.default_rng(5)

    def run(unfused):
        locs = np.zeros((nb, m), np.uint16)
        counts = np.zeros(nb, np.uint16)
        for b in range(nb):
            es = 1 + b % min(8, m - 1)
            src = np.sort(rng.choice(k, es, replace=False))
            # losing parity row 0 sends the block to the unfused kernels
            par = np.array([k], int) if b in unfused else np.array([], int)
            e = np.concatenate([src, par]).astype(np.uint16)
            locs[b, :len(e)] = e
            counts[b] = len(e)
        rx = clean.copy()
        for b in range(nb):
            rx[b, locs[b, :counts[b]]] = 0
        ref = rx.copy()
        st_ref = orc.decode_blocks(NFEC_RS8, k, m, vec, ref, locs, counts)
        dev = torch.from_numpy(rx).cuda()
        st = dec.decode_blocks(dev, torch.from_numpy(locs.astype(np.int16)).cuda(),
                               torch.from_numpy(counts.astype(np.int16)).cuda())
        torch.cuda.synchronize()
        assert np.array_equal(st.cpu().numpy(), st_ref)
        assert np.array_equal(dev.cpu().numpy(), ref)
        assert np.array_equal(dev.cpu().numpy()[:, :k], clean[:, :k])

    run({0, 7, 19})
    run(set())
    run({nb - 1})


@pytest.mark.parametrize("pinned", [True, False])
@pytest.mark.parametrize("bad_nd", [0, 65])
def test_host_decode_rejects_bad_num_data(orc, pinned, bad_nd):
    """a host batch whose numData list holds 0 or a count past k fails with NFEC_EINVAL before
    any slot moves (the zero-copy slot moves size their copies by numData + m), and leaves the
    caller's buffer alone, pinned or pageable"""
    import norm_amd as na
    from norm_amd import _native as N

    k, m, vec, nb = 64, 32, 1400, 8
    dec = na.NormDecoderRS8()
    assert dec.Init(k, m, vec)
    host = orc.make_blocks(k, m, vec, nb)
    if pinned:
        t = torch.empty(host.shape, dtype=torch.uint8, pin_memory=True)
        t.copy_(torch.from_numpy(host))
        arr = t.numpy()
    else:
        arr = host.copy()
    before = arr.copy()
    nd = np.full(nb, k, np.uint16)
    nd[nb - 1] = bad_nd
    locs = np.zeros((nb, m), np.uint16)
    counts = np.ones(nb, np.uint16)
    with pytest.raises(N.NfecError):
        dec.decode_blocks_host(arr, locs, counts, num_data=nd)
    assert np.array_equal(arr, before)
