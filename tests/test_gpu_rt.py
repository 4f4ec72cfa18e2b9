"""The runtime-coefficient RS8 kernel (gen_rs8_rt.hip) against the oracle, bit-exact: every RS8
shape the fixed (64, m) kernels do not cover and every shortened batch goes through it
(NormEncoderRS8::Encode, src/common/normEncoderRS8.cpp:473-483, for k + m <= 255; shortened
blocks stop at numData, parity at slot numData + r -- run flat, each 8-byte piece masked by its
own block's numData), the one-pass repair of those shapes (Decode, :652-757: the plan's closed-form
e x numData map, then one product; blocks of up to 8 rows on one wave, larger on two), and MDP
blocks of other shapes or lengths (normEncoderMDP.cpp:178-211).  Shapes pick each work split:
m <= 8 one wave per item group, m <= 16 two waves sharing columns, more four (and several pass
sets past 32 rows, looped inside the workgroup); segments longer than one 2 KiB item group;
padded strides; accumulate."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from norm_amd import NFEC_MDP, NFEC_RS8, NormDecoderRS8, NormEncoderMDP, NormEncoderRS8  # noqa: E402


def _enc(kind, k, m, vec):
    e = (NormEncoderRS8 if kind == NFEC_RS8 else NormEncoderMDP)()
    assert e.Init(k, m, vec)
    return e


FLAT = [
    # k, m, vec, seg_stride, nblocks
    (16, 4, 1400, 1400, 97),      # G = 1
    (8, 2, 1408, 1408, 301),
    (32, 16, 1400, 1400, 53),     # G = 2
    (32, 9, 64, 64, 40),          # G = 2, odd row split
    (128, 32, 1400, 1408, 11),    # G = 4
    (200, 55, 1400, 1400, 7),     # two pass sets
    (64, 48, 4096, 4096, 5),      # two item groups per segment
    (100, 3, 8, 8, 700),          # many blocks per item group
    (3, 100, 1400, 1400, 6),      # m > k
    (127, 128, 72, 72, 3),        # k + m = 255, 16 pass sets
    (64, 20, 1400, 1400, 64),     # not a fixed-kernel shape at k = 64
]


@pytest.mark.parametrize("k,m,vec,stride,nb", FLAT)
def test_rt_encode_flat(orc, k, m, vec, stride, nb):
    enc = _enc(NFEC_RS8, k, m, vec)
    host = orc.make_blocks(k, m, vec, nb, seg_stride=stride)
    host[:, k:, :] = 0xA5  # overwrite semantics
    ref = orc.encode_blocks(NFEC_RS8, k, m, vec, host.copy())
    dev = torch.from_numpy(host).cuda()
    enc.encode_blocks(dev)
    torch.cuda.synchronize()
    assert np.array_equal(dev.cpu().numpy(), ref)


SHORT = [
    # kind, k, m, vec, nblocks
    (NFEC_RS8, 64, 32, 1400, 300),   # the fixed shape, shortened: per-block mode
    (NFEC_RS8, 64, 16, 1408, 97),
    (NFEC_RS8, 200, 55, 136, 9),
    (NFEC_RS8, 16, 4, 4104, 13),     # three item groups per segment
    (NFEC_MDP, 64, 32, 1400, 41),
    (NFEC_MDP, 30, 20, 200, 17),
]


@pytest.mark.parametrize("kind,k,m,vec,nb", SHORT)
def test_rt_encode_shortened(orc, kind, k, m, vec, nb):
    rng = np.random.default_rng(k + m + nb)
    nd = rng.integers(1, k + 1, nb).astype(np.uint16)
    nd[0], nd[-1] = k, 1
    enc = _enc(kind, k, m, vec)
    host = orc.make_blocks(k, m, vec, nb, num_data=nd)
    ref = orc.encode_blocks(kind, k, m, vec, host.copy(), nd)
    dev = torch.from_numpy(host).cuda()
    enc.encode_blocks(dev, num_data=torch.from_numpy(nd.view(np.int16)).cuda())
    torch.cuda.synchronize()
    assert np.array_equal(dev.cpu().numpy(), ref)


@pytest.mark.parametrize("k,m,vec,nb,short", [(16, 4, 1400, 33, False), (128, 40, 1400, 5, False),
                                             (64, 32, 1400, 20, True)])
def test_rt_encode_accumulates(orc, k, m, vec, nb, short):
    rng = np.random.default_rng(3)
    nd = rng.integers(1, k + 1, nb).astype(np.uint16) if short else None
    enc = _enc(NFEC_RS8, k, m, vec)
    host = orc.make_blocks(k, m, vec, nb, num_data=nd)
    ref = orc.encode_blocks(NFEC_RS8, k, m, vec, host.copy(), nd)
    junk = rng.integers(0, 256, host.shape, dtype=np.uint8)
    expect = ref.copy()
    for b in range(nb):
        n = k if nd is None else int(nd[b])
        host[b, n:n + m] = junk[b, n:n + m]
        expect[b, n:n + m] = ref[b, n:n + m] ^ junk[b, n:n + m]
    dev = torch.from_numpy(host).cuda()
    enc.encode_blocks(dev, num_data=None if nd is None else torch.from_numpy(nd.view(np.int16)).cuda(),
                      accumulate=True)
    torch.cuda.synchronize()
    assert np.array_equal(dev.cpu().numpy(), expect)


def test_rt_round_trip_sweep_shapes(orc):
    """the rs8sweep shapes at a few thousand blocks: encode, erase, repair, every byte back"""
    for k, m, er in [(16, 4, 4), (32, 16, 16), (128, 32, 16), (200, 55, 16), (8, 2, 2)]:
        nb = max(64, 200000 // (k + m))
        enc = _enc(NFEC_RS8, k, m, 1400)
        dec = NormDecoderRS8()
        assert dec.Init(k, m, 1400)
        import norm_amd as na

        blocks = torch.zeros((nb, k + m, 1400), dtype=torch.uint8, device="cuda")
        na.fill_blocks(blocks, k, 1400, 0x77)
        enc.encode_blocks(blocks)
        keep = blocks.clone()
        locs, counts = na.make_erasures(nb, k, er, 0x99, m)
        na.zero_erasures(blocks, locs, counts, 1400)
        st = dec.decode_blocks(blocks, locs, counts)
        torch.cuda.synchronize()
        assert bool((st == er).all()) and torch.equal(blocks, keep), (k, m)
        # sampled blocks against the oracle's parity
        sample = keep[:3].cpu().numpy()
        ref = orc.encode_blocks(NFEC_RS8, k, m, 1400, sample.copy())
        assert np.array_equal(sample, ref), (k, m)


DEC = [
    # k, m, vec, nblocks, source erasures, parity erasures, shortened
    (16, 4, 1400, 31, 3, 1, False),
    (32, 16, 1408, 17, 10, 6, False),
    (128, 32, 1400, 9, 20, 5, False),
    (200, 55, 136, 7, 40, 10, True),
    (64, 32, 1400, 40, 16, 0, True),      # the headline shape, shortened: the one-pass runtime-coefficient repair
    (3, 100, 64, 9, 3, 50, False),        # m > k
    (127, 128, 72, 3, 100, 27, False),    # e = 100: four waves, several pass sets per stage
    (64, 20, 4096, 5, 12, 3, False),      # two item groups per segment
    (10, 7, 8, 200, 7, 0, False),         # e = m, one piece per segment
]


@pytest.mark.parametrize("k,m,vec,nb,es,ep,short", DEC)
def test_rt_decode_matches_oracle(orc, k, m, vec, nb, es, ep, short):
    rng = np.random.default_rng(k * 7 + m)
    nd = rng.integers(max(1, es), k + 1, nb).astype(np.uint16) if short else np.full(nb, k, np.uint16)
    host = orc.make_blocks(k, m, vec, nb, num_data=nd if short else None)
    clean = orc.encode_blocks(NFEC_RS8, k, m, vec, host, nd if short else None)
    locs = np.zeros((nb, m), np.uint16)
    counts = np.zeros(nb, np.uint16)
    rx = clean.copy()
    for b in range(nb):
        n = int(nd[b])
        e = np.sort(np.concatenate([rng.choice(n, min(es, n), replace=False),
                                    n + rng.choice(m, ep, replace=False)]))[:m]
        counts[b] = len(e)
        locs[b, :len(e)] = e
        for s in e:
            rx[b, s] = 0
    ref = rx.copy()
    st_ref = orc.decode_blocks(NFEC_RS8, k, m, vec, ref, locs, counts, nd if short else None)
    dec = NormDecoderRS8()
    assert dec.Init(k, m, vec)
    dev = torch.from_numpy(rx).cuda()
    st = dec.decode_blocks(dev, torch.from_numpy(locs.view(np.int16)).cuda(),
                           torch.from_numpy(counts.view(np.int16)).cuda(),
                           num_data=torch.from_numpy(nd.view(np.int16)).cuda() if short else None)
    torch.cuda.synchronize()
    assert np.array_equal(st.cpu().numpy(), st_ref)
    assert np.array_equal(dev.cpu().numpy(), ref)


def test_rt_decode_accumulates(orc):
    """erased buffers that are not zero: the repair XORs into them, as the reference's addmul does"""
    k, m, vec, nb = 32, 16, 1400, 6
    clean = orc.encode_blocks(NFEC_RS8, k, m, vec, orc.make_blocks(k, m, vec, nb))
    rng = np.random.default_rng(2)
    locs = np.zeros((nb, m), np.uint16)
    counts = np.full(nb, 9, np.uint16)
    rx = clean.copy()
    for b in range(nb):
        e = np.sort(rng.choice(k, 9, replace=False))
        locs[b, :9] = e
        rx[b, e] = rng.integers(0, 256, (9, vec), dtype=np.uint8)
    ref = rx.copy()
    st_ref = orc.decode_blocks(NFEC_RS8, k, m, vec, ref, locs, counts)
    dec = NormDecoderRS8()
    assert dec.Init(k, m, vec)
    dev = torch.from_numpy(rx).cuda()
    st = dec.decode_blocks(dev, torch.from_numpy(locs.view(np.int16)).cuda(),
                           torch.from_numpy(counts.view(np.int16)).cuda(), accumulate=True)
    torch.cuda.synchronize()
    assert np.array_equal(st.cpu().numpy(), st_ref) and np.array_equal(dev.cpu().numpy(), ref)


def test_rt_decode_blocks_without_erasures(orc):
    """blocks with nothing to repair (e = 0) beside ones with erasures: the plan writes no slot
    list or table for them, so the repair must not read any (tests/test_gpu_random.py seed 24)"""
    k, m, vec, nb = 77, 134, 1408, 40
    clean = orc.encode_blocks(NFEC_RS8, k, m, vec, orc.make_blocks(k, m, vec, nb))
    rng = np.random.default_rng(24)
    locs = np.zeros((nb, m), np.uint16)
    counts = np.zeros(nb, np.uint16)
    rx = clean.copy()
    for b in range(0, nb, 2):
        e = np.sort(rng.choice(k, 1 + b % 70, replace=False))
        locs[b, :len(e)] = e
        counts[b] = len(e)
        rx[b, e] = 0
    ref = rx.copy()
    st_ref = orc.decode_blocks(NFEC_RS8, k, m, vec, ref, locs, counts)
    dec = NormDecoderRS8()
    assert dec.Init(k, m, vec)
    dev = torch.from_numpy(rx).cuda()
    st = dec.decode_blocks(dev, torch.from_numpy(locs.view(np.int16)).cuda(),
                           torch.from_numpy(counts.view(np.int16)).cuda())
    torch.cuda.synchronize()
    assert np.array_equal(st.cpu().numpy(), st_ref) and np.array_equal(dev.cpu().numpy(), ref)


@pytest.mark.parametrize("k,m,vec,nb", [(16, 4, 1400, 200), (64, 16, 1408, 50), (100, 3, 8, 700)])
def test_rt_encode_shortened_flat_bad_counts(orc, k, m, vec, nb):
    """RS8 shortened batches run flat (item groups across blocks, each lane's pieces stopping at
    their block's numData); a block whose numData is 0 or past k is left untouched, as the
    per-block mode leaves it"""
    rng = np.random.default_rng(vec + nb)
    nd = rng.integers(1, k + 1, nb).astype(np.uint16)
    bad = rng.choice(nb, max(2, nb // 10), replace=False)
    nd_dev = nd.copy()
    nd_dev[bad[: len(bad) // 2]] = 0
    nd_dev[bad[len(bad) // 2:]] = k + 1
    enc = _enc(NFEC_RS8, k, m, vec)
    host = orc.make_blocks(k, m, vec, nb, num_data=nd)
    ref = orc.encode_blocks(NFEC_RS8, k, m, vec, host.copy(), nd)
    ref[bad] = host[bad]
    dev = torch.from_numpy(host).cuda()
    enc.encode_blocks(dev, num_data=torch.from_numpy(nd_dev.view(np.int16)).cuda())
    torch.cuda.synchronize()
    assert np.array_equal(dev.cpu().numpy(), ref)


@pytest.mark.parametrize("k,m,vec,nb,short", [(40, 20, 1400, 300, False), (100, 30, 2056, 60, True),
                                              (64, 32, 1400, 200, True)])
def test_rt_decode_mixed_erasure_counts(orc, k, m, vec, nb, short):
    """one batch whose blocks need 0..m rows: the repair runs blocks of up to 8 rows on one wave
    and larger ones on two (two launches, each skipping the other's blocks), a block with
    nothing to repair is left alone, and every byte matches the oracle"""
    rng = np.random.default_rng(k * 3 + nb)
    nd = rng.integers(max(1, m // 2), k + 1, nb).astype(np.uint16) if short else np.full(nb, k, np.uint16)
    host = orc.make_blocks(k, m, vec, nb, num_data=nd if short else None)
    clean = orc.encode_blocks(NFEC_RS8, k, m, vec, host, nd if short else None)
    locs = np.zeros((nb, m), np.uint16)
    counts = np.zeros(nb, np.uint16)
    rx = clean.copy()
    for b in range(nb):
        n = int(nd[b])
        es = int(rng.integers(0, min(n, m) + 1))        # 0 .. m source erasures
        ep = int(rng.integers(0, m - es + 1)) if b % 3 == 0 else 0
        e = np.sort(np.concatenate([rng.choice(n, es, replace=False), n + rng.choice(m, ep, replace=False)]))
        e = e.astype(np.uint16)[:m]
        counts[b] = len(e)
        locs[b, :len(e)] = e
        for s in e:
            rx[b, s] = 0
    counts[0] = 0  # nothing to repair
    locs[0] = 0
    rx[0] = clean[0]
    ref = rx.copy()
    st_ref = orc.decode_blocks(NFEC_RS8, k, m, vec, ref, locs, counts, nd if short else None)
    dec = NormDecoderRS8()
    assert dec.Init(k, m, vec)
    dev = torch.from_numpy(rx).cuda()
    st = dec.decode_blocks(dev, torch.from_numpy(locs.view(np.int16)).cuda(),
                           torch.from_numpy(counts.view(np.int16)).cuda(),
                           num_data=torch.from_numpy(nd.view(np.int16)).cuda() if short else None)
    torch.cuda.synchronize()
    assert np.array_equal(st.cpu().numpy(), st_ref)
    assert np.array_equal(dev.cpu().numpy(), ref)
