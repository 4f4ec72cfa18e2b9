"""RS16 on the tower kernel beyond the unshortened, source-loss case (round 5), bit-exact against
the oracle: lost parity (NORM loses source and parity alike, so the substitute parities are the
first SURVIVING rows, normEncoderRS16.cpp:696-709), shortened blocks (every object's last block,
:675-693, normObject.cpp:203-231), accumulate into non-zero erased buffers (:739-745 XOR the
repair in), and vector sizes that are not multiples of 8 (NORM codes segmentSize + 8 bytes,
normSession.cpp:883, e.g. 1452 -> 1460; RS16 codes vec / 2 symbols and never touches an odd
last byte, :479).  Encode: NormEncoderRS16::Encode (:472-482) per source segment."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from norm_amd import NFEC_RS16, NormDecoderRS16, NormEncoderRS16  # noqa: E402


def _codecs(k, m, vec):
    enc, dec = NormEncoderRS16(), NormDecoderRS16()
    assert enc.Init(k, m, vec) and dec.Init(k, m, vec)
    return enc, dec


def _stride(vec):
    return (vec + 7) // 8 * 8


def _i16(a):
    return torch.from_numpy(np.ascontiguousarray(a).astype(np.uint16).view(np.int16)).cuda()


@pytest.mark.parametrize("k,m,vec,nb", [
    (400, 100, 1400, 6),   # the C5 RS16 block type
    (40, 12, 72, 9),       # one row past a full tower pass
    (100, 20, 1460, 5),    # shortened and a 4-byte tail per segment
    (16, 4, 6, 7),         # vector shorter than one 8-byte piece: tail kernel only
])
def test_rs16_shortened_encode(orc, k, m, vec, nb):
    """numData drawn per block in [1, k]: columns past it read as zero, parity at numData + r"""
    rng = np.random.default_rng(k * 31 + vec)
    nd = rng.integers(1, k + 1, nb).astype(np.uint16)
    nd[0] = k  # a full block beside shortened ones
    host = orc.make_blocks(k, m, vec, nb, seg_stride=_stride(vec), num_data=nd)
    # junk past each block's parity (slots nd + m ..): never read, never written
    for b in range(nb):
        host[b, nd[b] + m:, :] = rng.integers(0, 256, (k - nd[b], host.shape[2]), dtype=np.uint8)
    ref = orc.encode_blocks(NFEC_RS16, k, m, vec, host.copy(), num_data=nd)
    enc, _ = _codecs(k, m, vec)
    dev = torch.from_numpy(host).cuda()
    enc.encode_blocks(dev, num_data=_i16(nd))
    torch.cuda.synchronize()
    assert np.array_equal(dev.cpu().numpy(), ref)


@pytest.mark.parametrize("k,m,vec,stride", [
    (100, 20, 1460, 1464),   # 1452-byte segments + 8: 2 tail symbols
    (64, 11, 1402, 1408),    # 1 tail symbol
    (40, 12, 1406, 1416),    # 3 tail symbols, padded stride
    (30, 8, 1461, 1464),     # odd vector: 1460 bytes coded, the last byte untouched
])
def test_rs16_encode_ragged_vectors(orc, k, m, vec, stride):
    nb = 5
    host = orc.make_blocks(k, m, vec, nb, seg_stride=stride)
    host[:, k:, :] = 0x5A   # parity slots (and the odd last byte) hold junk before the encode
    ref = orc.encode_blocks(NFEC_RS16, k, m, vec, host.copy())
    ref[:, k:, vec & ~1:] = 0x5A   # (the oracle zero-fills the whole parity vector first, as NORM does)
    enc, _ = _codecs(k, m, vec)
    dev = torch.from_numpy(host).cuda()
    enc.encode_blocks(dev)
    torch.cuda.synchronize()
    assert np.array_equal(dev.cpu().numpy(), ref)


@pytest.mark.parametrize("short", [False, True])
def test_rs16_encode_accumulates(orc, short):
    """accumulate: parity ^= the block's products (the reference's Encode adds into the parity
    buffers, normEncoderRS16.cpp:480)"""
    k, m, vec, nb = 60, 13, 1460, 4
    rng = np.random.default_rng(11)
    nd = rng.integers(1, k + 1, nb).astype(np.uint16) if short else None
    host = orc.make_blocks(k, m, vec, nb, seg_stride=_stride(vec), num_data=nd)
    clean = orc.encode_blocks(NFEC_RS16, k, m, vec, host.copy(), num_data=nd)
    junk = rng.integers(0, 256, host.shape, dtype=np.uint8)
    ref = clean.copy()
    for b in range(nb):
        n = k if nd is None else int(nd[b])
        host[b, n:n + m] = junk[b, n:n + m]
        ref[b, n:n + m, :vec & ~1] = clean[b, n:n + m, :vec & ~1] ^ junk[b, n:n + m, :vec & ~1]
        ref[b, n:n + m, vec & ~1:] = junk[b, n:n + m, vec & ~1:]
    enc, _ = _codecs(k, m, vec)
    dev = torch.from_numpy(host).cuda()
    enc.encode_blocks(dev, num_data=_i16(nd) if short else None, accumulate=True)
    torch.cuda.synchronize()
    assert np.array_equal(dev.cpu().numpy(), ref)


def _uniform_erasures(rng, nd, k, m, counts):
    nb = len(counts)
    locs = np.zeros((nb, m + 1), np.uint16)   # (room for one more than m: an undecodable list)
    for b, e in enumerate(counts):
        e = min(e, int(nd[b]) + m)
        pick = np.sort(rng.choice(int(nd[b]) + m, e, replace=False))
        locs[b, :e] = pick
        counts[b] = e
    return locs, np.asarray(counts, np.uint16)


def _decode_case(orc, k, m, vec, nd, counts, accumulate, seed, short):
    """encode (oracle), erase uniformly over numData + m slots; erased slots (source and parity)
    hold junk.  Reference: Decode with the erased source zeroed (overwrite) or holding the junk
    (accumulate: the repair is XORed in)."""
    nb = len(counts)
    rng = np.random.default_rng(seed)
    host = orc.encode_blocks(NFEC_RS16, k, m, vec,
                             orc.make_blocks(k, m, vec, nb, seg_stride=_stride(vec), num_data=nd if short else None),
                             num_data=nd if short else None)
    locs, cnt = _uniform_erasures(rng, nd, k, m, list(counts))
    ref = host.copy()
    for b in range(nb):
        for s in locs[b, :cnt[b]]:
            junk = rng.integers(0, 256, host.shape[2], dtype=np.uint8)
            host[b, s] = junk
            ref[b, s] = junk
            if not accumulate and s < nd[b]:
                ref[b, s, :vec & ~1] = 0   # NORM's zero-fill (the odd last byte is never coded)
    st_ref = orc.decode_blocks(NFEC_RS16, k, m, vec, ref, locs, cnt, num_data=nd if short else None)
    _, dec = _codecs(k, m, vec)
    dev = torch.from_numpy(host).cuda()
    st = dec.decode_blocks(dev, _i16(locs), _i16(cnt), num_data=_i16(nd) if short else None, accumulate=accumulate)
    torch.cuda.synchronize()
    got = dev.cpu().numpy()
    assert np.array_equal(st.cpu().numpy(), st_ref)
    # Decode writes the erased source of decodable blocks only (erased parity keeps its junk);
    # an undecodable block is left as it came
    want = host.copy()
    for b in range(nb):
        if st_ref[b] > 0:
            want[b, :nd[b]] = ref[b, :nd[b]]
    assert np.array_equal(got, want)


@pytest.mark.parametrize("k,m,vec", [(400, 100, 1400), (40, 12, 72), (100, 20, 1460), (12, 30, 64), (30, 8, 1461)])
@pytest.mark.parametrize("accumulate", [False, True])
def test_rs16_decode_uniform_loss(orc, k, m, vec, accumulate):
    """erasures over all k + m segments: lost parity shifts the substitutes to the next
    surviving rows; e from 0 to beyond m in one batch (the last one undecodable)"""
    counts = [min(k, m) // 2, 0, 1, m, min(k, m), m // 3, m + 1 if m + 1 <= k + m else m]
    nd = np.full(len(counts), k, np.uint16)
    _decode_case(orc, k, m, vec, nd, counts, accumulate, seed=k + m + vec, short=False)


@pytest.mark.parametrize("k,m,vec", [(400, 100, 1400), (40, 12, 72), (60, 13, 1460)])
@pytest.mark.parametrize("accumulate", [False, True])
def test_rs16_decode_shortened(orc, k, m, vec, accumulate):
    """shortened blocks with erasures over their numData + m slots, beside a full block"""
    rng = np.random.default_rng(vec + k)
    nb = 6
    nd = rng.integers(1, k + 1, nb).astype(np.uint16)
    nd[2] = k
    counts = [m // 2, m, 1, 0, min(int(nd[4]), m), 3]
    _decode_case(orc, k, m, vec, nd, counts, accumulate, seed=7 * k + m, short=True)


def test_rs16_decode_uniform_full_size(orc):
    """RS16(400, 100), 1400-byte segments, 50 erasures uniform over all 500 segments per block
    (bench_extra --workload rs16 --loss uniform's pattern) on 48 blocks"""
    k, m, vec, nb = 400, 100, 1400, 48
    nd = np.full(nb, k, np.uint16)
    _decode_case(orc, k, m, vec, nd, [50] * nb, False, seed=2024, short=False)
