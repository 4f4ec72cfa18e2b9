"""RS16 encode by the Toeplitz split (kernels_tmvp.hip + the tower kernel's multi launch) against
the oracle on the GPU, bit-exact, at one Karatsuba level (three (m/2)-row products) and two
(nine (m/4)-row products).  NFEC_OPT_RS16_TOEPLITZ_ON forces the split, at the most levels the
shape allows, where it is not chosen by default (NFEC_OPT_RS16_TOEPLITZ_OFF: never;
NFEC_OPT_RS16_TOEPLITZ_ONE_LEVEL: one level at most); by default the codec takes the form with the
lowest modelled cost (the products' passes on the cheapest of the tower kernel's 7-, 6- and 4-row
configurations, plus the prescale's traffic and the postscale's multiplies, fitted to the split
forced at each level, profiles/r05/tmvp_levels/): no split for (128, 32) and (256, 64), two levels
for (512, 128), RS16(400, 100) and C4.  Chunk widths need not be powers of two on the tower kernel
(its column map divides by a multiply-high)."""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from norm_amd import NFEC_RS16, NormDecoderRS16, NormEncoderRS16  # noqa: E402
from norm_amd._native import (NFEC_FEATURE_RS16_TOEPLITZ, NFEC_FEATURE_RS16_TOEPLITZ2,  # noqa: E402
                              NFEC_OPT_RS16_TOEPLITZ_OFF, NFEC_OPT_RS16_TOEPLITZ_ON,
                              NFEC_OPT_RS16_TOEPLITZ_ONE_LEVEL)

OPTS = {None: 0, "0": NFEC_OPT_RS16_TOEPLITZ_OFF, "1": NFEC_OPT_RS16_TOEPLITZ_ON,
        "1L1": NFEC_OPT_RS16_TOEPLITZ_ON | NFEC_OPT_RS16_TOEPLITZ_ONE_LEVEL, "L1": NFEC_OPT_RS16_TOEPLITZ_ONE_LEVEL}


def _encoder(k, m, vec, force):
    enc = NormEncoderRS16(options=OPTS[force])
    assert enc.Init(k, m, vec)
    return enc


def _levels(enc):
    f = enc.features()
    return 2 if f & NFEC_FEATURE_RS16_TOEPLITZ2 else 1 if f & NFEC_FEATURE_RS16_TOEPLITZ else 0


CASES = [
    # k, m, vec, seg_stride, nblocks, force, expected Karatsuba levels (0: no split)
    (64, 16, 1400, 1400, 5, "1", 2),
    (64, 16, 1400, 1400, 5, "1L1", 1),
    (128, 32, 64, 64, 37, "1", 2),        # several item groups, short segments
    (128, 32, 64, 64, 37, "1L1", 1),
    (128, 32, 1408, 1416, 3, "1", 2),     # padded segment stride
    # pass costs: 4 passes of 4 rows 292, 8 passes 584, 16 passes 1168, 6-row passes 100 each
    (128, 32, 1400, 1400, 4, None, 0),    # no split by default (measured 7.8 ms against 11.4 / 14.1 at one / two levels)
    (256, 64, 1400, 1400, 4, None, 0),    # likewise (14.2 against 16.4 / 15.9 ms)
    (256, 64, 1400, 1400, 4, "L1", 0),
    (256, 64, 1400, 1400, 4, "0", 0),
    (512, 128, 64, 64, 2, "1", 2),        # several passes per product
    (512, 128, 64, 64, 2, "1L1", 1),
    (32, 8, 8, 8, 7, "1", 2),             # one item per segment, chunk width 4, level-2 halves of 2
    (32, 8, 8, 8, 7, "1L1", 1),
    (16, 4, 64, 64, 3, "1", 2),           # the smallest level-2 shape: halves of one column
    (96, 16, 72, 72, 5, "1", 2),          # three chunk pairs
    (1024, 64, 1400, 1400, 2, "1", 2),
    (2048, 128, 64, 64, 2, "1", 2),
    (512, 128, 64, 64, 3, None, 2),       # two levels by default (23.5 ms against 27.6 / 26.0 at none / one)
    (512, 128, 64, 64, 3, "L1", 1),
    (96, 24, 1400, 1400, 3, "1", 2),      # chunks of 12 and 6 columns (the column map's division)
    (96, 24, 1400, 1400, 3, "1L1", 1),
    (40, 10, 72, 72, 6, "1", 1),          # m / 4 not whole: one level at most, chunks of 5
    (48, 12, 64, 64, 5, "1", 2),          # level-2 chunks of 3 columns
    (400, 100, 1400, 1400, 3, None, 2),   # RS16(400, 100): two levels by default (chunks of 50 and 25)
    (400, 100, 1400, 1400, 3, "L1", 1),
    (400, 100, 1400, 1400, 3, "0", 0),
    # vec % 8 != 0: the split over the 8-byte pieces, the tail kernel over the last 2-6 bytes
    (400, 100, 1460, 1464, 3, None, 2),   # NORM's 1452-byte segments (strides are multiples of 8)
    (64, 16, 1402, 1408, 5, "1", 2),      # 2-byte tail, padded stride
    (64, 16, 1406, 1408, 5, "1L1", 1),    # 6-byte tail at one level
    (32, 8, 14, 16, 7, "1", 2),           # one 8-byte piece and a 6-byte tail per segment
    (100, 20, 1400, 1400, 3, "1", 2),     # level-2 chunks of 5 columns
    (100, 24, 1400, 1400, 3, "1", 0),     # k not a multiple of m: not allowed
]


@pytest.mark.parametrize("k,m,vec,stride,nb,force,levels", CASES)
def test_toeplitz_encode_matches_oracle(orc, k, m, vec, stride, nb, force, levels):
    enc = _encoder(k, m, vec, force)
    assert _levels(enc) == levels
    host = orc.make_blocks(k, m, vec, nb, seg_stride=stride)
    host[:, k:, :] = 0xA5  # overwrite semantics: stale parity must not leak through
    ref = orc.encode_blocks(orc.RS16, k, m, vec, host.copy())  # zeroes the parity, then Encode()s
    dev = torch.from_numpy(host).cuda()
    enc.encode_blocks(dev)
    torch.cuda.synchronize()
    got = dev.cpu().numpy()
    assert np.array_equal(got[:, :, :vec], ref[:, :, :vec])
    assert np.array_equal(got[:, :, vec:], host[:, :, vec:])  # stride padding untouched


def test_toeplitz_encode_twice_and_accumulate(orc):
    """Back-to-back calls share the codec's scratch; accumulate mode takes the one-product path."""
    k, m, vec, nb = 128, 32, 1400, 6
    enc = _encoder(k, m, vec, "1")
    host = orc.make_blocks(k, m, vec, nb)
    ref = orc.encode_blocks(orc.RS16, k, m, vec, host.copy())
    a = torch.from_numpy(host).cuda()
    b = torch.from_numpy(orc.make_blocks(k, m, vec, nb, first_block=100)).cuda()
    ref_b = orc.encode_blocks(orc.RS16, k, m, vec, b.cpu().numpy().copy())
    s2 = torch.cuda.Stream()
    enc.encode_blocks(a)
    with torch.cuda.stream(s2):
        enc.encode_blocks(b, stream=s2)
    torch.cuda.synchronize()
    assert np.array_equal(a.cpu().numpy(), ref)
    assert np.array_equal(b.cpu().numpy(), ref_b)
    enc.encode_blocks(a, accumulate=True)  # parity ^= parity: zero
    torch.cuda.synchronize()
    assert not a[:, k:, :].any()


def test_toeplitz_round_trip_c4_shape(orc):
    """C4's code (4096, 256) at a reduced block count: encode through the split, erase 40
    source segments per block, decode, compare; sampled block against the oracle's encode."""
    k, m, vec, nb = 4096, 256, 1400, 6
    enc = _encoder(k, m, vec, None)
    assert enc.features() & NFEC_FEATURE_RS16_TOEPLITZ
    host = orc.make_blocks(k, m, vec, nb)
    dev = torch.from_numpy(host).cuda()
    enc.encode_blocks(dev)
    torch.cuda.synchronize()
    got = dev.cpu().numpy()
    ref0 = orc.encode_blocks(orc.RS16, k, m, vec, host[:1].copy())
    assert np.array_equal(got[:1], ref0)
    dec = NormDecoderRS16()
    assert dec.Init(k, m, vec)
    locs = np.zeros((nb, m), np.int16)
    counts = np.full(nb, 40, np.int16)
    for b in range(nb):
        locs[b, :40] = orc.erasure_pattern(b, k, 40)
    rx = got.copy()
    for b in range(nb):
        rx[b, locs[b, :40]] = 0
    d = torch.from_numpy(rx).cuda()
    st = dec.decode_blocks(d, torch.from_numpy(locs).cuda(), torch.from_numpy(counts).cuda())
    torch.cuda.synchronize()
    assert (st.cpu().numpy() == 40).all()
    assert np.array_equal(d.cpu().numpy()[:, :k], got[:, :k])


def test_stream_copy_matches_source():
    """nfec_util_stream_copy (the bench's achievable-copy kernel): exact bytes, odd sizes
    rejected, one-piece-per-wave grid covers the tail."""
    from norm_amd import stream_copy
    from norm_amd._native import NfecError

    for n in (16, 4096 + 16, (1 << 20) + 48):
        src = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda")
        dst = torch.zeros_like(src)
        stream_copy(dst, src)
        torch.cuda.synchronize()
        assert torch.equal(dst, src)
    with pytest.raises(NfecError):
        stream_copy(torch.zeros(24, dtype=torch.uint8, device="cuda"), torch.zeros(24, dtype=torch.uint8, device="cuda"))


@pytest.mark.parametrize("pinned", [False, True])
def test_toeplitz_host_pipeline_chunks(orc, pinned, monkeypatch):
    """Host-resident encode through the split: four chunks over the three slot streams share
    the codec's scratch (ordered by its event)."""
    k, m, vec, nb = 256, 64, 1400, 10
    enc = _encoder(k, m, vec, "1")
    assert enc.features() & NFEC_FEATURE_RS16_TOEPLITZ
    host = orc.make_blocks(k, m, vec, nb)
    ref = orc.encode_blocks(orc.RS16, k, m, vec, host.copy())
    if pinned:
        buf = torch.from_numpy(host).pin_memory()
        arr = buf.numpy()
    else:
        arr = host
    monkeypatch.setenv("NFEC_HOST_CHUNK_BLOCKS", "3")
    enc.encode_blocks_host(arr)
    assert np.array_equal(arr, ref)


def test_toeplitz_pipeline_sub_batches(orc):
    """A large batch runs the two-level split as sub-batches pipelined over the caller's stream
    and the codec's second stream (rs16_tmvp2_encode: about 3,072 product workgroups per
    sub-batch, i.e. ~1,000 RS16(400, 100) blocks, so 2,100 blocks make three).  The bytes equal
    the one-product encode of the same blocks, unshortened and with RFC 5052 numData in
    {k, k - 1}; the blocks at the sub-batch seams equal the oracle; and two batches encoded at once
    from two threads on two streams of one codec both come out right (the pipeline's fork, join
    and scratch hand-over between calls)."""
    import threading

    from norm_amd import fill_blocks

    k, m, vec, nb = 400, 100, 1400, 2100
    enc = _encoder(k, m, vec, None)
    assert _levels(enc) == 2
    one = _encoder(k, m, vec, "0")
    assert _levels(one) == 0

    def batch(first, nd=None):
        t = torch.zeros((nb, k + m, vec), dtype=torch.uint8, device="cuda")
        fill_blocks(t, k, vec, 0x4E4F524D, first_block=first, per_block_num_data=nd)
        t[:, k:] = 0xA5  # stale parity must not survive (the split overwrites)
        return t

    # unshortened: the split (pipelined) against the one-product kernel, and the seams against the oracle
    a = batch(0)
    ref = a.clone()
    enc.encode_blocks(a)
    one.encode_blocks(ref)
    torch.cuda.synchronize()
    assert torch.equal(a, ref)
    seams = [0, 699, 700, 1399, 1400, nb - 1]
    host = a[seams].cpu().numpy()
    want = orc.encode_blocks(orc.RS16, k, m, vec, host.copy())
    assert np.array_equal(host, want)

    # RFC 5052 shortened blocks through the pipeline (each sub-batch's numData slice)
    rng = np.random.default_rng(7)
    ndh = rng.integers(k - 1, k + 1, nb).astype(np.uint16)
    nd = torch.from_numpy(ndh.view(np.int16)).cuda()
    s = batch(0, nd)
    s_ref = s.clone()
    enc.encode_blocks(s, num_data=nd)
    one.encode_blocks(s_ref, num_data=nd)
    torch.cuda.synchronize()
    assert torch.equal(s, s_ref)

    # NORM's 1452-byte segments (vec 1460 = segmentSize + 8, % 8 != 0): the pipelined split over the
    # 8-byte pieces, then the tail kernel over the last 4 bytes, against the one-product path
    v2 = 1460
    enc2, one2 = _encoder(k, m, v2, None), _encoder(k, m, v2, "0")
    t = torch.zeros((nb, k + m, 1464), dtype=torch.uint8, device="cuda")
    fill_blocks(t, k, v2, 0x4E4F524D, first_block=3000)
    t_ref = t.clone()
    enc2.encode_blocks(t)
    one2.encode_blocks(t_ref)
    torch.cuda.synchronize()
    assert torch.equal(t, t_ref)
    del t, t_ref

    # two batches at once on one codec, two host threads and two streams
    x, y = batch(5000), batch(9000)
    x_ref, y_ref = x.clone(), y.clone()
    one.encode_blocks(x_ref)
    one.encode_blocks(y_ref)
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    errs = []

    def run(t, st):
        try:
            for _ in range(3):
                enc.encode_blocks(t, stream=st)
        except Exception as e:  # pragma: no cover - reported below
            errs.append(e)

    th = [threading.Thread(target=run, args=(t, st)) for t, st in ((x, streams[0]), (y, streams[1]))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    torch.cuda.synchronize()
    assert not errs
    assert torch.equal(x, x_ref) and torch.equal(y, y_ref)


def test_toeplitz_pipeline_c4_shape():
    """C4's code at 600 blocks: the pipelined two-level split (about 250 C4 blocks per sub-batch,
    so three, over two streams and two scratch halves) against the one-product encode of the same
    blocks, every byte."""
    from norm_amd import fill_blocks

    k, m, vec, nb = 4096, 256, 1400, 600
    enc, one = _encoder(k, m, vec, None), _encoder(k, m, vec, "0")
    assert _levels(enc) == 2 and _levels(one) == 0
    t = torch.zeros((nb, k + m, vec), dtype=torch.uint8, device="cuda")
    fill_blocks(t, k, vec, 0x4E4F524D, first_block=77)
    t_ref = t.clone()
    enc.encode_blocks(t)
    one.encode_blocks(t_ref)
    torch.cuda.synchronize()
    assert torch.equal(t, t_ref)
