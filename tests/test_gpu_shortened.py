"""Shortened blocks on the fast encode kernels (round 6), bit-exact against the oracle.

NORM's block partition gives whole runs of blocks numData = k - 1 (RFC 5052 small blocks,
normObject.cpp:203-231: large blocks of k, small blocks of k - 1), and every object's last block
is shorter still.  The reference encodes a shortened block by calling Encode() for its numData
source segments only (normEncoderRS8.cpp:473-483, normEncoderRS16.cpp:472-482): generator
columns 0 .. numData - 1, parity in the slots after them (numData + r, normObject.cpp:1610).

These batches now stay on the fast kernels:
  * RS16: the Toeplitz split (one or two Karatsuba levels) -- its prescale reads zeros for a
    source column at or past the block's numData, the products that read source columns through
    their column map mask the mapped slot, and the postscale writes slot numData + r;
  * RS8 (64, 32) / (64, 16) / (64, 8): the fixed-generator q4 kernels with each 8-byte piece's
    source data masked at its own block's numData; and their repair on the closed-form plan and
    the fused / bit-sliced repair kernels (a shortened block's columns past numData are skipped
    like erased ones, its parity read at slot numData + t).
nfec_codec_encode_paths() / decode_paths() tell which kernel family took each batch.  A block whose numData is 0
or past k (undefined in the reference) is left untouched."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from norm_amd import (NFEC_RS8, NFEC_RS16, NormDecoderRS8, NormEncoderRS8, NormEncoderRS16)  # noqa: E402
from norm_amd._native import (NFEC_FEATURE_RS16_TOEPLITZ, NFEC_FEATURE_RS16_TOEPLITZ2,  # noqa: E402
                              NFEC_OPT_RS16_TOEPLITZ_ON, NFEC_OPT_RS16_TOEPLITZ_ONE_LEVEL)


def _i16(a):
    return torch.from_numpy(np.ascontiguousarray(a).astype(np.uint16).view(np.int16)).cuda()


def _num_data(k, nb, seed, invalid=False):
    """a mix in one batch: numData below k/4, k/2 and 3k/4, k - 1 (RFC 5052 small blocks), k,
    and 1; the rest drawn from [1, k]"""
    rng = np.random.default_rng(seed)
    nd = rng.integers(1, k + 1, nb).astype(np.uint16)
    fixed = [max(1, k // 4 - 1), max(1, k // 2 - 1), max(1, 3 * k // 4 - 1), k - 1, k, 1, k - 1, k]
    nd[:min(nb, len(fixed))] = fixed[:nb]
    if invalid and nb > 10:
        nd[9] = 0          # undefined in the reference: left alone
        nd[10] = k + 1
    return nd


def _check(orc, kind, k, m, vec, stride, nb, nd, enc, expect_path, opts_note=""):
    host = orc.make_blocks(k, m, vec, nb, seg_stride=stride, num_data=np.clip(nd, 1, k))
    rng = np.random.default_rng(int(nd.sum()))
    # parity slots hold junk before an overwrite encode; slots past numData + m hold junk that is
    # never read nor written
    for b in range(nb):
        n = int(np.clip(nd[b], 1, k))
        host[b, n:, :] = rng.integers(0, 256, (k + m - n, host.shape[2]), dtype=np.uint8)
    valid = (nd >= 1) & (nd <= k)
    ref = host.copy()
    ref[valid] = orc.encode_blocks(kind, k, m, vec, host[valid].copy(), num_data=nd[valid])
    # the oracle zero-fills each block's parity vectors (NORM does, normObject.cpp:1919) and the
    # reference writes only vec bytes (RS16: vec & ~1): the stride padding keeps the junk
    cov = vec & ~1 if kind == NFEC_RS16 else vec
    for b in np.nonzero(valid)[0]:
        n = int(nd[b])
        ref[b, n:n + m, cov:] = host[b, n:n + m, cov:]
    dev = torch.from_numpy(host).cuda()
    before = enc.encode_paths()
    enc.encode_blocks(dev, num_data=_i16(nd))
    torch.cuda.synchronize()
    after = enc.encode_paths()
    got = dev.cpu().numpy()
    assert np.array_equal(got, ref), opts_note
    took = {p: after[p] - before[p] for p in after if after[p] != before[p]}
    assert took == {expect_path: 1}, took


RS16_CASES = [
    # k, m, vec, stride, nb, options, expected levels
    (400, 100, 1400, 1400, 12, 0, 2),                          # the C5 RS16 block type
    (400, 100, 1400, 1400, 12, NFEC_OPT_RS16_TOEPLITZ_ONE_LEVEL, 1),
    (400, 100, 1460, 1464, 12, 0, 2),                          # NORM's 1452-byte segments + 8
    (64, 16, 1400, 1400, 13, NFEC_OPT_RS16_TOEPLITZ_ON, 2),
    (64, 16, 1406, 1408, 13, NFEC_OPT_RS16_TOEPLITZ_ON | NFEC_OPT_RS16_TOEPLITZ_ONE_LEVEL, 1),
    (512, 128, 64, 64, 15, 0, 2),                              # many blocks per item group
    (96, 24, 72, 72, 40, NFEC_OPT_RS16_TOEPLITZ_ON, 2),        # chunks of 12 / 6 columns
    (40, 10, 72, 72, 21, NFEC_OPT_RS16_TOEPLITZ_ON, 1),        # m / 4 not whole: one level
    (32, 8, 8, 8, 37, NFEC_OPT_RS16_TOEPLITZ_ON, 2),           # one item per segment
]


@pytest.mark.parametrize("k,m,vec,stride,nb,opts,levels", RS16_CASES)
def test_rs16_shortened_encode_on_the_split(orc, k, m, vec, stride, nb, opts, levels):
    enc = NormEncoderRS16(options=opts) if opts else NormEncoderRS16()
    assert enc.Init(k, m, vec)
    f = enc.features()
    assert (2 if f & NFEC_FEATURE_RS16_TOEPLITZ2 else 1 if f & NFEC_FEATURE_RS16_TOEPLITZ else 0) == levels
    nd = _num_data(k, nb, k * 7 + m, invalid=True)
    _check(orc, NFEC_RS16, k, m, vec, stride, nb, nd, enc, "rs16_split", f"opts {opts}")


def test_rs16_rfc5052_partition_on_the_split(orc):
    """whole runs of numData = k and k - 1, as NORM's block partition makes them"""
    k, m, vec, nb = 400, 100, 1400, 16
    enc = NormEncoderRS16()
    assert enc.Init(k, m, vec)
    nd = np.array([k] * 5 + [k - 1] * 11, np.uint16)
    _check(orc, NFEC_RS16, k, m, vec, vec, nb, nd, enc, "rs16_split")


def test_rs16_c4_shape_shortened_on_the_split(orc):
    """C4's code (4096, 256) with shortened blocks, against the oracle's per-segment Encode with
    the codec's generator (pinned to the oracle's C4 fixture in test_c4_c5.py)"""
    k, m, vec, nb = 4096, 256, 1400, 4
    enc = NormEncoderRS16()
    assert enc.Init(k, m, vec)
    assert enc.features() & NFEC_FEATURE_RS16_TOEPLITZ2
    nd = np.array([k - 1, 1000, k, 2047], np.uint16)
    host = orc.make_blocks(k, m, vec, nb, num_data=nd)
    dev = torch.from_numpy(host).cuda()
    before = enc.encode_paths()["rs16_split"]
    enc.encode_blocks(dev, num_data=_i16(nd))
    torch.cuda.synchronize()
    assert enc.encode_paths()["rs16_split"] == before + 1
    got = dev.cpu().numpy()
    par = enc.generator()  # m x k
    full = np.zeros((k + m, k), np.uint16)
    full[:k] = np.eye(k, dtype=np.uint16)
    full[k:] = par
    for b in (0, 1):
        n = int(nd[b])
        src = host[b, :k, :].copy()
        src[n:] = 0  # a shortened block's columns past numData do not take part
        want = orc.encode_block_with_generator(orc.RS16, full, k, m, vec, src)
        assert np.array_equal(got[b, n:n + m, :vec], want)
        assert np.array_equal(got[b, :n], host[b, :n])


RS8_CASES = [(64, 32, 1400, 70), (64, 16, 1400, 33), (64, 8, 1408, 20), (64, 32, 8, 300), (64, 32, 1400, 1)]


@pytest.mark.parametrize("k,m,vec,nb", RS8_CASES)
def test_rs8_shortened_encode_on_the_fixed_kernels(orc, k, m, vec, nb):
    enc = NormEncoderRS8()
    assert enc.Init(k, m, vec)
    nd = _num_data(k, nb, k + m + vec, invalid=True)
    _check(orc, NFEC_RS8, k, m, vec, vec, nb, nd, enc, "fixed")


def test_rs8_rfc5052_partition_and_accumulate(orc):
    """numData in {k, k - 1} on the q4 kernel; accumulate XORs into the existing parity"""
    k, m, vec, nb = 64, 32, 1400, 64
    enc = NormEncoderRS8()
    assert enc.Init(k, m, vec)
    nd = np.where(np.arange(nb) % 3 == 0, k, k - 1).astype(np.uint16)
    _check(orc, NFEC_RS8, k, m, vec, vec, nb, nd, enc, "fixed")
    host = orc.make_blocks(k, m, vec, nb, num_data=nd)
    ref = orc.encode_blocks(NFEC_RS8, k, m, vec, host.copy(), num_data=nd)
    dev = torch.from_numpy(ref.copy()).cuda()
    enc.encode_blocks(dev, num_data=_i16(nd), accumulate=True)  # parity ^= parity: zero
    torch.cuda.synchronize()
    got = dev.cpu().numpy()
    for b in range(nb):
        n = int(nd[b])
        assert np.array_equal(got[b, :n], ref[b, :n])
        assert not got[b, n:n + m].any()


def test_rs8_shortened_other_shapes_stay_on_the_runtime_kernel(orc):
    """shapes without a fixed-generator kernel keep the runtime-coefficient kernel"""
    k, m, vec, nb = 48, 20, 1400, 9
    enc = NormEncoderRS8()
    assert enc.Init(k, m, vec)
    nd = _num_data(k, nb, 5)
    _check(orc, NFEC_RS8, k, m, vec, vec, nb, nd, enc, "runtime")


def _i16a(a):
    return torch.from_numpy(np.ascontiguousarray(a).astype(np.int16)).cuda()


@pytest.mark.parametrize("k,m,vec,nb,acc", [(64, 32, 1400, 48, False), (64, 16, 1408, 40, False),
                                             (64, 8, 64, 40, False), (64, 32, 1400, 24, True)])
def test_rs8_shortened_decode_on_the_fixed_kernels(orc, k, m, vec, nb, acc):
    """Shortened blocks (numData < k) repaired by the closed-form plan and the fused / bit-sliced
    repair kernels (normEncoderRS8.cpp:652-757 with :675-693): source erasures only (the fused
    kernel), source and parity erasures (substitute rows past 16: the unfused stage 1 + solve),
    more than 16 erasures, none, too many (status 0, untouched) and invalid numData (left alone)"""
    rng = np.random.default_rng(k + m + nb + int(acc))
    nd = _num_data(k, nb, 17 * m + nb, invalid=True)
    valid = (nd >= 1) & (nd <= k)
    host = orc.make_blocks(k, m, vec, nb, num_data=np.clip(nd, 1, k))
    enc = NormEncoderRS8()
    assert enc.Init(k, m, vec)
    clean = host.copy()
    clean[valid] = orc.encode_blocks(NFEC_RS8, k, m, vec, host[valid].copy(), num_data=nd[valid])
    ls = m + 1
    locs = np.zeros((nb, ls), np.uint16)
    counts = np.zeros(nb, np.uint16)
    for b in range(nb):
        n = int(np.clip(nd[b], 1, k))
        kind = b % 6
        if kind == 0:      # source erasures only, e <= 16: the fused kernel
            es, ep = min(n, int(rng.integers(1, 17))), 0
        elif kind == 1:    # source + parity: substitute parity rows shift upward
            es, ep = min(n, int(rng.integers(1, 9))), int(rng.integers(1, m // 2 + 1))
        elif kind == 2:    # more than 16 source erasures (m = 32): unfused
            es, ep = min(n, m // 2 + 4 if m > 16 else m), 0
        elif kind == 3:    # nothing lost
            es, ep = 0, 0
        elif kind == 4:    # lost parity only
            es, ep = 0, int(rng.integers(1, m + 1))
        else:              # everything a block can lose and still decode
            es = min(n, m // 2)
            ep = m - es
        es = min(es, n, m)
        ep = max(0, min(ep, m - es))
        e = np.sort(np.concatenate([rng.choice(n, es, replace=False), n + rng.choice(m, ep, replace=False)]))
        if b == 7:         # one past the parity count: undecodable, the block stays as it is
            e = np.sort(rng.choice(n + m, min(n + m, m + 1), replace=False))
        locs[b, :len(e)] = e
        counts[b] = len(e)
    rx = clean.copy()
    for b in range(nb):
        for s in locs[b, :counts[b]]:
            # erased source: zero (NORM's zero-fill), or junk under accumulate (XORed into)
            rx[b, s] = rng.integers(0, 256, rx.shape[2], dtype=np.uint8) if acc else 0
    want = rx.copy()
    st_ref = np.zeros(nb, np.int32)
    if valid.any():
        sub = want[valid].copy()
        st_ref[valid] = _oracle_decode(orc, k, m, vec, sub, locs[valid], counts[valid], nd[valid])
        want[valid] = sub
    dec = NormDecoderRS8()
    assert dec.Init(k, m, vec)
    dev = torch.from_numpy(rx).cuda()
    before = dec.decode_paths()
    st = dec.decode_blocks(dev, _i16a(locs), _i16a(counts), num_data=_i16(nd), accumulate=acc)
    torch.cuda.synchronize()
    after = dec.decode_paths()
    assert {p: after[p] - before[p] for p in after if after[p] != before[p]} == {"fixed": 1}
    got = dev.cpu().numpy()
    stg = st.cpu().numpy()
    assert np.array_equal(stg, st_ref), (stg, st_ref)
    assert np.array_equal(got, want)
    for b in np.nonzero(~valid)[0]:
        assert stg[b] == 0 and np.array_equal(got[b], rx[b])


def _oracle_decode(orc, k, m, vec, blocks, locs, counts, nd):
    """the oracle's Decode per block; a list longer than m (undecodable) gives status 0 and
    leaves the block alone, as the reference's dec_matrix build fails (normEncoderRS8.cpp:721-725)"""
    st = np.zeros(len(blocks), np.int32)
    for i in range(len(blocks)):
        if counts[i] > m:
            continue
        one = blocks[i:i + 1].copy()
        l1 = np.zeros((1, m), np.uint16)
        l1[0, :counts[i]] = locs[i, :counts[i]]
        st[i] = orc.decode_blocks(NFEC_RS8, k, m, vec, one, l1, counts[i:i + 1], nd[i:i + 1])[0]
        blocks[i] = one[0]
    return st
