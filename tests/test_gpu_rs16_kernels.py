"""RS16 products on both GPU kernels against the oracle, bit-exact: the tower-field kernel
(gen_gf16_tw.hip, the default) and the shared-table kernel (gen_gf16_t3.hip,
NFEC_OPT_RS16_SHARED_TABLES).  The option is per codec, so both run in one process.  Covers the one-product
encode, the Toeplitz split (C4's route) and decode stage 1 (the plan's by-encode blocks).
Reference: NormEncoderRS16::Encode / NormDecoderRS16::Decode, src/common/normEncoderRS16.cpp:472-482,
650-755."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from norm_amd import NFEC_RS16, NormDecoderRS16, NormEncoderRS16  # noqa: E402
from norm_amd._native import (NFEC_FEATURE_RS16_TOEPLITZ, NFEC_OPT_RS16_SHARED_TABLES,  # noqa: E402
                              NFEC_OPT_RS16_TOEPLITZ_OFF, NFEC_OPT_RS16_TOEPLITZ_ON)

KERNELS = ["1", "0"]   # tower, shared tables


def _codecs(monkeypatch, tw, k, m, vec, tmvp=None):
    opts = (0 if tw == "1" else NFEC_OPT_RS16_SHARED_TABLES) | \
        {None: 0, "0": NFEC_OPT_RS16_TOEPLITZ_OFF, "1": NFEC_OPT_RS16_TOEPLITZ_ON}[tmvp]
    enc, dec = NormEncoderRS16(options=opts), NormDecoderRS16(options=opts)
    assert enc.Init(k, m, vec) and dec.Init(k, m, vec)
    return enc, dec


@pytest.mark.parametrize("tw", KERNELS)
@pytest.mark.parametrize("k,m,vec,stride,nb,tmvp", [
    (100, 20, 1400, 1400, 3, "0"),     # one product: four 5-row passes (tower, 6-row kernel) / one of 44 (shared tables)
    (64, 11, 64, 64, 9, "0"),          # 11 rows: four passes of the 4-row kernel (the 11-row kernel's one full pass)
    (40, 12, 72, 80, 5, "0"),          # 12 rows, padded stride
    (128, 32, 1408, 1416, 3, "1"),     # Toeplitz split, padded stride
    (512, 128, 64, 64, 2, "1"),        # Toeplitz split, several passes per product
])
def test_rs16_encode_both_kernels(orc, monkeypatch, tw, k, m, vec, stride, nb, tmvp):
    enc, _ = _codecs(monkeypatch, tw, k, m, vec, tmvp)
    assert bool(enc.features() & NFEC_FEATURE_RS16_TOEPLITZ) == (tmvp == "1")
    host = orc.make_blocks(k, m, vec, nb, seg_stride=stride)
    host[:, k:, :] = 0x5A
    ref = orc.encode_blocks(NFEC_RS16, k, m, vec, host.copy())
    dev = torch.from_numpy(host).cuda()
    enc.encode_blocks(dev)
    torch.cuda.synchronize()
    assert np.array_equal(dev.cpu().numpy(), ref)


@pytest.mark.parametrize("tw", KERNELS)
@pytest.mark.parametrize("k,m,vec,nb,es", [(400, 100, 64, 3, 50), (100, 20, 1400, 4, 20), (40, 10, 72, 5, 3)])
def test_rs16_decode_both_kernels(orc, monkeypatch, tw, k, m, vec, nb, es):
    """source-only erasures: stage 1 runs on the product kernel for every block"""
    enc, dec = _codecs(monkeypatch, tw, k, m, vec)
    host = orc.encode_blocks(NFEC_RS16, k, m, vec, orc.make_blocks(k, m, vec, nb))
    locs = np.zeros((nb, m), np.uint16)
    counts = np.zeros(nb, np.uint16)
    for b in range(nb):
        e = max(1, es - b)   # different erasure counts per block: rows_lim is the largest
        src = orc.erasure_pattern(b + 77, k, e)
        locs[b, :e] = src
        counts[b] = e
        host[b, src, :] = 0
    ref = host.copy()
    st_ref = orc.decode_blocks(NFEC_RS16, k, m, vec, ref, locs, counts)
    dev = torch.from_numpy(host).cuda()
    st = dec.decode_blocks(dev, torch.from_numpy(locs.astype(np.int16)).cuda(),
                           torch.from_numpy(counts.astype(np.int16)).cuda())
    torch.cuda.synchronize()
    assert np.array_equal(st.cpu().numpy(), st_ref)
    assert np.array_equal(dev.cpu().numpy(), ref)


@pytest.mark.parametrize("k,m,vec,counts", [
    (40, 10, 72, [0, 1, 10, 3, 10, 0, 7]),      # e from 0 to M = min(k, m) in one batch
    (30, 12, 4104, [12, 1, 5]),                 # segments past one 4 KiB item group (two per block)
    (12, 30, 64, [12, 0, 11, 6]),               # k < m: M = k
])
def test_rs16_decode_per_block_rows(orc, monkeypatch, k, m, vec, counts):
    """decode stage 2 on the tower kernel in per-block mode: each block's own e (rows and
    columns), blocks with nothing to repair, several item groups per block"""
    nb = len(counts)
    enc, dec = _codecs(monkeypatch, "1", k, m, vec)
    host = orc.encode_blocks(NFEC_RS16, k, m, vec, orc.make_blocks(k, m, vec, nb))
    locs = np.zeros((nb, m), np.uint16)
    cnt = np.zeros(nb, np.uint16)
    for b, e in enumerate(counts):
        if e:
            src = orc.erasure_pattern(b + 5, k, e)
            locs[b, :e] = src
            host[b, src, :] = 0
        cnt[b] = e
    ref = host.copy()
    st_ref = orc.decode_blocks(NFEC_RS16, k, m, vec, ref, locs, cnt)
    dev = torch.from_numpy(host).cuda()
    st = dec.decode_blocks(dev, torch.from_numpy(locs.astype(np.int16)).cuda(),
                           torch.from_numpy(cnt.astype(np.int16)).cuda())
    torch.cuda.synchronize()
    assert np.array_equal(st.cpu().numpy(), st_ref)
    assert np.array_equal(dev.cpu().numpy(), ref)
