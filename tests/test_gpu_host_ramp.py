"""Pinned host batches large enough for the ramped pipeline (host_chunk_plan, nfec_api.cpp):
chunks of base / 8, / 4, / 2, base, then 4 x base through the middle and the same steps down,
with a slot holding the largest.  RS8(64,32) x 1400 B: base = 998 blocks, so 8,192 blocks take
the ramp (it needs 2 x 1,870 + 3,992).  The encode and the 16-erasure repair through the host
pipeline must give the bytes and statuses of the device-resident path on the same blocks (itself
checked against the oracle in test_gpu_parity.py)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import torch  # noqa: E402

from norm_amd import NormDecoderRS8, NormEncoderRS8, fill_blocks, make_erasures, zero_erasures  # noqa: E402


def test_ramped_host_pipeline_matches_device():
    k, m, vec, nb = 64, 32, 1400, 8192
    enc, dec = NormEncoderRS8(), NormDecoderRS8()
    assert enc.Init(k, m, vec) and dec.Init(k, m, vec)
    blocks = torch.zeros((nb, k + m, vec), dtype=torch.uint8, device="cuda")
    fill_blocks(blocks, k, vec, 0x5EED)
    host = torch.empty(blocks.shape, dtype=torch.uint8, pin_memory=True)
    host.copy_(blocks)
    # device-resident reference
    enc.encode_blocks(blocks)
    locs, counts = make_erasures(nb, k, 16, 0x5EED, m)
    clean = blocks.cpu().numpy()
    zero_erasures(blocks, locs, counts, vec)
    st_dev = dec.decode_blocks(blocks, locs, counts).cpu().numpy()
    torch.cuda.synchronize()
    assert (st_dev == 16).all()
    assert np.array_equal(blocks.cpu().numpy(), clean)
    del blocks
    # the same through the pinned host pipeline
    hnp = host.numpy()
    enc.encode_blocks_host(hnp)
    assert np.array_equal(hnp, clean)
    hl = locs.cpu().numpy().view(np.uint16)
    hc = counts.cpu().numpy().view(np.uint16)
    hnp[np.arange(nb)[:, None], hl[:, :16].astype(np.int64)] = 0
    st = dec.decode_blocks_host(hnp, hl, hc)
    assert (st == 16).all()
    assert np.array_equal(hnp, clean)
