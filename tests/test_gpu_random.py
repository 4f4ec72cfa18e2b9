"""Randomized parity sweep (fixed seeds): codec, (k, m), segment length, stride, block count,
shortened blocks and erasure patterns drawn at random, every encode and decode compared byte
for byte (and status for status) with the oracle's restatement of the reference calls
(Encode per segment, normObject.cpp:2203-2229; Decode, normObject.cpp:1548-1644)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from norm_amd import (NFEC_MDP, NFEC_RS8, NFEC_RS16, NormDecoderMDP, NormDecoderRS8,  # noqa: E402
                      NormDecoderRS16, NormEncoderMDP, NormEncoderRS8, NormEncoderRS16)

ENC = {NFEC_RS8: NormEncoderRS8, NFEC_RS16: NormEncoderRS16, NFEC_MDP: NormEncoderMDP}
DEC = {NFEC_RS8: NormDecoderRS8, NFEC_RS16: NormDecoderRS16, NFEC_MDP: NormDecoderMDP}


def _draw(seed):
    rng = np.random.default_rng(seed)
    kind = [NFEC_RS8, NFEC_RS8, NFEC_RS16, NFEC_MDP][seed % 4]
    if kind == NFEC_RS16:
        k = int(rng.integers(1, 300))
        m = int(rng.integers(1, 160))
        vec = int(rng.integers(2, 600))
    else:
        k = int(rng.integers(1, 200))
        m = int(rng.integers(1, (255 - k if rng.integers(0, 3) == 0 else min(255 - k, 64)) + 1))
        vec = int(rng.choice([int(rng.integers(1, 3000)), 1400, 1408, 8 * int(rng.integers(1, 200))]))
    stride = (vec + 7) // 8 * 8 + 8 * int(rng.integers(0, 3))
    nb = int(rng.integers(1, 40))
    short = bool(rng.integers(0, 2))
    return rng, kind, k, m, vec, stride, nb, short


@pytest.mark.parametrize("seed", range(160))
def test_random_encode_decode_matches_oracle(orc, seed):
    rng, kind, k, m, vec, stride, nb, short = _draw(seed)
    enc, dec = ENC[kind](), DEC[kind]()
    assert enc.Init(k, m, vec) and dec.Init(k, m, vec)
    nd = rng.integers(1, k + 1, nb).astype(np.uint16) if short else None
    host = orc.make_blocks(k, m, vec, nb, seg_stride=stride, num_data=nd, seed=seed)
    ref = orc.encode_blocks(kind, k, m, vec, host.copy(), nd)
    dev = torch.from_numpy(host).cuda()
    ndev = torch.from_numpy(nd.astype(np.int16)).cuda() if short else None
    enc.encode_blocks(dev, num_data=ndev)
    torch.cuda.synchronize()
    assert np.array_equal(dev.cpu().numpy(), ref), (kind, k, m, vec, stride, nb, short)

    # erasures: source then parity, sorted, at most m in all (some blocks lose nothing)
    locs = np.zeros((nb, m), np.uint16)
    counts = np.zeros(nb, np.uint16)
    rx = ref.copy()
    for b in range(nb):
        n_d = int(nd[b]) if short else k
        es = int(rng.integers(0, min(n_d, m) + 1))
        ep = int(rng.integers(0, m - es + 1)) if rng.integers(0, 3) == 0 else 0
        e = np.concatenate([np.sort(rng.choice(n_d, es, replace=False)),
                            n_d + np.sort(rng.choice(m, ep, replace=False))]).astype(np.uint16)
        locs[b, :len(e)] = e
        counts[b] = len(e)
        for s in e:
            rx[b, s, :vec] = 0
    want = rx.copy()
    st_ref = orc.decode_blocks(kind, k, m, vec, want, locs, counts, nd)
    dev = torch.from_numpy(rx).cuda()
    st = dec.decode_blocks(dev, torch.from_numpy(locs.astype(np.int16)).cuda(),
                           torch.from_numpy(counts.astype(np.int16)).cuda(), num_data=ndev)
    torch.cuda.synchronize()
    assert np.array_equal(st.cpu().numpy(), st_ref), (kind, k, m, vec, stride, nb, short)
    assert np.array_equal(dev.cpu().numpy(), want), (kind, k, m, vec, stride, nb, short)
