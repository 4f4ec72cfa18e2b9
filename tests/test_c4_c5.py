"""BASELINE.json configs C4 and C5 on the HIP path.

C4: RS16 k=4096, m=256, vec=1400.  The generator is pinned to the oracle's
restatement of NormEncoderRS16::Init (src/common/normEncoderRS16.cpp:399-461) through the
committed fixture tests/golden/rs16_c4_generator.json (SHA-256 of all 256 x 4096 parity rows
plus four rows in full; made by tests/golden/make_rs16_c4_fixture.py).  Encoded blocks are
compared byte for byte with the oracle's per-segment Encode (normEncoderRS16.cpp:472-482) on
sampled blocks; the full 4,096-block batch goes through encode -> erase -> decode.

C5: the mixed RS8(64,32) / RS16(400,100) stream at vec=1400 (the fecTest shape with NORM's
segment size, src/common/fecTest.cpp:13-16), blocks in host memory, driven through the
host-resident pipelines from two host threads at once, every block checked against the oracle.
"""
import hashlib
import json
import os
import threading

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
C4_K, C4_M, VEC = 4096, 256, 1400
SEED = 0x4E4F524D


def _c4_fixture():
    with open(os.path.join(ROOT, "tests", "golden", "rs16_c4_generator.json")) as f:
        return json.load(f)


def _check_c4_rows(par):
    fx = _c4_fixture()
    assert par.shape == (C4_M, C4_K)
    le = np.ascontiguousarray(par).astype("<u2")
    for r, hexrow in fx["rows"].items():
        assert le[int(r)].tobytes().hex() == hexrow, f"row {r}"
    assert hashlib.sha256(le.tobytes()).hexdigest() == fx["parity_rows_sha256"]


def test_c4_generator_host_matches_oracle_fixture():
    """nfec_build_generator (host closed form, no GPU) == the oracle's Vandermonde construction."""
    from norm_amd import NFEC_RS16, build_generator

    _check_c4_rows(build_generator(NFEC_RS16, C4_K, C4_M))


def _gpu():
    torch = pytest.importorskip("torch")
    from norm_amd import device_count

    assert torch.cuda.is_available() and device_count() >= 1, "GPU tests need a gfx950 device"
    return torch


@pytest.mark.gpu
def test_c4_codec_generator_matches_oracle_fixture():
    _gpu()
    from norm_amd import NormEncoderRS16

    enc = NormEncoderRS16()
    assert enc.Init(C4_K, C4_M, VEC)
    _check_c4_rows(enc.generator())


@pytest.mark.gpu
def test_c4_encode_sampled_blocks_match_oracle(orc):
    torch = _gpu()
    from norm_amd import NormEncoderRS16, fill_blocks

    nb = 192
    enc = NormEncoderRS16()
    assert enc.Init(C4_K, C4_M, VEC)
    gen = enc.generator()
    _check_c4_rows(gen)
    full = np.vstack([np.eye(C4_K, dtype=np.uint16), gen])
    blocks = torch.zeros((nb, C4_K + C4_M, VEC), dtype=torch.uint8, device="cuda")
    fill_blocks(blocks, C4_K, VEC, SEED)
    # junk in the parity slots: the batch encode overwrites them (no NFEC_ACCUMULATE)
    blocks[:, C4_K:].fill_(0xA5)
    enc.encode_blocks(blocks)
    torch.cuda.synchronize()
    for b in (0, 77, nb - 1):
        host = blocks[b].cpu().numpy()
        # the GPU fill is the oracle's splitmix64 stream (spot check one segment)
        assert np.array_equal(host[4095], orc.fill_segment(b, 4095, VEC))
        ref = orc.encode_block_with_generator(orc.RS16, full, C4_K, C4_M, VEC, host[:C4_K])
        assert np.array_equal(host[C4_K:], ref), f"block {b}"


@pytest.mark.gpu
@pytest.mark.parametrize("nb,erasures", [(4096, 32), (48, 256)])
def test_c4_round_trip(nb, erasures):
    """Full C4 batch (4,096 blocks, 25 GB) encode -> erase `erasures` random source symbols ->
    decode restores every byte; e = m = 256 on a smaller batch."""
    torch = _gpu()
    from norm_amd import NormDecoderRS16, NormEncoderRS16, fill_blocks, make_erasures, zero_erasures

    enc, dec = NormEncoderRS16(), NormDecoderRS16()
    assert enc.Init(C4_K, C4_M, VEC) and dec.Init(C4_K, C4_M, VEC)
    blocks = torch.zeros((nb, C4_K + C4_M, VEC), dtype=torch.uint8, device="cuda")
    fill_blocks(blocks, C4_K, VEC, SEED ^ 0xC4)
    enc.encode_blocks(blocks)
    keep = blocks.clone()
    if erasures <= 128:  # the device generator's limit
        locs, counts = make_erasures(nb, C4_K, erasures, SEED, C4_M)
    else:
        rng = np.random.default_rng(erasures)
        hl = np.stack([np.sort(rng.choice(C4_K, erasures, replace=False)) for _ in range(nb)]).astype(np.int16)
        locs = torch.from_numpy(hl).cuda()
        counts = torch.full((nb,), erasures, dtype=torch.int16, device="cuda")
    zero_erasures(blocks, locs, counts, VEC)
    st = dec.decode_blocks(blocks, locs, counts)
    torch.cuda.synchronize()
    assert bool((st == erasures).all())
    assert torch.equal(blocks, keep)
    del keep, blocks
    torch.cuda.empty_cache()


def _splitmix64(x):
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


@pytest.mark.gpu
@pytest.mark.parametrize("pinned", [True, False])
def test_c5_mixed_stream_two_host_threads(orc, pinned):
    """C5's block stream (RS16(400,100) where splitmix64(seed ^ b) % 8 == 0, else RS8(64,32),
    vec 1400; tools/bench_c5.py) in host memory, both sub-streams encoded and repaired through
    the host-resident pipelines from two host threads concurrently; parity and repaired bytes
    compared with the oracle block by block."""
    torch = _gpu()
    from norm_amd import NormDecoderRS8, NormDecoderRS16, NormEncoderRS8, NormEncoderRS16

    total = 640
    ids = np.arange(total, dtype=np.uint64)
    is16 = (_splitmix64(np.uint64(SEED) ^ ids) % np.uint64(8)) == 0
    specs = {"RS8": (orc.RS8, 64, 32, 16, NormEncoderRS8, NormDecoderRS8, np.flatnonzero(~is16)),
             "RS16": (orc.RS16, 400, 100, 50, NormEncoderRS16, NormDecoderRS16, np.flatnonzero(is16))}
    assert len(specs["RS16"][6]) > 40 and len(specs["RS8"][6]) > 400
    jobs = {}
    for name, (kind, k, m, er, E, D, sel) in specs.items():
        n = len(sel)
        src = np.zeros((n, k + m, VEC), np.uint8)
        for i, b in enumerate(sel):  # block id b of the stream, its own kind's source
            for s in range(k):
                src[i, s] = orc.fill_segment(int(b), s, VEC)
        ref = orc.encode_blocks(kind, k, m, VEC, src.copy())
        locs = np.zeros((n, m), np.uint16)
        cnts = np.full(n, er, np.uint16)
        for i, b in enumerate(sel):
            locs[i, :er] = orc.erasure_pattern(int(b), k, er)
        rx = ref.copy()
        for i in range(n):
            rx[i, locs[i, :er]] = 0
        want = rx.copy()
        st_ref = orc.decode_blocks(kind, k, m, VEC, want, locs, cnts)
        assert (st_ref == er).all() and np.array_equal(want, ref)
        if pinned:
            buf = torch.empty((n, k + m, VEC), dtype=torch.uint8, pin_memory=True).numpy()
            buf[:] = src
        else:
            buf = src
        enc, dec = E(), D()
        assert enc.Init(k, m, VEC) and dec.Init(k, m, VEC)
        jobs[name] = dict(buf=buf, ref=ref, rx=rx, locs=locs, cnts=cnts, enc=enc, dec=dec, k=k, er=er)

    errors = []

    def run(j):
        try:
            j["enc"].encode_blocks_host(j["buf"])
            j["parity_ok"] = np.array_equal(j["buf"], j["ref"])
            # the receiver side: erased copy repaired through the same kind of pipeline
            j["st"] = j["dec"].decode_blocks_host(j["rx"], j["locs"], j["cnts"])
        except Exception as e:  # surfaced in the main thread
            errors.append(e)

    th = [threading.Thread(target=run, args=(j,)) for j in jobs.values()]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not errors, errors
    for name, j in jobs.items():
        assert j["parity_ok"], f"{name} parity"
        assert (j["st"] == j["er"]).all(), f"{name} status"
        assert np.array_equal(j["rx"], j["ref"]), f"{name} repair"


@pytest.mark.gpu
def test_c5_full_share_device_resident(orc):
    """One GPU's whole C5 share (131,072 stream blocks: 114,726 RS8(64,32) + 16,346
    RS16(400,100), vec 1400, 26.8 GB in HBM, tools/bench_c5.py's device-resident step): encode
    both sub-streams, sampled blocks against the oracle's per-segment Encode, then erase 16 / 50
    source symbols per block and repair: every source byte of every block comes back."""
    torch = _gpu()
    import norm_amd as na

    total = 1 << 17
    ids = np.arange(total, dtype=np.uint64)
    is16 = (_splitmix64(np.uint64(SEED) ^ ids) % np.uint64(8)) == 0
    subs = [("RS8", orc.RS8, 64, 32, 16, na.NormEncoderRS8, na.NormDecoderRS8, int((~is16).sum()), SEED ^ 0x8),
            ("RS16", orc.RS16, 400, 100, 50, na.NormEncoderRS16, na.NormDecoderRS16, int(is16.sum()), SEED ^ 0x16)]
    assert (subs[0][7], subs[1][7]) == (114726, 16346)
    for name, kind, k, m, er, E, D, n, seed in subs:
        enc, dec = E(), D()
        assert enc.Init(k, m, VEC) and dec.Init(k, m, VEC)
        d = torch.zeros((n, k + m, VEC), dtype=torch.uint8, device="cuda")
        na.fill_blocks(d, k, VEC, seed)
        enc.encode_blocks(d)
        torch.cuda.synchronize()
        for b in (0, n // 2 + 3, n - 1):
            host = orc.make_blocks(k, m, VEC, 1, seed=seed, first_block=b)
            ref = orc.encode_blocks(kind, k, m, VEC, host)
            assert np.array_equal(d[b].cpu().numpy(), ref[0]), f"{name} block {b}"
        keep = d[:, :k].clone()
        locs, cnts = na.make_erasures(n, k, er, SEED, m)
        na.zero_erasures(d, locs, cnts, VEC)
        st = dec.decode_blocks(d, locs, cnts)
        torch.cuda.synchronize()
        assert bool((st == er).all()), name
        assert torch.equal(d[:, :k], keep), name
        del d, keep, st, locs, cnts
        torch.cuda.empty_cache()
