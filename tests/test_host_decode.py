"""One-block Decode on the host CPU (nfec_decode_vectors_host, the drop-in's default for RS8
and small RS16): the closed-form repair map of the block -- the first surviving parities in
place of the erased source (NormDecoderRS8::Decode, src/common/normEncoderRS8.cpp:652-757;
RS16 :650-755) -- applied with the host region products.  Against the oracle and against the
GPU per-call path (nfec_decode_vectors), byte for byte and status for status: full and
shortened blocks, parity erasures, NULL missing parity, erased buffers that are not zero
(the reference XORs into them), undecodable blocks and invalid lists."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from norm_amd import NFEC_MDP, NFEC_RS8, NFEC_RS16, NormDecoderMDP, NormDecoderRS8, NormDecoderRS16  # noqa: E402

DECODER = {NFEC_RS8: NormDecoderRS8, NFEC_RS16: NormDecoderRS16, NFEC_MDP: NormDecoderMDP}


def _case(orc, kind, k, m, vec, nd, es, ep, rng, junk=False):
    host = orc.make_blocks(k, m, vec, 1, num_data=np.array([nd], np.uint16) if nd < k else None,
                           seed=int(rng.integers(1, 1 << 30)))
    clean = orc.encode_blocks(kind, k, m, vec, host, np.array([nd], np.uint16) if nd < k else None)
    e = np.sort(np.concatenate([rng.choice(nd, es, replace=False), nd + rng.choice(m, ep, replace=False)]))
    rx = clean[0, :nd + m].copy()
    for s in e:
        rx[s] = 0
        if junk and s < nd:
            rx[s, :vec] = rng.integers(0, 256, vec, dtype=np.uint8)
    return clean, rx, [int(x) for x in e]


def _decode(dec, rx, nd, locs, host, null_parity):
    vl = [rx[s].copy() for s in range(rx.shape[0])]
    if null_parity:
        for s in locs:
            if s >= nd:
                vl[s] = None
    st = dec.Decode(vl, nd, len(locs), locs, host=host)
    return st, vl


CASES = [
    # kind, k, m, vec, nd, source erasures, parity erasures, junk in erased buffers, NULL parity
    (NFEC_RS8, 64, 32, 1408, 64, 16, 0, False, False),
    (NFEC_RS8, 64, 32, 1400, 64, 10, 5, False, True),
    (NFEC_RS8, 16, 4, 1408, 16, 4, 0, False, False),
    (NFEC_RS8, 200, 55, 1401, 150, 40, 10, True, True),
    (NFEC_RS8, 3, 100, 64, 3, 3, 50, False, True),
    (NFEC_RS8, 127, 128, 72, 100, 100, 27, True, False),
    (NFEC_RS8, 10, 7, 8, 4, 4, 3, False, False),
    (NFEC_RS16, 400, 20, 1400, 400, 12, 3, False, True),
    (NFEC_RS16, 300, 40, 1401, 250, 30, 5, True, False),
    (NFEC_RS16, 10, 4, 64, 10, 4, 0, False, False),
    # MDP: erased source arrives zero-filled (normObject.cpp:1579), missing parity NULL
    (NFEC_MDP, 64, 32, 1408, 64, 16, 0, False, False),
    (NFEC_MDP, 64, 32, 1400, 50, 10, 6, False, True),
    (NFEC_MDP, 200, 55, 1401, 150, 30, 20, False, True),
    (NFEC_MDP, 10, 7, 8, 4, 4, 3, False, False),
    (NFEC_MDP, 1, 1, 64, 1, 1, 0, False, False),
    # repairs past 8 MiB of products: the host path splits the vectors over threads
    (NFEC_RS8, 128, 127, 8192, 128, 100, 20, True, True),
    (NFEC_RS8, 128, 127, 8190, 120, 90, 30, False, False),
    (NFEC_MDP, 128, 127, 8192, 128, 100, 20, False, True),
    (NFEC_RS16, 300, 64, 8000, 300, 64, 0, False, False),
]


@pytest.mark.parametrize("kind,k,m,vec,nd,es,ep,junk,nullp", CASES)
def test_host_decode_matches_oracle_and_gpu(orc, kind, k, m, vec, nd, es, ep, junk, nullp):
    rng = np.random.default_rng(k * 131 + m + nd)
    clean, rx, locs = _case(orc, kind, k, m, vec, nd, es, ep, rng, junk)
    st_ref, ref = _oracle_one(orc, kind, k, m, vec, rx, nd, locs)
    dec = DECODER[kind]()
    assert dec.Init(k, m, vec)
    outs = {}
    for host in (True, False):
        st, vl = _decode(dec, rx, nd, locs, host, nullp)
        outs[host] = (st, [None if v is None else v.copy() for v in vl])
    assert outs[True][0] == outs[False][0] == st_ref
    for s in range(nd):
        assert np.array_equal(outs[True][1][s], ref[s]), s
        assert np.array_equal(outs[False][1][s], ref[s]), s
    if not junk:
        for s in range(nd):
            assert np.array_equal(outs[True][1][s], clean[0, s]), s


def _oracle_one(orc, kind, k, m, vec, rx, nd, locs):
    ref = rx[None].copy()
    if nd < k:
        ref = np.concatenate([ref, np.zeros((1, k - nd, ref.shape[2]), np.uint8)], 1)
    nloc = np.zeros((1, m), np.uint16)
    nloc[0, :len(locs)] = locs
    st = orc.decode_blocks(kind, k, m, vec, ref, nloc, np.array([len(locs)], np.uint16),
                           np.array([nd], np.uint16) if nd < k else None)
    return int(st[0]), ref[0]


@pytest.mark.parametrize("kind", [NFEC_RS8, NFEC_MDP])
def test_host_decode_random(orc, kind):
    """many random RS8 / MDP blocks: shapes, shortening, source and parity erasures"""
    rng = np.random.default_rng(99 + kind)
    for it in range(60):
        k = int(rng.integers(1, 120))
        m = int(rng.integers(1, min(100, 255 - k) + 1))
        vec = int(rng.choice([8, 64, 100, 1400, 1408]))
        nd = int(rng.integers(1, k + 1))
        es = int(rng.integers(0, min(nd, m) + 1))
        ep = int(rng.integers(0, m - es + 1))
        clean, rx, locs = _case(orc, kind, k, m, vec, nd, es, ep, rng)
        st_ref, ref = _oracle_one(orc, kind, k, m, vec, rx, nd, locs)
        dec = DECODER[kind]()
        assert dec.Init(k, m, vec)
        st, vl = _decode(dec, rx, nd, locs, True, kind == NFEC_MDP)
        assert st == st_ref, (it, k, m, nd, locs)
        for s in range(nd):
            assert np.array_equal(vl[s], ref[s]), (it, s)


@pytest.mark.parametrize("kind", [NFEC_RS8, NFEC_MDP])
def test_host_decode_undecodable_and_invalid(orc, kind):
    """more erasures than (surviving) parity, unsorted and out-of-range lists: status 0, block
    untouched, as the GPU path"""
    k, m, vec = 20, 4, 64
    dec = DECODER[kind]()
    assert dec.Init(k, m, vec)
    rng = np.random.default_rng(3)
    clean, rx, _ = _case(orc, kind, k, m, vec, k, 0, 0, rng)
    bad_lists = [[3, 1], [0, 25], [5, 5], [0, 1, 2, 3, 4]] + ([[0, 1, 2, 3, 21]] if kind == NFEC_RS8 else [])
    for locs in bad_lists:
        for host in (True, False):
            vl = [rx[s].copy() for s in range(k + m)]
            st = dec.Decode(vl, k, len(locs), locs, host=host)
            assert st == 0, (locs, host)
            for s in range(k + m):
                assert np.array_equal(vl[s], rx[s])


def test_drop_in_policy():
    """NORM-sized repairs on the host, big ones on the GPU"""
    from norm_amd import _native as N

    d8, d16, dm = NormDecoderRS8(), NormDecoderRS16(), NormDecoderMDP()
    b8, bm, b16 = NormDecoderRS8(), NormDecoderMDP(), NormDecoderRS16()
    assert d8.Init(64, 32, 1408) and d16.Init(400, 60, 1400) and dm.Init(64, 32, 1408)
    assert b8.Init(128, 127, 65535) and bm.Init(128, 127, 65535) and b16.Init(4000, 60, 65535)
    pref = N.lib().nfec_decode_host_preferred
    assert pref(d8._h, 64, 16) == 1 and pref(dm._h, 64, 16) == 1
    assert pref(d16._h, 400, 10) == 1 and pref(d16._h, 400, 50) == 1
    assert pref(b8._h, 128, 100) == 0 and pref(bm._h, 128, 100) == 0 and pref(b16._h, 4000, 60) == 0
    assert pref(b8._h, 128, 10) == 1


def test_host_decode_concurrent_calls(orc):
    """one decoder, four caller threads (the host path keeps no per-call state in the codec):
    every block repaired exactly, including the threaded-size ones"""
    import threading

    k, m = 128, 127
    dec = NormDecoderRS8()
    assert dec.Init(k, m, 8192)
    jobs = []
    for i in range(8):
        rng = np.random.default_rng(700 + i)
        es = 4 if i % 2 else 100   # 4 erasures: 4 MB of products, one thread; 100: threaded
        clean, rx, locs = _case(orc, NFEC_RS8, k, m, 8192, k, es, 0, rng)
        jobs.append((clean, rx, locs))
    errors = []

    def work(idx):
        for j in range(idx, len(jobs), 4):
            clean, rx, locs = jobs[j]
            for _ in range(3):
                vl = [rx[s].copy() for s in range(rx.shape[0])]
                st = dec.Decode(vl, k, len(locs), locs, host=True)
                if st != len(locs) or any(not np.array_equal(vl[s], clean[0, s]) for s in locs):
                    errors.append((j, st))

    th = [threading.Thread(target=work, args=(i,)) for i in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors
