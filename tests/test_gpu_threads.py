"""Thread safety of the C ABI (SURVEY.md 8b "Threading": must be thread-safe across codec
instances).  NORM runs one codec per session / remote sender, and an application may run
several NormInstances on their own threads (normApi.cpp:55,126), so codecs are driven from
several host threads at once here, every result checked against the oracle.  Host-batch
calls on ONE codec from two threads are serialised by the codec (nfec.h), also checked."""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from norm_amd import (NFEC_MDP, NFEC_RS8, NFEC_RS16, NormDecoderMDP, NormDecoderRS8,  # noqa: E402
                      NormDecoderRS16, NormEncoderMDP, NormEncoderRS8, NormEncoderRS16)

ENC = {NFEC_RS8: NormEncoderRS8, NFEC_RS16: NormEncoderRS16, NFEC_MDP: NormEncoderMDP}
DEC = {NFEC_RS8: NormDecoderRS8, NFEC_RS16: NormDecoderRS16, NFEC_MDP: NormDecoderMDP}


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    from norm_amd import device_count

    assert torch.cuda.is_available() and device_count() >= 1


def _case(orc, kind, k, m, vec, nb, er, off):
    host = orc.make_blocks(k, m, vec, nb, first_block=off)
    ref = orc.encode_blocks(kind, k, m, vec, host.copy())
    locs = np.zeros((nb, m), np.uint16)
    counts = np.full(nb, er, np.uint16)
    for b in range(nb):
        locs[b, :er] = orc.erasure_pattern(b + off, k, er)
    return host, ref, locs, counts


def _run_threads(fns):
    errors = []

    def wrap(f):
        try:
            f()
        except BaseException as e:  # noqa: BLE001 -- reported by the main thread
            errors.append(e)

    th = [threading.Thread(target=wrap, args=(f,)) for f in fns]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=600)
    assert not any(t.is_alive() for t in th), "a worker thread hung"
    if errors:
        raise errors[0]


def test_four_threads_own_codecs(orc):
    shapes = [(NFEC_RS8, 64, 32, 1400, 96, 16), (NFEC_RS16, 100, 20, 1400, 24, 12),
              (NFEC_MDP, 64, 16, 1400, 40, 9), (NFEC_RS8, 32, 8, 1397, 64, 8)]
    cases = [_case(orc, *s, off=1000 * i) for i, s in enumerate(shapes)]
    results = {}

    def worker(i):
        kind, k, m, vec, nb, er = shapes[i]
        host, ref, locs, counts = cases[i]
        enc, dec = ENC[kind](), DEC[kind]()
        assert enc.Init(k, m, vec) and dec.Init(k, m, vec)
        ok = True
        for it in range(3):
            # batch encode of a strided host batch
            buf = host.copy()
            enc.encode_blocks_host(buf)
            ok &= np.array_equal(buf, ref)
            # receiver repair of NORM-style segment lists (missing parity as None)
            rx = ref.copy()
            vecs = []
            for b in range(nb):
                rx[b, locs[b, :er]] = 0
                vecs.append([rx[b, s] for s in range(k)] + [rx[b, k + p] for p in range(m)])
            st = dec.decode_vectors_host(vecs, locs, counts)
            ok &= bool((st == er).all()) and np.array_equal(rx, ref)
            # per-call Decode (nfec_decode_vectors) on one block
            one = ref[it].copy()
            one[locs[it, :er]] = 0
            lst = [one[s] for s in range(k + m)]
            ok &= dec.Decode(lst, k, er, [int(x) for x in locs[it, :er]]) == er
            ok &= np.array_equal(one, ref[it])
        results[i] = ok

    _run_threads([lambda i=i: worker(i) for i in range(4)])
    assert results == {0: True, 1: True, 2: True, 3: True}


def test_two_threads_one_codec_host_batches(orc):
    """nfec_encode_host / nfec_decode_host on ONE codec from two threads: the codec's staging
    pipeline is shared, so the calls are serialised; both must come back exact."""
    k, m, vec = 64, 32, 1400
    a = _case(orc, NFEC_RS8, k, m, vec, 300, 16, 0)
    b = _case(orc, NFEC_RS8, k, m, vec, 200, 16, 5000)
    enc, dec = NormEncoderRS8(), NormDecoderRS8()
    assert enc.Init(k, m, vec) and dec.Init(k, m, vec)
    out = {}

    def worker(name, case):
        host, ref, locs, counts = case
        for it in range(3):
            buf = host.copy()
            enc.encode_blocks_host(buf)
            rx = buf.copy()
            for blk in range(rx.shape[0]):
                rx[blk, locs[blk, :16]] = 0
            st = dec.decode_blocks_host(rx, locs, counts)
            out[(name, it)] = np.array_equal(buf, ref) and bool((st == 16).all()) and np.array_equal(rx, ref)

    _run_threads([lambda: worker("a", a), lambda: worker("b", b)])
    assert all(out.values()) and len(out) == 6
