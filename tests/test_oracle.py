"""The oracle (CPU restatement) against the reference's own data and the code's invariants.

Pinning: GF(2^8) tables against tests/golden/galois_tables.json (compiled from the
reference's src/common/galois.cpp).  The RS generator/decoder and MDP LFSR have no
reference-produced vectors (the codec TUs need absent protolib headers; fecTest only
round-trips), so they are checked by the properties the reference algorithm guarantees:
systematic form, Lagrange/MDS structure, and encode -> erase -> decode round trips.
"""
import numpy as np
import pytest


def test_galois_tables_pinned(orc, galois_fixture):
    ginv, gexp, gm = orc.galois_tables()
    assert np.array_equal(ginv, galois_fixture["GINV"])
    assert np.array_equal(gexp, galois_fixture["GEXP"])
    assert np.array_equal(gm.reshape(-1), galois_fixture["GMULT"])


def test_rs8_field_is_reference_field(orc, galois_fixture):
    # RS8 builds its own tables from "101110001" (normEncoderRS8.cpp:81, :182-242); they
    # must be the same field as galois.cpp's constants.
    exp, log, inv = orc.gf8_tables()
    mul = orc.gf8_mul_table()
    assert np.array_equal(mul.reshape(-1), galois_fixture["GMULT"])
    assert np.array_equal(exp[:255], galois_fixture["GEXP"][:255])
    assert np.array_equal(exp[255:510], exp[:255])
    assert log[0] == 255                      # log(0) sentinel, normEncoderRS8.cpp:228
    assert inv[0] == 0 and galois_fixture["GINV"][0] == 1  # the two codebases' inverse(0) quirks
    assert np.array_equal(inv[1:], galois_fixture["GINV"][1:])
    for x in range(1, 256):
        assert mul[x, inv[x]] == 1


def test_gf16_field_polynomial(orc):
    exp, log, inv = orc.gf16_tables()
    assert exp[0] == 1 and exp[1] == 2
    assert exp[16] == 0x100B                  # alpha^16 = x^12 + x^3 + x + 1 (poly 0x1100B)
    assert len(set(exp[:65535].tolist())) == 65535
    assert log[0] == 65535


def test_splitmix64_known_answer(orc):
    # Vigna's splitmix64, state 0: first output mix(0x9E3779B97F4A7C15) = 0xE220A8397B1DCDAF
    assert orc.lib().orc_splitmix64_mix(0x9E3779B97F4A7C15) == 0xE220A8397B1DCDAF


def _gf8_lagrange(k, m, mul, exp, inv):
    x = [0] + [int(exp[(j - 1) % 255]) for j in range(1, k)]
    G = np.zeros((m, k), np.uint8)
    for p in range(m):
        y = int(exp[(k + p - 1) % 255])
        for j in range(k):
            num, den = 1, 1
            for l in range(k):
                if l != j:
                    num = mul[num, y ^ x[l]]
                    den = mul[den, x[j] ^ x[l]]
            G[p, j] = mul[num, inv[den]]
    return G


@pytest.mark.parametrize("k,m", [(1, 1), (2, 3), (16, 4), (64, 16), (64, 32), (40, 20)])
def test_rs8_generator_is_systematic_lagrange(orc, k, m):
    """The Vandermonde-invert-multiply generator (normEncoderRS8.cpp:428-450) equals the
    Lagrange basis of the points {0, a^0..a^(k-2)} at a^(k-1+p), computed independently."""
    exp, _, inv = orc.gf8_tables()
    mul = orc.gf8_mul_table()
    g = orc.generator(orc.RS8, k, m)
    assert np.array_equal(g[:k], np.eye(k, dtype=np.uint8))
    assert np.array_equal(g[k:], _gf8_lagrange(k, m, mul, exp, inv))


def test_rs8_generator_limits(orc):
    assert orc.generator(orc.RS8, 200, 56) is None   # k+m > 255 -> Init false
    assert orc.generator(orc.RS8, 200, 55) is not None
    assert np.all(orc.generator(orc.RS8, 64, 32)[64:] != 0)  # all 2048 coefficients non-zero


def _roundtrip(orc, kind, k, m, vec, nblocks, erasures, num_data=None, parity_erasures=0):
    blocks = orc.make_blocks(k, m, vec, nblocks, num_data=num_data)
    orc.encode_blocks(kind, k, m, vec, blocks, num_data)
    ref = blocks.copy()
    locs = np.zeros((nblocks, m), np.uint16)
    counts = np.zeros(nblocks, np.uint16)
    for b in range(nblocks):
        nd = k if num_data is None else int(num_data[b])
        src = orc.erasure_pattern(b, nd, min(erasures, nd))
        par = (nd + orc.erasure_pattern(b + 7777, m, parity_erasures)).astype(np.uint16)
        allp = np.concatenate([src, par])[: m]
        counts[b] = len(allp)
        locs[b, : len(allp)] = allp
        for s in allp:
            blocks[b, s, :] = 0
    status = orc.decode_blocks(kind, k, m, vec, blocks, locs, counts, num_data)
    assert np.array_equal(status, counts.astype(np.int32))
    for b in range(nblocks):
        nd = k if num_data is None else int(num_data[b])
        nb = vec if kind != orc.RS16 else vec // 2 * 2
        assert np.array_equal(blocks[b, :nd, :nb], ref[b, :nd, :nb])
        erased_par = [s for s in locs[b, : counts[b]] if s >= nd]
        for s in erased_par:
            assert not blocks[b, s].any()     # parity is never filled (normEncoderRS8.cpp:732)
    return ref


@pytest.mark.parametrize("kind", [1, 2, 3])
def test_roundtrip_full_blocks(orc, kind):
    _roundtrip(orc, kind, 64, 32, 200, 3, 16)
    _roundtrip(orc, kind, 64, 32, 200, 3, 32)


@pytest.mark.parametrize("kind", [1, 2, 3])
def test_roundtrip_mixed_source_and_parity_erasures(orc, kind):
    _roundtrip(orc, kind, 32, 16, 96, 4, 10, parity_erasures=6)


@pytest.mark.parametrize("kind", [1, 2, 3])
def test_roundtrip_shortened_blocks(orc, kind):
    nd = np.array([40, 64, 1, 17], np.uint16)
    _roundtrip(orc, kind, 64, 16, 120, 4, 12, num_data=nd, parity_erasures=2)


def test_rs16_odd_vector_size_ignores_last_byte(orc):
    ref = _roundtrip(orc, orc.RS16, 40, 10, 65, 2, 10)
    assert not ref[:, 40:, 64].any()           # parity's last byte stays 0


def test_rs16_fectest_shape(orc):
    # src/common/fecTest.cpp:13-16: RS16, k=400, m=100, seg=64, 2 erasures over all n positions
    _roundtrip(orc, orc.RS16, 400, 100, 64, 1, 2)


def test_decode_only_parity_erased(orc):
    k, m, vec = 16, 4, 32
    blocks = orc.make_blocks(k, m, vec, 1)
    orc.encode_blocks(orc.RS8, k, m, vec, blocks)
    ref = blocks.copy()
    locs = np.array([[17, 19, 0, 0]], np.uint16)
    blocks[0, 17] = 0
    blocks[0, 19] = 0
    st = orc.decode_blocks(orc.RS8, k, m, vec, blocks, locs, np.array([2], np.uint16))
    assert st[0] == 2
    assert np.array_equal(blocks[0, :k], ref[0, :k])
    assert not blocks[0, 17].any() and not blocks[0, 19].any()


def test_mdp_generator_roots(orc):
    exp, _, _ = orc.gf8_tables()
    mul = orc.gf8_mul_table()
    for m in (1, 4, 32):
        g = orc.mdp_generator_poly(m)
        assert g[m] == 1
        for n in range(1, m + 1):
            a, acc, p = int(exp[n]), 0, 1
            for c in g:
                acc ^= mul[int(c), p]
                p = mul[p, a]
            assert acc == 0


def test_erasure_pattern_spec(orc):
    e = orc.erasure_pattern(5, 64, 16)
    assert len(e) == 16 and len(set(e.tolist())) == 16
    assert np.all(np.diff(e.astype(int)) > 0) and e.max() < 64
    assert np.array_equal(e, orc.erasure_pattern(5, 64, 16))
