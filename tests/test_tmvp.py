"""RS16 Toeplitz split (norm_amd/csrc/kernels_tmvp.hip) on the CPU.

1. The factorisation the split relies on, against the oracle's restatement of the reference
   generator (NormEncoderRS16::Init, src/common/normEncoderRS16.cpp:399-461):
   G[p][j] = W(y_p) * T[p][j] * c_j with T Toeplitz, and one Karatsuba step of the Toeplitz
   product (three half-size products) reproducing the full product G d.
2. The bit-sliced constant multiply of gf16_bs.hpp (what the prescale / postscale kernels run),
   compiled for the host, against table multiplication.
"""
import os
import subprocess

import numpy as np
import pytest

from oracle import pyoracle as orc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
Q = 65535


@pytest.fixture(scope="module")
def gf():
    e, lg, inv = orc.gf16_tables()

    def mul(a, b):
        return 0 if a == 0 or b == 0 else int(e[(lg[a] + lg[b]) % Q])

    return e, lg, inv, mul


def _factors(gf, k, m):
    e, lg, inv, mul = gf
    ex = lambda n: int(e[n % Q])  # noqa: E731
    x = [0] + [ex(j - 1) for j in range(1, k)]
    y = [ex(k - 1 + p) for p in range(m)]

    def prod_diff(z, skip=None):
        r = 1
        for i, xl in enumerate(x):
            if i != skip:
                r = mul(r, z ^ xl)
        return r

    w = [prod_diff(v) for v in y]
    c = [0] + [mul(ex(-(j - 1)), int(inv[prod_diff(x[j], j)])) for j in range(1, k)]
    t = lambda p, j: int(inv[1 ^ ex(k + p - j)])  # noqa: E731
    return w, c, t


@pytest.mark.parametrize("k,m", [(64, 16), (128, 32), (40, 10)])
def test_generator_factorisation(orc, gf, k, m):
    _, _, inv, mul = gf
    G = orc.generator(orc.RS16, k, m)[k:]
    w, c, t = _factors(gf, k, m)
    for p in range(m):
        for j in range(1, k):
            assert int(G[p][j]) == mul(w[p], mul(t(p, j), c[j])), (p, j)
        # column 0 (the point 0): G[p][0] = W(y_p) / (y_p W'(0)), added by the postscale
        assert int(G[p][0]) != 0


@pytest.mark.parametrize("k,m", [(64, 16), (128, 32)])
def test_karatsuba_step_reproduces_product(orc, gf, k, m):
    _, _, _, mul = gf
    G = orc.generator(orc.RS16, k, m)[k:]
    w, c, t = _factors(gf, k, m)
    rng = np.random.default_rng(7)
    d = rng.integers(0, 65536, size=(k, 3))
    ref = np.zeros((m, 3), np.int64)
    for p in range(m):
        for j in range(k):
            for s in range(3):
                ref[p, s] ^= mul(int(G[p][j]), int(d[j, s]))
    cw, half = m // 2, k // 2
    p0 = np.zeros((cw, 3), np.int64)
    p1 = np.zeros_like(p0)
    p2 = np.zeros_like(p0)
    for v in range(half):
        a = 2 * (v // cw) * cw + v % cw
        b = a + cw
        sv = [mul(c[a], int(d[a, s])) ^ mul(c[b], int(d[b, s])) for s in range(3)]  # prescale
        for p in range(cw):
            A = t(p, a)
            e1 = mul(t(p, b) ^ A, c[b])
            e2 = mul(t(p + cw, a) ^ A, c[a])
            for s in range(3):
                p0[p, s] ^= mul(A, sv[s])
                p1[p, s] ^= mul(e1, int(d[b, s]))
                p2[p, s] ^= mul(e2, int(d[a, s]))
    out = np.zeros_like(ref)
    for p in range(cw):  # postscale
        for s in range(3):
            out[p, s] = mul(w[p], int(p0[p, s] ^ p1[p, s])) ^ mul(int(G[p][0]), int(d[0, s]))
            out[p + cw, s] = mul(w[p + cw], int(p0[p, s] ^ p2[p, s])) ^ mul(int(G[p + cw][0]), int(d[0, s]))
    assert np.array_equal(out, ref)


def test_bitsliced_constant_multiply(gf, tmp_path):
    e, lg, inv, mul = gf
    exe = tmp_path / "bs16_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", str(exe), os.path.join(ROOT, "tests", "native", "bs16_check.cpp")],
                   check=True)
    rng = np.random.default_rng(3)
    consts = [0, 1, 2, 0x8000, 0xFFFF] + [int(v) for v in rng.integers(1, 65536, 20)]
    lines, expect = [], []
    for cst in consts:
        rows = [0] * 16
        for q in range(16):
            v = mul(cst, 1 << q)
            for p in range(16):
                rows[p] |= ((v >> p) & 1) << q
        syms = [int(v) for v in rng.integers(0, 65536, 32)]
        syms[:3] = [0, 1, 0xFFFF]
        lines.append(" ".join(map(str, rows + syms)))
        expect.append([mul(cst, s) for s in syms])
    out = subprocess.run([str(exe)], input="\n".join(lines) + "\n", capture_output=True, text=True, check=True).stdout
    got = [[int(v) for v in ln.split()] for ln in out.strip().splitlines()]
    assert got == expect


def _level2(gf, k, m, d, G, w, c, t):
    """Two Karatsuba levels (kernels_tmvp.hip, rs16_tmvp_plan with two levels): level 1 as above;
    level 2 splits each of the three (m/2)-row products the same way within each cw-wide chunk of
    its columns, whose cw x cw blocks are Toeplitz: nine (m/4)-row products over k/4 columns.
    The diag(c) of P1 / P2 moves to their data side for the alpha products (sums of scaled
    columns) and stays in the coefficients of the beta / gamma products (raw columns)."""
    _, _, _, mul = gf
    cw, hw, nq = m // 2, m // 4, k // m
    S = d.shape[1]
    # N_X[p][a] for p < cw over level-1 virtual column (q, i), i < cw: the Toeplitz parts
    N = [lambda p, q, i: t(p, 2 * q * cw + i),
         lambda p, q, i: t(p, 2 * q * cw + cw + i) ^ t(p, 2 * q * cw + i),
         lambda p, q, i: t(p + cw, 2 * q * cw + i) ^ t(p, 2 * q * cw + i)]
    # level-1 inputs: z_0 = c_a d_a + c_b d_b, z_1 = c_b d_b, z_2 = c_a d_a (per (q, i))
    col = {0: None, 1: lambda q, i: 2 * q * cw + cw + i, 2: lambda q, i: 2 * q * cw + i}

    def z(X, q, i, s):
        a, b = 2 * q * cw + i, 2 * q * cw + cw + i
        if X == 0:
            return mul(c[a], int(d[a, s])) ^ mul(c[b], int(d[b, s]))
        j = col[X](q, i)
        return mul(c[j], int(d[j, s]))

    P = [np.zeros((cw, S), np.int64) for _ in range(3)]
    for X in range(3):
        pa = np.zeros((hw, S), np.int64)
        pb = np.zeros_like(pa)
        pg = np.zeros_like(pa)
        for q in range(nq):
            for i in range(hw):
                for p in range(hw):
                    al = N[X](p, q, i)
                    be = N[X](p, q, hw + i)       # top-right block
                    ga = N[X](hw + p, q, i)       # bottom-left block
                    assert N[X](hw + p, q, hw + i) == al   # bottom-right = top-left (Toeplitz)
                    for s in range(S):
                        z0, z1 = z(X, q, i, s), z(X, q, hw + i, s)
                        pa[p, s] ^= mul(al, z0 ^ z1)
                        pb[p, s] ^= mul(be ^ al, z1)
                        pg[p, s] ^= mul(ga ^ al, z0)
        P[X][:hw] = pa ^ pb
        P[X][hw:] = pa ^ pg
    out = np.zeros((m, S), np.int64)
    for p in range(cw):
        for s in range(S):
            out[p, s] = mul(w[p], int(P[0][p, s] ^ P[1][p, s])) ^ mul(int(G[p][0]), int(d[0, s]))
            out[p + cw, s] = mul(w[p + cw], int(P[0][p, s] ^ P[2][p, s])) ^ mul(int(G[p + cw][0]), int(d[0, s]))
    return out


@pytest.mark.parametrize("k,m", [(16, 8), (32, 8), (64, 16)])
def test_two_karatsuba_levels_reproduce_product(orc, gf, k, m):
    _, _, _, mul = gf
    G = orc.generator(orc.RS16, k, m)[k:]
    w, c, t = _factors(gf, k, m)
    rng = np.random.default_rng(11)
    d = rng.integers(0, 65536, size=(k, 2))
    ref = np.zeros((m, 2), np.int64)
    for p in range(m):
        for j in range(k):
            for s in range(2):
                ref[p, s] ^= mul(int(G[p][j]), int(d[j, s]))
    assert np.array_equal(_level2(gf, k, m, d, G, w, c, t), ref)


def _split_levels(gf, k, m, L, d, G, w, c, t):
    """L Karatsuba levels of the Toeplitz split, as rs16_tmvp_plan_levels / the level-L kernels lay
    them out (the general form of the two tests above).  A product is a path of L digits
    (0 alpha, 1 beta, 2 gamma; product index sum d_l 3^(L-l)).  The root takes the Toeplitz part
    T[p][q m + i] over the scaled source u_j = c_j d_j, chunk q of m columns; a node of width r
    (its Toeplitz blocks r x r, input per chunk r values) splits into alpha = top-left block over
    (input first half + second half), beta = top-right - top-left over the second half, gamma =
    bottom-left - top-left over the first half, r/2 rows each.  Output row block b (L bits, level
    1 the top bit) sums the products whose digits are alpha, or beta where b's bit is 0, or gamma
    where it is 1; parity = W (sum) + G[p][0] d_0."""
    _, _, _, mul = gf
    r, nq, S = m >> L, k // m, d.shape[1]
    u = [[mul(c[j], int(d[j, s])) for s in range(S)] for j in range(k)]

    def inp(path, q, i, s):
        if not path:
            return u[q * m + i][s]
        par, dg, half = path[:-1], path[-1], m >> len(path)
        if dg == 0:
            return inp(par, q, i, s) ^ inp(par, q, i + half, s)
        return inp(par, q, i + half, s) if dg == 1 else inp(par, q, i, s)

    def M(path, q, p, i):
        if not path:
            return t(p, q * m + i)
        par, dg, half = path[:-1], path[-1], m >> len(path)
        if dg == 0:
            return M(par, q, p, i)
        if dg == 1:
            return M(par, q, p, i + half) ^ M(par, q, p, i)
        return M(par, q, p + half, i) ^ M(par, q, p, i)

    import itertools
    paths = list(itertools.product(range(3), repeat=L))
    P = {}
    for path in paths:
        acc = np.zeros((r, S), np.int64)
        for q in range(nq):
            for i in range(r):
                x = [inp(path, q, i, s) for s in range(S)]
                for p in range(r):
                    co = M(path, q, p, i)
                    for s in range(S):
                        acc[p, s] ^= mul(co, x[s])
        P[path] = acc
    out = np.zeros((m, S), np.int64)
    for b in range(1 << L):
        R = np.zeros((r, S), np.int64)
        for path in paths:
            if all(dg == 0 or (dg == 1) == (((b >> (L - 1 - l)) & 1) == 0) for l, dg in enumerate(path)):
                R ^= P[path]
        for p in range(r):
            row = b * r + p
            for s in range(S):
                out[row, s] = mul(w[row], int(R[p, s])) ^ mul(int(G[row][0]), int(d[0, s]))
    return out


@pytest.mark.parametrize("k,m,L", [(16, 8, 1), (16, 8, 2), (16, 8, 3), (32, 8, 3), (64, 16, 3), (32, 16, 2)])
def test_karatsuba_levels_reproduce_product(orc, gf, k, m, L):
    _, _, _, mul = gf
    G = orc.generator(orc.RS16, k, m)[k:]
    w, c, t = _factors(gf, k, m)
    rng = np.random.default_rng(13 + L)
    d = rng.integers(0, 65536, size=(k, 2))
    ref = np.zeros((m, 2), np.int64)
    for p in range(m):
        for j in range(k):
            for s in range(2):
                ref[p, s] ^= mul(int(G[p][j]), int(d[j, s]))
    assert np.array_equal(_split_levels(gf, k, m, L, d, G, w, c, t), ref)
