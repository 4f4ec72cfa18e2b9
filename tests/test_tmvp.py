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
