"""The algebra behind the one-pass RS8 repair (rs8_plan_rt_kernel, kernels_plan.hip), on the CPU
against the oracle's generator (the reference's Init, normEncoderRS8.cpp:400-462):

  * the generator's parity rows are a scaled Cauchy matrix, G[p][j] = a_p b_j / (y_p + x_j) with
    x_j = 0 (j = 0) or alpha^(j-1) and y_p = alpha^(k-1+p) -- the points the plan uses;
  * the closed-form repair map W (e x numData) equals A^-1 [P_S | G_{S,R}] computed by plain
    Gauss-Jordan elimination, where A = G_{S,E} and S the first e surviving parities in slot
    order (the reference's substitute scan, normEncoderRS8.cpp:660-718):
        erased column E_r:  W[s][E_r] = A^-1[s][r]
        received column j:  W[s][j] = b_j / b_{E_s} * prod_s'(x_j + x_s') / prod_t(x_j + y_t)
                                     * prod_t(x_s + y_t) / prod_{s' != s}(x_s + x_s') / (x_s + x_j)
CPU only."""
import numpy as np
import pytest

from oracle import pyoracle as orc


def _field():
    ex, lg, inv = orc.gf8_tables()
    mul = orc.gf8_mul_table()
    return ex, lg, inv, mul


def _inv_matrix(A, mul, inv):
    n = A.shape[0]
    M = np.concatenate([A.copy(), np.eye(n, dtype=np.uint8)], axis=1)
    for c in range(n):
        p = next(r for r in range(c, n) if M[r, c])
        M[[c, p]] = M[[p, c]]
        M[c] = mul[inv[M[c, c]]][M[c]]
        for r in range(n):
            if r != c and M[r, c]:
                M[r] ^= mul[M[r, c]][M[c]]
    return M[:, n:]


def _matmul(A, B, mul):
    out = np.zeros((A.shape[0], B.shape[1]), np.uint8)
    for i in range(A.shape[0]):
        for t in range(A.shape[1]):
            if A[i, t]:
                out[i] ^= mul[A[i, t]][B[t]]
    return out


@pytest.mark.parametrize("k,m", [(64, 32), (16, 4), (200, 55), (3, 100), (127, 128)])
def test_generator_is_scaled_cauchy(k, m):
    ex, lg, inv, mul = _field()
    g = orc.generator(orc.RS8, k, m)[k:]
    x = [0] + [int(ex[j - 1]) for j in range(1, k)]
    y = [int(ex[(k - 1 + p) % 255]) for p in range(m)]
    # C[p][j] = G[p][j] * (y_p + x_j) must be rank one: a_p b_j
    C = np.array([[mul[g[p, j]][y[p] ^ x[j]] for j in range(k)] for p in range(m)], np.uint8)
    assert (C != 0).all()
    for p in range(m):
        ratio = mul[C[p, 0]][inv[C[0, 0]]]
        assert np.array_equal(C[p], mul[ratio][C[0]])


@pytest.mark.parametrize("k,m,nd,es,ep,seed", [(64, 32, 64, 16, 0, 1), (64, 32, 64, 16, 5, 2), (16, 4, 16, 4, 0, 3),
                                              (200, 55, 150, 40, 10, 4), (32, 16, 20, 9, 3, 5), (10, 7, 10, 7, 0, 6)])
def test_closed_form_repair_map(k, m, nd, es, ep, seed):
    ex, lg, inv, mul = _field()
    G = orc.generator(orc.RS8, k, m)[k:]
    rng = np.random.default_rng(seed)
    E = sorted(rng.choice(nd, es, replace=False).tolist())
    lost_par = set(rng.choice(m, ep, replace=False).tolist())
    S = [p for p in range(m) if p not in lost_par][:es]
    R = [j for j in range(nd) if j not in E]
    x = [0] + [int(ex[j - 1]) for j in range(1, k)]
    y = [int(ex[(k - 1 + p) % 255]) for p in range(m)]
    # column scalings from the rank-one structure (a_0 = 1): b_j = G[0][j] (y_0 + x_j)
    b = [int(mul[G[0, j]][y[0] ^ x[j]]) for j in range(k)]
    L = lambda v: int(lg[v])  # noqa: E731

    # direct: W = A^-1 [ I (parity columns) | G_{S,R} ]
    A = G[np.ix_(S, E)]
    Ai = _inv_matrix(A, mul, inv)
    direct = {}
    for r, e_col in enumerate(E):
        direct[e_col] = Ai[:, r]
    WR = _matmul(Ai, G[np.ix_(S, R)], mul)
    for i, j in enumerate(R):
        direct[j] = WR[:, i]

    # closed form (rs8_plan_rt_kernel): lA[s], lB[t], lC[j] in the log domain, mod 255
    xs = [x[c] for c in E]
    yt = [y[p] for p in S]
    lA = [(-L(b[E[s]]) + sum(L(xs[s] ^ yt[t]) for t in range(es))
           - sum(L(xs[s] ^ xs[u]) for u in range(es) if u != s)) % 255 for s in range(es)]
    a = [int(mul[mul[G[p, 0]][y[p] ^ x[0]]][inv[b[0]]]) for p in range(m)]  # a_p = G[p][0] (y_p + x_0) / b_0
    lB = [(-L(a[S[t]]) + sum(L(yt[t] ^ xs[s]) for s in range(es))
           - sum(L(yt[t] ^ yt[u]) for u in range(es) if u != t)) % 255 for t in range(es)]
    for j in range(nd):
        if j in E:
            r = E.index(j)
            col = [int(ex[(lA[s] + lB[r] - L(xs[s] ^ yt[r])) % 255]) for s in range(es)]
        else:
            lC = (L(b[j]) + sum(L(x[j] ^ xs[s]) for s in range(es)) - sum(L(x[j] ^ yt[t]) for t in range(es))) % 255
            col = [int(ex[(lA[s] + lC - L(xs[s] ^ x[j])) % 255]) for s in range(es)]
        assert col == [int(v) for v in direct[j]], j
