"""The closed form of the MDP repair coefficients (mdp_plan_kernel, kernels_plan.hip) against the
Forney sum the plan used to evaluate term by term (the reference decoder's algebra,
normEncoderMDP.cpp Decode): with Lambda the erasure locator, beta_r the inverse position of
erased source r, gamma_v the position of survivor v, w = gamma_v beta_r,

    Dinv_r gamma_v sum_{u<m} Lambda_u(beta_r) w^(m-1-u)
      == Dinv_r beta_r^m gamma_v^(m+1) Lambda(1/gamma_v) / (w + 1)

over random shortened blocks and erasure sets.  CPU only (GF(2^8) from the oracle's tables)."""
import numpy as np

from oracle import pyoracle as orc


def test_forney_closed_form():
    ex, lg, inv = orc.gf8_tables()
    mul = orc.gf8_mul_table()

    def M(a, b):
        return int(mul[a][b])

    def P(a, e):
        return (0 if e else 1) if a == 0 else int(ex[(int(lg[a]) * e) % 255])

    rng = np.random.default_rng(1)
    checked = 0
    for _ in range(120):
        k = int(rng.integers(2, 100))
        m = int(rng.integers(1, min(60, 255 - k) + 1))
        nd = int(rng.integers(1, k + 1))
        nvecs = nd + m
        locs = sorted(rng.choice(nvecs, int(rng.integers(1, m + 1)), replace=False).tolist())
        es = sum(1 for loc in locs if loc < nd)
        if es == 0:
            continue
        deg = 2 * m
        lam = [1] + [0] * (deg - 1)
        for loc in locs:
            X = int(ex[nvecs - 1 - loc])
            lam = [lam[0]] + [lam[j] ^ M(X, lam[j - 1]) for j in range(1, deg)]
        surv = [v for v in range(nvecs) if v not in locs]
        for r in range(es):
            beta = int(ex[(255 - (nvecs - 1 - locs[r])) % 255])
            denom = 0
            for j in range(1, deg, 2):
                denom ^= M(lam[j], P(beta, j - 1))
            dinv = int(inv[denom]) if denom else 1
            pre, acc = [], 0
            for u in range(m):
                acc ^= M(lam[u], P(beta, u))
                pre.append(acc)
            for v in surv:
                g = int(ex[(nvecs - 1 - v) % 255])
                w = M(g, beta)
                h = 0
                for u in range(m):
                    h ^= M(pre[u], P(w, m - 1 - u))
                lam_at = 0
                for j in range(deg):
                    lam_at ^= M(lam[j], P(int(inv[g]), j))
                closed = M(M(M(dinv, P(beta, m)), M(P(g, m + 1), lam_at)), int(inv[w ^ 1]))
                assert M(dinv, M(g, h)) == closed
                checked += 1
    assert checked > 1000
