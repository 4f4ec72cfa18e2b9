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


def mdp_syndrome_map(ex, lg, inv, mul, nvecs, locs):
    """The erasure-only MDP repair from ec = len(locs) syndromes (a candidate fused form, like
    the RS8 fused repair's 16 constant rows):
    S_j = sum_v r_v X_v^j (j = 1..ec, X_v = alpha^(nvecs-1-v), erased r_v = 0), and erased
    position i gets e_i = sum_j F[i][j] S_j with
        F[i][j] = coef_{j-1}(prod_{k != i} (x + X_k)) / (X_i prod_{k != i} (X_i + X_k))
    (the Vandermonde inverse of S_j = sum_i (e_i X_i) X_i^(j-1)).  Returns F [ec][ec]."""
    def M(a, b):
        return int(mul[a][b])

    X = [int(ex[nvecs - 1 - loc]) for loc in locs]
    ec = len(X)
    full = [1]                               # prod_k (x + X_k), low coefficient first
    for x in X:
        nxt = [0] * (len(full) + 1)
        for d, c in enumerate(full):
            nxt[d] ^= M(c, x)
            nxt[d + 1] ^= c
        full = nxt
    F = [[0] * ec for _ in range(ec)]
    for i in range(ec):
        # synthetic division of full by (x + X_i): q has degree ec - 1
        q = [0] * ec
        carry = 0
        for d in range(ec, 0, -1):
            carry = full[d] ^ M(carry, X[i]) if d < ec else full[d]
            q[d - 1] = carry
        den = X[i]
        for k2 in range(ec):
            if k2 != i:
                den = M(den, X[i] ^ X[k2])
        dinv = int(inv[den])
        for j in range(ec):
            F[i][j] = M(q[j], dinv)
    return F


def test_mdp_syndrome_form_repairs(orc):
    ex, lg, inv = orc.gf8_tables()
    mul = orc.gf8_mul_table()
    rng = np.random.default_rng(5)
    for it in range(60):
        k = int(rng.integers(2, 100))
        m = int(rng.integers(1, min(40, 255 - k) + 1))
        vec = 16
        blk = orc.make_blocks(k, m, vec, 1, seed=int(rng.integers(1, 1 << 30)))
        clean = orc.encode_blocks(orc_kind_mdp(), k, m, vec, blk)[0]
        nvecs = k + m
        ec = int(rng.integers(1, m + 1))
        locs = sorted(rng.choice(nvecs, ec, replace=False).tolist())
        rx = clean.copy()
        rx[locs] = 0
        F = mdp_syndrome_map(ex, lg, inv, mul, nvecs, locs)
        S = []
        for j in range(1, ec + 1):
            s = np.zeros(vec, np.uint8)
            for v in range(nvecs):
                c = int(ex[(j * (nvecs - 1 - v)) % 255])
                s ^= mul[c][rx[v]]
            S.append(s)
        for i, loc in enumerate(locs):
            d = np.zeros(vec, np.uint8)
            for j in range(ec):
                d ^= mul[F[i][j]][S[j]]
            assert np.array_equal(d, clean[loc]), (it, k, m, locs, loc)


def test_mdp_syndrome_form_off_codewords(orc):
    """Why the build does not use that form: the reference's Forney step reads all m syndromes
    (Omega_t = sum_{j<=t} S_j Lambda_{t-j}, t < m, normEncoderMDP.cpp:378-419), so when the
    survivors are not a codeword its output depends on S_(ec+1)..S_m as well; the ec-syndrome
    form then differs from the reference, while the closed-form map over every survivor
    (mdp_plan_kernel) stays equal to it (tests/test_gpu_parity.py, non-codeword survivors)."""
    ex, lg, inv = orc.gf8_tables()
    mul = orc.gf8_mul_table()
    rng = np.random.default_rng(8)
    k, m, vec = 64, 32, 16
    differ = 0
    for it in range(10):
        blk = orc.make_blocks(k, m, vec, 1, seed=int(rng.integers(1, 1 << 30)))
        clean = orc.encode_blocks(orc_kind_mdp(), k, m, vec, blk)[0]
        nvecs = k + m
        locs = sorted(rng.choice(k, 16, replace=False).tolist())
        rx = clean.copy()
        rx[locs] = 0
        surv = [v for v in range(nvecs) if v not in locs]
        rx[surv[int(rng.integers(0, len(surv)))]] ^= rng.integers(1, 256, vec, dtype=np.uint8)  # off the code
        ref = rx[None].copy()
        nloc = np.zeros((1, m), np.uint16)
        nloc[0, :16] = locs
        orc.decode_blocks(orc_kind_mdp(), k, m, vec, ref, nloc, np.array([16], np.uint16))
        F = mdp_syndrome_map(ex, lg, inv, mul, nvecs, locs)
        S = []
        for j in range(1, 17):
            sj = np.zeros(vec, np.uint8)
            for v in range(nvecs):
                sj ^= mul[int(ex[(j * (nvecs - 1 - v)) % 255])][rx[v]]
            S.append(sj)
        for i, loc in enumerate(locs):
            d = np.zeros(vec, np.uint8)
            for j in range(16):
                d ^= mul[F[i][j]][S[j]]
            differ += not np.array_equal(d, ref[0, loc])
    assert differ > 0


def orc_kind_mdp():
    from norm_amd import _native as N

    return N.NFEC_MDP
