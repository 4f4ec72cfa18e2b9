// gf_host.cpp -- host-side field tables, generator construction and kernel tables.
//
// Field construction follows generate_gf() (reference src/common/normEncoderRS8.cpp:182-242,
// normEncoderRS16.cpp:181-241): alpha = x over the primitive polynomials 0x11d / 0x1100B.
//
// The systematic generator is built in closed form.  The reference fills an n x k
// Vandermonde matrix whose row r evaluates the powers of the point p_r (p_0 = 0,
// p_r = alpha^(r-1)), inverts the top k x k block and multiplies the bottom rows by it
// (normEncoderRS8.cpp:428-450).  That product is the Lagrange basis of the top points
// evaluated at the bottom points:
//     G[k+p][j] = W(y_p) / ((y_p + x_j) * W'(x_j)),   W(z) = prod_l (z + x_l)
// which is unique, so it is byte-identical to the reference matrix while costing
// O(k^2 + m k) instead of O(m k^2) (the reference's RS16 Init takes 26 s at k = 4096).
// tests/ checks it against the oracle's Vandermonde construction.
#include <cstring>
#include <mutex>

#include "nfec_internal.hpp"

#include <functional>

namespace nfec {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }
int fail(int code, const std::string& msg)
{
    set_error(msg);
    return code;
}
int hip_fail(hipError_t e, const char* what)
{
    set_error(std::string(what) + ": " + hipGetErrorString(e));
    return NFEC_EDEVICE;
}
const char* last_error_cstr() { return g_last_error.c_str(); }

static void build_field(Field& f, int bits, uint32_t poly)
{
    f.bits = bits;
    f.q = (1u << bits) - 1u;
    f.exp.assign(2 * f.q, 0);
    f.log.assign(f.q + 1, 0);
    uint32_t v = 1;
    for (uint32_t i = 0; i < f.q; ++i) {
        f.exp[i] = v;
        f.log[v] = i;
        v <<= 1;
        if (v & (1u << bits)) v ^= poly;
    }
    f.log[0] = f.q;
    for (uint32_t i = 0; i < f.q; ++i) f.exp[i + f.q] = f.exp[i];
}

const Field& gf8()
{
    static Field f;
    static std::once_flag once;
    std::call_once(once, [] { build_field(f, 8, 0x11d); });
    return f;
}

const Field& gf16()
{
    static Field f;
    static std::once_flag once;
    std::call_once(once, [] { build_field(f, 16, 0x1100b); });
    return f;
}

int rs_generator(int bits, uint32_t k, uint32_t m, std::vector<uint32_t>& rows)
{
    const Field& f = bits == 8 ? gf8() : gf16();
    if (k == 0 || (uint64_t)k + m > f.q) return NFEC_ERANGE;
    // The reference computes the point exponents as int row*col (normEncoderRS8.cpp:433);
    // past 2^31 that is undefined behaviour, so such shapes are refused.
    if (k + m >= 2 && (uint64_t)(k + m - 2) * (k - 1) >= (1ull << 31)) return NFEC_ERANGE;
    const uint32_t q = f.q;
    std::vector<uint32_t> x(k);
    for (uint32_t j = 0; j < k; ++j) x[j] = rs_point(f, j);
    // log W'(x_j) = sum_{l != j} log(x_j + x_l)
    std::vector<uint64_t> lwp(k, 0);
    for (uint32_t j = 0; j < k; ++j) {
        uint64_t s = 0;
        for (uint32_t l = 0; l < k; ++l)
            if (l != j) s += f.log[x[j] ^ x[l]];
        lwp[j] = s % q;
    }
    rows.assign((size_t)m * k, 0);
    for (uint32_t p = 0; p < m; ++p) {
        const uint32_t y = rs_point(f, k + p);
        uint64_t lw = 0;
        for (uint32_t l = 0; l < k; ++l) lw += f.log[y ^ x[l]];
        lw %= q;
        for (uint32_t j = 0; j < k; ++j) {
            uint64_t e = lw + 2ull * q - f.log[y ^ x[j]] - lwp[j];
            rows[(size_t)p * k + j] = f.exp[e % q];
        }
    }
    return NFEC_OK;
}

void mdp_generator_poly(uint32_t m, std::vector<uint8_t>& g)
{
    // g(x) = prod_{n=1..m} (x + alpha^n), g[i] = coefficient of x^i
    const Field& f = gf8();
    g.assign(m + 1, 0);
    g[0] = 1;
    for (uint32_t n = 1; n <= m; ++n) {
        const uint32_t a = f.exp[n];
        for (uint32_t i = n; i > 0; --i) g[i] = (uint8_t)(g[i - 1] ^ f.mul(g[i], a));
        g[0] = (uint8_t)f.mul(g[0], a);
    }
}

void mdp_encode_matrix(const std::vector<uint8_t>& g, uint32_t m, uint32_t nd, uint8_t* out)
{
    // The MDP encoder (normEncoderMDP.cpp:178-211) is a linear shift register over the
    // parity vectors: fb = d ^ P[0];  P[i] = P[i+1] ^ g[m-1-i]*fb;  P[m-1] = g[0]*fb.
    // Column j of the block map is the register after an impulse at step j followed
    // by nd-1-j zero steps, so all columns come from one impulse response.
    const Field& f = gf8();
    std::vector<uint8_t> st(m, 0), nx(m);
    auto step = [&](uint32_t d) {
        uint32_t fb = d ^ st[0];
        for (uint32_t i = 0; i + 1 < m; ++i) nx[i] = (uint8_t)(st[i + 1] ^ f.mul(g[m - 1 - i], fb));
        nx[m - 1] = (uint8_t)f.mul(g[0], fb);
        st.swap(nx);
    };
    if (nd == 0) return;
    step(1);
    for (uint32_t j = nd; j-- > 0;) {
        for (uint32_t i = 0; i < m; ++i) out[(size_t)i * nd + j] = st[i];
        if (j) step(0);
    }
}

// coefficient table of the runtime-coefficient kernel (gen_rs8_rt.hip): entry (c, r) is the
// byte offset of coefficient rows[r][c]'s snippet (value << 7), columns rs8_rt_col_stride(m)
// bytes apart, 16 bytes of padding for the kernel's 8-row entry loads
std::vector<uint16_t> rs8_rt_table(const std::vector<uint32_t>& rows, uint32_t k, uint32_t m)
{
    const uint32_t cs = rs8_rt_col_stride(m) / 2;
    std::vector<uint16_t> t((size_t)k * cs + 4 * cs + 64, 0);  // padding: the kernel's touch loads
    for (uint32_t c = 0; c < k; ++c)
        for (uint32_t r = 0; r < m; ++r) t[(size_t)c * cs + r] = (uint16_t)((rows[(size_t)r * k + c] & 0xffu) << 7);
    return t;
}

void vperm_table(uint32_t c, uint32_t out[8])
{
    const Field& f = gf8();
    auto pack = [&](uint32_t a, uint32_t b, uint32_t cc, uint32_t d) {
        return f.mul(c, a) | (f.mul(c, b) << 8) | (f.mul(c, cc) << 16) | (f.mul(c, d) << 24);
    };
    out[0] = pack(0, 1, 2, 3);
    out[1] = pack(4, 5, 6, 7);
    out[2] = pack(0, 8, 16, 24);
    out[3] = pack(32, 40, 48, 56);
    out[4] = pack(0, 64, 128, 192);
    out[5] = out[6] = out[7] = 0;
}

}  // namespace nfec

namespace nfec {

// LDS byte offsets for the shared-table RS16 encode (gen_gf16_t3.hip): coefficient (c, r) is
// the 16 x 16 GF(2) matrix M of x -> G[r][c] * x (column q = G[r][c] * alpha^q); output plane
// p XORs input planes q with bit q of row p of M.  Input planes split into groups 0..5,
// 6..10 and 11..15 whose subset XORs sit in table rows [0, 64), [64, 96), [96, 128), 512 bytes
// apart: out[(c * m_pad + r) * 48 + p * 3 + g] = (table row) * 512.  Rows r >= m (padding up
// to gf16_t3_rows_padded) and the one extra column (the kernel prefetches one past the end)
// point at the zero rows.
void gf16_t3_offsets(const std::vector<uint32_t>& parity_rows, uint32_t k, uint32_t m, uint16_t* out)
{
    const Field& f = gf16();
    const uint32_t mp = gf16_t3_rows_padded(m);
    static const uint32_t first[3] = {0, 6, 11}, width[3] = {6, 5, 5}, row0[3] = {0, 64, 96};
    for (uint32_t c = 0; c <= k; ++c)
        for (uint32_t r = 0; r < mp; ++r) {
            const uint32_t g = (c < k && r < m) ? parity_rows[(size_t)r * k + c] : 0u;
            uint32_t col[16];
            for (int q = 0; q < 16; ++q) col[q] = f.mul(g, 1u << q);
            uint16_t* o = out + ((size_t)c * mp + r) * 48;
            for (int p = 0; p < 16; ++p) {
                uint32_t mask = 0;
                for (int q = 0; q < 16; ++q) mask |= ((col[q] >> p) & 1u) << q;
                for (int t = 0; t < 3; ++t) {
                    const uint32_t e = (mask >> first[t]) & ((1u << width[t]) - 1u);
                    o[p * 3 + t] = (uint16_t)((row0[t] + e) * 512u);
                }
            }
        }
}

}  // namespace nfec

namespace nfec {

// 16 row masks of x -> c * x over GF(2^16): M[p] bit q = bit p of c * 2^q (gf16_bs.hpp)
static void gf16_bitmatrix(const Field& f, uint32_t c, uint16_t* M)
{
    for (int p = 0; p < 16; ++p) M[p] = 0;
    for (int q = 0; q < 16; ++q) {
        const uint32_t v = f.mul(c, 1u << q);
        for (int p = 0; p < 16; ++p) M[p] |= (uint16_t)(((v >> p) & 1u) << q);
    }
}

// The Toeplitz split of the RS16 generator (kernels_tmvp.hip): G[p][j] = W(y_p) T[p][j] c_j for
// j >= 1 with T[p][j] = 1 / (1 + alpha^(k+p-j)).  Builds the three cw x (k/2) product matrices
// (row-major, virtual column q*cw + i for the column pair a = 2q*cw + i, b = a + cw):
//   prod[0] = A       = T[p][a]
//   prod[1] = (B-A) c = (T[p][b] + T[p][a]) c_b
//   prod[2] = (C-A) c = (T[p+cw][a] + T[p][a]) c_a      (c_0 = 0)
// and the row masks of c_j, W(y_p) and G[p][0].  Every G[p][j] is re-derived from the factors
// and compared with the generator; false (and nothing used) on any mismatch or shape the split
// does not cover (m even, k a multiple of m; the caller adds that the shared-table kernel's
// column map needs m/2 a power of two, the tower kernel's takes any width).
bool rs16_tmvp_plan(uint32_t k, uint32_t m, const std::vector<uint32_t>& gen, std::vector<uint32_t> prod[3],
                    std::vector<uint16_t>& cmat, std::vector<uint16_t>& wmat, std::vector<uint16_t>& gmat)
{
    return rs16_tmvp_plan_levels(k, m, gen, 1, prod, cmat, wmat, gmat);
}

// levels = L in 1..3: the general form (tests/test_tmvp.py::_split_levels restates it).  The root
// is the Toeplitz part T[p][q m + i] over the scaled source u_j = c_j d_j in chunks of m columns;
// a node of width r (its r x r blocks Toeplitz) splits into three of r/2 rows, per chunk
//   alpha = the top-left block      over (first half + second half of its input)
//   beta  = top-right - top-left    over the second half
//   gamma = bottom-left - top-left  over the first half,
// and the 3^L leaves (path digits d_1..d_L, 0 alpha / 1 beta / 2 gamma; product index
// sum d_l 3^(L-l)) have m >> L rows over k >> L virtual columns v = q (m >> L) + i.  A leaf
// whose path holds no alpha reads raw source columns j = q m + i + (sum of m >> l over its beta
// levels l), its c_j folded into the coefficients; the others read the alpha sums the prescale
// writes (kernels_tmvp.hip).  L = 1: prod[0] = A, prod[1] = (B - A) c_b, prod[2] = (C - A) c_a.
bool rs16_tmvp_plan_levels(uint32_t k, uint32_t m, const std::vector<uint32_t>& gen, int levels,
                           std::vector<uint32_t>* prod, std::vector<uint16_t>& cmat, std::vector<uint16_t>& wmat,
                           std::vector<uint16_t>& gmat)
{
    if (m < 2 || (m & 1u) || k % m || gen.size() != (size_t)m * k) return false;
    if (levels < 1 || levels > 3 || (m >> levels) == 0 || m % (1u << levels)) return false;
    const Field& f = gf16();
    const uint32_t q = f.q;
    std::vector<uint32_t> x(k);
    for (uint32_t j = 0; j < k; ++j) x[j] = rs_point(f, j);
    std::vector<uint32_t> c(k, 0), w(m), h(k + m, 0);
    for (uint32_t j = 1; j < k; ++j) {
        uint64_t lwp = 0;  // log W'(x_j)
        for (uint32_t l = 0; l < k; ++l)
            if (l != j) lwp += f.log[x[j] ^ x[l]];
        c[j] = f.exp[(2ull * q - (j - 1) % q - lwp % q) % q];
    }
    for (uint32_t p = 0; p < m; ++p) {
        const uint32_t y = rs_point(f, k + p);
        uint64_t lw = 0;
        for (uint32_t l = 0; l < k; ++l) lw += f.log[y ^ x[l]];
        w[p] = f.exp[lw % q];
    }
    for (uint32_t t = 1; t < k + m; ++t) {
        const uint32_t d = 1u ^ f.exp[t % q];
        if (d == 0) return false;
        h[t] = f.exp[(q - f.log[d]) % q];
    }
    for (uint32_t p = 0; p < m; ++p)
        for (uint32_t j = 1; j < k; ++j)
            if (gen[(size_t)p * k + j] != f.mul(w[p], f.mul(h[k + p - j], c[j]))) return false;
    const int L = levels;
    const uint32_t r = m >> L, cols = k >> L, nq = k / m;
    // block entry (p, i) of the node with digits dg[0..l) in chunk qq
    std::function<uint32_t(const int*, int, uint32_t, uint32_t, uint32_t)> M =
        [&](const int* dg, int l, uint32_t qq, uint32_t p, uint32_t i) -> uint32_t {
        if (l == 0) return h[k + p - qq * m - i];
        const uint32_t hf = m >> l;
        if (dg[l - 1] == 0) return M(dg, l - 1, qq, p, i);
        if (dg[l - 1] == 1) return M(dg, l - 1, qq, p, i + hf) ^ M(dg, l - 1, qq, p, i);
        return M(dg, l - 1, qq, p + hf, i) ^ M(dg, l - 1, qq, p, i);
    };
    uint32_t np = 1;
    for (int l = 0; l < L; ++l) np *= 3;
    for (uint32_t e = 0; e < np; ++e) {
        int dg[3] = {0, 0, 0};
        bool raw = true;
        uint32_t off = 0;
        for (int l = L, t = (int)e; l >= 1; --l, t /= 3) dg[l - 1] = t % 3;
        for (int l = 1; l <= L; ++l) {
            raw = raw && dg[l - 1] != 0;
            if (dg[l - 1] == 1) off += m >> l;
        }
        prod[e].assign((size_t)r * cols, 0);
        for (uint32_t qq = 0; qq < nq; ++qq)
            for (uint32_t i = 0; i < r; ++i) {
                const uint32_t v = qq * r + i, j = qq * m + i + off;
                for (uint32_t p = 0; p < r; ++p) {
                    uint32_t val = M(dg, L, qq, p, i);
                    if (raw) val = f.mul(val, c[j]);
                    prod[e][(size_t)p * cols + v] = val;
                }
            }
    }
    cmat.assign((size_t)k * 16, 0);
    wmat.assign((size_t)m * 16, 0);
    gmat.assign((size_t)m * 16, 0);
    for (uint32_t j = 0; j < k; ++j) gf16_bitmatrix(f, c[j], &cmat[(size_t)j * 16]);
    for (uint32_t p = 0; p < m; ++p) {
        gf16_bitmatrix(f, w[p], &wmat[(size_t)p * 16]);
        gf16_bitmatrix(f, gen[(size_t)p * k], &gmat[(size_t)p * 16]);
    }
    return true;
}

}  // namespace nfec
