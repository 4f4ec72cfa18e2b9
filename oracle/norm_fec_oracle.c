/*
 * norm_fec_oracle.c -- CPU restatement of NORM's FEC codecs.
 *
 * TEST INFRASTRUCTURE ONLY: this file is the parity checker and the CPU baseline
 * ("port") for bench.py.  The product path (norm_amd/, HIP kernels behind the C-ABI
 * in include/nfec.h) never links, loads or calls it.  See norm_fec_oracle.h for the
 * pinning status of each routine.
 *
 * Written from a reading of the reference's behaviour; every routine cites the
 * reference function it restates.  Field element types follow the reference: 8-bit
 * elements for RS8/MDP, 16-bit elements for RS16 (native-endian symbols).
 */
#define _GNU_SOURCE
#include "norm_fec_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

enum { ORC_RS8 = 1, ORC_RS16 = 2, ORC_MDP = 3 };

/* ======================================================================
 * GF(2^8), polynomial "101110001" (1+x^2+x^3+x^4+x^8 = 0x11d)
 * restates generate_gf() normEncoderRS8.cpp:182-242 and init_mul_table() :140-149
 * ====================================================================== */
#define Q8 255u
static uint8_t f8_exp[2 * Q8];
static int32_t f8_log[Q8 + 1];
static uint8_t f8_inv[Q8 + 1];
static uint8_t f8_mul[Q8 + 1][Q8 + 1];

/* GF(2^16), polynomial "11010000000010001" (1+x+x^3+x^12+x^16 = 0x1100B)
 * restates generate_gf() normEncoderRS16.cpp:181-241 */
#define Q16 65535u
static uint16_t f16_exp[2 * Q16];
static int32_t f16_log[Q16 + 1];
static uint16_t f16_inv[Q16 + 1];

/* galois.cpp tables, restated (galois.cpp:37 GINV, :58 GEXP, :95 GMULT) */
static uint8_t gal_inv[256];
static uint8_t gal_exp[512];
static uint8_t gal_mul[256][256];

static pthread_once_t tables_once = PTHREAD_ONCE_INIT;

/* x mod (2^bits - 1) without a divide: modnn() normEncoderRS8.cpp:109-117 */
static int reduce_mod(int x, int bits, int q)
{
    while (x >= q) {
        x -= q;
        x = (x >> bits) + (x & q);
    }
    return x;
}

/* Build exp/log/inverse for a binary field from its primitive polynomial given as the
 * reference's coefficient string (lowest power first). */
static void build_field(const char* poly, int bits, void* exp_tab, int32_t* log_tab,
                        void* inv_tab, int wide)
{
    const uint32_t q = (1u << bits) - 1u;
    uint32_t* e = (uint32_t*)malloc(sizeof(uint32_t) * 2 * q);
    uint32_t top = 0; /* alpha^bits in polynomial form */
    for (int i = 0; i < bits; ++i) {
        e[i] = 1u << i;
        log_tab[e[i]] = i;
        if (poly[i] == '1') top ^= 1u << i;
    }
    e[bits] = top;
    log_tab[top] = bits;
    const uint32_t hib = 1u << (bits - 1);
    for (uint32_t i = (uint32_t)bits + 1; i < q; ++i) {
        uint32_t prev = e[i - 1];
        e[i] = (prev >= hib) ? (top ^ ((prev ^ hib) << 1)) : (prev << 1);
        log_tab[e[i]] = (int32_t)i;
    }
    log_tab[0] = (int32_t)q; /* log(0) sentinel, :228 */
    for (uint32_t i = 0; i < q; ++i) e[i + q] = e[i];
    for (uint32_t i = 0; i < 2 * q; ++i) {
        if (wide) ((uint16_t*)exp_tab)[i] = (uint16_t)e[i];
        else ((uint8_t*)exp_tab)[i] = (uint8_t)e[i];
    }
    /* inverse[0] = 0, inverse[1] = 1, inverse[i] = alpha^(q - log i)  (:238-241) */
    for (uint32_t i = 0; i <= q; ++i) {
        uint32_t v = (i == 0) ? 0u : (i == 1) ? 1u : e[q - (uint32_t)log_tab[i]];
        if (wide) ((uint16_t*)inv_tab)[i] = (uint16_t)v;
        else ((uint8_t*)inv_tab)[i] = (uint8_t)v;
    }
    free(e);
}

static void init_tables(void)
{
    build_field("101110001", 8, f8_exp, f8_log, f8_inv, 0);
    for (int a = 0; a <= (int)Q8; ++a)
        for (int b = 0; b <= (int)Q8; ++b)
            f8_mul[a][b] = (a && b) ? f8_exp[reduce_mod(f8_log[a] + f8_log[b], 8, Q8)] : 0;
    build_field("11010000000010001", 16, f16_exp, f16_log, f16_inv, 1);

    /* galois.cpp: GEXP is alpha^i over the same 0x11d field for i < 510 with a trailing
     * 0x00; GINV[0] is 0x01 (galois.cpp:39); GMULT is the plain product table. */
    for (int i = 0; i < 510; ++i) gal_exp[i] = f8_exp[i];
    gal_exp[510] = 0x01;
    gal_exp[511] = 0x00;
    for (int i = 0; i < 256; ++i) gal_inv[i] = (i == 0) ? 0x01 : f8_inv[i];
    memcpy(gal_mul, f8_mul, sizeof(gal_mul));
}

static void ensure_tables(void) { pthread_once(&tables_once, init_tables); }

void orc_gf8_tables(uint8_t exp_out[510], int32_t log_out[256], uint8_t inv_out[256])
{
    ensure_tables();
    memcpy(exp_out, f8_exp, sizeof(f8_exp));
    memcpy(log_out, f8_log, sizeof(f8_log));
    memcpy(inv_out, f8_inv, sizeof(f8_inv));
}

void orc_gf8_mul_table(uint8_t out[65536])
{
    ensure_tables();
    memcpy(out, f8_mul, sizeof(f8_mul));
}

void orc_gf16_tables(uint16_t* exp_out, int32_t* log_out, uint16_t* inv_out)
{
    ensure_tables();
    memcpy(exp_out, f16_exp, sizeof(f16_exp));
    memcpy(log_out, f16_log, sizeof(f16_log));
    memcpy(inv_out, f16_inv, sizeof(f16_inv));
}

void orc_galois_tables(uint8_t ginv[256], uint8_t gexp[512], uint8_t gmult[65536])
{
    ensure_tables();
    memcpy(ginv, gal_inv, 256);
    memcpy(gexp, gal_exp, 512);
    memcpy(gmult, gal_mul, 65536);
}

/* ---- element multiply in each field (gf_mul macros, RS8 :133-138, RS16 :152-156) ---- */
static inline uint32_t mul8(uint32_t a, uint32_t b) { return f8_mul[a][b]; }
static inline uint32_t mul16(uint32_t a, uint32_t b)
{
    if (a == 0 || b == 0) return 0;
    return f16_exp[f16_log[a] + f16_log[b]];
}

/* addmul1(): dst[] ^= c * src[] (RS8 :262-299).  The reference unrolls by 16; the
 * result is the same byte for byte, so the oracle keeps the unroll for timing parity. */
static void addmul8(uint8_t* dst, const uint8_t* src, uint32_t c, unsigned n)
{
    if (c == 0) return; /* addmul macro :258-259 */
    const uint8_t* row = f8_mul[c];
    unsigned i = 0;
    for (; i + 16 <= n; i += 16) {
        dst[i + 0] ^= row[src[i + 0]];   dst[i + 1] ^= row[src[i + 1]];
        dst[i + 2] ^= row[src[i + 2]];   dst[i + 3] ^= row[src[i + 3]];
        dst[i + 4] ^= row[src[i + 4]];   dst[i + 5] ^= row[src[i + 5]];
        dst[i + 6] ^= row[src[i + 6]];   dst[i + 7] ^= row[src[i + 7]];
        dst[i + 8] ^= row[src[i + 8]];   dst[i + 9] ^= row[src[i + 9]];
        dst[i + 10] ^= row[src[i + 10]]; dst[i + 11] ^= row[src[i + 11]];
        dst[i + 12] ^= row[src[i + 12]]; dst[i + 13] ^= row[src[i + 13]];
        dst[i + 14] ^= row[src[i + 14]]; dst[i + 15] ^= row[src[i + 15]];
    }
    for (; i < n; ++i) dst[i] ^= row[src[i]];
}

/* RS16 addmul1 with GF_ADDMULC {if (x) dst ^= mulc[log x]} (RS16 :158-161, :261-298);
 * operates on native-endian 16-bit symbols. */
static void addmul16(uint16_t* dst, const uint16_t* src, uint32_t c, unsigned n)
{
    if (c == 0) return;
    const uint16_t* mulc = &f16_exp[f16_log[c]];
    for (unsigned i = 0; i < n; ++i) {
        uint32_t x = src[i];
        if (x) dst[i] ^= mulc[f16_log[x]];
    }
}

/* ======================================================================
 * Systematic generator: Vandermonde fill, invert top k x k, multiply bottom rows.
 * restates NormEncoderRS8::Init normEncoderRS8.cpp:400-462 with invert_vdm :322-376
 * and matmul :303-319.  Shared by RS8 and RS16 through the element width W.
 * ====================================================================== */
typedef uint32_t elem_t;

static elem_t fmul(int bits, elem_t a, elem_t b) { return bits == 8 ? mul8(a, b) : mul16(a, b); }
static elem_t finv(int bits, elem_t a) { return bits == 8 ? f8_inv[a] : f16_inv[a]; }
static elem_t fexp(int bits, int i) { return bits == 8 ? f8_exp[i] : f16_exp[i]; }

/* in-place inverse of a k x k Vandermonde matrix whose column 1 holds the points */
static void vandermonde_invert(elem_t* v, int k, int bits)
{
    if (k == 1) return; /* the 1x1 matrix is [1] */
    elem_t* c = (elem_t*)calloc((size_t)k, sizeof(elem_t));
    elem_t* b = (elem_t*)calloc((size_t)k, sizeof(elem_t));
    elem_t* pt = (elem_t*)calloc((size_t)k, sizeof(elem_t));
    for (int i = 0; i < k; ++i) pt[i] = v[i * k + 1];
    /* coefficients of P(x) = prod (x - p_i), leading 1 implicit */
    c[k - 1] = pt[0];
    for (int i = 1; i < k; ++i) {
        elem_t pi = pt[i];
        for (int j = k - 1 - (i - 1); j < k - 1; ++j) c[j] ^= fmul(bits, pi, c[j + 1]);
        c[k - 1] ^= pi;
    }
    for (int row = 0; row < k; ++row) {
        elem_t xx = pt[row], t = 1;
        b[k - 1] = 1;
        for (int i = k - 2; i >= 0; --i) {
            b[i] = c[i + 1] ^ fmul(bits, xx, b[i + 1]);
            t = fmul(bits, xx, t) ^ b[i];
        }
        elem_t it = finv(bits, t);
        for (int col = 0; col < k; ++col) v[col * k + row] = fmul(bits, it, b[col]);
    }
    free(c);
    free(b);
    free(pt);
}

static int build_generator(unsigned k, unsigned m, int bits, elem_t* enc)
{
    const unsigned q = (1u << bits) - 1u;
    if (k == 0 || k + m > q) return -1; /* :405-409 */
    const unsigned n = k + m;
    elem_t* t = (elem_t*)calloc((size_t)n * k, sizeof(elem_t));
    if (!t) return -1;
    t[0] = 1; /* row 0 = powers of the point 0 */
    for (unsigned r = 0; r + 1 < n; ++r)
        for (unsigned col = 0; col < k; ++col)
            t[(size_t)(r + 1) * k + col] = fexp(bits, reduce_mod((int)(r * col), bits, (int)q));
    vandermonde_invert(t, (int)k, bits);
    /* bottom (n-k) rows times the inverted top block */
    for (unsigned row = 0; row < n - k; ++row)
        for (unsigned col = 0; col < k; ++col) {
            elem_t acc = 0;
            for (unsigned i = 0; i < k; ++i)
                acc ^= fmul(bits, t[(size_t)(k + row) * k + i], t[(size_t)i * k + col]);
            enc[(size_t)(k + row) * k + col] = acc;
        }
    for (unsigned r = 0; r < k; ++r)
        for (unsigned col = 0; col < k; ++col) enc[(size_t)r * k + col] = (r == col);
    free(t);
    return 0;
}

int orc_rs8_generator(unsigned k, unsigned m, uint8_t* enc_out)
{
    ensure_tables();
    size_t cnt = (size_t)(k + m) * k;
    elem_t* tmp = (elem_t*)malloc(cnt * sizeof(elem_t));
    int rc = build_generator(k, m, 8, tmp);
    if (rc == 0)
        for (size_t i = 0; i < cnt; ++i) enc_out[i] = (uint8_t)tmp[i];
    free(tmp);
    return rc;
}

int orc_rs16_generator(unsigned k, unsigned m, uint16_t* enc_out)
{
    ensure_tables();
    size_t cnt = (size_t)(k + m) * k;
    elem_t* tmp = (elem_t*)malloc(cnt * sizeof(elem_t));
    int rc = build_generator(k, m, 16, tmp);
    if (rc == 0)
        for (size_t i = 0; i < cnt; ++i) enc_out[i] = (uint16_t)tmp[i];
    free(tmp);
    return rc;
}

/* ---- incremental encode: NormEncoderRS8::Encode :473-483 (RS16 :472-482) ---- */
void orc_rs8_encode(const uint8_t* enc, unsigned k, unsigned m, unsigned vec,
                    unsigned segment_id, const uint8_t* data, uint8_t** parity)
{
    ensure_tables();
    for (unsigned i = 0; i < m; ++i)
        addmul8(parity[i], data, enc[(size_t)(i + k) * k + segment_id], vec);
}

void orc_rs16_encode(const uint16_t* enc, unsigned k, unsigned m, unsigned vec,
                     unsigned segment_id, const uint8_t* data, uint8_t** parity)
{
    ensure_tables();
    for (unsigned i = 0; i < m; ++i)
        addmul16((uint16_t*)parity[i], (const uint16_t*)data,
                 enc[(size_t)(i + k) * k + segment_id], vec / 2);
}

/* ======================================================================
 * Decode: dec_matrix build, Gauss-Jordan inversion, repair.
 * restates NormDecoderRS8::Decode :652-757 and InvertDecodingMatrix :766-889.
 * ====================================================================== */
static int gauss_jordan(elem_t* src, unsigned k, int bits)
{
    unsigned* ndxc = (unsigned*)calloc(k, sizeof(unsigned));
    unsigned* ndxr = (unsigned*)calloc(k, sizeof(unsigned));
    unsigned* pivt = (unsigned*)calloc(k, sizeof(unsigned));
    elem_t* idrow = (elem_t*)calloc(k, sizeof(elem_t));
    int ok = 1;
    for (unsigned col = 0; col < k && ok; ++col) {
        int irow = -1, icol = -1;
        if (pivt[col] != 1 && src[(size_t)col * k + col] != 0) {
            irow = (int)col;
            icol = (int)col;
        } else {
            for (unsigned row = 0; row < k && icol < 0 && ok; ++row) {
                if (pivt[row] == 1) continue;
                for (unsigned ix = 0; ix < k; ++ix) {
                    if (pivt[ix] == 0) {
                        if (src[(size_t)row * k + ix] != 0) {
                            irow = (int)row;
                            icol = (int)ix;
                            break;
                        }
                    } else if (pivt[ix] > 1) {
                        ok = 0; /* singular */
                        break;
                    }
                }
            }
            if (ok && icol < 0) ok = 0; /* pivot not found */
        }
        if (!ok) break;
        pivt[icol]++;
        if (irow != icol)
            for (unsigned ix = 0; ix < k; ++ix) {
                elem_t tmp = src[(size_t)irow * k + ix];
                src[(size_t)irow * k + ix] = src[(size_t)icol * k + ix];
                src[(size_t)icol * k + ix] = tmp;
            }
        ndxr[col] = (unsigned)irow;
        ndxc[col] = (unsigned)icol;
        elem_t* prow = &src[(size_t)icol * k];
        elem_t c = prow[icol];
        if (c == 0) { ok = 0; break; }
        if (c != 1) {
            c = finv(bits, c);
            prow[icol] = 1;
            for (unsigned ix = 0; ix < k; ++ix) prow[ix] = fmul(bits, c, prow[ix]);
        }
        idrow[icol] = 1;
        if (memcmp(prow, idrow, k * sizeof(elem_t)) != 0) {
            for (unsigned ix = 0; ix < k; ++ix) {
                if (ix == (unsigned)icol) continue;
                elem_t* p = &src[(size_t)ix * k];
                elem_t f = p[icol];
                p[icol] = 0;
                if (f)
                    for (unsigned j = 0; j < k; ++j) p[j] ^= fmul(bits, f, prow[j]);
            }
        }
        idrow[icol] = 0;
    }
    if (ok) {
        for (int col = (int)k - 1; col >= 0; --col) {
            if (ndxr[col] >= k || ndxc[col] >= k || ndxr[col] == ndxc[col]) continue;
            for (unsigned row = 0; row < k; ++row) {
                elem_t tmp = src[(size_t)row * k + ndxr[col]];
                src[(size_t)row * k + ndxr[col]] = src[(size_t)row * k + ndxc[col]];
                src[(size_t)row * k + ndxc[col]] = tmp;
            }
        }
    }
    free(ndxc);
    free(ndxr);
    free(pivt);
    free(idrow);
    return ok;
}

static int rs_decode(const void* encv, int bits, unsigned ndata, unsigned npar, unsigned vec,
                     uint8_t** vectors, unsigned num_data, unsigned erasure_count,
                     const unsigned* locs)
{
    ensure_tables();
    const unsigned bsz = ndata + npar;
    elem_t* dec = (elem_t*)calloc((size_t)ndata * ndata, sizeof(elem_t));
    unsigned* parity_loc = (unsigned*)calloc(npar ? npar : 1, sizeof(unsigned));
    const uint8_t* enc8 = (const uint8_t*)encv;
    const uint16_t* enc16 = (const uint16_t*)encv;
#define ENC(r, c) (bits == 8 ? (elem_t)enc8[(size_t)(r) * ndata + (c)] : (elem_t)enc16[(size_t)(r) * ndata + (c)])
    unsigned next = 0, ne = 0, src_erasures = 0, pcount = 0;
    /* (1) decoding matrix, :656-718 */
    for (unsigned i = 0; i < bsz; ++i) {
        int erased = (next < erasure_count) && (i == locs[next]);
        if (i < num_data) {
            if (erased) {
                next++;
                src_erasures++;
            } else {
                dec[(size_t)ndata * i + i] = 1;
            }
        } else if (i < ndata) {
            dec[(size_t)ndata * i + i] = 1; /* virtual zero symbol of a shortened block */
            if (erased) {
                next++;
            } else if (pcount < src_erasures) {
                parity_loc[pcount++] = i;
                elem_t* row = &dec[(size_t)ndata * locs[ne++]];
                for (unsigned c = 0; c < ndata; ++c) row[c] = ENC(ndata - num_data + i, c);
            }
        } else if (pcount < src_erasures) {
            if (erased) {
                next++;
            } else {
                parity_loc[pcount++] = i;
                elem_t* row = &dec[(size_t)ndata * locs[ne++]];
                for (unsigned c = 0; c < ndata; ++c) row[c] = ENC(ndata - num_data + i, c);
            }
        } else {
            break;
        }
    }
#undef ENC
    /* (2) invert, :720-725 */
    if (!gauss_jordan(dec, ndata, bits)) {
        free(dec);
        free(parity_loc);
        return 0;
    }
    /* (3) repair erased source rows only, :727-756 */
    const unsigned nel = (bits == 8) ? vec : vec / 2;
    for (unsigned e = 0; e < erasure_count; ++e) {
        unsigned row = locs[e];
        if (row >= num_data) break;
        unsigned nxt = 0;
        for (unsigned i = 0; i < num_data; ++i) {
            const uint8_t* src;
            if (nxt < erasure_count && i == locs[nxt]) {
                src = vectors[parity_loc[nxt]];
                nxt++;
            } else {
                src = vectors[i];
            }
            elem_t c = dec[(size_t)row * ndata + i];
            if (bits == 8) addmul8(vectors[row], src, c, nel);
            else addmul16((uint16_t*)vectors[row], (const uint16_t*)src, c, nel);
        }
    }
    free(dec);
    free(parity_loc);
    return (int)erasure_count;
}

int orc_rs8_decode(const uint8_t* enc, unsigned k, unsigned m, unsigned vec, uint8_t** vectors,
                   unsigned num_data, unsigned erasure_count, const unsigned* erasure_locs)
{
    return rs_decode(enc, 8, k, m, vec, vectors, num_data, erasure_count, erasure_locs);
}

int orc_rs16_decode(const uint16_t* enc, unsigned k, unsigned m, unsigned vec, uint8_t** vectors,
                    unsigned num_data, unsigned erasure_count, const unsigned* erasure_locs)
{
    return rs_decode(enc, 16, k, m, vec, vectors, num_data, erasure_count, erasure_locs);
}

/* ======================================================================
 * MDP (fec_id 129): normEncoderMDP.cpp, using the galois.cpp tables.
 * ====================================================================== */
static inline uint8_t gmul(uint32_t a, uint32_t b) { return gal_mul[a][b]; }

/* CreateGeneratorPolynomial :102-170 -- g(x) = prod_{n=1..m} (x + alpha^n), coefficient of
 * x^i in gen_poly[i].  The reference's scratch-array convolution is replaced by the
 * equivalent in-place multiply by (x + alpha^n). */
int orc_mdp_generator_poly(unsigned m, uint8_t* g)
{
    ensure_tables();
    if (m == 0 || m > 254) return -1;
    memset(g, 0, m + 1);
    g[0] = 1;
    for (unsigned n = 1; n <= m; ++n) {
        uint8_t a = gal_exp[n];
        for (unsigned i = n; i > 0; --i) g[i] = g[i - 1] ^ gmul(g[i], a);
        g[0] = gmul(g[0], a);
    }
    return 0;
}

/* Encode :178-211 -- one LFSR step per source vector, in order; parity zeroed by the
 * caller at block start. */
void orc_mdp_encode(const uint8_t* g, unsigned m, unsigned vec, const uint8_t* data,
                    uint8_t** parity, uint8_t* scratch)
{
    ensure_tables();
    memcpy(scratch, parity[0], vec);
    const uint8_t* gp = &g[m - 1];
    for (unsigned i = 0; i + 1 < m; ++i) {
        uint8_t* d = parity[i];
        const uint8_t* s = parity[i + 1];
        for (unsigned j = 0; j < vec; ++j) d[j] = s[j] ^ gmul(*gp, data[j] ^ scratch[j]);
        gp--;
    }
    uint8_t* last = parity[m - 1];
    for (unsigned j = 0; j < vec; ++j) last[j] = gmul(*gp, data[j] ^ scratch[j]);
}

/* Decode :333-430 -- syndromes, erasure locator, Omega, Forney fill of source erasures. */
int orc_mdp_decode(unsigned m, unsigned vec, uint8_t** dvec, unsigned num_data,
                   unsigned erasure_count, const unsigned* locs)
{
    ensure_tables();
    const unsigned nvecs = m + num_data;
    const unsigned degree = 2 * m;
    uint8_t* zero = (uint8_t*)calloc(vec ? vec : 1, 1);
    uint8_t* syn = (uint8_t*)calloc((size_t)m * vec + 1, 1);
    uint8_t* omega = (uint8_t*)calloc((size_t)m * vec + 1, 1);
    uint8_t* lambda = (uint8_t*)calloc(degree + 1, 1);
    /* (A) syndromes S_i = Horner over all vectors with X = alpha^(i+1); NULL reads zero */
    for (unsigned i = 0; i < m; ++i) {
        uint32_t x = gal_exp[i + 1];
        uint8_t* s = &syn[(size_t)i * vec];
        for (unsigned j = 0; j < nvecs; ++j) {
            const uint8_t* d = dvec[j] ? dvec[j] : zero;
            for (unsigned n = 0; n < vec; ++n) s[n] = d[n] ^ gmul(x, s[n]);
        }
    }
    /* (B) lambda(x) = prod over erasures of (1 + X x), X = alpha^(nvecs-1-loc) */
    lambda[0] = 1;
    for (unsigned i = 0; i < erasure_count; ++i) {
        uint32_t x = gal_exp[nvecs - 1 - locs[i]];
        for (int j = (int)degree - 1; j > 0; --j) lambda[j] ^= gmul(x, lambda[j - 1]);
    }
    /* (C) Omega_i = sum_{j<=i} lambda[i-j] * S_j */
    for (unsigned i = 0; i < m; ++i) {
        uint8_t* o = &omega[(size_t)i * vec];
        int kk = (int)i;
        for (unsigned j = 0; j <= i; ++j) {
            uint32_t lk = lambda[kk--];
            const uint8_t* s = &syn[(size_t)j * vec];
            for (unsigned n = 0; n < vec; ++n) o[n] ^= gmul(s[n], lk);
        }
    }
    /* (D) fill source erasures only */
    for (unsigned i = 0; i < erasure_count; ++i) {
        if (locs[i] >= num_data) break;
        unsigned kk = nvecs - 1 - locs[i];
        uint32_t denom = 0;
        for (unsigned j = 1; j < degree; j += 2)
            denom ^= gmul(lambda[j], gal_exp[((255 - kk) * (j - 1)) % 255]);
        denom = gal_inv[denom];
        uint8_t* e = dvec[locs[i]];
        for (unsigned j = 0; j < m; ++j) {
            uint32_t x = gal_exp[((255 - kk) * j) % 255];
            const uint8_t* o = &omega[(size_t)j * vec];
            for (unsigned n = 0; n < vec; ++n) e[n] ^= gmul(o[n], x);
        }
        for (unsigned n = 0; n < vec; ++n) e[n] = gmul(e[n], denom);
    }
    free(zero);
    free(syn);
    free(omega);
    free(lambda);
    return (int)erasure_count;
}

/* ======================================================================
 * Contiguous-block helpers (tests)
 * ====================================================================== */
int orc_encode_blocks(int kind, unsigned k, unsigned m, unsigned vec, uint8_t* blocks,
                      uint64_t block_stride, unsigned seg_stride, const uint16_t* num_data,
                      unsigned nblocks)
{
    ensure_tables();
    void* enc = NULL;
    uint8_t* gp = NULL;
    uint8_t* scratch = NULL;
    if (kind == ORC_RS8) {
        enc = malloc((size_t)(k + m) * k);
        if (orc_rs8_generator(k, m, (uint8_t*)enc)) { free(enc); return -1; }
    } else if (kind == ORC_RS16) {
        enc = malloc((size_t)(k + m) * k * 2);
        if (orc_rs16_generator(k, m, (uint16_t*)enc)) { free(enc); return -1; }
    } else if (kind == ORC_MDP) {
        if (k + m > 255) return -1;
        gp = (uint8_t*)malloc(m + 1);
        orc_mdp_generator_poly(m, gp);
        scratch = (uint8_t*)malloc(vec ? vec : 1);
    } else {
        return -1;
    }
    uint8_t** par = (uint8_t**)malloc(sizeof(uint8_t*) * (m ? m : 1));
    for (unsigned b = 0; b < nblocks; ++b) {
        uint8_t* blk = blocks + (size_t)b * block_stride;
        unsigned nd = num_data ? num_data[b] : k;
        for (unsigned p = 0; p < m; ++p) {
            par[p] = blk + (size_t)(nd + p) * seg_stride;
            memset(par[p], 0, vec); /* caller-zeroed parity, normObject.cpp:2240-2252 */
        }
        for (unsigned j = 0; j < nd; ++j) {
            const uint8_t* d = blk + (size_t)j * seg_stride;
            if (kind == ORC_RS8) orc_rs8_encode((uint8_t*)enc, k, m, vec, j, d, par);
            else if (kind == ORC_RS16) orc_rs16_encode((uint16_t*)enc, k, m, vec, j, d, par);
            else orc_mdp_encode(gp, m, vec, d, par, scratch);
        }
    }
    free(par);
    free(enc);
    free(gp);
    free(scratch);
    return 0;
}

int orc_decode_blocks(int kind, unsigned k, unsigned m, unsigned vec, uint8_t* blocks,
                      uint64_t block_stride, unsigned seg_stride, const uint16_t* num_data,
                      const uint16_t* erasure_locs, unsigned erasure_stride,
                      const uint16_t* erasure_counts, int32_t* status, unsigned nblocks)
{
    ensure_tables();
    void* enc = NULL;
    if (kind == ORC_RS8) {
        enc = malloc((size_t)(k + m) * k);
        if (orc_rs8_generator(k, m, (uint8_t*)enc)) { free(enc); return -1; }
    } else if (kind == ORC_RS16) {
        enc = malloc((size_t)(k + m) * k * 2);
        if (orc_rs16_generator(k, m, (uint16_t*)enc)) { free(enc); return -1; }
    } else if (kind != ORC_MDP) {
        return -1;
    }
    uint8_t** vecs = (uint8_t**)malloc(sizeof(uint8_t*) * (k + m));
    unsigned* locs = (unsigned*)malloc(sizeof(unsigned) * (m + 1));
    for (unsigned b = 0; b < nblocks; ++b) {
        uint8_t* blk = blocks + (size_t)b * block_stride;
        unsigned nd = num_data ? num_data[b] : k;
        unsigned ec = erasure_counts[b];
        for (unsigned s = 0; s < nd + m; ++s) vecs[s] = blk + (size_t)s * seg_stride;
        for (unsigned e = 0; e < ec; ++e) locs[e] = erasure_locs[(size_t)b * erasure_stride + e];
        if (kind == ORC_MDP) {
            /* missing parity is passed as NULL, as NormObject does for absent segments */
            for (unsigned e = 0; e < ec; ++e)
                if (locs[e] >= nd) vecs[locs[e]] = NULL;
        }
        int rc;
        if (kind == ORC_RS8) rc = orc_rs8_decode((uint8_t*)enc, k, m, vec, vecs, nd, ec, locs);
        else if (kind == ORC_RS16) rc = orc_rs16_decode((uint16_t*)enc, k, m, vec, vecs, nd, ec, locs);
        else rc = orc_mdp_decode(m, vec, vecs, nd, ec, locs);
        if (status) status[b] = rc;
    }
    free(vecs);
    free(locs);
    free(enc);
    return 0;
}

/* ======================================================================
 * Synthetic workload: splitmix64 counter streams.
 * ====================================================================== */
#define SM64_GAMMA 0x9E3779B97F4A7C15ULL

uint64_t orc_splitmix64_mix(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

void orc_fill_segment(uint64_t seed, uint64_t block, uint32_t seg, uint8_t* out, unsigned nbytes)
{
    uint64_t s0 = seed ^ (block << 20) ^ (uint64_t)seg;
    for (unsigned w = 0; w * 8 < nbytes; ++w) {
        uint64_t v = orc_splitmix64_mix(s0 + (uint64_t)(w + 1) * SM64_GAMMA);
        for (unsigned b = 0; b < 8 && w * 8 + b < nbytes; ++b) out[w * 8 + b] = (uint8_t)(v >> (8 * b));
    }
}

unsigned orc_erasure_pattern(uint64_t seed, uint64_t block, unsigned range, unsigned count,
                             uint16_t* out)
{
    if (count > range) count = range;
    uint16_t* perm = (uint16_t*)malloc(sizeof(uint16_t) * (range ? range : 1));
    for (unsigned i = 0; i < range; ++i) perm[i] = (uint16_t)i;
    uint64_t s0 = seed ^ 0xE7A5E7A500000000ULL ^ block;
    for (unsigned i = 0; i < count; ++i) {
        uint64_t r = orc_splitmix64_mix(s0 + (uint64_t)(i + 1) * SM64_GAMMA);
        unsigned j = i + (unsigned)(r % (uint64_t)(range - i));
        uint16_t t = perm[i];
        perm[i] = perm[j];
        perm[j] = t;
    }
    for (unsigned i = 0; i < count; ++i) out[i] = perm[i];
    for (unsigned i = 1; i < count; ++i) { /* insertion sort, count is small */
        uint16_t v = out[i];
        int j = (int)i - 1;
        while (j >= 0 && out[j] > v) { out[j + 1] = out[j]; --j; }
        out[j + 1] = v;
    }
    free(perm);
    return count;
}

/* ======================================================================
 * CPU baseline timing (C1): reference call pattern -- per-segment Encode into zeroed
 * parity, then erase `erasures` random source symbols (zeroed) and Decode.
 * ====================================================================== */
typedef struct {
    unsigned k, m, vec, erasures, b0, b1;
    uint64_t seed;
    const uint8_t* enc;
    uint8_t* buf; /* [nb][k+m][vec] */
    uint8_t* keep; /* copy of the erased source for verification */
    uint16_t* locs; /* [nb][erasures] */
    uint64_t bad;
    int phase;
} bench_job;

static void* bench_worker(void* arg)
{
    bench_job* j = (bench_job*)arg;
    const unsigned n = j->k + j->m;
    uint8_t* par[256];
    uint8_t* vecs[256];
    unsigned locs[256];
    for (unsigned b = j->b0; b < j->b1; ++b) {
        uint8_t* blk = j->buf + (size_t)(b - j->b0) * n * j->vec;
        if (j->phase == 0) {
            for (unsigned p = 0; p < j->m; ++p) par[p] = blk + (size_t)(j->k + p) * j->vec;
            for (unsigned s = 0; s < j->k; ++s)
                orc_rs8_encode(j->enc, j->k, j->m, j->vec, s, blk + (size_t)s * j->vec, par);
        } else {
            for (unsigned s = 0; s < n; ++s) vecs[s] = blk + (size_t)s * j->vec;
            const uint16_t* l = &j->locs[(size_t)(b - j->b0) * j->erasures];
            for (unsigned e = 0; e < j->erasures; ++e) locs[e] = l[e];
            orc_rs8_decode(j->enc, j->k, j->m, j->vec, vecs, j->k, j->erasures, locs);
        }
    }
    return NULL;
}

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

int orc_bench_rs8(unsigned k, unsigned m, unsigned vec, unsigned nblocks, unsigned erasures,
                  unsigned threads, uint64_t seed, double* t_encode, double* t_decode,
                  uint64_t* bad_blocks)
{
    ensure_tables();
    if (threads == 0) threads = 1;
    if (k + m > 255 || erasures > m || erasures > k) return -1;
    const unsigned n = k + m;
    uint8_t* enc = (uint8_t*)malloc((size_t)n * k);
    orc_rs8_generator(k, m, enc);
    uint8_t* buf = (uint8_t*)calloc((size_t)nblocks * n * vec, 1);
    uint8_t* keep = (uint8_t*)malloc((size_t)nblocks * erasures * vec + 1);
    uint16_t* locs = (uint16_t*)malloc(sizeof(uint16_t) * ((size_t)nblocks * erasures + 1));
    if (!buf || !keep || !locs) return -2;
    for (unsigned b = 0; b < nblocks; ++b)
        for (unsigned s = 0; s < k; ++s)
            orc_fill_segment(seed, b, s, buf + ((size_t)b * n + s) * vec, vec);
    bench_job* jobs = (bench_job*)calloc(threads, sizeof(bench_job));
    pthread_t* tids = (pthread_t*)calloc(threads, sizeof(pthread_t));
    for (unsigned t = 0; t < threads; ++t) {
        jobs[t].k = k; jobs[t].m = m; jobs[t].vec = vec; jobs[t].erasures = erasures;
        jobs[t].b0 = (unsigned)((uint64_t)nblocks * t / threads);
        jobs[t].b1 = (unsigned)((uint64_t)nblocks * (t + 1) / threads);
        jobs[t].seed = seed; jobs[t].enc = enc;
        jobs[t].buf = buf + (size_t)jobs[t].b0 * n * vec;
        jobs[t].locs = locs + (size_t)jobs[t].b0 * erasures;
    }
    /* encode phase */
    double t0 = now_s();
    for (unsigned t = 0; t < threads; ++t) { jobs[t].phase = 0; pthread_create(&tids[t], NULL, bench_worker, &jobs[t]); }
    for (unsigned t = 0; t < threads; ++t) pthread_join(tids[t], NULL);
    double t1 = now_s();
    /* erase (untimed): keep a copy, zero the erased source segments */
    for (unsigned b = 0; b < nblocks; ++b) {
        uint16_t* l = &locs[(size_t)b * erasures];
        orc_erasure_pattern(seed, b, k, erasures, l);
        for (unsigned e = 0; e < erasures; ++e) {
            uint8_t* s = buf + ((size_t)b * n + l[e]) * vec;
            memcpy(keep + ((size_t)b * erasures + e) * vec, s, vec);
            memset(s, 0, vec);
        }
    }
    double t2 = now_s();
    for (unsigned t = 0; t < threads; ++t) { jobs[t].phase = 1; pthread_create(&tids[t], NULL, bench_worker, &jobs[t]); }
    for (unsigned t = 0; t < threads; ++t) pthread_join(tids[t], NULL);
    double t3 = now_s();
    uint64_t bad = 0;
    for (unsigned b = 0; b < nblocks; ++b) {
        const uint16_t* l = &locs[(size_t)b * erasures];
        for (unsigned e = 0; e < erasures; ++e)
            if (memcmp(keep + ((size_t)b * erasures + e) * vec, buf + ((size_t)b * n + l[e]) * vec, vec)) {
                bad++;
                break;
            }
    }
    *t_encode = t1 - t0;
    *t_decode = t3 - t2;
    if (bad_blocks) *bad_blocks = bad;
    free(jobs); free(tids); free(enc); free(buf); free(keep); free(locs);
    return 0;
}
