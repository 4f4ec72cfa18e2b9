// host_gf8.cpp -- GF(2^8) / GF(2^16) region products on the host CPU, for the per-call patterns a
// GPU cannot serve well.  First NORM's incremental sender, which calls Encode once per source segment
// and reads the parity without telling the encoder when a block ends
// (NormObject::NextSenderMsg -> NormSession::SenderEncode, normObject.cpp:2038-2052 ->
// NormEncoderRS8::Encode, normEncoderRS8.cpp:473-483).  One such call is m products of a
// 1.4 KB segment: a GPU round trip costs ~80 us of copies and launch against a few us of work.
//
//   dst[0..n) ^= c * src[0..n)   over GF(2^8) with polynomial 0x11d (normEncoderRS8.cpp:81)
//
// Three forms, chosen once per process from the CPU's features:
//   GFNI: vgf2p8affineqb applies the 8 x 8 bit matrix of c (any field: the matrix is built from
//         the field's own products, not GFNI's fixed 0x11b multiply), 32 bytes per instruction;
//   AVX2: the split-nibble table form, two vpshufb lookups of 16-entry product tables;
//   scalar: a 256 x 256 product table (the reference's own method, normEncoderRS8.cpp:140-149).
// c = 0 leaves dst alone, as the reference's addmul macro does (:258-259).  GF(2^16) (RS16
// Encode, normEncoderRS16.cpp:472-482) below: GFNI affine transforms on deinterleaved bytes, or
// log/exp tables.  Row dot products (sum_j c_j * src_j into one destination) serve the one-block
// host repair (nfec_decode_vectors_host); the batch paths stay on the GPU.
// (host code only: the library's .cpp files go through the HIP compiler, whose device pass
// has no x86 builtins)
#ifndef __HIP_DEVICE_COMPILE__
#include <immintrin.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <vector>

#include "nfec_internal.hpp"

namespace nfec {
namespace {

struct Gf8HostTables {
    uint8_t mul[256][256];        // scalar products
    uint8_t lo[256][16];          // c * n,        n < 16
    uint8_t hi[256][16];          // c * (n << 4), n < 16
    uint64_t affine[256];         // GFNI matrix of multiplication by c
};

const Gf8HostTables& tables()
{
    static Gf8HostTables t;
    static std::once_flag once;
    std::call_once(once, [] {
        const Field& f = gf8();
        for (uint32_t a = 0; a < 256; ++a)
            for (uint32_t b = 0; b < 256; ++b) t.mul[a][b] = (uint8_t)f.mul(a, b);
        for (uint32_t c = 0; c < 256; ++c) {
            for (uint32_t n = 0; n < 16; ++n) {
                t.lo[c][n] = t.mul[c][n];
                t.hi[c][n] = t.mul[c][n << 4];
            }
            // output bit i = parity(row_i & x), row_i bit b = bit i of c * 2^b; GFNI takes row i
            // from byte 7 - i of the matrix operand
            uint64_t m = 0;
            for (uint32_t i = 0; i < 8; ++i) {
                uint32_t row = 0;
                for (uint32_t b = 0; b < 8; ++b) row |= ((t.mul[c][1u << b] >> i) & 1u) << b;
                m |= (uint64_t)row << (8 * (7 - i));
            }
            t.affine[c] = m;
        }
    });
    return t;
}

void addmul_scalar(uint8_t* dst, const uint8_t* src, uint32_t c, size_t n)
{
    const uint8_t* row = tables().mul[c];
    for (size_t i = 0; i < n; ++i) dst[i] ^= row[src[i]];
}

__attribute__((target("avx2"))) void addmul_avx2(uint8_t* dst, const uint8_t* src, uint32_t c, size_t n)
{
    const Gf8HostTables& t = tables();
    const __m256i lo = _mm256_broadcastsi128_si256(_mm_loadu_si128(reinterpret_cast<const __m128i*>(t.lo[c])));
    const __m256i hi = _mm256_broadcastsi128_si256(_mm_loadu_si128(reinterpret_cast<const __m128i*>(t.hi[c])));
    const __m256i nib = _mm256_set1_epi8(0x0f);
    size_t i = 0;
    for (; i + 32 <= n; i += 32) {
        const __m256i x = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i));
        const __m256i pl = _mm256_shuffle_epi8(lo, _mm256_and_si256(x, nib));
        const __m256i ph = _mm256_shuffle_epi8(hi, _mm256_and_si256(_mm256_srli_epi64(x, 4), nib));
        __m256i d = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(dst + i));
        d = _mm256_xor_si256(d, _mm256_xor_si256(pl, ph));
        _mm256_storeu_si256(reinterpret_cast<__m256i*>(dst + i), d);
    }
    addmul_scalar(dst + i, src + i, c, n - i);
}

// The last n < 32 bytes of a vector: whole dwords by masked loads and stores (masked-out lanes
// are neither read nor written), so a 1400-byte segment's 24-byte tail stays vectorised; the
// final 0-3 bytes go scalar.
__attribute__((target("avx2"))) inline __m256i tail_mask(size_t bytes)
{
    return _mm256_cmpgt_epi32(_mm256_set1_epi32((int)(bytes / 4)), _mm256_setr_epi32(0, 1, 2, 3, 4, 5, 6, 7));
}

__attribute__((target("avx2"))) inline __m256i load_tail(const void* p, __m256i mask)
{
    return _mm256_maskload_epi32(static_cast<const int*>(p), mask);
}

__attribute__((target("avx2"))) inline void store_tail(void* p, __m256i mask, __m256i v)
{
    _mm256_maskstore_epi32(static_cast<int*>(p), mask, v);
}

__attribute__((target("avx2,gfni"))) void addmul_gfni(uint8_t* dst, const uint8_t* src, uint32_t c, size_t n)
{
    const __m256i a = _mm256_set1_epi64x((long long)tables().affine[c]);
    size_t i = 0;
    for (; i + 32 <= n; i += 32) {
        const __m256i x = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i));
        __m256i d = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(dst + i));
        d = _mm256_xor_si256(d, _mm256_gf2p8affine_epi64_epi8(x, a, 0));
        _mm256_storeu_si256(reinterpret_cast<__m256i*>(dst + i), d);
    }
    if (n - i >= 4) {
        const __m256i mask = tail_mask(n - i);
        const __m256i d = _mm256_xor_si256(load_tail(dst + i, mask),
                                           _mm256_gf2p8affine_epi64_epi8(load_tail(src + i, mask), a, 0));
        store_tail(dst + i, mask, d);
        i += (n - i) & ~(size_t)3;
    }
    addmul_scalar(dst + i, src + i, c, n - i);
}

using AddMul = void (*)(uint8_t*, const uint8_t*, uint32_t, size_t);

int best_isa()
{
    static const int isa = [] {
        __builtin_cpu_init();
        if (__builtin_cpu_supports("avx2") && __builtin_cpu_supports("gfni")) return NFEC_HOST_GF_GFNI;
        if (__builtin_cpu_supports("avx2")) return NFEC_HOST_GF_AVX2;
        return NFEC_HOST_GF_SCALAR;
    }();
    return isa;
}

AddMul pick(int isa)
{
    switch (isa) {
        case NFEC_HOST_GF_GFNI: return addmul_gfni;
        case NFEC_HOST_GF_AVX2: return addmul_avx2;
        default: return addmul_scalar;
    }
}

// ---- GF(2^16) (poly 0x1100B, normEncoderRS16.cpp:88), native-endian 16-bit symbols ----
// y = c * x splits over the symbol's bytes: y_lo = A x_lo + B x_hi, y_hi = C x_lo + D x_hi with
// four 8 x 8 GF(2) matrices taken from c * 2^j.  GFNI applies one matrix to every byte, so a
// 32-byte step is four affine transforms whose results are picked by byte position (16-bit
// shifts move the odd byte of a product to the even position and back).

void addmul16_scalar(uint16_t* dst, const uint16_t* src, uint32_t c, size_t n)
{
    const Field& f = gf16();
    const uint32_t lc = f.log[c];
    for (size_t i = 0; i < n; ++i)
        if (src[i]) dst[i] ^= (uint16_t)f.exp[lc + f.log[src[i]]];
}

struct Gf16Mats {
    uint64_t a, b, c, d;
};

// 8 x 8 bit transpose: byte j of x holds row j; afterwards byte i holds column i
inline uint64_t transpose8(uint64_t x)
{
    uint64_t t = (x ^ (x >> 7)) & 0x00AA00AA00AA00AAull;
    x ^= t ^ (t << 7);
    t = (x ^ (x >> 14)) & 0x0000CCCC0000CCCCull;
    x ^= t ^ (t << 14);
    t = (x ^ (x >> 28)) & 0x00000000F0F0F0F0ull;
    return x ^ t ^ (t << 28);
}

Gf16Mats gf16_mats_direct(uint32_t c)
{
    // v[j] = c * x^j by doubling (alpha = x; r = x^16 mod the field polynomial)
    static const uint32_t r = gf16().exp[16];
    uint32_t v[16];
    v[0] = c & 0xffffu;
    for (uint32_t j = 1; j < 16; ++j) v[j] = ((v[j - 1] << 1) & 0xffffu) ^ ((v[j - 1] >> 15) ? r : 0u);
    // matrix (jbase, ibase): row i = bit (ibase + i) of v[jbase + 0..7]; GFNI takes row i from
    // byte 7 - i, so transpose the bytes (v[jbase + j] >> ibase) and reverse them
    auto mat = [&](uint32_t jbase, uint32_t ibase) {
        uint64_t w = 0;
        for (uint32_t j = 0; j < 8; ++j) w |= (uint64_t)((v[jbase + j] >> ibase) & 0xffu) << (8 * j);
        return __builtin_bswap64(transpose8(w));
    };
    return {mat(0, 0), mat(8, 0), mat(0, 8), mat(8, 8)};
}

// The matrices are GF(2)-linear in c, so M(c) = M(c & 0xff) ^ M(c & 0xff00): two 256-entry
// tables (16 KiB) built once, two loads and an XOR per coefficient.
struct Gf16MatTables {
    Gf16Mats lo[256], hi[256];
};

const Gf16MatTables& gf16_mat_tables()
{
    static Gf16MatTables t;
    static std::once_flag once;
    std::call_once(once, [] {
        for (uint32_t b = 0; b < 256; ++b) {
            t.lo[b] = gf16_mats_direct(b);
            t.hi[b] = gf16_mats_direct(b << 8);
        }
    });
    return t;
}

inline Gf16Mats gf16_mats(uint32_t c)
{
    const Gf16MatTables& t = gf16_mat_tables();
    const Gf16Mats& l = t.lo[c & 0xffu];
    const Gf16Mats& h = t.hi[(c >> 8) & 0xffu];
    return {l.a ^ h.a, l.b ^ h.b, l.c ^ h.c, l.d ^ h.d};
}

// GFNI applies one matrix per 64-bit lane.  Deinterleaving each 128-bit lane's 8 symbols into
// [8 low bytes | 8 high bytes] lets one transform apply A to the low bytes and D to the high
// ones ([A, D] per lane pair), a second C and B ([C, B]); y_lo = A x_lo + B x_hi and
// y_hi = C x_lo + D x_hi are then the first result plus the second with its two lanes swapped:
// two affine transforms per 16 symbols instead of four.
__attribute__((target("avx2,gfni"))) inline __m256i gf16_deint()
{
    return _mm256_setr_epi8(0, 2, 4, 6, 8, 10, 12, 14, 1, 3, 5, 7, 9, 11, 13, 15, 0, 2, 4, 6, 8, 10, 12, 14, 1, 3, 5, 7,
                            9, 11, 13, 15);
}

__attribute__((target("avx2,gfni"))) inline __m256i gf16_inter()
{
    return _mm256_setr_epi8(0, 8, 1, 9, 2, 10, 3, 11, 4, 12, 5, 13, 6, 14, 7, 15, 0, 8, 1, 9, 2, 10, 3, 11, 4, 12, 5, 13,
                            6, 14, 7, 15);
}

__attribute__((target("avx2,gfni"))) void addmul16_gfni(uint16_t* dst, const uint16_t* src, uint32_t c, size_t n)
{
    const Gf16Mats g = gf16_mats(c);
    const __m256i m1 = _mm256_setr_epi64x((long long)g.a, (long long)g.d, (long long)g.a, (long long)g.d);
    const __m256i m2 = _mm256_setr_epi64x((long long)g.c, (long long)g.b, (long long)g.c, (long long)g.b);
    const __m256i deint = gf16_deint(), inter = gf16_inter();
    size_t i = 0;
    for (; i + 16 <= n; i += 16) {
        const __m256i x = _mm256_shuffle_epi8(_mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i)), deint);
        const __m256i r = _mm256_xor_si256(_mm256_gf2p8affine_epi64_epi8(x, m1, 0),
                                           _mm256_shuffle_epi32(_mm256_gf2p8affine_epi64_epi8(x, m2, 0), 0x4e));
        __m256i d = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(dst + i));
        _mm256_storeu_si256(reinterpret_cast<__m256i*>(dst + i), _mm256_xor_si256(d, _mm256_shuffle_epi8(r, inter)));
    }
    if (n - i >= 2) {
        const __m256i mask = tail_mask(2 * (n - i));
        const __m256i x = _mm256_shuffle_epi8(load_tail(src + i, mask), deint);
        const __m256i r = _mm256_xor_si256(_mm256_gf2p8affine_epi64_epi8(x, m1, 0),
                                           _mm256_shuffle_epi32(_mm256_gf2p8affine_epi64_epi8(x, m2, 0), 0x4e));
        store_tail(dst + i, mask, _mm256_xor_si256(load_tail(dst + i, mask), _mm256_shuffle_epi8(r, inter)));
        i += (n - i) & ~(size_t)1;
    }
    addmul16_scalar(dst + i, src + i, c, n - i);
}

// ---- dot products: dst[0..n) (^)= sum_j coef[j] * src[j][off + 0..n) ----
// One accumulator set per 128 bytes (GF(2^8)) / 32 symbols (GF(2^16)) over all columns: one
// load per product instead of the region form's load-load-store, and the destination written
// once.  GF(2^16) keeps the four affine partial products apart across columns (the byte masks
// and shifts that combine them are linear) and combines them once at the end.

__attribute__((target("avx2,gfni"))) void dot_gfni(uint8_t* dst, const uint8_t* const* src, size_t off,
                                                   const uint16_t* coef, uint32_t nc, size_t n, bool acc)
{
    const Gf8HostTables& t = tables();
    size_t i = 0;
    for (; i + 128 <= n; i += 128) {
        __m256i a0, a1, a2, a3;
        if (acc) {
            a0 = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(dst + i));
            a1 = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(dst + i + 32));
            a2 = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(dst + i + 64));
            a3 = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(dst + i + 96));
        } else {
            a0 = a1 = a2 = a3 = _mm256_setzero_si256();
        }
        for (uint32_t j = 0; j < nc; ++j) {
            const __m256i m = _mm256_set1_epi64x((long long)t.affine[coef[j] & 0xffu]);
            const uint8_t* p = src[j] + off + i;
            a0 = _mm256_xor_si256(a0, _mm256_gf2p8affine_epi64_epi8(_mm256_loadu_si256(reinterpret_cast<const __m256i*>(p)), m, 0));
            a1 = _mm256_xor_si256(a1, _mm256_gf2p8affine_epi64_epi8(_mm256_loadu_si256(reinterpret_cast<const __m256i*>(p + 32)), m, 0));
            a2 = _mm256_xor_si256(a2, _mm256_gf2p8affine_epi64_epi8(_mm256_loadu_si256(reinterpret_cast<const __m256i*>(p + 64)), m, 0));
            a3 = _mm256_xor_si256(a3, _mm256_gf2p8affine_epi64_epi8(_mm256_loadu_si256(reinterpret_cast<const __m256i*>(p + 96)), m, 0));
        }
        _mm256_storeu_si256(reinterpret_cast<__m256i*>(dst + i), a0);
        _mm256_storeu_si256(reinterpret_cast<__m256i*>(dst + i + 32), a1);
        _mm256_storeu_si256(reinterpret_cast<__m256i*>(dst + i + 64), a2);
        _mm256_storeu_si256(reinterpret_cast<__m256i*>(dst + i + 96), a3);
    }
    for (; i + 32 <= n; i += 32) {
        __m256i a0 = acc ? _mm256_loadu_si256(reinterpret_cast<const __m256i*>(dst + i)) : _mm256_setzero_si256();
        for (uint32_t j = 0; j < nc; ++j) {
            const __m256i m = _mm256_set1_epi64x((long long)t.affine[coef[j] & 0xffu]);
            a0 = _mm256_xor_si256(a0, _mm256_gf2p8affine_epi64_epi8(
                                          _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src[j] + off + i)), m, 0));
        }
        _mm256_storeu_si256(reinterpret_cast<__m256i*>(dst + i), a0);
    }
    if (n - i >= 4) {
        const __m256i mask = tail_mask(n - i);
        __m256i a0 = acc ? load_tail(dst + i, mask) : _mm256_setzero_si256();
        for (uint32_t j = 0; j < nc; ++j) {
            const __m256i m = _mm256_set1_epi64x((long long)t.affine[coef[j] & 0xffu]);
            a0 = _mm256_xor_si256(a0, _mm256_gf2p8affine_epi64_epi8(load_tail(src[j] + off + i, mask), m, 0));
        }
        store_tail(dst + i, mask, a0);
        i += (n - i) & ~(size_t)3;
    }
    if (i < n) {
        if (!acc) std::memset(dst + i, 0, n - i);
        for (uint32_t j = 0; j < nc; ++j) addmul_scalar(dst + i, src[j] + off + i, coef[j] & 0xffu, n - i);
    }
}

__attribute__((target("avx2,gfni"))) void dot16_gfni(uint16_t* dst, const uint16_t* const* src, size_t off,
                                                     const uint16_t* coef, uint32_t nc, size_t n, bool acc)
{
    const Gf16MatTables& t = gf16_mat_tables();
    const __m256i deint = gf16_deint(), inter = gf16_inter();
    size_t i = 0;
    for (; i + 64 <= n; i += 64) {
        __m256i p1[4], p2[4];
        for (int q = 0; q < 4; ++q) p1[q] = p2[q] = _mm256_setzero_si256();
        for (uint32_t j = 0; j < nc; ++j) {
            const uint32_t c = coef[j];
            const __m256i mm = _mm256_xor_si256(
                _mm256_loadu_si256(reinterpret_cast<const __m256i*>(&t.lo[c & 0xffu])),
                _mm256_loadu_si256(reinterpret_cast<const __m256i*>(&t.hi[c >> 8])));
            const __m256i m1 = _mm256_permute4x64_epi64(mm, 0xcc);  // [A, D, A, D]
            const __m256i m2 = _mm256_permute4x64_epi64(mm, 0x66);  // [C, B, C, B]
            const uint16_t* p = src[j] + off + i;
            for (int q = 0; q < 4; ++q) {
                const __m256i x =
                    _mm256_shuffle_epi8(_mm256_loadu_si256(reinterpret_cast<const __m256i*>(p + 16 * q)), deint);
                p1[q] = _mm256_xor_si256(p1[q], _mm256_gf2p8affine_epi64_epi8(x, m1, 0));
                p2[q] = _mm256_xor_si256(p2[q], _mm256_gf2p8affine_epi64_epi8(x, m2, 0));
            }
        }
        for (int q = 0; q < 4; ++q) {
            __m256i y = _mm256_shuffle_epi8(_mm256_xor_si256(p1[q], _mm256_shuffle_epi32(p2[q], 0x4e)), inter);
            if (acc) y = _mm256_xor_si256(y, _mm256_loadu_si256(reinterpret_cast<const __m256i*>(dst + i + 16 * q)));
            _mm256_storeu_si256(reinterpret_cast<__m256i*>(dst + i + 16 * q), y);
        }
    }
    // the rest: 16-symbol steps, then one masked step, then an odd last symbol
    while (n - i >= 2) {
        const size_t len = std::min<size_t>(16, n - i);
        const __m256i mask = tail_mask(2 * len);
        __m256i p1 = _mm256_setzero_si256(), p2 = p1;
        for (uint32_t j = 0; j < nc; ++j) {
            const uint32_t c = coef[j];
            const __m256i mm = _mm256_xor_si256(
                _mm256_loadu_si256(reinterpret_cast<const __m256i*>(&t.lo[c & 0xffu])),
                _mm256_loadu_si256(reinterpret_cast<const __m256i*>(&t.hi[c >> 8])));
            const __m256i x = _mm256_shuffle_epi8(load_tail(src[j] + off + i, mask), deint);
            p1 = _mm256_xor_si256(p1, _mm256_gf2p8affine_epi64_epi8(x, _mm256_permute4x64_epi64(mm, 0xcc), 0));
            p2 = _mm256_xor_si256(p2, _mm256_gf2p8affine_epi64_epi8(x, _mm256_permute4x64_epi64(mm, 0x66), 0));
        }
        __m256i y = _mm256_shuffle_epi8(_mm256_xor_si256(p1, _mm256_shuffle_epi32(p2, 0x4e)), inter);
        if (acc) y = _mm256_xor_si256(y, load_tail(dst + i, mask));
        store_tail(dst + i, mask, y);
        i += len & ~(size_t)1;
    }
    if (i < n) {
        if (!acc) dst[i] = 0;
        for (uint32_t j = 0; j < nc; ++j)
            if (coef[j]) addmul16_scalar(dst + i, src[j] + off + i, coef[j], n - i);
    }
}

// ---- one source into many rows: dst[r][0..n) ^= coef[r * cstride] * src[0..n) ----
// The per-segment Encode's m products share their source: a 128-byte piece of it stays in
// registers while every row takes it (one load of the source per piece instead of per row).

__attribute__((target("avx2,gfni"))) void rows_gfni(uint8_t* const* dst, const uint8_t* src, const uint32_t* coef,
                                                    size_t cstride, uint32_t nr, size_t n)
{
    const Gf8HostTables& t = tables();
    size_t i = 0;
    for (; i + 128 <= n; i += 128) {
        const __m256i x0 = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i));
        const __m256i x1 = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i + 32));
        const __m256i x2 = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i + 64));
        const __m256i x3 = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i + 96));
        for (uint32_t r = 0; r < nr; ++r) {
            const uint32_t c = coef[r * cstride] & 0xffu;
            if (!c) continue;
            const __m256i m = _mm256_set1_epi64x((long long)t.affine[c]);
            __m256i* d = reinterpret_cast<__m256i*>(dst[r] + i);
            _mm256_storeu_si256(d, _mm256_xor_si256(_mm256_loadu_si256(d), _mm256_gf2p8affine_epi64_epi8(x0, m, 0)));
            _mm256_storeu_si256(d + 1, _mm256_xor_si256(_mm256_loadu_si256(d + 1), _mm256_gf2p8affine_epi64_epi8(x1, m, 0)));
            _mm256_storeu_si256(d + 2, _mm256_xor_si256(_mm256_loadu_si256(d + 2), _mm256_gf2p8affine_epi64_epi8(x2, m, 0)));
            _mm256_storeu_si256(d + 3, _mm256_xor_si256(_mm256_loadu_si256(d + 3), _mm256_gf2p8affine_epi64_epi8(x3, m, 0)));
        }
    }
    if (i < n)
        for (uint32_t r = 0; r < nr; ++r) {
            const uint32_t c = coef[r * cstride] & 0xffu;
            if (c) addmul_gfni(dst[r] + i, src + i, c, n - i);
        }
}

__attribute__((target("avx2,gfni"))) void rows16_gfni(uint16_t* const* dst, const uint16_t* src, const uint32_t* coef,
                                                      size_t cstride, uint32_t nr, size_t n)
{
    const Gf16MatTables& t = gf16_mat_tables();
    const __m256i deint = gf16_deint(), inter = gf16_inter();
    // rows in groups of 64, their two lane-pair matrices built once per group
    constexpr uint32_t kGroup = 64;
    __m256i m1[kGroup], m2[kGroup];
    for (uint32_t r0 = 0; r0 < nr; r0 += kGroup) {
        const uint32_t gn = std::min(kGroup, nr - r0);
        for (uint32_t r = 0; r < gn; ++r) {
            const uint32_t c = coef[(r0 + r) * cstride] & 0xffffu;
            const __m256i mm = _mm256_xor_si256(_mm256_loadu_si256(reinterpret_cast<const __m256i*>(&t.lo[c & 0xffu])),
                                                _mm256_loadu_si256(reinterpret_cast<const __m256i*>(&t.hi[c >> 8])));
            m1[r] = _mm256_permute4x64_epi64(mm, 0xcc);  // [A, D, A, D]
            m2[r] = _mm256_permute4x64_epi64(mm, 0x66);  // [C, B, C, B]
        }
        size_t i = 0;
        for (; i + 64 <= n; i += 64) {
            __m256i x[4];
            for (int q = 0; q < 4; ++q)
                x[q] = _mm256_shuffle_epi8(_mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i + 16 * q)), deint);
            for (uint32_t r = 0; r < gn; ++r) {
                if (!(coef[(r0 + r) * cstride] & 0xffffu)) continue;
                __m256i* d = reinterpret_cast<__m256i*>(dst[r0 + r] + i);
                for (int q = 0; q < 4; ++q) {
                    const __m256i y = _mm256_xor_si256(_mm256_gf2p8affine_epi64_epi8(x[q], m1[r], 0),
                                                       _mm256_shuffle_epi32(_mm256_gf2p8affine_epi64_epi8(x[q], m2[r], 0), 0x4e));
                    _mm256_storeu_si256(d + q, _mm256_xor_si256(_mm256_loadu_si256(d + q), _mm256_shuffle_epi8(y, inter)));
                }
            }
        }
        if (i < n)
            for (uint32_t r = r0; r < r0 + gn; ++r) {
                const uint32_t c = coef[r * cstride] & 0xffffu;
                if (c) addmul16_gfni(dst[r] + i, src + i, c, n - i);
            }
    }
}

// ---- the MDP encoder's LFSR step (normEncoderMDP.cpp:178-211), one pass per 128-byte piece:
// s = data ^ P0; P_i = P_(i+1) ^ g[m-1-i] * s (i < m-1); P_(m-1) = g[0] * s.  Pieces are
// independent, so each one reads the old P_(i+1) before it is overwritten, with s in registers.

__attribute__((target("avx2,gfni"))) void mdp_step_gfni(uint8_t* const* par, const uint8_t* data, const uint8_t* g,
                                                        uint32_t m, size_t n, size_t& done)
{
    const Gf8HostTables& t = tables();
    size_t i = 0;
    for (; i + 128 <= n; i += 128) {
        __m256i sv[4];
        for (int q = 0; q < 4; ++q)
            sv[q] = _mm256_xor_si256(_mm256_loadu_si256(reinterpret_cast<const __m256i*>(data + i + 32 * q)),
                                     _mm256_loadu_si256(reinterpret_cast<const __m256i*>(par[0] + i + 32 * q)));
        for (uint32_t r = 0; r + 1 < m; ++r) {
            const __m256i mt = _mm256_set1_epi64x((long long)t.affine[g[m - 1 - r]]);
            const uint8_t* nx = par[r + 1] + i;
            uint8_t* d = par[r] + i;
            for (int q = 0; q < 4; ++q)
                _mm256_storeu_si256(reinterpret_cast<__m256i*>(d + 32 * q),
                                    _mm256_xor_si256(_mm256_loadu_si256(reinterpret_cast<const __m256i*>(nx + 32 * q)),
                                                     _mm256_gf2p8affine_epi64_epi8(sv[q], mt, 0)));
        }
        const __m256i m0 = _mm256_set1_epi64x((long long)t.affine[g[0]]);
        for (int q = 0; q < 4; ++q)
            _mm256_storeu_si256(reinterpret_cast<__m256i*>(par[m - 1] + i + 32 * q), _mm256_gf2p8affine_epi64_epi8(sv[q], m0, 0));
    }
    done = i;
}

}  // namespace

void host_gf16_addmul(uint16_t* dst, const uint16_t* src, uint32_t c, size_t nsym, int isa)
{
    if (c == 0 || nsym == 0) return;
    if ((isa < 0 ? best_isa() : isa) == NFEC_HOST_GF_GFNI) addmul16_gfni(dst, src, c & 0xffffu, nsym);
    else addmul16_scalar(dst, src, c & 0xffffu, nsym);
}

void host_gf8_dot(uint8_t* dst, const uint8_t* const* src, size_t off, const uint16_t* coef, uint32_t nc, size_t n,
                  bool acc, int isa)
{
    if (n == 0) return;
    if ((isa < 0 ? best_isa() : isa) == NFEC_HOST_GF_GFNI) return dot_gfni(dst, src, off, coef, nc, n, acc);
    if (!acc) std::memset(dst, 0, n);
    for (uint32_t j = 0; j < nc; ++j) host_gf8_addmul(dst, src[j] + off, coef[j] & 0xffu, n, isa);
}

void host_gf16_dot(uint16_t* dst, const uint16_t* const* src, size_t off, const uint16_t* coef, uint32_t nc,
                   size_t nsym, bool acc, int isa)
{
    if (nsym == 0) return;
    if ((isa < 0 ? best_isa() : isa) == NFEC_HOST_GF_GFNI) return dot16_gfni(dst, src, off, coef, nc, nsym, acc);
    if (!acc) std::memset(dst, 0, nsym * 2);
    for (uint32_t j = 0; j < nc; ++j) host_gf16_addmul(dst, src[j] + off, coef[j], nsym, isa);
}

void host_gf8_addmul_rows(uint8_t* const* dst, const uint8_t* src, const uint32_t* coef, size_t cstride, uint32_t nrows,
                          size_t n, int isa)
{
    if (n == 0) return;
    if ((isa < 0 ? best_isa() : isa) == NFEC_HOST_GF_GFNI) return rows_gfni(dst, src, coef, cstride, nrows, n);
    for (uint32_t r = 0; r < nrows; ++r) host_gf8_addmul(dst[r], src, coef[r * cstride], n, isa);
}

void host_gf16_addmul_rows(uint16_t* const* dst, const uint16_t* src, const uint32_t* coef, size_t cstride,
                           uint32_t nrows, size_t nsym, int isa)
{
    if (nsym == 0) return;
    if ((isa < 0 ? best_isa() : isa) == NFEC_HOST_GF_GFNI) return rows16_gfni(dst, src, coef, cstride, nrows, nsym);
    for (uint32_t r = 0; r < nrows; ++r) host_gf16_addmul(dst[r], src, coef[r * cstride], nsym, isa);
}

void host_mdp_step(uint8_t* const* parity, const uint8_t* data, const uint8_t* g, uint32_t m, size_t n, int isa)
{
    size_t i = 0;
    if (m && (isa < 0 ? best_isa() : isa) == NFEC_HOST_GF_GFNI) mdp_step_gfni(parity, data, g, m, n, i);
    if (i >= n || m == 0) return;
    // the rest (and the other forms): the same step through a scratch copy of s
    const size_t len = n - i;
    thread_local std::vector<uint8_t> sv;
    sv.resize(len);
    for (size_t j = 0; j < len; ++j) sv[j] = data[i + j] ^ parity[0][i + j];
    for (uint32_t r = 0; r + 1 < m; ++r) {
        std::memcpy(parity[r] + i, parity[r + 1] + i, len);
        host_gf8_addmul(parity[r] + i, sv.data(), g[m - 1 - r], len, isa);
    }
    std::memset(parity[m - 1] + i, 0, len);
    host_gf8_addmul(parity[m - 1] + i, sv.data(), g[0], len, isa);
}

int host_gf8_isa() { return best_isa(); }

void host_gf8_addmul(uint8_t* dst, const uint8_t* src, uint32_t c, size_t n, int isa)
{
    if (c == 0 || n == 0) return;
    pick(isa < 0 ? best_isa() : isa)(dst, src, c & 0xffu, n);
}

}  // namespace nfec

extern "C" int nfec_gf16_addmul_host(void* dst, const void* src, uint16_t c, size_t symbols, int isa)
{
    using namespace nfec;
    if ((!dst || !src) && symbols) return fail(NFEC_EINVAL, "null buffer");
    if (isa > NFEC_HOST_GF_GFNI) return fail(NFEC_EINVAL, "unknown host form");
    const int best = best_isa();
    if (isa > best) return fail(NFEC_ENOTSUP, "this CPU lacks the instructions of that form");
    // (the AVX2 form has no GF(2^16) variant: it runs the scalar one)
    const int form = (isa < 0 ? best : isa) == NFEC_HOST_GF_GFNI ? NFEC_HOST_GF_GFNI : NFEC_HOST_GF_SCALAR;
    // unaligned symbol arrays are fine (byte loads in both forms)
    host_gf16_addmul(static_cast<uint16_t*>(dst), static_cast<const uint16_t*>(src), c, symbols, form);
    return form;
}

extern "C" int nfec_gf8_addmul_host(void* dst, const void* src, uint8_t c, size_t bytes, int isa)
{
    using namespace nfec;
    if ((!dst || !src) && bytes) return fail(NFEC_EINVAL, "null buffer");
    if (isa > NFEC_HOST_GF_GFNI) return fail(NFEC_EINVAL, "unknown host form");
    const int best = best_isa();
    if (isa > best) return fail(NFEC_ENOTSUP, "this CPU lacks the instructions of that form");
    host_gf8_addmul(static_cast<uint8_t*>(dst), static_cast<const uint8_t*>(src), c, bytes, isa < 0 ? best : isa);
    return isa < 0 ? best : isa;
}

extern "C" int nfec_gf_dot_host(int bits, void* dst, const void* const* src, const uint16_t* coef, uint32_t ncols,
                                size_t n, int accumulate, int isa)
{
    using namespace nfec;
    if (bits != 8 && bits != 16) return fail(NFEC_EINVAL, "bits must be 8 or 16");
    if (n && (!dst || (ncols && (!src || !coef)))) return fail(NFEC_EINVAL, "null buffer");
    for (uint32_t j = 0; n && j < ncols; ++j)
        if (!src[j]) return fail(NFEC_EINVAL, "null source vector");
    if (isa > NFEC_HOST_GF_GFNI) return fail(NFEC_EINVAL, "unknown host form");
    const int best = best_isa();
    if (isa > best) return fail(NFEC_ENOTSUP, "this CPU lacks the instructions of that form");
    int form = isa < 0 ? best : isa;
    if (bits == 16) {
        form = form == NFEC_HOST_GF_GFNI ? NFEC_HOST_GF_GFNI : NFEC_HOST_GF_SCALAR;
        host_gf16_dot(static_cast<uint16_t*>(dst), reinterpret_cast<const uint16_t* const*>(src), 0, coef, ncols, n,
                      accumulate != 0, form);
    } else {
        host_gf8_dot(static_cast<uint8_t*>(dst), reinterpret_cast<const uint8_t* const*>(src), 0, coef, ncols, n,
                     accumulate != 0, form);
    }
    return form;
}
#endif  // __HIP_DEVICE_COMPILE__
