// host_gf8.cpp -- GF(2^8) region multiply-accumulate on the host CPU, for the one call pattern a
// GPU cannot serve well: NORM's incremental sender, which calls Encode once per source segment
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
// c = 0 leaves dst alone, as the reference's addmul macro does (:258-259).  The batch and repair
// paths stay on the GPU; this serves nfec_encode_segment_host only.  GF(2^16) (RS16 Encode,
// normEncoderRS16.cpp:472-482) below: GFNI affine transforms per byte half, or log/exp tables.
// (host code only: the library's .cpp files go through the HIP compiler, whose device pass
// has no x86 builtins)
#ifndef __HIP_DEVICE_COMPILE__
#include <immintrin.h>

#include <cstring>
#include <mutex>

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

Gf16Mats gf16_mats(uint32_t c)
{
    const Field& f = gf16();
    uint32_t v[16];
    for (uint32_t j = 0; j < 16; ++j) v[j] = f.mul(c, 1u << j);
    auto mat = [&](uint32_t jbase, uint32_t ibase) {
        uint64_t m = 0;
        for (uint32_t i = 0; i < 8; ++i) {
            uint32_t row = 0;
            for (uint32_t j = 0; j < 8; ++j) row |= ((v[jbase + j] >> (ibase + i)) & 1u) << j;
            m |= (uint64_t)row << (8 * (7 - i));
        }
        return m;
    };
    return {mat(0, 0), mat(8, 0), mat(0, 8), mat(8, 8)};
}

__attribute__((target("avx2,gfni"))) void addmul16_gfni(uint16_t* dst, const uint16_t* src, uint32_t c, size_t n)
{
    const Gf16Mats g = gf16_mats(c);
    const __m256i ma = _mm256_set1_epi64x((long long)g.a), mb = _mm256_set1_epi64x((long long)g.b);
    const __m256i mc = _mm256_set1_epi64x((long long)g.c), md = _mm256_set1_epi64x((long long)g.d);
    const __m256i lo = _mm256_set1_epi16(0x00ff), hi = _mm256_set1_epi16((short)0xff00);
    size_t i = 0;
    for (; i + 16 <= n; i += 16) {
        const __m256i x = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i));
        const __m256i pa = _mm256_gf2p8affine_epi64_epi8(x, ma, 0);   // A x_lo at the even bytes
        const __m256i pb = _mm256_gf2p8affine_epi64_epi8(x, mb, 0);   // B x_hi at the odd bytes
        const __m256i pc = _mm256_gf2p8affine_epi64_epi8(x, mc, 0);   // C x_lo at the even bytes
        const __m256i pd = _mm256_gf2p8affine_epi64_epi8(x, md, 0);   // D x_hi at the odd bytes
        __m256i y = _mm256_xor_si256(_mm256_and_si256(pa, lo), _mm256_srli_epi16(pb, 8));
        y = _mm256_xor_si256(y, _mm256_xor_si256(_mm256_and_si256(pd, hi), _mm256_slli_epi16(pc, 8)));
        __m256i d = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(dst + i));
        _mm256_storeu_si256(reinterpret_cast<__m256i*>(dst + i), _mm256_xor_si256(d, y));
    }
    addmul16_scalar(dst + i, src + i, c, n - i);
}

}  // namespace

void host_gf16_addmul(uint16_t* dst, const uint16_t* src, uint32_t c, size_t nsym, int isa)
{
    if (c == 0 || nsym == 0) return;
    if ((isa < 0 ? best_isa() : isa) == NFEC_HOST_GF_GFNI) addmul16_gfni(dst, src, c & 0xffffu, nsym);
    else addmul16_scalar(dst, src, c & 0xffffu, nsym);
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
#endif  // __HIP_DEVICE_COMPILE__
