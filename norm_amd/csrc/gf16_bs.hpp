// Bit-sliced GF(2^16) helpers for the RS16 Toeplitz split (kernels_tmvp.hip; host-compilable for
// the CPU unit test).  A lane's 32 symbols are 16 dwords of two native-endian uint16 symbols
// each; transpose() turns them into 16 bit planes (plane q = bit q of every symbol, the low and
// high halves of the dwords kept apart), and mulc() multiplies the planes by a constant c given
// as its 16 x 16 GF(2) matrix: M[p] bit q = bit p of c * 2^q (the column of x -> c*x for the
// basis symbol 2^q), so plane p of c*x is the XOR of the planes q selected by M[p].
#pragma once
#include <cstdint>

#if defined(__HIPCC__)
#define NFEC_HD __host__ __device__
#else
#define NFEC_HD
#endif

namespace nfec {
namespace bs16 {

// in place, its own inverse: swapmove stages 8, 4, 2, 1 on both 16-bit halves at once
NFEC_HD inline void transpose(uint32_t x[16])
{
    const uint32_t mask[4] = {0x00FF00FFu, 0x0F0F0F0Fu, 0x33333333u, 0x55555555u};
#pragma unroll
    for (int st = 0; st < 4; ++st) {
        const int s = 8 >> st;
#pragma unroll
        for (int d = 0; d < 16; ++d) {
            if (d & s) continue;
            const uint32_t t = ((x[d] >> s) ^ x[d + s]) & mask[st];
            x[d + s] ^= t;
            x[d] ^= t << s;
        }
    }
}

// out ^= c * in (planes), M = the 16 row masks of c (4-byte aligned).  On the device M must be
// wave-uniform: its rows are read into scalar registers, so the selects are scalar masks.
NFEC_HD inline void mulc_acc(const uint32_t in[16], uint32_t out[16], const uint16_t* M)
{
    uint32_t rows[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint32_t w = reinterpret_cast<const uint32_t*>(M)[i];
#if defined(__HIP_DEVICE_COMPILE__)
        rows[i] = __builtin_amdgcn_readfirstlane(w);
#else
        rows[i] = w;
#endif
    }
#pragma unroll
    for (int p = 0; p < 16; ++p) {
        uint32_t o = out[p];
        const uint32_t row = (rows[p >> 1] >> (16 * (p & 1))) & 0xFFFFu;
#pragma unroll
        for (int q = 0; q < 16; ++q) o ^= in[q] & (0u - ((row >> q) & 1u));
        out[p] = o;
    }
}

}  // namespace bs16
}  // namespace nfec
