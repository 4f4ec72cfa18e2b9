// Host check of norm_amd/csrc/gf16_bs.hpp (built with g++ by tests/test_tmvp.py): reads lines of
// "c s0 s1 ... s31" (decimal) and prints c*s_i for the 32 symbols, computed the way the device
// kernels do it (16 dwords -> bit planes -> multiply by the constant's row masks -> back).
// Row masks come from the caller as 16 numbers before the symbols: "M0..M15 s0..s31".
#include <cstdint>
#include <cstdio>
#include "../../norm_amd/csrc/gf16_bs.hpp"

int main()
{
    uint16_t M[16];
    uint32_t sym[32];
    for (;;) {
        for (int p = 0; p < 16; ++p) {
            unsigned v;
            if (scanf("%u", &v) != 1) return 0;
            M[p] = (uint16_t)v;
        }
        for (int i = 0; i < 32; ++i)
            if (scanf("%u", &sym[i]) != 1) return 1;
        uint32_t x[16], o[16];
        for (int d = 0; d < 16; ++d) x[d] = sym[2 * d] | (sym[2 * d + 1] << 16);
        nfec::bs16::transpose(x);
        for (int p = 0; p < 16; ++p) o[p] = 0;
        nfec::bs16::mulc_acc(x, o, M);
        nfec::bs16::transpose(o);
        for (int d = 0; d < 16; ++d) printf("%u %u ", o[d] & 0xFFFFu, o[d] >> 16);
        printf("\n");
    }
}
