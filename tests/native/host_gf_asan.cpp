// host_gf_asan.cpp -- the host GF(2^8) / GF(2^16) products (norm_amd/csrc/host_gf8.cpp: region
// multiply-accumulate and the row dot products of the one-block host repair) under AddressSanitizer
// and UBSan, on buffers of exactly n bytes, every length 0..299 and every form this CPU has: the
// masked-vector tails must neither read nor write past a vector.  Host code only (the library's
// .cpp files compiled for the host with the sanitizers, no GPU); `make -C tests/native asan`.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>
#include "nfec_internal.hpp"
extern "C" int nfec_gf_dot_host(int, void*, const void* const*, const uint16_t*, uint32_t, size_t, int, int);
extern "C" int nfec_gf8_addmul_host(void*, const void*, uint8_t, size_t, int);
extern "C" int nfec_gf16_addmul_host(void*, const void*, uint16_t, size_t, int);
int main()
{
    srand(3);
    for (int bits : {8, 16})
        for (size_t n = 0; n < 300; ++n)
            for (int isa = 0; isa <= 2; ++isa) {
                const size_t es = bits / 8;
                const uint32_t nc = 1 + rand() % 5;
                std::vector<void*> src(nc);
                std::vector<uint16_t> co(nc);
                for (uint32_t j = 0; j < nc; ++j) {
                    src[j] = malloc(n * es ? n * es : 1);  // exact size: ASan catches any overread
                    for (size_t b = 0; b < n * es; ++b) ((uint8_t*)src[j])[b] = rand();
                    co[j] = rand() & (bits == 8 ? 0xff : 0xffff);
                }
                void* dst = malloc(n * es ? n * es : 1);
                memset(dst, 0, n * es);
                nfec_gf_dot_host(bits, dst, src.data(), co.data(), nc, n, rand() & 1, isa);
                if (bits == 8) nfec_gf8_addmul_host(dst, src[0], co[0], n, isa);
                else nfec_gf16_addmul_host(dst, src[0], co[0], n, isa);
                for (auto p : src) free(p);
                free(dst);
            }
    std::printf("asan driver done\n");
}
