// host_gf_asan.cpp -- the host GF(2^8) / GF(2^16) products (norm_amd/csrc/host_gf8.cpp: region
// multiply-accumulate, the per-segment Encode's one-source-many-rows form, checked against it, and
// the row dot products of the one-block host repair) under AddressSanitizer
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
    // one source into many rows (the per-segment Encode) against the region products, row by row
    for (int bits : {8, 16})
        for (size_t n = 0; n < 300; n += (n < 40 ? 1 : 7))
            for (int isa = 0; isa <= 2; ++isa) {
                const size_t es = bits / 8;
                const uint32_t nr = 1 + rand() % 40;
                const size_t stride = 3;
                std::vector<uint32_t> co(nr * stride);
                for (auto& v : co) v = rand() & (bits == 8 ? 0xff : 0xffff);
                co[0] = 0;
                uint8_t* src = (uint8_t*)malloc(n * es ? n * es : 1);
                for (size_t b = 0; b < n * es; ++b) src[b] = rand();
                std::vector<uint8_t*> a(nr), b(nr);
                for (uint32_t r = 0; r < nr; ++r) {
                    a[r] = (uint8_t*)malloc(n * es ? n * es : 1);
                    b[r] = (uint8_t*)malloc(n * es ? n * es : 1);
                    for (size_t q = 0; q < n * es; ++q) a[r][q] = b[r][q] = rand();
                }
                if (bits == 8) {
                    nfec::host_gf8_addmul_rows(a.data(), src, co.data(), stride, nr, n, isa);
                    for (uint32_t r = 0; r < nr; ++r) nfec_gf8_addmul_host(b[r], src, co[r * stride], n, isa);
                } else {
                    nfec::host_gf16_addmul_rows(reinterpret_cast<uint16_t* const*>(a.data()), (const uint16_t*)src,
                                                co.data(), stride, nr, n, isa);
                    for (uint32_t r = 0; r < nr; ++r) nfec_gf16_addmul_host(b[r], src, co[r * stride], n, isa);
                }
                for (uint32_t r = 0; r < nr; ++r) {
                    if (std::memcmp(a[r], b[r], n * es) != 0) {
                        std::printf("rows mismatch bits %d n %zu isa %d row %u\n", bits, n, isa, r);
                        return 1;
                    }
                    free(a[r]);
                    free(b[r]);
                }
                free(src);
            }
    // the MDP step against a byte-by-byte restatement
    for (size_t n = 0; n < 300; n += (n < 40 ? 1 : 7))
        for (int isa = 0; isa <= 2; ++isa) {
            const uint32_t m = 1 + rand() % 40;
            std::vector<uint8_t> g(m + 1);
            for (auto& v : g) v = rand();
            uint8_t* data = (uint8_t*)malloc(n ? n : 1);
            for (size_t q = 0; q < n; ++q) data[q] = rand();
            std::vector<uint8_t*> a(m);
            std::vector<std::vector<uint8_t>> b(m, std::vector<uint8_t>(n));
            for (uint32_t r = 0; r < m; ++r) {
                a[r] = (uint8_t*)malloc(n ? n : 1);
                for (size_t q = 0; q < n; ++q) a[r][q] = b[r][q] = rand();
            }
            nfec::host_mdp_step(a.data(), data, g.data(), m, n, isa);
            const nfec::Field& f = nfec::gf8();
            for (size_t q = 0; q < n; ++q) {
                const uint32_t sv = data[q] ^ b[0][q];
                for (uint32_t r = 0; r + 1 < m; ++r) b[r][q] = (uint8_t)(b[r + 1][q] ^ f.mul(g[m - 1 - r], sv));
                b[m - 1][q] = (uint8_t)f.mul(g[0], sv);
            }
            for (uint32_t r = 0; r < m; ++r) {
                if (n && std::memcmp(a[r], b[r].data(), n) != 0) {
                    std::printf("mdp step mismatch n %zu isa %d row %u\n", n, isa, r);
                    return 1;
                }
                free(a[r]);
            }
            free(data);
        }
    std::printf("asan driver done\n");
}
