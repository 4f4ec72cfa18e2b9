// Achievable device-to-device copy rate on this GPU: 16-byte-per-lane copy kernels over 4 GiB
// with and without non-temporal hints, for several grid sizes and loads in flight per lane.
// Picks the form nfec_util_stream_copy uses for bench.py's achievable_copy figure.
//   hipcc --offload-arch=gfx950 -O3 -o copy_rate copy_rate.hip && ./copy_rate
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int U, bool NT>
__global__ __launch_bounds__(256) void copy_k(u32x4* __restrict__ dst, const u32x4* __restrict__ src, uint64_t n16)
{
    const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    const uint32_t lane = threadIdx.x & 63;
    for (uint64_t base = wave * 64 * U; base < n16; base += nwaves * 64 * U) {
        u32x4 v[U];
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const uint64_t i = base + j * 64 + lane;
            if (i < n16) v[j] = NT ? __builtin_nontemporal_load(src + i) : src[i];
        }
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const uint64_t i = base + j * 64 + lane;
            if (i < n16) {
                if (NT) __builtin_nontemporal_store(v[j], dst + i);
                else dst[i] = v[j];
            }
        }
    }
}

template <int U, bool NT>
void run(u32x4* d, const u32x4* s, uint64_t n16, uint32_t grid, hipEvent_t e0, hipEvent_t e1)
{
    hipLaunchKernelGGL((copy_k<U, NT>), dim3(grid), dim3(256), 0, 0, d, s, n16);
    hipEventRecord(e0);
    for (int i = 0; i < 5; ++i) hipLaunchKernelGGL((copy_k<U, NT>), dim3(grid), dim3(256), 0, 0, d, s, n16);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    ms /= 5;
    printf("{\"unroll\": %d, \"nt\": %d, \"grid\": %u, \"ms\": %.4f, \"TBps\": %.3f}\n", U, (int)NT, grid, ms,
           2.0 * n16 * 16 / (ms * 1e-3) / 1e12);
    fflush(stdout);
}

int main()
{
    const uint64_t bytes = 1ull << 32, n16 = bytes / 16;
    u32x4 *s, *d;
    if (hipMalloc(&s, bytes) != hipSuccess || hipMalloc(&d, bytes) != hipSuccess) return 1;
    (void)hipMemset(s, 1, bytes);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (uint32_t grid : {1024u, 2048u, 4096u, 16384u, (uint32_t)(n16 / 1024)}) {
        run<4, true>(d, s, n16, grid, e0, e1);
        run<4, false>(d, s, n16, grid, e0, e1);
        run<1, false>(d, s, n16, grid, e0, e1);
        run<8, false>(d, s, n16, grid, e0, e1);
    }
    return 0;
}
