// Memory-depth microbenchmark for the RS8 encode's HBM stream, in the real block layout:
// 65,536 blocks of (64 + 32) segments x 1400 B, contiguous; items of 8 bytes flat over the
// batch (175 per segment), 256 items per wave (4 per lane, 64 items apart).  Each wave reads its
// items' 64 source columns with D columns in flight and writes 32 parity columns; no arithmetic
// beyond XORs that keep the loads live.  Occupancy is capped with dynamic LDS (WPC = waves per
// CU).  Prints ms and TB/s of algorithmic bytes per (D, WPC).  The q4 encode corresponds to
// D = 2 at WPC = 16.
//   hipcc --offload-arch=gfx950 -O3 -o stream_depth stream_depth.hip && ./stream_depth
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

constexpr int K = 64, M = 32, VEC = 1400, IPS = VEC / 8;  // items per segment
constexpr uint64_t NB = 65536, BSTRIDE = (uint64_t)(K + M) * VEC;

template <int D>
__global__ __launch_bounds__(64) void stream(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, uint64_t items)
{
    extern __shared__ uint8_t cap[];  // occupancy cap only
    const uint32_t lane = threadIdx.x;
    const uint64_t base = (uint64_t)blockIdx.x * 256;
    uint64_t off[4];
    bool live[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint64_t it = base + j * 64 + lane;
        live[j] = it < items;
        off[j] = live[j] ? (it / IPS) * BSTRIDE + (it % IPS) * 8 : 0;
    }
    uint2 acc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = uint2{0, 0};
    for (int c = 0; c < K; c += D) {
        uint2 v[D][4];
#pragma unroll
        for (int d = 0; d < D; ++d)
#pragma unroll
            for (int j = 0; j < 4; ++j) v[d][j] = *reinterpret_cast<const uint2*>(src + off[j] + (uint64_t)(c + d) * VEC);
#pragma unroll
        for (int d = 0; d < D; ++d)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                acc[j].x ^= v[d][j].x;
                acc[j].y ^= v[d][j].y;
            }
    }
    if (lane == 1000) cap[0] = 0;
#pragma unroll 4
    for (int r = 0; r < M; ++r)
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (live[j]) {
                uint2 w = acc[j];
                w.x += r;
                *reinterpret_cast<uint2*>(dst + off[j] + (uint64_t)(K + r) * VEC) = w;
            }
}

int main()
{
    const uint64_t items = NB * IPS;
    uint8_t* buf;
    hipMalloc(&buf, NB * BSTRIDE);
    hipMemset(buf, 1, NB * BSTRIDE);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const double bytes = (double)(K + M) * VEC * NB;
    const unsigned grid = (unsigned)((items + 255) / 256);
    for (int wpc : {8, 16, 32}) {
        const size_t lds = 160 * 1024 / wpc;
        for (int d : {1, 2, 4, 8, 16}) {
            auto launch = [&] {
                switch (d) {
                case 1: hipLaunchKernelGGL(stream<1>, dim3(grid), dim3(64), lds, 0, buf, buf, items); break;
                case 2: hipLaunchKernelGGL(stream<2>, dim3(grid), dim3(64), lds, 0, buf, buf, items); break;
                case 4: hipLaunchKernelGGL(stream<4>, dim3(grid), dim3(64), lds, 0, buf, buf, items); break;
                case 8: hipLaunchKernelGGL(stream<8>, dim3(grid), dim3(64), lds, 0, buf, buf, items); break;
                default: hipLaunchKernelGGL(stream<16>, dim3(grid), dim3(64), lds, 0, buf, buf, items); break;
                }
            };
            launch();
            hipEventRecord(e0);
            for (int i = 0; i < 10; ++i) launch();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            ms /= 10;
            printf("{\"waves_per_cu\": %d, \"cols_in_flight\": %d, \"ms\": %.4f, \"TBps\": %.3f}\n", wpc, d, ms,
                   bytes / (ms * 1e-3) / 1e12);
            fflush(stdout);
        }
    }
    return 0;
}
