// Streaming-width microbenchmark for the RS8 encode's memory pattern: per 2 KiB chunk of a
// column, read 64 source columns and write 32 parity columns (2:1 bytes), either as 8-byte
// (dwordx2) or 16-byte (dwordx4) accesses per lane.  No arithmetic beyond an XOR that keeps
// the loads live.  Prints ms per pass and TB/s for each width.
//   hipcc --offload-arch=gfx950 -O3 -o ldst_width ldst_width.hip && ./ldst_width
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int K = 64, M = 32;
constexpr uint64_t CHUNK = 2048;  // bytes per column handled by one wave

template <int W>  // W = 8 or 16 bytes per lane per access
__global__ __launch_bounds__(256) void stream(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                              uint64_t chunks)
{
    const uint64_t wave = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63;
    if (wave >= chunks) return;
    constexpr int PER = CHUNK / (64 * W);  // accesses per lane per column
    using T = typename std::conditional<W == 8, uint2, uint4>::type;
    T acc[PER];
#pragma unroll
    for (int i = 0; i < PER; ++i) acc[i] = T{};
    const uint8_t* s = src + wave * CHUNK;
    for (int c = 0; c < K; ++c) {
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const T v = *reinterpret_cast<const T*>(s + (uint64_t)c * chunks * CHUNK + (uint64_t)(i * 64 + lane) * W);
            acc[i].x ^= v.x;
            acc[i].y ^= v.y;
            if constexpr (W == 16) {
                acc[i].z ^= v.z;
                acc[i].w ^= v.w;
            }
        }
    }
    uint8_t* d = dst + wave * CHUNK;
    for (int r = 0; r < M; ++r) {
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            T v = acc[i];
            v.x += r;
            *reinterpret_cast<T*>(d + (uint64_t)r * chunks * CHUNK + (uint64_t)(i * 64 + lane) * W) = v;
        }
    }
}

int main()
{
    const uint64_t chunks = 65536ull * 1400 / CHUNK;  // the headline batch: 65,536 blocks x 1400 B per column
    uint8_t *src, *dst;
    hipMalloc(&src, K * chunks * CHUNK);
    hipMalloc(&dst, M * chunks * CHUNK);
    hipMemset(src, 1, K * chunks * CHUNK);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const double bytes = (double)(K + M) * chunks * CHUNK;
    for (int rep = 0; rep < 2; ++rep) {
        for (int w : {8, 16}) {
            const dim3 grid((unsigned)((chunks + 3) / 4)), block(256);
            auto launch = [&] {
                if (w == 8) hipLaunchKernelGGL(stream<8>, grid, block, 0, 0, src, dst, chunks);
                else hipLaunchKernelGGL(stream<16>, grid, block, 0, 0, src, dst, chunks);
            };
            launch();
            hipEventRecord(e0);
            for (int i = 0; i < 10; ++i) launch();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            ms /= 10;
            printf("{\"width_bytes\": %d, \"ms\": %.4f, \"TBps\": %.3f}\n", w, ms, bytes / (ms * 1e-3) / 1e12);
        }
    }
    return 0;
}
