// Host <-> device transfer rates on this GPU for the host-resident decode:
// DMA (hipMemcpyAsync from/to pinned memory) against kernels that read or write the pinned host
// buffer directly (zero-copy), for several grid sizes and loads in flight per lane.
//   hipcc --offload-arch=gfx950 -O3 -o zc_rate zc_rate.hip && ./zc_rate
#include <hip/hip_runtime.h>
#include <cstdint>
#include <chrono>
#include <cstdio>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int U>
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
            if (i < n16) v[j] = __builtin_nontemporal_load(src + i);
        }
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const uint64_t i = base + j * 64 + lane;
            if (i < n16) __builtin_nontemporal_store(v[j], dst + i);
        }
    }
}

// the host decode's access pattern: per block of 96 slots x 1400 B, copy `nsel` slots (the first
// nsel of every 3-slot group pattern when skip, else the first nsel), one wave per slot, W-byte
// lane accesses
template <typename T>
__global__ __launch_bounds__(256) void seg_k(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src,
                                            uint32_t nblocks, uint32_t skip)
{
    const uint32_t wave = (blockIdx.x * 256 + threadIdx.x) >> 6, nwaves = (gridDim.x * 256) >> 6;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t nw = 1400 / sizeof(T);
    for (uint32_t job = wave; job < nblocks * 64; job += nwaves) {
        const uint32_t b = job / 64, j = job % 64;
        const uint32_t slot = skip ? (j / 2) * 3 + (j & 1) : j;  // 64 of 96 slots
        const T* s8 = reinterpret_cast<const T*>(src + (uint64_t)b * 134400 + slot * 1400);
        T* d8 = reinterpret_cast<T*>(dst + (uint64_t)b * 134400 + slot * 1400);
        for (uint32_t i = lane; i < nw; i += 64) d8[i] = __builtin_nontemporal_load(s8 + i);
    }
}

static float timed(hipStream_t s, hipEvent_t e0, hipEvent_t e1, void (*fn)(void*), void* arg, int reps)
{
    fn(arg);
    (void)hipEventRecord(e0, s);
    for (int i = 0; i < reps; ++i) fn(arg);
    (void)hipEventRecord(e1, s);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms / reps;
}

struct K {
    u32x4 *dst;
    const u32x4* src;
    uint64_t n16;
    uint32_t grid;
    int unroll;
    hipStream_t s;
    void* hd;
    const void* hs;
    size_t bytes;
    hipMemcpyKind kind;
};

static void launch(void* p)
{
    K* k = (K*)p;
    if (k->unroll == 1) hipLaunchKernelGGL(copy_k<1>, dim3(k->grid), dim3(256), 0, k->s, k->dst, k->src, k->n16);
    else if (k->unroll == 2) hipLaunchKernelGGL(copy_k<2>, dim3(k->grid), dim3(256), 0, k->s, k->dst, k->src, k->n16);
    else hipLaunchKernelGGL(copy_k<4>, dim3(k->grid), dim3(256), 0, k->s, k->dst, k->src, k->n16);
}

static void dma(void* p)
{
    K* k = (K*)p;
    (void)hipMemcpyAsync(k->hd, k->hs, k->bytes, k->kind, k->s);
}

int main()
{
    const size_t bytes = 1ull << 30;
    void *h, *d;
    if (hipHostMalloc(&h, bytes, hipHostMallocDefault) != hipSuccess || hipMalloc(&d, bytes) != hipSuccess) return 1;
    for (size_t i = 0; i < bytes; i += 4096) ((char*)h)[i] = 1;
    hipPointerAttribute_t at;
    if (hipPointerGetAttributes(&at, h) != hipSuccess) return 2;
    printf("{\"host_ptr\": \"%p\", \"device_ptr\": \"%p\", \"type\": %d}\n", h, at.devicePointer, (int)at.type);
    hipStream_t s;
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    K k{};
    k.s = s;
    k.bytes = bytes;
    k.hd = d;
    k.hs = h;
    k.kind = hipMemcpyHostToDevice;
    float ms = timed(s, e0, e1, dma, &k, 5);
    printf("{\"what\": \"dma_h2d\", \"ms\": %.3f, \"GBps\": %.1f}\n", ms, bytes / (ms * 1e-3) / 1e9);
    k.hd = h;
    k.hs = d;
    k.kind = hipMemcpyDeviceToHost;
    ms = timed(s, e0, e1, dma, &k, 5);
    printf("{\"what\": \"dma_d2h\", \"ms\": %.3f, \"GBps\": %.1f}\n", ms, bytes / (ms * 1e-3) / 1e9);
    u32x4* hdev = (u32x4*)at.devicePointer;
    k.n16 = bytes / 16;
    for (int u : {1, 2, 4})
        for (uint32_t grid : {256u, 1024u, 4096u}) {
            k.unroll = u;
            k.grid = grid;
            k.dst = (u32x4*)d;
            k.src = hdev;
            ms = timed(s, e0, e1, launch, &k, 3);
            printf("{\"what\": \"zc_read\", \"unroll\": %d, \"grid\": %u, \"ms\": %.3f, \"GBps\": %.1f}\n", u, grid, ms,
                   bytes / (ms * 1e-3) / 1e9);
            k.dst = hdev;
            k.src = (const u32x4*)d;
            ms = timed(s, e0, e1, launch, &k, 3);
            printf("{\"what\": \"zc_write\", \"unroll\": %d, \"grid\": %u, \"ms\": %.3f, \"GBps\": %.1f}\n", u, grid, ms,
                   bytes / (ms * 1e-3) / 1e9);
            fflush(stdout);
        }
    {
        const uint32_t nb = (uint32_t)(bytes / 134400);
        for (int skip : {0, 1})
            for (uint32_t grid : {256u, 1024u}) {
                for (int w : {8, 16}) {
                    (void)hipDeviceSynchronize();
                    (void)hipEventRecord(e0, s);
                    for (int r = 0; r < 3; ++r) {
                        if (w == 8)
                            hipLaunchKernelGGL(seg_k<uint64_t>, dim3(grid), dim3(256), 0, s, (uint8_t*)d, (const uint8_t*)hdev,
                                               nb, (uint32_t)skip);
                        else
                            hipLaunchKernelGGL(seg_k<u32x4>, dim3(grid), dim3(256), 0, s, (uint8_t*)d, (const uint8_t*)hdev,
                                               nb, (uint32_t)skip);
                    }
                    (void)hipEventRecord(e1, s);
                    (void)hipEventSynchronize(e1);
                    (void)hipEventElapsedTime(&ms, e0, e1);
                    ms /= 3;
                    printf("{\"what\": \"seg_read\", \"skip\": %d, \"grid\": %u, \"lane_bytes\": %d, \"ms\": %.3f, \"GBps\": %.1f}\n",
                           skip, grid, w, ms, (double)nb * 64 * 1400 / (ms * 1e-3) / 1e9);
                    fflush(stdout);
                }
            }
    }
    // both directions at once: DMA H2D on one stream while a zero-copy write kernel runs
    hipStream_t s2;
    (void)hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
    void* d2;
    if (hipMalloc(&d2, bytes) != hipSuccess) return 3;
    (void)hipDeviceSynchronize();
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < 3; ++i) (void)hipMemcpyAsync(d2, h, bytes / 2, hipMemcpyHostToDevice, s);
    for (int i = 0; i < 3; ++i)
        hipLaunchKernelGGL(copy_k<2>, dim3(1024), dim3(256), 0, s2, (u32x4*)((char*)hdev + bytes / 2), (const u32x4*)d,
                           bytes / 2 / 16);
    (void)hipDeviceSynchronize();
    ms = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
    printf("{\"what\": \"dma_h2d_with_zc_write\", \"ms\": %.3f, \"GBps_total\": %.1f}\n", ms, 3.0 * bytes / (ms * 1e-3) / 1e9);
    return 0;
}
