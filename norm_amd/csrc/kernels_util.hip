// kernels_util.hip -- synthetic-workload and receiver helpers (device side).
//
// fill:      splitmix64 counter streams per (block, slot), generated in
//            HBM so the bench never moves gigabytes over PCIe.
// erasures:  per-block partial Fisher-Yates over [0, range) with a sparse swap map,
//            identical to the oracle's full-array shuffle (orc_erasure_pattern).
// zero:      the receiver's zero-fill of erased segments before Decode
//            (reference src/common/normObject.cpp:1579).
#include <algorithm>

#include "nfec_internal.hpp"

namespace nfec {

namespace {

constexpr uint64_t kGamma = 0x9E3779B97F4A7C15ull;

__device__ __forceinline__ uint64_t mix64(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ void fill_kernel(uint8_t* base, uint64_t block_stride, uint32_t seg_stride, uint32_t nblocks,
                            const uint16_t* num_data, uint32_t k, uint32_t vec, uint64_t seed,
                            uint64_t first_block)
{
    const uint32_t words = (vec + 7) / 8;
    const uint64_t per_block = (uint64_t)k * words;
    const uint64_t total = per_block * nblocks;
    for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < total;
         g += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t b = (uint32_t)(g / per_block);
        const uint32_t rem = (uint32_t)(g % per_block);
        const uint32_t s = rem / words, w = rem % words;
        const uint32_t nd = num_data ? num_data[b] : k;
        if (s >= nd) continue;
        const uint64_t s0 = seed ^ ((first_block + b) << 20) ^ (uint64_t)s;
        const uint64_t v = mix64(s0 + (uint64_t)(w + 1) * kGamma);
        uint8_t* p = base + (uint64_t)b * block_stride + (uint64_t)s * seg_stride + (uint64_t)w * 8;
        const uint32_t nbytes = min(8u, vec - w * 8);
        if (nbytes == 8) {
            *reinterpret_cast<uint64_t*>(p) = v;
        } else {
            for (uint32_t i = 0; i < nbytes; ++i) p[i] = (uint8_t)(v >> (8 * i));
        }
    }
}

__global__ void erasure_kernel(uint16_t* locs, uint32_t stride, uint16_t* counts, uint32_t nblocks,
                               uint32_t range, uint32_t count, uint64_t seed, uint64_t first_block)
{
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nblocks) return;
    if (count > range) count = range;
    if (count > stride) count = stride;
    // sparse Fisher-Yates: only positions touched by swaps are recorded
    uint16_t pos[256], val[256];
    uint32_t n = 0;
    auto get = [&](uint32_t p) -> uint32_t {
        for (uint32_t i = 0; i < n; ++i)
            if (pos[i] == p) return val[i];
        return p;
    };
    auto set = [&](uint32_t p, uint32_t v) {
        for (uint32_t i = 0; i < n; ++i)
            if (pos[i] == p) { val[i] = (uint16_t)v; return; }
        pos[n] = (uint16_t)p;
        val[n] = (uint16_t)v;
        ++n;
    };
    const uint64_t s0 = seed ^ 0xE7A5E7A500000000ull ^ (first_block + b);
    uint16_t* out = locs + (uint64_t)b * stride;
    count = min(count, 128u);
    for (uint32_t i = 0; i < count; ++i) {
        const uint64_t r = mix64(s0 + (uint64_t)(i + 1) * kGamma);
        const uint32_t j = i + (uint32_t)(r % (uint64_t)(range - i));
        const uint32_t vi = get(i), vj = get(j);
        set(i, vj);
        set(j, vi);
        out[i] = (uint16_t)vj;
    }
    for (uint32_t i = 1; i < count; ++i) {
        const uint16_t v = out[i];
        int32_t j = (int32_t)i - 1;
        while (j >= 0 && out[j] > v) { out[j + 1] = out[j]; --j; }
        out[j + 1] = v;
    }
    counts[b] = (uint16_t)count;
}

__global__ void zero_kernel(uint8_t* base, uint64_t block_stride, uint32_t seg_stride, uint32_t nblocks,
                            const uint16_t* locs, uint32_t stride, const uint16_t* counts, uint32_t vec)
{
    // one workgroup per (block, erasure index) pair
    const uint32_t b = blockIdx.x / stride;
    const uint32_t e = blockIdx.x % stride;
    if (b >= nblocks || e >= counts[b]) return;
    uint8_t* p = base + (uint64_t)b * block_stride + (uint64_t)locs[(uint64_t)b * stride + e] * seg_stride;
    for (uint32_t i = threadIdx.x; i * 8 < vec; i += blockDim.x) {
        if (i * 8 + 8 <= vec) *reinterpret_cast<uint64_t*>(p + i * 8) = 0;
        else
            for (uint32_t j = i * 8; j < vec; ++j) p[j] = 0;
    }
}

// slot moves of the host-resident decode (launch_slot_move): one workgroup per block.  The
// block's erasure list becomes an LDS bitmap; lane 0 of wave 0 finds the end of the parity
// range the decode reads; then each wave copies every fourth selected slot, 8 bytes per lane
// (slots are 8-byte aligned: NORM's segment pool rounds to 8, normSegment.cpp:25-27).
constexpr uint32_t kMoveMaxSlots = 65536;

__device__ void slot_move_block(const SlotMoveArgs& a, uint32_t b, uint32_t* erased, uint32_t& sh_end,
                                uint32_t& sh_bad, uint32_t& sh_es)
{
    const uint32_t nd_in = a.num_data ? a.num_data[b] : a.k;
    // an out-of-range numData marks the block bad and the slot range stays the block's own
    // k + m slots: the moves never reach past a block (nor the erased bitmap past its size)
    const bool nd_bad = nd_in == 0 || nd_in > a.k;
    const uint32_t nd = nd_bad ? a.k : nd_in;
    const uint32_t nvec = nd + a.m;
    const uint32_t words = (nvec + 31) / 32;
    for (uint32_t w = threadIdx.x; w < words; w += blockDim.x) erased[w] = 0;
    if (threadIdx.x == 0) {
        sh_bad = (nd_bad || a.counts[b] > a.lstride) ? 1u : 0u;
        sh_es = 0;
    }
    __syncthreads();
    const uint32_t ec = min((uint32_t)a.counts[b], a.lstride);
    const uint16_t* l = a.locs + (uint64_t)b * a.lstride;
    for (uint32_t i = threadIdx.x; i < ec; i += blockDim.x) {
        const uint32_t v = l[i];
        if (v >= nvec) {
            sh_bad = 1u;
            continue;
        }
        atomicOr(&erased[v / 32], 1u << (v % 32));
        if (v < nd) atomicAdd(&sh_es, 1u);
    }
    __syncthreads();
    const bool bad = sh_bad != 0;
    if (a.mode == SLOTS_OUT && (bad || !a.status || a.status[b] <= 0)) {
        __syncthreads();  // every thread leaves together: the LDS is reused by the next block
        return;
    }
    if (threadIdx.x == 0) {
        uint32_t end = nvec;
        if (!bad && a.mode == SLOTS_RS_IN) {
            // the first es surviving parities; fewer than es: undecodable, nothing is read,
            // and copying every surviving slot is harmless
            uint32_t used = 0;
            end = nd;
            for (uint32_t v = nd; v < nvec && used < sh_es; ++v)
                if (!((erased[v / 32] >> (v % 32)) & 1u)) {
                    ++used;
                    end = v + 1;
                }
            if (used < sh_es) end = nvec;
        }
        sh_end = end;
    }
    __syncthreads();
    const uint32_t end = a.mode == SLOTS_OUT ? nd : sh_end;
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint8_t* sb = a.src + (uint64_t)b * a.src_block_stride;
    uint8_t* db = a.dst + (uint64_t)b * a.dst_block_stride;
    const uint32_t nw = a.bytes / 8, tail = a.bytes - nw * 8;
    uint32_t pick = 0;  // selected slots seen so far: slot j goes to wave j % 4
    for (uint32_t v = 0; v < end; ++v) {
        const bool is_erased = (erased[v / 32] >> (v % 32)) & 1u;
        bool sel;
        if (bad) sel = a.mode != SLOTS_OUT;
        else if (a.mode == SLOTS_OUT) sel = is_erased;                        // v < nd here
        else if (v < nd) sel = !is_erased || (a.accumulate && a.mode == SLOTS_RS_IN);
        else sel = !is_erased;
        if (!sel) continue;
        if ((pick++ & 3u) != wave) continue;
        const uint64_t* s8 = reinterpret_cast<const uint64_t*>(sb + (uint64_t)v * a.src_seg_stride);
        uint64_t* d8 = reinterpret_cast<uint64_t*>(db + (uint64_t)v * a.dst_seg_stride);
        for (uint32_t i = lane; i < nw; i += 64) d8[i] = __builtin_nontemporal_load(s8 + i);
        if (lane < tail) {
            const uint8_t* s1 = sb + (uint64_t)v * a.src_seg_stride + nw * 8;
            uint8_t* d1 = db + (uint64_t)v * a.dst_seg_stride + nw * 8;
            d1[lane] = s1[lane];
        }
    }
    __syncthreads();
}

// A few hundred workgroups loop over the blocks: the copies are PCIe-bound (one workgroup per
// CU already reaches the link's 55-57 GB/s, tools/diag/zc_rate.hip), and a grid of one
// workgroup per block filled every CU with waves parked on PCIe reads, starving the decode
// kernels of the other pipeline chunks (rs_plan2 1.5 ms instead of 0.07 per 2k blocks).
constexpr uint32_t kMoveGrid = 256;

__global__ __launch_bounds__(256) void slot_move_kernel(SlotMoveArgs a)
{
    __shared__ uint32_t erased[kMoveMaxSlots / 32];
    __shared__ uint32_t sh_end, sh_bad, sh_es;
    for (uint32_t b = blockIdx.x; b < a.nblocks; b += gridDim.x) slot_move_block(a, b, erased, sh_end, sh_bad, sh_es);
}

// streaming copy for the bench's achievable-HBM figure: 16 bytes per lane, four loads in
// flight per lane before the stores, grid-stride over 4 KiB per wave
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void stream_copy_kernel(u32x4* __restrict__ dst, const u32x4* __restrict__ src,
                                                          uint64_t n16)
{
    const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    const uint32_t lane = threadIdx.x & 63;
    for (uint64_t base = wave * 256; base < n16; base += nwaves * 256) {
        u32x4 v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint64_t i = base + j * 64 + lane;
            if (i < n16) v[j] = __builtin_nontemporal_load(src + i);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint64_t i = base + j * 64 + lane;
            if (i < n16) __builtin_nontemporal_store(v[j], dst + i);
        }
    }
}

}  // namespace

int launch_stream_copy(void* dst, const void* src, uint64_t bytes, hipStream_t s)
{
    if (bytes == 0) return NFEC_OK;
    if ((reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src) | bytes) & 15)
        return fail(NFEC_EINVAL, "stream_copy: pointers and size must be multiples of 16 bytes");
    const uint64_t n16 = bytes / 16;
    // one 4 KiB piece per wave, no grid-stride loop: 6.29 TB/s on a 4 GiB copy, against
    // 5.5-5.8 TB/s with 1-16 K resident workgroups looping (tools/diag/copy_rate.hip,
    // profiles/r02/copy_rate.jsonl)
    if ((n16 + 1023) / 1024 >= (1ull << 31)) return fail(NFEC_EINVAL, "stream_copy: size too large");
    const uint32_t grid = (uint32_t)((n16 + 1023) / 1024);
    hipLaunchKernelGGL(stream_copy_kernel, dim3(grid), dim3(256), 0, s, static_cast<u32x4*>(dst),
                       static_cast<const u32x4*>(src), n16);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? NFEC_OK : hip_fail(e, "stream_copy launch");
}

int launch_fill(uint8_t* base, uint64_t block_stride, uint32_t seg_stride, uint32_t nblocks,
                const uint16_t* num_data, uint32_t k, uint32_t vec, uint64_t seed, uint64_t first_block,
                hipStream_t s)
{
    if (nblocks == 0 || vec == 0) return NFEC_OK;
    const uint64_t total = (uint64_t)nblocks * k * ((vec + 7) / 8);
    const uint32_t grid = (uint32_t)std::min<uint64_t>((total + 255) / 256, 65536);
    hipLaunchKernelGGL(fill_kernel, dim3(grid), dim3(256), 0, s, base, block_stride, seg_stride, nblocks,
                       num_data, k, vec, seed, first_block);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? NFEC_OK : hip_fail(e, "fill launch");
}

int launch_erasures(uint16_t* locs, uint32_t stride, uint16_t* counts, uint32_t nblocks, uint32_t range,
                    uint32_t count, uint64_t seed, uint64_t first_block, hipStream_t s)
{
    if (nblocks == 0) return NFEC_OK;
    if (count > 128) return fail(NFEC_EINVAL, "erasure generator supports at most 128 erasures per block");
    hipLaunchKernelGGL(erasure_kernel, dim3((nblocks + 63) / 64), dim3(64), 0, s, locs, stride, counts, nblocks,
                       range, count, seed, first_block);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? NFEC_OK : hip_fail(e, "erasure launch");
}

int launch_slot_move(const SlotMoveArgs& a, hipStream_t s)
{
    if (a.nblocks == 0) return NFEC_OK;
    if ((uint64_t)a.k + a.m > kMoveMaxSlots) return fail(NFEC_ENOTSUP, "slot_move: more than 65536 slots");
    if (!a.src || !a.dst || !a.locs || !a.counts || a.lstride == 0) return fail(NFEC_EINVAL, "slot_move: bad arguments");
    if ((reinterpret_cast<uintptr_t>(a.src) | reinterpret_cast<uintptr_t>(a.dst) | a.src_block_stride |
         a.dst_block_stride | a.src_seg_stride | a.dst_seg_stride) & 7)
        return fail(NFEC_EINVAL, "slot_move: slots must be 8-byte aligned");
    static const uint32_t g = (uint32_t)diag_knob("NFEC_MOVE_GRID", kMoveGrid, 1, 4096);
    static const uint32_t go = (uint32_t)diag_knob("NFEC_MOVE_GRID_OUT", kMoveGrid, 1, 4096);
    hipLaunchKernelGGL(slot_move_kernel, dim3(std::min(a.nblocks, a.mode == SLOTS_OUT ? go : g)), dim3(256), 0, s, a);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? NFEC_OK : hip_fail(e, "slot_move launch");
}

int launch_zero_slots(uint8_t* base, uint64_t block_stride, uint32_t seg_stride, uint32_t nblocks,
                      const uint16_t* locs, uint32_t stride, const uint16_t* counts, uint32_t vec,
                      hipStream_t s)
{
    if (nblocks == 0 || stride == 0) return NFEC_OK;
    const uint64_t groups = (uint64_t)nblocks * stride;
    if (groups >= (1ull << 31)) return fail(NFEC_EINVAL, "zero_slots: too many blocks");
    hipLaunchKernelGGL(zero_kernel, dim3((uint32_t)groups), dim3(64), 0, s, base, block_stride, seg_stride, nblocks,
                       locs, stride, counts, vec);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? NFEC_OK : hip_fail(e, "zero launch");
}

}  // namespace nfec
