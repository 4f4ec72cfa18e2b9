// kernels_crc.hip -- per-segment CRC-32 of a block batch and the erasure lists it implies.
//
// npc (the reference's offline precoder) closes every output segment with a big-endian
// CRC-32 of its data part and, on decode, treats a segment whose CRC does not match as an
// erasure (src/common/normPrecode.cpp:780-783 encode, :1039-1050 and :1077-1089 decode).  The
// CRC is the reflected 0x04C11DB7 code with init and final XOR 0xFFFFFFFF
// (ComputeCRC32 / CRC32_TABLE, normPrecode.cpp:1236-1313).
//
// One lane per segment: a segment is a dependent chain, and a batch holds far more segments
// than the chip has lanes.  The slice-by-4 tables (4 KiB) are built in LDS by each workgroup;
// the data comes in 8-byte loads (segment strides are 8-byte multiples).
#include "nfec_internal.hpp"

namespace nfec {

namespace {

constexpr int kCrcThreads = 256;
constexpr uint32_t kPolyRev = 0xEDB88320u;

__device__ __forceinline__ uint32_t crc_word(const uint32_t* t, uint32_t crc, uint32_t w)
{
    crc ^= w;
    return t[768 + (crc & 0xff)] ^ t[512 + ((crc >> 8) & 0xff)] ^ t[256 + ((crc >> 16) & 0xff)] ^ t[crc >> 24];
}

__global__ __launch_bounds__(kCrcThreads) void crc32_slots_kernel(CrcArgs a)
{
    __shared__ uint32_t tab[1024];  // tab[j*256 + i]: byte i followed by j zero bytes
    for (uint32_t i = threadIdx.x; i < 256; i += kCrcThreads) {
        uint32_t c = i;
        for (int s = 0; s < 8; ++s) c = (c >> 1) ^ ((c & 1) ? kPolyRev : 0u);
        tab[i] = c;
    }
    __syncthreads();
    for (int j = 1; j < 4; ++j) {
        for (uint32_t i = threadIdx.x; i < 256; i += kCrcThreads) {
            const uint32_t p = tab[(j - 1) * 256 + i];
            tab[j * 256 + i] = (p >> 8) ^ tab[p & 0xff];
        }
        __syncthreads();
    }

    const uint64_t idx = (uint64_t)blockIdx.x * kCrcThreads + threadIdx.x;
    if (idx >= (uint64_t)a.nblocks * a.slots) return;
    const uint32_t b = (uint32_t)(idx / a.slots), s = (uint32_t)(idx % a.slots);
    const uint8_t* p = a.base + (uint64_t)b * a.block_stride + (uint64_t)s * a.seg_stride;
    uint32_t crc = 0xffffffffu;
    uint32_t i = 0;
    for (; i + 8 <= a.len; i += 8) {
        const uint2 v = *reinterpret_cast<const uint2*>(p + i);
        crc = crc_word(tab, crc, v.x);
        crc = crc_word(tab, crc, v.y);
    }
    for (; i < a.len; ++i) crc = tab[(crc ^ p[i]) & 0xff] ^ (crc >> 8);
    crc ^= 0xffffffffu;
    if (a.crc) a.crc[idx] = crc;
    if (a.bad) {
        // the stored CRC follows the data, big-endian (htonl, normPrecode.cpp:781-782)
        const uint32_t stored = ((uint32_t)p[a.len] << 24) | ((uint32_t)p[a.len + 1] << 16) |
                                ((uint32_t)p[a.len + 2] << 8) | p[a.len + 3];
        a.bad[idx] = stored != crc;
    }
}

// One wave per block: the block's bad slots among its first num_data + m, in ascending
// order (the order npc appends them, normPrecode.cpp:1077-1083), compacted with a ballot.
// counts[b] is the full count (it may exceed the list stride: the caller rejects that block).
__global__ __launch_bounds__(64) void erasure_list_kernel(ErasureListArgs a)
{
    const uint32_t b = blockIdx.x;
    const uint32_t lane = threadIdx.x;
    const uint32_t nd = a.num_data ? a.num_data[b] : a.k;
    const uint32_t n = nd + a.m;
    const uint8_t* bad = a.bad + (uint64_t)b * a.slots;
    uint16_t* locs = a.locs + (uint64_t)b * a.stride;
    uint32_t count = 0;
    for (uint32_t s0 = 0; s0 < n; s0 += 64) {
        const uint32_t s = s0 + lane;
        const bool e = s < n && bad[s];
        const uint64_t mask = __ballot(e);
        const uint32_t before = __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                                          __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
        if (e && count + before < a.stride) locs[count + before] = (uint16_t)s;
        count += (uint32_t)__popcll(mask);
    }
    if (lane == 0) a.counts[b] = count > 0xffffu ? 0xffffu : (uint16_t)count;
}

}  // namespace

int launch_crc32_slots(const CrcArgs& a, hipStream_t s)
{
    const uint64_t n = (uint64_t)a.nblocks * a.slots;
    if (n == 0) return NFEC_OK;
    const uint64_t grid = (n + kCrcThreads - 1) / kCrcThreads;
    if (grid > 0x7fffffffu) return fail(NFEC_EINVAL, "crc32: batch too large");
    hipLaunchKernelGGL(crc32_slots_kernel, dim3((uint32_t)grid), dim3(kCrcThreads), 0, s, a);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? NFEC_OK : hip_fail(e, "crc32 launch");
}

int launch_erasure_list(const ErasureListArgs& a, hipStream_t s)
{
    if (a.nblocks == 0) return NFEC_OK;
    hipLaunchKernelGGL(erasure_list_kernel, dim3(a.nblocks), dim3(64), 0, s, a);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? NFEC_OK : hip_fail(e, "erasure list launch");
}

}  // namespace nfec
