// kernels_gf16.hip -- batched GF(2^16) segment-matrix product (RS16) for gfx950.
//
// Same contract as the GF(2^8) kernel but over native-endian 16-bit symbols, the unit of
// the reference RS16 codec (addmul1 with GF_ADDMULC, src/common/normEncoderRS16.cpp:
// 158-161, 261-298; vector_size/2 symbols, :479).  Multiplication is exp[log c + log x]:
// the 65,535-entry exp table (128 KiB) is staged in LDS, the data logs come from a
// 128 KiB log table that stays L2-resident and are computed once per (column, symbol)
// then reused for every output row.  Logs are stored doubled so the sum is directly a
// byte offset; a zero symbol maps to a sentinel that v_min3 clamps onto a zero entry.
#include "nfec_internal.hpp"

namespace nfec {

namespace {

constexpr int kWave = 64;
constexpr int kWaves = 16;
constexpr int kThreads = kWave * kWaves;
constexpr uint32_t kQ2 = 2u * 65535u;      // doubled field order (byte offset period)
constexpr uint32_t kZeroLog = 0x40000u;    // doubled-log sentinel for a zero symbol

__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

__device__ __forceinline__ uint32_t dlog(const uint16_t* __restrict__ log_tab, uint32_t x)
{
    return x ? 2u * (uint32_t)log_tab[x] : kZeroLog;
}

// one wave per block; NI dwords (2 symbols each) per lane per group; RC rows per pass
template <int NI, int RC>
__global__ __launch_bounds__(kThreads) void gf16_matmul_kernel(Gf16MatmulArgs a)
{
    extern __shared__ uint8_t lds_raw[];
    uint16_t* exp_lds = reinterpret_cast<uint16_t*>(lds_raw);
    for (uint32_t i = threadIdx.x; i < 65536u; i += kThreads) exp_lds[i] = i < 65535u ? a.exp_tab[i] : 0;
    __syncthreads();
    const uint8_t* lds_bytes = reinterpret_cast<const uint8_t*>(exp_lds);

    const uint32_t lane = threadIdx.x & (kWave - 1);
    const uint32_t b = uni(blockIdx.x * kWaves + (threadIdx.x >> 6));
    if (b >= a.nblocks) return;
    const int32_t rows = a.row_count ? (int32_t)uni((uint32_t)a.row_count[b]) : (int32_t)a.rows_const;
    if (rows <= 0) return;
    const uint32_t cols = a.in_count ? uni(a.in_count[b]) : a.cols_const;
    const uint32_t dws = (a.vec_bytes + 3) >> 2;  // dwords per segment (2 symbols each)
    const uint32_t ngroups = (dws + NI * kWave - 1) / (NI * kWave);
    const uint16_t* islots = a.in_slots ? a.in_slots + (uint64_t)b * a.slots_stride : nullptr;
    const uint16_t* oslots = a.out_slots ? a.out_slots + (uint64_t)b * a.slots_stride : nullptr;
    const uint16_t* coef_blk = a.coef + (uint64_t)(a.coef_by_count ? (cols ? cols - 1 : 0) : b) * a.coef_block_stride;
    const uint8_t* in_blk = a.in_base + (uint64_t)b * a.in_block_stride;
    uint8_t* out_blk = a.out_base + (uint64_t)b * a.out_block_stride;

    for (uint32_t grp = 0; grp < ngroups; ++grp) {
        uint32_t dw[NI];
        bool valid[NI];
#pragma unroll
        for (int j = 0; j < NI; ++j) {
            dw[j] = (grp * NI + j) * kWave + lane;
            valid[j] = dw[j] < dws;
        }
        for (int32_t r0 = 0; r0 < rows; r0 += RC) {
            uint32_t acc_lo[RC][NI], acc_hi[RC][NI];
#pragma unroll
            for (int r = 0; r < RC; ++r)
#pragma unroll
                for (int j = 0; j < NI; ++j) acc_lo[r][j] = acc_hi[r][j] = 0;
            for (uint32_t c = 0; c < cols; ++c) {
                const uint32_t slot = islots ? uni(islots[c]) : c;
                uint32_t l0[NI], l1[NI];
#pragma unroll
                for (int j = 0; j < NI; ++j) {
                    uint32_t x = 0;
                    if (valid[j]) x = *reinterpret_cast<const uint32_t*>(in_blk + (uint64_t)slot * a.in_seg_stride + dw[j] * 4u);
                    l0[j] = dlog(a.log_tab, x & 0xffffu);
                    l1[j] = dlog(a.log_tab, x >> 16);
                }
                const uint16_t* cc = coef_blk + (uint64_t)c * a.coef_col_stride + r0;
#pragma unroll
                for (int r = 0; r < RC; ++r) {
                    const uint32_t cv = (r0 + r < rows) ? uni(cc[r]) : 0u;
                    if (cv != 0) {
                        const uint32_t lc = 2u * (uint32_t)a.log_tab[cv];
                        const uint32_t lcm = lc - kQ2;
#pragma unroll
                        for (int j = 0; j < NI; ++j) {
                            const uint32_t i0 = min(min(lc + l0[j], lcm + l0[j]), kQ2);
                            const uint32_t i1 = min(min(lc + l1[j], lcm + l1[j]), kQ2);
                            acc_lo[r][j] ^= *reinterpret_cast<const uint16_t*>(lds_bytes + i0);
                            acc_hi[r][j] ^= *reinterpret_cast<const uint16_t*>(lds_bytes + i1);
                        }
                    }
                }
            }
#pragma unroll
            for (int r = 0; r < RC; ++r) {
                if (r0 + r >= rows) continue;
                uint32_t slot;
                if (a.out_slot_mode == OUT_SLOT_LIST) slot = oslots[r0 + r];
                else if (a.out_slot_mode == OUT_SLOT_AFTER_INPUT) slot = cols + r0 + r;
                else slot = r0 + r;
                uint8_t* o = out_blk + (uint64_t)slot * a.out_seg_stride;
#pragma unroll
                for (int j = 0; j < NI; ++j) {
                    if (!valid[j]) continue;
                    uint32_t v = acc_lo[r][j] | (acc_hi[r][j] << 16);
                    const uint32_t byte0 = dw[j] * 4u;
                    if (byte0 + 4u <= a.vec_bytes) {
                        uint32_t* p = reinterpret_cast<uint32_t*>(o + byte0);
                        if (a.accumulate) v ^= *p;
                        *p = v;
                    } else {
                        // last symbol of an odd symbol count: only the low 16 bits
                        uint16_t* p = reinterpret_cast<uint16_t*>(o + byte0);
                        uint16_t w = (uint16_t)v;
                        if (a.accumulate) w ^= *p;
                        *p = w;
                    }
                }
            }
        }
    }
}

}  // namespace

int launch_gf16_matmul(const Gf16MatmulArgs& a, hipStream_t s)
{
    if (a.nblocks == 0 || a.vec_bytes < 2) return NFEC_OK;
    if (a.vec_bytes & 1) return fail(NFEC_EINVAL, "gf16 matmul: odd byte count");
    const uint32_t dws = (a.vec_bytes + 3) / 4;
    const uint32_t groups = (a.nblocks + kWaves - 1) / kWaves;
    const size_t lds = 65536 * sizeof(uint16_t);
    hipError_t e;
    if (dws <= kWave) {
        static bool attr1 = false;
        if (!attr1) {
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&gf16_matmul_kernel<1, 16>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            attr1 = true;
        }
        hipLaunchKernelGGL((gf16_matmul_kernel<1, 16>), dim3(groups), dim3(kThreads), lds, s, a);
    } else {
        static bool attr2 = false;
        if (!attr2) {
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&gf16_matmul_kernel<2, 16>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            attr2 = true;
        }
        hipLaunchKernelGGL((gf16_matmul_kernel<2, 16>), dim3(groups), dim3(kThreads), lds, s, a);
    }
    e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "gf16_matmul launch");
    return NFEC_OK;
}

}  // namespace nfec
