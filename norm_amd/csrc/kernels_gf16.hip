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

// exp-table byte offset of (doubled) log a + log b: the sum mod 2q, or the zero entry when
// either operand is the zero sentinel.  lcm = a - 2q (wraps for a < 2q), so one v_min3.
__device__ __forceinline__ uint32_t eidx(uint32_t lc, uint32_t lcm, uint32_t l)
{
    return min(min(lc + l, lcm + l), kQ2);  // v_min3_u32
}

// One wave per block.  NI dwords (2 symbols) per lane per item group, RC output rows per
// pass, accumulators packed (low symbol | high symbol << 16).  Per source column the wave
//  - already holds the column's data and its doubled logs (computed one column earlier),
//  - holds the column's RC coefficient logs distributed over lanes 0..RC-1 (also one column
//    earlier), read back with v_readlane into SGPRs,
//  - issues the next column's data load, its log gathers and its coefficient logs,
//  - and does RC x NI x 2 exp lookups in LDS.
// No dependent global load sits on the per-row path.
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
            uint32_t acc[RC][NI];
#pragma unroll
            for (int r = 0; r < RC; ++r)
#pragma unroll
                for (int j = 0; j < NI; ++j) acc[r][j] = 0;

            // column c's inputs: data x, its logs (l0 low, l1 high), coefficient logs (lane r)
            auto col_data = [&](uint32_t c, uint32_t (&x)[NI]) {
                const uint32_t slot = islots ? uni(islots[c]) : c;
                const uint8_t* src = in_blk + (uint64_t)slot * a.in_seg_stride;
#pragma unroll
                for (int j = 0; j < NI; ++j)
                    x[j] = valid[j] ? *reinterpret_cast<const uint32_t*>(src + dw[j] * 4u) : 0u;
            };
            auto col_clog = [&](uint32_t c) -> uint32_t {
                const int32_t r = r0 + (int32_t)lane;
                const uint32_t cv = (lane < (uint32_t)RC && r < rows)
                                        ? (uint32_t)coef_blk[(uint64_t)c * a.coef_col_stride + r] : 0u;
                return dlog(a.log_tab, cv);
            };
            uint32_t x[NI], l0[NI], l1[NI];
            uint32_t clog = 0;
            if (cols > 0) {
                col_data(0, x);
                clog = col_clog(0);
#pragma unroll
                for (int j = 0; j < NI; ++j) {
                    l0[j] = dlog(a.log_tab, x[j] & 0xffffu);
                    l1[j] = dlog(a.log_tab, x[j] >> 16);
                }
            }
            for (uint32_t c = 0; c < cols; ++c) {
                // next column's loads and gathers first, then this column's lookups
                uint32_t xn[NI], clogn = 0;
                const uint32_t cn = min(c + 1, cols - 1);
                col_data(cn, xn);
                clogn = col_clog(cn);
#pragma unroll
                for (int r = 0; r < RC; ++r) {
                    const uint32_t lc = (uint32_t)__builtin_amdgcn_readlane((int)clog, r);
                    const uint32_t lcm = lc - kQ2;
#pragma unroll
                    for (int j = 0; j < NI; ++j) {
                        const uint32_t lo = *reinterpret_cast<const uint16_t*>(lds_bytes + eidx(lc, lcm, l0[j]));
                        const uint32_t hi = *reinterpret_cast<const uint16_t*>(lds_bytes + eidx(lc, lcm, l1[j]));
                        acc[r][j] ^= lo | (hi << 16);
                    }
                }
#pragma unroll
                for (int j = 0; j < NI; ++j) {
                    l0[j] = dlog(a.log_tab, xn[j] & 0xffffu);
                    l1[j] = dlog(a.log_tab, xn[j] >> 16);
                }
                clog = clogn;
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
                    uint32_t v = acc[r][j];
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
    const uint32_t groups = (a.nblocks + kWaves - 1) / kWaves;
    const size_t lds = 65536 * sizeof(uint16_t);
    // one dword (2 symbols) per lane per item group, 32 rows per pass: the LDS lookups are
    // the same for any split, the log gathers scale with the number of row passes
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&gf16_matmul_kernel<1, 32>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        attr = true;
    }
    hipError_t e;
    hipLaunchKernelGGL((gf16_matmul_kernel<1, 32>), dim3(groups), dim3(kThreads), lds, s, a);
    e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "gf16_matmul launch");
    return NFEC_OK;
}

}  // namespace nfec
