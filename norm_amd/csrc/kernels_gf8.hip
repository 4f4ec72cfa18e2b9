// kernels_gf8.hip -- batched GF(2^8) segment-matrix product for gfx950 (MI355X).
//
// out[b][slot_out(r)] (^)= XOR_c coef[b][c][r] (x) in[b][slot_in(c)]   over vec bytes.
//
// This is the repair/parity loop of the reference (addmul1, src/common/normEncoderRS8.cpp:
// 262-299, called per (parity row, source column) by Encode :473-483 and Decode :727-756),
// restructured for CDNA4: a wavefront owns 64 x 8-byte items of segment columns, keeps
// RC output rows x 8 bytes per lane in VGPRs, streams each source column through once
// with coalesced 512-byte wave loads, and multiplies bytes by the column's constants with
// v_perm_b32 table lookups: a byte x = lo3 | mid3<<3 | hi2<<6 and, GF multiplication
// being GF(2)-linear,  c*x = c*lo3 ^ c*(mid3<<3) ^ c*(hi2<<6)  -- three 8-entry byte
// tables held in 5 dwords, so one v_perm_b32 performs four byte lookups.  Per (row,
// column, dword) that is 3 v_perm + ~1.5 v_bitop3/xor; the per-value tables (256 x 32 B)
// sit in LDS and are read with uniform (broadcast) ds_read_b128/_b32.
#include <cstdlib>

#include "nfec_internal.hpp"

namespace nfec {

namespace {

constexpr int kWave = 64;
constexpr int kWavesPerGroup = 4;
constexpr int kThreads = kWave * kWavesPerGroup;

__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

struct Sel {
    uint32_t s0, s1, s2;
};

__device__ __forceinline__ Sel selectors(uint32_t x)
{
    Sel s;
    s.s0 = x & 0x07070707u;
    s.s1 = (x >> 3) & 0x07070707u;
    s.s2 = (x >> 6) & 0x03030303u;
    return s;
}

__device__ __forceinline__ uint32_t gfmul4(const uint4& t, uint32_t t4, const Sel& s)
{
    const uint32_t a = __builtin_amdgcn_perm(t.y, t.x, s.s0);
    const uint32_t b = __builtin_amdgcn_perm(t.w, t.z, s.s1);
    const uint32_t c = __builtin_amdgcn_perm(t4, t4, s.s2);
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

__device__ __forceinline__ uint2 load8(const uint8_t* p) { return *reinterpret_cast<const uint2*>(p); }

__device__ __forceinline__ void store_bytes(uint8_t* p, uint2 v, uint32_t nbytes)
{
    if (nbytes >= 8) {
        *reinterpret_cast<uint2*>(p) = v;
    } else {
        for (uint32_t i = 0; i < nbytes; ++i) {
            const uint32_t w = i < 4 ? v.x : v.y;
            p[i] = (uint8_t)(w >> (8 * (i & 3)));
        }
    }
}

// NI items (8 bytes each) per lane, RC output rows per pass.
// FLAT: all blocks share one coefficient matrix and identity input slots; the wave's
//       items are consecutive in the flattened (block, item) space.
// !FLAT: one wave per block (per-block coefficients / slot lists, uniform per wave).
template <int NI, int RC, bool FLAT>
__global__ __launch_bounds__(kThreads) void gf8_matmul_kernel(Gf8MatmulArgs a)
{
    __shared__ uint4 lds_tab[256 * 2];  // 256 x 32 bytes
    // !FLAT: the wave's per-block coefficient matrix, staged once so the per-column
    // coefficient reads are LDS broadcasts instead of dependent global loads
    constexpr uint32_t kCoefLds = FLAT ? 1u : 1024u;  // dwords per wave
    __shared__ uint32_t lds_coef[kWavesPerGroup][kCoefLds];
    {
        const uint4* g = reinterpret_cast<const uint4*>(a.vtab);
        for (int i = threadIdx.x; i < 512; i += kThreads) lds_tab[i] = g[i];
    }
    __syncthreads();
    const uint32_t* tab32 = reinterpret_cast<const uint32_t*>(lds_tab);

    const uint32_t lane = threadIdx.x & (kWave - 1);
    const uint32_t wave = uni(blockIdx.x * kWavesPerGroup + (threadIdx.x >> 6));
    const uint32_t ips = (a.vec_bytes + 7) >> 3;  // 8-byte items per segment

    // ---- per-lane item geometry ----
    uint32_t blk[NI], item[NI];
    bool valid[NI];
    uint32_t ngroups = 1;
    uint32_t wblock = 0;
    if constexpr (FLAT) {
        const uint64_t total = (uint64_t)a.nblocks * ips;
#pragma unroll
        for (int j = 0; j < NI; ++j) {
            const uint64_t gi = ((uint64_t)wave * NI + j) * kWave + lane;
            valid[j] = gi < total;
            blk[j] = valid[j] ? (uint32_t)(gi / ips) : 0;
            item[j] = valid[j] ? (uint32_t)(gi % ips) : 0;
        }
    } else {
        wblock = wave;
        if (wblock >= a.nblocks) return;
        ngroups = (ips + NI * kWave - 1) / (NI * kWave);
    }

    int32_t rows = (int32_t)a.rows_const;
    uint32_t cols = a.cols_const;
    if constexpr (!FLAT) {
        if (a.row_count) rows = (int32_t)uni((uint32_t)a.row_count[wblock]);
        if (a.in_count) cols = uni(a.in_count[wblock]);
        if (rows <= 0) return;
    }

    for (uint32_t grp = 0; grp < ngroups; ++grp) {
        if constexpr (!FLAT) {
#pragma unroll
            for (int j = 0; j < NI; ++j) {
                item[j] = (grp * NI + j) * kWave + lane;
                blk[j] = wblock;
                valid[j] = item[j] < ips;
            }
        }
        // per-lane column limits (FLAT: shortened blocks differ per lane)
        uint32_t ncol[NI];
#pragma unroll
        for (int j = 0; j < NI; ++j)
            ncol[j] = (FLAT && a.in_count) ? (valid[j] ? a.in_count[blk[j]] : 0u) : cols;

        const uint8_t* in_ptr[NI];
#pragma unroll
        for (int j = 0; j < NI; ++j)
            in_ptr[j] = a.in_base + (uint64_t)blk[j] * a.in_block_stride + (uint64_t)item[j] * 8u;

        const uint8_t* coef_blk = a.coef;
        if constexpr (!FLAT)
            coef_blk += (uint64_t)(a.coef_by_count ? (cols ? cols - 1 : 0) : wblock) * a.coef_block_stride;
        bool staged = false;
        if constexpr (!FLAT) {
            const uint32_t cdw = (cols * a.coef_col_stride + 3) / 4;
            if (grp == 0 && cdw <= kCoefLds && (reinterpret_cast<uintptr_t>(coef_blk) & 3) == 0) {
                const uint32_t* src = reinterpret_cast<const uint32_t*>(coef_blk);
                uint32_t* dst = lds_coef[threadIdx.x >> 6];
                for (uint32_t i = lane; i < cdw; i += kWave) dst[i] = src[i];
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
            staged = cdw <= kCoefLds && (reinterpret_cast<uintptr_t>(coef_blk) & 3) == 0;
        }
        const uint16_t* islots = (!FLAT && a.in_slots) ? a.in_slots + (uint64_t)wblock * a.slots_stride : nullptr;

        for (int32_t r0 = 0; r0 < rows; r0 += RC) {
            uint32_t acc[RC][2 * NI];
#pragma unroll
            for (int r = 0; r < RC; ++r)
#pragma unroll
                for (int d = 0; d < 2 * NI; ++d) acc[r][d] = 0;

            // software pipeline: load column c+1 while multiplying column c
            uint2 cur[NI];
            auto load_col = [&](uint32_t c, uint2* dst) {
                const uint32_t slot = islots ? (uint32_t)uni(islots[c]) : c;
                const uint64_t off = (uint64_t)slot * a.in_seg_stride;
#pragma unroll
                for (int j = 0; j < NI; ++j) {
                    if (valid[j] && c < ncol[j]) dst[j] = load8(in_ptr[j] + off);
                    else dst[j] = make_uint2(0u, 0u);
                }
            };
            if (cols > 0) load_col(0, cur);
            for (uint32_t c = 0; c < cols; ++c) {
                uint2 nxt[NI];
                if (c + 1 < cols) load_col(c + 1, nxt);
                Sel sel[2 * NI];
#pragma unroll
                for (int j = 0; j < NI; ++j) {
                    sel[2 * j] = selectors(cur[j].x);
                    sel[2 * j + 1] = selectors(cur[j].y);
                }
                const uint32_t* cw =
                    staged ? &lds_coef[threadIdx.x >> 6][((uint64_t)c * a.coef_col_stride + r0) >> 2]
                           : reinterpret_cast<const uint32_t*>(coef_blk + (uint64_t)c * a.coef_col_stride + r0);
#pragma unroll
                for (int r4 = 0; r4 < RC / 4; ++r4) {
                    const uint32_t word = cw[r4];
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr) {
                        const int r = r4 * 4 + rr;
                        if (FLAT || r0 + r < rows) {
                            const uint32_t cv = (word >> (8 * rr)) & 0xffu;
                            const uint4 t = lds_tab[cv * 2];
                            const uint32_t t4 = tab32[cv * 8 + 4];
#pragma unroll
                            for (int d = 0; d < 2 * NI; ++d) acc[r][d] ^= gfmul4(t, t4, sel[d]);
                        }
                    }
                }
                if (c + 1 < cols) {
#pragma unroll
                    for (int j = 0; j < NI; ++j) cur[j] = nxt[j];
                }
            }

            // ---- write back rows [r0, r0+RC) ----
            const uint16_t* oslots = (a.out_slot_mode == OUT_SLOT_LIST)
                                         ? a.out_slots + (uint64_t)(FLAT ? 0 : wblock) * a.slots_stride
                                         : nullptr;
#pragma unroll
            for (int r = 0; r < RC; ++r) {
                if (r0 + r >= rows) continue;
#pragma unroll
                for (int j = 0; j < NI; ++j) {
                    if (!valid[j]) continue;
                    uint32_t slot;
                    if (a.out_slot_mode == OUT_SLOT_LIST) slot = oslots[r0 + r];
                    else if (a.out_slot_mode == OUT_SLOT_AFTER_INPUT) slot = ncol[j] + r0 + r;
                    else slot = r0 + r;
                    uint8_t* p = a.out_base + (uint64_t)blk[j] * a.out_block_stride +
                                 (uint64_t)slot * a.out_seg_stride + (uint64_t)item[j] * 8u;
                    uint2 v = make_uint2(acc[r][2 * j], acc[r][2 * j + 1]);
                    if (a.accumulate) {
                        const uint2 o = load8(p);
                        v.x ^= o.x;
                        v.y ^= o.y;
                    }
                    store_bytes(p, v, a.vec_bytes - item[j] * 8u);
                }
            }
        }
    }
}

template <int NI, int RC, bool FLAT>
hipError_t launch_one(const Gf8MatmulArgs& a, hipStream_t s)
{
    const uint32_t ips = (a.vec_bytes + 7) / 8;
    uint64_t waves;
    if (FLAT) waves = ((uint64_t)a.nblocks * ips + NI * kWave - 1) / (NI * kWave);
    else waves = a.nblocks;
    const uint64_t groups = (waves + kWavesPerGroup - 1) / kWavesPerGroup;
    hipLaunchKernelGGL((gf8_matmul_kernel<NI, RC, FLAT>), dim3((uint32_t)groups), dim3(kThreads), 0, s, a);
    return hipGetLastError();
}

// ---- per-block square solve (decode stage 2 of the fast RS8 path) ----
// out[b][out_slots[b][r]] (^)= XOR_t coef[b][t][r] (x) z[b][t]   for r < rows(b) <= RC, t < cols(b).
// One wave per block.  The block's RC x cols coefficient tables (5 dwords each) are expanded
// into LDS once, zero-padded to RC rows and an even column count, so the main loop is
// branch-free: per column pair the wave issues the next pair's z loads, then for each of
// the RC rows reads its table with uniform (broadcast) LDS loads whose addresses do not
// depend on data, and applies 3 v_perm + 1 bitop3 + 1 xor per output dword.
template <int NI, int RC, int LA>
__global__ __launch_bounds__(kThreads) void gf8_solve_kernel(Gf8SolveArgs a)
{
    constexpr int kMaxCols = 32;
    __shared__ uint4 lds_t4[kWavesPerGroup][kMaxCols * RC + LA];  // +LA: pipelined reads past the end
    __shared__ uint32_t lds_t1[kWavesPerGroup][kMaxCols * RC + LA];
    const uint32_t lane = threadIdx.x & (kWave - 1);
    const uint32_t w = threadIdx.x >> 6;
    if (a.gate && *a.gate != a.gate_gen) return;  // every block repaired by the fused kernel
    const uint32_t blk = uni(blockIdx.x * kWavesPerGroup + w);
    if (blk >= a.nblocks) return;
    const int32_t rows = (int32_t)uni((uint32_t)a.rows[blk]);
    if (rows <= 0 || rows <= a.min_rows) return;
    const uint32_t cols = min(uni((uint32_t)a.cols[blk]), (uint32_t)kMaxCols);
    const uint32_t cols2 = (cols + 1) & ~1u;

    for (int32_t r0 = 0; r0 < rows; r0 += RC) {
    // expand the tables of rows [r0, r0+RC): entry (t, r) for t < cols2
    {
        const uint8_t* cb = a.coef + (uint64_t)blk * a.coef_block_stride + r0;
        __builtin_amdgcn_wave_barrier();
        for (uint32_t e = lane; e < cols2 * RC; e += kWave) {
            const uint32_t t = e / RC, r = e % RC;
            const uint32_t cv = (t < cols && r0 + (int32_t)r < rows) ? cb[(uint64_t)t * a.coef_col_stride + r] : 0u;
            const uint32_t* src = a.vtab + cv * 8;
            lds_t4[w][e] = make_uint4(src[0], src[1], src[2], src[3]);
            lds_t1[w][e] = src[4];
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    const uint32_t ips = (a.vec_bytes + 7) >> 3;
    const uint8_t* zb = a.z + (uint64_t)blk * a.z_block_stride;
    const uint16_t* oslots = a.out_slots + (uint64_t)blk * a.slots_stride;
    for (uint32_t g0 = 0; g0 < ips; g0 += NI * kWave) {
        uint32_t zoff[NI];
        bool valid[NI];
#pragma unroll
        for (int j = 0; j < NI; ++j) {
            const uint32_t it = g0 + (uint32_t)j * kWave + lane;
            valid[j] = it < ips;
            zoff[j] = (valid[j] ? it : g0) * 8u;
        }
        uint32_t acc[RC][2 * NI];
#pragma unroll
        for (int r = 0; r < RC; ++r)
#pragma unroll
            for (int d = 0; d < 2 * NI; ++d) acc[r][d] = 0;

        auto load_pair = [&](uint32_t t, uint2 (&dst)[2][NI]) {
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const uint32_t tt = min(t + (uint32_t)u, cols - 1);
                const uint8_t* zr = zb + (uint64_t)tt * a.z_stride;
#pragma unroll
                for (int j = 0; j < NI; ++j) dst[u][j] = load8(zr + zoff[j]);
            }
        };
        uint2 cur[2][NI], nxt[2][NI];
        load_pair(0, cur);
        // tables are software-pipelined LA rows ahead (LDS latency off the VALU chain)
        const uint4* t4 = lds_t4[w];
        const uint32_t* t1 = lds_t1[w];
        uint4 tb[LA + 1];
        uint32_t tc[LA + 1];
#pragma unroll
        for (int q = 0; q < LA; ++q) {
            tb[q] = t4[q];
            tc[q] = t1[q];
        }
        for (uint32_t t = 0; t < cols2; t += 2) {
            load_pair(min(t + 2, cols2 - 2), nxt);
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                Sel sel[2 * NI];
#pragma unroll
                for (int j = 0; j < NI; ++j) {
                    sel[2 * j] = selectors(cur[u][j].x);
                    sel[2 * j + 1] = selectors(cur[u][j].y);
                }
                const uint32_t e0 = (t + u) * RC;
#pragma unroll
                for (int r = 0; r < RC; ++r) {
                    tb[LA] = t4[e0 + r + LA];
                    tc[LA] = t1[e0 + r + LA];
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int d = 0; d < 2 * NI; ++d) acc[r][d] ^= gfmul4(tb[0], tc[0], sel[d]);
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int q = 0; q < LA; ++q) {
                        tb[q] = tb[q + 1];
                        tc[q] = tc[q + 1];
                    }
                }
            }
#pragma unroll
            for (int u = 0; u < 2; ++u)
#pragma unroll
                for (int j = 0; j < NI; ++j) cur[u][j] = nxt[u][j];
        }
#pragma unroll
        for (int r = 0; r < RC; ++r) {
            if (r0 + (int32_t)r >= rows) continue;
            uint8_t* orow = a.out + (uint64_t)blk * a.out_block_stride + (uint64_t)oslots[r0 + r] * a.out_seg_stride;
#pragma unroll
            for (int j = 0; j < NI; ++j) {
                if (!valid[j]) continue;
                uint8_t* p = orow + zoff[j];
                uint2 v = make_uint2(acc[r][2 * j], acc[r][2 * j + 1]);
                if (a.accumulate) {
                    const uint2 o = load8(p);
                    v.x ^= o.x;
                    v.y ^= o.y;
                }
                store_bytes(p, v, a.vec_bytes - zoff[j]);
            }
        }
    }
    }
}

template <int NI, int RC, int LA = 1>
hipError_t launch_solve(const Gf8SolveArgs& a, hipStream_t s)
{
    const uint32_t groups = (a.nblocks + kWavesPerGroup - 1) / kWavesPerGroup;
    hipLaunchKernelGGL((gf8_solve_kernel<NI, RC, LA>), dim3(groups), dim3(kThreads), 0, s, a);
    return hipGetLastError();
}

}  // namespace

int launch_gf8_solve(const Gf8SolveArgs& a, uint32_t max_rows, uint32_t max_cols, hipStream_t s)
{
    if (a.nblocks == 0 || a.vec_bytes == 0) return NFEC_OK;
    if (max_cols > 32) return NFEC_ENOTSUP;
    const uint32_t ni = (((a.vec_bytes + 7) / 8) + kWave - 1) / kWave;
    // NFEC_SOLVE_CFG (A/B runs, diagnostic library): 1 = 8-row bands, 2 = tables two rows ahead
    static const int cfg = (int)diag_knob("NFEC_SOLVE_CFG", 0, 0, 2);
    hipError_t e;
    if (max_rows <= 8 || cfg == 1) e = ni <= 2 ? launch_solve<2, 8>(a, s) : launch_solve<3, 8>(a, s);
    else if (cfg == 2) e = ni <= 2 ? launch_solve<2, 16, 2>(a, s) : launch_solve<3, 16, 2>(a, s);
    else e = ni <= 2 ? launch_solve<2, 16>(a, s) : launch_solve<3, 16>(a, s);
    if (e != hipSuccess) return hip_fail(e, "gf8_solve launch");
    return NFEC_OK;
}

int launch_gf8_matmul(const Gf8MatmulArgs& a, bool shared_coef, hipStream_t s)
{
    if (a.nblocks == 0 || a.vec_bytes == 0) return NFEC_OK;
    const uint32_t ips = (a.vec_bytes + 7) / 8;
    hipError_t e;
    if (shared_coef) {
        // encode: flat item space, 2 items (16 bytes) per lane, up to 32 rows per pass
        if (a.rows_const <= 16) e = launch_one<2, 16, true>(a, s);
        else e = launch_one<2, 32, true>(a, s);
    } else {
        // per-block matrices: one wave per block
        const uint32_t ni = (ips + kWave - 1) / kWave;
        if (ni <= 1) e = launch_one<1, 16, false>(a, s);
        else if (ni == 2) e = launch_one<2, 16, false>(a, s);
        else if (ni == 3) e = launch_one<3, 16, false>(a, s);
        else e = launch_one<4, 16, false>(a, s);
    }
    if (e != hipSuccess) return hip_fail(e, "gf8_matmul launch");
    return NFEC_OK;
}

}  // namespace nfec
