// kernels_gf16bs.hip -- RS16 encode, bit-sliced, with per-lane four-Russians tables in LDS.
//
// The table kernel (kernels_gf16.hip) spends one random LDS lookup per GF(2^16) multiply-add,
// and random 16-bit lookups into a 128 KiB table conflict on the LDS banks (~8.5 cycles per
// wave lookup).  Here every lane owns 32 symbols of one segment (64 bytes) as 16 bit-planes
// (plane p = bit p of the 32 symbols).  Multiplying by a constant c is linear over GF(2):
//     Y[p] = XOR_{j : bit p of (c * alpha^j) is set} X[j]        (alpha^j = 1 << j, j < 16)
// Splitting the 16 input planes into 4 groups of 4, each lane writes the 16 XOR-combinations
// of each group once per source column into LDS (layout [group*16 + combination][lane], so a
// wave reads a uniform entry with no bank conflict) and each output plane of each parity row
// is then 4 reads and 2 three-input XORs.  The entry indices are wave-uniform (they depend only
// on the generator coefficient) and precomputed on the host: sel[col][row][plane*4 + group].
//
// Work split: one wave = 64 items (block, 64-byte chunk) x one pass of RC parity rows; items
// run across blocks (the generator is shared), passes across waves (each re-reads its columns).
// Reference semantics kept: parity[r] (^)= sum_c G[k+r][c] * data_c over vec/2 native-endian
// symbols (normEncoderRS16.cpp:472-482), source columns >= numData are zero (shortened
// blocks), parity written to slots numData + r, an odd last byte never touched.
#include "nfec_internal.hpp"

namespace nfec {

namespace {

constexpr int kBsWaves = 4;
constexpr int kBsRows = 8;                 // parity rows per pass: 8 x 16 accumulator planes
constexpr uint32_t kTabDwords = 64 * 64;   // per wave: 64 entries x 64 lanes

// 16 x 16 bit transpose of the low halves and of the high halves of x[0..15] at once:
// afterwards bit j of x[p] (j < 16) is bit p of the low symbol of input dword j, and bit
// 16 + j that of the high symbol.  Swapmove stages 8, 4, 2, 1; the network is its own inverse.
__device__ __forceinline__ void transpose16(uint32_t (&x)[16])
{
#pragma unroll
    for (int st = 0; st < 4; ++st) {
        const int s = 8 >> st;
        const uint32_t mask = st == 0 ? 0x00ff00ffu : st == 1 ? 0x0f0f0f0fu : st == 2 ? 0x33333333u : 0x55555555u;
#pragma unroll
        for (int d = 0; d < 16; ++d) {
            if (d & s) continue;
            const uint32_t t = ((x[d] >> s) ^ x[d + s]) & mask;
            x[d + s] ^= t;
            x[d] ^= t << s;
        }
    }
}

__global__ __launch_bounds__(kBsWaves * 64, 2) void gf16_bs_encode_kernel(Gf16BsEncArgs a, const uint16_t* __restrict__ sel,
                                                                         const uint8_t* __restrict__ src_base,
                                                                         uint8_t* __restrict__ out_base)
{
    extern __shared__ uint32_t lds_tab[];
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint32_t* T = lds_tab + wave * kTabDwords + lane;

    const uint32_t passes = (a.m + kBsRows - 1) / kBsRows;
    // workgroups are dealt to the 8 XCDs round-robin; renumber them so consecutive logical
    // groups (the row passes of one item group, which read the same columns) share an XCD's L2
    const uint32_t ng = gridDim.x, wg = blockIdx.x;
    const uint32_t per = ng / 8, rem = ng % 8, xcd = wg % 8, idx = wg / 8;
    const uint32_t lwg = (ng >= 8 && wg < per * 8) ? xcd * per + idx : wg;
    (void)rem;
    const uint64_t gw = (uint64_t)lwg * kBsWaves + wave;
    const uint64_t item_wave = gw / passes;
    const uint32_t pass = (uint32_t)(gw % passes);
    const uint64_t items = (uint64_t)a.nblocks * a.chunks;
    if (item_wave * 64 >= items) return;  // wave-uniform
    const uint64_t item = item_wave * 64 + lane;
    const bool valid = item < items;
    const uint32_t b = valid ? (uint32_t)(item / a.chunks) : 0u;
    const uint32_t byte0 = valid ? (uint32_t)(item % a.chunks) * 64u : 0u;
    const uint32_t nd = valid ? (a.num_data ? (uint32_t)a.num_data[b] : a.k) : 0u;
    const uint32_t nbytes = valid ? min(64u, a.vec_bytes - byte0) : 0u;  // even
    const uint8_t* blk = src_base + (uint64_t)b * a.block_stride + byte0;
    const uint32_t r0 = pass * kBsRows;
    const uint32_t rows = min((uint32_t)kBsRows, a.m - r0);

    uint32_t acc[kBsRows][16];
#pragma unroll
    for (int r = 0; r < kBsRows; ++r)
#pragma unroll
        for (int p = 0; p < 16; ++p) acc[r][p] = 0;

    // column c's selectors: 8 rows x 64 uint16 = 1 KB, 16 bytes per lane, loaded one column
    // ahead (vector loads: no scalar loads in flight, so the LDS waits stay counted)
    const uint4* selp = reinterpret_cast<const uint4*>(sel + (uint64_t)r0 * 64) + lane;
    const uint64_t sel_col = (uint64_t)a.m_pad * 64 / 8;  // uint4 per column
    uint4 sv = selp[0];
    for (uint32_t c = 0; c < a.k; ++c) {
        uint32_t x[16];
        const uint8_t* src = blk + (uint64_t)c * a.seg_stride;
        if (c < nd && nbytes == 64) {
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const uint2 v = *reinterpret_cast<const uint2*>(src + 8 * q);
                x[2 * q] = v.x;
                x[2 * q + 1] = v.y;
            }
        } else {
#pragma unroll
            for (int d = 0; d < 16; ++d) {
                uint32_t v = 0;
                if (c < nd) {
                    if (4u * d + 4u <= nbytes) v = *reinterpret_cast<const uint32_t*>(src + 4 * d);
                    else if (4u * d + 2u <= nbytes) v = *reinterpret_cast<const uint16_t*>(src + 4 * d);
                }
                x[d] = v;
            }
        }
        const uint4 cur = sv;
        if (c + 1 < a.k) sv = selp[(uint64_t)(c + 1) * sel_col];
        transpose16(x);
        // the 16 combinations of each group of 4 planes
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const uint32_t e0 = x[4 * g], e1 = x[4 * g + 1], e2 = x[4 * g + 2], e3 = x[4 * g + 3];
            uint32_t* t = T + g * 16 * 64;
            const uint32_t e01 = e0 ^ e1, e23 = e2 ^ e3;
            t[0 * 64] = 0;
            t[1 * 64] = e0;
            t[2 * 64] = e1;
            t[3 * 64] = e01;
            t[4 * 64] = e2;
            t[5 * 64] = e0 ^ e2;
            t[6 * 64] = e1 ^ e2;
            t[7 * 64] = e01 ^ e2;
            t[8 * 64] = e3;
            t[9 * 64] = e0 ^ e3;
            t[10 * 64] = e1 ^ e3;
            t[11 * 64] = e01 ^ e3;
            t[12 * 64] = e23;
            t[13 * 64] = e0 ^ e23;
            t[14 * 64] = e1 ^ e23;
            t[15 * 64] = e01 ^ e23;
        }
        // offsets of (row r, plane p): lane r*8 + p/2 holds them in dwords (p%2)*2, +1
#pragma unroll
        for (int r = 0; r < kBsRows; ++r) {
            uint32_t v[16][4];
#pragma unroll
            for (int p = 0; p < 16; ++p) {
                const int ln = r * 8 + p / 2;
                const uint32_t w0 = (uint32_t)__builtin_amdgcn_readlane((int)((p & 1) ? cur.z : cur.x), ln);
                const uint32_t w1 = (uint32_t)__builtin_amdgcn_readlane((int)((p & 1) ? cur.w : cur.y), ln);
                v[p][0] = T[w0 & 0xffffu];
                v[p][1] = T[w0 >> 16];
                v[p][2] = T[w1 & 0xffffu];
                v[p][3] = T[w1 >> 16];
            }
#pragma unroll
            for (int p = 0; p < 16; ++p) acc[r][p] ^= v[p][0] ^ v[p][1] ^ v[p][2] ^ v[p][3];
        }
    }

    if (!valid) return;
#pragma unroll
    for (int r = 0; r < kBsRows; ++r) {
        if ((uint32_t)r >= rows) break;
        transpose16(acc[r]);
        uint8_t* dst = out_base + (uint64_t)b * a.block_stride + (uint64_t)(nd + r0 + r) * a.seg_stride + byte0;
        if (nbytes == 64) {
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                uint2 v = make_uint2(acc[r][2 * q], acc[r][2 * q + 1]);
                uint2* pq = reinterpret_cast<uint2*>(dst + 8 * q);
                if (a.accumulate) {
                    const uint2 o = *pq;
                    v.x ^= o.x;
                    v.y ^= o.y;
                }
                *pq = v;
            }
        } else {
#pragma unroll
            for (int d = 0; d < 16; ++d) {
                if (4u * d + 4u <= nbytes) {
                    uint32_t* pd = reinterpret_cast<uint32_t*>(dst + 4 * d);
                    *pd = a.accumulate ? (*pd ^ acc[r][d]) : acc[r][d];
                } else if (4u * d + 2u <= nbytes) {
                    uint16_t* ph = reinterpret_cast<uint16_t*>(dst + 4 * d);
                    const uint16_t v = (uint16_t)acc[r][d];
                    *ph = a.accumulate ? (uint16_t)(*ph ^ v) : v;
                }
            }
        }
    }
}

}  // namespace

int launch_gf16_bs_encode(const Gf16BsEncArgs& a, hipStream_t s)
{
    if (a.nblocks == 0 || a.vec_bytes < 2 || a.m == 0) return NFEC_OK;
    if ((a.seg_stride & 7) || (a.block_stride & 7) || (reinterpret_cast<uintptr_t>(a.base) & 7))
        return NFEC_ENOTSUP;  // 8-byte loads (check_batch guarantees this alignment)
    const uint64_t items = (uint64_t)a.nblocks * a.chunks;
    const uint64_t waves = (items + 63) / 64 * ((a.m + kBsRows - 1) / kBsRows);
    const uint64_t groups = (waves + kBsWaves - 1) / kBsWaves;
    if (groups > 0x7fffffffu) return NFEC_ENOTSUP;
    const size_t lds = (size_t)kBsWaves * kTabDwords * 4;
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&gf16_bs_encode_kernel),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        attr = true;
    }
    hipLaunchKernelGGL(gf16_bs_encode_kernel, dim3((uint32_t)groups), dim3(kBsWaves * 64), lds, s, a, a.sel, a.base, a.out_base);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? NFEC_OK : hip_fail(e, "gf16 bit-sliced encode launch");
}

// sel[c][r][p*4 + g] = dword offset in the lane's table of the combination of group g that
// output plane p of G[r][c] * x needs (see the kernel comment).
void gf16_bs_selectors(const std::vector<uint32_t>& parity_rows, uint32_t k, uint32_t m, uint16_t* sel)
{
    const Field& f = gf16();
    const uint32_t mp = gf16_bs_rows_padded(m);
    for (uint32_t c = 0; c < k; ++c) {
        for (uint32_t r = 0; r < mp; ++r) {
            const uint32_t g = r < m ? parity_rows[(size_t)r * k + c] : 0u;
            uint32_t col[16];  // column j of the multiplication matrix: g * alpha^j
            for (int j = 0; j < 16; ++j) col[j] = f.mul(g, 1u << j);
            uint16_t* o = sel + ((size_t)c * mp + r) * 64;
            for (int p = 0; p < 16; ++p)
                for (int q = 0; q < 4; ++q) {
                    uint32_t s = 0;
                    for (int i = 0; i < 4; ++i) s |= ((col[4 * q + i] >> p) & 1u) << i;
                    o[p * 4 + q] = (uint16_t)((q * 16 + s) * 64);
                }
        }
    }
}

}  // namespace nfec
