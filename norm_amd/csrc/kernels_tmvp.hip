// RS16 encode by the Toeplitz split of the generator (rs16_tmvp in nfec_api.cpp).
//
// The RS16 generator of NormEncoderRS16::Init (src/common/normEncoderRS16.cpp:399-461) is the
// Lagrange basis of the points x_0 = 0, x_j = alpha^(j-1) evaluated at y_p = alpha^(k-1+p):
//   G[p][j] = W(y_p) / ((y_p + x_j) W'(x_j)),  W(z) = prod_l (z + x_l),
// and for j >= 1, y_p + x_j = alpha^(j-1) (1 + alpha^(k+p-j)), so
//   G[p][j] = W(y_p) * T[p][j] * c_j,  T[p][j] = 1 / (1 + alpha^(k+p-j)),  c_j = alpha^-(j-1) / W'(x_j):
// a row scaling, a Toeplitz matrix and a column scaling.  With the rows split in halves R0, R1
// of cw = m/2 and the columns in chunk pairs (C0, C1) of cw each, T's blocks are [[A, B], [C, A]]
// and one Karatsuba step needs three products instead of four:
//   P0 = A (v_C0 + v_C1)  (v = c * d, the prescaled data: prescale_kernel)
//   P1 = (B - A) c_C1 d_C1,  P2 = (C - A) c_C0 d_C0   (coefficients absorb c)
//   parity_R0 = W (P0 + P1) + G[.][0] d_0,  parity_R1 = W (P0 + P2) + G[.][0] d_0  (postscale_kernel)
// The products run in one launch of the tower kernel (gen_gf16_tw.hip; the shared-table kernel,
// gen_gf16_t3.hip, under NFEC_OPT_RS16_SHARED_TABLES, one level only); the kernels here are the elementwise steps around
// them: bit-sliced multiplies by wave-uniform constants.  Two Karatsuba levels (nine products)
// use the tmvp2_* pair below.  Any chunk width; vec % 8 != 0 runs over the 8-byte pieces and the
// tail kernel takes the rest (rs16_tmvp_encode, nfec_api.cpp).
#include "nfec_internal.hpp"
#include "gf16_bs.hpp"
#include "bitslice.hpp"

#include <algorithm>

namespace nfec {
namespace {

// ---- two Karatsuba levels (rs16_tmvp_plan_levels, levels = 2) ----
// Scratch per block (sc, sc_block_stride; columns of vec bytes): the level-1 pair sums v at
// [0, k/2) (virtual column q*cw + i), the level-2 scaled sums s_0, s_1, s_2 at k/2 + X*k/4 + u
// (u = q*hw + i, i < hw), then the nine hw-row products at k/2 + 3k/4 + e*hw + p.
__device__ __forceinline__ uint32_t tmvp2_prow0(const Rs16TmvpArgs& a) { return a.k / 2u + 3u * (a.k / 4u); }

// per (q, i < hw): u_j = c_j d_j for j = a0, a1 = a0 + hw, b0 = a0 + cw, b1 = b0 + hw, then
//   v at q cw + i = u_a0 + u_b0, at q cw + hw + i = u_a1 + u_b1   (the level-1 pair sums, halves)
//   s_0 = both pair sums, s_1 = u_b0 + u_b1, s_2 = u_a0 + u_a1      (level 2's alpha inputs)
// (the products are linear, so the sums are taken after transposing back to symbols)
// buffer addressing for the prescale and postscale kernels: descriptors over the wave's first block (of the
// batch and of the scratch) and per item a 32-bit offset into each (0x80000000 outside the batch:
// its loads read zeros, its stores drop, no branches).  With 64-bit addresses per item and
// branches the postscale spilled (332 bytes per lane) and took 1.44 ms per 2,048 C4 blocks.
struct ItemMapB {
    uint32_t vs[8], vc[8];
    __amdgpu_buffer_rsrc_t src, sc;
};

// (sc, sc_stride: the scratch the kernel reads or writes -- level 2: a.sc; level 1: a.s or a.x)
// nd[j] = the numData of item j's block (k without a.num_data, and outside the batch); an item
// whose block has numData 0 or past k is treated as outside the batch (left alone).  Unshortened
// batches take the same code with nd = k: the parity addressed as the item offset + k x stride
// and a small slot offset measured 2 % faster over the whole RS16(400,100) encode than the item
// offset + (k + row) x stride (postscale 138 -> 126 VGPRs, 4 waves per SIMD instead of 3;
// profiles/r06/tmvp_sh_ab.jsonl)
__device__ __forceinline__ void map_items_b(const Rs16TmvpArgs& a, uint32_t chunk, uint32_t lane, ItemMapB& m,
                                            uint8_t* sc, uint64_t sc_stride, uint32_t nd[8])
{
    const uint32_t ipb = a.vec / 8u, items = a.nblocks * ipb;
    const uint32_t blk0 = __builtin_amdgcn_readfirstlane((chunk * 512u) / ipb);
    m.src = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(a.base) + (uint64_t)blk0 * a.block_stride, (short)0,
                                              (int)0x80000000u, 0x00020000);
    m.sc = __builtin_amdgcn_make_buffer_rsrc(sc + (uint64_t)blk0 * sc_stride, (short)0, (int)0x80000000u, 0x00020000);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const uint32_t it = chunk * 512u + (uint32_t)j * 64u + lane;
        const uint32_t b = it / ipb, off = (it - b * ipb) * 8u, db = b - blk0;
        bool ok = it < items;
        nd[j] = a.k;
        if (ok && a.num_data) {
            const uint32_t v = a.num_data[b];
            ok = v >= 1u && v <= a.k;
            nd[j] = ok ? v : a.k;
        }
        m.vs[j] = ok ? db * (uint32_t)a.block_stride + off : 0x80000000u;
        m.vc[j] = ok ? db * (uint32_t)sc_stride + off : 0x80000000u;
    }
}

// item offsets for source column col (wave-uniform): bit 31 (reads zeros) where col is at or
// past the item's numData
__device__ __forceinline__ void col_offsets(uint32_t o[8], const uint32_t v[8], const uint32_t nd[8], uint32_t col)
{
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = col < nd[j] ? v[j] : 0x80000000u;
}

// item offsets of the block's parity slot 0 (slot numData): stores past the batch drop
__device__ __forceinline__ void parity_offsets(uint32_t o[8], const uint32_t v[8], const uint32_t nd[8], uint32_t ss)
{
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = v[j] == 0x80000000u ? v[j] : v[j] + nd[j] * ss;
}

template <int AUX = 0>
__device__ __forceinline__ void load16_b(uint32_t x[16], __amdgpu_buffer_rsrc_t rs, uint32_t soff, const uint32_t v[8])
{
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const bs::u32x2 w = __builtin_amdgcn_raw_buffer_load_b64(rs, v[j], soff, AUX);
        x[2 * j] = w.x;
        x[2 * j + 1] = w.y;
    }
}

template <int AUX = 0>
__device__ __forceinline__ void store16_b(const uint32_t x[16], __amdgpu_buffer_rsrc_t rs, uint32_t soff, const uint32_t v[8])
{
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        bs::u32x2 w;
        w.x = x[2 * j];
        w.y = x[2 * j + 1];
        __builtin_amdgcn_raw_buffer_store_b64(w, rs, v[j], soff, AUX);
    }
}

// the postscale's offsets fit 32 bits: a wave's 512 items span at most 512 / ipb + 2 blocks
static bool tmvp2_offsets_fit(const Rs16TmvpArgs& a)
{
    const uint64_t ipb = a.vec / 8u, nb = 512u / std::max<uint64_t>(ipb, 1) + 2u;
    const uint64_t slots = (uint64_t)a.k + 2u * a.cw;
    return nb * a.block_stride + slots * a.seg_stride < (1ull << 31) && (nb + 1) * a.sc_block_stride < (1ull << 31);
}

// level 1's offsets fit 32 bits (its scratch: the pair sums a.s, the P1 rows a.x)
static bool tmvp1_offsets_fit(const Rs16TmvpArgs& a)
{
    const uint64_t ipb = a.vec / 8u, nb = 512u / std::max<uint64_t>(ipb, 1) + 2u;
    const uint64_t slots = (uint64_t)a.k + 2u * a.cw;
    return nb * a.block_stride + slots * a.seg_stride < (1ull << 31) && (nb + 1) * a.s_block_stride < (1ull << 31) &&
           (nb + 1) * a.x_block_stride < (1ull << 31);
}

// items of 8 bytes (4 symbols), 8 per lane, 512 per wave: item j of the lane is
// chunk * 512 + j * 64 + lane, flat over (block, position in the segment), addressed as above.
// v = c_a d_a + c_b d_b for every chunk pair: virtual column q*cw + i from columns
// a = 2q*cw + i and b = a + cw (c_0 = 0: column 0 is added by the postscale)
__global__ __launch_bounds__(256, 4) void tmvp_prescale_kernel(Rs16TmvpArgs a)
{
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wid = __builtin_amdgcn_readfirstlane(blockIdx.x * 4u + (threadIdx.x >> 6));
    const uint32_t half = a.k / 2;
    const uint32_t v = wid % half, chunk = wid / half;
    const uint32_t ipb = a.vec / 8u, items = a.nblocks * ipb;
    if (chunk * 512u >= items) return;
    const uint32_t q = v / a.cw, i = v - q * a.cw;
    const uint32_t ca = 2u * q * a.cw + i, cb = ca + a.cw;
    ItemMapB m;
    uint32_t nd[8];
    map_items_b(a, chunk, lane, m, a.s, a.s_block_stride, nd);
    uint32_t x[16], y[16], z[16];
    {  // shortened blocks: source columns at or past numData read zeros
        uint32_t o[8];
        col_offsets(o, m.vs, nd, ca);
        load16_b(x, m.src, ca * a.seg_stride, o);
        col_offsets(o, m.vs, nd, cb);
        load16_b(y, m.src, cb * a.seg_stride, o);
    }
    bs16::transpose(x);
    bs16::transpose(y);
#pragma unroll
    for (int p = 0; p < 16; ++p) z[p] = 0;
    bs16::mulc_acc(x, z, a.cmat + 16u * ca);
    bs16::mulc_acc(y, z, a.cmat + 16u * cb);
    bs16::transpose(z);
    store16_b(z, m.sc, v * a.vec, m.vc);
}

// parity row p < cw and p + cw from P0 (parity row p), P1 (x row p), P2 (parity row cw + p)
// and source column 0 (shortened blocks: the parity rows at slot numData + r)
__global__ __launch_bounds__(256, 4) void tmvp_postscale_kernel(Rs16TmvpArgs a)
{
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wid = __builtin_amdgcn_readfirstlane(blockIdx.x * 4u + (threadIdx.x >> 6));
    const uint32_t p = wid % a.cw, chunk = wid / a.cw;
    const uint32_t ipb = a.vec / 8u, items = a.nblocks * ipb;
    if (chunk * 512u >= items) return;
    ItemMapB m;
    uint32_t nd[8], pv[8];
    map_items_b(a, chunk, lane, m, a.x, a.x_block_stride, nd);
    parity_offsets(pv, m.vs, nd, a.seg_stride);  // parity rows from slot numData (k unshortened)
    const uint32_t r0 = p * a.seg_stride, r1 = (a.cw + p) * a.seg_stride;
    uint32_t t0[16], t1[16], d0[16], o[16];
    load16_b(t0, m.src, r0, pv);
    load16_b(d0, m.src, 0u, m.vs);
    load16_b(t1, m.sc, p * a.vec, m.vc);
#pragma unroll
    for (int j = 0; j < 16; ++j) t1[j] ^= t0[j];  // P0 + P1
    bs16::transpose(t1);
    bs16::transpose(d0);
#pragma unroll
    for (int j = 0; j < 16; ++j) o[j] = 0;
    bs16::mulc_acc(t1, o, a.wmat + 16u * p);
    bs16::mulc_acc(d0, o, a.gmat + 16u * p);
    bs16::transpose(o);
    load16_b(t1, m.src, r1, pv);
    store16_b(o, m.src, r0, pv);
#pragma unroll
    for (int j = 0; j < 16; ++j) t1[j] ^= t0[j];  // P0 + P2
    bs16::transpose(t1);
#pragma unroll
    for (int j = 0; j < 16; ++j) o[j] = 0;
    bs16::mulc_acc(t1, o, a.wmat + 16u * (a.cw + p));
    bs16::mulc_acc(d0, o, a.gmat + 16u * (a.cw + p));
    bs16::transpose(o);
    store16_b(o, m.src, r1, pv);
}

// (SP / LP: cache policy of the scratch stores / source loads, NFEC_TMVP_POLICY A/B, knob library)
template <int SP, int LP>
__global__ __launch_bounds__(256, 4) void tmvp2_prescale_kernel(Rs16TmvpArgs a)
{
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wid = __builtin_amdgcn_readfirstlane(blockIdx.x * 4u + (threadIdx.x >> 6));
    const uint32_t quarter = a.k / 4u;
    const uint32_t u = wid % quarter, chunk = wid / quarter;
    const uint32_t ipb = a.vec / 8u, items = a.nblocks * ipb;
    if (chunk * 512u >= items) return;
    const uint32_t q = u / a.hw, i = u - q * a.hw;
    const uint32_t a0 = 2u * q * a.cw + i;
    const uint32_t col[4] = {a0, a0 + a.hw, a0 + a.cw, a0 + a.cw + a.hw};  // a0, a1, b0, b1
    ItemMapB m;
    uint32_t nd[8];
    map_items_b(a, chunk, lane, m, a.sc, a.sc_block_stride, nd);
    // all four columns' loads in flight first, then each scaled in place (shortened blocks:
    // columns at or past numData read zeros)
    uint32_t r[4][16];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        uint32_t o[8];
        col_offsets(o, m.vs, nd, col[t]);
        load16_b<LP>(r[t], m.src, col[t] * a.seg_stride, o);
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        uint32_t o[16];
        bs16::transpose(r[t]);
#pragma unroll
        for (int p = 0; p < 16; ++p) o[p] = 0;
        bs16::mulc_acc(r[t], o, a.cmat + 16u * col[t]);
        bs16::transpose(o);
#pragma unroll
        for (int p = 0; p < 16; ++p) r[t][p] = o[p];
    }
    uint32_t o[16];
#pragma unroll
    for (int p = 0; p < 16; ++p) o[p] = r[0][p] ^ r[2][p];
    store16_b<SP>(o, m.sc, (q * a.cw + i) * a.vec, m.vc);
#pragma unroll
    for (int p = 0; p < 16; ++p) o[p] = r[1][p] ^ r[3][p];
    store16_b<SP>(o, m.sc, (q * a.cw + a.hw + i) * a.vec, m.vc);
#pragma unroll
    for (int p = 0; p < 16; ++p) o[p] = r[0][p] ^ r[1][p] ^ r[2][p] ^ r[3][p];
    store16_b<SP>(o, m.sc, (a.k / 2u + u) * a.vec, m.vc);
#pragma unroll
    for (int p = 0; p < 16; ++p) o[p] = r[2][p] ^ r[3][p];
    store16_b<SP>(o, m.sc, (a.k / 2u + quarter + u) * a.vec, m.vc);
#pragma unroll
    for (int p = 0; p < 16; ++p) o[p] = r[0][p] ^ r[1][p];
    store16_b<SP>(o, m.sc, (a.k / 2u + 2u * quarter + u) * a.vec, m.vc);
}

// per p < hw: level-1 product X's rows p (top) and hw + p (bottom) are P_aX + P_bX and
// P_aX + P_gX (products e = 3X, 3X + 1, 3X + 2); parity rows p and hw + p (R0) take X = 0, 1,
// rows cw + p and cw + hw + p (R1) take X = 0, 2, then W(y_r) and G[r][0] d_0 as at one level.
// The wave loads each of the nine products once into four sums (143 VGPRs, no spill; one
// output at a time, reloading the products, measured 1.82 against 1.56 ms per 16,384
// RS16(400,100) blocks).
template <int SP, int LP>
__global__ __launch_bounds__(256, 3) void tmvp2_postscale_kernel(Rs16TmvpArgs a)
{
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wid = __builtin_amdgcn_readfirstlane(blockIdx.x * 4u + (threadIdx.x >> 6));
    const uint32_t p = wid % a.hw, chunk = wid / a.hw;
    const uint32_t ipb = a.vec / 8u, items = a.nblocks * ipb;
    if (chunk * 512u >= items) return;
    ItemMapB m;
    uint32_t nd[8];
    map_items_b(a, chunk, lane, m, a.sc, a.sc_block_stride, nd);
    const uint32_t pr = (tmvp2_prow0(a) + p) * a.vec;  // product e's row p at pr + e hw vec
    // output rows (R0 top, R0 bottom, R1 top, R1 bottom): bit t of uses[e] = product e feeds output t
    constexpr uint8_t uses[9] = {0xF, 0x5, 0xA, 0x3, 0x1, 0x2, 0xC, 0x4, 0x8};
    uint32_t sum[4][16], x[16];
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int j = 0; j < 16; ++j) sum[t][j] = 0;
#pragma unroll
    for (int e = 0; e < 9; ++e) {
        load16_b<LP>(x, m.sc, pr + (uint32_t)e * a.hw * a.vec, m.vc);
#pragma unroll
        for (int t = 0; t < 4; ++t)
            if (uses[e] & (1u << t))
#pragma unroll
                for (int j = 0; j < 16; ++j) sum[t][j] ^= x[j];
    }
    load16_b(x, m.src, 0u, m.vs);
    bs16::transpose(x);  // d_0, bit-sliced
    // parity rows at slot numData + row (k unshortened)
    uint32_t pv[8];
    parity_offsets(pv, m.vs, nd, a.seg_stride);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const uint32_t row = (uint32_t)(t >> 1) * a.cw + (uint32_t)(t & 1) * a.hw + p;
        bs16::transpose(sum[t]);
        uint32_t o[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) o[j] = 0;
        bs16::mulc_acc(sum[t], o, a.wmat + 16u * row);
        bs16::mulc_acc(x, o, a.gmat + 16u * row);
        bs16::transpose(o);
        store16_b<SP>(o, m.src, row * a.seg_stride, pv);
    }
}

// cache policy of the level-2 scale kernels (NFEC_TMVP_POLICY, knob library A/B): 0 none,
// 1 non-temporal stores (the product library), 2 non-temporal stores and loads, 3 non-temporal
// loads.  One box, alternating twice (profiles/r06/tmvp_policy_ab/): RS16(400,100) prescale 4.98 ->
// 4.71 ms with non-temporal stores (encode 19.65 -> 19.38 ms), postscale 1.65 -> 1.62 ms; C4
// encode unchanged (95.5-96.0 ms either way); non-temporal loads slower (prescale 5.5 ms)
static int tmvp_policy()
{
    static const int v = (int)diag_knob("NFEC_TMVP_POLICY", 1, 0, 3);
    return v;
}

}  // namespace

int launch_tmvp2_prescale(const Rs16TmvpArgs& a, hipStream_t s)
{
    const uint64_t items = (uint64_t)a.nblocks * (a.vec / 8u);
    const uint64_t waves = (items + 511) / 512 * (a.k / 4);
    // (the postscale's 32-bit offsets: checked here too, before anything is written)
    if (!a.hw || !a.sc || items >= (1ull << 32) || waves >= (1ull << 32) || !tmvp2_offsets_fit(a)) return NFEC_ENOTSUP;
    if (waves == 0) return NFEC_OK;
    const dim3 g((uint32_t)((waves + 3) / 4));
    switch (tmvp_policy()) {
    case 1: hipLaunchKernelGGL((tmvp2_prescale_kernel<2, 0>), g, dim3(256), 0, s, a); break;
    case 2: hipLaunchKernelGGL((tmvp2_prescale_kernel<2, 2>), g, dim3(256), 0, s, a); break;
    case 3: hipLaunchKernelGGL((tmvp2_prescale_kernel<0, 2>), g, dim3(256), 0, s, a); break;
    default: hipLaunchKernelGGL((tmvp2_prescale_kernel<0, 0>), g, dim3(256), 0, s, a); break;
    }
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? NFEC_OK : hip_fail(e, "tmvp level-2 prescale launch");
}

int launch_tmvp2_postscale(const Rs16TmvpArgs& a, hipStream_t s)
{
    const uint64_t items = (uint64_t)a.nblocks * (a.vec / 8u);
    const uint64_t waves = (items + 511) / 512 * a.hw;
    if (!a.hw || !a.sc || items >= (1ull << 32) || waves >= (1ull << 32) || !tmvp2_offsets_fit(a)) return NFEC_ENOTSUP;
    if (waves == 0) return NFEC_OK;
    const dim3 g((uint32_t)((waves + 3) / 4));
    switch (tmvp_policy()) {
    case 1: hipLaunchKernelGGL((tmvp2_postscale_kernel<2, 0>), g, dim3(256), 0, s, a); break;
    case 2: hipLaunchKernelGGL((tmvp2_postscale_kernel<2, 2>), g, dim3(256), 0, s, a); break;
    case 3: hipLaunchKernelGGL((tmvp2_postscale_kernel<0, 2>), g, dim3(256), 0, s, a); break;
    default: hipLaunchKernelGGL((tmvp2_postscale_kernel<0, 0>), g, dim3(256), 0, s, a); break;
    }
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? NFEC_OK : hip_fail(e, "tmvp level-2 postscale launch");
}

int launch_tmvp_prescale(const Rs16TmvpArgs& a, hipStream_t s)
{
    const uint64_t items = (uint64_t)a.nblocks * (a.vec / 8u);
    const uint64_t waves = (items + 511) / 512 * (a.k / 2);
    // (the postscale's 32-bit offsets: checked here too, before anything is written)
    if (items >= (1ull << 32) || waves >= (1ull << 32) || !tmvp1_offsets_fit(a)) return NFEC_ENOTSUP;
    if (waves == 0) return NFEC_OK;
    hipLaunchKernelGGL(tmvp_prescale_kernel, dim3((uint32_t)((waves + 3) / 4)), dim3(256), 0, s, a);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? NFEC_OK : hip_fail(e, "tmvp prescale launch");
}

int launch_tmvp_postscale(const Rs16TmvpArgs& a, hipStream_t s)
{
    const uint64_t items = (uint64_t)a.nblocks * (a.vec / 8u);
    const uint64_t waves = (items + 511) / 512 * a.cw;
    if (items >= (1ull << 32) || waves >= (1ull << 32) || !tmvp1_offsets_fit(a)) return NFEC_ENOTSUP;
    if (waves == 0) return NFEC_OK;
    hipLaunchKernelGGL(tmvp_postscale_kernel, dim3((uint32_t)((waves + 3) / 4)), dim3(256), 0, s, a);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? NFEC_OK : hip_fail(e, "tmvp postscale launch");
}

namespace {

// RS16 decode stage 2 on the tower kernel (per-block mode, gen_gf16_tw.hip): block b's inverse
// A^-1 (coef2, column t = z row t, row s = erased output s) becomes the kernel's snippet table
// [t][sweep][s][2] as gf16_tw_offsets lays out an encode's generator (the kernel spreads the
// block's e rows over its passes itself), and the output rows' byte offsets row_off[b][s] =
// erased slot s * seg_stride.  One workgroup per block; columns at or past the block's column
// count (cols[b], else e) and rows at or past its e are never read.
__device__ __forceinline__ uint32_t gf8_mul_11d(uint32_t a, uint32_t b)
{
    uint32_t r = 0;
    for (int i = 0; i < 8; ++i) {
        if (b & 1u) r ^= a;
        b >>= 1;
        a <<= 1;
        if (a & 0x100u) a ^= 0x11du;
    }
    return r;
}

__global__ __launch_bounds__(256) void tw_dec_tables_kernel(TwDecTablesArgs a)
{
    // one workgroup per block: the e x e entries and the M + 12 row offsets
    const uint32_t b = blockIdx.x;
    const int32_t e = a.rows[b];
    uint32_t* ro = a.row_off + (uint64_t)b * (a.M + 12u);
    for (uint32_t r = threadIdx.x; r < a.M + 12u; r += blockDim.x)
        ro[r] = (int32_t)r < e ? (uint32_t)a.out_slots[(uint64_t)b * a.slots_stride + r] * a.seg_stride : 0u;
    if (e <= 0) return;
    const uint32_t ue = (uint32_t)e, nc = a.cols ? (uint32_t)a.cols[b] : ue;
    const uint16_t* c2 = a.coef2 + (uint64_t)b * (a.coef2_block ? a.coef2_block : (uint64_t)a.dcs * a.dcs);
    for (uint32_t idx = threadIdx.x; idx < nc * ue; idx += blockDim.x) {
        const uint32_t t = idx / ue, row = idx - t * ue;
        const uint32_t g = c2[(uint64_t)t * a.dcs + row];
        uint32_t tt = 0;
#pragma unroll
        for (int k = 0; k < 16; ++k)
            if ((g >> k) & 1u) tt ^= a.phi[k];
        const uint32_t c0 = tt & 255u, c1 = tt >> 8;
        uint32_t* col = reinterpret_cast<uint32_t*>(a.tw + (uint64_t)b * a.tw_block_stride + (uint64_t)t * 4u * a.M);
        col[row] = (c0 << 7) | (c1 << 23);
        col[a.M + row] = (gf8_mul_11d(a.lam, c1) << 7) | ((c0 ^ c1) << 23);
    }
}

}  // namespace

int launch_tw_dec_tables(const TwDecTablesArgs& a, hipStream_t s)
{
    if (a.nblocks == 0 || a.M == 0) return NFEC_OK;
    hipLaunchKernelGGL(tw_dec_tables_kernel, dim3(a.nblocks), dim3(256), 0, s, a);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? NFEC_OK : hip_fail(e, "tw decode tables launch");
}

}  // namespace nfec
