// kernels_gf16tail.hip -- the segment tails of the RS16 tower-kernel products.
//
// The tower kernel (gen_gf16_tw.hip) works in 8-byte lane pieces, so it covers the first
// vec & ~7 bytes of each segment.  NORM's vectors are segmentSize + 8 bytes (normSession.cpp:883)
// and RS16 codes vec / 2 symbols (normEncoderRS16.cpp:479), so a segment of e.g. 1452 bytes
// leaves 4 bytes (2 symbols) past the last piece.  This kernel computes those 1-3 symbols per
// segment with the same arguments, layouts and coefficient table as the tower kernel: the
// table's four GF(2^8) snippet entries of coefficient g are the tower product's constants,
//     phi(g x) = (c0 x0 + (lam c1) x1) + (c1 x0 + (c0 + c1) x1) y,   phi(x) = x0 + x1 y,
// so the products run through phi, GF(2^8) log / exp lookups and phi^-1 here.  One thread per
// (block, output row); the columns' tail symbols are read with uniform (scalar) loads.
#include "nfec_internal.hpp"

namespace nfec {

namespace {

struct Gf8Tables {
    uint8_t exp[512];
    uint8_t log[256];
};

constexpr Gf8Tables make_gf8_tables()
{
    Gf8Tables t{};
    uint32_t v = 1;
    for (uint32_t i = 0; i < 255; ++i) {
        t.exp[i] = (uint8_t)v;
        t.exp[i + 255] = (uint8_t)v;
        t.log[v] = (uint8_t)i;
        v <<= 1;
        if (v & 0x100u) v ^= 0x11du;  // the RS8 field, the tower's base field
    }
    t.exp[510] = t.exp[511] = 0;
    return t;
}

__constant__ Gf8Tables kGf8Tables = make_gf8_tables();

struct TailConsts {
    uint16_t phi[16], phi_inv[16];
};

constexpr uint32_t kTailRowsPerWg = 64;
constexpr uint32_t kTailMaxSym = 3;
constexpr uint32_t kNoLog = 0xffffu;

__global__ __launch_bounds__(kTailRowsPerWg) void gf16_tw_tail_kernel(Gf16T3Args a, uint32_t off, uint32_t nsym,
                                                                      TailConsts tc)
{
    __shared__ uint8_t ex[512];
    __shared__ uint16_t lg[256];
    __shared__ uint16_t ph0[256], ph1[256], pi0[256], pi1[256];  // phi / phi^-1 of the low / high byte
    const uint32_t lane = threadIdx.x;
    const uint32_t wpb = (a.m + kTailRowsPerWg - 1u) / kTailRowsPerWg;
    const uint32_t blk = blockIdx.x / wpb, rchunk = blockIdx.x - blk * wpb;
    if (blk >= a.nblocks) return;
    // rows and columns of this block, as the tower kernel takes them
    const bool pb = a.blk_rows != nullptr;
    uint32_t rlim = a.m, kk = a.k, nd = a.k;
    if (a.rows_lim) rlim = min(rlim, *a.rows_lim);
    if (pb) {
        const int32_t e = a.blk_rows[blk];
        rlim = e > 0 ? min(rlim, (uint32_t)e) : 0u;
        kk = a.blk_cols ? min(kk, (uint32_t)a.blk_cols[blk]) : min(kk, rlim);
    } else if (a.num_data) {
        nd = a.num_data[blk];
        if (nd < 1u || nd > a.k) return;  // left alone, as the tower kernel does
        kk = nd;
    }
    if (rlim == 0u || kk == 0u || rchunk * kTailRowsPerWg >= rlim) return;  // workgroup-uniform
    for (uint32_t i = lane; i < 512; i += kTailRowsPerWg) ex[i] = kGf8Tables.exp[i];
    for (uint32_t i = lane; i < 256; i += kTailRowsPerWg) {
        lg[i] = i ? kGf8Tables.log[i] : (uint16_t)kNoLog;
        uint32_t f0 = 0, f1 = 0, g0 = 0, g1 = 0;
        for (int j = 0; j < 8; ++j)
            if ((i >> j) & 1u) f0 ^= tc.phi[j], f1 ^= tc.phi[8 + j], g0 ^= tc.phi_inv[j], g1 ^= tc.phi_inv[8 + j];
        ph0[i] = (uint16_t)f0, ph1[i] = (uint16_t)f1, pi0[i] = (uint16_t)g0, pi1[i] = (uint16_t)g1;
    }
    __syncthreads();
    const uint32_t r = rchunk * kTailRowsPerWg + lane;
    const bool live = r < rlim;
    const uint8_t* in = a.base + (uint64_t)blk * a.block_stride + off;
    const uint16_t* tab = a.tw + (pb ? (uint64_t)blk * a.tw_block_stride : 0u);
    uint32_t acc0[kTailMaxSym] = {0, 0, 0}, acc1[kTailMaxSym] = {0, 0, 0};
    // columns in batches of 8, their loads issued together (the loop is latency-bound otherwise):
    // a column's tail symbols as one 8-byte load (the segment stride is a multiple of 8 and at
    // least vec, so the 8 bytes at the tail offset stay inside the slot), uniform across the
    // workgroup; the row's two table dwords
    const uint32_t* tab32 = reinterpret_cast<const uint32_t*>(tab);
    for (uint32_t c0 = 0; c0 < kk; c0 += 8u) {
        uint2 xv[8];
        uint32_t e0[8], e1[8];
#pragma unroll
        for (uint32_t j = 0; j < 8u; ++j) {
            const uint32_t c = min(c0 + j, kk - 1u);
            xv[j] = *reinterpret_cast<const uint2*>(in + (uint64_t)c * a.seg_stride);
            const uint64_t eb = ((uint64_t)c * 4u * a.m + 2u * r) / 2u;  // dword index of (c, sweep 0, r)
            e0[j] = live ? tab32[eb] : 0u;
            e1[j] = live ? tab32[eb + a.m] : 0u;
        }
#pragma unroll
        for (uint32_t j = 0; j < 8u; ++j) {
            if (c0 + j >= kk) break;
            // the column's tail symbols in the tower basis
            uint32_t lx0[kTailMaxSym], lx1[kTailMaxSym];
#pragma unroll
            for (uint32_t s = 0; s < kTailMaxSym; ++s) {
                const uint32_t w = s < 2u ? xv[j].x : xv[j].y;
                const uint32_t v = s < nsym ? (w >> (16u * (s & 1u))) & 0xFFFFu : 0u;
                const uint32_t t = (uint32_t)ph0[v & 255u] ^ (uint32_t)ph1[v >> 8];
                lx0[s] = lg[t & 255u];
                lx1[s] = lg[t >> 8];
            }
            // entries (c0, c1) of sweep 0 and (lam c1, c0 ^ c1) of sweep 1, each (value << 7)
            const uint32_t l00 = lg[(e0[j] >> 7) & 255u], l01 = lg[e0[j] >> 23];  // x0 -> out0, out1
            const uint32_t l10 = lg[(e1[j] >> 7) & 255u], l11 = lg[e1[j] >> 23];  // x1 -> out0, out1
#pragma unroll
            for (uint32_t s = 0; s < kTailMaxSym; ++s) {
                const uint32_t a0 = lx0[s], a1 = lx1[s];
                if (a0 != kNoLog) {
                    if (l00 != kNoLog) acc0[s] ^= ex[a0 + l00];
                    if (l01 != kNoLog) acc1[s] ^= ex[a0 + l01];
                }
                if (a1 != kNoLog) {
                    if (l10 != kNoLog) acc0[s] ^= ex[a1 + l10];
                    if (l11 != kNoLog) acc1[s] ^= ex[a1 + l11];
                }
            }
        }
    }
    if (!live) return;
    uint8_t* out;
    const uint8_t* accsrc = nullptr;
    if (pb) {
        out = a.out_base + (uint64_t)blk * a.out_block_stride + a.row_off[(uint64_t)blk * a.row_off_stride + r] + off;
    } else {
        out = a.out_base + (uint64_t)blk * a.out_block_stride +
              (uint64_t)(a.out_slot0 + (a.out_after_data ? nd : 0u) + r) * a.out_seg_stride + off;
        if (a.accumulate)
            accsrc = a.acc_base + (uint64_t)blk * a.acc_block_stride +
                     (uint64_t)(a.acc_slot0 + (a.acc_after_data ? nd : 0u) + r) * a.acc_seg_stride + off;
    }
    for (uint32_t s = 0; s < nsym; ++s) {
        uint32_t v = (uint32_t)pi0[acc0[s]] ^ (uint32_t)pi1[acc1[s]];
        if (accsrc) v ^= reinterpret_cast<const uint16_t*>(accsrc)[s];
        reinterpret_cast<uint16_t*>(out)[s] = (uint16_t)v;
    }
}

}  // namespace

bool gf16_tw_tail_covers(const Gf16T3Args& in, uint32_t bytes)
{
    if (bytes == 0) return true;
    return !((bytes & 1u) || bytes > 2u * kTailMaxSym || !in.tw || in.k == 0 || in.m == 0 || in.col_chunk ||
             (in.num_data && in.blk_rows) || (in.blk_rows && (!in.row_off || !in.tw_block_stride || in.accumulate)));
}

int launch_gf16_tw_tail(const Gf16T3Args& in, uint32_t off, uint32_t bytes, hipStream_t s)
{
    if (in.nblocks == 0 || bytes == 0) return NFEC_OK;
    if ((off & 1u) || !gf16_tw_tail_covers(in, bytes)) return NFEC_ENOTSUP;
    Gf16T3Args a = in;
    // default layouts, as the tower kernel's launcher fills them (encode: parity in place)
    if (!a.out_base) {
        a.out_base = const_cast<uint8_t*>(in.base);
        a.out_block_stride = in.block_stride;
        a.out_seg_stride = in.seg_stride;
        a.out_slot0 = in.num_data ? 0u : in.k;
        a.out_after_data = in.num_data ? 1u : 0u;
    }
    if (!a.acc_base) {
        a.acc_base = a.out_base;
        a.acc_block_stride = a.out_block_stride;
        a.acc_seg_stride = a.out_seg_stride;
        a.acc_slot0 = a.out_slot0;
        a.acc_after_data = a.out_after_data;
    }
    if (!in.num_data) a.out_after_data = a.acc_after_data = 0u;
    TailConsts tc;
    uint32_t lam = 0;
    gf16_tw_field(tc.phi, &lam, tc.phi_inv);
    const uint64_t wgs = (uint64_t)a.nblocks * ((a.m + kTailRowsPerWg - 1u) / kTailRowsPerWg);
    if (wgs >= (1ull << 31)) return NFEC_ENOTSUP;
    hipLaunchKernelGGL(gf16_tw_tail_kernel, dim3((uint32_t)wgs), dim3(kTailRowsPerWg), 0, s, a, off, bytes / 2u, tc);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? NFEC_OK : hip_fail(e, "gf16 tower tail launch");
}

}  // namespace nfec
