// bitslice.hpp -- device helpers for the bit-sliced GF(2^8) kernels (generated code).
//
// A lane owns 32 byte positions of a segment (4 items of 8 bytes, each item index
// = item_base + i*64 + lane so every wave-wide load is one contiguous 512-byte run).
// The 32 bytes are held as 8 dwords w[0..7] and transposed into 8 bit-planes X[0..7]
// (per byte column q: an 8x8 bit transpose of the bytes of the 8 dwords), so that plane
// X_b bit (8q+d) = bit b of byte q of dword d.  Multiplying every byte by a constant c is
// then the GF(2) 8x8 matrix of c applied to the planes (XORs only); the transpose is an
// involution, so the same network maps parity planes back to bytes.
#pragma once

#include "nfec_internal.hpp"

namespace nfec {
namespace bs {

__device__ __forceinline__ uint32_t x3(uint32_t a, uint32_t b, uint32_t c)
{
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// accumulator XOR as an opaque op: keeps LLVM's reassociation from regrouping the long
// per-accumulator XOR chains across source columns (that blows up register pressure)
__device__ __forceinline__ uint32_t x2(uint32_t a, uint32_t b)
{
    uint32_t r;
    asm("v_xor_b32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

// bit-select: (m & a) | (~m & b)
__device__ __forceinline__ uint32_t sel(uint32_t m, uint32_t a, uint32_t b)
{
    return __builtin_amdgcn_bitop3_b32(m, a, b, 0xca);
}

// swap M[r][c+s] <-> M[r+s][c] for the bit columns selected by mask (per byte)
template <int S, uint32_t MASK>
__device__ __forceinline__ void swapmove(uint32_t& lo, uint32_t& hi)
{
    const uint32_t u = lo >> S;   // lo's high columns moved down
    const uint32_t v = hi << S;   // hi's low columns moved up
    hi = sel(MASK, u, hi);
    lo = sel(MASK << S, v, lo);
}

// 8x8 bit transpose in each of the 4 byte columns of w[0..7] (involution).
__device__ __forceinline__ void transpose8(uint32_t& w0, uint32_t& w1, uint32_t& w2, uint32_t& w3, uint32_t& w4,
                                           uint32_t& w5, uint32_t& w6, uint32_t& w7)
{
    swapmove<4, 0x0F0F0F0Fu>(w0, w4);
    swapmove<4, 0x0F0F0F0Fu>(w1, w5);
    swapmove<4, 0x0F0F0F0Fu>(w2, w6);
    swapmove<4, 0x0F0F0F0Fu>(w3, w7);
    swapmove<2, 0x33333333u>(w0, w2);
    swapmove<2, 0x33333333u>(w1, w3);
    swapmove<2, 0x33333333u>(w4, w6);
    swapmove<2, 0x33333333u>(w5, w7);
    swapmove<1, 0x55555555u>(w0, w1);
    swapmove<1, 0x55555555u>(w2, w3);
    swapmove<1, 0x55555555u>(w4, w5);
    swapmove<1, 0x55555555u>(w6, w7);
}

// Buffer descriptor over a wave-uniform base: loads/stores then take a 32-bit VGPR offset
// (the item) plus an SGPR offset (the slot), so no 64-bit address arithmetic per column.
// num_records = 2^32-1: the launchers keep every offset a wave uses below 2^31.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, -1, 0x00020000);
}

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// a wave's items span at most 3 blocks and 256 slots: every buffer offset stays < 2^31
inline bool offsets_fit(uint64_t block_stride, uint64_t seg_stride)
{
    return 3 * block_stride + 256 * seg_stride < (1ull << 31);
}

__device__ __forceinline__ uint2 bld8(__amdgpu_buffer_rsrc_t rs, uint32_t voff, uint32_t soff)
{
    const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(rs, voff, soff, 0);
    return make_uint2(v.x, v.y);
}

struct EncArgs {
    const uint8_t* base = nullptr;   // block 0 slot 0
    uint8_t* out = nullptr;          // parity destination base (== base for in-place encode)
    uint64_t block_stride = 0;
    uint32_t seg_stride = 0;
    uint32_t nblocks = 0;
    uint32_t vec = 0;
    const uint16_t* num_data = nullptr;  // per block (null: k)
    uint32_t accumulate = 0;
    uint32_t xcd_remap = 0;   // nonzero: give each XCD a contiguous range of workgroups
    uint32_t nt_store = 0;    // nonzero: nontemporal parity stores
};

// per-lane item geometry for the 4 items of a lane (all blocks hold k source symbols; the
// bit-sliced kernels are only used for unshortened batches).  Addresses are a wave-uniform
// base (the first block the wave touches) plus 32-bit per-lane offsets, so every load is a
// global_load with an SGPR base: no 64-bit per-lane pointer arithmetic per column.
struct Items {
    const uint8_t* wbase;   // uniform: slot 0 of the wave's first block
    uint8_t* obase;         // uniform: same block in the output batch
    __amdgpu_buffer_rsrc_t rs;   // buffer descriptors over wbase / obase (32-bit offsets)
    __amdgpu_buffer_rsrc_t ors;
    uint32_t off[4];        // per lane: byte offset of item i (clamped to a valid item)
    uint32_t nbytes[4];     // valid bytes in the item (0 if out of range, <8 for the tail)
};

__device__ __forceinline__ void make_items(const EncArgs& a, uint32_t item_base, uint32_t lane, Items& it)
{
    const uint32_t ips = (a.vec + 7) >> 3;
    const uint32_t total = a.nblocks * ips;  // launcher guarantees < 2^31
    const uint32_t b0 = __builtin_amdgcn_readfirstlane(min(item_base, total - 1) / ips);
    it.wbase = a.base + (uint64_t)b0 * a.block_stride;
    it.obase = a.out + (uint64_t)b0 * a.block_stride;
    it.rs = rsrc(it.wbase);
    it.ors = rsrc(it.obase);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t g = item_base + (uint32_t)i * 64u + lane;
        const bool ok = g < total;
        const uint32_t gg = ok ? g : item_base;
        const uint32_t b = gg / ips;
        const uint32_t o = gg - b * ips;
        it.off[i] = (uint32_t)((b - b0) * a.block_stride) + o * 8u;
        it.nbytes[i] = ok ? min(8u, a.vec - o * 8u) : 0u;
    }
}

// decode stage 1 (re-encode of the surviving source with the erased columns masked out)
struct DecArgs {
    const uint8_t* base = nullptr;
    uint64_t block_stride = 0;
    uint32_t seg_stride = 0;
    uint32_t nblocks = 0;
    uint32_t vec = 0;
    const uint32_t* emask = nullptr;  // [b][2] erased source columns
    const uint32_t* psel = nullptr;   // [b][2] parity rows used
    const uint8_t* pmap = nullptr;    // [b][m] row -> index t in P
    uint8_t* z = nullptr;             // [b][cs][z_stride] stage-1 output z_t
    uint64_t z_block_stride = 0;
    uint32_t z_stride = 0;
    uint32_t xcd_remap = 0;
    const uint32_t* gate = nullptr;   // non-null: skip the launch unless *gate == gate_gen
    uint32_t gate_gen = 0;            // (RsPlan2Args::gate)
    const uint16_t* num_data = nullptr;  // per block (null: k): parity row p at slot numData + p
};

// Workgroup -> work index.  The dispatcher deals workgroups round-robin over the 8 XCDs
// (each with its own L2); with remap on, XCD x gets the contiguous index range
// [x*q + min(x, r), ...) so neighbouring items (which share 128-byte lines at their
// boundaries) are fetched through one L2 instead of two.
__device__ __forceinline__ uint32_t wg_index(uint32_t remap)
{
    const uint32_t bid = blockIdx.x;
    if (!remap) return bid;
    constexpr uint32_t kXcd = 8;
    const uint32_t n = gridDim.x, q = n / kXcd, r = n % kXcd;
    const uint32_t x = bid % kXcd, i = bid / kXcd;
    return x < r ? x * (q + 1) + i : r * (q + 1) + (x - r) * q + i;
}

// LDS byte address (what ds_read/ds_write take) of a __shared__ object
__device__ __forceinline__ uint32_t lds_addr(const void* p)
{
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

struct DecItems {
    const uint8_t* wbase;   // uniform: slot 0 of the wave's first block
    __amdgpu_buffer_rsrc_t rs;   // num_records = 2^31: offsets with bit 31 set read as zero
    uint32_t item_base;     // uniform
    uint32_t off[4];        // per lane: byte offset of item i from wbase (slot 0)
    uint32_t em0[4], em1[4];  // erased source columns of item i's block
    uint32_t need;          // OR of the used parity rows of the lane's blocks
};

// per-item data only the z stores need: rebuilt after the column loop so it is not live
// across it
struct DecTail {
    uint32_t blk[4];        // absolute block index of item i
    uint32_t ib[4];         // byte offset of item i inside a segment
    uint32_t nbytes[4];
    uint32_t sel[4];        // parity rows used by item i's block (m <= 32)
};

__device__ __forceinline__ void make_dec_items(const DecArgs& a, uint32_t item_base, uint32_t lane, DecItems& it)
{
    const uint32_t ips = (a.vec + 7) >> 3;
    const uint32_t total = a.nblocks * ips;
    const uint32_t b0 = __builtin_amdgcn_readfirstlane(min(item_base, total - 1) / ips);
    it.wbase = a.base + (uint64_t)b0 * a.block_stride;
    it.rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(it.wbase), (short)0, (int)0x80000000u, 0x00020000);
    it.item_base = item_base;
    it.need = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t g = item_base + (uint32_t)i * 64u + lane;
        const bool ok = g < total;
        const uint32_t gg = ok ? g : item_base;
        const uint32_t b = gg / ips;
        const uint32_t o = gg - b * ips;
        it.off[i] = (uint32_t)((b - b0) * a.block_stride) + o * 8u;
        it.em0[i] = a.emask[2 * (uint64_t)b];
        it.em1[i] = a.emask[2 * (uint64_t)b + 1];
        it.need |= ok ? a.psel[2 * (uint64_t)b] : 0u;
    }
}

__device__ __forceinline__ void make_dec_tail(const DecArgs& a, const DecItems& it, DecTail& tl)
{
    const uint32_t lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
    const uint32_t ips = (a.vec + 7) >> 3;
    const uint32_t total = a.nblocks * ips;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t g = it.item_base + (uint32_t)i * 64u + lane;
        const bool ok = g < total;
        const uint32_t gg = ok ? g : it.item_base;
        const uint32_t b = gg / ips;
        const uint32_t o = gg - b * ips;
        tl.blk[i] = b;
        tl.ib[i] = o * 8u;
        tl.nbytes[i] = ok ? min(8u, a.vec - o * 8u) : 0u;
        tl.sel[i] = ok ? a.psel[2 * (uint64_t)b] : 0u;
    }
}

// Load offset of item (offset o) in source column j: erased columns get bit 31 set, which
// puts the access past the decode descriptor's num_records (2^31), so the buffer load
// returns zeros without touching memory -- masking and skipping in one VALU op.
template <int J>
__device__ __forceinline__ uint32_t dec_off(uint32_t o, uint32_t em0, uint32_t em1)
{
    const uint32_t t = J < 32 ? (em0 << (31 - J)) : (em1 << (63 - J));
    return __builtin_amdgcn_bitop3_b32(t, 0x80000000u, o, 0xEA);  // (t & bit31) | o
}

__device__ __forceinline__ uint2 ld8(const uint8_t* base, uint32_t off)
{
    return *reinterpret_cast<const uint2*>(base + off);
}

__device__ __forceinline__ void st8(uint8_t* p, uint32_t x, uint32_t y, uint32_t nbytes, uint32_t accumulate)
{
    if (nbytes == 0) return;
    if (accumulate) {
        const uint2 o = *reinterpret_cast<const uint2*>(p);
        x ^= o.x;
        y ^= o.y;
    }
    if (nbytes >= 8) {
        *reinterpret_cast<uint2*>(p) = make_uint2(x, y);
    } else {
        for (uint32_t i = 0; i < nbytes; ++i) p[i] = (uint8_t)((i < 4 ? x : y) >> (8 * (i & 3)));
    }
}

// parity store through the output descriptor (full items), byte stores for the tail
__device__ __forceinline__ void bst8(const Items& it, uint32_t voff, uint32_t soff, uint32_t x, uint32_t y,
                                     uint32_t nbytes, uint32_t accumulate, uint32_t nt)
{
    if (nbytes >= 8 && !accumulate) {
        u32x2 v;
        v.x = x;
        v.y = y;
        if (nt) __builtin_amdgcn_raw_buffer_store_b64(v, it.ors, voff, soff, 2);
        else __builtin_amdgcn_raw_buffer_store_b64(v, it.ors, voff, soff, 0);
        return;
    }
    st8(it.obase + soff + voff, x, y, nbytes, accumulate);
}

}  // namespace bs

// generated (gen_rs8_bitsliced.hip): NFEC_ENOTSUP when (k, m) has no specialised kernel or
// the batch is shortened (per-block numData)
int launch_rs8_bitsliced_encode(uint32_t k, uint32_t m, const bs::EncArgs& a, hipStream_t s);
// gen_rs8_asm.hip: hand-allocated assembly bodies; NFEC_ENOTSUP for tails / shortened batches
int launch_rs8_asm_encode(uint32_t k, uint32_t m, const bs::EncArgs& a, hipStream_t s);
// gen_rs8_asm.hip: MDP encode of full blocks with the same assembly bodies (NFEC_ENOTSUP otherwise)
int launch_mdp_asm_encode(uint32_t k, uint32_t m, const bs::EncArgs& a, hipStream_t s);
// gen_rs8_q4.hip: 4 role waves per workgroup sharing each column's transpose through LDS
int launch_rs8_q4_encode(uint32_t k, uint32_t m, const bs::EncArgs& a, hipStream_t s);
int launch_mdp_q4_encode(uint32_t k, uint32_t m, const bs::EncArgs& a, hipStream_t s);
int launch_rs8_bitsliced_reencode(uint32_t k, uint32_t m, const bs::DecArgs& a, hipStream_t s);
int bitsliced_encode_generator(uint32_t k, uint32_t m, uint8_t* out);

}  // namespace nfec
