// nfec_internal.hpp -- shared declarations of the MI355X FEC engine (not part of the ABI).
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <atomic>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/nfec.h"

namespace nfec {

// ---------------------------------------------------------------------------------
// Error plumbing: the ABI never throws; failures set a thread-local message.
// ---------------------------------------------------------------------------------
void set_error(const std::string& msg);
const char* last_error_cstr();  // this thread's last message
int fail(int code, const std::string& msg);
int hip_fail(hipError_t e, const char* what);

#define NFEC_HIP(call)                                    \
    do {                                                  \
        hipError_t e_ = (call);                           \
        if (e_ != hipSuccess) return ::nfec::hip_fail(e_, #call); \
    } while (0)

// A/B switches between correct alternative paths (kernels on or off, tuning choices).  Only
// the diagnostic library (make -C norm_amd diag, -DNFEC_DIAG) reads them from the
// environment; the product library always takes the default, so no stray variable changes
// what it runs.  Values outside [lo, hi] fall back to the default.
inline long diag_knob(const char* name, long def, long lo = 0, long hi = 1)
{
#if defined(NFEC_DIAG) || defined(NFEC_KNOBS)  // (NFEC_KNOBS: an A/B build of the product kernels, tools/ab_build.sh)
    const char* e = std::getenv(name);
    if (!e || !*e) return def;
    const long v = std::strtol(e, nullptr, 0);
    return v < lo || v > hi ? def : v;
#else
    (void)name, (void)lo, (void)hi;
    return def;
#endif
}

// ---------------------------------------------------------------------------------
// Host worker pool (host_pool.cpp): one per process, sized to the cores the job may use (the
// affinity mask capped by the cgroup cpu.max quota; NFEC_HOST_THREADS overrides, at most 64).
// host_parallel_for runs fn(0..n-1) on it and returns when all are done; every host-batch copy
// of every codec and stripe shares these workers, so N stripes never put more than
// host_pool_size() copy threads on the cores.
// ---------------------------------------------------------------------------------
unsigned host_visible_cores();
unsigned host_usable_cores();
unsigned host_pool_size();
unsigned host_pool_workers();  // workers actually running (starts the pool)
unsigned host_pool_max_active(bool reset);  // most pool pieces that ran at once (since the last reset)
// returns NFEC_OK, or the status of the first piece that threw (NFEC_ENOMEM for std::bad_alloc,
// NFEC_EINVAL for anything else; nfec_last_error names it) after every piece has run
[[nodiscard]] int host_parallel_for(unsigned n, const std::function<void(unsigned)>& fn);

// ---------------------------------------------------------------------------------
// Host field arithmetic (gf_host.cpp).  GF(2^8) on 0x11d and GF(2^16) on 0x1100B with
// alpha = x, exactly the fields of normEncoderRS8.cpp:81 / normEncoderRS16.cpp:88.
// ---------------------------------------------------------------------------------
struct Field {
    int bits = 0;
    uint32_t q = 0;                 // 2^bits - 1
    std::vector<uint32_t> exp;      // 2q entries (exp[i] = alpha^(i mod q))
    std::vector<uint32_t> log;      // q+1 entries, log[0] = q
    uint32_t mul(uint32_t a, uint32_t b) const { return (a && b) ? exp[log[a] + log[b]] : 0; }
    uint32_t inv(uint32_t a) const { return a <= 1 ? a : exp[q - log[a]]; }
    uint32_t div(uint32_t a, uint32_t b) const { return a ? exp[log[a] + q - log[b]] : 0; }
};
const Field& gf8();
const Field& gf16();

// Systematic generator parity rows (m x k, row-major) of the reference's Rizzo code, built
// in closed (Lagrange) form; identical to Vandermonde-invert-and-multiply because the
// systematic matrix is unique for the reference's evaluation points.
int rs_generator(int bits, uint32_t k, uint32_t m, std::vector<uint32_t>& parity_rows);
// Evaluation point of generator row r (0 -> 0, r >= 1 -> alpha^(r-1)).
inline uint32_t rs_point(const Field& f, uint32_t row) { return row == 0 ? 0u : f.exp[(row - 1) % f.q]; }

// MDP: generator polynomial (normEncoderMDP.cpp:102-170) and the linear map of the
// in-order LFSR encoder for a block of nd source symbols (m x nd, row-major).
void mdp_generator_poly(uint32_t m, std::vector<uint8_t>& g);
void mdp_encode_matrix(const std::vector<uint8_t>& g, uint32_t m, uint32_t nd, uint8_t* out);

// host_gf8.cpp: dst ^= c * src over n bytes on the host CPU (isa: NFEC_HOST_GF_*, < 0 best)
void host_gf8_addmul(uint8_t* dst, const uint8_t* src, uint32_t c, size_t n, int isa);
// ... and over nsym 16-bit symbols in the RS16 field (GFNI or scalar)
void host_gf16_addmul(uint16_t* dst, const uint16_t* src, uint32_t c, size_t nsym, int isa);
int host_gf8_isa();
// dst[0..n) = (acc ? dst : 0) + sum_j coef[j] * src[j][off + 0..n) (GF(2^8) bytes / GF(2^16)
// symbols; off and n in elements); the host repair's row products
void host_gf8_dot(uint8_t* dst, const uint8_t* const* src, size_t off, const uint16_t* coef, uint32_t nc, size_t n,
                  bool acc, int isa);
void host_gf16_dot(uint16_t* dst, const uint16_t* const* src, size_t off, const uint16_t* coef, uint32_t nc,
                   size_t nsym, bool acc, int isa);
// dst[r][0..n) ^= coef[r * cstride] * src[0..n) for r < nrows (the per-segment Encode's m rows)
void host_gf8_addmul_rows(uint8_t* const* dst, const uint8_t* src, const uint32_t* coef, size_t cstride, uint32_t nrows,
                          size_t n, int isa);
void host_gf16_addmul_rows(uint16_t* const* dst, const uint16_t* src, const uint32_t* coef, size_t cstride,
                           uint32_t nrows, size_t nsym, int isa);
// one MDP encoder step (normEncoderMDP.cpp:178-211) over n bytes: s = data ^ P0,
// P_i = P_(i+1) ^ g[m-1-i] * s for i < m-1, P_(m-1) = g[0] * s (g: the generator polynomial)
void host_mdp_step(uint8_t* const* parity, const uint8_t* data, const uint8_t* g, uint32_t m, size_t n, int isa);

// v_perm product tables for one GF(2^8) constant c: 8 dwords (32 bytes)
//   t0 = c*{0,1,2,3}   t1 = c*{4,5,6,7}       (low 3 bits)
//   t2 = c*{0,8,16,24} t3 = c*{32,40,48,56}   (middle 3 bits)
//   t4 = c*{0,64,128,192}                     (top 2 bits), t5..t7 = 0
void vperm_table(uint32_t c, uint32_t out[8]);

// ---------------------------------------------------------------------------------
// Device kernels (launchers live next to the kernels).
// ---------------------------------------------------------------------------------
enum OutSlotMode : uint32_t {
    OUT_SLOT_LIST = 0,      // slot = out_slots[b][r]
    OUT_SLOT_AFTER_INPUT = 1,// slot = in_count(b) + r   (parity after the block's numData sources)
    OUT_SLOT_ROW = 2        // slot = r
};

// Generic batched GF(2^8) matrix product over segment vectors:
//   out[b][slot_out(r)] (^)= sum_c coef[b][c][r] * in[b][slot_in(c)]   for r < rows(b), c < cols(b)
struct Gf8MatmulArgs {
    const uint8_t* in_base = nullptr;
    uint64_t in_block_stride = 0;
    uint32_t in_seg_stride = 0;
    const uint16_t* in_slots = nullptr;  // [b*slots_stride + c] or null (identity)
    const uint16_t* in_count = nullptr;  // per block column count or null (cols_const)
    uint32_t cols_const = 0;
    uint8_t* out_base = nullptr;
    uint64_t out_block_stride = 0;
    uint32_t out_seg_stride = 0;
    const uint16_t* out_slots = nullptr; // [b*slots_stride + r]
    uint32_t out_slot_mode = OUT_SLOT_AFTER_INPUT;
    const int32_t* row_count = nullptr;  // per block rows (<=0: skip block) or null (rows_const)
    uint32_t rows_const = 0;
    uint32_t slots_stride = 0;
    const uint8_t* coef = nullptr;       // coef[b*coef_block_stride + c*coef_col_stride + r]
    uint64_t coef_block_stride = 0;
    uint32_t coef_col_stride = 0;
    const uint32_t* vtab = nullptr;      // 256 x 8 dword v_perm tables (device)
    uint32_t coef_by_count = 0;          // coef block = coef + (cols(b)-1)*coef_block_stride (MDP encode)
    uint32_t nblocks = 0;
    uint32_t vec_bytes = 0;
    uint32_t accumulate = 0;
};
int launch_gf8_matmul(const Gf8MatmulArgs& a, bool shared_coef, hipStream_t s);

// per-block square solve: out[b][out_slots[b][r]] (^)= XOR_t coef[b][t][r] (x) z[b][t]
// (rows(b) <= 16, cols(b) <= 32; NFEC_ENOTSUP beyond)
struct Gf8SolveArgs {
    const uint8_t* z = nullptr;
    uint64_t z_block_stride = 0;
    uint32_t z_stride = 0;
    const uint16_t* cols = nullptr;      // per block: z rows used
    const int32_t* rows = nullptr;       // per block: outputs (<= 0: skip block)
    const uint16_t* out_slots = nullptr; // [b*slots_stride + r]
    uint32_t slots_stride = 0;
    uint8_t* out = nullptr;
    uint64_t out_block_stride = 0;
    uint32_t out_seg_stride = 0;
    const uint8_t* coef = nullptr;       // coef[b*coef_block_stride + t*coef_col_stride + r]
    uint64_t coef_block_stride = 0;
    uint32_t coef_col_stride = 0;
    const uint32_t* vtab = nullptr;
    uint32_t nblocks = 0;
    uint32_t vec_bytes = 0;
    uint32_t accumulate = 0;
    int32_t min_rows = 0;                // skip blocks with rows <= min_rows (done by another kernel)
    const uint32_t* gate = nullptr;      // non-null: skip the launch unless *gate == gate_gen
    uint32_t gate_gen = 0;
};
int launch_gf8_solve(const Gf8SolveArgs& a, uint32_t max_rows, uint32_t max_cols, hipStream_t s);
// gen_solve_asm.hip: bit-sliced solve for blocks with rows <= 16 (NFEC_ENOTSUP: other shapes)
int launch_gf8_solve_bs(const Gf8SolveArgs& a, hipStream_t s);

// GF(2^16) variant (log/exp); coef holds generator elements (uint16) at the same indexing.
struct Gf16MatmulArgs {
    const uint8_t* in_base = nullptr;
    uint64_t in_block_stride = 0;
    uint32_t in_seg_stride = 0;
    const uint16_t* in_slots = nullptr;
    const uint16_t* in_count = nullptr;
    uint32_t cols_const = 0;
    uint8_t* out_base = nullptr;
    uint64_t out_block_stride = 0;
    uint32_t out_seg_stride = 0;
    const uint16_t* out_slots = nullptr;
    uint32_t out_slot_mode = OUT_SLOT_AFTER_INPUT;
    const int32_t* row_count = nullptr;
    uint32_t rows_const = 0;
    uint32_t slots_stride = 0;
    const uint16_t* coef = nullptr;      // element values (0 allowed)
    uint32_t coef_by_count = 0;
    uint64_t coef_block_stride = 0;
    uint32_t coef_col_stride = 0;
    const uint16_t* exp_tab = nullptr;   // device exp table, 2q entries
    const uint16_t* log_tab = nullptr;   // device log table, q+1 entries (log 0 = q)
    uint32_t nblocks = 0;
    uint32_t vec_bytes = 0;              // even number of bytes processed
    uint32_t accumulate = 0;
};
int launch_gf16_matmul(const Gf16MatmulArgs& a, hipStream_t s);

// RS16 encode, bit-sliced with per-lane four-Russians tables in LDS (kernels_gf16bs.hip).
// In and out share the batch layout; parity row r goes to slot numData_b + r.
struct Gf16BsEncArgs {
    const uint8_t* base = nullptr;
    uint8_t* out_base = nullptr;
    uint64_t block_stride = 0;
    uint32_t seg_stride = 0;
    uint32_t nblocks = 0;
    const uint16_t* num_data = nullptr;  // per block or null (k)
    uint32_t k = 0, m = 0;
    uint32_t vec_bytes = 0;              // even
    uint32_t chunks = 0;                 // 64-byte chunks per segment
    const uint16_t* sel = nullptr;       // [k][m_pad][64] table offsets (gf16_bs_selectors)
    uint32_t m_pad = 0;                  // gf16_bs_rows_padded(m)
    uint32_t accumulate = 0;
};
inline uint32_t gf16_bs_rows_padded(uint32_t m) { return (m + 7u) & ~7u; }

// RS16 encode, bit-sliced with three shared four-Russians tables per column (gen_gf16_t3.hip):
// one builder wave + 11 row waves of 4 parity rows per workgroup, 44 rows per pass.
struct Gf16T3Args {
    const uint8_t* base = nullptr;       // batch (parity written in place, slot k + r)
    uint64_t block_stride = 0;
    uint32_t seg_stride = 0;
    uint32_t nblocks = 0;
    // per block numData (tower kernel, flat mode only: columns whose source slot -- through the
    // column map -- is at or past it read as zeros; the shared-table kernel takes unshortened
    // batches only).  nd_limit: the largest valid numData (0: k; the Toeplitz split's products
    // have k >> L columns but mask the codec's k source slots); nd_outputs_only: numData only
    // places the output / accumulate rows (out_after_data), the loads are not masked (products
    // over scratch columns)
    const uint16_t* num_data = nullptr;
    uint32_t nd_limit = 0, nd_outputs_only = 0;
    uint32_t k = 0, m = 0, m_pad = 0;    // m_pad = gf16_t3_rows_padded(m)
    uint32_t vec_bytes = 0;              // multiple of 8
    const uint16_t* offs = nullptr;      // [k + 1][m_pad][48] LDS offsets (gf16_t3_offsets)
    uint32_t accumulate = 0;
    uint32_t passes = 0;                 // set by the launcher
    // output and accumulate-source layouts (null: parity in place, slot k + r, as encode does);
    // decode stage 1 writes z rows (slot r of a z batch) XORed with the received parity row
    uint8_t* out_base = nullptr;
    uint64_t out_block_stride = 0;
    uint32_t out_seg_stride = 0, out_slot0 = 0;
    const uint8_t* acc_base = nullptr;
    uint64_t acc_block_stride = 0;
    uint32_t acc_seg_stride = 0, acc_slot0 = 0;
    // with num_data: output / accumulate row r at slot slot0 + numData + r (encode: the parity
    // after the block's numData sources; decode stage 1: the received parity rows)
    uint32_t out_after_data = 0, acc_after_data = 0;
    const uint32_t* rows_lim = nullptr;  // device word: rows needed (<= m), null: m
    // column map: column c is read from slot ((c >> col_shift) * col_chunk + (c & col_mask) +
    // col_base) (identity by default); in_slots bounds the slots read (0: k + m).  The tower
    // kernel also takes any chunk width: col_div != 0 reads slot (c / col_div) * col_chunk +
    // c % col_div + col_base (col_magic: set by its launcher)
    uint32_t col_shift = 31, col_mask = 0xFFFFFFFFu, col_chunk = 0, col_base = 0, in_slots = 0;
    uint32_t col_div = 0, col_magic = 0;
    const uint16_t* tw = nullptr;   // [k][2][m][2] snippet offsets (gf16_tw_offsets)
    // per-block mode (RS16 decode stage 2 on the tower kernel): item groups stay inside one
    // block; block b has its own table (tw + b * tw_block_stride), e = blk_rows[b] rows,
    // blk_cols[b] columns (null: e), and its rows' output byte offsets row_off[b *
    // row_off_stride + r] (from out_base + b * out_block_stride); no accumulate source
    const int32_t* blk_rows = nullptr;
    const uint16_t* blk_cols = nullptr;
    uint64_t tw_block_stride = 0;
    const uint32_t* row_off = nullptr;
    uint32_t row_off_stride = 0;
};
struct Gf16T3Multi {
    Gf16T3Args e[3];
    uint32_t wg_end[3] = {0, 0, 0};
};
// several independent products in one tower-kernel launch (the Toeplitz split: 3 at one level,
// 9 at two): workgroups [wg_end[i-1], wg_end[i]) run problem i
constexpr uint32_t kTwMultiMax = 9;
struct Gf16TwMulti {
    Gf16T3Args e[kTwMultiMax];
    uint32_t wg_end[kTwMultiMax] = {};
    uint32_t n = 0;
};
constexpr uint32_t kGf16T3RowsPerPass = 44;  // 11 row waves x 4 rows (gen_gf16_t3.py asserts it)
constexpr uint32_t gf16_t3_rows_padded(uint32_t m)
{
    return (m + kGf16T3RowsPerPass - 1) / kGf16T3RowsPerPass * kGf16T3RowsPerPass;
}
// RS16 encode by the Toeplitz split of the generator (kernels_tmvp.hip): the elementwise steps
// around the three shared-table products
struct Rs16TmvpArgs {
    const uint8_t* base = nullptr;  // batch: source slots [0, k), parity slots [k, k + m)
    uint64_t block_stride = 0;
    uint32_t seg_stride = 0, nblocks = 0;
    uint32_t vec = 0;               // bytes, multiple of 8
    uint32_t k = 0, cw = 0;         // cw = m / 2 (chunk width and half the parity rows)
    uint8_t* s = nullptr;           // prescaled chunk-pair sums: block b, virtual column v at s + b*s_block_stride + v*vec
    uint64_t s_block_stride = 0;
    uint8_t* x = nullptr;           // P1 rows: block b, row p at x + b*x_block_stride + p*vec
    uint64_t x_block_stride = 0;
    const uint16_t* cmat = nullptr; // [k][16] row masks of c_j (c_0 = 0)
    const uint16_t* wmat = nullptr; // [m][16] of W(y_p)
    const uint16_t* gmat = nullptr; // [m][16] of G[p][0]
    // two Karatsuba levels: hw = m / 4, and one scratch per block (sc + b * sc_block_stride,
    // columns of vec bytes): pair sums [0, k/2), scaled sums s_X at k/2 + X k/4, the nine
    // hw-row products from k/2 + 3k/4 (kernels_tmvp.hip, tmvp2_*)
    uint32_t hw = 0;
    uint8_t* sc = nullptr;
    uint64_t sc_block_stride = 0;
    // shortened blocks (null: every block has k sources): block b's source columns at or past
    // num_data[b] read as zeros in the prescale, and the postscale reads and writes its parity
    // at slot num_data[b] + p; a block whose numData is 0 or past k is left alone
    const uint16_t* num_data = nullptr;
};
bool rs16_tmvp_plan(uint32_t k, uint32_t m, const std::vector<uint32_t>& gen, std::vector<uint32_t> prod[3],
                    std::vector<uint16_t>& cmat, std::vector<uint16_t>& wmat, std::vector<uint16_t>& gmat);
// levels L = 1..3: prod[0 .. 3^L), (m >> L) x (k >> L) each (gf_host.cpp; the codec uses 1 or 2)
bool rs16_tmvp_plan_levels(uint32_t k, uint32_t m, const std::vector<uint32_t>& gen, int levels,
                           std::vector<uint32_t>* prod, std::vector<uint16_t>& cmat, std::vector<uint16_t>& wmat,
                           std::vector<uint16_t>& gmat);
int launch_tmvp_prescale(const Rs16TmvpArgs& a, hipStream_t s);
int launch_tmvp_postscale(const Rs16TmvpArgs& a, hipStream_t s);
int launch_tmvp2_prescale(const Rs16TmvpArgs& a, hipStream_t s);
int launch_tmvp2_postscale(const Rs16TmvpArgs& a, hipStream_t s);
int launch_gf16_t3_encode(const Gf16T3Args& a, hipStream_t s);  // NFEC_ENOTSUP: shape not covered
bool gf16_t3_covers(const Gf16T3Args& a);  // launch_gf16_t3_encode would take it
int launch_gf16_t3_multi(const Gf16T3Args* e, uint32_t n, hipStream_t s);  // n <= 3 independent products
// the same products through the tower field GF((2^8)^2) (gen_gf16_tw.hip): reads a.tw, not a.offs
int launch_gf16_tw_encode(const Gf16T3Args& a, hipStream_t s);  // NFEC_ENOTSUP: shape not covered
bool gf16_tw_covers(const Gf16T3Args& a);
int launch_gf16_tw_multi(const Gf16T3Args* e, uint32_t n, hipStream_t s);  // n <= kTwMultiMax
void gf16_tw_offsets(const std::vector<uint32_t>& parity_rows, uint32_t k, uint32_t m, uint16_t* out);
// The library holds the kernel in several configurations (rows per wave: 7 and 6 at 3 waves per SIMD,
// 4 at 4); each launch takes the cheapest for its rows (gen_gf16_tw.py CONFIGS / PASS_COST).
uint32_t gf16_tw_passes(uint32_t m, uint32_t rows);  // passes for m rows at `rows` per wave (a multiple of 4)
uint32_t gf16_tw_rows(uint32_t m);   // the configuration a launch of m rows takes
uint64_t gf16_tw_cost(uint32_t m);   // its relative cost per column (pass cost x passes)
size_t gf16_tw_table_elems(uint32_t k, uint32_t m);  // u16 elements of a k-column, m-row table
// the tower isomorphism's constants: phi's columns (phi(x^i)), lam, and phi^-1's columns (optional)
void gf16_tw_field(uint16_t phi_cols[16], uint32_t* lam, uint16_t* phi_inv_cols = nullptr);
// the segment tails of the same products: bytes [off, off + bytes) of every segment (even, at
// most 6: the part of vec & ~1 past the tower kernel's 8-byte pieces), same arguments and
// layouts as launch_gf16_tw_encode (flat or per-block mode, numData, accumulate; a.vec_bytes is
// ignored; no column map).  kernels_gf16tail.hip
int launch_gf16_tw_tail(const Gf16T3Args& a, uint32_t off, uint32_t bytes, hipStream_t s);
bool gf16_tw_tail_covers(const Gf16T3Args& a, uint32_t bytes);  // launch_gf16_tw_tail would take it
// RS16 decode stage 2 on the tower kernel: per-block snippet tables and output row offsets from
// the plan's e x e inverses (kernels_tmvp.hip)
struct TwDecTablesArgs {
    const uint16_t* coef2 = nullptr;  // [b][columns][dcs] inverse, column-major ([t][s])
    uint32_t dcs = 0;
    uint64_t coef2_block = 0;         // elements per block (0: dcs * dcs)
    const int32_t* rows = nullptr;    // e per block
    const uint16_t* cols = nullptr;   // columns per block (null: e)
    const uint16_t* out_slots = nullptr;  // [b][slots_stride] erased source slots
    uint32_t slots_stride = 0;
    uint32_t seg_stride = 0;          // output segment stride (bytes)
    uint32_t nblocks = 0, M = 0;      // M rows at most (min(k, m))
    uint64_t tw_block_stride = 0;     // u16 elements per block table
    uint16_t* tw = nullptr;           // [b][gf16_tw_table_elems(columns, M)]: [t][sweep][row][2]
    uint32_t* row_off = nullptr;      // [b][M + 12]
    uint16_t phi[16] = {};
    uint32_t lam = 0;
};
int launch_tw_dec_tables(const TwDecTablesArgs& a, hipStream_t s);
void gf16_t3_offsets(const std::vector<uint32_t>& parity_rows, uint32_t k, uint32_t m, uint16_t* out);
int launch_gf16_bs_encode(const Gf16BsEncArgs& a, hipStream_t s);  // NFEC_ENOTSUP: layout not 8-byte aligned
void gf16_bs_selectors(const std::vector<uint32_t>& parity_rows, uint32_t k, uint32_t m, uint16_t* sel);

// GF(2^8) block-matrix products with runtime coefficients (gen_rs8_rt.hip): bit-sliced, each
// coefficient a jump into a 256-entry snippet table.  out[b][oslot(r)] (^)= sum_c coef[c][r] *
// in[b][islot(c)] for r < rows(b), c < cols(b).  The table holds snippet byte offsets (u16,
// c << 7): entry (c, r) at tab + [block or count] * tab_block_stride + c * tab_col_stride + 2 r
// (bytes), or, pass-major (tab_pass_stride != 0, the plans' per-block tables), entry i of pass p
// (row pass_row0(p) + i) at tab + block * tab_block_stride + p * tab_pass_stride +
// c * tab_col_stride + 2 i: a pass's entries of consecutive columns share scalar-cache lines.
// Padded by 128 bytes past the last entry (the kernel touches lines ahead of its reads).
//   flat mode (per_block = 0): item groups run across the blocks; cols = k, rows = m, islot =
//     in_slot0 + c, oslot = out_slot0 + r (unshortened encode); with num_data (shortened encode,
//     "flat shortened") each 8-byte piece takes its own block's numData: columns at or past it
//     read as zeros and its parity row r lands at slot numData + r
//   per-block mode: item groups inside one block; cols = blk_cols[b] (else num_data[b], else k),
//     rows = blk_rows[b] (<= 0: skip; else m); islot = in_slots[b][c] or in_slot0 + c; oslot =
//     out_slots[b][r] or out_slot0 (+ num_data[b] with out_after_data) + r; table per block
//     (tab_block_stride) or per numData (tab_by_count: block nd - 1, MDP) or shared (stride 0)
struct Rs8RtArgs {
    const uint8_t* in_base = nullptr;
    uint64_t in_block_stride = 0;
    uint32_t in_seg_stride = 0;
    uint8_t* out_base = nullptr;
    uint64_t out_block_stride = 0;
    uint32_t out_seg_stride = 0;
    uint32_t nblocks = 0;
    uint32_t vec_bytes = 0;              // multiple of 8
    uint32_t k = 0, m = 0;               // columns / rows (per-block mode: the largest)
    uint32_t per_block = 0;
    const uint16_t* num_data = nullptr;
    const uint16_t* blk_cols = nullptr;
    const int32_t* blk_rows = nullptr;
    const uint16_t* in_slots = nullptr;
    uint32_t in_slots_stride = 0, in_slot0 = 0;
    const uint16_t* out_slots = nullptr;
    uint32_t out_slots_stride = 0, out_slot0 = 0, out_after_data = 0;
    const uint16_t* tab = nullptr;
    uint64_t tab_block_stride = 0;       // bytes
    uint32_t tab_col_stride = 0;         // bytes, multiple of 4
    uint32_t tab_by_count = 0;
    uint64_t tab_pass_stride = 0;        // bytes; 0: entries by row (2 r)
    uint32_t rows_lo = 0, rows_hi = ~0u; // per-block: only blocks with rows in [lo, hi] (set by the launcher)
    uint32_t probe_noapply = 0;          // diagnostic probes only (set by the launcher)
    uint32_t accumulate = 0;             // XOR into the output slots
    uint32_t slot_bound = 0;             // slot lists hold slots below this (0: 65536)
    uint32_t pass_sets = 0;              // set by the launcher
};
constexpr uint32_t kRs8RtRows = 8;       // parity rows per pass (gen_rs8_rt.py asserts it)
// rows [row0, row1) of pass p of a block with `rows` rows: the fewest passes of at most 8 rows,
// rows spread evenly with even boundaries (the kernel's split; plans writing pass-major tables
// use the same)
__host__ __device__ inline void rs8_rt_pass_rows(uint32_t rows, uint32_t p, uint32_t& row0, uint32_t& row1)
{
    const uint32_t P = rows > kRs8RtRows ? (rows + kRs8RtRows - 1u) / kRs8RtRows : 1u;
    const uint32_t h = (rows + 1u) / 2u;
    row0 = p < P ? (2u * (p * h / P) < rows ? 2u * (p * h / P) : rows) : rows;
    row1 = p < P ? (2u * ((p + 1u) * h / P) < rows ? 2u * ((p + 1u) * h / P) : rows) : rows;
}
__host__ __device__ inline uint32_t rs8_rt_passes(uint32_t rows) { return rows > kRs8RtRows ? (rows + kRs8RtRows - 1u) / kRs8RtRows : 1u; }
int launch_rs8_rt(const Rs8RtArgs& a, hipStream_t s);  // NFEC_ENOTSUP: layout not covered
bool rs8_rt_covers(const Rs8RtArgs& a);                // launch_rs8_rt would take it
// snippet-offset table of an m x k generator (row-major parity rows): [c][r] u16, column stride
// round_up(2m, 4) bytes, padded by 4 columns + 128 bytes
std::vector<uint16_t> rs8_rt_table(const std::vector<uint32_t>& rows, uint32_t k, uint32_t m);
inline uint32_t rs8_rt_col_stride(uint32_t m) { return (2u * m + 3u) & ~3u; }

// RS decode planning (per block): pick parities, invert the e x e system, emit the
// stage-1 (gather) and stage-2 (inverse) matrices and slot lists.
struct RsPlanArgs {
    int bits = 8;
    uint32_t k = 0, m = 0;
    uint32_t nblocks = 0;
    const uint16_t* num_data = nullptr;      // per block or null (k)
    const uint16_t* erasure_locs = nullptr;
    uint32_t erasure_stride = 0;
    const uint16_t* erasure_counts = nullptr;
    const void* gen_parity = nullptr;        // device m x k generator parity rows (elements)
    const void* exp_tab = nullptr;           // device exp (2q) table of the field (elements)
    const uint16_t* log_tab = nullptr;       // device log table (q+1 entries)
    // outputs
    int32_t* status = nullptr;               // per block decode return value
    int32_t* rows = nullptr;                 // per block source-erasure count e_s (0: nothing to do)
    uint16_t* in_slots1 = nullptr;           // [b][k]   stage-1 input slots
    uint16_t* out_slots2 = nullptr;          // [b][k]   stage-2 output slots (erased source)
    uint16_t* cols2 = nullptr;               // per block stage-2 column count (= e_s)
    uint32_t coef_stride = 0;                // padded row count of coef1/coef2 (multiple of 16)
    void* coef1 = nullptr;                   // [b][k][cs] gathered generator / unit columns
    void* coef2 = nullptr;                   // [b][cs][cs] inverse (column-major: [t][s])
    void* work = nullptr;                    // [b] work_block_bytes: e x 2e matrix, then the E/P
                                             // lists and pivot factors (used when e > 64 / > 256)
    uint64_t work_block_bytes = 0;
    // stage 1 by encode (RS16, gen_gf16_t3.hip): blocks whose substitute parities are rows
    // 0..e-1 get z_t = encode row t of the block with its erased source zeroed ^ parity t.  For
    // them the plan writes rows1 = 0 (the gather stage skips them), no gather matrix, raises
    // *rmax to e and zeroes the erased source slots (zero_*: the batch).  Others: rows1 = e.
    int32_t* rows1 = nullptr;
    uint32_t* rmax = nullptr;
    // by_row (tower decode, rs16_plan_cf_kernel): EVERY decodable block is repaired by encode,
    // whatever its substitute parities or numData: stage 1 computes z rows 0..P_last (the block's
    // last substitute parity row - nd), *rmax rises to P_last + 1, cols2 = P_last + 1, and coef2
    // is laid out by parity row (column P_t - nd holds A^-1's column t, lost rows zero).
    // zero_base null: the erased source is not zeroed (accumulate: stage 2 overwrites with
    // d_E ^ X, see rs16_plan_cf_kernel)
    uint32_t by_row = 0;
    uint64_t coef2_block = 0;           // coef2 elements per block (0: coef_stride^2)
    uint8_t* zero_base = nullptr;
    uint64_t zero_block_stride = 0;
    uint32_t zero_seg_stride = 0, zero_vec = 0;   // zero_vec: bytes (even; rs_plan_kernel: multiple of 8)
    // RS16 closed form (rs16_plan_cf_kernel, when both are set and min(k, m) <= kPlanCfMaxE):
    // A^-1 from the Cauchy form of the Lagrange generator instead of Gauss-Jordan
    const uint16_t* lwp = nullptr;      // [k] log W'(x_j)
    const uint16_t* lw = nullptr;       // [m] log W(y_p)
};
constexpr uint32_t kPlanCfMaxE = 256;
// per-block scratch of launch_rs_plan for decode row stride cs (elements of sym bytes)
inline uint64_t rs_plan_work_bytes(uint32_t cs, uint32_t sym)
{
    return ((uint64_t)cs * 2 * cs * sym + (uint64_t)cs * (4 + sym) + 7) & ~7ull;
}
int launch_rs_plan(const RsPlanArgs& a, hipStream_t s);
// RS8 closed-form plan for the runtime-coefficient repair: rs_plan's outputs with coef1 as
// [b][k][cst] and coef2 as [b][min(k, m)][cst] snippet-offset tables (u16, cst even and >=
// min(k, m)); needs lwp / lw.  Entries past a block's e are not written.
// writes coef1 pass-major: [block][pass < npass][column < k][8 entries] (u16), npass = passes of min(k, m)
int launch_rs8_plan_rt(const RsPlanArgs& a, uint32_t npass, hipStream_t s);

// RS decode planning, closed form (RS8, m <= 64): the systematic generator is the Lagrange
// basis of the points x_j = point(j) evaluated at y_p = point(k+p), so the e x e system
// A[t][s] = G[P_t][E_s] is a row/column-scaled Cauchy matrix with the explicit inverse
//   Ainv[s][t] = W'(x_s) Q(y_t) M_t(x_s) / (W(y_t) Q'(x_s))
// (W over all k points, Q over the erased points, M_t the Lagrange basis of the parity
// points).  Per block this is O(e^2) log-domain additions instead of a Gauss-Jordan
// elimination; the inverse is unique, so the bytes equal the reference's.
struct RsPlan2Args {
    uint32_t k = 0, m = 0, nblocks = 0;
    const uint16_t* num_data = nullptr;  // per block (null: k); parity p at slot numData + p
    const uint16_t* erasure_locs = nullptr;
    uint32_t erasure_stride = 0;
    const uint16_t* erasure_counts = nullptr;
    const uint8_t* exp_tab = nullptr;   // 510-entry GF(2^8) exp table (device)
    const uint16_t* log_tab = nullptr;  // 256-entry log table (device)
    const uint16_t* lwp = nullptr;      // [k] log W'(x_j)   (codec constant)
    const uint16_t* lw = nullptr;       // [m] log W(y_p)    (codec constant)
    // outputs
    int32_t* status = nullptr;
    int32_t* rows = nullptr;            // e_s per block (0: nothing to repair)
    uint16_t* cols2 = nullptr;          // e_s per block
    uint16_t* out_slots2 = nullptr;     // [b][k]: erased source slots E_s
    uint32_t* emask = nullptr;          // [b][2]: bit j set = source column j erased or past numData
    uint32_t* psel = nullptr;           // [b][2]: bit p set = parity row p used (P)
    uint8_t* pmap = nullptr;            // [b][m]: index t of parity row p in P
    uint32_t coef_stride = 0;
    uint8_t* coef2 = nullptr;           // [b][cs][cs]: Ainv column-major ([t][s])
    // gate word: set to gate_gen when some block needs the unfused stage 1 + solve (one the
    // fused kernel does not take); those kernels skip their whole launch unless *gate == gate_gen.
    // The generation changes per call, so the word never needs clearing.
    uint32_t* gate = nullptr;
    uint32_t gate_gen = 0;
    // fused repair runs after the plan (gen_fdec_asm.hip, rows fused_rows = min(16, m)): for a
    // block with e <= 16 whose substitute parities are all below fused_rows the inverse is
    // written by parity ROW ([row][s], zero rows for unused rows) instead of by rank, and the
    // block does not open the gate.  0: no fused kernel follows.
    uint32_t fused_rows = 0;
};
int launch_rs_plan2(const RsPlan2Args& a, hipStream_t s);

// Fused RS8 repair (gen_fdec_asm.hip): re-encode + e x e solve in registers, one wave per block,
// for blocks with e <= 16 whose substitute parities are rows below min(16, m).  Marks the blocks it repaired
// (rows = 0, psel = 0) so the unfused kernels that follow skip them.
struct FdecArgs {
    uint8_t* base = nullptr;
    uint64_t block_stride = 0;
    uint32_t seg_stride = 0;
    uint32_t nblocks = 0;
    uint32_t vec = 0;
    uint32_t ips = 0;                    // vec / 8
    int32_t* rows = nullptr;             // plan outputs (consumed and cleared)
    uint32_t* psel = nullptr;
    const uint32_t* emask = nullptr;
    const uint8_t* coef = nullptr;       // [b][t][s], column stride 32
    uint64_t coef_block_stride = 0;
    uint32_t coef_col_stride = 0;
    const uint16_t* out_slots = nullptr; // [b][slots_stride]: erased source slots
    uint32_t slots_stride = 0;
    uint32_t accumulate = 0;
    uint32_t lane_major = 0;             // lane L holds items 4L..4L+3; lanes without one exit
    const uint16_t* num_data = nullptr;  // per block (null: k): parity row t read at slot numData + t
};
int launch_rs8_fused_decode(uint32_t k, uint32_t m, const FdecArgs& a, hipStream_t s);
bool rs8_fused_decode_covers(uint32_t k, uint32_t m, const FdecArgs& a);

// MDP decode planning: per block one-stage coefficient matrix over the surviving slots.
struct MdpPlanArgs {
    uint32_t k = 0, m = 0, nblocks = 0;
    const uint16_t* num_data = nullptr;
    const uint16_t* erasure_locs = nullptr;
    uint32_t erasure_stride = 0;
    const uint16_t* erasure_counts = nullptr;
    const uint8_t* exp_tab = nullptr;        // 510-entry GF(2^8) exp table (device)
    const uint16_t* log_tab = nullptr;       // 256-entry log table (device)
    int32_t* status = nullptr;
    int32_t* rows = nullptr;
    uint16_t* cols = nullptr;                // number of surviving input slots
    uint16_t* in_slots = nullptr;            // [b][k+m]
    uint16_t* out_slots = nullptr;           // [b][k+m]
    uint32_t coef_stride = 0;                // padded row count (multiple of 16)
    uint8_t* coef = nullptr;                 // [b][k+m][cs]
    uint16_t* coef16 = nullptr;              // set: snippet offsets (value << 7) for gen_rs8_rt.hip,
                                             // pass-major [b][pass < npass16][k+m][8], instead of coef
    uint32_t npass16 = 0;
};
int launch_mdp_plan(const MdpPlanArgs& a, hipStream_t s);

// MDP decode, bit-sliced snippet solve (gen_solve_asm.hip): erased source r = XOR_j C[r][j] v_j
// over the block's surviving vectors, for blocks with rows (source erasures) <= 16 and cols
// (survivors) <= 96; marks them done (rows = 0) so the generic kernel that follows skips them.
// The scalar loads of the slot lists read up to 128 entries past a block's list: the lists'
// allocation must be padded by that much.
struct MdpSolveArgs {
    uint8_t* base = nullptr;             // the batch (inputs and outputs in place)
    uint64_t block_stride = 0;
    uint32_t seg_stride = 0;
    uint32_t nblocks = 0;
    uint32_t vec = 0;
    int32_t* rows = nullptr;             // plan outputs (consumed and cleared)
    const uint16_t* cols = nullptr;
    const uint16_t* in_slots = nullptr;  // [b][slots_stride]
    const uint16_t* out_slots = nullptr; // [b][slots_stride]
    uint32_t slots_stride = 0;
    const uint8_t* coef = nullptr;       // [b][j][r], column stride 32
    uint64_t coef_block_stride = 0;
    uint32_t coef_col_stride = 0;
};
int launch_mdp_solve_bs(const MdpSolveArgs& a, hipStream_t s);

// utilities
int launch_fill(uint8_t* base, uint64_t block_stride, uint32_t seg_stride, uint32_t nblocks,
                const uint16_t* num_data, uint32_t k, uint32_t vec, uint64_t seed, uint64_t first_block,
                hipStream_t s);
int launch_erasures(uint16_t* locs, uint32_t stride, uint16_t* counts, uint32_t nblocks, uint32_t range,
                    uint32_t count, uint64_t seed, uint64_t first_block, hipStream_t s);
int launch_stream_copy(void* dst, const void* src, uint64_t bytes, hipStream_t s);
int launch_zero_slots(uint8_t* base, uint64_t block_stride, uint32_t seg_stride, uint32_t nblocks,
                      const uint16_t* locs, uint32_t stride, const uint16_t* counts, uint32_t vec,
                      hipStream_t s);

// Host-resident decode transfers by kernels that read / write pinned host memory directly
// (zero-copy: 55-57 GB/s either way on one MI355X, as fast as the DMA engine, but per segment,
// tools/diag/zc_rate.hip).  Per block, the slots a mode selects from the block's erasure list:
//   SLOTS_RS_IN:  surviving source slots [0, numData) (erased ones too when accumulating) and
//                 the first e surviving parities -- what an RS decode reads (normEncoderRS8.cpp:
//                 680-700: the erased source rows are replaced by the first surviving parities)
//   SLOTS_ALL_IN: every surviving slot (MDP decode reads all of them, normEncoderMDP.cpp:346-361)
//   SLOTS_OUT:    the erased source slots, for blocks whose status is > 0 (the only bytes a
//                 decode writes, normEncoderRS8.cpp:732)
// An invalid erasure list (a location >= numData + m, or more entries than the stride) moves
// every slot [0, numData + m) in the IN modes and nothing in SLOTS_OUT.
enum SlotMoveMode : uint32_t { SLOTS_RS_IN = 0, SLOTS_ALL_IN = 1, SLOTS_OUT = 2 };
struct SlotMoveArgs {
    const uint8_t* src = nullptr;
    uint64_t src_block_stride = 0;
    uint32_t src_seg_stride = 0;
    uint8_t* dst = nullptr;
    uint64_t dst_block_stride = 0;
    uint32_t dst_seg_stride = 0;
    uint32_t nblocks = 0;
    uint32_t k = 0, m = 0;
    uint32_t bytes = 0;                    // bytes per slot to move
    const uint16_t* num_data = nullptr;    // device, per block (null: k)
    const uint16_t* locs = nullptr;        // device [b * lstride + i]
    uint32_t lstride = 0;
    const uint16_t* counts = nullptr;      // device
    const int32_t* status = nullptr;       // SLOTS_OUT: device decode status per block
    uint32_t mode = SLOTS_RS_IN;
    uint32_t accumulate = 0;
};
int launch_slot_move(const SlotMoveArgs& a, hipStream_t s);

// npc segment checksums (kernels_crc.hip): CRC-32 of the first len bytes of every slot
// (crc[b*slots + s], optional) and, optionally, whether it differs from the big-endian CRC
// stored right after them (bad[b*slots + s]).
struct CrcArgs {
    const uint8_t* base = nullptr;
    uint64_t block_stride = 0;
    uint32_t seg_stride = 0;
    uint32_t nblocks = 0;
    uint32_t slots = 0;
    uint32_t len = 0;
    uint32_t* crc = nullptr;
    uint8_t* bad = nullptr;
};
int launch_crc32_slots(const CrcArgs& a, hipStream_t s);

// Per block: ascending list of bad slots among [0, num_data + m) -> locs[b*stride ..] (at most
// stride entries), counts[b] = the full count (saturated at 65535).
struct ErasureListArgs {
    const uint8_t* bad = nullptr;        // [b][slots]
    uint32_t slots = 0;
    const uint16_t* num_data = nullptr;  // per block, or null = k
    uint32_t k = 0, m = 0;
    uint32_t nblocks = 0;
    uint16_t* locs = nullptr;
    uint32_t stride = 0;
    uint16_t* counts = nullptr;
};
int launch_erasure_list(const ErasureListArgs& a, hipStream_t s);

}  // namespace nfec
