#!/usr/bin/env python3
"""Generate norm_amd/csrc/gen_solve_asm.hip: the RS8 decode stage-2 solve d_E = A^-1 z as a
bit-sliced kernel whose per-block GF(2^8) coefficients are applied by jumping into a table of
256 code snippets, one per coefficient value.

Stage 2 of the closed-form RS8 decode (the reference computes the same
bytes through its k x k inverse, src/common/normEncoderRS8.cpp:652-757): for every block,
erased source symbol s = XOR_t c[s][t] * z_t over the e <= 16 rows z_t that stage 1 wrote, with
the block's e x e coefficient matrix c from rs_plan2_kernel.  One wave per block, so the
coefficients are wave-uniform scalars:

  * z_t is loaded, bit-transposed (8 planes) and expanded into the method-of-four-Russians
    tables of its even planes (group A, VGPR bank 0) and odd planes (group B, bank 1):
    48 + 22 VALU per row;
  * for every output s the wave jumps (s_swappc) to snippet[c[s][t]]: the 8 updates
    acc[s][i] ^= A[a_i(c)] ^ B[b_i(c)] of the 8x8 bit matrix of c, with the accumulator
    operands relative to M0 (VGPR index mode, M0 = 16 s), then returns (s_setpc).  No table
    lookups and no v_perm: 8 VALU + 7 SALU per (s, t), where the v_perm kernel
    (gf8_solve_kernel) spends three half-rate permutes per output dword.
  * acc[s][i] = acc[0][i] + 16 s in VGPR banks 2/3 (the layout of gen_rs8_asm.py), so every
    update reads three different banks.

Blocks with more than 16 rows, segment tails (vec % 8 != 0) and vec > 2048 keep
gf8_solve_kernel.

Usage: gen_solve_asm.py OUT.hip
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gen_rs8_asm import MASKS, MULTI, S_MASK, acc_reg, bank, combo_reg, split, transpose  # noqa: E402
from gen_rs8_bitsliced import bitmatrix_rows  # noqa: E402

IN_REGS = [0, 1, 4, 5, 8, 9, 12, 13]          # compiler-placed inputs: item / store offsets
TEMP = {0: [16, 20, 24, 28], 1: [17, 21, 25, 29]}
WIN_P0 = 19                                    # window: pairs 19..22 hold the planes of z_t
PRE_P0 = 23                                    # z row ring: pairs 23..38
S_RET = 56                                     # s56:57 return address of a snippet call
S_TI, S_ZOFF = 58, 59                          # row counter, z row offset
S_ZRS, S_ORS = 64, 68                          # z / output buffer descriptors
S_T = 78
S_COEF = 80                                    # s80..s83: c[0..15][t]
S_SLOT = 84                                    # s84..s91: erased slots (16 x u16)
S_TAB = 92                                     # s92:93 snippet table, s94:95 jump target
GPR_MODE = 0x9000                              # M0[15:12]: index SRC0 and DST
SNIP_ALIGN = 7                                 # 128-byte snippets


def pairs(p0):
    w = []
    for q in range(4):
        w += [4 * (p0 + q), 4 * (p0 + q) + 1]
    return w


def pool_ring():
    avail = {0: list(TEMP[0]), 1: list(TEMP[1])}

    def pick(avoid):
        return avail[1 if avoid == 0 else 0].pop(0)
    return pick


def pool_epi():
    free = [combo_reg(g, a) for a in MULTI for g in (0, 1)] + TEMP[0] + TEMP[1]

    def pick(avoid):
        for i, r in enumerate(free):
            if bank(r) != avoid:
                return free.pop(i)
        raise RuntimeError("no temporary")
    return pick


def all_tables(w):
    """every multi-plane combination of group A (w[0,2,4,6]) and group B (w[1,3,5,7])"""
    code, regs = [], [{}, {}]
    for g in (0, 1):
        single = [w[2 * t + g] for t in range(4)]
        built = {1 << t: single[t] for t in range(4)}
        for a in sorted(MULTI, key=lambda a: bin(a).count("1")):
            top = a.bit_length() - 1
            dst = combo_reg(g, a)
            code.append(f"v_xor_b32 v{dst}, v{built[a & ~(1 << top)]}, v{single[top]}")
            built[a] = dst
        regs[g] = built
    return code, regs


def snippet_table(regs):
    A, B = regs
    out = []
    for c in range(256):
        out.append(f".p2align {SNIP_ALIGN}")
        if c == 0:
            out.append("Lsnip0_%=:")
        rows = bitmatrix_rows(c) if c else [0] * 8
        for i in range(8):
            a, b = split(rows[i])
            acc = acc_reg(0, i)
            if a and b:
                out.append(f"v_bitop3_b32 v{acc}, v{acc}, v{A[a]}, v{B[b]} bitop3:0x96")
            elif a:
                out.append(f"v_xor_b32 v{acc}, v{acc}, v{A[a]}")
            elif b:
                out.append(f"v_xor_b32 v{acc}, v{acc}, v{B[b]}")
        out.append(f"s_setpc_b64 s[{S_RET}:{S_RET + 1}]")
    return out


NROW = 4                                       # z rows in flight (ring of pairs 23..38)
S_COEF2 = 60                                   # s60..s63: second coefficient buffer


def ring_slot(t):
    return pairs(PRE_P0 + 4 * (t % NROW))


def solve_asm():
    L = []
    offs = ["%[o0]", "%[o1]", "%[o2]", "%[o3]"]
    soffs = ["%[s0]", "%[s1]", "%[s2]", "%[s3]"]
    win = pairs(WIN_P0)
    coefbuf = [S_COEF, S_COEF2]
    L += [f"s_mov_b64 s[{S_ZRS}:{S_ZRS + 1}], %[zb]", f"s_mov_b32 s{S_ZRS + 2}, -1",
          f"s_mov_b32 s{S_ZRS + 3}, 0x00020000",
          f"s_mov_b64 s[{S_ORS}:{S_ORS + 1}], %[ob]", f"s_mov_b32 s{S_ORS + 2}, 0x80000000",
          f"s_mov_b32 s{S_ORS + 3}, 0x00020000"]
    for i, mk in enumerate(MASKS):
        L.append(f"s_mov_b32 s{S_MASK + i}, 0x{mk:08x}")
    L += [f"s_load_dwordx8 s[{S_SLOT}:{S_SLOT + 7}], %[sp], 0x0",
          f"s_load_dwordx4 s[{S_COEF}:{S_COEF + 3}], %[cp], 0x0",
          f"s_getpc_b64 s[{S_TAB}:{S_TAB + 1}]",
          "Lpc_%=:",
          f"s_add_u32 s{S_TAB}, s{S_TAB}, Lsnip0_%=-Lpc_%=",
          f"s_addc_u32 s{S_TAB + 1}, s{S_TAB + 1}, 0"]

    def zload(t):
        # rows past e are issued (the vmcnt accounting stays static) but as out-of-range loads
        # (num_records 0): no memory traffic
        w = ring_slot(t)
        out = [f"s_mul_i32 s{S_ZOFF}, %[zs], {t}",
               f"s_cmp_lt_u32 {t}, %[e]",
               f"s_cselect_b32 s{S_ZRS + 2}, -1, 0"]
        for q in range(4):
            out.append(f"buffer_load_dwordx2 v[{w[2 * q]}:{w[2 * q + 1]}], {offs[q]}, s[{S_ZRS}:{S_ZRS + 3}], s{S_ZOFF} offen")
        return out

    # rows 0..NROW-1 in flight (rows past e read unused workspace rows: in bounds, cs = 32)
    for t in range(NROW):
        L += zload(t)
    for s in range(16):
        for i in range(8):
            L.append(f"v_mov_b32 v{acc_reg(s, i)}, 0")
    # ---- rows z_t, unrolled; the wave leaves at t = e ----
    for t in range(16):
        L += [f"s_cmp_le_u32 %[e], {t}", "s_cbranch_scc1 Lrows_%="]
        L.append(f"s_waitcnt vmcnt({4 * (NROW - 1)})")
        w = ring_slot(t)
        for d in range(8):
            L.append(f"v_mov_b32 v{win[d]}, v{w[d]}")
        if t + NROW < 32:
            L += zload(t + NROW)
        cur = coefbuf[t % 2]
        L.append("s_waitcnt lgkmcnt(0)")
        if t + 1 < 16:
            nxt = coefbuf[(t + 1) % 2]
            L.append(f"s_load_dwordx4 s[{nxt}:{nxt + 3}], %[cp], 0x{32 * (t + 1):x}")
        L += transpose(win, pool_ring)
        tcode, regs = all_tables(win)
        L += tcode
        L += [f"s_mov_b32 s{S_T}, 0",
              f"s_set_gpr_idx_on s{S_T}, gpr_idx(SRC0,DST)"]
        for s in range(16):
            # one bound check per four outputs: mdp_plan_kernel zero-fills the coefficient rows
            # past e (to cs), so the calls of the outputs s >= e left in a group jump into the
            # empty snippet, and their accumulators are never stored
            if s % 4 == 0:
                L += [f"s_cmp_le_u32 %[e], {s}", f"s_cbranch_scc1 Lsend{t}_%="]
            L += [f"s_bfe_u32 s{S_T}, s{cur + s // 4}, 0x{(8 << 16) | (8 * (s % 4)):x}",
                  f"s_lshl_b32 s{S_T}, s{S_T}, {SNIP_ALIGN}",
                  f"s_add_u32 s{S_TAB + 2}, s{S_TAB}, s{S_T}",
                  f"s_addc_u32 s{S_TAB + 3}, s{S_TAB + 1}, 0",
                  f"s_movk_i32 m0, 0x{GPR_MODE | (16 * s):x}",
                  f"s_swappc_b64 s[{S_RET}:{S_RET + 1}], s[{S_TAB + 2}:{S_TAB + 3}]"]
        L += [f"Lsend{t}_%=:", "s_set_gpr_idx_off"]
    L.append("Lrows_%=:")
    # ---- outputs: planes back to bytes, optional accumulate, store into the erased slots ----
    L.append("s_waitcnt vmcnt(0) lgkmcnt(0)")
    tmp = [4 * (8 + p) + h for p in range(4) for h in (0, 1)]   # combination pairs, free now
    for s in range(16):
        L += [f"s_cmp_le_u32 %[e], {s}", "s_cbranch_scc1 Lout_%="]
        w = [acc_reg(s, i) for i in range(8)]
        L += transpose(w, pool_epi)
        L += [f"s_bfe_u32 s{S_T}, s{S_SLOT + s // 2}, 0x{(16 << 16) | (16 * (s % 2)):x}",
              f"s_mul_i32 s{S_T}, s{S_T}, %[ss]",
              "s_cmp_eq_u32 %[acc], 0", f"s_cbranch_scc1 Lna{s}_%="]
        for q in range(4):
            L.append(f"buffer_load_dwordx2 v[{tmp[2 * q]}:{tmp[2 * q + 1]}], {soffs[q]}, s[{S_ORS}:{S_ORS + 3}], s{S_T} offen")
        L.append("s_waitcnt vmcnt(0)")
        for q in range(4):
            L.append(f"v_xor_b32 v{w[2 * q]}, v{tmp[2 * q]}, v{w[2 * q]}")
            L.append(f"v_xor_b32 v{w[2 * q + 1]}, v{tmp[2 * q + 1]}, v{w[2 * q + 1]}")
        L.append(f"Lna{s}_%=:")
        for q in range(4):
            L.append(f"buffer_store_dwordx2 v[{w[2 * q]}:{w[2 * q + 1]}], {soffs[q]}, s[{S_ORS}:{S_ORS + 3}], s{S_T} offen")
    L.append("Lout_%=:")
    L.append("s_branch Lend_%=")
    L += snippet_table(regs)
    L.append("Lend_%=:")
    return L


MDP_NT = 96                                    # surviving vectors per block (k + m <= 97)
S_ISL = [40, 48]                               # s40..s55: input slot lists, 16 x u16 each


def mdp_solve_asm():
    """MDP decode in one pass per block: erased source r = XOR_j C[r][j] * v_j over the ns
    surviving vectors v_j of the block itself (mdp_plan_kernel's coefficients; the reference's
    syndrome / Forney chain, normEncoderMDP.cpp:333-430, is linear in them).  Same machinery as
    solve_asm, but the input rows are the block's surviving slots, read through the plan's slot
    list, and there are up to MDP_NT of them."""
    L = []
    offs = ["%[o0]", "%[o1]", "%[o2]", "%[o3]"]
    soffs = ["%[s0]", "%[s1]", "%[s2]", "%[s3]"]
    win = pairs(WIN_P0)
    coefbuf = [S_COEF, S_COEF2]
    L += [f"s_mov_b64 s[{S_ZRS}:{S_ZRS + 1}], %[ib]", f"s_mov_b32 s{S_ZRS + 2}, -1",
          f"s_mov_b32 s{S_ZRS + 3}, 0x00020000",
          f"s_mov_b64 s[{S_ORS}:{S_ORS + 1}], %[ib]", f"s_mov_b32 s{S_ORS + 2}, 0x80000000",
          f"s_mov_b32 s{S_ORS + 3}, 0x00020000"]
    for i, mk in enumerate(MASKS):
        L.append(f"s_mov_b32 s{S_MASK + i}, 0x{mk:08x}")
    L += [f"s_load_dwordx8 s[{S_SLOT}:{S_SLOT + 7}], %[sp], 0x0",
          f"s_load_dwordx4 s[{S_COEF}:{S_COEF + 3}], %[cp], 0x0",
          f"s_load_dwordx8 s[{S_ISL[0]}:{S_ISL[0] + 7}], %[ip], 0x0",
          f"s_load_dwordx8 s[{S_ISL[1]}:{S_ISL[1] + 7}], %[ip], 0x20",
          f"s_getpc_b64 s[{S_TAB}:{S_TAB + 1}]",
          "Lpc_%=:",
          f"s_add_u32 s{S_TAB}, s{S_TAB}, Lsnip0_%=-Lpc_%=",
          f"s_addc_u32 s{S_TAB + 1}, s{S_TAB + 1}, 0",
          "s_waitcnt lgkmcnt(0)"]

    def vload(t):
        # rows past ns are issued (static vmcnt accounting) as out-of-range loads
        w = ring_slot(t)
        sl = S_ISL[(t // 16) % 2] + (t % 16) // 2
        out = [f"s_bfe_u32 s{S_ZOFF}, s{sl}, 0x{(16 << 16) | (16 * (t % 2)):x}",
               f"s_mul_i32 s{S_ZOFF}, s{S_ZOFF}, %[ss]",
               f"s_cmp_lt_u32 {t}, %[ns]",
               f"s_cselect_b32 s{S_ZRS + 2}, -1, 0"]
        for q in range(4):
            out.append(f"buffer_load_dwordx2 v[{w[2 * q]}:{w[2 * q + 1]}], {offs[q]}, s[{S_ZRS}:{S_ZRS + 3}], s{S_ZOFF} offen")
        return out

    for t in range(NROW):
        L += vload(t)
    for s in range(16):
        for i in range(8):
            L.append(f"v_mov_b32 v{acc_reg(s, i)}, 0")
    regs = None
    for t in range(MDP_NT):
        L += [f"s_cmp_le_u32 %[ns], {t}", "s_cbranch_scc1 Lrows_%="]
        L.append(f"s_waitcnt vmcnt({4 * (NROW - 1)})")
        w = ring_slot(t)
        for d in range(8):
            L.append(f"v_mov_b32 v{win[d]}, v{w[d]}")
        if t + NROW < MDP_NT:
            L += vload(t + NROW)
        cur = coefbuf[t % 2]
        L.append("s_waitcnt lgkmcnt(0)")
        if t + 1 < MDP_NT:
            nxt = coefbuf[(t + 1) % 2]
            L.append(f"s_load_dwordx4 s[{nxt}:{nxt + 3}], %[cp], 0x{32 * (t + 1):x}")
        if t % 16 == 12 and t + 20 < MDP_NT:
            # slots of rows 16j.. (j = the next-but-one group of 16) into the buffer whose last
            # reader was row t-1's load of row t+3; their first load is issued at row 16j-4
            j = (t + 20) // 16
            L.append(f"s_load_dwordx8 s[{S_ISL[j % 2]}:{S_ISL[j % 2] + 7}], %[ip], 0x{32 * j:x}")
        L += transpose(win, pool_ring)
        tcode, regs = all_tables(win)
        L += tcode
        L += [f"s_mov_b32 s{S_T}, 0",
              f"s_set_gpr_idx_on s{S_T}, gpr_idx(SRC0,DST)"]
        for s in range(16):
            # one bound check per four outputs: mdp_plan_kernel zero-fills the coefficient rows
            # past e (to cs), so the calls of the outputs s >= e left in a group jump into the
            # empty snippet, and their accumulators are never stored
            if s % 4 == 0:
                L += [f"s_cmp_le_u32 %[e], {s}", f"s_cbranch_scc1 Lsend{t}_%="]
            L += [f"s_bfe_u32 s{S_T}, s{cur + s // 4}, 0x{(8 << 16) | (8 * (s % 4)):x}",
                  f"s_lshl_b32 s{S_T}, s{S_T}, {SNIP_ALIGN}",
                  f"s_add_u32 s{S_TAB + 2}, s{S_TAB}, s{S_T}",
                  f"s_addc_u32 s{S_TAB + 3}, s{S_TAB + 1}, 0",
                  f"s_movk_i32 m0, 0x{GPR_MODE | (16 * s):x}",
                  f"s_swappc_b64 s[{S_RET}:{S_RET + 1}], s[{S_TAB + 2}:{S_TAB + 3}]"]
        L += [f"Lsend{t}_%=:", "s_set_gpr_idx_off"]
    L.append("Lrows_%=:")
    L.append("s_waitcnt vmcnt(0) lgkmcnt(0)")
    tmp = [4 * (8 + p) + h for p in range(4) for h in (0, 1)]
    for s in range(16):
        L += [f"s_cmp_le_u32 %[e], {s}", "s_cbranch_scc1 Lout_%="]
        w = [acc_reg(s, i) for i in range(8)]
        L += transpose(w, pool_epi)
        L += [f"s_bfe_u32 s{S_T}, s{S_SLOT + s // 2}, 0x{(16 << 16) | (16 * (s % 2)):x}",
              f"s_mul_i32 s{S_T}, s{S_T}, %[ss]"]
        for q in range(4):
            L.append(f"buffer_store_dwordx2 v[{w[2 * q]}:{w[2 * q + 1]}], {soffs[q]}, s[{S_ORS}:{S_ORS + 3}], s{S_T} offen")
    L.append("Lout_%=:")
    L.append("s_branch Lend_%=")
    L += snippet_table(regs)
    L.append("Lend_%=:")
    return L


def mdp_clobbers():
    v = [f'"v{i}"' for i in range(256) if i not in IN_REGS]
    s = [f'"s{i}"' for i in range(S_ISL[0], 96)]
    return ", ".join(v + s + ['"m0"', '"scc"', '"memory"'])


def clobbers():
    v = [f'"v{i}"' for i in range(256) if i not in IN_REGS]
    s = [f'"s{i}"' for i in range(S_RET, 96)]
    return ", ".join(v + s + ['"m0"', '"scc"', '"memory"'])


def main():
    path = sys.argv[1]
    body = "\\n\"\n        \"".join(solve_asm())
    mbody = "\\n\"\n        \"".join(mdp_solve_asm())
    src = f"""// GENERATED by tools/codegen/gen_solve_asm.py -- do not edit by hand.
// RS8 decode stage 2 (d_E = A^-1 z, e <= 16 rows per block): bit-sliced, the block's
// coefficients applied through a table of 256 code snippets (see the generator's docstring).
#include "nfec_internal.hpp"

namespace nfec {{
namespace {{

__global__ __launch_bounds__(256, 2) void gf8_solve_bs_kernel(Gf8SolveArgs a, uint32_t ips)
{{
    if (a.gate && *a.gate != a.gate_gen) return;  // every block repaired by the fused kernel
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t blk = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
    if (blk >= a.nblocks) return;
    const int32_t rows = (int32_t)__builtin_amdgcn_readfirstlane((uint32_t)a.rows[blk]);
    if (rows <= 0 || rows > 16) return;  // more rows: gf8_solve_kernel
    const uint32_t e = (uint32_t)rows;
    uint32_t o[4], so[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {{
        const uint32_t item = (uint32_t)q * 64u + lane;
        const bool ok = item < ips;
        o[q] = ok ? item * 8u : 0u;
        so[q] = ok ? item * 8u : 0x80000000u;   // past the output descriptor's records: dropped
    }}
    const uint8_t* zb = a.z + (uint64_t)blk * a.z_block_stride;
    uint8_t* ob = a.out + (uint64_t)blk * a.out_block_stride;
    const uint8_t* cp = a.coef + (uint64_t)blk * a.coef_block_stride;
    const uint16_t* sp = a.out_slots + (uint64_t)blk * a.slots_stride;
    asm volatile(
        "{body}\\n"
        :
        : [zb] "s"(zb), [ob] "s"(ob), [cp] "s"(cp), [sp] "s"(sp), [e] "s"(e), [zs] "s"(a.z_stride),
          [ss] "s"(a.out_seg_stride), [acc] "s"(a.accumulate),
          [o0] "v"(o[0]), [o1] "v"(o[1]), [o2] "v"(o[2]), [o3] "v"(o[3]),
          [s0] "v"(so[0]), [s1] "v"(so[1]), [s2] "v"(so[2]), [s3] "v"(so[3])
        : {clobbers()});
}}

__global__ __launch_bounds__(256, 2) void mdp_solve_bs_kernel(MdpSolveArgs a, uint32_t ips)
{{
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t blk = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
    if (blk >= a.nblocks) return;
    const int32_t rows = (int32_t)__builtin_amdgcn_readfirstlane((uint32_t)a.rows[blk]);
    const uint32_t ns = __builtin_amdgcn_readfirstlane((uint32_t)a.cols[blk]);
    if (rows <= 0 || rows > 16 || ns > {MDP_NT}u) return;  // the generic kernel that follows takes it
    const uint32_t e = (uint32_t)rows;
    if (lane == 0) a.rows[blk] = 0;  // hand the block off: the generic kernel skips it
    // lane-major items, ceil(items / 4) lanes per load (item q*l4 + lane): the lanes past the
    // segment leave EXEC instead of computing garbage bytes (as the fused RS8 repair does)
    const uint32_t l4 = (ips + 3u) / 4u;
    if (lane >= l4) return;
    uint32_t o[4], so[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {{
        const uint32_t item = (uint32_t)q * l4 + lane;
        const bool ok = item < ips;
        o[q] = ok ? item * 8u : 0u;
        so[q] = ok ? item * 8u : 0x80000000u;   // past the output descriptor's records: dropped
    }}
    const uint8_t* ib = a.base + (uint64_t)blk * a.block_stride;
    const uint8_t* cp = a.coef + (uint64_t)blk * a.coef_block_stride;
    const uint16_t* sp = a.out_slots + (uint64_t)blk * a.slots_stride;
    const uint16_t* ip = a.in_slots + (uint64_t)blk * a.slots_stride;
    asm volatile(
        "{mbody}\\n"
        :
        : [ib] "s"(ib), [cp] "s"(cp), [sp] "s"(sp), [ip] "s"(ip), [e] "s"(e), [ns] "s"(ns),
          [ss] "s"(a.seg_stride),
          [o0] "v"(o[0]), [o1] "v"(o[1]), [o2] "v"(o[2]), [o3] "v"(o[3]),
          [s0] "v"(so[0]), [s1] "v"(so[1]), [s2] "v"(so[2]), [s3] "v"(so[3])
        : {mdp_clobbers()});
}}

}}  // namespace

// MDP decode of the blocks with <= 16 erased source vectors and <= {MDP_NT} survivors (marks them
// done: rows = 0); NFEC_ENOTSUP for layouts it does not cover
int launch_mdp_solve_bs(const MdpSolveArgs& a, hipStream_t s)
{{
    if (a.nblocks == 0) return NFEC_OK;
    if ((a.vec & 7u) || a.vec > 2048 || a.coef_col_stride != 32 || (a.coef_block_stride & 15) ||
        (a.slots_stride & 1) || (uint64_t)a.seg_stride * 256 + a.vec >= (1ull << 31))
        return NFEC_ENOTSUP;
    hipLaunchKernelGGL(mdp_solve_bs_kernel, dim3((a.nblocks + 3) / 4), dim3(256), 0, s, a, a.vec / 8);
    return hipGetLastError() == hipSuccess ? NFEC_OK : NFEC_EDEVICE;
}}

// NFEC_ENOTSUP when the shape needs the general kernel (segment tails, vec > 2048, other
// coefficient strides, odd slot-list strides, offsets past 2^31)
int launch_gf8_solve_bs(const Gf8SolveArgs& a, hipStream_t s)
{{
    if (a.nblocks == 0) return NFEC_OK;
    if ((a.vec_bytes & 7u) || a.vec_bytes > 2048 || a.coef_col_stride != 32 || (a.coef_block_stride & 15) ||
        (a.slots_stride & 1) || a.z_stride < a.vec_bytes || (a.z_stride & 7u) ||
        (uint64_t)a.out_seg_stride * 256 + a.vec_bytes >= (1ull << 31))
        return NFEC_ENOTSUP;
    hipLaunchKernelGGL(gf8_solve_bs_kernel, dim3((a.nblocks + 3) / 4), dim3(256), 0, s, a, a.vec_bytes / 8);
    return hipGetLastError() == hipSuccess ? NFEC_OK : NFEC_EDEVICE;
}}

}}  // namespace nfec
"""
    open(path, "w").write(src)


if __name__ == "__main__":
    main()
