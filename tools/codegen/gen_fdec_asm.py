#!/usr/bin/env python3
"""Generate norm_amd/csrc/gen_fdec_asm.hip: fused RS8 erasure repair, one wavefront per block.

The closed-form RS8 decode (same bytes as the reference's k x k inverse,
src/common/normEncoderRS8.cpp:652-757) has two linear stages:
    z_t = parity(P_t) ^ sum_{c present} G[P_t][c] * d_c         (constant generator rows)
    d_E = A^-1 z                                                (per-block e x e matrix)
The unfused path writes z to HBM between the two (gen_rs8_bitsliced.hip stage 1, then
gen_solve_asm.hip).  Here one wave owns one block, so the block's erasure pattern and its
coefficients are wave-uniform and both stages run back to back in registers:

  * stage 1 = the bit-sliced re-encode of gen_rs8_asm.py (bank-separated VGPR layout, 11-column
    load ring) over the 64 source columns plus the e used parity rows as 16 extra "columns"
    (identity coefficient on their own row).  Erased columns are neither read (their loads go
    through a descriptor with 0 records) nor computed (uniform branch).
  * stage 2 = the snippet-table solve of gen_solve_asm.py: for each row t, z_t's planes are
    copied into a fixed window and expanded into M4RM tables; for each output s the wave jumps
    into the 128-byte snippet of c[s][t], whose accumulator operands are relative to M0.
    Outputs are produced in two halves of 8 (64 accumulators in the freed load ring).
  * z never leaves the register file: the block's HBM traffic is the 48 + 16 segments read and
    the e repaired segments written.

A block qualifies when e <= 16 and the used parity rows are exactly rows 0..e-1 (no parity
erasures among them: NORM's usual case); the kernel marks the blocks it repaired (rows = 0,
psel = 0) so the unfused kernels that run after it on the same stream skip them.

Usage: gen_fdec_asm.py OUT.hip [k,m ...]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gen_rs8_asm import (MASKS, MULTI, NSLOT, S_MASK, TEMP, acc_reg, bank, combo_reg, ring_temps,  # noqa: E402
                         slot_regs, split, table_code, transpose)
from gen_rs8_bitsliced import bitmatrix_rows, generator  # noqa: E402

DEFAULT_SHAPES = [(64, 32), (64, 16), (64, 8)]
IN_REGS = [0, 1, 4, 5, 8, 9, 12, 13]      # compiler-placed inputs: load / store offsets
S_RET, S_EM = 56, 58                       # return address; erased-column mask (64 bit)
S_COEF2 = 60
S_LRS, S_SRS = 64, 68
S_COL, S_T = 78, 79
S_COEF1 = 80
S_SLOT = 84
S_TAB = 92                                 # s92:93 snippet table, s94:95 jump target
GPR_MODE = 0x9000                          # M0[15:12]: index SRC0 and DST
SNIP_ALIGN = 7
D_P0 = 19                                  # solve accumulators d[sl][i]: pairs 19..50 (ring)
WIN_P0 = 51                                # solve window: pairs 51..54
NCOLS_PAR = 16                             # parity rows handled as extra columns


def d_reg(sl, i):
    return 4 * (D_P0 + 4 * sl + i // 2) + (i & 1)


def win_regs():
    w = []
    for q in range(4):
        w += [4 * (WIN_P0 + q), 4 * (WIN_P0 + q) + 1]
    return w


def solve_pool():
    """transpose temporaries for the outputs (d in banks 0/1; banks 2/3 still hold z)"""
    free = list(TEMP[0]) + list(TEMP[1]) + [combo_reg(g, a) for a in MULTI for g in (0, 1)]

    def make():
        avail = list(free)

        def pick(avoid):
            for i, r in enumerate(avail):
                if bank(r) != avoid:
                    return avail.pop(i)
            return avail.pop(0)
        return pick
    return make


def all_tables(w):
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


def snippets(regs):
    A, B = regs
    # 64 KiB-aligned table start: in the e = 16 solve a snippet address's low word is the table
    # address's high half packed with the u16 offset (s_pack_*_b32_b16), no extract, no add
    out = [".p2align 16"]
    for c in range(256):
        out.append(f".p2align {SNIP_ALIGN}")
        if c == 0:
            out.append("Lsnip0_%=:")
        rows = bitmatrix_rows(c) if c else [0] * 8
        for i in range(8):
            a, b = split(rows[i])
            d = d_reg(0, i)
            if a and b:
                out.append(f"v_bitop3_b32 v{d}, v{d}, v{A[a]}, v{B[b]} bitop3:0x96")
            elif a:
                out.append(f"v_xor_b32 v{d}, v{d}, v{A[a]}")
            elif b:
                out.append(f"v_xor_b32 v{d}, v{d}, v{B[b]}")
        out.append(f"s_setpc_b64 s[{S_RET}:{S_RET + 1}]")
    return out


def fdec_asm(k, m, probe=None, e16=False):
    G = generator(k, m)
    nr = min(NCOLS_PAR, m)  # z rows that can be in use (e <= m)
    L = []
    offs = ["%[o0]", "%[o1]", "%[o2]", "%[o3]"]
    soffs = ["%[s0]", "%[s1]", "%[s2]", "%[s3]"]
    ncol = k + nr
    # load records 2^31: item offsets with bit 31 set (items past the segment) read as zero
    # without a memory access; erased columns switch the records to 0
    L += [f"s_mov_b64 s[{S_LRS}:{S_LRS + 1}], %[base]", f"s_mov_b32 s{S_LRS + 2}, 0x80000000",
          f"s_mov_b32 s{S_LRS + 3}, 0x00020000",
          f"s_mov_b64 s[{S_SRS}:{S_SRS + 1}], %[base]", f"s_mov_b32 s{S_SRS + 2}, 0x80000000",
          f"s_mov_b32 s{S_SRS + 3}, 0x00020000",
          f"s_mov_b64 s[{S_EM}:{S_EM + 1}], %[em]"]
    for i, mk in enumerate(MASKS):
        L.append(f"s_mov_b32 s{S_MASK + i}, 0x{mk:08x}")
    L += [f"s_load_dwordx8 s[{S_SLOT}:{S_SLOT + 7}], %[sp], 0x0",
          f"s_load_dwordx4 s[{S_COEF1}:{S_COEF1 + 3}], %[cp], 0x0",
          f"s_getpc_b64 s[{S_TAB}:{S_TAB + 1}]",
          "Lpc_%=:",
          f"s_add_u32 s{S_TAB}, s{S_TAB}, Lsnip0_%=-Lpc_%=",
          f"s_addc_u32 s{S_TAB + 1}, s{S_TAB + 1}, 0"]

    def loads(c):
        """column c: source slot c (c < k) or parity row c - k (slot c); unused ones read nothing"""
        if probe == "noload":
            return []
        w = slot_regs(c % NSLOT)
        if c < k:
            out = [f"s_bitcmp1_b64 s[{S_EM}:{S_EM + 1}], {c}", f"s_cselect_b32 s{S_LRS + 2}, 0, 0x80000000"]
        else:  # parity row c - k: read when the block uses it (bit of the parity-row mask)
            out = [f"s_bitcmp1_b32 %[ps], {c - k}", f"s_cselect_b32 s{S_LRS + 2}, 0x80000000, 0"]
        if c < k:
            out.append(f"s_mul_i32 s{S_COL}, %[ss], {c}")
        else:  # (slot numData + t: a shortened block's parity follows its numData sources)
            out += [f"s_add_u32 s{S_COL}, %[pk], {c - k}", f"s_mul_i32 s{S_COL}, s{S_COL}, %[ss]"]
        for q in range(4):
            out.append(f"buffer_load_dwordx2 v[{w[2 * q]}:{w[2 * q + 1]}], {offs[q]}, s[{S_LRS}:{S_LRS + 3}], s{S_COL} offen{LPOL}")
        return out

    for r in range(16):
        for i in range(8):
            L.append(f"v_mov_b32 v{acc_reg(r, i)}, 0")
    issued = -1
    for c in range(min(NSLOT, ncol)):
        L += loads(c)
        issued = c
    # ---- stage 1: z_t for rows 0..15 (rows >= e are computed but unused) ----
    if probe == "prio1":
        L.append("s_setprio 2")  # A/B: the loading stage ahead of the other wave's solve
    for c in range(ncol):
        w = slot_regs(c % NSLOT)
        if probe != "noload":
            L.append(f"s_waitcnt vmcnt({4 * (issued - c)})")
        if probe == "nos1":
            for i in range(8):  # keep the loaded data live
                L.append(f"v_xor_b32 v{acc_reg(0, i)}, v{w[i]}, v{acc_reg(0, i)}")
        elif c < k:
            L += [f"s_bitcmp1_b64 s[{S_EM}:{S_EM + 1}], {c}", f"s_cbranch_scc1 Lskip{c}_%="]
            L += transpose(w, ring_temps())
            ups, need = [], [set(), set()]
            for r in range(nr):
                mat = bitmatrix_rows(G[r][c])
                for i in range(8):
                    a, b = split(mat[i])
                    ups.append((acc_reg(r, i), a, b))
                    if a:
                        need[0].add(a)
                    if b:
                        need[1].add(b)
            L += table_code(w, need)
            A, B = need
            for acc, a, b in ups:
                if a and b:
                    L.append(f"v_bitop3_b32 v{acc}, v{acc}, v{A[a]}, v{B[b]} bitop3:0x96")
                elif a:
                    L.append(f"v_xor_b32 v{acc}, v{A[a]}, v{acc}")
                elif b:
                    L.append(f"v_xor_b32 v{acc}, v{B[b]}, v{acc}")
        else:
            t = c - k
            L += [f"s_bitcmp0_b32 %[ps], {t}", f"s_cbranch_scc1 Lskip{c}_%="]
            L += transpose(w, ring_temps())
            for i in range(8):
                L.append(f"v_xor_b32 v{acc_reg(t, i)}, v{w[i]}, v{acc_reg(t, i)}")
        L.append(f"Lskip{c}_%=:")
        if probe and probe.startswith("sync") and ((c + 1) % int(probe[4:]) == 0 or c + 1 == ncol):
            # A/B: keep the workgroup's four waves (four blocks) within N columns of each other,
            # so they stream the same stage-1 code through the instruction cache
            L.append("s_barrier")
        if c + NSLOT < ncol:
            L += loads(c + NSLOT)
            issued = c + NSLOT
    # ---- stage 2: d_s = sum_t c[s][t] z_t, outputs in two halves of 8 ----
    if probe == "prio1":
        L.append("s_setprio 0")
    if probe == "prio2":
        L.append("s_setprio 2")  # A/B: the solve ahead of the other wave's loading stage
    win = win_regs()
    cbuf = [S_COEF1, S_COEF2]
    tmp = [4 * (WIN_P0 + p) + h for p in range(4) for h in (0, 1)]
    regs = all_tables(win)[1]

    def stage2(x, full):
        """x: label suffix; full: the block has e = 16 (then every output is live and the used
        parity rows are 0..15), so the per-output and per-row bound checks are left out, and the
        snippet addresses add only their low word (the wave checked that no offset carries).
        The plan writes each coefficient as its snippet's byte offset (u16, c << 7); row t holds
        16 of them (32 bytes), half h loads its 8 (16 bytes at 32 t + 16 h)."""
        S = []
        for h in range(2):
            if h == 1 and not full:
                S.extend(["s_cmp_le_u32 %[e], 8", "s_cbranch_scc1 Ldone_%="])
            for sl in range(8):
                for i in range(8):
                    S.append(f"v_mov_b32 v{d_reg(sl, i)}, 0")
            for t in range(0 if probe == "nos2" else 16):
                if not full:
                    S.extend([f"s_cmp_le_u32 %[tmax], {t}", f"s_cbranch_scc1 Lrows{h}{x}_%="])
                cur = cbuf[t % 2]
                S.append("s_waitcnt lgkmcnt(0)")
                # next coefficient row (after row 15: row 0 again, for the second half)
                nt = (t + 1) % 16
                S.append(f"s_load_dwordx4 s[{cbuf[nt % 2]}:{cbuf[nt % 2] + 3}], %[cp], 0x{32 * nt + 16 * h:x}")
                for i in range(8):
                    S.append(f"v_mov_b32 v{win[i]}, v{acc_reg(t, i)}")
                S.extend(all_tables(win)[0])
                S.extend([f"s_mov_b32 s{S_T}, 0", f"s_set_gpr_idx_on s{S_T}, gpr_idx(SRC0,DST)"])
                for sl in range(8):
                    s = 8 * h + sl
                    if not full:
                        S.extend([f"s_cmp_le_u32 %[e], {s}", f"s_cbranch_scc1 Lsend{h}_{t}{x}_%="])
                    if full:
                        op = "s_pack_lh_b32_b16" if sl % 2 == 0 else "s_pack_hh_b32_b16"
                        S.append(f"{op} s{S_TAB + 2}, s{cur + sl // 2}, s{S_TAB}")
                    else:
                        S.extend([f"s_bfe_u32 s{S_T}, s{cur + sl // 2}, 0x{(16 << 16) | (16 * (sl % 2)):x}",
                                  f"s_add_u32 s{S_TAB + 2}, s{S_TAB}, s{S_T}",
                                  f"s_addc_u32 s{S_TAB + 3}, s{S_TAB + 1}, 0"])
                    S.extend([f"s_movk_i32 m0, 0x{GPR_MODE | (16 * sl):x}",
                              f"s_swappc_b64 s[{S_RET}:{S_RET + 1}], s[{S_TAB + 2}:{S_TAB + 3}]"])
                S.extend([f"Lsend{h}_{t}{x}_%=:", "s_set_gpr_idx_off"])
            S.append(f"Lrows{h}{x}_%=:")
            # the coefficient row that leaving early left in flight must land before the next half
            S.append("s_waitcnt lgkmcnt(0)")
            if h == 0:
                # the next half starts at row 0, which must sit in buffer 0
                S.append(f"s_load_dwordx4 s[{S_COEF1}:{S_COEF1 + 3}], %[cp], 0x10")
            for sl in range(8):
                s = 8 * h + sl
                if not full:
                    S.extend([f"s_cmp_le_u32 %[e], {s}",
                              "s_cbranch_scc1 Ldone_%=" if h == 1 else f"s_cbranch_scc1 Lhalf{h}{x}_%="])
                w = [d_reg(sl, i) for i in range(8)]
                S.extend(transpose(w, solve_pool()))
                S.extend([f"s_bfe_u32 s{S_T}, s{S_SLOT + s // 2}, 0x{(16 << 16) | (16 * (s % 2)):x}",
                          f"s_mul_i32 s{S_T}, s{S_T}, %[ss]",
                          "s_cmp_eq_u32 %[acc], 0", f"s_cbranch_scc1 Lna{s}{x}_%="])
                for q in range(4):
                    S.append(f"buffer_load_dwordx2 v[{tmp[2 * q]}:{tmp[2 * q + 1]}], {soffs[q]}, s[{S_SRS}:{S_SRS + 3}], s{S_T} offen")
                S.append("s_waitcnt vmcnt(0)")
                for q in range(4):
                    S.append(f"v_xor_b32 v{w[2 * q]}, v{tmp[2 * q]}, v{w[2 * q]}")
                    S.append(f"v_xor_b32 v{w[2 * q + 1]}, v{tmp[2 * q + 1]}, v{w[2 * q + 1]}")
                S.append(f"Lna{s}{x}_%=:")
                for q in range(4):
                    S.append(f"buffer_store_dwordx2 v[{w[2 * q]}:{w[2 * q + 1]}], {soffs[q]}, s[{S_SRS}:{S_SRS + 3}], s{S_T} offen{SPOL}")
            if h == 0:
                S.append(f"Lhalf{h}{x}_%=:")
        return S

    if e16:
        # the e = 16 copy packs a snippet address from the table address's high half and the
        # offset: taken when the table starts at a 64 KiB boundary in memory
        L += ["s_cmp_eq_u32 %[e], 16", "s_cbranch_scc0 Lgen_%=",
              f"s_mov_b32 s{S_TAB + 3}, s{S_TAB + 1}", f"s_and_b32 s{S_T}, s{S_TAB}, 0xffff",
              f"s_cmp_lg_u32 s{S_T}, 0", "s_cbranch_scc1 Lgen_%="]
        L += stage2("f", True)
        L += ["s_branch Ldone_%=", "Lgen_%=:"]
    L += stage2("", False)
    L.append("Ldone_%=:")
    L.append("s_waitcnt lgkmcnt(0)")
    L.append("s_branch Lend_%=")
    L += snippets(regs)
    L.append("Lend_%=:")
    return L


def clobbers():
    v = [f'"v{i}"' for i in range(256) if i not in IN_REGS]
    s = [f'"s{i}"' for i in range(S_RET, 96)]
    return ", ".join(v + s + ['"m0"', '"scc"', '"memory"'])


# A/B probes of the (64, 32) kernel, NFEC_FDEC_VARIANT=<id> (never the default): no stage-2 solve,
# no stage-1 arithmetic (loads only), no stage-1 loads, no e = 16 specialisation of stage 2
# (measured: 1.992 ms without it, 1.981 with it, 64k blocks)
# Also generable (add to PROBES): "prio1" (stage 1 at issue priority 2: 2.12-2.14 ms, slower) and
# "prio2" (stage 2 at priority 2: 1.993-1.996 ms, no change against 1.989-1.992).
# "dephase" / "dephase2" (first-generation second workgroups start 30 / 17 us late, so the two
# waves of a SIMD do not ramp their loads in phase): 1.999-2.002 / 1.984-1.987 ms against
# 1.983-1.986, no gain; generable, not built.
PROBES = {1: "nos2", 2: "nos1", 3: "noload", 4: "gen", 5: "sync4", 6: "sync8", 7: "sync16", 8: "sync80",
          9: "persist"}
# "persist" (A/B): a grid of 1,024 workgroups whose waves loop over the blocks (no wave launch
# and prologue per block, no tail of partly filled workgroups)


def persist_kernel(K, nr, body, k):
    """the fused repair as a persistent loop: each wave walks blocks w, w + 4 * gridDim.x, ...;
    the item offsets are the same for every block (o doubles as the store offsets)"""
    return f"""__global__ __launch_bounds__(256, 2) void {K}(FdecArgs a)
{{
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t l4 = (a.ips + 3u) / 4u;
    if (lane >= l4) return;  // lane-major items (lane_major 2 only in this probe)
    uint32_t o[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {{
        const uint32_t item = (uint32_t)q * l4 + lane;
        o[q] = item < a.ips ? item * 8u : 0x80000000u;
    }}
    const uint32_t stride = gridDim.x * 4u;
    for (uint32_t blk = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6)); blk < a.nblocks;
         blk += stride) {{
        const int32_t rows = (int32_t)__builtin_amdgcn_readfirstlane((uint32_t)a.rows[blk]);
        const uint32_t ps0 = __builtin_amdgcn_readfirstlane(a.psel[2 * (uint64_t)blk]);
        const uint32_t ps1 = __builtin_amdgcn_readfirstlane(a.psel[2 * (uint64_t)blk + 1]);
        if (rows <= 0 || rows > 16 || ps1 != 0 || (ps0 >> {nr}) != 0u) continue;
        const uint32_t e = (uint32_t)rows;
        const uint32_t tmax = 32u - (uint32_t)__builtin_clz(ps0);
        const uint64_t em = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane(a.emask[2 * (uint64_t)blk]) |
                            ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane(a.emask[2 * (uint64_t)blk + 1]) << 32);
        const uint32_t pk = a.num_data ? __builtin_amdgcn_readfirstlane((uint32_t)a.num_data[blk]) : {k}u;
        if (lane == 0) {{
            a.rows[blk] = 0;
            a.psel[2 * (uint64_t)blk] = 0;
        }}
        const uint8_t* base = a.base + (uint64_t)blk * a.block_stride;
        const uint8_t* cp = a.coef + (uint64_t)blk * a.coef_block_stride;
        const uint16_t* sp = a.out_slots + (uint64_t)blk * a.slots_stride;
        asm volatile(
            "{body}\\n"
            :
            : [base] "s"(base), [em] "s"(em), [cp] "s"(cp), [sp] "s"(sp), [e] "s"(e), [ss] "s"(a.seg_stride),
              [acc] "s"(a.accumulate), [ps] "s"(ps0), [tmax] "s"(tmax), [pk] "s"(pk),
              [o0] "v"(o[0]), [o1] "v"(o[1]), [o2] "v"(o[2]), [o3] "v"(o[3]),
              [s0] "v"(o[0]), [s1] "v"(o[1]), [s2] "v"(o[2]), [s3] "v"(o[3])
            : {clobbers()});
    }}
}}
"""


def gen_kernel(k, m, probe=None):
    K = f"rs8_fdec_k{k}_m{m}" + (f"_probe_{probe}" if probe else "")
    nr = min(NCOLS_PAR, m)
    # e = 16 blocks (every output live) get a copy of stage 2 without the bound checks; m < 16
    # codes never have them
    asm = fdec_asm(k, m, None if probe in ("gen", "dephase", "dephase2", "persist") else probe,
                   e16=((probe in (None, "prio1", "prio2", "dephase", "dephase2", "persist") or probe.startswith("sync"))
                        and nr == 16))
    # A/B probe: the first generation's second workgroup per CU (dispatch order 256..511) starts
    # ~half (dephase) / ~a quarter (dephase2) of a block later, so the two waves of a SIMD stop
    # ramping their loads in phase
    nsleep = {"dephase": 9, "dephase2": 5}.get(probe, 0)
    dephase = (f"    if (blockIdx.x >= 256u && blockIdx.x < 512u)\n"
               f"        for (int i = 0; i < {nsleep}; ++i) __builtin_amdgcn_s_sleep(127);\n") if nsleep else ""
    body = "\\n\"\n        \"".join(asm)
    if probe == "persist":
        return persist_kernel(K, nr, body, k)
    return f"""__global__ __launch_bounds__(256, 2) void {K}(FdecArgs a)
{{
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t blk = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
    if (blk >= a.nblocks) return;
{dephase}    const int32_t rows = (int32_t)__builtin_amdgcn_readfirstlane((uint32_t)a.rows[blk]);
    const uint32_t ps0 = __builtin_amdgcn_readfirstlane(a.psel[2 * (uint64_t)blk]);
    const uint32_t ps1 = __builtin_amdgcn_readfirstlane(a.psel[2 * (uint64_t)blk + 1]);
    // qualifies: 1..16 source erasures repaired from parity rows below {nr} (the z rows this
    // kernel computes); the plan then wrote the inverse by parity row, zero for unused rows
    if (rows <= 0 || rows > 16 || ps1 != 0 || (ps0 >> {nr}) != 0u) return;
    const uint32_t e = (uint32_t)rows;
    const uint32_t tmax = 32u - (uint32_t)__builtin_clz(ps0);  // highest used parity row + 1
    // (readfirstlane yields int: widen through uint32_t, or bit 31 would sign-extend into the
    // high word)
    const uint64_t em = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane(a.emask[2 * (uint64_t)blk]) |
                        ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane(a.emask[2 * (uint64_t)blk + 1]) << 32);
    // the block's parity slot 0: numData (a shortened block; the plan put its columns
    // [numData, k) into em, so they are neither read nor computed), else k
    const uint32_t pk = a.num_data ? __builtin_amdgcn_readfirstlane((uint32_t)a.num_data[blk]) : {k}u;
    // hand the block off: the unfused stage 1 and solve that follow on the stream skip it
    if (lane == 0) {{
        a.rows[blk] = 0;
        a.psel[2 * (uint64_t)blk] = 0;
    }}
    // lane-major items: a 1400-byte segment occupies lanes 0..43 and the lanes past it drop out
    // of every instruction (EXEC) instead of computing garbage bytes, a third of the lane work.
    // lane_major 1: lane L holds items 4L..4L+3 (strided loads; measured slower, off);
    // lane_major 2: item q*L4 + L with L4 = ceil(items / 4), so each load stays contiguous
    const uint32_t l4 = (a.ips + 3u) / 4u;
    if ((a.lane_major == 1u && lane * 4u >= a.ips) || (a.lane_major == 2u && lane >= l4)) return;
    uint32_t o[4], so[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {{
        const uint32_t item = a.lane_major == 1u   ? lane * 4u + (uint32_t)q
                              : a.lane_major == 2u ? (uint32_t)q * l4 + lane
                                                   : (uint32_t)q * 64u + lane;
        const bool ok = item < a.ips;
        o[q] = ok ? item * 8u : 0x80000000u;  // past the load records: zeros, no memory access
        so[q] = ok ? item * 8u : 0x80000000u;  // past the store descriptor's records: dropped
    }}
    const uint8_t* base = a.base + (uint64_t)blk * a.block_stride;
    const uint8_t* cp = a.coef + (uint64_t)blk * a.coef_block_stride;
    const uint16_t* sp = a.out_slots + (uint64_t)blk * a.slots_stride;
    asm volatile(
        "{body}\\n"
        :
        : [base] "s"(base), [em] "s"(em), [cp] "s"(cp), [sp] "s"(sp), [e] "s"(e), [ss] "s"(a.seg_stride),
          [acc] "s"(a.accumulate), [ps] "s"(ps0), [tmax] "s"(tmax), [pk] "s"(pk),
          [o0] "v"(o[0]), [o1] "v"(o[1]), [o2] "v"(o[2]), [o3] "v"(o[3]),
          [s0] "v"(so[0]), [s1] "v"(so[1]), [s2] "v"(so[2]), [s3] "v"(so[3])
        : {clobbers()});
}}
"""


LPOL = SPOL = ""   # cache-policy suffixes (main: --nt-loads / --nt-stores)


def main():
    # --diag: also emit the A/B probes and their NFEC_FDEC_VARIANT switch (the diagnostic
    # library, make -C norm_amd diag); the product library ships the default kernels only.
    # --nt-loads / --nt-stores: non-temporal column loads / repaired-row stores (A/B builds)
    global LPOL, SPOL
    diag = "--diag" in sys.argv
    LPOL = " nt" if "--nt-loads" in sys.argv else ""
    SPOL = " nt" if "--nt-stores" in sys.argv else ""
    argv = [a for a in sys.argv if a not in ("--diag", "--nt-loads", "--nt-stores")]
    path = argv[1]
    shapes = DEFAULT_SHAPES
    if len(argv) > 2:
        shapes = [tuple(int(v) for v in s.split(",")) for s in argv[2:]]
    parts = [
        "// GENERATED by tools/codegen/gen_fdec_asm.py -- do not edit by hand.",
        "// Fused RS8 erasure repair (re-encode + e x e solve in registers, one wave per block) for",
        "// (k, m) in: " + ", ".join(f"({k},{m})" for k, m in shapes),
        "#include <cstdlib>",
        '#include "nfec_internal.hpp"',
        "",
        "namespace nfec {",
        "namespace {",
    ]
    for k, m in shapes:
        parts.append(gen_kernel(k, m))
        if diag and (k, m) == (64, 32):
            for probe in PROBES.values():
                parts.append(gen_kernel(k, m, probe))
    parts.append("}  // namespace")
    parts.append("")
    if diag:
        parts.append("static int fdec_variant()")
        parts.append("{")
        parts.append("    static const int v = [] { const char* e = std::getenv(\"NFEC_FDEC_VARIANT\"); return e ? std::atoi(e) : 0; }();")
        parts.append("    return v;")
        parts.append("}")
        parts.append("")
    parts.append("// true when launch_rs8_fused_decode runs a kernel for this shape and layout (the plan then")
    parts.append("// writes the inverse of the blocks it will take by parity row)")
    parts.append("bool rs8_fused_decode_covers(uint32_t k, uint32_t m, const FdecArgs& a)")
    parts.append("{")
    parts.append("    if ((a.vec & 7u) || a.vec > 2048 || a.coef_col_stride != 32 || (a.coef_block_stride & 15) ||")
    parts.append("        (a.slots_stride & 1) || (uint64_t)a.seg_stride * (k + 16) + a.vec >= (1ull << 31))")
    parts.append("        return false;")
    parts.append("    return " + " || ".join(f"(k == {k} && m == {m})" for k, m in shapes) + ";")
    parts.append("}")
    parts.append("")
    parts.append("// NFEC_ENOTSUP when (k, m) has no fused kernel or the batch shape needs the unfused path")
    parts.append("int launch_rs8_fused_decode(uint32_t k, uint32_t m, const FdecArgs& a, hipStream_t s)")
    parts.append("{")
    parts.append("    if (a.nblocks == 0) return NFEC_OK;")
    parts.append("    if (!rs8_fused_decode_covers(k, m, a)) return NFEC_ENOTSUP;")
    for v, probe in (PROBES.items() if diag else ()):
        parts.append(f"    if (k == 64 && m == 32 && fdec_variant() == {v}) {{")
        grid = "std::min((a.nblocks + 3) / 4, 1024u)" if probe == "persist" else "(a.nblocks + 3) / 4"
        parts.append(f"        hipLaunchKernelGGL(rs8_fdec_k64_m32_probe_{probe}, dim3({grid}), dim3(256), 0, s, a);")
        parts.append("        return hipGetLastError() == hipSuccess ? NFEC_OK : NFEC_EDEVICE;")
        parts.append("    }")
    for k, m in shapes:
        parts.append(f"    if (k == {k} && m == {m}) {{")
        parts.append(f"        hipLaunchKernelGGL(rs8_fdec_k{k}_m{m}, dim3((a.nblocks + 3) / 4), dim3(256), 0, s, a);")
        parts.append("        return hipGetLastError() == hipSuccess ? NFEC_OK : NFEC_EDEVICE;")
        parts.append("    }")
    parts.append("    return NFEC_ENOTSUP;")
    parts.append("}")
    parts.append("")
    parts.append("}  // namespace nfec")
    open(path, "w").write("\n".join(parts) + "\n")


if __name__ == "__main__":
    main()
