#!/usr/bin/env python3
"""Generate norm_amd/csrc/gen_fdec_q2.hip: fused RS8 erasure repair with TWO waves per block that
share every column's bit transpose through LDS (168 VGPRs: 3 waves per SIMD).

Same two linear stages as gen_fdec_asm.py (closed-form decode; bytes equal
to the reference's k x k inverse, src/common/normEncoderRS8.cpp:652-757):
    z_t = parity(P_t) ^ sum_{c present} G[P_t][c] * d_c          (constant generator rows)
    d_E = A^-1 z                                                 (per-block e x e matrix)
with P_t = parity row t (the block qualifies when its e <= 16 substitute parities are rows
0..e-1).  The one-wave kernel holds all 16 z rows (128 accumulator VGPRs) plus an 11-column load
ring: 256 VGPRs, 2 waves per SIMD.  Here the block's rows are dealt to two waves:

  * stage 1: wave w owns z rows t = 2r + w (r < R = min(16, m) / 2; 64 accumulators).  In step
    n wave w loads source column 2n + w (a 6-slot VGPR ring, buffer loads; erased columns read
    nothing), transposes it once and writes its 8 planes to LDS; after one s_barrier it reads
    the other wave's column back and applies both columns to its rows.  Then its own parity
    rows enter as identity columns (transpose + 8 XORs).
  * stage 2: the z rows move out of the accumulator registers (which become the output
    accumulators d); in step j both waves publish their row 2j + w through LDS, and each wave
    applies rows 2j and 2j + 1 to its outputs s = 2sl + w with the snippet-table solve of
    gen_solve_asm.py (the wave jumps into the 128-byte snippet of c[s][t]; accumulator operands
    are M0-relative).
  * z never leaves the chip: the block's HBM traffic is the 48 + 16 segments read and the e
    repaired segments written, as before.

VGPR map (v0..v167; bank = index mod 4; every bitop3 reads three banks):
  stage 1: accumulators in banks 2/3 of quads 0..4R-1 (acc_reg as gen_rs8_q4.py), M4RM
           combinations quads 0..10 banks 0/1, the other wave's planes quads 11..14, ring slots
           quads 15..38, compiler-placed inputs (4 item offsets + LDS address) quads 39..41;
  stage 2: outputs d in the accumulator registers, window (the row being applied) quads 11..14,
           its combinations quads 0..10, the wave's z rows in ring quads (rows 0..5) and banks
           2/3 of quads 32..39 (rows 6, 7).

Usage: gen_fdec_q2.py OUT.hip
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gen_rs8_asm import MASKS, S_MASK, split, transpose  # noqa: E402
from gen_rs8_bitsliced import bitmatrix_rows, generator  # noqa: E402

SHAPES = [(64, 32), (64, 16), (64, 8)]
NW = 2
NQ = 42                                    # quads: v0..v167
MULTI = [a for a in range(1, 16) if bin(a).count("1") >= 2]
COMBO_Q0, PBUF_Q0, RING_Q0 = 0, 11, 15
NS = 6                                     # ring slots per wave (quads 15..38)
IN_REGS = [156, 157, 160, 161, 164]        # quads 39..41, banks 0/1
ZHI_Q0 = 32                                # z rows 6, 7 in banks 2/3 of quads 32..39
S_RET, S_EM = 56, 58
S_C0, S_C1 = 60, 80                        # coefficient rows 2j, 2j+1 (4 SGPRs each)
S_LRS, S_SRS = 64, 68
S_COL, S_T = 78, 79
S_SLOT = 84
S_TAB = 92
GPR_MODE = 0x9000                          # M0[15:12]: index SRC0 and DST
SNIP_ALIGN = 7
COL_BYTES = 4 * 512                        # one column's 8 planes: 4 b64 rows of 64 lanes
ST2_BASE = 4 * COL_BYTES                   # stage-2 row exchange after the stage-1 slots
LDS_BYTES = 8 * COL_BYTES


def acc_reg(r, i):
    return 4 * (4 * r + i // 2) + 2 + (i & 1)


def combo_reg(g, a):
    return 4 * (COMBO_Q0 + MULTI.index(a)) + g


def quad_pairs(q0):
    w = []
    for q in range(4):
        w += [4 * (q0 + q), 4 * (q0 + q) + 1]
    return w


def ring(i):
    return quad_pairs(RING_Q0 + 4 * i)


PBUF = quad_pairs(PBUF_Q0)


def zreg(r, i):
    if r < 6:
        return 4 * (RING_Q0 + 4 * r + i // 2) + (i & 1)
    return 4 * (ZHI_Q0 + 4 * (r - 6) + i // 2) + 2 + (i & 1)


def combo_temps():
    """transpose temporaries from the combination registers (dead while a column transposes)"""
    def make():
        avail = {0: [combo_reg(0, MULTI[i]) for i in range(4)], 1: [combo_reg(1, MULTI[i]) for i in range(4)]}

        def pick(avoid):
            return avail[1 if avoid == 0 else 0].pop(0)
        return pick
    return make


def low_temps():
    """temporaries in banks 0/1 for the output transposes (operands in banks 2/3)"""
    def make():
        free = [4 * q + b for q in range(COMBO_Q0, RING_Q0 + 4 * NS) for b in (0, 1)]

        def pick(avoid):
            for i, r in enumerate(free):
                if r % 4 != avoid:
                    return free.pop(i)
            raise RuntimeError("no temp")
        return pick
    return make


def combos(w, need):
    """group A = w[0,2,4,6] (bank 0), group B = w[1,3,5,7] (bank 1); only the combinations in
    need[g] are built.  Returns (code, A map, B map)."""
    code, tabs = [], []
    for g in (0, 1):
        single = [w[2 * t + g] for t in range(4)]
        built = {1 << t: single[t] for t in range(4)}
        for a in sorted({a for a in need[g] if a in MULTI}, key=lambda a: bin(a).count("1")):
            dst = combo_reg(g, a)
            top = a.bit_length() - 1
            rest = a & ~(1 << top)
            if rest in built:
                code.append(f"v_xor_b32 v{dst}, v{built[rest]}, v{single[top]}")
            else:
                bits = [t for t in range(4) if (a >> t) & 1]
                code.append(f"v_bitop3_b32 v{dst}, v{single[bits[0]]}, v{single[bits[1]]}, v{single[bits[2]]} bitop3:0x96")
                if len(bits) == 4:
                    code.append(f"v_xor_b32 v{dst}, v{dst}, v{single[bits[3]]}")
            built[a] = dst
        tabs.append(built)
    return code, tabs[0], tabs[1]


def column_code(G, w_idx, R, nr, c, w):
    """updates of the wave's rows t = 2r + w (t < nr) by source column c with planes in w"""
    ups, need = [], [set(), set()]
    for r in range(R):
        t = NW * r + w_idx
        if t >= nr:
            continue
        mat = bitmatrix_rows(G[t][c])
        for i in range(8):
            a, b = split(mat[i])
            ups.append((acc_reg(r, i), a, b))
            if a:
                need[0].add(a)
            if b:
                need[1].add(b)
    code, A, B = combos(w, need)
    for acc, a, b in ups:
        if a and b:
            code.append(f"v_bitop3_b32 v{acc}, v{acc}, v{A[a]}, v{B[b]} bitop3:0x96")
        elif a:
            code.append(f"v_xor_b32 v{acc}, v{A[a]}, v{acc}")
        elif b:
            code.append(f"v_xor_b32 v{acc}, v{B[b]}, v{acc}")
    return code


def window_tables():
    """all 22 combinations of the stage-2 window (PBUF); returns (code, A, B)"""
    return combos(PBUF, [set(MULTI), set(MULTI)])


def snippets(A, B):
    out = []
    for c in range(256):
        out.append(f".p2align {SNIP_ALIGN}")
        if c == 0:
            out.append("Lsnip0_%=:")
        rows = bitmatrix_rows(c) if c else [0] * 8
        for i in range(8):
            a, b = split(rows[i])
            d = acc_reg(0, i)
            if a and b:
                out.append(f"v_bitop3_b32 v{d}, v{d}, v{A[a]}, v{B[b]} bitop3:0x96")
            elif a:
                out.append(f"v_xor_b32 v{d}, v{d}, v{A[a]}")
            elif b:
                out.append(f"v_xor_b32 v{d}, v{d}, v{B[b]}")
        out.append(f"s_setpc_b64 s[{S_RET}:{S_RET + 1}]")
    return out


def role_asm(G, k, m, w, probe=None):
    nr = min(16, m)            # z rows that can be in use (e <= m)
    R = nr // NW
    K2 = k // NW
    nolds = probe == "nolds"
    # the wave's loads in order: its source columns (every column with "nolds"), then its parity rows
    seq = [("src", c) for c in range(k)] if nolds else [("src", NW * n + w) for n in range(K2)]
    seq += [("par", NW * j + w) for j in range(R)]
    NL = len(seq)
    P = f"r{w}_"
    offs = ["%[o0]", "%[o1]", "%[o2]", "%[o3]"]
    L = []

    def loads(n):
        if probe == "noload":
            return []
        rs = ring(n % NS)
        kind, x = seq[n]
        if kind == "src":
            out = [f"s_bitcmp1_b64 s[{S_EM}:{S_EM + 1}], {x}", f"s_cselect_b32 s{S_LRS + 2}, 0, 0x80000000"]
            slot = x
        else:
            out = [f"s_cmp_lt_u32 {x}, %[e]", f"s_cselect_b32 s{S_LRS + 2}, 0x80000000, 0"]
            slot = k + x
        out.append(f"s_mul_i32 s{S_COL}, %[ss], {slot}")
        for q in range(4):
            out.append(f"buffer_load_dwordx2 v[{rs[2 * q]}:{rs[2 * q + 1]}], {offs[q]}, s[{S_LRS}:{S_LRS + 3}], s{S_COL} offen")
        return out

    def wait(n):
        return [] if probe == "noload" else [f"s_waitcnt vmcnt({4 * (issued - n)})"]

    for r in range(R):
        for i in range(8):
            L.append(f"v_mov_b32 v{acc_reg(r, i)}, 0")
    issued = -1
    for n in range(min(NS, NL)):
        L += loads(n)
        issued = n
    # ---- stage 1: source columns, two per step (one per wave) ----
    nsrc = k if nolds else K2
    for n in range(nsrc):
        rs = ring(n % NS)
        if nolds:  # probe: the wave loads and transposes every column itself, no LDS, no barrier
            L += wait(n)
            L += [f"s_bitcmp1_b64 s[{S_EM}:{S_EM + 1}], {n}", f"s_cbranch_scc1 {P}Lna{n}_%="]
            L += transpose(rs, combo_temps())
            L += column_code(G, w, R, nr, n, rs)
            L.append(f"{P}Lna{n}_%=:")
            if n + NS < NL:
                L += loads(n + NS)
                issued = n + NS
            continue
        own, oth = NW * n + w, NW * n + 1 - w
        slot = n % 2
        L += wait(n)
        L += [f"s_bitcmp1_b64 s[{S_EM}:{S_EM + 1}], {own}", f"s_cbranch_scc1 {P}Lnw{n}_%="]
        L += transpose(rs, combo_temps())
        for i in range(4):
            L.append(f"ds_write_b64 %[la], v[{rs[2 * i]}:{rs[2 * i + 1]}] offset:{(slot * NW + w) * COL_BYTES + i * 512}")
        L.append(f"{P}Lnw{n}_%=:")
        L.append("s_waitcnt lgkmcnt(0)")
        L.append("s_barrier")
        L += [f"s_bitcmp1_b64 s[{S_EM}:{S_EM + 1}], {oth}", f"s_cbranch_scc1 {P}Lnr{n}_%="]
        for i in range(4):
            L.append(f"ds_read_b64 v[{PBUF[2 * i]}:{PBUF[2 * i + 1]}], %[la] offset:{(slot * NW + 1 - w) * COL_BYTES + i * 512}")
        L.append(f"{P}Lnr{n}_%=:")
        L += [f"s_bitcmp1_b64 s[{S_EM}:{S_EM + 1}], {own}", f"s_cbranch_scc1 {P}Lna{n}_%="]
        L += column_code(G, w, R, nr, own, rs)
        L.append(f"{P}Lna{n}_%=:")
        if n + NS < NL:
            L += loads(n + NS)
            issued = n + NS
        L += [f"s_bitcmp1_b64 s[{S_EM}:{S_EM + 1}], {oth}", f"s_cbranch_scc1 {P}Lno{n}_%="]
        L.append("s_waitcnt lgkmcnt(0)")
        L += column_code(G, w, R, nr, oth, PBUF)
        L.append(f"{P}Lno{n}_%=:")
    # ---- stage 1: the wave's parity rows as identity columns ----
    for j in range(R):
        n = nsrc + j
        t = NW * j + w
        rs = ring(n % NS)
        L += wait(n)
        L += [f"s_cmp_le_u32 %[e], {t}", f"s_cbranch_scc1 {P}Lpz{j}_%="]
        L += transpose(rs, combo_temps())
        for i in range(8):
            L.append(f"v_xor_b32 v{acc_reg(j, i)}, v{rs[i]}, v{acc_reg(j, i)}")
        L.append(f"{P}Lpz{j}_%=:")
        if n + NS < NL:
            L += loads(n + NS)
            issued = n + NS
    # ---- z rows out of the accumulators, which become the outputs d ----
    for r in range(R):
        for i in range(8):
            L.append(f"v_mov_b32 v{zreg(r, i)}, v{acc_reg(r, i)}")
    for r in range(R):
        for i in range(8):
            L.append(f"v_mov_b32 v{acc_reg(r, i)}, 0")
    # ---- stage 2: rows 2j, 2j+1 per step, d_s += c[s][t] z_t for the wave's s = 2sl + w ----
    tcode, A, B = window_tables()

    def apply_row(t, creg):
        if probe == "nos2":
            return []
        out = list(tcode)
        out += [f"s_mov_b32 s{S_T}, 0", f"s_set_gpr_idx_on s{S_T}, gpr_idx(SRC0,DST)"]
        for sl in range(R):
            s = NW * sl + w
            out += [f"s_cmp_le_u32 %[e], {s}", f"s_cbranch_scc1 {P}Lse{t}_%="]
            out += [f"s_bfe_u32 s{S_T}, s{creg + s // 4}, 0x{(8 << 16) | (8 * (s % 4)):x}",
                    f"s_lshl_b32 s{S_T}, s{S_T}, {SNIP_ALIGN}",
                    f"s_add_u32 s{S_TAB + 2}, s{S_TAB}, s{S_T}",
                    f"s_addc_u32 s{S_TAB + 3}, s{S_TAB + 1}, 0",
                    f"s_mov_b32 m0, 0x{GPR_MODE | (16 * sl):x}",
                    f"s_swappc_b64 s[{S_RET}:{S_RET + 1}], s[{S_TAB + 2}:{S_TAB + 3}]"]
        out += [f"{P}Lse{t}_%=:", "s_set_gpr_idx_off"]
        return out

    for j in range(R):
        t_own, t_oth = NW * j + w, NW * j + 1 - w
        creg = {NW * j: S_C0, NW * j + 1: S_C1}
        zp = [zreg(j, i) for i in range(8)]
        L += [f"s_cmp_le_u32 %[e], {NW * j}", f"s_cbranch_scc1 {P}Ls2done_%="]
        L.append(f"s_load_dwordx4 s[{S_C0}:{S_C0 + 3}], %[cp], 0x{32 * NW * j:x}")
        L.append(f"s_load_dwordx4 s[{S_C1}:{S_C1 + 3}], %[cp], 0x{32 * (NW * j + 1):x}")
        L += [f"s_cmp_le_u32 %[e], {t_own}", f"s_cbranch_scc1 {P}Lzw{j}_%="]
        for i in range(4):
            L.append(f"ds_write_b64 %[la], v[{zp[2 * i]}:{zp[2 * i + 1]}] offset:{ST2_BASE + ((j % 2) * NW + w) * COL_BYTES + i * 512}")
        L.append(f"{P}Lzw{j}_%=:")
        L.append("s_waitcnt lgkmcnt(0)")
        L.append("s_barrier")
        # the other wave's row: read into the window (j = 0) or into the registers of the
        # wave's row j - 1 (applied already), so the read overlaps the own row's work
        L += [f"s_cmp_le_u32 %[e], {t_oth}", f"s_cbranch_scc1 {P}Lzr{j}_%="]
        dst = PBUF if j == 0 else [zreg(j - 1, i) for i in range(8)]
        for i in range(4):
            L.append(f"ds_read_b64 v[{dst[2 * i]}:{dst[2 * i + 1]}], %[la] offset:{ST2_BASE + ((j % 2) * NW + 1 - w) * COL_BYTES + i * 512}")
        if j == 0:
            L.append("s_waitcnt lgkmcnt(0)")
            L += apply_row(t_oth, creg[t_oth])
        L.append(f"{P}Lzr{j}_%=:")
        L += [f"s_cmp_le_u32 %[e], {t_own}", f"s_cbranch_scc1 {P}Lzo{j}_%="]
        for i in range(8):
            L.append(f"v_mov_b32 v{PBUF[i]}, v{zp[i]}")
        L += apply_row(t_own, creg[t_own])
        L.append(f"{P}Lzo{j}_%=:")
        if j > 0:
            L += [f"s_cmp_le_u32 %[e], {t_oth}", f"s_cbranch_scc1 {P}Lzq{j}_%="]
            L.append("s_waitcnt lgkmcnt(0)")
            for i in range(8):
                L.append(f"v_mov_b32 v{PBUF[i]}, v{dst[i]}")
            L += apply_row(t_oth, creg[t_oth])
            L.append(f"{P}Lzq{j}_%=:")
    L.append(f"{P}Ls2done_%=:")
    # ---- outputs: planes back to bytes, optional accumulate, store into the erased slots ----
    soffs = offs
    tmp = ring(0)
    for sl in range(R):
        s = NW * sl + w
        L += [f"s_cmp_le_u32 %[e], {s}", f"s_cbranch_scc1 {P}Lout_%="]
        d = [acc_reg(sl, i) for i in range(8)]
        L += transpose(d, low_temps())
        L += [f"s_bfe_u32 s{S_T}, s{S_SLOT + s // 2}, 0x{(16 << 16) | (16 * (s % 2)):x}",
              f"s_mul_i32 s{S_T}, s{S_T}, %[ss]",
              "s_cmp_eq_u32 %[acc], 0", f"s_cbranch_scc1 {P}Lna_o{s}_%="]
        for q in range(4):
            L.append(f"buffer_load_dwordx2 v[{tmp[2 * q]}:{tmp[2 * q + 1]}], {soffs[q]}, s[{S_SRS}:{S_SRS + 3}], s{S_T} offen")
        L.append("s_waitcnt vmcnt(0)")
        for q in range(4):
            L.append(f"v_xor_b32 v{d[2 * q]}, v{tmp[2 * q]}, v{d[2 * q]}")
            L.append(f"v_xor_b32 v{d[2 * q + 1]}, v{tmp[2 * q + 1]}, v{d[2 * q + 1]}")
        L.append(f"{P}Lna_o{s}_%=:")
        for q in range(4):
            L.append(f"buffer_store_dwordx2 v[{d[2 * q]}:{d[2 * q + 1]}], {soffs[q]}, s[{S_SRS}:{S_SRS + 3}], s{S_T} offen")
    L.append(f"{P}Lout_%=:")
    L.append("s_waitcnt lgkmcnt(0)")
    L.append("s_branch Lend_%=")
    return L, (A, B)


def fdq2_asm(k, m, probe=None):
    G = generator(k, m)
    L = [f"s_mov_b64 s[{S_LRS}:{S_LRS + 1}], %[base]", f"s_mov_b32 s{S_LRS + 2}, 0x80000000",
         f"s_mov_b32 s{S_LRS + 3}, 0x00020000",
         f"s_mov_b64 s[{S_SRS}:{S_SRS + 1}], %[base]", f"s_mov_b32 s{S_SRS + 2}, 0x80000000",
         f"s_mov_b32 s{S_SRS + 3}, 0x00020000",
         f"s_mov_b64 s[{S_EM}:{S_EM + 1}], %[em]"]
    for i, mk in enumerate(MASKS):
        L.append(f"s_mov_b32 s{S_MASK + i}, 0x{mk:08x}")
    L += [f"s_load_dwordx8 s[{S_SLOT}:{S_SLOT + 7}], %[sp], 0x0",
          f"s_getpc_b64 s[{S_TAB}:{S_TAB + 1}]",
          "Lpc_%=:",
          f"s_add_u32 s{S_TAB}, s{S_TAB}, Lsnip0_%=-Lpc_%=",
          f"s_addc_u32 s{S_TAB + 1}, s{S_TAB + 1}, 0",
          "s_cmp_eq_u32 %[wave], 0",
          "s_cbranch_scc0 Lrole1_%="]
    r0, tabs = role_asm(G, k, m, 0, probe)
    r1, _ = role_asm(G, k, m, 1, probe)
    L += r0
    L.append("Lrole1_%=:")
    L += r1
    L += snippets(*tabs)
    L.append("Lend_%=:")
    return L


def clobbers():
    v = [f'"v{i}"' for i in range(4 * NQ) if i not in IN_REGS]
    s = [f'"s{i}"' for i in range(S_RET, 96)]
    return ", ".join(v + s + ['"m0"', '"scc"', '"memory"'])


# A/B probes and variants of the (64, 32) kernel, NFEC_FDEC_VARIANT=<id>: no stage-1 loads, no
# stage-2 solve, no stage-1 LDS exchange (each wave loads and transposes every column)
PROBES = {1: "noload", 2: "nos2", 3: "nolds"}


def gen_kernel(k, m, probe=None):
    K = f"rs8_fdq2_k{k}_m{m}" + (f"_probe_{probe}" if probe else "")
    body = "\\n\"\n        \"".join(fdq2_asm(k, m, probe))
    return f"""__global__ __launch_bounds__(128, 3) void {K}(FdecArgs a)
{{
    __shared__ uint32_t lds[{LDS_BYTES // 4}];
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t blk = blockIdx.x;
    if (blk >= a.nblocks) return;
    const int32_t rows = (int32_t)__builtin_amdgcn_readfirstlane((uint32_t)a.rows[blk]);
    const uint32_t ps0 = __builtin_amdgcn_readfirstlane(a.psel[2 * (uint64_t)blk]);
    const uint32_t ps1 = __builtin_amdgcn_readfirstlane(a.psel[2 * (uint64_t)blk + 1]);
    // qualifies: 1..16 source erasures repaired from parity rows 0..e-1 (both waves decide alike)
    if (rows <= 0 || rows > 16 || ps1 != 0 || ps0 != ((1u << rows) - 1u)) return;
    const uint32_t e = (uint32_t)rows;
    const uint64_t em = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane(a.emask[2 * (uint64_t)blk]) |
                        ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane(a.emask[2 * (uint64_t)blk + 1]) << 32);
    // both waves have read the plan outputs before wave 0 hands the block off (the unfused
    // stage 1 and solve that follow on the stream skip it)
    __syncthreads();
    if (threadIdx.x == 0) {{
        a.rows[blk] = 0;
        a.psel[2 * (uint64_t)blk] = 0;
    }}
    uint32_t o[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {{
        const uint32_t item = (uint32_t)q * 64u + lane;
        o[q] = item < a.ips ? item * 8u : 0x80000000u;  // past the records: loads read zero, stores drop
    }}
    const uint32_t la = bs::lds_addr(lds) + lane * 8u;
    const uint8_t* base = a.base + (uint64_t)blk * a.block_stride;
    const uint8_t* cp = a.coef + (uint64_t)blk * a.coef_block_stride;
    const uint16_t* sp = a.out_slots + (uint64_t)blk * a.slots_stride;
    asm volatile(
        "{body}\\n"
        :
        : [base] "s"(base), [em] "s"(em), [cp] "s"(cp), [sp] "s"(sp), [e] "s"(e), [ss] "s"(a.seg_stride),
          [acc] "s"(a.accumulate), [wave] "s"(wave),
          [o0] "v"(o[0]), [o1] "v"(o[1]), [o2] "v"(o[2]), [o3] "v"(o[3]), [la] "v"(la)
        : {clobbers()});
}}
"""


def main():
    path = sys.argv[1]
    parts = [
        "// GENERATED by tools/codegen/gen_fdec_q2.py -- do not edit by hand.",
        "// Fused RS8 erasure repair, two waves per block sharing each column's transpose through LDS,",
        "// (k, m) in: " + ", ".join(f"({k},{m})" for k, m in SHAPES),
        "#include <cstdlib>",
        '#include "bitslice.hpp"',
        "",
        "namespace nfec {",
        "namespace {",
    ]
    for k, m in SHAPES:
        parts.append(gen_kernel(k, m))
        if (k, m) == (64, 32):
            for probe in PROBES.values():
                parts.append(gen_kernel(k, m, probe))
    parts.append("}  // namespace")
    parts.append("")
    parts.append("static int fdq2_variant()")
    parts.append("{")
    parts.append("    static const int v = [] { const char* e = std::getenv(\"NFEC_FDEC_VARIANT\"); return e ? std::atoi(e) : 0; }();")
    parts.append("    return v;")
    parts.append("}")
    parts.append("")
    parts.append("// NFEC_ENOTSUP when (k, m) has no kernel or the batch shape needs the unfused path")
    parts.append("int launch_rs8_fused_decode_q2(uint32_t k, uint32_t m, const FdecArgs& a, hipStream_t s)")
    parts.append("{")
    parts.append("    if (a.nblocks == 0) return NFEC_OK;")
    parts.append("    if ((a.vec & 7u) || a.vec > 2048 || a.coef_col_stride != 32 || (a.coef_block_stride & 15) ||")
    parts.append("        (a.slots_stride & 1) || (uint64_t)a.seg_stride * (k + 16) + a.vec >= (1ull << 31))")
    parts.append("        return NFEC_ENOTSUP;")
    for v, probe in PROBES.items():
        parts.append(f"    if (k == 64 && m == 32 && fdq2_variant() == {v}) {{")
        parts.append(f"        hipLaunchKernelGGL(rs8_fdq2_k64_m32_probe_{probe}, dim3(a.nblocks), dim3(128), 0, s, a);")
        parts.append("        return hipGetLastError() == hipSuccess ? NFEC_OK : NFEC_EDEVICE;")
        parts.append("    }")
    for k, m in SHAPES:
        parts.append(f"    if (k == {k} && m == {m}) {{")
        parts.append(f"        hipLaunchKernelGGL(rs8_fdq2_k{k}_m{m}, dim3(a.nblocks), dim3(128), 0, s, a);")
        parts.append("        return hipGetLastError() == hipSuccess ? NFEC_OK : NFEC_EDEVICE;")
        parts.append("    }")
    parts.append("    return NFEC_ENOTSUP;")
    parts.append("}")
    parts.append("")
    parts.append("}  // namespace nfec")
    open(path, "w").write("\n".join(parts) + "\n")


if __name__ == "__main__":
    main()
