#!/usr/bin/env python3
"""Generate norm_amd/csrc/gen_rs8_rt.hip: GF(2^8) block-matrix products with RUNTIME
coefficients, bit-sliced, each coefficient applied by a jump into a 256-entry snippet table.

Every RS8 product the fixed-shape kernels do not cover goes through this kernel: the encode of
any (k, m) with k + m <= 255 (NormEncoderRS8::Encode, src/common/normEncoderRS8.cpp:473-483;
the generator comes from Init, :400-462), shortened blocks (numData < k: the reference just stops
calling Encode at numData, so the product runs over the block's numData columns and the parity
lands at slot numData + r), and the two stages of the generic erasure repair (Decode, :652-757):
z_t = sum over the block's columns of the gathered generator, then d_E = A^-1 z.

The arithmetic is the fixed-shape kernels' (gen_rs8_q4.py): per source column an 8 x 8 bit
transpose of the lane's 32 bytes, the 22 four-Russians combinations of its even planes (group A,
VGPR bank 0) and odd planes (group B, bank 1), then per parity row one v_bitop3 per output plane.
The coefficient is a runtime value, so per (row, column) the wave jumps (s_swappc) into the
128-byte snippet of that value: its 8 updates acc[i] ^= A[a_i(c)] ^ B[b_i(c)] with the
accumulator operands relative to M0 (VGPR index mode on SRC0 and DST), then back (s_setpc).  The
coefficient table holds each coefficient as its snippet's byte offset (u16, c << 7), [column]
[row]; with the table code at a 64 KiB boundary a call target is one s_pack of the table address
and the entry (the RS16 tower kernel's mechanism, gen_gf16_tw.py).

Work split: an item group is 64 lanes x 32 bytes (lane L holds the 8-byte pieces at flat
positions f0 + 512 i + 8 L, so each load is a 512-byte run); a wave owns one pass of at most 8
parity rows of it (64 accumulators in banks 2/3; 128 VGPRs in all: 4 waves per SIMD).  G waves
share an item group (G = 1, 2 or 4, chosen by the row count): in a step of G columns wave w
loads and transposes column G s + w only and hands its planes to the others through LDS; after
one s_barrier every wave applies the G columns to its rows.  More than 8 G rows take several
pass sets (workgroups), each reading the columns again (through L2).

Modes (Rs8RtArgs): flat (item groups run across the blocks of an unshortened batch: one table,
k columns, m rows) or per-block (each item group inside one block: the block's column count,
row count, column slot list, output slot list or numData-relative output slots, and its own
table when the plan made one).

Usage: gen_rs8_rt.py OUT.hip
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gen_rs8_asm import MASKS, S_MASK, acc_reg, split, transpose  # noqa: E402
from gen_rs8_bitsliced import bitmatrix_rows  # noqa: E402

R = 8                     # rows per wave (pass)
SNIP_ALIGN = 7            # 128-byte snippet slots
GPR_MODE = 0x9000         # M0[15:12]: index SRC0 and DST
MULTI = [a for a in range(1, 16) if bin(a).count("1") >= 2]
GS = (1, 2, 4, 8)         # waves per item group


def q2(q):
    """banks 0/1 of quad q"""
    return [4 * q, 4 * q + 1]


def quads(q0, n=4):
    """8 registers: banks 0/1 of quads q0..q0+n-1 (pairs (4q, 4q+1): dwords 2i, 2i+1)"""
    out = []
    for q in range(q0, q0 + n):
        out += q2(q)
    return out


# ---- VGPRs (v0..v127; banks 2/3 = the 8 rows' accumulators, acc_reg(r, i) = acc_reg(0, i) + 16 r) ----
IN_REGS = [0, 1, 4, 5, 8, 9, 112, 113, 116, 117]   # compiler-placed inputs: 4 load offsets, LDS exchange,
                                                   # LDS out offsets, 4 per-piece numData - 1
FREE = [124, 125]                     # left to the compiler as well (it needs a register beside the inputs)
SLOT = quads(3)                       # column being loaded -> transposed planes
S = quads(7)                          # next column's planes (LDS prefetch) / second load slot (G = 1)
W = quads(11)                         # planes being applied (the snippets' single-plane operands)
CA = [4 * (15 + n) for n in range(11)]       # combinations of group A (bank 0)
CB = [4 * (15 + n) + 1 for n in range(11)]   # ... of group B (bank 1)
TMP = quads(26, 2)                    # spare: epilogue temporaries
V_LAST = 127

# ---- SGPRs (clobbered s36..s79; the compiler places the inputs elsewhere) ----
S_DESC, S_ODESC = 36, 40
S_SNIP, S_TGT, S_RET = 44, 46, 48
S_C, S_SB, S_BUF, S_COL, S_T0, S_T1, S_T2, S_WV = 50, 51, 52, 53, 54, 55, 56, 57
S_TBN = 58                            # 2: table address of the column being fetched
S_OFF = [60, 64]                      # 2 x 4: the entries of a column (8 rows, u16 each)
S_SLW = 68                            # the slot-list dword being read
S_TOUCH = 78                          # destination of the scalar-cache touch loads (never read)
S_LAST = 78
S_UNUSED = (69, 70, 71)               # left to the compiler (its SGPR pressure is high around the asm)
assert S_MASK == 72


def operand_maps():
    """A[a] / B[b]: register of the XOR of planes {0,2,4,6} / {1,3,5,7} selected by a / b"""
    A = {1 << t: W[2 * t] for t in range(4)}
    B = {1 << t: W[2 * t + 1] for t in range(4)}
    for n, a in enumerate(MULTI):
        A[a] = CA[n]
        B[a] = CB[n]
    return A, B


def combos_code():
    A, B = operand_maps()
    out = []
    for M in (A, B):
        for a in sorted(MULTI, key=lambda a: bin(a).count("1")):
            top = a.bit_length() - 1
            out.append(f"v_xor_b32 v{M[a]}, v{M[a & ~(1 << top)]}, v{M[1 << top]}")
    return out


def snippets():
    # 64 KiB-aligned table start: a call target is then the table address's high half packed
    # with the 16-bit entry (s_pack_*_b32_b16)
    A, B = operand_maps()
    out = [".p2align 16"]
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


def temps_pool():
    """transpose temporaries: 4 per bank 0/1 per stage, from the combination registers (dead
    while a column is transposed)"""
    def make():
        avail = {0: list(CA[:4]), 1: list(CB[:4])}

        def pick(avoid):
            return avail[1 if avoid == 0 else 0].pop(0)
        return pick
    return make


def epi_pool():
    """temporaries for an accumulator transpose (accumulators in banks 2/3)"""
    def make():
        free = W + CA + CB

        def pick(avoid):
            for i, r in enumerate(free):
                if r % 4 != avoid:
                    return free.pop(i)
            raise RuntimeError("no temp")
        return pick
    return make


def call(r, fast, ebuf):
    """jump into the snippet of row r's entry (in s[ebuf + r // 2], half r % 2); M0 = 16 r"""
    dw, half = ebuf + r // 2, r % 2
    if fast:
        op = "s_pack_lh_b32_b16" if half == 0 else "s_pack_hh_b32_b16"
        L = [f"{op} s{S_TGT}, s{dw}, s{S_SNIP}"]
    else:
        L = [f"s_bfe_u32 s{S_T1}, s{dw}, 0x{(16 << 16) | (16 * half):x}",
             f"s_add_u32 s{S_TGT}, s{S_SNIP}, s{S_T1}",
             f"s_addc_u32 s{S_TGT + 1}, s{S_SNIP + 1}, 0"]
    m0 = "s_mov_b32" if M0_LITERAL else "s_movk_i32"   # (--m0-literal: the round-4 8-byte form, A/B only)
    return L + [f"{m0} m0, 0x{GPR_MODE | (16 * r):x}",
                f"s_swappc_b64 s[{S_RET}:{S_RET + 1}], s[{S_TGT}:{S_TGT + 1}]"]


def sweep(nr, x, ebuf):
    """the rows' jumps for the column whose planes are in W; nr: a fixed row count (fast
    targets), or None (generic targets, rows checked against %[nr])"""
    fast = nr is not None
    L = [f"s_mov_b32 s{S_T0}, 0", f"s_set_gpr_idx_on s{S_T0}, gpr_idx(SRC0,DST)"]
    for r in range(nr if fast else R):
        if not fast:
            L += [f"s_cmp_le_u32 %[nr], {r}", f"s_cbranch_scc1 Lsw{x}_%="]
        L += call(r, fast, ebuf)
    L += [f"Lsw{x}_%=:", "s_set_gpr_idx_off", "s_nop 1"]
    return L


def col_offset(col_sgpr):
    """column index s[col_sgpr] -> its slot's byte offset s[S_COL]: slot = islot0 + c, or the
    per-block slot list isl[c] (u16) when isl != 0 (one scalar load, waited for)"""
    return slot_prefetch(col_sgpr) + ["s_waitcnt lgkmcnt(0)"] + col_offset_slw(col_sgpr)


def slot_prefetch(col_sgpr, add=0):
    """issue the scalar load of the slot-list dword holding column s[col_sgpr] + add into
    s[S_SLW] (nothing in identity mode); a later lgkmcnt(0) wait makes it usable"""
    L = [f"s_cmp_eq_u64 %[isl], 0", f"s_cbranch_scc1 Lpf_%=_{{uid}}",
         f"s_add_u32 s{S_T2}, s{col_sgpr}, %[iph]"]
    if add:
        L.append(f"s_add_u32 s{S_T2}, s{S_T2}, {add}")
    L += [f"s_lshr_b32 s{S_T2}, s{S_T2}, 1", f"s_lshl_b32 s{S_T2}, s{S_T2}, 2",
          f"s_load_dword s{S_SLW}, %[isl], s{S_T2}", f"Lpf_%=_{{uid}}:"]
    return L


def col_offset_slw(col_sgpr):
    """s[S_COL] = byte offset of column s[col_sgpr], its slot read from the prefetched s[S_SLW]"""
    return [f"s_cmp_eq_u64 %[isl], 0", f"s_cbranch_scc1 Lid_%=_{{uid}}",
            f"s_add_u32 s{S_T2}, s{col_sgpr}, %[iph]", f"s_and_b32 s{S_T2}, s{S_T2}, 1",
            f"s_lshl_b32 s{S_T2}, s{S_T2}, 4",
            f"s_lshr_b32 s{S_COL}, s{S_SLW}, s{S_T2}", f"s_and_b32 s{S_COL}, s{S_COL}, 0xffff",
            f"s_branch Lcs_%=_{{uid}}",
            f"Lid_%=_{{uid}}:", f"s_add_u32 s{S_COL}, s{col_sgpr}, %[islot0]",
            f"Lcs_%=_{{uid}}:", f"s_mul_i32 s{S_COL}, s{S_COL}, %[ss]"]


_uid = [0]


def uniq(code):
    _uid[0] += 1
    return [ln.replace("{uid}", str(_uid[0])) for ln in code]


def loads(dst):
    """column s[S_C]'s 4 pieces -> dst.  Flat shortened mode (lnd != 0): a piece whose block has
    numData <= c reads zeros (its offset gets bit 31: past num_records), so each lane's blocks
    stop at their own numData"""
    plain = [f"buffer_load_dwordx2 v[{dst[2 * i]}:{dst[2 * i + 1]}], %[o{i}], s[{S_DESC}:{S_DESC + 3}], s{S_COL} offen"
             for i in range(4)]
    nd = []
    for i in range(4):
        t = TMP[i]
        nd += [f"v_subrev_u32 v{t}, s{S_C}, %[q{i}]",                          # numData - 1 - c
               f"v_and_or_b32 v{t}, v{t}, s{S_DESC + 2}, %[o{i}]",              # sign -> bit 31
               f"buffer_load_dwordx2 v[{dst[2 * i]}:{dst[2 * i + 1]}], v{t}, s[{S_DESC}:{S_DESC + 3}], s{S_COL} offen"]
    return uniq(["s_bitcmp1_b32 %[acc], 1", "s_cbranch_scc0 Lld_%=_{uid}"] + nd +
                ["s_branch Lldx_%=_{uid}", "Lld_%=_{uid}:"] + plain + ["Lldx_%=_{uid}:"])


def table_fetch(col_sgpr, ebuf, add=None):
    """entries of column s[col_sgpr] (+ add) of this wave's rows -> s[ebuf .. ebuf + 3]"""
    L = []
    if add:
        L.append(f"s_add_u32 s{S_T2}, s{col_sgpr}, {add}")
        L.append(f"s_mul_i32 s{S_T2}, s{S_T2}, %[tstep]")
    else:
        L.append(f"s_mul_i32 s{S_T2}, s{col_sgpr}, %[tstep]")
    L += [f"s_add_u32 s{S_TBN}, %[twl], s{S_T2}", f"s_addc_u32 s{S_TBN + 1}, %[twh], 0",
          f"s_load_dwordx4 s[{ebuf}:{ebuf + 3}], s[{S_TBN}:{S_TBN + 1}], 0x0",
          f"s_load_dword s{S_TOUCH}, s[{S_TBN}:{S_TBN + 1}], %[tpf]"]   # warm a line ahead
    return L


XCH_COL = 4 * 512        # bytes per column in the exchange: 4 plane pairs x 64 lanes x 8 bytes


def xch_buf_bytes(G):
    return G * XCH_COL


def step_loop_shared(G, x, nr):
    """G >= 2: a step of G columns shared through LDS.  nr: fixed rows (fast targets), 0 (no
    rows: the wave only loads and shares), None (generic targets)"""
    L = [f"Lstep{x}_%=:", "s_waitcnt vmcnt(0)",
         f"s_cmp_lt_u32 s{S_C}, %[k]", f"s_cbranch_scc0 Lnotr{x}_%="]
    L += transpose(SLOT, temps_pool())
    # my column's planes -> exchange buffer S_BUF, column slot S_WV
    L += [f"s_mul_i32 s{S_T0}, s{S_WV}, {XCH_COL}", f"s_add_u32 s{S_T0}, s{S_T0}, s{S_BUF}",
          f"v_add_u32 v{TMP[0]}, s{S_T0}, %[xl]"]
    for p in range(4):
        L.append(f"ds_write_b64 v{TMP[0]}, v[{SLOT[2 * p]}:{SLOT[2 * p + 1]}] offset:{512 * p}")
    L.append(f"Lnotr{x}_%=:")
    # the slot's data went to LDS: wait before the next column's loads overwrite it
    # (the wait also covers the slot-list dword of the next column, prefetched a step ago)
    L += ["s_waitcnt lgkmcnt(0)",
          f"s_add_u32 s{S_C}, s{S_C}, {G}", f"s_cmp_lt_u32 s{S_C}, %[k]", f"s_cbranch_scc0 Lnl{x}_%="]
    L += uniq(col_offset_slw(S_C)) + loads(SLOT) + uniq(slot_prefetch(S_C, G))
    L += [f"Lnl{x}_%=:", "s_barrier"]
    if nr != 0:
        # fetch column 0 of the step: planes -> S, entries -> buffer 0 (a wave whose item
        # group has fewer columns than the workgroup's longest only keeps the barriers)
        L += [f"s_cmp_lt_u32 s{S_SB}, %[k]", f"s_cbranch_scc0 Lend{x}_%="]
        L += [f"v_add_u32 v{TMP[0]}, s{S_BUF}, %[xl]"]
        L += [f"ds_read_b64 v[{S[2 * p]}:{S[2 * p + 1]}], v{TMP[0]} offset:{512 * p}" for p in range(4)]
        L += table_fetch(S_SB, S_OFF[0])
        for j in range(G):
            y = f"{x}{j}"
            eb = S_OFF[j % 2]
            if j:
                L += [f"s_add_u32 s{S_T0}, s{S_SB}, {j}", f"s_cmp_lt_u32 s{S_T0}, %[k]", f"s_cbranch_scc0 Lend{x}_%="]
            L.append("s_waitcnt lgkmcnt(0)")
            L += [f"v_mov_b32 v{W[i]}, v{S[i]}" for i in range(8)]
            if j + 1 < G:
                L += [f"s_add_u32 s{S_T0}, s{S_SB}, {j + 1}", f"s_cmp_lt_u32 s{S_T0}, %[k]", f"s_cbranch_scc0 Lnf{y}_%="]
                L += [f"v_add_u32 v{TMP[0]}, s{S_BUF}, %[xl]"]
                L += [f"ds_read_b64 v[{S[2 * p]}:{S[2 * p + 1]}], v{TMP[0]} offset:{XCH_COL * (j + 1) + 512 * p}"
                      for p in range(4)]
                L += table_fetch(S_SB, S_OFF[(j + 1) % 2], add=j + 1)
                L.append(f"Lnf{y}_%=:")
            L += combos_code()
            L += sweep(nr, y, eb)
    L += [f"Lend{x}_%=:", f"s_xor_b32 s{S_BUF}, s{S_BUF}, {xch_buf_bytes(G)}", f"s_add_u32 s{S_SB}, s{S_SB}, {G}",
          f"s_cmp_lt_u32 s{S_SB}, %[kl]", f"s_cbranch_scc1 Lstep{x}_%="]
    return L


def step_loop_single(x, nr):
    """G = 1: the wave loads every column itself, one column ahead (slots SLOT / S
    alternate); no LDS, no barrier.  Unrolled by two columns."""
    L = [f"Lstep{x}_%=:"]
    for half, (cur, nxt) in enumerate(((SLOT, S), (S, SLOT))):
        y = f"{x}{half}"
        if half:
            L += [f"s_cmp_lt_u32 s{S_SB}, %[k]", f"s_cbranch_scc0 Lend{x}_%="]
        # this column's entries (fetched a column ago) are in; then the next column's loads
        # (into the other slot) and entries go out
        L += ["s_waitcnt lgkmcnt(0)",
              f"s_add_u32 s{S_C}, s{S_SB}, 1", f"s_cmp_lt_u32 s{S_C}, %[k]", f"s_cbranch_scc0 Lnl{y}_%="]
        L += uniq(col_offset_slw(S_C)) + loads(nxt)
        L += table_fetch(S_C, S_OFF[(half + 1) % 2]) + uniq(slot_prefetch(S_C, 1))
        L += ["s_waitcnt vmcnt(4)", f"s_branch Lgo{y}_%=",
              f"Lnl{y}_%=:", "s_waitcnt vmcnt(0)", f"Lgo{y}_%=:"]
        L += transpose(cur, temps_pool())
        L += [f"v_mov_b32 v{W[i]}, v{cur[i]}" for i in range(8)]
        L += combos_code()
        L += sweep(nr, y, S_OFF[half % 2])
        L += [f"s_add_u32 s{S_SB}, s{S_SB}, 1"]
    L += [f"s_cmp_lt_u32 s{S_SB}, %[k]", f"s_cbranch_scc1 Lstep{x}_%=", f"Lend{x}_%=:"]
    return L


def body(G):
    L = [f"s_mov_b64 s[{S_DESC}:{S_DESC + 1}], %[wb]", f"s_mov_b32 s{S_DESC + 2}, 0x80000000",
         f"s_mov_b32 s{S_DESC + 3}, 0x00020000"]
    for i, mk in enumerate(MASKS):
        L.append(f"s_mov_b32 s{S_MASK + i}, 0x{mk:08x}")
    L += [f"s_getpc_b64 s[{S_SNIP}:{S_SNIP + 1}]",
          "Lpc_%=:",
          f"s_add_u32 s{S_SNIP}, s{S_SNIP}, Lsnip0_%=-Lpc_%=",
          f"s_addc_u32 s{S_SNIP + 1}, s{S_SNIP + 1}, 0",
          f"s_mov_b32 s{S_WV}, %[wv]", f"s_mov_b32 s{S_SB}, 0", f"s_mov_b32 s{S_BUF}, 0"]
    for r in range(R):
        for i in range(8):
            L.append(f"v_mov_b32 v{acc_reg(r, i)}, 0")
    if G == 1:
        # column 0 and its entries; column 1's slot-list dword
        L += [f"s_mov_b32 s{S_C}, 0", f"s_cmp_lt_u32 s{S_C}, %[k]", "s_cbranch_scc0 Lnl0_%="]
        L += uniq(col_offset(S_C)) + loads(SLOT)
        L += table_fetch(S_C, S_OFF[0]) + uniq(slot_prefetch(S_C, 1))
    else:
        L += [f"s_mov_b32 s{S_C}, %[wv]", f"s_cmp_lt_u32 s{S_C}, %[k]", "s_cbranch_scc0 Lnl0_%="]
        L += uniq(col_offset(S_C)) + loads(SLOT) + uniq(slot_prefetch(S_C, G))
    L += ["Lnl0_%=:", f"s_mov_b32 s{S_TGT + 1}, s{S_SNIP + 1}"]
    # helpers (G >= 2, no rows) only load and share
    if G > 1:
        L += ["s_cmp_eq_u32 %[nr], 0", "s_cbranch_scc1 Lstepn_%="]
    # the fast loops pack call targets from the table address's high half: taken when the
    # table starts at a 64 KiB boundary in memory (else the generic loop)
    L += [f"s_and_b32 s{S_T0}, s{S_SNIP}, 0xffff", f"s_cmp_lg_u32 s{S_T0}, 0", "s_cbranch_scc1 Lstepg_%="]
    for nr in range(R, 0, -1):
        L += [f"s_cmp_eq_u32 %[nr], {nr}", f"s_cbranch_scc1 Lstepr{nr}_%="]
    L.append("s_branch Lstepg_%=")
    loops = [(f"r{nr}", nr) for nr in range(R, 0, -1)] + [("g", None)]
    if G > 1:
        loops.append(("n", 0))
    for x, nr in loops:
        L += step_loop_single(x, nr) if G == 1 else step_loop_shared(G, x, nr)
        L.append("s_branch Lepi0_%=")
    L += ["Lepi0_%=:", "s_cmp_eq_u32 %[nr], 0", "s_cbranch_scc1 Lend_%="]
    L += epilogue()
    return L


def epilogue():
    """planes back to bytes per row, optional accumulate, store; then the snippet table"""
    L = [f"s_mov_b64 s[{S_ODESC}:{S_ODESC + 1}], %[ob]", f"s_mov_b32 s{S_ODESC + 2}, 0x80000000",
         f"s_mov_b32 s{S_ODESC + 3}, 0x00020000"]
    so = TMP[:4]   # the lanes' output offsets of the 4 pieces
    for i in range(4):
        L.append(f"ds_read_b32 v{so[i]}, %[lo] offset:{4 * i}")
    # the rows' output slots -> s[S_OFF .. +7] (slot list, or oslot + r)
    # (the list address is 4-byte aligned; oph = 1 when the rows start at its upper half)
    L += ["s_cmp_eq_u64 %[osl], 0", "s_cbranch_scc1 Lflat_%=",
          f"s_load_dwordx8 s[{S_OFF[0]}:{S_OFF[0] + 7}], %[osl], 0x0", "s_waitcnt lgkmcnt(0)",
          "s_cmp_eq_u32 %[oph], 0", "s_cbranch_scc0 Loph_%="]
    # unpack 8 u16 slots in place, back to front (slot r -> s[S_OFF[0] + r]; s60..67 contiguous)
    assert S_OFF[1] == S_OFF[0] + 4
    for ph, lab in ((0, "Lunp0_%="), (1, "Loph_%=")):
        L.append(f"{lab}:")
        for r in range(R - 1, -1, -1):
            u = r + ph
            L.append(f"s_bfe_u32 s{S_OFF[0] + r}, s{S_OFF[0] + u // 2}, 0x{(16 << 16) | (16 * (u % 2)):x}")
        L.append("s_branch Lrows_%=")
    L += ["Lflat_%=:"]
    for r in range(R):
        L.append(f"s_add_u32 s{S_OFF[0] + r}, %[oslot], {r}")
    L.append("Lrows_%=:")
    L.append("s_waitcnt lgkmcnt(0)")
    tmp = S + SLOT
    for r in range(R):
        if r:
            L += [f"s_cmp_le_u32 %[nr], {r}", "s_cbranch_scc1 Lepi_%="]
        d = S_OFF[0] + r
        w = [acc_reg(r, i) for i in range(8)]
        L += transpose(w, epi_pool())
        L += [f"s_mul_i32 s{S_T1}, s{d}, %[oss]", "s_bitcmp1_b32 %[acc], 0", f"s_cbranch_scc0 Lna{r}_%="]
        for i in range(4):
            L.append(f"buffer_load_dwordx2 v[{tmp[2 * i]}:{tmp[2 * i + 1]}], v{so[i]}, s[{S_ODESC}:{S_ODESC + 3}], s{S_T1} offen")
        L.append("s_waitcnt vmcnt(0)")
        for i in range(8):
            L.append(f"v_xor_b32 v{w[i]}, v{w[i]}, v{tmp[i]}")
        L.append(f"Lna{r}_%=:")
        for i in range(4):
            L.append(f"buffer_store_dwordx2 v[{w[2 * i]}:{w[2 * i + 1]}], v{so[i]}, s[{S_ODESC}:{S_ODESC + 3}], s{S_T1} offen")
    L += ["Lepi_%=:", "s_branch Lend_%="]
    L += snippets()
    L.append("Lend_%=:")
    return L


def clobbers():
    v = [f'"v{i}"' for i in range(0, V_LAST + 1) if i not in IN_REGS + FREE]
    s = [f'"s{i}"' for i in range(S_DESC, S_LAST + 1) if i not in S_UNUSED]
    return ", ".join(v + s + ['"m0"', '"scc"', '"memory"'])


M0_LITERAL = False


def main():
    global M0_LITERAL
    if "--m0-literal" in sys.argv:   # A/B builds (tools/ab_build.sh): M0 written with a 32-bit literal
        sys.argv.remove("--m0-literal")
        M0_LITERAL = True
    path = sys.argv[1]
    asms = {G: "\\n\"\n            \"".join(body(G)) for G in GS}
    ins = ", ".join([f'[o{i}] "v"(o[{i}])' for i in range(4)] + [f'[q{i}] "v"(q[{i}])' for i in range(4)])
    common = ("[wb] \"s\"(wb), [ob] \"s\"(ob), [ss] \"s\"(a.in_seg_stride), [oss] \"s\"(a.out_seg_stride), "
              "[k] \"s\"(k), [kl] \"s\"(kl), [nr] \"s\"(nr), [twl] \"s\"(twl), [twh] \"s\"(twh), "
              "[tstep] \"s\"(a.tab_col_stride), [tpf] \"s\"(tpf), [isl] \"s\"(isl), [islot0] \"s\"(a.in_slot0), [osl] \"s\"(osl), "
              "[oslot] \"s\"(oslot), [acc] \"s\"(mode), [wv] \"s\"(pw), [iph] \"s\"(iph), [oph] \"s\"(oph), "
              
              "[lo] \"v\"(lo), [xl] \"v\"(xl), " + ins)
    blocks = []
    for G in GS:
        kw = "if constexpr" if G == GS[0] else "else if constexpr"
        blocks.append(f"""    {kw} (G == {G}) {{
        asm volatile(
            "{asms[G]}\\n"
            :
            : {common}
            : {clobbers()});
    }}""")
    asm_blocks = "\n".join(blocks)
    src = f"""// GENERATED by tools/codegen/gen_rs8_rt.py -- do not edit by hand.
// GF(2^8) block-matrix products with runtime coefficients: bit-sliced, snippet jumps.
#include "nfec_internal.hpp"
#include "bitslice.hpp"

namespace nfec {{
static_assert(kRs8RtRows == {R}u, "gen_rs8_rt.py and nfec_internal.hpp disagree on the rows per pass");
namespace {{

constexpr uint32_t kGroupBytes = 2048;   // 64 lanes x 4 pieces x 8 bytes

template <int G, int NG>
__device__ __forceinline__ void rt_body(const Rs8RtArgs& a, uint32_t wg)
{{
    // NG item groups per workgroup, G waves each
    __shared__ uint32_t lds[G * NG * 64 * 4];                   // the lanes' output offsets (epilogue)
    __shared__ uint64_t xch[(G > 1 ? NG * 2 * G * {XCH_COL} / 8 : 1)];  // column planes exchange
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t gi = wave / G, pw = wave % G;                // item group in the workgroup, wave in the group
    const uint32_t group = wg * NG + gi;
    const bool pb = a.per_block != 0u;
    const uint32_t chunks = (a.vec_bytes + kGroupBytes - 1u) / kGroupBytes;
    const uint32_t blk = pb ? group / chunks : 0u;
    const uint64_t total = pb ? (uint64_t)a.vec_bytes : (uint64_t)a.nblocks * a.vec_bytes;
    const uint64_t f0 = pb ? (uint64_t)(group - blk * chunks) * kGroupBytes : (uint64_t)group * kGroupBytes;
    const bool live = pb ? blk < a.nblocks : f0 < total;
    // this item group's columns and rows
    uint32_t kk = a.k, rows = a.m;
    uint32_t nd = a.k;
    if (live && pb) {{
        if (a.num_data) nd = __builtin_amdgcn_readfirstlane((uint32_t)a.num_data[blk]);
        kk = a.blk_cols ? __builtin_amdgcn_readfirstlane((uint32_t)a.blk_cols[blk]) : (a.num_data ? nd : a.k);
        if (a.blk_rows) {{
            const int32_t e = (int32_t)__builtin_amdgcn_readfirstlane((uint32_t)a.blk_rows[blk]);
            rows = e > 0 ? min((uint32_t)e, a.m) : 0u;
        }}
        // a block with nothing to compute reads nothing: a plan writes no slot list or table for
        // a block it rejected or that has no erasure (e = 0), so they must not be read
        if (rows == 0u || kk == 0u || kk > a.k || nd == 0u || nd > a.k) rows = 0u, kk = 0u;
        if (rows < a.rows_lo || rows > a.rows_hi) rows = 0u, kk = 0u;  // another launch's blocks
    }}
    if (!live) rows = 0u, kk = 0u;
    // the workgroup's largest row and column counts: its waves run the pass sets (8 G rows
    // each) and steps of the longest item group together, with the same barriers (G > 1)
    if (!pb && a.num_data && live) {{
        // flat shortened: columns past every numData of the item group's blocks read zeros, so
        // the group stops at their largest (no valid block: nothing to compute or store)
        const uint32_t bf = (uint32_t)(f0 / a.vec_bytes), bl = (uint32_t)((min(f0 + kGroupBytes, total) - 1u) / a.vec_bytes);
        uint32_t mx = 0;
        for (uint32_t b = bf + lane; b <= bl; b += 64u) {{
            const uint32_t v = a.num_data[b];
            if (v >= 1u && v <= a.k) mx = max(mx, v);
        }}
        for (int off = 32; off > 0; off >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, off));
        kk = __builtin_amdgcn_readfirstlane(mx);
        if (kk == 0u) rows = 0u;
    }}
    uint32_t kl = kk, rl = rows;
    if constexpr (G > 1) {{
        if (NG > 1) {{
            __shared__ uint32_t kmax, rmax;
            if (threadIdx.x == 0) kmax = 0u, rmax = 0u;
            __syncthreads();
            if (lane == 0 && pw == 0) atomicMax(&kmax, kk), atomicMax(&rmax, rows);
            __syncthreads();
            kl = __builtin_amdgcn_readfirstlane(kmax);
            rl = __builtin_amdgcn_readfirstlane(rmax);
        }}
    }}
    if (kl == 0u) return;  // workgroup-uniform (G > 1) / this wave (G = 1): nothing to compute
    const uint32_t b0 = pb ? blk : __builtin_amdgcn_readfirstlane((uint32_t)(min(f0, total - 1) / a.vec_bytes));
    const uint8_t* wb = a.in_base + (uint64_t)b0 * a.in_block_stride;
    const uint8_t* ob = a.out_base + (uint64_t)b0 * a.out_block_stride;
    // flat shortened mode: every piece's block has its own numData (columns at or past it read
    // zeros, parity at slot numData + r); numData is 1..k (a.num_data was validated by the host)
    const uint32_t lnd = !pb && a.num_data ? 1u : 0u;
    uint32_t o[4], q[4];
    uint32_t* po = lds + (wave * 64u + lane) * 4u;
#pragma unroll
    for (int i = 0; i < 4; ++i) {{
        const uint64_t f = f0 + (uint64_t)i * 512u + lane * 8u;
        const uint32_t b = pb ? b0 : (uint32_t)(f / a.vec_bytes);
        const uint32_t p = (uint32_t)(f - (uint64_t)(pb ? 0u : b) * a.vec_bytes);
        const uint32_t raw = lnd && live && f < total ? (uint32_t)a.num_data[b] : a.k;
        // a block whose numData is 0 or past k is left alone, as in per-block mode
        const bool ok = live && f < total && raw >= 1u && raw <= a.k;
        const uint32_t pnd = ok ? raw : 1u;
        q[i] = pnd - 1u;
        o[i] = ok ? (uint32_t)((uint64_t)(b - b0) * a.in_block_stride) + p : 0x80000000u;
        po[i] = ok ? (uint32_t)((uint64_t)(b - b0) * a.out_block_stride + (uint64_t)(lnd ? pnd : 0u) * a.out_seg_stride) + p
                   : 0x80000000u;
    }}
    const uint32_t lo = bs::lds_addr(po);
    const uint32_t xl = bs::lds_addr(xch) + gi * (2u * G * {XCH_COL}u) + lane * 8u;
    const uint8_t* tblk = reinterpret_cast<const uint8_t*>(a.tab) +
                          (pb && a.tab_block_stride ? (uint64_t)(a.tab_by_count ? nd - 1u : blk) * a.tab_block_stride : 0u);
    // scalar-cache touch distance: per-block tables are read once, so the line 4 columns ahead
    // is requested early (a dummy load); shared tables stay cached (touch the current line)
    const uint32_t tpf = __builtin_amdgcn_readfirstlane(pb ? 4u * a.tab_col_stride : 0u);
    // slot lists: 4-byte aligned addresses for the scalar loads, plus the u16 phase
    const uintptr_t isa = pb && a.in_slots ? (uintptr_t)(a.in_slots + (uint64_t)blk * a.in_slots_stride) : 0;
    const uint16_t* isl = reinterpret_cast<const uint16_t*>(isa & ~(uintptr_t)3);
    const uint32_t iph = (uint32_t)(isa >> 1) & 1u;
    const uint32_t mode = __builtin_amdgcn_readfirstlane((a.accumulate ? 1u : 0u) | (lnd << 1));  // bit 0: accumulate, bit 1: flat shortened
    // Pass sets: 8 G rows each, one after another in this workgroup (their second read of a
    // column hits this XCD's L2), as many as the workgroup's largest row count needs.  The row
    // pass of a wave is rotated by the workgroup, so that when some waves of an item group have
    // no rows (rows < 8 G) the busy ones land on different SIMDs from one workgroup to the next.
    const uint32_t pr = (pw + wg % G) % G;
    for (uint32_t set = 0; set * G * {R}u < rl; ++set) {{
        if constexpr (G > 1) {{
            if (set) __syncthreads();  // the exchange buffers are reused
        }}
        uint32_t row0 = 0, row1 = 0;
        rs8_rt_pass_rows(rows, set * G + pr, row0, row1);
        const uint32_t nr = a.probe_noapply ? 0u : __builtin_amdgcn_readfirstlane(row1 - row0);
        // (an item group whose rows end before this set only keeps the workgroup's barriers)
        const uint32_t k = __builtin_amdgcn_readfirstlane(set * G * {R}u < rows ? kk : 0u);
        const uint8_t* tb = tblk + (a.tab_pass_stride ? (uint64_t)(set * G + pr) * a.tab_pass_stride : 2u * row0);
        const uint32_t twl = (uint32_t)(uintptr_t)tb, twh = (uint32_t)((uintptr_t)tb >> 32);
        const uintptr_t osa = pb && a.out_slots ? (uintptr_t)(a.out_slots + (uint64_t)blk * a.out_slots_stride + row0) : 0;
        const uint16_t* osl = reinterpret_cast<const uint16_t*>(osa & ~(uintptr_t)3);
        const uint32_t oph = (uint32_t)(osa >> 1) & 1u;
        const uint32_t oslot = a.out_slot0 + (a.out_after_data && !lnd ? nd : 0u) + row0;  // (lnd: numData in po)
{asm_blocks}
    }}
}}

template <int G, int NG>
__global__ __launch_bounds__(64 * G * NG, 4) void rs8_rt_kernel(Rs8RtArgs a)
{{
    rt_body<G, NG>(a, bs::wg_index(1));
}}

}}  // namespace

bool rs8_rt_covers(const Rs8RtArgs& a)
{{
    if ((a.vec_bytes & 7u) || a.vec_bytes == 0 || !a.tab || a.k == 0 || (a.tab_col_stride & 3u) ||
        (a.per_block && (a.tab_block_stride & 3u)) || (a.tab_pass_stride & 3u))
        return false;
    // every offset a wave forms stays below 2^31 (a flat item group spans at most
    // 2048 / vec + 2 blocks), as do the slot offsets
    const uint64_t nbg = a.per_block ? 1u : kGroupBytes / a.vec_bytes + 2u;
    const uint64_t bound = a.slot_bound ? a.slot_bound : 65536u;
    const uint64_t in_slots = a.in_slots ? bound : (uint64_t)a.in_slot0 + a.k;
    const uint64_t out_slots = a.out_slots ? bound : (uint64_t)a.out_slot0 + (a.out_after_data ? a.k : 0u) + a.m;
    return nbg * a.in_block_stride + in_slots * a.in_seg_stride + a.vec_bytes < (1ull << 31) &&
           nbg * a.out_block_stride + out_slots * a.out_seg_stride + a.vec_bytes < (1ull << 31);
}}

int launch_rs8_rt(const Rs8RtArgs& in, hipStream_t s)
{{
    if (in.nblocks == 0 || in.m == 0) return NFEC_OK;
    if (!rs8_rt_covers(in)) return NFEC_ENOTSUP;
    Rs8RtArgs a = in;
    // waves per item group: by the row count when every block has m rows (every wave busy);
    // launches whose rows differ per block (the repairs, e usually well below capacity) one wave
    // up to 8 rows, else two
    // (measured: four waves there leave two mostly idle, profiles/r04/rt_gsplit.jsonl)
    const bool var_rows = a.per_block && a.blk_rows;  // rows differ per block (the repairs)
    uint32_t G = a.m <= {R}u ? 1u : (a.m <= {2 * R}u || var_rows) ? 2u : 4u;
    // (NFEC_RT_G=1/2/4: that split for every launch, A/B only; NFEC_RT_GPB: per-block launches)
    // more than 32 rows (every block the same): eight waves of 8 rows share each column's load
    // and transpose, one pass set up to 64 rows instead of two (NFEC_RT_G8=0: four waves, A/B)
    static const long g8 = diag_knob("NFEC_RT_G8", 1);
    if (G == 4 && g8 && a.m > 4u * {R}u) G = 8;
    static const long g_all = diag_knob("NFEC_RT_G", 0, 0, 8), g_pb = diag_knob("NFEC_RT_GPB", 0, 0, 8);
    const long gk = a.per_block && g_pb ? g_pb : g_all;
    if (gk == 1 || gk == 2 || gk == 4 || gk == 8) G = (uint32_t)gk;
    a.pass_sets = (a.m + G * {R}u - 1u) / (G * {R}u);  // (informational: the kernel loops over them)
    // NFEC_RT_PROBE=1 (diagnostic library only, wrong results): every column reads slot 0 of its
    // block, so the loads hit the cache -- the kernel's time without HBM read latency
    // =2: every coefficient the empty snippet (calls kept, their VALU gone: the table reads
    // one zeroed line); =3: no rows applied (loads, transposes and exchange only)
    static const long probe = diag_knob("NFEC_RT_PROBE", 0, 0, 3);
    if (probe == 1) a.in_seg_stride = 0;
    if (probe == 2) {{
        static uint16_t* zeros = nullptr;
        if (!zeros) {{
            if (hipMalloc(&zeros, 256) != hipSuccess || hipMemset(zeros, 0, 256) != hipSuccess) return NFEC_EDEVICE;
        }}
        a.tab = zeros;
        a.tab_block_stride = 0;
        a.tab_pass_stride = 0;
        a.tab_col_stride = 0;
        a.tab_by_count = 0;
    }}
    if (probe == 3) a.probe_noapply = 1;
    const uint64_t groups = a.per_block ? (uint64_t)a.nblocks * ((a.vec_bytes + kGroupBytes - 1u) / kGroupBytes)
                                        : ((uint64_t)a.nblocks * a.vec_bytes + kGroupBytes - 1u) / kGroupBytes;
    // item groups per workgroup: four waves per workgroup, except per-block launches of two-wave
    // groups, one group per workgroup (its barriers then hold only its own two waves, not
    // another block's; NFEC_RT_PBNG=2: two groups, A/B)
    static const long pbng = diag_knob("NFEC_RT_PBNG", 1, 1, 2);
    const uint32_t ng2 = a.per_block ? (uint32_t)pbng : 2u;
    const uint32_t NGs = G == 1 ? 4u : G == 2 ? ng2 : 1u;
    const uint64_t wgs = (groups + NGs - 1u) / NGs;
    if (wgs >= (1ull << 31)) return NFEC_ENOTSUP;
    auto launch2 = [&](const Rs8RtArgs& x) {{
        if (ng2 == 1) hipLaunchKernelGGL((rs8_rt_kernel<2, 1>), dim3((uint32_t)wgs), dim3(128), 0, s, x);
        else hipLaunchKernelGGL((rs8_rt_kernel<2, 2>), dim3((uint32_t)wgs), dim3(256), 0, s, x);
    }};
    if (var_rows && G == 2 && !gk) {{
        // per-block rows vary: blocks of at most {R} rows by one wave each (its own columns, no
        // exchange), the others by two waves sharing columns -- two launches, each skipping the
        // other's blocks (one wave loses to two from 9 rows up, two waves with one of them idle
        // lose to one below; profiles/r04/rt_gsplit.jsonl)
        Rs8RtArgs lo = a, hi = a;
        lo.rows_hi = {R}u;
        hi.rows_lo = {R + 1}u;
        const uint64_t wgs1 = (groups + 3u) / 4u;
        if (wgs1 >= (1ull << 31)) return NFEC_ENOTSUP;
        hipLaunchKernelGGL((rs8_rt_kernel<1, 4>), dim3((uint32_t)wgs1), dim3(256), 0, s, lo);
        launch2(hi);
    }} else if (G == 1) hipLaunchKernelGGL((rs8_rt_kernel<1, 4>), dim3((uint32_t)wgs), dim3(256), 0, s, a);
    else if (G == 2) launch2(a);
    else if (G == 4) hipLaunchKernelGGL((rs8_rt_kernel<4, 1>), dim3((uint32_t)wgs), dim3(256), 0, s, a);
    else hipLaunchKernelGGL((rs8_rt_kernel<8, 1>), dim3((uint32_t)wgs), dim3(512), 0, s, a);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? NFEC_OK : hip_fail(e, "rs8 runtime-coefficient product launch");
}}

}}  // namespace nfec
"""
    open(path, "w").write(src)


if __name__ == "__main__":
    main()
