#!/usr/bin/env python3
"""Generate norm_amd/csrc/gen_gf16_t3.hip: RS16 (GF(2^16)) encode, bit-sliced, with the
four-Russians tables of each source column built ONCE per workgroup in LDS and shared by 11
row waves.

The reference multiplies symbol by symbol through log/exp tables (NormEncoderRS16::Encode,
src/common/normEncoderRS16.cpp:472-482, addmul1 :261-298).  Over GF(2) multiplication by a
constant c is a 16 x 16 bit matrix M_c, so with the data bit-sliced (plane q = bit q of 32
symbols) output plane p of c*x is the XOR of the input planes q with bit q of row p of M_c.
The 16 input planes are split into three groups of 6, 5 and 5 planes; per source column the
XOR of every subset of each group is tabulated (64 + 32 + 32 rows), so each output plane is
three table reads and two XORs.  The row of M_c for a plane only picks table rows: the
generator's coefficients become a precomputed list of LDS offsets (gf16_t3_offsets, 96 bytes
per coefficient) read by scalar loads.

Workgroup = 12 waves on one item group (64 lanes x 64 symbols: lane L holds 16 pieces of
8 bytes, piece i at flat position f0 + 512 i + 8 L, so every load is a 512-byte run):
  * wave 0 (builder) loads source column c+2 (16 x buffer_load_dwordx2 per lane), transposes
    column c+1 (two 16 x 16 bit transposes: the lane's 64 symbols are 2 x 32), and writes its
    tables into the LDS buffer (c+1) % 2 (Gray-code order, one XOR per row and half);
  * waves 1..11 (row waves) each own 4 parity rows (16 planes x 2 halves = 128 accumulator
    VGPRs) and apply column c from buffer c % 2: per plane three v_add_u32_sdwa address
    (16-bit offset from the SGPR list + lane base) + ds_read_b64, a bitop3 and a xor per half;
  * one s_barrier per column; tables 2 x 64 KiB.
A workgroup covers 44 rows; the grid runs ceil(m / 44) passes per item group.

VGPR banks (index mod 4): the table reads land as pairs (banks 0,1 / 2,3), so half 0 of an
accumulator sits in an odd bank and half 1 in an even one -- every bitop3 reads three banks.

Usage: gen_gf16_t3.py OUT.hip
"""
import sys

ROWS = 4                 # parity rows per row wave
RWAVES = 11              # row waves per workgroup (15 x 3 rows at 4 waves/SIMD measured no faster)
RP = ROWS * RWAVES       # rows per pass
NWAVES = RWAVES + 1
GROUPS = [(0, 6, 0), (6, 5, 64), (11, 5, 96)]   # (first plane, planes, first table row)
TROWS = 128
BUF = TROWS * 512        # one table buffer: 128 rows x 64 lanes x 8 bytes
OFF_LDS = 2 * BUF        # piece offsets in the output layout (epilogue stores): 64 lanes x 16 dwords
OFF_ACC = OFF_LDS + 4096 # ... and in the accumulate-source layout
S_ODESC, S_ADESC = 60, 64  # row-wave epilogue: output / accumulate-source descriptors (over S_SB[1])
MASKS = {8: 0x00FF00FF, 4: 0x0F0F0F0F, 2: 0x33333333, 1: 0x55555555}

# ---- SGPRs used inside the asm bodies (clobbered) ----
S_SB = [36, 60]          # row waves: offsets double buffer, 24 SGPRs each (4-aligned)
S_DESC = 84              # buffer descriptor (4)
S_PTR = 88               # row waves: offsets pointer (2)
S_CNT = 90               # column counter
S_T0, S_T1 = 91, 92      # scratch
S_T2 = 93                # builder: column-map scratch
S_MASK = 36              # s36..s43 transpose masks (builder; row waves: epilogue, over S_SB[0])
S_LAST = 92


# ---- row-wave VGPRs ----
def acc(r, p, h):
    """half 0 in an odd bank, half 1 in the even one below it"""
    return 2 * (16 * r + p) + (1 - h)


T_BASE = 32 * ROWS
DEPTH = 4                # planes whose table reads are in flight beyond the one computed
NSLOT = DEPTH + 1        # read-target slots: quads v128.., pairs after them
A_BASE = T_BASE + 6 * NSLOT          # 4 rotating address registers
V_B0, V_B1 = A_BASE + 4, A_BASE + 5  # lane*8 + buffer base (0 / 64 KiB), pinned inputs


def row_slot(pp):
    """(tA, tB, tC) register pairs for read slot pp: tA banks (0,1), tB (2,3), tC even pair"""
    quad = T_BASE + 4 * pp
    tc = T_BASE + 4 * NSLOT + 2 * pp
    return (quad, quad + 1), (quad + 2, quad + 3), (tc, tc + 1)


def transpose16(x, temps):
    """16 x 16 bit transpose (low and high halves of x[0..15] at once), in place;
    swapmove stages 8, 4, 2, 1 (kernels_gf16bs.hip transpose16)."""
    out = []
    ti = 0
    for s in (8, 4, 2, 1):
        mi = {8: 0, 4: 2, 2: 4, 1: 6}[s]
        for d in range(16):
            if d & s:
                continue
            lo, hi = x[d], x[d + s]
            tu, tv = temps[ti % len(temps)], temps[(ti + 1) % len(temps)]
            ti += 2
            out.append(f"v_lshrrev_b32 v{tu}, {s}, v{lo}")
            out.append(f"v_lshlrev_b32 v{tv}, {s}, v{hi}")
            out.append(f"v_bitop3_b32 v{hi}, s{S_MASK + mi}, v{tu}, v{hi} bitop3:0xca")
            out.append(f"v_bitop3_b32 v{lo}, s{S_MASK + mi + 1}, v{tv}, v{lo} bitop3:0xca")
    return out


def mask_init():
    out = []
    for s, mi in ((8, 0), (4, 2), (2, 4), (1, 6)):
        out.append(f"s_mov_b32 s{S_MASK + mi}, 0x{MASKS[s]:08x}")
        out.append(f"s_mov_b32 s{S_MASK + mi + 1}, 0x{(MASKS[s] << s) & 0xFFFFFFFF:08x}")
    return out


# ---- builder (wave 0) ----
B_RING = [0, 32]         # two 32-register data slots: v0..v31, v32..v63
B_TMP = [64, 65, 66, 67]
B_CUR = [(68, 69), (70, 71)]   # Gray-code running values (ping-pong), half 0 / half 1
B_ZERO = (72, 73)


# builder variants (NFEC_T3_VARIANT=<id> for A/B runs; add them to BUILDER_VARIANTS to build):
#   "prio"    raise the builder's issue priority above the row waves on its SIMD
#   "ilp"     build the three groups' Gray-code chains interleaved (6 independent XOR chains)
#   "deep"    three source columns in flight instead of two
#   "nochain" / "notr": timing probes (wrong parity): no Gray-code XORs / no transposes
# Measured on C4 (4,096 blocks, Toeplitz split, one MI355X): default 179.2-180.2 ms; prio 179.9,
# ilp 180.0, prio+ilp 180.3, deep 180.4, deep+ilp 180.0; nochain 188.8, notr 176.1, both 175.6.
# The builder does not set the column step: the row waves' VALU does (7 per row, plane and
# 64 symbols: 3 address adds for the table reads, a bitop3 and a xor per half), DESIGN.md RS16.
#   "nodrain" (row waves): timing probe without the lgkmcnt(0) at each row start that waits for
#             the row's scalar-loaded offsets: 178.6-178.8 against 179.8-180.2 ms, under 1 %.
#   "timed"   probe: s_memtime around the builder's phases, printf from workgroup 0
#             (profiles/r02/t3_builder_timing.txt): per column the builder's build + table-write
#             drain takes ~5,000 shader clocks and it then waits ~2,500 (44 rows) / ~1,600 (20
#             rows) at the barrier for the row waves; loads wait ~130.
BUILDER_VARIANTS = {0: ()}
DIAG_BUILDER_VARIANTS = {0: (), 1: ("timed",)}   # --diag (make -C norm_amd diag) only
T3_DEFAULT = 0
B_CUR3 = [[(68, 69), (70, 71)], [(74, 75), (76, 77)], [(78, 79), (80, 81)]]  # per group (ilp)
# "deep" register map: three 32-register slots v0..v95, then temporaries (four slots leave the
# compiler too few registers for the asm's inputs)
D_NS = 3
D_RING = [0, 32, 64]
D_TMP = [96, 97, 98, 99]
D_CUR = [(100, 101), (102, 103)]
D_CUR3 = [[(100, 101), (102, 103)], [(104, 105), (106, 107)], [(108, 109), (110, 111)]]
D_ZERO = (112, 113)


def builder_regs(flags):
    if "deep" in flags:
        return D_RING, D_TMP, D_CUR, D_CUR3, D_ZERO
    return B_RING, B_TMP, B_CUR, B_CUR3, B_ZERO


def STAMP(acc):
    """timing probe: add the shader clocks since the last stamp to s<acc>"""
    return ["s_memtime s[94:95]", "s_waitcnt lgkmcnt(0)", "s_sub_u32 s100, s94, s99",
            f"s_add_u32 s{acc}, s{acc}, s100", "s_mov_b32 s99, s94"]


def builder_asm(flags=()):
    ring, tmp, bcur, bcur3, bzero = builder_regs(flags)
    L = []
    if "prio" in flags:
        L.append("s_setprio 3")
    L += [f"s_mov_b64 s[{S_DESC}:{S_DESC + 1}], %[wb]", f"s_mov_b32 s{S_DESC + 2}, 0x80000000",
          f"s_mov_b32 s{S_DESC + 3}, 0x00020000"]
    L += mask_init()
    offs = [f"%[o{i}]" for i in range(16)]

    def loads(slot):
        # column index in S_T0 (set by the caller) -> byte offset in S_T1 through the column
        # map: ((c >> csh) * cck + (c & cmk) * ss + cbb; identity: csh 31, cck 0, cmk ~0, cbb 0)
        out = [f"s_lshr_b32 s{S_T2}, s{S_T0}, %[csh]", f"s_mul_i32 s{S_T2}, s{S_T2}, %[cck]",
               f"s_and_b32 s{S_T1}, s{S_T0}, %[cmk]", f"s_mul_i32 s{S_T1}, s{S_T1}, %[ss]",
               f"s_add_u32 s{S_T1}, s{S_T1}, s{S_T2}", f"s_add_u32 s{S_T1}, s{S_T1}, %[cbb]"]
        base = ring[slot]
        for i in range(16):
            out.append(f"buffer_load_dwordx2 v[{base + 2 * i}:{base + 2 * i + 1}], {offs[i]}, s[{S_DESC}:{S_DESC + 3}], s{S_T1} offen")
        return out

    def build(slot, buf):
        """transpose the slot, write its tables into LDS buffer buf"""
        out = []
        base = ring[slot]
        halves = [[base + d for d in range(16)], [base + 16 + d for d in range(16)]]
        for h in (0, 1):
            if "notr" not in flags:
                out += transpose16(halves[h], tmp)
        lb = "%[lb0]" if buf == 0 else "%[lb1]"

        def chain(gi):
            """(instructions of one Gray-code step) for group gi, in order"""
            first, n, row0 = GROUPS[gi]
            cur = bcur3[gi] if "ilp" in flags else bcur
            steps, prev, k = [], 0, 0
            for i in range(1, 1 << n):
                g = i ^ (i >> 1)
                q = (g ^ prev).bit_length() - 1
                dst, srcp = cur[k % 2], cur[(k + 1) % 2]
                st = []
                for h in (0, 1):
                    plane = halves[h][first + q]
                    if "nochain" in flags:
                        continue
                    if prev == 0:
                        st.append(f"v_mov_b32 v{dst[h]}, v{plane}")
                    else:
                        st.append(f"v_xor_b32 v{dst[h]}, v{srcp[h]}, v{plane}")
                st.append(f"ds_write_b64 {lb}, v[{dst[0]}:{dst[1]}] offset:{(row0 + g) * 512}")
                steps.append(st)
                prev, k = g, k + 1
            return steps

        chains = [chain(gi) for gi in range(len(GROUPS))]
        if "ilp" in flags:
            # round-robin over the groups: the 63-step chain of group 0 with the two 31-step
            # chains of groups 1 and 2 beside it
            for i in range(max(len(c) for c in chains)):
                for c in chains:
                    if i < len(c):
                        out += c[i]
        else:
            for c in chains:
                for st in c:
                    out += st
        return out

    # zero rows of both buffers; piece offsets for the row waves' epilogue
    L += [f"v_mov_b32 v{bzero[0]}, 0", f"v_mov_b32 v{bzero[1]}, 0"]
    for lb in ("%[lb0]", "%[lb1]"):
        for _, _, row0 in GROUPS:
            L.append(f"ds_write_b64 {lb}, v[{bzero[0]}:{bzero[1]}] offset:{row0 * 512}")
    if "deep" in flags:
        return L + deep_loop(loads, build)
    # prologue: column 0 -> slot 0 (wait), column 1 -> slot 1 (in flight), build column 0
    L += [f"s_mov_b32 s{S_T0}, 0"] + loads(0)
    L += ["s_cmp_gt_u32 %[k], 1", "s_cbranch_scc0 Lb_one_%=", f"s_mov_b32 s{S_T0}, 1"] + loads(1)
    L += ["s_waitcnt vmcnt(16)", "s_branch Lb_built0_%=", "Lb_one_%=:", "s_waitcnt vmcnt(0)", "Lb_built0_%=:"]
    L += build(0, 0)
    # column 2 into the slot column 0 just left
    L += ["s_cmp_gt_u32 %[k], 2", "s_cbranch_scc0 Lb_no2_%=", f"s_mov_b32 s{S_T0}, 2"] + loads(0) + ["Lb_no2_%=:"]
    L += ["s_waitcnt lgkmcnt(0)", "s_barrier"]
    timed = "timed" in flags
    if timed:  # probe: s96 load wait, s97 build + table-write drain, s98 barrier (shader clocks)
        L += ["s_memtime s[94:95]", "s_waitcnt lgkmcnt(0)", "s_mov_b32 s99, s94", "s_mov_b32 s96, 0",
              "s_mov_b32 s97, 0", "s_mov_b32 s98, 0"]
    # loop: at column c build c+1 (slot (c+1)%2, buffer (c+1)%2), load c+3 into slot c%2...
    # unrolled by two so slots and buffers are compile-time: iteration A has c even.
    L += [f"s_mov_b32 s{S_CNT}, 0"]
    for par in (0, 1):
        L.append(f"Lb_it{par}_%=:")
        nxt = 1 - par                    # slot / buffer of column c+1
        # done when c == k-1 (nothing left to build); the last barrier still happens
        L += [f"s_add_u32 s{S_T0}, s{S_CNT}, 1", "s_cmp_ge_u32 s%d, %%[k]" % S_T0, "s_cbranch_scc1 Lb_tail_%="]
        # data of column c+1 must be in: if column c+2 was issued, 16 loads are younger
        L += [f"s_add_u32 s{S_T1}, s{S_CNT}, 2", "s_cmp_lt_u32 s%d, %%[k]" % S_T1,
              f"s_cbranch_scc0 Lb_w0_{par}_%=", "s_waitcnt vmcnt(16)", f"s_branch Lb_w1_{par}_%=",
              f"Lb_w0_{par}_%=:", "s_waitcnt vmcnt(0)", f"Lb_w1_{par}_%=:"]
        if timed:
            L += STAMP(96)
        L += build(nxt, nxt)
        # column c+3 into slot (c+1)%2 ... no: slot of column c+3 is (c+3)%2 = (c+1)%2, which
        # holds column c+1 until its tables are written: issue after the build
        L += [f"s_add_u32 s{S_T0}, s{S_CNT}, 3", "s_cmp_lt_u32 s%d, %%[k]" % S_T0, f"s_cbranch_scc0 Lb_nl_{par}_%="]
        L += loads(nxt)
        L.append(f"Lb_nl_{par}_%=:")
        L += ["s_waitcnt lgkmcnt(0)"]
        if timed:
            L += STAMP(97)
        L += ["s_barrier"]
        if timed:
            L += STAMP(98)
        L += [f"s_add_u32 s{S_CNT}, s{S_CNT}, 1"]
        if par == 0:
            pass
        else:
            L.append("s_branch Lb_it0_%=")
    L += ["Lb_tail_%=:", "s_waitcnt vmcnt(0)", "s_barrier"]
    return L


def deep_loop(loads, build):
    """D_NS slots: column j in slot j % D_NS, tables in buffer j % 2; at column step c the
    builder builds column c + 1, then loads column c + 1 + D_NS into the slot c + 1 just left"""
    ns = D_NS
    L = []
    # prologue: columns 0..ns-1 in flight, wait for column 0, build it, load column ns
    L += [f"s_mov_b32 s{S_T0}, 0"] + loads(0)
    for j in range(1, ns):
        L += [f"s_cmp_gt_u32 %[k], {j}", f"s_cbranch_scc0 Lb_pl{j}_%=", f"s_mov_b32 s{S_T0}, {j}"] + loads(j)
        L.append(f"Lb_pl{j}_%=:")
    L += wait_for(f"s_sub_u32 s{S_T1}, %[k], 1", "p", ns - 1)
    L += build(0, 0)
    L += [f"s_cmp_gt_u32 %[k], {ns}", f"s_cbranch_scc0 Lb_pln_%=", f"s_mov_b32 s{S_T0}, {ns}"] + loads(0) + ["Lb_pln_%=:"]
    L += ["s_waitcnt lgkmcnt(0)", "s_barrier", f"s_mov_b32 s{S_CNT}, 0"]
    unroll = ns * 2 // (2 if ns % 2 == 0 else 1)  # lcm(ns, 2)
    for u in range(unroll):
        L.append(f"Lb_it{u}_%=:")
        nslot, nbuf = (u + 1) % ns, (u + 1) % 2
        L += [f"s_add_u32 s{S_T0}, s{S_CNT}, 1", "s_cmp_ge_u32 s%d, %%[k]" % S_T0, "s_cbranch_scc1 Lb_tail_%="]
        # columns issued beyond c+1: c+2 .. min(k-1, c+ns), i.e. clamp(k - c - 2, 0, ns-1)
        L += wait_for(f"s_sub_u32 s{S_T1}, %[k], s{S_CNT}", f"i{u}", ns - 1, extra=[f"s_sub_u32 s{S_T1}, s{S_T1}, 2"])
        L += build(nslot, nbuf)
        L += [f"s_add_u32 s{S_T0}, s{S_CNT}, {1 + ns}", "s_cmp_lt_u32 s%d, %%[k]" % S_T0, f"s_cbranch_scc0 Lb_nl_{u}_%="]
        L += loads(nslot)
        L.append(f"Lb_nl_{u}_%=:")
        L += ["s_waitcnt lgkmcnt(0)", "s_barrier", f"s_add_u32 s{S_CNT}, s{S_CNT}, 1"]
    L.append("s_branch Lb_it0_%=")
    L += ["Lb_tail_%=:", "s_waitcnt vmcnt(0)", "s_barrier"]
    return L


def wait_for(first, tag, nmax, extra=()):
    """s_waitcnt vmcnt(16 * n) with n = clamp(S_T1, 0, nmax) computed by `first` (+ `extra`):
    the loads of the n columns issued after the one needed may stay in flight (S_T1 is a
    signed count; the comparisons are signed)"""
    L = [first] + list(extra)
    L += [f"s_cmp_ge_i32 s{S_T1}, {nmax}", f"s_cbranch_scc1 Lb_w{nmax}{tag}_%="]
    for n in range(nmax - 1, 0, -1):
        L += [f"s_cmp_eq_i32 s{S_T1}, {n}", f"s_cbranch_scc1 Lb_w{n}{tag}_%="]
    L += ["s_waitcnt vmcnt(0)", f"s_branch Lb_wd{tag}_%="]
    for n in range(1, nmax + 1):
        L += [f"Lb_w{n}{tag}_%=:", f"s_waitcnt vmcnt({16 * n})"]
        if n < nmax:
            L.append(f"s_branch Lb_wd{tag}_%=")
    L.append(f"Lb_wd{tag}_%=:")
    return L


def builder_clobbers(flags=()):
    if "deep" in flags:
        return ", ".join([f'"v{i}"' for i in range(D_ZERO[1] + 1)] + [f'"s{i}"' for i in range(S_DESC, S_T2 + 1)] +
                         ['"scc"', '"memory"'])
    v = [f'"v{i}"' for i in range(82)]
    s = [f'"s{i}"' for i in range(S_DESC, (100 if "timed" in flags else S_T2) + 1)]
    return ", ".join(v + s + ['"scc"', '"memory"'])


# ---- row waves ----
def row_asm(flags=()):
    L = []
    L += [f"s_mov_b64 s[{S_DESC}:{S_DESC + 1}], %[wb]", f"s_mov_b32 s{S_DESC + 2}, 0x80000000",
          f"s_mov_b32 s{S_DESC + 3}, 0x00020000"]
    for r in range(ROWS):
        for p in range(16):
            for h in (0, 1):
                L.append(f"v_mov_b32 v{acc(r, p, h)}, 0")
    L += [f"s_mov_b64 s[{S_PTR}:{S_PTR + 1}], %[op]"]
    sb = S_SB

    def sload(dst):
        return [f"s_load_dwordx8 s[{dst + 8 * i}:{dst + 8 * i + 7}], s[{S_PTR}:{S_PTR + 1}], 0x{32 * i:x}" for i in range(3)]

    def advance(row_in_wave):
        """move the pointer to the next (column, row): +96 within a column, else to the next
        column's first row of this wave"""
        if row_in_wave < ROWS - 1:
            return [f"s_add_u32 s{S_PTR}, s{S_PTR}, 96", f"s_addc_u32 s{S_PTR + 1}, s{S_PTR + 1}, 0"]
        return [f"s_add_u32 s{S_PTR}, s{S_PTR}, %[cstep]", f"s_addc_u32 s{S_PTR + 1}, s{S_PTR + 1}, 0"]

    # prologue: offsets of (column 0, row 0)
    L += sload(sb[0]) + advance(0) + ["s_waitcnt lgkmcnt(0)", "s_barrier", f"s_mov_b32 s{S_CNT}, 0"]

    def column(buf):
        """the column's 4 rows x 16 planes as one pipeline: the three table reads of plane
        i + DEPTH are issued before plane i is applied (counted lgkmcnt waits; LDS returns in
        order, and the offsets' scalar loads in flight only make a count wait longer)"""
        out = []
        vb = V_B0 if buf == 0 else V_B1
        seq = [(r, p) for r in range(ROWS) for p in range(16)]
        n = len(seq)
        areg = [0]

        def issue(i):
            r, p = seq[i]
            cur = sb[r % 2]
            o = []
            for g, t in enumerate(row_slot(i % NSLOT)):
                idx = 3 * p + g
                a = A_BASE + areg[0] % 4
                areg[0] += 1
                o.append(f"v_add_u32_sdwa v{a}, s{cur + idx // 2}, v{vb} dst_sel:DWORD dst_unused:UNUSED_PAD "
                         f"src0_sel:WORD_{idx % 2} src1_sel:DWORD")
                o.append(f"ds_read_b64 v[{t[0]}:{t[1]}], v{a}")
            if p == 0:
                # this row's offsets are in use: fetch the next (column, row)'s into the other buffer
                o += sload(sb[(r + 1) % 2]) + advance((r + 1) % ROWS)
            return o

        def compute(i):
            r, p = seq[i]
            ta, tb, tc = row_slot(i % NSLOT)
            o = []
            for h in (0, 1):
                a_ = acc(r, p, h)
                o.append(f"v_bitop3_b32 v{a_}, v{a_}, v{ta[h]}, v{tb[h]} bitop3:0x96")
            for h in (0, 1):
                a_ = acc(r, p, h)
                o.append(f"v_xor_b32 v{a_}, v{tc[h]}, v{a_}")
            return o

        for i in range(min(DEPTH, n)):
            out += issue(i)
        for i in range(n):
            j = i + DEPTH
            if j < n:
                if j % 16 == 0 and "nodrain" not in flags:
                    out.append("s_waitcnt lgkmcnt(0)")  # row j // 16's offsets (and all reads)
                out += issue(j)
            ahead = min(j, n - 1) - i
            out.append(f"s_waitcnt lgkmcnt({3 * ahead})")
            out += compute(i)
        return out

    for par in (0, 1):
        L.append(f"Lr_it{par}_%=:")
        L += ["s_cmp_ge_u32 s%d, %%[k]" % S_CNT, "s_cbranch_scc1 Lr_done_%="]
        L += column(par)
        L += ["s_barrier", f"s_add_u32 s{S_CNT}, s{S_CNT}, 1"]
        if par == 1:
            L.append("s_branch Lr_it0_%=")
    L.append("Lr_done_%=:")
    # the prefetched offsets load past the last column may still be in flight
    L.append("s_waitcnt lgkmcnt(0)")
    L += mask_init()
    # epilogue: piece offsets (output layout) from LDS, inverse transposes, stores of the rows
    # below the limit; with accumulate the old bytes come from the accumulate-source layout
    # (encode: the parity slot itself; decode stage 1: the received parity row, output z)
    L += [f"s_mov_b64 s[{S_ODESC}:{S_ODESC + 1}], %[ob]", f"s_mov_b32 s{S_ODESC + 2}, 0x80000000",
          f"s_mov_b32 s{S_ODESC + 3}, 0x00020000",
          f"s_mov_b64 s[{S_ADESC}:{S_ADESC + 1}], %[ab]", f"s_mov_b32 s{S_ADESC + 2}, 0x80000000",
          f"s_mov_b32 s{S_ADESC + 3}, 0x00020000"]
    offv = list(range(T_BASE, T_BASE + 16))          # piece offsets v128..v143
    lo = T_BASE + 16                                 # lane*64 + OFF_LDS (from vb0 = lane*8 + base)
    L += [f"v_lshlrev_b32 v{lo}, 3, v{V_B0}", f"v_add_u32 v{lo}, %[loadj], v{lo}"]
    for i in range(4):
        L.append(f"ds_read_b128 v[{offv[4 * i]}:{offv[4 * i + 3]}], v{lo} offset:{16 * i}")
    L.append("s_waitcnt lgkmcnt(0)")
    ao = T_BASE + 17
    tmp = list(range(T_BASE + 18, T_BASE + 26))
    for r in range(ROWS):
        L += [f"s_add_u32 s{S_T0}, %[row0], {r}", "s_cmp_ge_u32 s%d, %%[rlim]" % S_T0, f"s_cbranch_scc1 Lr_skip{r}_%="]
        L += [f"s_add_u32 s{S_T1}, s{S_T0}, %[aslot]", f"s_mul_i32 s{S_CNT}, s{S_T1}, %[ass]",
              f"s_add_u32 s{S_T0}, s{S_T0}, %[oslot]", f"s_mul_i32 s{S_T1}, s{S_T0}, %[oss]"]
        for h in (0, 1):
            x = [acc(r, p, h) for p in range(16)]
            L += transpose16(x, tmp[:4])
            for i in range(8):
                piece = 8 * h + i
                d0, d1 = tmp[4], tmp[5]
                L += [f"v_mov_b32 v{d0}, v{x[2 * i]}", f"v_mov_b32 v{d1}, v{x[2 * i + 1]}"]
                L += ["s_cmp_eq_u32 %[acc], 0", f"s_cbranch_scc1 Lr_na{r}_{piece}_%="]
                L += [f"ds_read_b32 v{ao}, v{lo} offset:{OFF_ACC - OFF_LDS + 4 * piece}", "s_waitcnt lgkmcnt(0)",
                      f"buffer_load_dwordx2 v[{tmp[6]}:{tmp[7]}], v{ao}, s[{S_ADESC}:{S_ADESC + 3}], s{S_CNT} offen",
                      "s_waitcnt vmcnt(0)", f"v_xor_b32 v{d0}, v{d0}, v{tmp[6]}", f"v_xor_b32 v{d1}, v{d1}, v{tmp[7]}"]
                L.append(f"Lr_na{r}_{piece}_%=:")
                L.append(f"buffer_store_dwordx2 v[{d0}:{d1}], v{offv[piece]}, s[{S_ODESC}:{S_ODESC + 3}], s{S_T1} offen")
        L.append(f"Lr_skip{r}_%=:")
    return L


def row_clobbers():
    v = [f'"v{i}"' for i in range(V_B0)]
    s = [f'"s{i}"' for i in range(S_SB[0], S_LAST + 1)]
    return ", ".join(v + s + ['"scc"', '"memory"'])


def main():
    # --diag: build DIAG_BUILDER_VARIANTS with their NFEC_T3_VARIANT switch (the diagnostic
    # library, make -C norm_amd diag); the product library ships the default builder only
    global BUILDER_VARIANTS
    diag = "--diag" in sys.argv
    path = [a for a in sys.argv if a != "--diag"][1]
    if diag:
        BUILDER_VARIANTS = DIAG_BUILDER_VARIANTS
    bbs = {v: "\\n\"\n        \"".join(builder_asm(f) + (["s_mov_b32 %[oa], s96", "s_mov_b32 %[ob], s97",
                                                                 "s_mov_b32 %[oc], s98"] if "timed" in f else []))
           for v, f in BUILDER_VARIANTS.items()}
    rbs = {v: "\\n\"\n        \"".join(row_asm(f)) for v, f in BUILDER_VARIANTS.items()}
    ins = ", ".join(f'[o{i}] "v"(off[{i}])' for i in range(16))
    blocks = []
    for v in BUILDER_VARIANTS:
        kw = "if constexpr" if v == 0 else "else if constexpr"
        timed = "timed" in BUILDER_VARIANTS[v]
        outs = '[oa] "=s"(ta), [ob] "=s"(tb), [oc] "=s"(tc)' if timed else ""
        decl = "uint32_t ta, tb, tc;\n            " if timed else ""
        prt = ('\n            if (wg == 0 && lane == 0) printf("t3 builder k=%u m=%u: load wait %u, build+drain %u, '
               'barrier %u shader clocks\\n", a.k, a.m, ta, tb, tc);') if timed else ""
        blocks.append(f"""        {kw} (V == {v}) {{
            {decl}asm volatile(
            "{bbs[v]}\\n"
            : {outs}
            : [wb] "s"(wb), [ss] "s"(a.seg_stride), [k] "s"(a.k), [lb0] "v"(lb0), [lb1] "v"(lb1),
              [csh] "s"(a.col_shift), [cmk] "s"(a.col_mask), [cck] "s"(cck), [cbb] "s"(cbb), {ins}
            : {builder_clobbers(BUILDER_VARIANTS[v])});{prt}
        }}""")
    builder_blocks = "\n".join(blocks)
    rblocks = []
    for v in BUILDER_VARIANTS:
        kw = "if constexpr" if v == 0 else "else if constexpr"
        rblocks.append(f"""        {kw} (V == {v}) {{
            asm volatile(
            "{rbs[v]}\\n"
            :
            : [wb] "s"(wb), [op] "s"(op), [k] "s"(a.k), [rlim] "s"(rlim), [row0] "s"(row0),
              [cstep] "s"(cstep), [acc] "s"(a.accumulate), [loadj] "s"(loadj), [ob] "s"(ob), [ab] "s"(ab),
              [oslot] "s"(a.out_slot0), [oss] "s"(a.out_seg_stride), [aslot] "s"(a.acc_slot0),
              [ass] "s"(a.acc_seg_stride), [vb0] "{{v{V_B0}}}"(vb0), [vb1] "{{v{V_B1}}}"(vb1)
            : {row_clobbers()});
        }}""")
    row_blocks = "\n".join(rblocks)
    multi_cases = "\n".join(
        f"    case {v}: hipLaunchKernelGGL(gf16_t3_multi_kernel<{v}>, dim3((uint32_t)end), dim3({64 * NWAVES}), 0, s, mm); break;"
        for v in BUILDER_VARIANTS)
    enc_cases = "\n".join(
        f"    case {v}: hipLaunchKernelGGL(gf16_t3_encode_kernel<{v}>, dim3((uint32_t)wgs), dim3({64 * NWAVES}), 0, s, b); break;"
        for v in BUILDER_VARIANTS)
    if diag:
        t3_variant = f"""int t3_variant()
{{
    static const int v = [] {{
        const char* e = std::getenv("NFEC_T3_VARIANT");
        const int x = e ? std::atoi(e) : {T3_DEFAULT};
        return x >= 0 && x < {len(BUILDER_VARIANTS)} ? x : {T3_DEFAULT};
    }}();
    return v;
}}"""
    else:
        t3_variant = f"constexpr int t3_variant() {{ return {T3_DEFAULT}; }}"
    src = f"""// GENERATED by tools/codegen/gen_gf16_t3.py -- do not edit by hand.
// RS16 encode: bit-sliced, three shared four-Russians tables per source column in LDS.
#include <cstdlib>
#include "nfec_internal.hpp"
#include "bitslice.hpp"

namespace nfec {{
static_assert(kGf16T3RowsPerPass == {RP}u, "gen_gf16_t3.py and nfec_internal.hpp disagree on the rows per pass");
namespace {{

template <int V>
__device__ __forceinline__ void t3_body(const Gf16T3Args& a, uint32_t wg)
{{
    __shared__ uint32_t lds[{(OFF_ACC + 64 * 64) // 4}];
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t group = wg / a.passes, pass = wg - group * a.passes;
    // rows actually needed (decode stage 1: the largest erasure count among the blocks it
    // serves, written by the plan); passes past them leave at once, every wave together
    uint32_t rlim = a.m;
    if (a.rows_lim) rlim = min(rlim, __builtin_amdgcn_readfirstlane(*a.rows_lim));
    if (pass * {RP}u >= rlim) return;
    const uint64_t total = (uint64_t)a.nblocks * a.vec_bytes;   // flat bytes over blocks
    const uint64_t f0 = (uint64_t)group * 8192u;
    const uint32_t b0 = __builtin_amdgcn_readfirstlane((uint32_t)(min(f0, total - 1) / a.vec_bytes));
    const uint8_t* wb = a.base + (uint64_t)b0 * a.block_stride;
    const uint32_t lbase = bs::lds_addr(lds);
    if (wave == 0) {{
        uint32_t off[16];
        uint32_t* po = lds + {OFF_LDS // 4} + lane * 16;
        uint32_t* pa = lds + {OFF_ACC // 4} + lane * 16;
#pragma unroll
        for (int i = 0; i < 16; ++i) {{
            const uint64_t f = f0 + (uint64_t)i * 512u + lane * 8u;
            const uint32_t b = (uint32_t)(f / a.vec_bytes);
            const uint32_t p = (uint32_t)(f - (uint64_t)b * a.vec_bytes);
            const bool ok = f < total;
            off[i] = ok ? (uint32_t)((uint64_t)(b - b0) * a.block_stride) + p : 0x80000000u;
            po[i] = ok ? (uint32_t)((uint64_t)(b - b0) * a.out_block_stride) + p : 0x80000000u;
            pa[i] = ok ? (uint32_t)((uint64_t)(b - b0) * a.acc_block_stride) + p : 0x80000000u;
        }}
        const uint32_t lb0 = lbase + lane * 8u, lb1 = lb0 + {BUF}u;
        const uint32_t cck = a.col_chunk * a.seg_stride, cbb = a.col_base * a.seg_stride;
{builder_blocks}
    }} else {{
        const uint32_t row0 = pass * {RP}u + (wave - 1u) * {ROWS}u;
        // a row wave whose rows are all past the limit (the last pass of m = 100, decode stage 1
        // with e = 50) leaves before its first barrier: the builder and the other row waves
        // synchronise among the waves still running, and its SIMD's issue slots go to them
        if (row0 >= rlim) return;
        const uint8_t* op = reinterpret_cast<const uint8_t*>(a.offs) + (uint64_t)row0 * 96u;
        const uint32_t cstep = (a.m_pad - {ROWS - 1}u) * 96u;   // last row of a column -> first row of the next
        const uint32_t vb0 = lbase + lane * 8u, vb1 = vb0 + {BUF}u;
        const uint32_t loadj = lbase + {OFF_LDS}u - 8u * lbase;   // 8 * vb0 + loadj = piece offsets of the lane
        rlim = __builtin_amdgcn_readfirstlane(rlim);  // uniform: keep it in an SGPR for the asm
        const uint8_t* ob = a.out_base + (uint64_t)b0 * a.out_block_stride;
        const uint8_t* ab = a.acc_base + (uint64_t)b0 * a.acc_block_stride;
{row_blocks}
    }}
}}

template <int V>
__global__ __launch_bounds__({64 * NWAVES}, 1) void gf16_t3_encode_kernel(Gf16T3Args a)
{{
    t3_body<V>(a, bs::wg_index(1));
}}

// several independent products in one grid (the RS16 Toeplitz split, rs16_tmvp): workgroup
// ranges [wg_end[i-1], wg_end[i]) run problem i, so their tails share one launch
template <int V>
__global__ __launch_bounds__({64 * NWAVES}, 1) void gf16_t3_multi_kernel(Gf16T3Multi mm)
{{
    const uint32_t wg = bs::wg_index(1);
    if (wg < mm.wg_end[0]) t3_body<V>(mm.e[0], wg);
    else if (wg < mm.wg_end[1]) t3_body<V>(mm.e[1], wg - mm.wg_end[0]);
    else t3_body<V>(mm.e[2], wg - mm.wg_end[1]);
}}

{t3_variant}

// checks the shape, fills the default output / accumulate layouts and the pass count
int t3_prepare(const Gf16T3Args& a, Gf16T3Args& b, uint64_t& wgs)
{{
    if ((a.vec_bytes & 7u) || a.vec_bytes == 0 || !a.offs || a.num_data ||
        a.m_pad != (a.m + {RP - 1}u) / {RP}u * {RP}u)
        return NFEC_ENOTSUP;
    // every piece offset of a group (8 KiB of flat positions) plus slot offsets within 2^31
    const uint64_t nbg = 8192u / a.vec_bytes + 2u;
    const uint64_t in_slots = a.in_slots ? a.in_slots : (uint64_t)a.k + a.m;
    if (nbg * a.block_stride + in_slots * a.seg_stride >= (1ull << 31) ||
        (a.out_base && nbg * a.out_block_stride + (uint64_t)(a.out_slot0 + a.m) * a.out_seg_stride >= (1ull << 31)) ||
        (a.acc_base && nbg * a.acc_block_stride + (uint64_t)(a.acc_slot0 + a.m) * a.acc_seg_stride >= (1ull << 31)))
        return NFEC_ENOTSUP;
    const uint64_t total = (uint64_t)a.nblocks * a.vec_bytes;
    b = a;
    if (!b.out_base) {{  // encode: parity in place, slot k + r; accumulate against it
        b.out_base = const_cast<uint8_t*>(a.base);
        b.out_block_stride = a.block_stride;
        b.out_seg_stride = a.seg_stride;
        b.out_slot0 = a.k;
    }}
    if (!b.acc_base) {{
        b.acc_base = b.out_base;
        b.acc_block_stride = b.out_block_stride;
        b.acc_seg_stride = b.out_seg_stride;
        b.acc_slot0 = b.out_slot0;
    }}
    b.passes = (a.m + {RP - 1}u) / {RP}u;
    const uint64_t groups = (total + 8191u) / 8192u;
    wgs = groups * b.passes;
    return wgs >= (1ull << 31) ? NFEC_ENOTSUP : NFEC_OK;
}}

}}  // namespace

// whether launch_gf16_t3_encode takes this shape and layout (decode asks before its plan marks
// blocks for stage 1 by the encode kernel, so an uncovered layout keeps the gather stage)
bool gf16_t3_covers(const Gf16T3Args& a)
{{
    Gf16T3Args b;
    uint64_t wgs = 0;
    return t3_prepare(a, b, wgs) == NFEC_OK;
}}

int launch_gf16_t3_multi(const Gf16T3Args* e, uint32_t n, hipStream_t s)
{{
    if (n == 0 || n > 3) return NFEC_EINVAL;
    Gf16T3Multi mm;
    uint64_t end = 0;
    for (uint32_t i = 0; i < 3; ++i) {{
        uint64_t w = 0;
        if (i < n && e[i].nblocks) {{
            const int rc = t3_prepare(e[i], mm.e[i], w);
            if (rc) return rc;
        }}
        end += w;
        if (end >= (1ull << 31)) return NFEC_ENOTSUP;
        mm.wg_end[i] = (uint32_t)end;
    }}
    if (end == 0) return NFEC_OK;
    switch (t3_variant()) {{
{multi_cases}
    }}
    const hipError_t err = hipGetLastError();
    return err == hipSuccess ? NFEC_OK : hip_fail(err, "gf16 t3 multi launch");
}}

int launch_gf16_t3_encode(const Gf16T3Args& a, hipStream_t s)
{{
    if (a.nblocks == 0) return NFEC_OK;
    Gf16T3Args b;
    uint64_t wgs = 0;
    const int rc = t3_prepare(a, b, wgs);
    if (rc) return rc;
    switch (t3_variant()) {{
{enc_cases}
    }}
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? NFEC_OK : hip_fail(e, "gf16 t3 encode launch");
}}

}}  // namespace nfec
"""
    open(path, "w").write(src)


if __name__ == "__main__":
    main()
