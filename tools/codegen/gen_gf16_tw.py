#!/usr/bin/env python3
"""Generate norm_amd/csrc/gen_gf16_tw.hip: RS16 (GF(2^16)) parity products through the tower
field GF((2^8)^2), multiplications as jumps into a 256-entry GF(2^8) snippet table.

The reference multiplies symbol by symbol through log/exp tables (NormEncoderRS16::Encode,
src/common/normEncoderRS16.cpp:472-482, addmul1 :261-298).  Any GF(2)-linear isomorphism phi
from the reference's field (x^16 + x^12 + x^3 + x + 1, src/common/galois.h) onto the tower
GF(2^8)[y] / (y^2 + y + lam) keeps products: phi(g * x) = phi(g) (x) phi(x).  With
phi(g) = c0 + c1 y and phi(x) = x0 + x1 y (x0, x1 in the RS8 field 0x11d):

    (g * x)_0 = c0 x0 + (lam c1) x1          (g * x)_1 = c1 x0 + (c0 + c1) x1

four GF(2^8) products by constants.  Bit-sliced (plane b = bit b of 32 symbols), a product
by a GF(2^8) constant is one v_bitop3 per output plane over the four-Russians combinations of
the source's planes 0..3 and 4..7 -- the same 8-instruction snippets the RS8 solve jumps into
(gen_solve_asm.py), 256 of them in 32 KiB of code.  No LDS tables, no per-symbol lookups.

One wave owns one (item group, pass): 64 lanes x 32 symbols (lane L holds 8 pieces of 8 bytes,
piece i at flat position f0 + 512 i + 8 L, so each load is a 512-byte run) and 11 parity rows
(16 accumulator planes each, 176 VGPRs).  Per source column:
  * 8 x buffer_load_dwordx2 (issued one column ahead), a 16 x 16 bit transpose, the XOR
    network of phi into x0 (8 planes) and x1 (8 planes);
  * combinations of x0; per row a jump into snippet[c0] (target out0) and snippet[c1]
    (target out1); then x1's combinations and jumps into snippet[lam c1] and
    snippet[c0 ^ c1].  The targets are M0-relative (gpr-index mode on SRC0 and DST), the
    snippet byte offsets (four 16-bit values per row) come from the coefficient table by scalar
    loads.
After the last column each row goes back through phi^-1 and the transpose and is stored (XORed
with the accumulate source when asked).  Workgroup = 4 independent waves (consecutive jobs:
passes of one item group share their column reads through L2).

Usage: gen_gf16_tw.py OUT.hip [--diag] [--rows N] [--noprefetch] [--waves N]

The library holds the kernel in the configurations of CONFIGS (rows per wave), and each launch
takes the one with the lowest PASS_COST x passes for its rows.  6 rows hold 96 accumulator VGPRs
(164 in all: 3 waves per SIMD, which hide the snippet calls' branch redirects: RS16(400,100)
encode 27.1 -> 22.9 ms, C4 133.4 -> 125.8 ms against 11 rows, profiles/r05/tw_rows_ab); 4 rows
hold 64 (125 in all: 4 waves per SIMD, more column work per row: C4's 64-row products 0.946x the
6-row time, RS16(400,100)'s 100 rows 1.044x, profiles/r05/tw_rows4_ab).  --rows N builds one
configuration of N rows (A/B builds, tools/ab_build.sh; 11 rows: the round-3/4 kernel at 2 waves
per SIMD).  --noprefetch reads each sweep's planes into W after the previous sweep instead of
into S during it (8 VGPRs fewer, 16 moves per column fewer; measured neutral at 6 rows).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gen_rs8_bitsliced import bitmatrix_rows  # noqa: E402
from gen_rs8_bitsliced import mul as gf8_mul  # noqa: E402  (the RS8 field, 0x11d)

P16 = 0x1100B            # the reference's GF(2^16) polynomial
ROWS = 6                 # parity rows per wave (pass); set_rows() below fixes what follows from it
NWAVES = 4               # waves per workgroup (passes of one item group sharing its columns; --waves)
GROUP_BYTES = 4096       # flat bytes per item group: 64 lanes x 8 pieces x 8 bytes
SNIP_ALIGN = 7           # 128-byte snippet slots
TBL_HALF = 48            # 16-bit table entries per (column, pass): 11 rows x 4 + 4 padding
GPR_MODE = 0x9000        # M0[15:12]: index SRC0 and DST

# ---- VGPRs ----
# v0..v3: the asm's three inputs (lo, xl, lq; placed by the compiler below the first clobber)
PREFETCH = True          # x1 / next x0 planes read into S while a sweep runs (--noprefetch: into W after it)
# The library holds one kernel per configuration (rows per wave, prefetch) and each launch takes
# the one with the lowest PASS_COST x passes: 7 rows without the prefetch and 6 rows with it fit
# 3 waves per SIMD (166 / 158 VGPRs), 4 rows 4 (125).  Relative pass costs measured on one box
# (profiles/r05/tw_rows4_ab/, tw_r7/): a 4-row pass ~0.73 of a 6-row one (C4's 64-row products
# 16 passes vs 12, 0.946x the time; RS16(400, 100) 28 vs 20, 1.044x), a 7-row pass ~1.2 (RS16
# encode m = 100: 16 passes vs 20, 0.957x; m = 50: 8 vs 16 4-row passes, 0.85x).
CONFIGS = [(7, False), (6, True), (4, True)]
PASS_COST = {7: 120, 6: 100, 4: 73}


def layout():
    """register map for ROWS and PREFETCH (set_rows / set_prefetch call it)"""
    global V_SLOT, V_W, V_S, V_X1, V_CA, V_CB, V_TMP, ACC0, V_LAST
    V_SLOT = 4           # 16: raw column (loads) -> transposed planes; epilogue: output planes
    V_W = 20             # 8: current source planes (x0, then x1); epilogue: store offsets
    V_S = 28 if PREFETCH else None   # 8: x1 while x0 is applied (prefetch only)
    V_CA = 36 if PREFETCH else 28    # 11: combinations of planes 0..3 of the source
    V_CB = V_CA + 11     # 11: combinations of planes 4..7
    V_X1 = V_S if PREFETCH else V_CA  # phi's x1 planes before the exchange write
    V_TMP = [V_CB + 11 + i for i in range(4)]
    ACC0 = V_CB + 15     # row r: out0 planes ACC0 + 16 r + (0..7), out1 + 8
    V_LAST = ACC0 + 16 * ROWS - 1


layout()
# (register pairs of loads, stores and LDS reads start at even registers: V_SLOT, V_W, V_S,
# V_CA and V_CB + 1 are even)
MULTI = [a for a in range(1, 16) if bin(a).count("1") >= 2]

# ---- SGPRs (clobbered) ----
S_DESC, S_ODESC, S_ADESC = 36, 40, 44
S_MASK = 48              # 8: transpose masks (mask, mask << s) for s = 8, 4, 2, 1
S_SNIP, S_TGT, S_RET = 56, 58, 60
S_C, S_COL, S_T0, S_T1, S_T2 = 64, 65, 66, 67, 68
S_OFF = 72               # 24: the column's table entries (sweep 0: 72..83, sweep 1: 84..95)
S_LAST = 95
MASKS = {8: 0x00FF00FF, 4: 0x0F0F0F0F, 2: 0x33333333, 1: 0x55555555}

def set_prefetch(on):
    global PREFETCH
    PREFETCH = on
    layout()


def set_waves(n):
    """waves per workgroup and what follows from it"""
    global NWAVES, XCH_BUF
    NWAVES = n
    XCH_BUF = NWAVES * 8 * 64 * 8


def set_rows(n):
    """parity rows per wave and what follows from it"""
    global ROWS, SPECIAL_ROWS
    ROWS = n
    layout()
    # pass row counts with their own (unchecked) step loop
    SPECIAL_ROWS = tuple(range(ROWS, max(ROWS - 6, 0), -1))


# timing probes (wrong parity on purpose), diagnostic library only (--diag, NFEC_TW_VARIANT=<id>):
#   "nosweep"  no jumps: loads, transpose, phi and combinations only
#   "noload"   no column loads (the slot keeps stale data)
#   "empty"    every jump goes to the empty snippet: the call overhead without its VALU
VARIANTS = {0: ()}
DIAG_VARIANTS = {0: (), 1: ("nosweep",), 2: ("noload",), 3: ("empty",)}
FLAGS = ()
NT_STORES = False        # --nt-stores: the rows' stores non-temporal (A/B builds)


# ---------------------------------------------------------------- field
def gf16_mul(a, b):
    r = 0
    while b:
        if b & 1:
            r ^= a
        b >>= 1
        a <<= 1
        if a & 0x10000:
            a ^= P16
    return r


def gf8_trace(v):
    t, x = 0, v
    for _ in range(8):
        t ^= x
        x = gf8_mul(x, x)
    return t


def tw_mul(a, b, lam):
    """tower product: a = a0 + a1 y (a0 low byte), y^2 = y + lam"""
    a0, a1, b0, b1 = a & 255, a >> 8, b & 255, b >> 8
    p1 = gf8_mul(a1, b1)
    lo = gf8_mul(a0, b0) ^ gf8_mul(lam, p1)
    hi = gf8_mul(a1, b0) ^ gf8_mul(a0, b1) ^ p1
    return lo | (hi << 8)


def _vec_tables():
    import numpy as np
    exp = np.zeros(512, dtype=np.int64)
    log = np.zeros(256, dtype=np.int64)
    v = 1
    for i in range(255):
        exp[i] = v
        log[v] = i
        v <<= 1
        if v & 0x100:
            v ^= 0x11D
    exp[255:510] = exp[0:255]
    return exp, log


def _roots(lam):
    """the 16 roots of P16 in the tower field of lam (vectorised over all elements)"""
    import numpy as np
    exp, log = _vec_tables()

    def m8(a, b):
        r = exp[(log[a] + log[b]) % 255]
        return np.where((a == 0) | (b == 0), 0, r)

    x = np.arange(1 << 16, dtype=np.int64)
    x0, x1 = x & 255, x >> 8
    acc = np.zeros_like(x)
    p = np.ones_like(x)            # x^i, starting at 1
    lam_a = np.full_like(x, lam)
    for i in range(17):
        if (P16 >> i) & 1:
            acc ^= p
        p0, p1 = p & 255, p >> 8
        q1 = m8(p1, x1)
        lo = m8(p0, x0) ^ m8(lam_a, q1)
        hi = m8(p1, x0) ^ m8(p0, x1) ^ q1
        p = lo | (hi << 8)
    return [int(v) for v in np.nonzero(acc == 0)[0] if v]


def gf2_inverse(cols):
    """inverse of a 16 x 16 GF(2) matrix given by its columns (ints), as columns"""
    n = 16
    rows = [sum(((cols[j] >> i) & 1) << j for j in range(n)) for i in range(n)]
    aug = [(rows[i], 1 << i) for i in range(n)]
    for c in range(n):
        piv = next(r for r in range(c, n) if (aug[r][0] >> c) & 1)
        aug[c], aug[piv] = aug[piv], aug[c]
        for r in range(n):
            if r != c and (aug[r][0] >> c) & 1:
                aug[r] = (aug[r][0] ^ aug[c][0], aug[r][1] ^ aug[c][1])
    inv_rows = [aug[i][1] for i in range(n)]
    return [sum(((inv_rows[i] >> j) & 1) << i for i in range(n)) for j in range(n)]


def row_masks(cols):
    """output bit j of M x = parity(row_j & x)"""
    return [sum(((cols[i] >> j) & 1) << i for i in range(16)) for j in range(16)]


def xor_cost(masks):
    c = 0
    for w in (bin(r).count("1") for r in masks):
        c += 1 if w <= 1 else (w // 2)   # mov / ceil((w - 1) / 2) three-input XORs
    return c


def choose_tower():
    """the isomorphism (lam, beta) whose phi network is cheapest: phi(x^i) = beta^i"""
    best = None
    lams = [v for v in range(1, 256) if gf8_trace(v) == 1]
    for lam in lams:
        for beta in _roots(lam):
            cols, inv = tower_basis(lam, beta)
            key = (xor_cost(row_masks(cols)), xor_cost(row_masks(inv)), lam, beta)
            if best is None or key < best[0]:
                best = (key, lam, beta, cols, inv)
    return best[1], best[2], best[3], best[4]


def tower_basis(lam, beta):
    """phi's columns (phi(x^i) = beta^i) and those of its inverse"""
    cols, p = [], 1
    for _ in range(16):
        cols.append(p)
        p = tw_mul(p, beta, lam)
    return cols, gf2_inverse(cols)


# choose_tower()'s pick (about 15 s of search; `gen_gf16_tw.py --search` reruns it):
# 49 / 53 three-input XORs for phi / phi^-1
LAM, BETA = 0x6B, 0xCF34
PHI, PHI_INV = tower_basis(LAM, BETA)


def phi(v, cols=None):
    cols = cols or PHI
    r = 0
    for i in range(16):
        if (v >> i) & 1:
            r ^= cols[i]
    return r


# ---------------------------------------------------------------- instruction lists
def mask_init():
    out = []
    for s, mi in ((8, 0), (4, 2), (2, 4), (1, 6)):
        out.append(f"s_mov_b32 s{S_MASK + mi}, 0x{MASKS[s]:08x}")
        out.append(f"s_mov_b32 s{S_MASK + mi + 1}, 0x{(MASKS[s] << s) & 0xFFFFFFFF:08x}")
    return out


def transpose16(x, temps):
    """16 x 16 bit transpose of x[0..15] (both 16-bit halves at once), in place: afterwards
    x[q] holds bit q of the 32 symbols (an involution: the epilogue applies it again)"""
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


def xor_network(masks, src, dst):
    """dst[j] = XOR of src[i] over the set bits i of masks[j] (three-input XOR chains)"""
    out = []
    for j, mk in enumerate(masks):
        ins = [src[i] for i in range(16) if (mk >> i) & 1]
        d = dst[j]
        if not ins:
            out.append(f"v_mov_b32 v{d}, 0")
            continue
        if len(ins) == 1:
            out.append(f"v_mov_b32 v{d}, v{ins[0]}")
            continue
        if len(ins) == 2:
            out.append(f"v_xor_b32 v{d}, v{ins[0]}, v{ins[1]}")
            ins = []
        else:
            out.append(f"v_bitop3_b32 v{d}, v{ins[0]}, v{ins[1]}, v{ins[2]} bitop3:0x96")
            ins = ins[3:]
        while ins:
            if len(ins) == 1:
                out.append(f"v_xor_b32 v{d}, v{d}, v{ins[0]}")
                ins = []
            else:
                out.append(f"v_bitop3_b32 v{d}, v{d}, v{ins[0]}, v{ins[1]} bitop3:0x96")
                ins = ins[2:]
    return out


def slot():
    return [V_SLOT + i for i in range(16)]


def w_regs():
    return [V_W + i for i in range(8)]


def x1_regs():
    return [V_X1 + i for i in range(8)]


def phi_code():
    """transposed planes (slot) -> x0 planes (W) and x1 planes (S, or CA without the prefetch)"""
    return xor_network(row_masks(PHI), slot(), w_regs() + x1_regs())


def phi_inv_code(r):
    """row r's accumulators (tower planes) -> polynomial-basis planes in the slot"""
    src = [ACC0 + 16 * r + i for i in range(16)]
    return xor_network(row_masks(PHI_INV), src, slot())


def operand_maps():
    """A[a] / B[b]: register of the XOR of source planes {0..3} / {4..7} selected by a / b"""
    w = w_regs()
    A = {1 << t: w[t] for t in range(4)}
    B = {1 << t: w[4 + t] for t in range(4)}
    for n, a in enumerate(MULTI):
        A[a] = V_CA + n
        B[a] = V_CB + n
    return A, B


def combos_code():
    A, B = operand_maps()
    out = []
    for M in (A, B):
        for a in sorted(MULTI, key=lambda a: bin(a).count("1")):
            top = a.bit_length() - 1
            out.append(f"v_xor_b32 v{M[a]}, v{M[a & ~(1 << top)]}, v{M[1 << top]}")
    return out


def snippet_body(c):
    """acc plane i (register ACC0 + i + M0 index) ^= plane i of c * source (c in GF(2^8))"""
    A, B = operand_maps()
    out = []
    rows = bitmatrix_rows(c) if c else [0] * 8
    for i in range(8):
        a, b = rows[i] & 15, rows[i] >> 4
        d = ACC0 + i
        if a and b:
            out.append(f"v_bitop3_b32 v{d}, v{d}, v{A[a]}, v{B[b]} bitop3:0x96")
        elif a:
            out.append(f"v_xor_b32 v{d}, v{d}, v{A[a]}")
        elif b:
            out.append(f"v_xor_b32 v{d}, v{d}, v{B[b]}")
    return out


def snippets():
    # 64 KiB-aligned table start: a snippet address is then the table address's high half
    # packed with the 16-bit entry (s_pack_*_b32_b16), with no add (the specialised loops)
    out = [".p2align 16"]
    for c in range(256):
        out.append(f".p2align {SNIP_ALIGN}")
        if c == 0:
            out.append("Lsnip0_%=:")
        out += snippet_body(c)
        out.append(f"s_setpc_b64 s[{S_RET}:{S_RET + 1}]")
    return out


def table_entries(g):
    """the four snippet byte offsets of coefficient g: sweep 1 (source x0) out0 / out1, sweep 2
    (source x1) out0 / out1"""
    t = phi(g)
    c0, c1 = t & 255, t >> 8
    return [v << SNIP_ALIGN for v in (c0, c1, gf8_mul(LAM, c1), c0 ^ c1)]


# ---------------------------------------------------------------- kernel body
def entry(n, r, j):
    """(dword, half) of the table entry of pass row r, sweep n (source x_n), output j: the
    entries of sweep 0 fill dwords 0..10 and those of sweep 1 dwords 12..22, so one sweep's
    entries load while the other sweep runs"""
    return S_OFF + 12 * n + r, j


def call(n, r, j, generic=True):
    """jump into the snippet of entry (n, r, j), target accumulators 16 r + 8 j.  generic=False
    (the specialised loops, taken when the table sits at a 64 KiB boundary): the target's high
    word is set once (s[S_TGT + 1] = s[S_SNIP + 1]) and its low word is the table address's
    high half packed with the entry; generic: extract the entry, add with carry"""
    dw, half = entry(n, r, j)
    if "empty" in FLAGS:
        L = [f"s_mov_b32 s{S_T1}, 0", f"s_add_u32 s{S_TGT}, s{S_SNIP}, s{S_T1}"]
        if generic:
            L.append(f"s_addc_u32 s{S_TGT + 1}, s{S_SNIP + 1}, 0")
    elif generic:
        L = [f"s_bfe_u32 s{S_T1}, s{dw}, 0x{(16 << 16) | (16 * half):x}",
             f"s_add_u32 s{S_TGT}, s{S_SNIP}, s{S_T1}",
             f"s_addc_u32 s{S_TGT + 1}, s{S_SNIP + 1}, 0"]
    else:
        op = "s_pack_lh_b32_b16" if half == 0 else "s_pack_hh_b32_b16"
        L = [f"{op} s{S_TGT}, s{dw}, s{S_SNIP}"]
    # s_movk_i32: a 4-byte SOPK instead of an 8-byte s_mov with a literal (M0's upper half takes
    # copies of bit 15, which gpr-index mode ignores); the calls measured 5.7 % faster at three
    # waves per SIMD (profiles/r05/callchain/)
    return L + [f"s_movk_i32 m0, 0x{GPR_MODE | (16 * r + 8 * j):x}",
                f"s_swappc_b64 s[{S_RET}:{S_RET + 1}], s[{S_TGT}:{S_TGT + 1}]"]


def sweep(n, x, nrows):
    """the pass rows' jumps for source x_n; nrows: a fixed row count (no bound checks), or None
    (rows checked against %[nr])"""
    if "nosweep" in FLAGS:
        return []
    L = [f"s_mov_b32 s{S_T0}, 0", f"s_set_gpr_idx_on s{S_T0}, gpr_idx(SRC0,DST)"]
    for r in range(nrows or ROWS):
        if r and nrows is None:
            L += [f"s_cmp_le_u32 %[nr], {r}", f"s_cbranch_scc1 Lsw{n}{x}_%="]
        L += call(n, r, 0, nrows is None)
        L += call(n, r, 1, nrows is None)
    L += [f"Lsw{n}{x}_%=:", "s_set_gpr_idx_off", "s_nop 1"]
    return L


# ---------------------------------------------------------------- kernel body
# The four waves of a workgroup run four passes of the same item group (64 lanes x 32 symbols).
# In step s wave w loads, transposes and maps (phi) column 4 s + w only and writes its 16 tower
# planes to an LDS exchange slot; after one s_barrier every wave applies columns 4 s .. 4 s + 3
# to its rows, reading their planes back from LDS.  The per-column transpose and phi network
# (~180 VALU) run once per workgroup, and each column is read from memory once per workgroup.
# The LDS planes and the scalar table entries of the next half-column are fetched while the
# current sweep runs (into S and the other half of the entry registers), so no sweep waits on
# them.  Exchange: 2 buffers x 4 columns x 8 plane pairs x 64 lanes x 8 bytes = 32 KiB (pair p
# of a lane at ((buf * 4 + col) * 8 + p) * 512 + lane * 8).
S_SB, S_BUF, S_WV = 69, 70, 71   # step's first column; exchange buffer byte offset; wave index
S_TB = 96                        # 2: table base (this pass's entries of column 0)
S_TBN = 98                       # 2: table address of the column being fetched
S_LAST4 = 99
XCH_BUF = NWAVES * 8 * 64 * 8    # bytes per exchange buffer (NWAVES columns; set_waves)
SPECIAL_ROWS = (6, 5, 4, 3, 2, 1)   # pass row counts with their own (unchecked) step loop (set_rows)


def col_offset():
    """column index s[S_C] -> byte offset s[S_COL] through the column map: q = c / d by the
    multiply-high with cmg = ceil(2^32 / d) (exact for c, d < 2^16), then
    q * cck + (c - q d) * crs + cbb.  Identity: cmg 0 (q = 0), crs = ss, cck = cbb = 0; d = 1:
    cmg 0 with crs = the chunk stride (set up by the wrapper, chunk_map)"""
    return [f"s_mul_hi_u32 s{S_T2}, s{S_C}, %[cmg]", f"s_mul_i32 s{S_COL}, s{S_T2}, %[cdv]",
            f"s_sub_u32 s{S_COL}, s{S_C}, s{S_COL}", f"s_mul_i32 s{S_COL}, s{S_COL}, %[crs]",
            f"s_mul_i32 s{S_T2}, s{S_T2}, %[cck]", f"s_add_u32 s{S_COL}, s{S_COL}, s{S_T2}",
            f"s_add_u32 s{S_COL}, s{S_COL}, %[cbb]"]


_uid = [0]


def loads():
    """column s[S_C]'s 8 pieces -> the slot.  The pieces' byte offsets come from LDS (%[lo] + 80,
    shared by the workgroup's waves).  Flat shortened mode (bit 0 of %[md]): a piece whose block
    has numData <= the column's source slot reads zeros (its offset gets bit 31: past
    num_records; q = the piece's numData - 1, u16 pairs at %[lq]), so each piece's block stops at
    its own numData.  The slot is the column map's (s[S_COL] = slot * seg_stride, so the sign of
    q * seg_stride - s[S_COL] decides): the Toeplitz split's products that read source columns
    through the map (chunks, halves) mask the source slot, not their own column index"""
    x = slot()
    if "noload" in FLAGS:
        return []
    _uid[0] += 1
    u = _uid[0]
    o = [V_CA + i for i in range(8)]       # (free: the combinations are rebuilt per column)
    q = [V_CB + 1 + i for i in range(4)]
    t = V_CB + 5
    L = [f"ds_read_b128 v[{o[0]}:{o[3]}], %[lo] offset:80", f"ds_read_b128 v[{o[4]}:{o[7]}], %[lo] offset:96"]
    plain = ["s_waitcnt lgkmcnt(0)"]
    plain += [f"buffer_load_dwordx2 v[{x[2 * i]}:{x[2 * i + 1]}], v{o[i]}, s[{S_DESC}:{S_DESC + 3}], s{S_COL} offen"
              for i in range(8)]
    masked = [f"ds_read_b64 v[{q[0]}:{q[1]}], %[lq]", f"ds_read_b64 v[{q[2]}:{q[3]}], %[lq] offset:8",
              "s_waitcnt lgkmcnt(0)"]
    for i in range(8):
        src = q[i // 2]
        masked += [f"v_lshrrev_b32 v{t}, 16, v{src}" if i & 1 else f"v_and_b32 v{t}, 0xffff, v{src}",
                   f"v_mul_u32_u24 v{t}, %[ss], v{t}",
                   f"v_subrev_u32 v{t}, s{S_COL}, v{t}",                        # (numData - 1 - slot) ss
                   f"v_and_or_b32 v{o[i]}, v{t}, s{S_DESC + 2}, v{o[i]}",       # sign -> bit 31
                   f"buffer_load_dwordx2 v[{x[2 * i]}:{x[2 * i + 1]}], v{o[i]}, s[{S_DESC}:{S_DESC + 3}], s{S_COL} offen"]
    return (L + [f"s_bitcmp1_b32 %[md], 0", f"s_cbranch_scc0 Lldp{u}_%="] + masked +
            [f"s_branch Lldx{u}_%=", f"Lldp{u}_%=:"] + plain + [f"Lldx{u}_%=:"])


def xch_addr(j=None, sgpr=None):
    """v_tmp0 = the lane's exchange address in the current buffer: of column slot j (a
    constant, returned as the ds offset base) or of the slot held in SGPR s[sgpr]"""
    if sgpr is None:
        return [f"v_add_u32 v{V_TMP[0]}, s{S_BUF}, %[xl]"], 4096 * j
    return [f"s_lshl_b32 s{S_T0}, s{sgpr}, 12", f"s_add_u32 s{S_T0}, s{S_T0}, s{S_BUF}",
            f"v_add_u32 v{V_TMP[0]}, s{S_T0}, %[xl]"], 0


def fetch_planes(j, n, dst):
    """planes of source x_n of column slot j -> dst (LDS)"""
    code, base = xch_addr(j)
    return code + [f"ds_read_b64 v[{dst + 2 * p}:{dst + 2 * p + 1}], v{V_TMP[0]} offset:{base + 512 * (4 * n + p)}"
                   for p in range(4)]


def fetch_entries(j, n):
    """table entries of sweep n of column slot j -> their half of the entry registers"""
    L = []
    if n == 0:  # a new column: its table address
        L += [f"s_add_u32 s{S_T2}, s{S_SB}, {j}", f"s_mul_i32 s{S_T2}, s{S_T2}, %[tstep]",
              f"s_add_u32 s{S_TBN}, s{S_TB}, s{S_T2}", f"s_addc_u32 s{S_TBN + 1}, s{S_TB + 1}, 0"]
    o = S_OFF + 12 * n
    if n == 1:  # the column's sweep-1 entries follow its m sweep-0 rows
        L += [f"s_add_u32 s{S_TBN}, s{S_TBN}, %[t1off]", f"s_addc_u32 s{S_TBN + 1}, s{S_TBN + 1}, 0"]
    L += [f"s_load_dwordx8 s[{o}:{o + 7}], s[{S_TBN}:{S_TBN + 1}], 0x0",
          f"s_load_dwordx4 s[{o + 8}:{o + 11}], s[{S_TBN}:{S_TBN + 1}], 0x20"]
    return L


def fetch(j, n):
    """prefetch form: planes of x_n of column slot j -> S, table entries of sweep n -> their half"""
    if n == 0:
        return fetch_entries(j, 0)[:4] + fetch_planes(j, 0, V_S) + fetch_entries(j, 0)[4:]
    return fetch_planes(j, 1, V_S) + fetch_entries(j, 1)


def apply_col(j, x, nrows):
    """apply column slot j of the step (prefetch: entering with x0's planes in S and the sweep-0
    entries in flight; else with the entries in flight only)"""
    y = f"{x}{j}"
    L = []
    if j:
        L += [f"s_add_u32 s{S_T2}, s{S_SB}, {j}", f"s_cmp_lt_u32 s{S_T2}, %[k]", f"s_cbranch_scc0 Lend{x}_%="]
    if not PREFETCH:
        # each sweep's planes go straight into W once the previous sweep is done (the LDS latency
        # is exposed to this wave; the SIMD's other waves run meanwhile)
        L += fetch_planes(j, 0, V_W)
        L.append("s_waitcnt lgkmcnt(0)")
        L += fetch_entries(j, 1)
        L += combos_code()
        L += sweep(0, y, nrows)
        L += fetch_planes(j, 1, V_W)
        L.append("s_waitcnt lgkmcnt(0)")
        if j < NWAVES - 1:
            L += [f"s_add_u32 s{S_T2}, s{S_SB}, {j + 1}", f"s_cmp_lt_u32 s{S_T2}, %[k]", f"s_cbranch_scc0 Lnf{y}_%="]
            L += fetch_entries(j + 1, 0)
            L.append(f"Lnf{y}_%=:")
        L += combos_code()
        L += sweep(1, y, nrows)
        return L
    L.append("s_waitcnt lgkmcnt(0)")
    L += [f"v_mov_b32 v{V_W + i}, v{V_S + i}" for i in range(8)]
    L += fetch(j, 1)
    L += combos_code()
    L += sweep(0, y, nrows)
    L.append("s_waitcnt lgkmcnt(0)")
    L += [f"v_mov_b32 v{V_W + i}, v{V_S + i}" for i in range(8)]
    if j < NWAVES - 1:
        L += [f"s_add_u32 s{S_T2}, s{S_SB}, {j + 1}", f"s_cmp_lt_u32 s{S_T2}, %[k]", f"s_cbranch_scc0 Lnf{y}_%="]
        L += fetch(j + 1, 0)
        L.append(f"Lnf{y}_%=:")
    L += combos_code()
    L += sweep(1, y, nrows)
    return L


def step_loop(x, nrows):
    """nrows: the pass's row count for a specialised loop, None: checked rows (helper waves with
    no rows skip the applies)"""
    L = [f"Lstep{x}_%=:", "s_waitcnt vmcnt(0)",
         f"s_cmp_lt_u32 s{S_C}, %[k]", f"s_cbranch_scc0 Lnotr{x}_%="]
    L += transpose16(slot(), V_TMP)
    L += phi_code()
    code, _ = xch_addr(sgpr=S_WV)
    L += code
    for p in range(4):
        L.append(f"ds_write_b64 v{V_TMP[0]}, v[{V_W + 2 * p}:{V_W + 2 * p + 1}] offset:{512 * p}")
    for p in range(4):
        L.append(f"ds_write_b64 v{V_TMP[0]}, v[{V_X1 + 2 * p}:{V_X1 + 2 * p + 1}] offset:{512 * (4 + p)}")
    L.append(f"Lnotr{x}_%=:")
    # the wave's column of the next step goes into the (now free) slot
    L += [f"s_add_u32 s{S_C}, s{S_C}, {NWAVES}", f"s_cmp_lt_u32 s{S_C}, %[k]", f"s_cbranch_scc0 Lnl{x}_%="]
    L += col_offset() + loads()
    L += [f"Lnl{x}_%=:", "s_waitcnt lgkmcnt(0)", "s_barrier"]
    if nrows is None:
        L += ["s_cmp_eq_u32 %[nr], 0", f"s_cbranch_scc1 Lend{x}_%="]
    L += fetch(0, 0) if PREFETCH else fetch_entries(0, 0)
    for j in range(NWAVES):
        L += apply_col(j, x, nrows)
    L += [f"Lend{x}_%=:", f"s_xor_b32 s{S_BUF}, s{S_BUF}, {XCH_BUF}", f"s_add_u32 s{S_SB}, s{S_SB}, {NWAVES}",
          f"s_cmp_lt_u32 s{S_SB}, %[k]", f"s_cbranch_scc1 Lstep{x}_%="]
    return L


def body():
    L = [f"s_mov_b64 s[{S_DESC}:{S_DESC + 1}], %[wb]", f"s_mov_b32 s{S_DESC + 2}, 0x80000000",
         f"s_mov_b32 s{S_DESC + 3}, 0x00020000"]
    L += mask_init()
    L += [f"s_getpc_b64 s[{S_SNIP}:{S_SNIP + 1}]",
          "Lpc_%=:",
          f"s_add_u32 s{S_SNIP}, s{S_SNIP}, Lsnip0_%=-Lpc_%=",
          f"s_addc_u32 s{S_SNIP + 1}, s{S_SNIP + 1}, 0",
          f"s_mov_b64 s[{S_TB}:{S_TB + 1}], %[tw]",
          f"s_mov_b32 s{S_WV}, %[wv]", f"s_mov_b32 s{S_C}, %[wv]",
          f"s_mov_b32 s{S_SB}, 0", f"s_mov_b32 s{S_BUF}, 0"]
    for v in range(ACC0, V_LAST + 1):
        L.append(f"v_mov_b32 v{v}, 0")
    L += [f"s_cmp_lt_u32 s{S_C}, %[k]", "s_cbranch_scc0 Lnl0_%="]
    L += col_offset() + loads()
    # the specialised loops pack a snippet address from the table address's high half and the
    # entry: taken when the table starts at a 64 KiB boundary in memory (else the generic loop)
    L += ["Lnl0_%=:", f"s_mov_b32 s{S_TGT + 1}, s{S_SNIP + 1}",
          f"s_and_b32 s{S_T0}, s{S_SNIP}, 0xffff", f"s_cmp_lg_u32 s{S_T0}, 0", "s_cbranch_scc1 Lstepg_%="]
    for nr in SPECIAL_ROWS:
        L += [f"s_cmp_eq_u32 %[nr], {nr}", f"s_cbranch_scc1 Lstepr{nr}_%="]
    L.append("s_branch Lstepg_%=")
    for nr in SPECIAL_ROWS:
        L += step_loop(f"r{nr}", nr)
        L.append("s_branch Lepi0_%=")
    L += step_loop("g", None)
    L += ["Lepi0_%=:", "s_cmp_eq_u32 %[nr], 0", "s_cbranch_scc1 Lend_%="]
    L += epilogue()
    return L


def epilogue():
    """phi^-1, transpose back, store the wave's rows (XOR the accumulate source first); then
    the snippet table"""
    L = []
    L += [f"s_mov_b64 s[{S_ODESC}:{S_ODESC + 1}], %[ob]", f"s_mov_b32 s{S_ODESC + 2}, 0x80000000",
          f"s_mov_b32 s{S_ODESC + 3}, 0x00020000",
          f"s_mov_b64 s[{S_ADESC}:{S_ADESC + 1}], %[ab]", f"s_mov_b32 s{S_ADESC + 2}, 0x80000000",
          f"s_mov_b32 s{S_ADESC + 3}, 0x00020000"]
    for i in range(8):
        L.append(f"ds_read_b32 v{V_W + i}, %[lo] offset:{4 * i}")
    # the rows' output byte offsets (the table entries' registers are free now): per-block mode
    # from the row table, else (oslot + r) * oss
    L += ["s_cmp_eq_u64 %[rp], 0", "s_cbranch_scc1 Lflat_%=",
          f"s_load_dwordx8 s[{S_OFF}:{S_OFF + 7}], %[rp], 0x0",
          f"s_load_dwordx4 s[{S_OFF + 8}:{S_OFF + 11}], %[rp], 0x20", "s_branch Lrows_%=", "Lflat_%=:"]
    for r in range(ROWS):
        L += [f"s_add_u32 s{S_OFF + r}, %[oslot], {r}", f"s_mul_i32 s{S_OFF + r}, s{S_OFF + r}, %[oss]"]
    L += ["Lrows_%=:", "s_waitcnt lgkmcnt(0)"]
    x = slot()
    tmp = [V_CA + i for i in range(16)]
    for r in range(ROWS):
        if r:
            L += [f"s_cmp_le_u32 %[nr], {r}", "s_cbranch_scc1 Lepi_%="]
        L += phi_inv_code(r)
        L += transpose16(x, V_TMP)
        L += [f"s_mov_b32 s{S_T1}, s{S_OFF + r}",
              "s_cmp_eq_u32 %[acc], 0", f"s_cbranch_scc1 Lna{r}_%=",
              f"s_add_u32 s{S_T2}, %[aslot], {r}", f"s_mul_i32 s{S_T2}, s{S_T2}, %[ass]"]
        # the accumulate source's piece offsets (LDS) in the loads' own destination registers
        L += [f"ds_read_b32 v{tmp[2 * i]}, %[lo] offset:{32 + 4 * i}" for i in range(8)]
        L.append("s_waitcnt lgkmcnt(0)")
        for i in range(8):
            L.append(f"buffer_load_dwordx2 v[{tmp[2 * i]}:{tmp[2 * i + 1]}], v{tmp[2 * i]}, s[{S_ADESC}:{S_ADESC + 3}], s{S_T2} offen")
        L.append("s_waitcnt vmcnt(0)")
        for i in range(16):
            L.append(f"v_xor_b32 v{x[i]}, v{x[i]}, v{tmp[i]}")
        L.append(f"Lna{r}_%=:")
        for i in range(8):
            L.append(f"buffer_store_dwordx2 v[{x[2 * i]}:{x[2 * i + 1]}], v{V_W + i}, s[{S_ODESC}:{S_ODESC + 3}], s{S_T1} offen"
                     + (" nt" if NT_STORES else ""))
    L += ["Lepi_%=:", "s_branch Lend_%="]
    L += snippets()
    L.append("Lend_%=:")
    return L


def pass_rows(m, passes, p):
    """rows [lo, hi) of pass p when m rows are spread evenly over `passes` passes"""
    return p * m // passes, (p + 1) * m // passes


def n_passes(m):
    """passes of a product with m rows: the fewest of at most ROWS rows, rounded up to whole
    workgroups of four"""
    return (((m + ROWS - 1) // ROWS) + NWAVES - 1) // NWAVES * NWAVES


def clobbers(last_s=None):
    v = [f'"v{i}"' for i in range(V_SLOT, V_LAST + 1)]
    s = [f'"s{i}"' for i in range(S_DESC, (last_s or S_LAST) + 1)]
    return ", ".join(v + s + ['"m0"', '"scc"', '"memory"'])


def asm_block(cond, text, last_s):
    return f"""    {cond} {{
        asm volatile(
            "{text}\\n"
            :
            : {ASM_INPUTS}
            : {clobbers(last_s)});
    }}"""


ASM_INPUTS = """[wb] "s"(wb), [ss] "s"(a.seg_stride), [k] "s"(kk), [tw] "s"(tw), [tstep] "s"(tstep), [t1off] "s"(t1off), [nr] "s"(nr),
              [cmg] "s"(cm.magic), [cdv] "s"(cm.div), [crs] "s"(cm.rem_stride), [cck] "s"(cck), [cbb] "s"(cbb),
              [acc] "s"(a.accumulate), [ob] "s"(ob), [ab] "s"(ab), [oslot] "s"(a.out_slot0 + row0),
              [oss] "s"(a.out_seg_stride), [aslot] "s"(a.acc_slot0 + row0), [ass] "s"(a.acc_seg_stride),
              [wv] "s"(wave), [rp] "s"(rp), [md] "s"(md), [lo] "v"(lo), [xl] "v"(xl), [lq] "v"(lq)"""


def main():
    if "--search" in sys.argv:
        lam, beta, _, _ = choose_tower()
        print(f"LAM, BETA = 0x{lam:02X}, 0x{beta:04X}")
        return
    global FLAGS, CONFIGS, NT_STORES
    diag = "--diag" in sys.argv
    args = [a for a in sys.argv[1:] if a != "--diag"]
    if "--noprefetch" in args:
        args.remove("--noprefetch")
        CONFIGS = [(r, False) for r, _ in CONFIGS]
    if "--rows" in args:   # one configuration only (A/B builds)
        i = args.index("--rows")
        r = int(args[i + 1])
        CONFIGS = [(r, dict(CONFIGS).get(r, True) and PREFETCH)]
        del args[i:i + 2]
    if "--nt-stores" in args:
        args.remove("--nt-stores")
        NT_STORES = True
    if "--waves" in args:
        i = args.index("--waves")
        set_waves(int(args[i + 1]))
        del args[i:i + 2]
    path = args[0]
    variants = DIAG_VARIANTS if diag else VARIANTS
    blocks, kernels, waves = [], [], {}
    for ci, (rows, pf) in enumerate(CONFIGS):
        set_prefetch(pf)
        set_rows(rows)
        # waves per SIMD the register file allows (512 VGPRs per lane, allocated in granules of 8)
        waves[rows] = min(8, 512 // ((V_LAST + 1 + 7) // 8 * 8))
        for v, f in variants.items():
            FLAGS = f
            text = "\\n\"\n            \"".join(body())
            kw = "if constexpr" if not blocks else "else if constexpr"
            blocks.append(asm_block(f"{kw} (R == {rows} && V == {v})", text, S_LAST4))
        FLAGS = ()
        kernels.append(f"""template <int V>
__global__ __launch_bounds__({64 * NWAVES}, {waves[rows]}) void gf16_tw_encode_kernel_r{rows}(Gf16T3Args a)
{{
    tw_body<{rows}, V>(a, bs::wg_index(1));
}}

// several independent products in one grid (the RS16 Toeplitz split, rs16_tmvp): workgroup
// ranges [wg_end[i-1], wg_end[i]) run problem i, so their tails share one launch
template <int V>
__global__ __launch_bounds__({64 * NWAVES}, {waves[rows]}) void gf16_tw_multi_kernel_r{rows}(Gf16TwMulti mm)
{{
    const uint32_t wg = bs::wg_index(1);
    // one body instance (one per problem would hold their argument sets live: more registers,
    // fewer waves); the problem index is workgroup-uniform
    uint32_t i = 0;
    while (i + 1u < mm.n && wg >= mm.wg_end[i]) ++i;
    tw_body<{rows}, V>(mm.e[i], wg - (i ? mm.wg_end[i - 1] : 0u));
}}""")
    set_prefetch(True)
    set_rows(6)
    asm_blocks = "\n".join(blocks)
    kernel_defs = "\n\n".join(kernels)

    def cases(kern, grid, arg):
        out = []
        for rows, _ in CONFIGS:
            inner = "\n".join(f"        case {v}: hipLaunchKernelGGL({kern}_r{rows}<{v}>, dim3((uint32_t){grid}), "
                               f"dim3({64 * NWAVES}), 0, s, {arg}); break;" for v in variants)
            out.append(f"    case {rows}:\n        switch (tw_variant()) {{\n{inner}\n        }}\n        break;")
        return "\n".join(out)
    enc_cases = cases("gf16_tw_encode_kernel", "wgs", "b")
    multi_cases = cases("gf16_tw_multi_kernel", "end", "mm")
    cfg_rows = ", ".join(str(r) for r, _ in CONFIGS)
    cfg_cost = ", ".join(str(PASS_COST.get(r, 100)) for r, _ in CONFIGS)
    if diag:
        tw_variant = """int tw_variant()
{
    static const int v = [] {
        const char* e = std::getenv("NFEC_TW_VARIANT");
        const int x = e ? std::atoi(e) : 0;
        return x >= 0 && x < %d ? x : 0;
    }();
    return v;
}""" % len(variants)
    else:
        tw_variant = "constexpr int tw_variant() { return 0; }"
    phi_cols = ", ".join(f"0x{c:04x}" for c in PHI)
    phi_inv_cols = ", ".join(f"0x{c:04x}" for c in PHI_INV)
    src = f"""// GENERATED by tools/codegen/gen_gf16_tw.py -- do not edit by hand.
// RS16 products through the tower field GF((2^8)^2): bit-sliced, GF(2^8) snippet jumps.
// Isomorphism: lam = 0x{LAM:02x}, beta = 0x{BETA:04x} (phi(x^i) = beta^i).
#include <cstdlib>
#include "nfec_internal.hpp"
#include "bitslice.hpp"

namespace nfec {{
namespace {{

// kernel configurations: rows per wave and the relative cost of one pass
constexpr uint32_t kTwRows[] = {{{cfg_rows}}};
constexpr uint32_t kTwPassCost[] = {{{cfg_cost}}};
constexpr uint32_t kTwConfigs = {len(CONFIGS)};

// the column map's scalars (col_offset): the multiply-high constant, the divisor and the stride of
// the remainder (the segment stride; the chunk stride when the divisor is 1, cmg then 0)
struct ChunkMap {{
    uint32_t magic, div, rem_stride;
}};

__device__ __forceinline__ ChunkMap chunk_map(const Gf16T3Args& a, uint32_t cck)
{{
    return {{a.col_magic, a.col_div ? a.col_div : 1u, a.col_div == 1u ? cck : a.seg_stride}};
}}

template <int R>
__device__ __forceinline__ uint32_t gf16_tw_passes_dev(uint32_t m)
{{
    return ((m + R - 1u) / R + {NWAVES - 1}u) / {NWAVES}u * {NWAVES}u;
}}

template <int R, int V>
__device__ __forceinline__ void tw_body(const Gf16T3Args& a, uint32_t wg)
{{
    // per lane, shared by the workgroup's waves (each writes the same values and reads only
    // what it wrote itself, so no barrier): 8 output and 8 accumulate-source offsets (epilogue),
    // the 8 pieces' numData - 1 as u16 pairs (flat shortened loads), the 8 pieces' offsets
    __shared__ uint32_t lds[64 * 28];
    __shared__ uint64_t xch[2 * {XCH_BUF // 8}];       // column planes exchange (body)
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t quads = a.passes / {NWAVES}u;   // workgroups per item group
    // the group's workgroups in a rotated order: when the rows in play leave some of its passes
    // idle (decode stages: rows_lim, per-block e), the idle workgroups are spread over the
    // dispatcher's round-robin instead of falling on the same shader engines every group (with
    // 4 workgroups per group and 2 idle, half of them idled: 2x per pass, r05k)
    const uint32_t group = wg / quads, slot = wg - group * quads;
    const uint32_t quad = (slot + group) % quads;
    // flat mode: item groups run over the batch's bytes across blocks (one coefficient table);
    // per-block mode (blk_rows): each group lies in one block, which has its own table, row
    // count e, column count (blk_cols, else e) and output row offsets
    const bool pb = a.blk_rows != nullptr;
    const uint32_t chunks = (a.vec_bytes + {GROUP_BYTES - 1}u) / {GROUP_BYTES}u;
    const uint32_t pblk = pb ? group / chunks : 0u;
    const uint64_t total = pb ? (uint64_t)a.vec_bytes : (uint64_t)a.nblocks * a.vec_bytes;
    const uint64_t f0 = pb ? (uint64_t)(group - pblk * chunks) * {GROUP_BYTES}u : (uint64_t)group * {GROUP_BYTES}u;
    if ((pb && pblk >= a.nblocks) || f0 >= total) return;  // workgroup-uniform, as the next exits
    // flat shortened mode (num_data): every piece's block has its own numData; columns whose
    // source slot is at or past it read zeros, and the output / accumulate rows may sit after it
    // (out_after_data / acc_after_data: slot numData + r).  The item group runs to the largest
    // numData among its blocks (the column map never maps a column below its own index); a
    // block whose numData is 0 or past nd_limit (0: k) is left alone.  nd_outputs_only: numData
    // places the rows but the loads are not masked (a Toeplitz product over scratch columns)
    const uint32_t lnd = !pb && a.num_data ? 1u : 0u;
    const uint32_t lmask = lnd && !a.nd_outputs_only ? 1u : 0u;
    const uint32_t ndk = a.nd_limit ? a.nd_limit : a.k;
    // rows actually needed (decode stage 1: the last substitute-parity row among the blocks it
    // serves, written by the plan; per-block mode: the block's e); workgroups past them leave
    // at once, waves past them only load, transpose and share their columns
    uint32_t rlim = a.m, kk = a.k;
    if (a.rows_lim) rlim = min(rlim, __builtin_amdgcn_readfirstlane(*a.rows_lim));
    if (pb) {{
        const int32_t e = (int32_t)__builtin_amdgcn_readfirstlane((uint32_t)a.blk_rows[pblk]);
        rlim = e > 0 ? min(rlim, (uint32_t)e) : 0u;
        kk = a.blk_cols ? min(kk, (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)a.blk_cols[pblk])) : min(kk, rlim);
    }} else if (lmask) {{
        const uint32_t bf = (uint32_t)(f0 / a.vec_bytes), bl = (uint32_t)((min(f0 + {GROUP_BYTES}u, total) - 1u) / a.vec_bytes);
        uint32_t mx = 0;
        for (uint32_t b = bf + lane; b <= bl; b += 64u) {{
            const uint32_t v = a.num_data[b];
            if (v >= 1u && v <= ndk) mx = max(mx, v);
        }}
        for (int off = 32; off > 0; off >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, off));
        kk = __builtin_amdgcn_readfirstlane(min(kk, mx));
    }}
    // the rows in play spread evenly over whole workgroups of four passes (the table holds any
    // row range); the launch sized the grid for a.m rows, so later workgroups may leave
    const uint32_t npass = gf16_tw_passes_dev<R>(rlim);
    if (rlim == 0u || kk == 0u || quad * {NWAVES}u >= npass) return;
    const uint32_t pass = quad * {NWAVES}u + wave;
    const uint32_t row0 = pass * rlim / npass, row1 = (pass + 1u) * rlim / npass;
    const uint32_t nr = __builtin_amdgcn_readfirstlane(row1 - row0);
    const uint32_t b0 = pb ? pblk : __builtin_amdgcn_readfirstlane((uint32_t)(f0 / a.vec_bytes));
    const uint8_t* wb = a.base + (uint64_t)b0 * a.block_stride;
    uint32_t q[8];
    uint32_t* po = lds + lane * 28u;
#pragma unroll
    for (int i = 0; i < 8; ++i) {{
        const uint64_t f = f0 + (uint64_t)i * 512u + lane * 8u;
        const uint32_t b = pb ? b0 : (uint32_t)(f / a.vec_bytes);
        const uint32_t p = (uint32_t)(f - (uint64_t)(pb ? 0u : b) * a.vec_bytes);
        const uint32_t raw = lnd && f < total ? (uint32_t)a.num_data[b] : ndk;
        const bool ok = f < total && raw >= 1u && raw <= ndk;
        const uint32_t pnd = ok ? raw : 1u;
        q[i] = pnd - 1u;
        po[20 + i] = ok ? (uint32_t)((uint64_t)(b - b0) * a.block_stride) + p : 0x80000000u;
        po[i] = ok ? (uint32_t)((uint64_t)(b - b0) * a.out_block_stride +
                                (a.out_after_data ? (uint64_t)pnd * a.out_seg_stride : 0u)) + p
                   : 0x80000000u;
        po[8 + i] = ok ? (uint32_t)((uint64_t)(b - b0) * a.acc_block_stride +
                                    (a.acc_after_data ? (uint64_t)pnd * a.acc_seg_stride : 0u)) + p
                       : 0x80000000u;
    }}
#pragma unroll
    for (int i = 0; i < 4; ++i) po[16 + i] = (q[2 * i] & 0xFFFFu) | (q[2 * i + 1] << 16);
    const uint32_t md = __builtin_amdgcn_readfirstlane(lmask);
    const uint32_t lo = bs::lds_addr(po);
    const uint32_t lq = lo + 64u;
    const uint32_t xl = bs::lds_addr(xch) + lane * 8u;
    // table [column][sweep][row][2 entries]: this pass's rows start 2 * row0 elements in
    const uint16_t* tw = a.tw + (uint64_t)b0 * (pb ? a.tw_block_stride : 0u) + 2u * row0;
    // per-block mode: byte offsets of the pass's output rows (row_off[b][row0 ..]); flat: null
    const uint32_t* rp = pb ? a.row_off + (uint64_t)b0 * a.row_off_stride + row0 : nullptr;
    const uint32_t tstep = 8u * a.m, t1off = 4u * a.m;   // bytes per column; sweep 1's offset
    const uint8_t* ob = a.out_base + (uint64_t)b0 * a.out_block_stride;
    const uint8_t* ab = a.acc_base + (uint64_t)b0 * a.acc_block_stride;
    const uint32_t cck = a.col_chunk * a.seg_stride, cbb = a.col_base * a.seg_stride;
    const ChunkMap cm = chunk_map(a, cck);
{asm_blocks}
}}

{kernel_defs}

{tw_variant}

// checks the shape, fills the default output / accumulate layouts and the pass count
int tw_prepare(const Gf16T3Args& a, Gf16T3Args& b, uint64_t& wgs, uint32_t rows)
{{
    // (numData masking is a flat-mode feature; with a column map it masks the mapped source slot,
    // whose byte offset it compares with numData x seg_stride in 24-bit multiplies)
    if ((a.vec_bytes & 7u) || a.vec_bytes == 0 || !a.tw || a.k == 0 || (a.num_data && a.blk_rows) ||
        (a.num_data && (a.seg_stride >= (1u << 24) || a.nd_limit >= (1u << 16))))
        return NFEC_ENOTSUP;
    const uint64_t ndk = a.nd_limit ? a.nd_limit : a.k;
    b = a;
    // the column map: chunks of col_div columns (or 2^col_shift), q = c / d by a multiply-high
    // with ceil(2^32 / d), exact for c, d < 2^16
    if (!b.col_div && a.col_shift < 31) {{
        if (a.col_mask != (1u << a.col_shift) - 1u) return NFEC_ENOTSUP;
        b.col_div = 1u << a.col_shift;
    }}
    if (b.col_div && (b.col_div >= 65536u || a.k >= 65536u)) return NFEC_ENOTSUP;
    b.col_magic = b.col_div >= 2u ? (uint32_t)((0xFFFFFFFFull + b.col_div) / b.col_div) : 0u;
    if (!b.out_base) {{  // encode: parity in place, slot k + r (numData + r when shortened); accumulate against it
        b.out_base = const_cast<uint8_t*>(a.base);
        b.out_block_stride = a.block_stride;
        b.out_seg_stride = a.seg_stride;
        b.out_slot0 = a.num_data ? 0u : a.k;
        b.out_after_data = a.num_data ? 1u : 0u;
    }}
    if (!b.acc_base) {{
        b.acc_base = b.out_base;
        b.acc_block_stride = b.out_block_stride;
        b.acc_seg_stride = b.out_seg_stride;
        b.acc_slot0 = b.out_slot0;
        b.acc_after_data = b.out_after_data;
    }}
    if (!a.num_data) b.out_after_data = b.acc_after_data = 0u;
    // every piece offset of a group ({GROUP_BYTES} bytes of flat positions) plus slot offsets within 2^31
    const uint64_t nbg = {GROUP_BYTES}u / a.vec_bytes + 2u;
    const uint64_t in_slots = a.in_slots ? a.in_slots : (uint64_t)a.k + a.m;
    const uint64_t oslots = (uint64_t)b.out_slot0 + (b.out_after_data ? ndk : 0u) + a.m;
    const uint64_t aslots = (uint64_t)b.acc_slot0 + (b.acc_after_data ? ndk : 0u) + a.m;
    if (nbg * a.block_stride + in_slots * a.seg_stride >= (1ull << 31) ||
        nbg * b.out_block_stride + oslots * b.out_seg_stride >= (1ull << 31) ||
        nbg * b.acc_block_stride + aslots * b.acc_seg_stride >= (1ull << 31))
        return NFEC_ENOTSUP;
    const uint64_t total = (uint64_t)a.nblocks * a.vec_bytes;
    b.passes = gf16_tw_passes(a.m, rows);
    // per-block mode: one table and one set of row offsets per block, no accumulate source
    if (a.blk_rows && (!a.row_off || !a.tw_block_stride || a.accumulate)) return NFEC_ENOTSUP;
    const uint64_t groups = a.blk_rows ? (uint64_t)a.nblocks * ((a.vec_bytes + {GROUP_BYTES - 1}u) / {GROUP_BYTES}u)
                                       : (total + {GROUP_BYTES - 1}u) / {GROUP_BYTES}u;
    wgs = groups * (b.passes / {NWAVES}u);
    return wgs >= (1ull << 31) ? NFEC_ENOTSUP : NFEC_OK;
}}

const uint16_t kPhiCol[16] = {{{phi_cols}}};
const uint16_t kPhiInvCol[16] = {{{phi_inv_cols}}};

}}  // namespace

bool gf16_tw_covers(const Gf16T3Args& a)
{{
    Gf16T3Args b;
    uint64_t wgs = 0;
    return tw_prepare(a, b, wgs, kTwRows[0]) == NFEC_OK;
}}

int launch_gf16_tw_multi(const Gf16T3Args* e, uint32_t n, hipStream_t s)
{{
    if (n == 0 || n > kTwMultiMax) return NFEC_EINVAL;
    // one configuration for the launch: the lowest cost of all its products' passes
    uint32_t rows = kTwRows[0];
    uint64_t best = ~0ull;
    for (uint32_t c = 0; c < kTwConfigs; ++c) {{
        uint64_t cost = 0;
        for (uint32_t i = 0; i < n; ++i)
            cost += (uint64_t)kTwPassCost[c] * gf16_tw_passes(e[i].m, kTwRows[c]) * e[i].k * e[i].nblocks;
        if (cost < best) best = cost, rows = kTwRows[c];
    }}
    Gf16TwMulti mm;
    mm.n = n;
    uint64_t end = 0;
    for (uint32_t i = 0; i < n; ++i) {{
        uint64_t w = 0;
        if (e[i].nblocks) {{
            const int rc = tw_prepare(e[i], mm.e[i], w, rows);
            if (rc) return rc;
        }}
        end += w;
        if (end >= (1ull << 31)) return NFEC_ENOTSUP;
        mm.wg_end[i] = (uint32_t)end;
    }}
    if (end == 0) return NFEC_OK;
    switch (rows) {{
{multi_cases}
    }}
    const hipError_t err = hipGetLastError();
    return err == hipSuccess ? NFEC_OK : hip_fail(err, "gf16 tower multi launch");
}}

int launch_gf16_tw_encode(const Gf16T3Args& a, hipStream_t s)
{{
    if (a.nblocks == 0) return NFEC_OK;
    Gf16T3Args b;
    uint64_t wgs = 0;
    const uint32_t rows = gf16_tw_rows(a.m);
    const int rc = tw_prepare(a, b, wgs, rows);
    if (rc) return rc;
    switch (rows) {{
{enc_cases}
    }}
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? NFEC_OK : hip_fail(e, "gf16 tower encode launch");
}}

void gf16_tw_field(uint16_t phi_cols[16], uint32_t* lam, uint16_t* phi_inv_cols)
{{
    for (int i = 0; i < 16; ++i) phi_cols[i] = kPhiCol[i];
    for (int i = 0; phi_inv_cols && i < 16; ++i) phi_inv_cols[i] = kPhiInvCol[i];
    *lam = 0x{LAM:02x}u;
}}

uint32_t gf16_tw_passes(uint32_t m, uint32_t rows)
{{
    return ((m + rows - 1u) / rows + {NWAVES - 1}u) / {NWAVES}u * {NWAVES}u;
}}

uint32_t gf16_tw_rows(uint32_t m)
{{
    uint32_t rows = kTwRows[0];
    uint64_t best = ~0ull;
    for (uint32_t c = 0; c < kTwConfigs; ++c) {{
        const uint64_t cost = (uint64_t)kTwPassCost[c] * gf16_tw_passes(m, kTwRows[c]);
        if (cost < best) best = cost, rows = kTwRows[c];
    }}
    return rows;
}}

uint64_t gf16_tw_cost(uint32_t m)
{{
    uint64_t best = ~0ull;
    for (uint32_t c = 0; c < kTwConfigs; ++c)
        best = std::min<uint64_t>(best, (uint64_t)kTwPassCost[c] * gf16_tw_passes(m, kTwRows[c]));
    return best;
}}

size_t gf16_tw_table_elems(uint32_t k, uint32_t m)
{{
    return (size_t)k * 4u * m + 32u;   // + the overread of a pass's 12-row entry loads
}}

// snippet byte offsets of the tower kernel: coefficient g = parity_rows[r][c] maps to
// phi(g) = c0 + c1 y.  Table [c][sweep][row][2]: sweep 0 (source x0) = (c0, c1), sweep 1
// (source x1) = (lam c1, c0 ^ c1), each the snippet's byte offset c << {SNIP_ALIGN}.  Rows are
// contiguous, so the kernel can spread any number of rows over its passes at run time.
void gf16_tw_offsets(const std::vector<uint32_t>& parity_rows, uint32_t k, uint32_t m, uint16_t* out)
{{
    const Field& f8 = gf8();
    for (size_t i = 0; i < gf16_tw_table_elems(k, m); ++i) out[i] = 0;
    for (uint32_t c = 0; c < k; ++c)
        for (uint32_t row = 0; row < m; ++row) {{
            const uint32_t g = parity_rows[(size_t)row * k + c];
            uint32_t t = 0;
            for (int i = 0; i < 16; ++i)
                if ((g >> i) & 1u) t ^= kPhiCol[i];
            const uint32_t c0 = t & 255u, c1 = t >> 8;
            uint16_t* o = out + (size_t)c * 4u * m + 2u * row;
            o[0] = (uint16_t)(c0 << {SNIP_ALIGN});
            o[1] = (uint16_t)(c1 << {SNIP_ALIGN});
            o[2u * m] = (uint16_t)(f8.mul(0x{LAM:02x}u, c1) << {SNIP_ALIGN});
            o[2u * m + 1] = (uint16_t)((c0 ^ c1) << {SNIP_ALIGN});
        }}
}}

}}  // namespace nfec
"""
    open(path, "w").write(src)


if __name__ == "__main__":
    main()
