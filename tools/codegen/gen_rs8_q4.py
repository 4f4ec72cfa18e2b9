#!/usr/bin/env python3
"""Generate norm_amd/csrc/gen_rs8_q4.hip: bit-sliced RS8 (and full-block MDP) encode kernels in
which FOUR role waves share every source column's bit transpose through LDS.

Same arithmetic as gen_rs8_asm.py (8x8 bit transpose per source column, method of four
Russians over the constant generator of NormEncoderRS8, src/common/normEncoderRS8.cpp:400-462,
one v_bitop3 per parity bit-plane and column), different work split:

  * a workgroup is 4 waves over the same 256 items (8 bytes each, 32 bytes per lane); wave w
    owns parity rows [w*m/4, (w+1)*m/4): m/4 x 8 plane accumulators (64 VGPRs at m = 32);
  * source columns are dealt round-robin: in step s wave w loads column 4s+w (a 2-slot VGPR
    ring, buffer loads), transposes it (48 VALU) and writes its 8 planes to an LDS slot
    (4 x ds_write_b64); after one s_barrier every wave reads the other three columns' planes
    back (ds_read_b64, double-buffered) and applies all four columns to its rows;
  * the transpose is done once per column instead of once per role, and the register file
    fits in 128 VGPRs, so 4 waves per SIMD are resident (the 2-role kernel holds 256 VGPRs:
    2 waves per SIMD, and its VALU and memory phases overlap badly).

VGPR banks (index mod 4; a VOP3 whose operands share a bank stalls): accumulators in banks 2/3
of quads 0..31, everything a bitop3 reads besides the accumulator in banks 0/1 -- M4RM group A
(even planes and their combinations) in bank 0, group B (odd planes) in bank 1.  A
buffer_load_dwordx2 / ds_read_b64 into the aligned pair (4P, 4P+1) lands dword/plane pair
(2q, 2q+1) in banks (0, 1); the in-place transpose leaves plane b in dword b's register.

Usage: gen_rs8_q4.py OUT.hip
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gen_rs8_asm import MASKS, mdp_matrix, split, transpose  # noqa: E402
from gen_rs8_bitsliced import bitmatrix_rows, generator  # noqa: E402

SHAPES = [(64, 32), (64, 16), (64, 8)]
MDP_SHAPES = [(64, 32), (64, 16)]
NW = 4                       # role waves per workgroup (share each column's transpose)
MULTI = [a for a in range(1, 16) if bin(a).count("1") >= 2]   # 11 combination indices

# ---- register map (v0..v127) ----
COMBO_Q0 = 3                 # combos: quads 3..13, A at 4q (bank 0), B at 4q+1 (bank 1)
RING_Q0 = 14                 # ring slots 0, 1: quads 14..21
P_Q0 = 22                    # 2 LDS plane buffers x 4 quads: quads 22..29
NQUAD = 32


def acc_reg(r, i):
    return 4 * (4 * r + i // 2) + 2 + (i & 1)


def combo_reg(group, a):
    return 4 * (COMBO_Q0 + MULTI.index(a)) + group


class Cfg:
    """nslot: own-column loads in flight per wave (VGPR ring slots)
    lazy:  build group-A combinations one at a time, updates grouped by A entry (2 VGPRs
           instead of 11: room for a third ring slot)
    share: what a column's owner hands the other waves through LDS -- "planes" (the 8
           transposed planes; every wave builds the 22 combinations itself), "A" (planes and
           the 11 group-A combinations), "AB" (all combinations: one slot, two barriers per
           step)"""

    def __init__(self, nslot=2, lazy=False, share="planes", lpol="", spol=""):
        self.nslot, self.lazy, self.share = nslot, lazy, share
        self.lpol, self.spol = lpol, spol  # cache-policy suffixes of the source loads / parity stores
        assert share == "planes" or not lazy
        if lazy:
            # 4 item offsets + LDS address in freed A-combination registers (bank 0)
            self.in_regs = [20, 24, 28, 32, 36]
            self.areg = [12, 16]
            self.temps = {0: [12, 16, 40, 44], 1: [13, 17, 21, 25]}
            slot2 = [0, 1, 2, 30]
        else:
            self.in_regs = [0, 1, 4, 5, 8] + ([9] if share == "A" else [])
            self.areg = None
            self.temps = {0: [combo_reg(0, MULTI[i]) for i in range(4)], 1: [combo_reg(1, MULTI[i]) for i in range(4)]}
            slot2 = None
        self.slot_quads = [[RING_Q0 + q for q in range(4)], [RING_Q0 + 4 + q for q in range(4)]]
        if nslot == 3:
            assert lazy, "the third ring slot needs the lazy A combinations' registers"
            self.slot_quads.append(slot2)
        assert nslot in (2, 3)

    def ring_slot(self, i):
        w = []
        for q in self.slot_quads[i]:
            w += [4 * q, 4 * q + 1]
        return w


DEFAULT = Cfg(2, False)
# variants of the (64, 32) kernel selectable with NFEC_Q4_VARIANT=<id> for A/B runs
VARIANTS = {1: Cfg(3, True), 2: Cfg(2, True), 3: Cfg(2, share="A"), 4: Cfg(2, share="AB"),
            5: Cfg(lpol=" nt"), 6: Cfg(spol=" nt"), 7: Cfg(lpol=" nt", spol=" nt")}
S_LRS, S_SRS = 64, 68        # load / store buffer descriptors
S_MASK = 72                  # s72..s77 transpose masks (gen_rs8_asm.transpose reads them here)
S_COL, S_ROW = 78, 79
SLOT_BYTES = NW * 4 * 512    # one LDS slot: 4 columns x 4 plane pairs x 64 lanes x 8 bytes
# A/B probes of the (64, 32) kernel, NFEC_Q4_VARIANT=<id> (never the default): VALU + LDS only
# (no source loads), memory only (loads and stores, no arithmetic, no LDS), no LDS exchange
# (every wave reuses its own column's planes: the cost of the exchange and its barrier)
PROBES = {8: "noload", 9: "nocompute", 10: "nolds"}


def quad_planes(q0):
    """w[d], d = 0..7, of the 4 quads starting at q0 (pairs (4q, 4q+1))."""
    w = []
    for q in range(4):
        w += [4 * (q0 + q), 4 * (q0 + q) + 1]
    return w


def pbuf(b):
    return quad_planes(P_Q0 + 4 * b)


def combo_temps(cfg):
    """transpose temporaries (4 per bank per stage) from the combination registers, which are
    dead while a column is transposed"""
    def make():
        avail = {0: list(cfg.temps[0]), 1: list(cfg.temps[1])}

        def pick(avoid):
            return avail[1 if avoid == 0 else 0].pop(0)
        return pick
    return make


def epi_temps(cfg):
    """temporaries for an accumulator transpose (accs in banks 2/3): ring/P registers"""
    def make():
        free = cfg.ring_slot(0) + cfg.ring_slot(1) + pbuf(0) + pbuf(1)

        def pick(avoid):
            for i, r in enumerate(free):
                if r % 4 != avoid:
                    return free.pop(i)
            raise RuntimeError("no temp")
        return pick
    return make


def combos(w, need):
    """the multi-plane combinations needed for this column (group A = w[0,2,4,6] in bank 0,
    group B = w[1,3,5,7] in bank 1); returns (code, {a: reg} for A, {b: reg} for B)"""
    code = []
    tabs = []
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


def update(acc, A, B, a, b, first):
    if first:
        if a and b:
            return f"v_xor_b32 v{acc}, v{A[a]}, v{B[b]}"
        if a or b:
            return f"v_mov_b32 v{acc}, v{A[a] if a else B[b]}"
        return f"v_mov_b32 v{acc}, 0"
    if a and b:
        return f"v_bitop3_b32 v{acc}, v{acc}, v{A[a]}, v{B[b]} bitop3:0x96"
    if a:
        return f"v_xor_b32 v{acc}, v{A[a]}, v{acc}"
    if b:
        return f"v_xor_b32 v{acc}, v{B[b]}, v{acc}"
    return None


def lazy_column(w, ups, need, areg, first):
    """group-B combinations up front, group-A ones built one at a time into two alternating
    registers, each followed by the updates that use it"""
    code, _, B = combos(w, [set(), need[1]])
    single = [w[2 * t] for t in range(4)]
    order = sorted({a for _, a, _ in ups}, key=lambda a: (bin(a).count("1"), a))
    if 15 in order:  # build 15 right after a 3-subset, from it
        order.remove(15)
        order.append(15)
    A = {1 << t: single[t] for t in range(4)}
    prev, k = None, 0
    for a in order:
        if a in MULTI:
            dst = areg[k % 2]
            k += 1
            bits = [t for t in range(4) if (a >> t) & 1]
            if prev is not None and prev[0] & a == prev[0] and bin(a & ~prev[0]).count("1") == 1:
                code.append(f"v_xor_b32 v{dst}, v{prev[1]}, v{single[(a & ~prev[0]).bit_length() - 1]}")
            elif len(bits) == 2:
                code.append(f"v_xor_b32 v{dst}, v{single[bits[0]]}, v{single[bits[1]]}")
            else:
                code.append(f"v_bitop3_b32 v{dst}, v{single[bits[0]]}, v{single[bits[1]]}, v{single[bits[2]]} bitop3:0x96")
                if len(bits) == 4:
                    code.append(f"v_xor_b32 v{dst}, v{dst}, v{single[bits[3]]}")
            A[a] = dst
            prev = (a, dst)
        for acc, ua, ub in ups:
            if ua == a:
                u = update(acc, A, B, ua, ub, first)
                if u:
                    code.append(u)
    return code


def column_code(G, r0, rows, j, w, first, cfg=None):
    """updates of rows [r0, r0+rows) by source column j whose planes are in w[0..7]"""
    mats = [bitmatrix_rows(G[r0 + r][j]) for r in range(rows)]
    ups, need = [], [set(), set()]
    for r in range(rows):
        for i in range(8):
            a, b = split(mats[r][i])
            ups.append((acc_reg(r, i), a, b))
            if a:
                need[0].add(a)
            if b:
                need[1].add(b)
    if cfg is not None and cfg.lazy:
        return lazy_column(w, ups, need, cfg.areg, first)
    code, A, B = combos(w, need)
    for acc, a, b in ups:
        if first:
            if a and b:
                code.append(f"v_xor_b32 v{acc}, v{A[a]}, v{B[b]}")
            elif a or b:
                code.append(f"v_mov_b32 v{acc}, v{A[a] if a else B[b]}")
            else:
                code.append(f"v_mov_b32 v{acc}, 0")
        elif a and b:
            code.append(f"v_bitop3_b32 v{acc}, v{acc}, v{A[a]}, v{B[b]} bitop3:0x96")
        elif a:
            code.append(f"v_xor_b32 v{acc}, v{A[a]}, v{acc}")
        elif b:
            code.append(f"v_xor_b32 v{acc}, v{B[b]}, v{acc}")
    return code


def lds_off(slot, c, i):
    return ((slot * NW + c) * 4 + i) * 512


def updates(ups, A, B, first):
    out = []
    for acc, a, b in ups:
        u = update(acc, A, B, a, b, first)
        if u:
            out.append(u)
    return out


def column_ups(G, r0, rows, j):
    mats = [bitmatrix_rows(G[r0 + r][j]) for r in range(rows)]
    ups, need = [], [set(), set()]
    for r in range(rows):
        for i in range(8):
            a, b = split(mats[r][i])
            ups.append((acc_reg(r, i), a, b))
            if a:
                need[0].add(a)
            if b:
                need[1].add(b)
    return ups, need


# ---- shared-combination layouts (Cfg.share "A" / "AB") ----
A_COL = 4 * 512 + 11 * 256          # "A": per column 4 plane pairs (b64) + 11 A combos (b32)


def a_off(slot, c, part, i):
    """share "A" LDS offsets: part 0 = plane pair i (lane*8 addressing), part 1 = A combo i
    (lane*4 addressing, stored after the pairs)"""
    base = (slot * NW + c) * A_COL
    return base + (i * 512 if part == 0 else 4 * 512 + i * 256)


def ab_off(c, i):
    """share "AB" LDS offsets (one slot): 15 b64 pairs per column -- pairs 0..3 planes (2i, 2i+1),
    pairs 4..14 the combinations (A[m], B[m]) of MULTI[i - 4]"""
    return (c * 15 + i) * 512


# shortened batches (per-block numData, RFC 5052 small blocks / an object's last block): every
# piece's block has its own numData; source column c of a piece whose numData <= c counts as
# zero and the parity goes to slot numData + r.  The column loads are issued unmasked (so no
# load waits on the numData fetch: a masked load offset would put a dependent memory round trip
# in front of every workgroup's first column, measured +13 % at RS8(64,32)); the loaded
# dwords of a masked piece are zeroed before the transpose (one SDWA compare of c with the
# piece's numData byte, two v_cndmask).  A column at or past numData lies inside the block (its
# parity or unused slots), read but never used.  The four pieces' numData are fetched inside the
# asm (buffer_load_ushort through a descriptor over num_data + the wave's first block, the
# pieces' block deltas packed in %[nd]) and packed as bytes into SHORT_TMP[0] (k <= 64; an
# invalid numData -- 0 or past k -- packs as 0: every column masked, every store dropped).
SHORT_TMP = [120, 121, 124, 125]
SHORT_ND = 9
S_NDD = 80                   # numData descriptor (shortened kernels)


def short_fetch_nd(k):
    """the four pieces' numData (block deltas in %[nd]) -> SHORT_TMP (issued before any column load)"""
    L = [f"s_mov_b64 s[{S_NDD}:{S_NDD + 1}], %[ndb]", f"s_mov_b32 s{S_NDD + 2}, 0x80000000",
         f"s_mov_b32 s{S_NDD + 3}, 0x00020000"]
    for q, t in enumerate(SHORT_TMP):
        L += [f"v_bfe_u32 v{t}, %[nd], {8 * q}, 8", f"v_lshlrev_b32 v{t}, 1, v{t}",
              f"buffer_load_ushort v{t}, v{t}, s[{S_NDD}:{S_NDD + 3}], 0 offen"]
    return L


def short_pack_nd(k):
    """after the first column wait (the numData loads are older): SHORT_TMP[0] = the four
    numData as bytes, 0 for a value outside [1, k]"""
    L = []
    for q, t in enumerate(SHORT_TMP):
        L += [f"v_subrev_u32 v{t}, 1, v{t}",                                         # numData - 1
              f"v_cmp_gt_u32 vcc, {k}, v{t}",
              f"v_add_u32 v{t}, 1, v{t}",
              f"v_cndmask_b32 v{t}, 0, v{t}, vcc"]
        if q:
            L.append(f"v_lshl_or_b32 v{SHORT_TMP[0]}, v{t}, {8 * q}, v{SHORT_TMP[0]}")
    # the lane's smallest numData (SHORT_TMP[1]): a step whose column is below it in every lane
    # skips the masking (RFC 5052 blocks of k and k - 1 mask in the last step only)
    t0, t1, t2, t3 = SHORT_TMP
    L += [f"v_min3_u32 v{t1}, v{t1}, v{t2}, v{t3}", f"v_and_b32 v{t2}, 0xff, v{t0}", f"v_min_u32 v{t1}, v{t1}, v{t2}"]
    return L


_mask_id = [0]


def short_mask(col, w, tail):
    """zero the loaded dwords w[2q], w[2q+1] of every piece q whose numData <= col.  The common
    case -- no lane holds such a piece -- falls through a not-taken branch; the masking itself
    sits out of line (appended to `tail`, placed after the epilogue) and jumps back"""
    _mask_id[0] += 1
    i = _mask_id[0]
    L = [f"v_cmp_gt_u32 vcc, {col + 1}, v{SHORT_TMP[1]}", f"s_cbranch_vccnz Lmask{i}_%=", f"Lback{i}_%=:"]
    tail.append(f"Lmask{i}_%=:")
    for q in range(4):
        tail += [f"v_cmp_lt_u32_sdwa vcc, {col}, v{SHORT_TMP[0]} src0_sel:DWORD src1_sel:BYTE_{q}",
                 f"v_cndmask_b32 v{w[2 * q]}, 0, v{w[2 * q]}, vcc",
                 f"v_cndmask_b32 v{w[2 * q + 1]}, 0, v{w[2 * q + 1]}, vcc"]
    tail.append(f"s_branch Lback{i}_%=")
    return L


def role_asm(G, k, m, w, probe=None, cfg=DEFAULT, short=False):
    noload, nocompute, nolds = probe == "noload", probe == "nocompute", probe == "nolds"
    assert not short or (k <= 64 and cfg is DEFAULT and probe is None)
    NS = cfg.nslot
    rows = m // NW
    r0 = w * rows
    tail = []  # out-of-line blocks (shortened masking), after the epilogue
    steps = k // NW
    L = []
    L.append(f"s_mov_b64 s[{S_LRS}:{S_LRS + 1}], %[ib]")
    L.append(f"s_mov_b32 s{S_LRS + 2}, 0x80000000")   # offsets with bit 31 set read as zero
    L.append(f"s_mov_b32 s{S_LRS + 3}, 0x00020000")
    L.append(f"s_mov_b64 s[{S_SRS}:{S_SRS + 1}], %[ob]")
    L.append(f"s_mov_b32 s{S_SRS + 2}, 0x80000000")   # ... and stores there are dropped
    L.append(f"s_mov_b32 s{S_SRS + 3}, 0x00020000")
    for i, mk in enumerate(MASKS):
        L.append(f"s_mov_b32 s{S_MASK + i}, 0x{mk:08x}")
    offs = ["%[o0]", "%[o1]", "%[o2]", "%[o3]"]

    def loads(step):
        if noload:
            return []
        col = NW * step + w
        rs = cfg.ring_slot(step % NS)
        out = [f"s_mul_i32 s{S_COL}, %[ss], {col}"]
        for q in range(4):
            out.append(f"buffer_load_dwordx2 v[{rs[2 * q]}:{rs[2 * q + 1]}], {offs[q]}, s[{S_LRS}:{S_LRS + 3}], s{S_COL} offen{cfg.lpol}")
        return out

    if short and SH_PROBE != "nofetch":
        L += short_fetch_nd(k)
    elif short:  # (A/B probe: every piece numData k, no fetch, no masking -- timing only)
        L += [f"v_mov_b32 v{SHORT_TMP[0]}, 0x{k:02x}{k:02x}{k:02x}{k:02x}", f"v_mov_b32 v{SHORT_TMP[1]}, {k}"]
    for s in range(min(NS, steps)):
        L += loads(s)
    for s in range(steps):
        slot = s % 2
        own = cfg.ring_slot(s % NS)
        pending = min(steps, s + NS) - (s + 1)  # later steps' loads in flight behind ours
        if not noload:
            L.append(f"s_waitcnt vmcnt({4 * pending})")
        if short and SH_PROBE != "nofetch":
            if s == 0:
                L += short_pack_nd(k)
            if SH_PROBE != "nomask":
                L += short_mask(NW * s + w, own, tail)
        if nocompute:
            for i in range(8):  # keep the loaded data live
                L.append(f"v_xor_b32 v{acc_reg(0, i)}, v{own[i]}, v{acc_reg(0, i)}")
            if s + NS < steps:
                L += loads(s + NS)
            continue
        L += transpose(own, combo_temps(cfg))
        if nolds:
            for c in range(NW):
                L += column_code(G, r0, rows, NW * s + c, own, first=(s == 0 and c == 0), cfg=cfg)
            if s + NS < steps:
                L += loads(s + NS)
            continue
        others = [(w + d) % NW for d in range(1, NW)]
        if cfg.share in ("A", "AB"):
            L += shared_step(G, r0, rows, s, w, own, others, cfg)
            if s + NS < steps:
                # issued at the end of the step: the ring slot's planes are dead only then
                L += loads(s + NS)
            continue
        for i in range(4):
            L.append(f"ds_write_b64 %[la], v[{own[2 * i]}:{own[2 * i + 1]}] offset:{lds_off(slot, w, i)}")
        L += column_code(G, r0, rows, NW * s + w, own, first=(s == 0), cfg=cfg)
        if s + NS < steps:
            L += loads(s + NS)
        L.append("s_waitcnt lgkmcnt(0)")
        L.append("s_barrier")

        def reads(c, buf):
            p = pbuf(buf)
            return [f"ds_read_b64 v[{p[2 * i]}:{p[2 * i + 1]}], %[la] offset:{lds_off(slot, c, i)}" for i in range(4)]

        L += reads(others[0], 0)
        L += reads(others[1], 1)
        for t, c in enumerate(others):
            buf = t % 2
            more = t + 1 < len(others)  # the next column's reads are in flight
            L.append(f"s_waitcnt lgkmcnt({4 if more else 0})")
            L += column_code(G, r0, rows, NW * s + c, pbuf(buf), first=False, cfg=cfg)
            if t + 2 < len(others):
                L += reads(others[t + 2], buf)
    # epilogue: planes back to bytes, optional accumulate, store (shortened: the items' parity
    # slot 0 is numData, so the row offsets are the items' offsets + numData * seg_stride)
    if short:
        # piece offset + numData * seg_stride; numData 0 (invalid) sets bit 31: the stores drop
        # (the packed numData sit in SHORT_TMP[0], so piece 0's offset goes there last)
        x = pbuf(1)[-1]  # (free until the first row's transpose)
        for q in (1, 2, 3, 0):
            t = SHORT_TMP[q]
            L += [f"v_bfe_u32 v{x}, v{SHORT_TMP[0]}, {8 * q}, 8", f"v_mad_u32_u24 v{t}, v{x}, %[ss], {offs[q]}",
                  f"v_subrev_u32 v{x}, 1, v{x}", f"v_and_or_b32 v{t}, v{x}, s{S_LRS + 2}, v{t}"]
        offs = [f"v{t}" for t in SHORT_TMP]
    for r in range(rows):
        acc = [acc_reg(r, i) for i in range(8)]
        L += transpose(acc, epi_temps(cfg))
        L.append(f"s_mul_i32 s{S_ROW}, %[ss], {(0 if short else k) + r0 + r}")
        tmp = cfg.ring_slot(0)
        L.append("s_cmp_eq_u32 %[acc], 0")
        L.append(f"s_cbranch_scc1 Lnoacc_{r}_%=")
        for q in range(4):
            L.append(f"buffer_load_dwordx2 v[{tmp[2 * q]}:{tmp[2 * q + 1]}], {offs[q]}, s[{S_SRS}:{S_SRS + 3}], s{S_ROW} offen")
        L.append("s_waitcnt vmcnt(0)")
        for q in range(4):
            L.append(f"v_xor_b32 v{acc[2 * q]}, v{tmp[2 * q]}, v{acc[2 * q]}")
            L.append(f"v_xor_b32 v{acc[2 * q + 1]}, v{tmp[2 * q + 1]}, v{acc[2 * q + 1]}")
        L.append(f"Lnoacc_{r}_%=:")
        for q in range(4):
            L.append(f"buffer_store_dwordx2 v[{acc[2 * q]}:{acc[2 * q + 1]}], {offs[q]}, s[{S_SRS}:{S_SRS + 3}], s{S_ROW} offen{cfg.spol}")
    if tail:
        L += ["s_branch Lroleend_%="] + tail + ["Lroleend_%=:"]
    return L


def shared_step(G, r0, rows, s, w, own, others, cfg):
    """one step of the shared-combination variants (after the own column's transpose)"""
    L = []
    j_own = NW * s + w
    ups, need = column_ups(G, r0, rows, j_own)
    # the owner builds every combination the other waves may need
    full = [set(MULTI), set(MULTI) if cfg.share == "AB" else need[1]]
    code, A, B = combos(own, full)
    L += code
    if cfg.share == "A":
        slot = s % 2
        for i in range(4):
            L.append(f"ds_write_b64 %[la], v[{own[2 * i]}:{own[2 * i + 1]}] offset:{a_off(slot, w, 0, i)}")
        for i, a in enumerate(MULTI):
            L.append(f"ds_write_b32 %[la4], v{combo_reg(0, a)} offset:{a_off(slot, w, 1, i)}")
        L += updates(ups, A, B, s == 0)
        L.append("s_waitcnt lgkmcnt(0)")
        L.append("s_barrier")

        def reads(c, buf):
            p = pbuf(buf)
            return [f"ds_read_b64 v[{p[2 * i]}:{p[2 * i + 1]}], %[la] offset:{a_off(slot, c, 0, i)}" for i in range(4)]

        def areads(c):
            return [f"ds_read_b32 v{combo_reg(0, a)}, %[la4] offset:{a_off(slot, c, 1, i)}" for i, a in enumerate(MULTI)]

        L += reads(others[0], 0) + areads(others[0])
        L += reads(others[1], 1)
        for t, c in enumerate(others):
            buf = t % 2
            # in flight behind this column's reads: the next column's planes (4)
            L.append(f"s_waitcnt lgkmcnt({4 if t + 1 < len(others) else 0})")
            p = pbuf(buf)
            u, nd = column_ups(G, r0, rows, NW * s + c)
            code, _, Bc = combos(p, [set(), nd[1]])
            Ac = {1 << q: p[2 * q] for q in range(4)}
            Ac.update({a: combo_reg(0, a) for a in MULTI})
            L += code
            L += updates(u, Ac, Bc, False)
            if t + 1 < len(others):
                L += areads(others[t + 1])
            if t + 2 < len(others):
                L += reads(others[t + 2], buf)
        return L
    # "AB": one slot; the barrier before the write keeps it from overwriting what the other
    # waves still read of the previous step
    pairs = [(own[2 * i], own[2 * i + 1]) for i in range(4)] + [(combo_reg(0, a), combo_reg(1, a)) for a in MULTI]
    L.append("s_barrier")
    for i, (x, y) in enumerate(pairs):
        L.append(f"ds_write_b64 %[la], v[{x}:{y}] offset:{ab_off(w, i)}")
    L += updates(ups, A, B, s == 0)
    L.append("s_waitcnt lgkmcnt(0)")
    L.append("s_barrier")
    for t, c in enumerate(others):
        p = pbuf(t % 2)
        if t == 0:
            L += [f"ds_read_b64 v[{p[2 * i]}:{p[2 * i + 1]}], %[la] offset:{ab_off(c, i)}" for i in range(4)]
        L += [f"ds_read_b64 v[{combo_reg(0, a)}:{combo_reg(1, a)}], %[la] offset:{ab_off(c, 4 + i)}"
              for i, a in enumerate(MULTI)]
        if t + 1 < len(others):
            q = pbuf((t + 1) % 2)
            L += [f"ds_read_b64 v[{q[2 * i]}:{q[2 * i + 1]}], %[la] offset:{ab_off(others[t + 1], i)}" for i in range(4)]
        L.append(f"s_waitcnt lgkmcnt({4 if t + 1 < len(others) else 0})")
        u, _ = column_ups(G, r0, rows, NW * s + c)
        Ac = {1 << q: p[2 * q] for q in range(4)}
        Bc = {1 << q: p[2 * q + 1] for q in range(4)}
        Ac.update({a: combo_reg(0, a) for a in MULTI})
        Bc.update({a: combo_reg(1, a) for a in MULTI})
        L += updates(u, Ac, Bc, False)
    return L


def clobbers(cfg, short=False):
    keep = cfg.in_regs + ([SHORT_ND] if short else [])
    v = [f'"v{i}"' for i in range(4 * NQUAD) if i not in keep]
    s = [f'"s{i}"' for i in range(S_LRS, (S_NDD + 3 if short else S_ROW) + 1)]
    return ", ".join(v + s + (['"vcc"'] if short else []) + ['"scc"', '"memory"'])


def lds_bytes(cfg):
    if cfg.share == "A":
        return 2 * NW * A_COL
    if cfg.share == "AB":
        return NW * 15 * 512
    return 2 * SLOT_BYTES


def gen_kernel(k, m, G=None, prefix="rs8_q4_enc", probe=None, suffix="", cfg=DEFAULT, short=False):
    assert k % NW == 0 and m % NW == 0
    G = G if G is not None else generator(k, m)
    K = f"{prefix}{suffix}{'_sh' if short else ''}_k{k}_m{m}"
    out = []
    la4 = ', [la4] "v"(la4)' if cfg.share == "A" else ""
    nd_in = ', [ndb] "s"(ndb), [nd] "v"(ndp)' if short else ""
    nd_out = ""
    for w in range(NW):
        body = role_asm(G, k, m, w, probe, cfg, short)
        s = "\\n\"\n        \"".join(body)
        out.append(f"""__device__ __forceinline__ void {K}_role{w}(const bs::EncArgs& a, const bs::Items& it, const uint32_t o[4], uint32_t la, uint32_t la4, uint32_t ndp, const uint16_t* ndb)
{{
    asm volatile(
        "{s}\\n"
        : {nd_out}
        : [ib] "s"(it.wbase), [ob] "s"(it.obase), [ss] "s"(a.seg_stride), [acc] "s"(a.accumulate),
          [o0] "v"(o[0]), [o1] "v"(o[1]), [o2] "v"(o[2]), [o3] "v"(o[3]), [la] "v"(la){la4}{nd_in}
        : {clobbers(cfg, short)});
}}""")
    body = [f"__global__ __launch_bounds__({64 * NW}, {NW}) void {K}(bs::EncArgs a)", "{"]
    body.append(f"    __shared__ uint32_t lds[{lds_bytes(cfg) // 4}];")
    body.append("    const uint32_t lane = threadIdx.x & 63;")
    body.append("    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);")
    body.append("    bs::Items it;")
    body.append("    uint32_t o[4];")
    body.append("    uint32_t ndp = 0;")
    body.append("    const uint16_t* ndb = nullptr;")
    if not short:
        body.append("    bs::make_items(a, bs::wg_index(a.xcd_remap) * 256u, lane, it);")
        body.append("    // out-of-range items: loads read zero, stores are dropped (bit 31 past num_records)")
        body.append("#pragma unroll")
        body.append("    for (int i = 0; i < 4; ++i) o[i] = it.nbytes[i] == 8 ? it.off[i] : 0x80000000u;")
    else:
        body.append("    // make_items' geometry (vec % 8 == 0), plus the pieces' block deltas from the wave's first")
        body.append("    // block as bytes (a workgroup's 256 pieces span at most 256 blocks): the asm fetches their")
        body.append("    // numData from ndb = num_data + that block")
        body.append("    const uint32_t ips = a.vec >> 3, ib = bs::wg_index(a.xcd_remap) * 256u, total = a.nblocks * ips;")
        body.append("    const uint32_t b0 = __builtin_amdgcn_readfirstlane(min(ib, total - 1u) / ips);")
        body.append("    it.wbase = a.base + (uint64_t)b0 * a.block_stride;")
        body.append("    it.obase = a.out + (uint64_t)b0 * a.block_stride;")
        body.append("    ndb = a.num_data + b0;")
        body.append("#pragma unroll")
        body.append("    for (int i = 0; i < 4; ++i) {")
        body.append("        const uint32_t g = ib + (uint32_t)i * 64u + lane, gg = g < total ? g : ib;")
        body.append("        const uint32_t db = gg / ips - b0;")
        body.append("        o[i] = g < total ? db * (uint32_t)a.block_stride + (gg - (db + b0) * ips) * 8u : 0x80000000u;")
        body.append("        ndp |= db << (8 * i);")
        body.append("    }")
    body.append("    const uint32_t la = bs::lds_addr(lds) + lane * 8u;   // b64 rows: 8 bytes per lane")
    body.append("    const uint32_t la4 = bs::lds_addr(lds) + lane * 4u;  // b32 rows")
    for w in range(NW):
        kw = "if" if w == 0 else "else if"
        body.append(f"    {kw} (wave == {w}) {K}_role{w}(a, it, o, la, la4, ndp, ndb);")
    body.append("}")
    out.append("\n".join(body))
    out.append(f"""
static int launch_{K}(const bs::EncArgs& a, hipStream_t s)
{{
    const uint64_t items = (uint64_t)a.nblocks * ((a.vec + 7) / 8);
    if ({"!a.num_data" if short else "a.num_data"} || (a.vec & 7u) || a.nt_store || items >= (1ull << 31) ||
        !bs::offsets_fit(a.block_stride, a.seg_stride))
        return NFEC_ENOTSUP;
    const uint64_t wgs = (items + 255) / 256;
    hipLaunchKernelGGL({K}, dim3((uint32_t)wgs), dim3({64 * NW}), 0, s, a);
    return hipGetLastError() == hipSuccess ? NFEC_OK : NFEC_EDEVICE;
}}""")
    return "\n\n".join(out)


SH_PROBE = None   # A/B timing probes of the shortened kernels (wrong bytes for masked pieces): --sh-probe nomask|nofetch


def main():
    # --diag: also emit the A/B variants and probes and their NFEC_Q4_VARIANT switch (the
    # diagnostic library, make -C norm_amd diag); the product library ships the defaults only
    global SH_PROBE
    if "--sh-probe" in sys.argv:
        i = sys.argv.index("--sh-probe")
        SH_PROBE = sys.argv[i + 1]
        del sys.argv[i:i + 2]
    diag = "--diag" in sys.argv
    path = [a for a in sys.argv if a != "--diag"][1]
    parts = [
        "// GENERATED by tools/codegen/gen_rs8_q4.py -- do not edit by hand.",
        "// Bit-sliced RS8 / MDP encode: 4 role waves per workgroup share each column's transpose",
        "// through LDS; (k, m) in: " + ", ".join(f"({k},{m})" for k, m in SHAPES),
        "#include <cstdlib>",
        '#include "bitslice.hpp"',
        "",
        "namespace nfec {",
        "namespace {",
    ]
    for k, m in SHAPES:
        parts.append(gen_kernel(k, m))
        parts.append(gen_kernel(k, m, short=True))
        if diag and (k, m) == (64, 32):
            for v, probe in PROBES.items():
                parts.append(gen_kernel(k, m, probe=probe, suffix=f"_probe_{probe}"))
            for v, cfg in VARIANTS.items():
                parts.append(gen_kernel(k, m, suffix=f"_v{v}", cfg=cfg))
    for k, m in MDP_SHAPES:
        parts.append(gen_kernel(k, m, G=mdp_matrix(k, m), prefix="mdp_q4_enc"))
    parts.append("}  // namespace")
    parts.append("")
    if diag:
        parts.append("static int q4_variant()")
        parts.append("{")
        parts.append("    static const int v = [] { const char* e = std::getenv(\"NFEC_Q4_VARIANT\"); return e ? std::atoi(e) : 0; }();")
        parts.append("    return v;")
        parts.append("}")
        parts.append("")
    parts.append("// NFEC_ENOTSUP when no kernel covers (k, m) or the batch (tails, shortened blocks)")
    parts.append("int launch_rs8_q4_encode(uint32_t k, uint32_t m, const bs::EncArgs& a, hipStream_t s)")
    parts.append("{")
    for v, probe in (PROBES.items() if diag else ()):
        parts.append(f"    if (k == 64 && m == 32 && q4_variant() == {v}) return launch_rs8_q4_enc_probe_{probe}_k64_m32(a, s);")
    for v in (VARIANTS if diag else ()):
        parts.append(f"    if (k == 64 && m == 32 && q4_variant() == {v}) return launch_rs8_q4_enc_v{v}_k64_m32(a, s);")
    for k, m in SHAPES:
        parts.append(f"    if (k == {k} && m == {m}) return a.num_data ? launch_rs8_q4_enc_sh_k{k}_m{m}(a, s) : launch_rs8_q4_enc_k{k}_m{m}(a, s);")
    parts.append("    return NFEC_ENOTSUP;")
    parts.append("}")
    parts.append("")
    parts.append("int launch_mdp_q4_encode(uint32_t k, uint32_t m, const bs::EncArgs& a, hipStream_t s)")
    parts.append("{")
    for k, m in MDP_SHAPES:
        parts.append(f"    if (k == {k} && m == {m}) return launch_mdp_q4_enc_k{k}_m{m}(a, s);")
    parts.append("    return NFEC_ENOTSUP;")
    parts.append("}")
    parts.append("")
    parts.append("}  // namespace nfec")
    open(path, "w").write("\n".join(parts) + "\n")


if __name__ == "__main__":
    main()
