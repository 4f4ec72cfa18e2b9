"""CPU checks of the tower-field RS16 kernel's generator (tools/codegen/gen_gf16_tw.py).

The kernel's arithmetic is straight-line VALU code emitted by the generator: the bit transpose,
the XOR networks of phi and phi^-1, the four-Russians combinations and the 256 GF(2^8)
snippets.  These tests run those exact instruction lists on a small interpreter of the few
VALU opcodes they use (one 32-bit lane; 32 symbols in bit-sliced form) and compare the result
with GF(2^16) products computed the reference's way (polynomial 0x1100B,
src/common/normEncoderRS16.cpp).  What they cannot see (the jumps, M0 indexing, loads and
stores) is covered by the GPU parity tests."""
import os
import random
import re
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools", "codegen"))
import gen_gf16_tw as g  # noqa: E402

M32 = 0xFFFFFFFF


class Lane:
    """one lane of the VALU ops the generator emits; `idx` plays gpr-index mode (SRC0, DST)"""

    def __init__(self):
        self.v = [0] * 256
        self.s = {}

    def val(self, tok, idx=0):
        tok = tok.strip()
        if tok.startswith("v"):
            return self.v[int(tok[1:]) + idx]
        if tok.startswith("s"):
            return self.s[int(tok[1:])]
        return int(tok, 0)

    def run(self, ops, idx=0):
        for op in ops:
            m = re.match(r"(\S+)\s+(.*)", op)
            name, rest = m.group(1), m.group(2)
            if name == "s_mov_b32":
                d, x = rest.split(",")
                self.s[int(d.strip()[1:])] = int(x, 0)
                continue
            tt = None
            if "bitop3:" in rest:
                rest, t = rest.split("bitop3:")
                tt = int(t, 0)
            a = [x.strip() for x in rest.split(",")]
            d = int(a[0][1:]) + idx
            if name == "v_mov_b32":
                r = self.val(a[1])
            elif name == "v_xor_b32":
                r = self.val(a[1], idx) ^ self.val(a[2])
            elif name == "v_lshrrev_b32":
                r = self.val(a[2]) >> int(a[1])
            elif name == "v_lshlrev_b32":
                r = (self.val(a[2]) << int(a[1])) & M32
            elif name == "v_bitop3_b32":
                x, y, z = self.val(a[1], idx), self.val(a[2]), self.val(a[3])
                r = 0
                for bit in range(32):
                    i = (((x >> bit) & 1) << 2) | (((y >> bit) & 1) << 1) | ((z >> bit) & 1)
                    r |= ((tt >> i) & 1) << bit
            else:
                raise AssertionError(f"interpreter lacks {name}")
            self.v[d] = r


def test_tower_is_a_field_isomorphism():
    rnd = random.Random(1)
    # beta is a root of the reference polynomial in the tower field
    acc, p = 0, 1
    for i in range(17):
        if (g.P16 >> i) & 1:
            acc ^= p
        p = g.tw_mul(p, g.BETA, g.LAM)
    assert acc == 0
    assert g.gf8_trace(g.LAM) == 1   # y^2 + y + lam irreducible over GF(2^8)
    for _ in range(2000):
        a, b = rnd.randrange(1 << 16), rnd.randrange(1 << 16)
        assert g.phi(g.gf16_mul(a, b)) == g.tw_mul(g.phi(a), g.phi(b), g.LAM)
        assert g.phi(g.phi(a), g.PHI_INV) == a


def test_table_entries_give_the_product():
    rnd = random.Random(2)
    for _ in range(2000):
        c, x = rnd.randrange(1 << 16), rnd.randrange(1 << 16)
        e = [v >> g.SNIP_ALIGN for v in g.table_entries(c)]
        t = g.phi(x)
        x0, x1 = t & 255, t >> 8
        out0 = g.gf8_mul(e[0], x0) ^ g.gf8_mul(e[2], x1)
        out1 = g.gf8_mul(e[1], x0) ^ g.gf8_mul(e[3], x1)
        assert out0 | (out1 << 8) == g.phi(g.gf16_mul(c, x))


def _load(lane, syms):
    """32 symbols of one lane as the 8 pieces land in the slot: dword j = symbols 2j, 2j+1"""
    for j in range(16):
        lane.v[g.V_SLOT + j] = syms[2 * j] | (syms[2 * j + 1] << 16)


def _store(lane):
    out = []
    for j in range(16):
        d = lane.v[g.V_SLOT + j]
        out += [d & 0xFFFF, d >> 16]
    return out


@pytest.mark.parametrize("k,rows,seed,prefetch", [(1, 1, 3, True), (3, 11, 4, True), (5, 4, 5, True),
                                                  (5, 7, 6, False)])
def test_column_flow_matches_gf16_products(k, rows, seed, prefetch):
    """the kernel's per-column sequence (transpose, phi, [x1 planes through the LDS exchange],
    combos, row snippets on x0, x1 -> W, combos, row snippets) and its epilogue (phi^-1,
    transpose), row targets by index; both register layouts"""
    g.set_prefetch(prefetch)
    try:
        _column_flow(k, rows, seed)
    finally:
        g.set_prefetch(True)


def _column_flow(k, rows, seed):
    rnd = random.Random(seed)
    data = [[rnd.randrange(1 << 16) for _ in range(32)] for _ in range(k)]
    data[0][:4] = [0, 1, 0xFFFF, 0x8000]
    G = [[rnd.randrange(1 << 16) for _ in range(k)] for _ in range(rows)]
    if rows > 1:
        G[1][0] = 0
    lane = Lane()
    lane.run(g.mask_init())
    snip = {c: g.snippet_body(c) for c in range(256)}
    for c in range(k):
        _load(lane, data[c])
        lane.run(g.transpose16(g.slot(), g.V_TMP))
        lane.run(g.phi_code())
        x1 = [lane.v[r] for r in g.x1_regs()]   # (written to the exchange before the combinations)
        lane.run(g.combos_code())
        for r in range(rows):
            e = [v >> g.SNIP_ALIGN for v in g.table_entries(G[r][c])]
            lane.run(snip[e[0]], idx=16 * r)
            lane.run(snip[e[1]], idx=16 * r + 8)
        for i in range(8):
            lane.v[g.V_W + i] = x1[i]
        lane.run(g.combos_code())
        for r in range(rows):
            e = [v >> g.SNIP_ALIGN for v in g.table_entries(G[r][c])]
            lane.run(snip[e[2]], idx=16 * r)
            lane.run(snip[e[3]], idx=16 * r + 8)
    for r in range(rows):
        lane.run(g.phi_inv_code(r))
        lane.run(g.transpose16(g.slot(), g.V_TMP))
        got = _store(lane)
        want = [0] * 32
        for c in range(k):
            for s in range(32):
                want[s] ^= g.gf16_mul(G[r][c], data[c][s])
        assert got == want, f"row {r}"


def test_snippets_fit_their_slots():
    """each snippet (8 VALU at most + the return) fits its 128-byte slot, so the table offset
    of coefficient c is c << 7"""
    for c in range(256):
        body = g.snippet_body(c)
        assert len(body) <= 8
        size = sum(8 if op.startswith("v_bitop3") else 4 for op in body) + 4
        assert size <= 1 << g.SNIP_ALIGN


@pytest.mark.parametrize("rows,prefetch", [(6, True), (7, False), (6, False), (4, True), (11, True)])
def test_register_map_is_disjoint(rows, prefetch):
    """the VGPR regions of each layout are disjoint, above the asm's inputs (v0..v3), with the
    pairs of loads, stores and LDS reads at even registers and the occupancy the layout is for"""
    try:
        g.set_prefetch(prefetch)
        g.set_rows(rows)
        regions = [range(g.V_SLOT, g.V_SLOT + 16), range(g.V_W, g.V_W + 8),
                   range(g.V_CA, g.V_CA + 11), range(g.V_CB, g.V_CB + 11), g.V_TMP,
                   range(g.ACC0, g.V_LAST + 1)]
        if prefetch:
            regions.append(range(g.V_S, g.V_S + 8))
        seen = set()
        for r in regions:
            for v in r:
                assert v not in seen and 4 <= v <= 255
                seen.add(v)
        assert g.V_SLOT % 2 == 0 and g.V_W % 2 == 0 and g.V_CA % 2 == 0 and (g.V_CB + 1) % 2 == 0
        assert g.V_X1 % 2 == 0 and (not prefetch or g.V_S % 2 == 0)
        if rows == 7 or rows == 6:
            assert g.V_LAST < 168   # three waves per SIMD
        if rows == 4:
            assert g.V_LAST < 128   # four
    finally:
        g.set_prefetch(True)
        g.set_rows(6)


@pytest.mark.parametrize("m", [1, 4, 11, 12, 44, 45, 50, 100, 128, 200, 256])
def test_pass_partition(m):
    """rows spread evenly over whole workgroups of NWAVES passes, at most ROWS rows per pass,
    every row in exactly one pass (the kernel's row0/nr and gf16_tw_offsets use the same split)"""
    P = g.n_passes(m)
    assert P % g.NWAVES == 0 and P >= g.NWAVES
    rows = []
    for p in range(P):
        lo, hi = g.pass_rows(m, P, p)
        assert 0 <= hi - lo <= g.ROWS
        rows += range(lo, hi)
    assert rows == list(range(m))


def test_entry_registers():
    """a pass's entries: sweep 0 in the first 12 entry dwords, sweep 1 in the next 12 (so one
    half loads while the other sweep reads), 16-bit halves j; matches gf16_tw_offsets'
    2 r + j / 24 + 2 r + j layout"""
    seen = set()
    for n in (0, 1):
        for r in range(g.ROWS):
            for j in (0, 1):
                dw, half = g.entry(n, r, j)
                e = 2 * (dw - g.S_OFF) + half
                assert e == 24 * n + 2 * r + j
                assert g.S_OFF + 12 * n <= dw < g.S_OFF + 12 * n + 12
                seen.add(e)
    assert len(seen) == 4 * g.ROWS


def test_column_map_division_is_exact():
    """The column map's division (col_offset): q = mulhi(c, ceil(2^32 / d)), remainder c - q d,
    as the generated launcher sets col_magic (d >= 2; d = 1 and the identity use magic 0).
    Exact for every column c < 2^16 and chunk width d < 2^16 (tw_prepare rejects larger)."""
    import numpy as np

    c = np.arange(1 << 16, dtype=np.uint64)
    widths = list(range(2, 1025)) + [3 << 10, 25 << 8, 65535]
    for d in widths:
        magic = ((1 << 32) - 1 + d) // d
        assert magic < (1 << 32)
        q = (c * np.uint64(magic)) >> np.uint64(32)
        assert np.array_equal(q, c // np.uint64(d)), d
    src = g.col_offset()
    assert src[0].startswith("s_mul_hi_u32") and "%[cmg]" in src[0]
