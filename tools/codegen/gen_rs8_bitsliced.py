#!/usr/bin/env python3
"""Generate norm_amd/csrc/gen_rs8_bitsliced.hip: bit-sliced RS8 encode kernels specialised
to the reference generator of fixed (k, m) shapes.

Why generate code: the encode matrix of NormEncoderRS8 (src/common/normEncoderRS8.cpp:400-462)
is a constant of (k, m).  Over GF(2) the map parity = G * data is a (8m x 8k) bit matrix; with
the data bit-sliced (bitslice.hpp) every parity bit-plane is an XOR of data bit-planes, i.e.
pure v_bitop3/v_xor work with the constants folded into the instruction stream -- no table
lookups and no v_perm (which gfx950 issues at half the rate of v_bitop3, measured in
profiles/r01/ubench_valu_rates.jsonl).  Per source column j the 8 data planes are combined
four at a time (method of four Russians): T_lo[a] = XOR of planes {b<4 : a_b}, T_hi likewise
(22 XORs), then each parity plane row (p, i) takes one 3-input XOR:
    acc[p][i] ^= T_lo[R & 15] ^ T_hi[R >> 4],   R = row i of the 8x8 matrix of G[p][j].
The code is straight-line (~100 KiB per role); measurements showed no instruction-cache
penalty for streams of that size.

Parity rows are split into roles of Cfg.rows rows; each role is one wavefront that keeps
rows x 8 plane accumulators in VGPRs (the register budget, hence the occupancy, is set by
the role size; see Cfg).

Usage: gen_rs8_bitsliced.py OUT.hip [k,m ...]
"""
import sys

POLY = 0x11D
DEFAULT_SHAPES = [(64, 32), (64, 16), (64, 8)]


class Cfg:
    """Code shape of one kernel build.
    rows: parity rows per role (one wavefront keeps rows x 8 plane accumulators)
    pf:   source columns in flight per wave (register prefetch ring)
    wpe:  occupancy target (waves per SIMD) handed to the register allocator, or None
    lazy: emit the plane updates grouped by low-table entry, so at most one low entry is
          live at a time (shorter live ranges; lets higher occupancy targets fit)"""

    def __init__(self, rows=16, pf=3, wpe=None, lazy=False, suffix="", probe=None):
        self.rows, self.pf, self.wpe, self.lazy, self.suffix = rows, pf, wpe, lazy, suffix
        # probe (A/B only, never the default): "noload" replaces the source loads with
        # synthetic registers (VALU-only time), "nocompute" keeps loads/stores but drops the
        # GF arithmetic (memory-only time)
        self.probe = probe


DEFAULT = Cfg(rows=16, pf=3, lazy=True)
DEC_DEFAULT = Cfg(rows=16, pf=3, lazy=False)
# extra (64,32) encode builds selectable with NFEC_BS_VARIANT=<id> for A/B runs
VARIANTS_64_32 = {
    2: Cfg(rows=12, pf=3, wpe=3, lazy=True, suffix="_v2"),
    3: Cfg(rows=8, pf=3, wpe=4, lazy=True, suffix="_v3"),
    4: Cfg(rows=16, pf=4, lazy=True, suffix="_v4"),
    8: Cfg(rows=16, pf=3, lazy=True, suffix="_probe_noload", probe="noload"),
    9: Cfg(rows=16, pf=3, lazy=True, suffix="_probe_nocompute", probe="nocompute"),
}


def gf_tables():
    exp = [0] * 510
    log = [0] * 256
    v = 1
    for i in range(255):
        exp[i] = v
        log[v] = i
        v <<= 1
        if v & 0x100:
            v ^= POLY
    for i in range(255, 510):
        exp[i] = exp[i - 255]
    log[0] = 255
    return exp, log


EXP, LOG = gf_tables()


def mul(a, b):
    return EXP[LOG[a] + LOG[b]] if a and b else 0


def inv(a):
    return EXP[255 - LOG[a]] if a > 1 else a


def point(row):
    return 0 if row == 0 else EXP[(row - 1) % 255]


def generator(k, m):
    """Parity rows (m x k) of the reference's systematic Rizzo generator, Lagrange form."""
    x = [point(j) for j in range(k)]
    G = []
    for p in range(m):
        y = point(k + p)
        row = []
        for j in range(k):
            num, den = 1, 1
            for l in range(k):
                if l != j:
                    num = mul(num, y ^ x[l])
                    den = mul(den, x[j] ^ x[l])
            row.append(mul(num, inv(den)))
        G.append(row)
    return G


def bitmatrix_rows(c):
    """R_i for i in 0..7: bit b of R_i = bit i of c * 2^b  ((c*x)_i = parity(R_i & x))."""
    cols = [mul(c, 1 << b) for b in range(8)]
    return [sum(((cols[b] >> i) & 1) << b for b in range(8)) for i in range(8)]


def table_expr(prefix, base, a):
    """Expression for the XOR of planes base+b over the set bits b of a (a in 1..15)."""
    bits = [b for b in range(4) if (a >> b) & 1]
    if len(bits) == 1:
        return f"w{base + bits[0]}"
    return f"{prefix}{a}"


def table_defs(prefix, base, needed):
    """Definitions of the multi-plane combinations actually used."""
    out = []
    for a in sorted(needed):
        bits = [b for b in range(4) if (a >> b) & 1]
        if len(bits) < 2:
            continue
        ws = [f"w{base + b}" for b in bits]
        if len(ws) == 2:
            out.append(f"const uint32_t {prefix}{a} = {ws[0]} ^ {ws[1]};")
        elif len(ws) == 3:
            out.append(f"const uint32_t {prefix}{a} = bs::x3({ws[0]}, {ws[1]}, {ws[2]});")
        else:
            out.append(f"const uint32_t {prefix}{a} = bs::x3({ws[0]}, {ws[1]}, {ws[2]}) ^ {ws[3]};")
    return out


def acc_update(acc, R):
    lo, hi = R & 15, R >> 4
    if lo and hi:
        return f"{acc} = bs::x3({acc}, {table_expr('L', 0, lo)}, {table_expr('H', 4, hi)});"
    if lo:
        return f"{acc} = bs::x2({acc}, {table_expr('L', 0, lo)});"
    if hi:
        return f"{acc} = bs::x2({acc}, {table_expr('H', 4, hi)});"
    return None


def col_loads(q, col, masked=False, probe=None):
    """Refill prefetch slot q with source column col (buffer loads: VGPR item offset + SGPR
    slot offset).  masked (decode): erased columns read as zeros (bs::dec_off)."""
    if probe == "noload":
        return "; ".join(f"n{q}_{i} = make_uint2(o{i} * 0x9E3779B1u ^ {col}u, (o{i} + {col}u) * 0x85EBCA6Bu)"
                         for i in range(4)) + ";"
    if masked:
        return "; ".join(f"n{q}_{i} = bs::bld8(it.rs, bs::dec_off<{col}>(o{i}, it.em0[{i}], it.em1[{i}]), {col}u * sstride)"
                         for i in range(4)) + ";"
    return "; ".join(f"n{q}_{i} = bs::bld8(it.rs, o{i}, {col}u * sstride)" for i in range(4)) + ";"


def prologue_loads(L, k, cfg, masked=False):
    L.append("    uint32_t w0, w1, w2, w3, w4, w5, w6, w7;")
    for r in range(cfg.pf):
        L.append(f"    uint2 n{r}_0, n{r}_1, n{r}_2, n{r}_3;")
    for r in range(min(cfg.pf, k)):
        L.append(f"    " + col_loads(r, r, masked, cfg.probe))


def column_body(L, G, k, r0, rows, j, masked, cfg):
    """Code for source column j: take it from the prefetch ring, refill the ring slot with
    column j+pf, (mask erased), transpose, M4RM update."""
    pf = cfg.pf
    L.append(f"    // ---- source column {j} ----")
    q = j % pf
    L.append(f"    w0 = n{q}_0.x; w1 = n{q}_0.y; w2 = n{q}_1.x; w3 = n{q}_1.y; w4 = n{q}_2.x; w5 = n{q}_2.y; "
             f"w6 = n{q}_3.x; w7 = n{q}_3.y;")
    if j + pf < k:
        L.append("    " + col_loads(q, j + pf, masked, cfg.probe))
    L.append("    __builtin_amdgcn_sched_barrier(0);")
    if cfg.probe == "nocompute":
        for i in range(8):
            L.append(f"    a0_{i} ^= w{i};")
        return
    L.append("    bs::transpose8(w0, w1, w2, w3, w4, w5, w6, w7);")
    mats = [bitmatrix_rows(G[r0 + r][j]) for r in range(rows)]
    outs = [(f"a{r}_{i}", mats[r][i]) for r in range(rows) for i in range(8)]
    need_lo = {R & 15 for _, R in outs if R & 15}
    need_hi = {R >> 4 for _, R in outs if R >> 4}
    L.append("    {")
    if not cfg.lazy:
        for d in table_defs("L", 0, need_lo) + table_defs("H", 4, need_hi):
            L.append("        " + d)
        for acc, R in outs:
            u = acc_update(acc, R)
            if u:
                L.append("        " + u)
    else:
        # high entries first (<= 11 multi-plane ones live), then one low entry at a time
        # together with all of its users
        for d in table_defs("H", 4, need_hi):
            L.append("        " + d)
        for acc, R in outs:
            if not R & 15 and R >> 4:
                L.append("        " + acc_update(acc, R))
        for lo in sorted(need_lo):
            L.append("        {")
            for d in table_defs("L", 0, {lo}):
                L.append("            " + d)
            for acc, R in outs:
                if R & 15 == lo:
                    L.append("            " + acc_update(acc, R))
            L.append("        }")
    L.append("    }")
    accs = [a for a, _ in outs]
    for c0 in range(0, len(accs), 16):
        grp = accs[c0:c0 + 16]
        L.append('    asm volatile("" : ' + ", ".join(f'"+v"({x})' for x in grp) + ' :: "memory");')


def kernel_attrs(cfg, threads=256):
    a = f"__launch_bounds__({threads}, 2)"
    if cfg.wpe:
        a += f" __attribute__((amdgpu_waves_per_eu({cfg.wpe}, {cfg.wpe})))"
    return a


def role_split(m, cfg):
    roles = (m + cfg.rows - 1) // cfg.rows
    return [(r * cfg.rows, min(cfg.rows, m - r * cfg.rows)) for r in range(roles)]


def gen_dec_role(k, m, role, r0, rows, cfg):
    """Decode stage 1 for parity rows [r0, r0+rows): z_t = parity_p ^ G[p][present] * data."""
    G = generator(k, m)
    L = []
    L.append(f"__device__ __forceinline__ void dec{cfg.suffix}_k{k}_m{m}_role{role}(const bs::DecArgs& a, "
             f"const bs::DecItems& it)")
    L.append("{")
    L.append("    const uint32_t sstride = a.seg_stride;")
    L.append("    const uint32_t o0 = it.off[0], o1 = it.off[1], o2 = it.off[2], o3 = it.off[3];")
    for r in range(rows):
        L.append("    uint32_t " + ", ".join(f"a{r}_{i} = 0" for i in range(8)) + ";")
    prologue_loads(L, k, cfg, masked=True)
    for j in range(k):
        column_body(L, G, k, r0, rows, j, True, cfg)
    L.append("    // ---- z_t = received parity p ^ re-encoded row p, for the rows P uses ----")
    L.append("    bs::DecTail tl;")
    L.append("    bs::make_dec_tail(a, it, tl);")
    L.append("    // t = rank of row p among the used rows (P is the first e surviving parity rows in")
    L.append("    // ascending order), so no table lookup; received parity is prefetched 4 rows ahead.")
    ahead = min(4, rows)
    # parity slot 0 of each item's block: numData (shortened blocks), else k
    L.append("    uint32_t " + ", ".join(f"p{i} = o{i} + (a.num_data ? (uint32_t)a.num_data[tl.blk[{i}]] : {k}u) * sstride"
                                       for i in range(4)) + ";")
    for r in range(ahead):
        p = r0 + r
        L.append(f"    uint2 " + ", ".join(f"q{r}_{i} = bs::bld8(it.rs, p{i}, {p}u * sstride)" for i in range(4)) + ";")
    for r in range(rows):
        p = r0 + r
        q = r % ahead
        L.append("    {")
        L.append(f"        const uint2 c0 = q{q}_0, c1 = q{q}_1, c2 = q{q}_2, c3 = q{q}_3;")
        if r + ahead < rows:
            pn = r0 + r + ahead
            L.append("        " + "; ".join(f"q{q}_{i} = bs::bld8(it.rs, p{i}, {pn}u * sstride)" for i in range(4)) + ";")
        L.append(f"        bs::transpose8(a{r}_0, a{r}_1, a{r}_2, a{r}_3, a{r}_4, a{r}_5, a{r}_6, a{r}_7);")
        for i in range(4):
            L.append(f"        if ((tl.sel[{i}] >> {p}) & 1u) {{")
            L.append(f"            const uint32_t t = __builtin_popcount(tl.sel[{i}] & 0x{(1 << p) - 1:08x}u);")
            L.append(f"            bs::st8(a.z + (uint64_t)tl.blk[{i}] * a.z_block_stride + (uint64_t)t * a.z_stride + tl.ib[{i}],")
            L.append(f"                    a{r}_{2 * i} ^ c{i}.x, a{r}_{2 * i + 1} ^ c{i}.y, tl.nbytes[{i}], 0u);")
            L.append("        }")
        L.append("    }")
    L.append("}")
    return "\n".join(L)


def gen_dec_kernel(k, m, cfg):
    split = role_split(m, cfg)
    out = [gen_dec_role(k, m, role, r0, rows, cfg) for role, (r0, rows) in enumerate(split)]
    groups = 4
    K = f"rs8_dec{cfg.suffix}_k{k}_m{m}"
    body = [f"__global__ {kernel_attrs(cfg)} void {K}(bs::DecArgs a)", "{"]
    # every block already repaired by the fused kernel: nothing to re-encode
    body.append("    if (a.gate && *a.gate != a.gate_gen) return;")
    body.append("    const uint32_t lane = threadIdx.x & 63;")
    body.append("    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);")
    body.append(f"    const uint64_t group = (uint64_t)bs::wg_index(a.xcd_remap) * {groups} + wave;")
    body.append("    bs::DecItems it;")
    body.append("    bs::make_dec_items(a, (uint32_t)group * 256u, lane, it);")
    body.append("    const uint32_t need = it.need;")
    for role, (r0, rows) in enumerate(split):
        rmask = ((1 << rows) - 1) << r0
        # every wave handles all roles its blocks need (usually only the first ones: P is
        # the first e surviving parity rows); unused roles cost nothing
        body.append(f"    if (__any(need & 0x{rmask:08x}u)) dec{cfg.suffix}_k{k}_m{m}_role{role}(a, it);")
    body.append("}")
    out.append("\n".join(body))
    out.append(f"""
static int launch_{K}(const bs::DecArgs& a, hipStream_t s)
{{
    const uint64_t items = (uint64_t)a.nblocks * ((a.vec + 7) / 8);
    if (items >= (1ull << 31) || !bs::offsets_fit(a.block_stride, a.seg_stride)) return NFEC_ENOTSUP;
    const uint64_t groups = (items + 255) / 256;
    const uint64_t wgs = (groups + {groups} - 1) / {groups};
    hipLaunchKernelGGL({K}, dim3((uint32_t)wgs), dim3(256), 0, s, a);
    return hipGetLastError() == hipSuccess ? NFEC_OK : NFEC_EDEVICE;
}}""")
    return "\n\n".join(out)


def gen_role(k, m, role, r0, rows, cfg):
    """Device function computing parity rows [r0, r0+rows) of one lane's 4 items."""
    G = generator(k, m)
    L = []
    L.append(f"__device__ __forceinline__ void enc{cfg.suffix}_k{k}_m{m}_role{role}(const bs::EncArgs& a, "
             f"const bs::Items& it)")
    L.append("{")
    L.append("    const uint32_t sstride = a.seg_stride;")
    L.append("    const uint32_t o0 = it.off[0], o1 = it.off[1], o2 = it.off[2], o3 = it.off[3];")
    for r in range(rows):
        L.append("    uint32_t " + ", ".join(f"a{r}_{i} = 0" for i in range(8)) + ";")
    prologue_loads(L, k, cfg)
    for j in range(k):
        column_body(L, G, k, r0, rows, j, False, cfg)
    L.append("    // ---- parity planes back to bytes, store ----")
    for r in range(rows):
        p = r0 + r
        L.append(f"    bs::transpose8(a{r}_0, a{r}_1, a{r}_2, a{r}_3, a{r}_4, a{r}_5, a{r}_6, a{r}_7);")
        for i in range(4):
            L.append(f"    bs::bst8(it, o{i}, {k + p}u * sstride, a{r}_{2 * i}, a{r}_{2 * i + 1}, "
                     f"it.nbytes[{i}], a.accumulate, a.nt_store);")
    L.append("}")
    return "\n".join(L)


def gen_kernel(k, m, cfg):
    """One workgroup = `groups` item groups x `roles` role-waves (<= 4 waves)."""
    split = role_split(m, cfg)
    roles = len(split)
    groups = max(1, 4 // roles)
    threads = 64 * roles * groups
    out = [gen_role(k, m, role, r0, rows, cfg) for role, (r0, rows) in enumerate(split)]
    K = f"rs8_enc{cfg.suffix}_k{k}_m{m}"
    body = [f"__global__ {kernel_attrs(cfg, threads)} void {K}(bs::EncArgs a)", "{"]
    body.append("    const uint32_t lane = threadIdx.x & 63;")
    body.append("    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);")
    body.append(f"    const uint32_t role = wave % {roles};")
    body.append(f"    const uint64_t group = (uint64_t)bs::wg_index(a.xcd_remap) * {groups} + wave / {roles};")
    body.append("    bs::Items it;")
    body.append("    bs::make_items(a, (uint32_t)group * 256u, lane, it);")
    for role in range(roles):
        kw = "if" if role == 0 else "else if"
        body.append(f"    {kw} (role == {role}) enc{cfg.suffix}_k{k}_m{m}_role{role}(a, it);")
    body.append("}")
    out.append("\n".join(body))
    out.append(f"""
static int launch_{K}(const bs::EncArgs& a, hipStream_t s)
{{
    const uint64_t items = (uint64_t)a.nblocks * ((a.vec + 7) / 8);
    // shortened batches, huge batches or strides beyond 32-bit buffer offsets: generic kernel
    if (a.num_data || items >= (1ull << 31) || !bs::offsets_fit(a.block_stride, a.seg_stride)) return NFEC_ENOTSUP;
    const uint64_t groups = (items + 255) / 256;
    const uint64_t wgs = (groups + {groups} - 1) / {groups};
    hipLaunchKernelGGL({K}, dim3((uint32_t)wgs), dim3({threads}), 0, s, a);
    return hipGetLastError() == hipSuccess ? NFEC_OK : NFEC_EDEVICE;
}}""")
    return "\n\n".join(out)


def main():
    # --diag: also emit the (64, 32) A/B builds and probes and their NFEC_BS_VARIANT switch (the
    # diagnostic library, make -C norm_amd diag); the product library ships the defaults only
    diag = "--diag" in sys.argv
    argv = [a for a in sys.argv if a != "--diag"]
    path = argv[1]
    shapes = DEFAULT_SHAPES
    if len(argv) > 2:
        shapes = [tuple(int(v) for v in s.split(",")) for s in argv[2:]]
    parts = [
        "// GENERATED by tools/codegen/gen_rs8_bitsliced.py -- do not edit by hand.",
        "// Bit-sliced RS8 encode / decode-stage-1 kernels specialised to the reference generator",
        "// of each (k, m): " + ", ".join(f"({k},{m})" for k, m in shapes),
        '#include <cstdlib>',
        '#include "bitslice.hpp"',
        "",
        "namespace nfec {",
        "namespace {",
    ]
    extra = {}
    for k, m in shapes:
        parts.append(gen_kernel(k, m, DEFAULT))
        if m <= 32:
            parts.append(gen_dec_kernel(k, m, DEC_DEFAULT))
        if diag and (k, m) == (64, 32):
            extra[(k, m)] = VARIANTS_64_32
            for v, cfg in VARIANTS_64_32.items():
                parts.append(gen_kernel(k, m, cfg))
    parts.append("}  // namespace")
    parts.append("")
    if diag:
        parts.append("static int bs_variant()")
        parts.append("{")
        parts.append("    static const int v = [] { const char* e = std::getenv(\"NFEC_BS_VARIANT\"); return e ? std::atoi(e) : 0; }();")
        parts.append("    return v;")
        parts.append("}")
        parts.append("")
    parts.append("// Returns NFEC_ENOTSUP when no specialised kernel exists for (k, m).")
    parts.append("int launch_rs8_bitsliced_encode(uint32_t k, uint32_t m, const bs::EncArgs& a, hipStream_t s)")
    parts.append("{")
    for k, m in shapes:
        for v, cfg in extra.get((k, m), {}).items():
            parts.append(f"    if (k == {k} && m == {m} && bs_variant() == {v}) return launch_rs8_enc{cfg.suffix}_k{k}_m{m}(a, s);")
        parts.append(f"    if (k == {k} && m == {m}) return launch_rs8_enc_k{k}_m{m}(a, s);")
    parts.append("    return NFEC_ENOTSUP;")
    parts.append("}")
    parts.append("")
    parts.append("int launch_rs8_bitsliced_reencode(uint32_t k, uint32_t m, const bs::DecArgs& a, hipStream_t s)")
    parts.append("{")
    for k, m in shapes:
        if m <= 32:
            parts.append(f"    if (k == {k} && m == {m}) return launch_rs8_dec_k{k}_m{m}(a, s);")
    parts.append("    return NFEC_ENOTSUP;")
    parts.append("}")
    parts.append("")
    parts.append("// generator parity rows compiled into the kernels (checked against the host build in tests)")
    parts.append("int bitsliced_encode_generator(uint32_t k, uint32_t m, uint8_t* out)")
    parts.append("{")
    for k, m in shapes:
        G = generator(k, m)
        flat = ",".join(str(v) for row in G for v in row)
        parts.append(f"    if (k == {k} && m == {m}) {{ static const uint8_t g[] = {{{flat}}};")
        parts.append(f"        for (uint32_t i = 0; i < {k * m}; ++i) out[i] = g[i]; return NFEC_OK; }}")
    parts.append("    return NFEC_ENOTSUP;")
    parts.append("}")
    parts.append("")
    parts.append("}  // namespace nfec")
    open(path, "w").write("\n".join(parts) + "\n")


if __name__ == "__main__":
    main()
