#!/usr/bin/env python3
"""Generate norm_amd/csrc/gen_rs8_asm.hip: bit-sliced RS8 encode kernels whose role bodies are
hand-scheduled gfx950 assembly with explicit VGPR assignment.

Same algorithm as gen_rs8_bitsliced.py (8x8 bit transpose per source column, method of four
Russians over the fixed generator of NormEncoderRS8, src/common/normEncoderRS8.cpp:400-462,
one v_bitop3 per parity bit-plane and column), but the register file is laid out by hand:

  * VGPR bank = index mod 4.  A VOP3 whose VGPR operands share a bank stalls
    (profiles/r01/ubench_icache.jsonl: 3 distinct banks run 15 % faster than random
    operands).  The 128 parity-plane accumulators live in banks 2 and 3, the source planes
    of M4RM group A (planes 0,2,4,6) and all their combinations in bank 0, group B
    (planes 1,3,5,7) in bank 1, so every update  acc ^= A[a] ^ B[b]  reads three banks.
  * The prefetch ring holds NSLOT source columns in flight per wave (no VGPR budget
    left to the compiler's allocator, no spills), with counted vmcnt waits.
  * A buffer_load_dwordx2 lands item q's two dwords in the aligned pair (4P, 4P+1): dword
    2q in bank 0 and 2q+1 in bank 1; the in-place transpose then leaves plane b in the
    register of dword b, i.e. the even planes in bank 0 and the odd planes in bank 1 --
    which is why the M4RM groups are the even and the odd planes.

The C++ wrapper computes the lane's item offsets (bitslice.hpp make_items) and hands them to
one asm statement per role; everything inside is straight-line.  Only batches whose segment
length is a multiple of 8 bytes use these kernels (tails and shortened batches fall back).

Usage: gen_rs8_asm.py OUT.hip [k,m ...]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gen_rs8_bitsliced import EXP, bitmatrix_rows, generator, mul  # noqa: E402

DEFAULT_SHAPES = [(64, 32), (64, 16), (64, 8)]
MDP_SHAPES = [(64, 32), (64, 16)]
ROWS = 16            # parity rows per role (one wavefront)
# A/B probes for (64, 32), NFEC_ASM_VARIANT=<id>: VALU only (no source loads) / memory only
# (measured and dropped: nt loads 2.42 ms / nt stores 2.42 / one role loading for both 1.91 in the
# memory-only probe -- none beat the default policy)
PROBES = {8: ("noload", "_probe_noload"), 9: ("nocompute", "_probe_nocompute"),
          10: ("nocompute,nostore", "_probe_readonly"), 11: ("nocompute,noload", "_probe_writeonly")}
# (measured and dropped: "halftr", transposing only every other column -- the upper bound of
# sharing the transposes of the two role waves through LDS -- 2.27 -> 2.12 ms before any LDS or
# barrier cost)

# ---- register map ----
IN_REGS = [0, 1, 4, 5, 8, 9, 12, 13]         # left to the compiler for the asm inputs
TEMP = {0: [16, 20, 24, 28], 1: [17, 21, 25, 29]}   # transpose temporaries by bank
COMBO_P0 = 8                                   # combos: pairs 8..18 (A at 4P, B at 4P+1)
RING_P0 = 19
NSLOT = 11                                     # ring pairs 19..62
S_LRS, S_SRS = 64, 68                          # load / store buffer descriptors s[64:67], s[68:71]
S_MASK = 72                                    # s72..s77 transpose masks
S_COL, S_ROW = 78, 79
MASKS = [0x0F0F0F0F, 0xF0F0F0F0, 0x33333333, 0xCCCCCCCC, 0x55555555, 0xAAAAAAAA]
MULTI = [a for a in range(1, 16) if bin(a).count("1") >= 2]   # 11 combination indices


def acc_reg(r, i):
    return 4 * (4 * r + i // 2) + 2 + (i & 1)


def slot_regs(s):
    """w[d], d = 0..7, of ring slot s."""
    w = []
    for q in range(4):
        p = RING_P0 + 4 * s + q
        w += [4 * p, 4 * p + 1]
    return w


def combo_reg(group, a):
    return 4 * (COMBO_P0 + MULTI.index(a)) + group


def bank(v):
    return v % 4


def transpose(w, temps):
    """8x8 bit transpose of the byte columns of w[0..7] in place (bitslice.hpp transpose8).
    temps(bank_to_avoid) -> iterator of free temporaries not in that bank."""
    out = []
    for S, (mlo, mhi), pairs in ((4, (0, 1), [(0, 4), (1, 5), (2, 6), (3, 7)]),
                                 (2, (2, 3), [(0, 2), (1, 3), (4, 6), (5, 7)]),
                                 (1, (4, 5), [(0, 1), (2, 3), (4, 5), (6, 7)])):
        shifts, sels = [], []
        pool = temps()
        for lo, hi in pairs:
            L, H = w[lo], w[hi]
            tu = pool(bank(H))
            tv = pool(bank(L))
            shifts.append(f"v_lshrrev_b32 v{tu}, {S}, v{L}")
            shifts.append(f"v_lshlrev_b32 v{tv}, {S}, v{H}")
            sels.append(f"v_bitop3_b32 v{H}, s{S_MASK + mlo}, v{tu}, v{H} bitop3:0xca")
            sels.append(f"v_bitop3_b32 v{L}, s{S_MASK + mhi}, v{tv}, v{L} bitop3:0xca")
        out += shifts + sels
    return out


def ring_temps():
    """temporaries for a ring-slot transpose: four per bank 0/1, handed out per stage"""
    def make():
        avail = {0: list(TEMP[0]), 1: list(TEMP[1])}

        def pick(avoid):
            b = 1 if avoid == 0 else 0
            return avail[b].pop(0)
        return pick
    return make


def epi_temps():
    """temporaries for an accumulator transpose (acc in banks 2/3): ring registers are free"""
    def make():
        free = [r for s in range(NSLOT) for r in slot_regs(s)]

        def pick(avoid):
            for i, r in enumerate(free):
                if bank(r) != avoid:
                    return free.pop(i)
            raise RuntimeError("no temp")
        return pick
    return make


def table_code(w, need):
    """Combination entries needed this column.  Group A = planes (0,2,4,6) = w[0,2,4,6]
    (bank 0), group B = planes (1,3,5,7) = w[1,3,5,7] (bank 1)."""
    code = []
    for g in (0, 1):
        single = [w[2 * t + g] for t in range(4)]
        built = {1 << t: single[t] for t in range(4)}
        # closure: to build a we use a minus its top bit when that is available
        todo = sorted({a for a in need[g] if a in MULTI}, key=lambda a: bin(a).count("1"))
        for a in todo:
            dst = combo_reg(g, a)
            top = a.bit_length() - 1
            rest = a & ~(1 << top)
            if rest in built:
                code.append(f"v_xor_b32 v{dst}, v{built[rest]}, v{single[top]}")
            else:
                bits = [t for t in range(4) if (a >> t) & 1]
                if len(bits) == 3:
                    code.append(f"v_bitop3_b32 v{dst}, v{single[bits[0]]}, v{single[bits[1]]}, v{single[bits[2]]} bitop3:0x96")
                else:  # 4 bits, no 3-subset built
                    code.append(f"v_bitop3_b32 v{dst}, v{single[bits[0]]}, v{single[bits[1]]}, v{single[bits[2]]} bitop3:0x96")
                    code.append(f"v_xor_b32 v{dst}, v{dst}, v{single[bits[3]]}")
            built[a] = dst
        need[g] = built
    return code


def split(R):
    a = sum(((R >> (2 * t)) & 1) << t for t in range(4))
    b = sum(((R >> (2 * t + 1)) & 1) << t for t in range(4))
    return a, b


def role_asm(G, k, m, r0, rows, probe=None):
    flags = set(probe.split(",")) if probe else set()
    noload = "noload" in flags or ("r0load" in flags and r0 > 0)
    nocompute = "nocompute" in flags
    lpol = " nt" if "ntload" in flags else ""
    spol = " nt" if "ntstore" in flags else ""
    L = []
    # descriptors and masks
    L.append(f"s_mov_b64 s[{S_LRS}:{S_LRS + 1}], %[ib]")
    L.append(f"s_mov_b32 s{S_LRS + 2}, -1")
    L.append(f"s_mov_b32 s{S_LRS + 3}, 0x00020000")
    L.append(f"s_mov_b64 s[{S_SRS}:{S_SRS + 1}], %[ob]")
    L.append(f"s_mov_b32 s{S_SRS + 2}, 0x80000000")
    L.append(f"s_mov_b32 s{S_SRS + 3}, 0x00020000")
    for i, mk in enumerate(MASKS):
        L.append(f"s_mov_b32 s{S_MASK + i}, 0x{mk:08x}")
    offs = ["%[o0]", "%[o1]", "%[o2]", "%[o3]"]
    soffs = ["%[s0]", "%[s1]", "%[s2]", "%[s3]"]

    def loads(col):
        if noload:
            return []
        s = col % NSLOT
        w = slot_regs(s)
        out = [f"s_mul_i32 s{S_COL}, %[ss], {col}"]
        for q in range(4):
            out.append(f"buffer_load_dwordx2 v[{w[2 * q]}:{w[2 * q + 1]}], {offs[q]}, s[{S_LRS}:{S_LRS + 3}], s{S_COL} offen{lpol}")
        return out

    issued = -1
    for col in range(min(NSLOT, k)):
        L += loads(col)
        issued = col
    mk_ring = ring_temps()
    for j in range(k):
        w = slot_regs(j % NSLOT)
        if not noload:
            L.append(f"s_waitcnt vmcnt({4 * (issued - j)})")
        if nocompute:
            for i in range(8):
                L.append(f"v_xor_b32 v{acc_reg(0, i)}, v{w[i]}, v{acc_reg(0, i)}")
            if j + NSLOT < k:
                L += loads(j + NSLOT)
                issued = j + NSLOT
            continue
        if not ("halftr" in flags and j % 2 == 1):  # probe: upper bound of sharing transposes
            L += transpose(w, mk_ring)
        mats = [bitmatrix_rows(G[r0 + r][j]) for r in range(rows)]
        ups = []
        need = [set(), set()]
        for r in range(rows):
            for i in range(8):
                a, b = split(mats[r][i])
                ups.append((acc_reg(r, i), a, b))
                if a:
                    need[0].add(a)
                if b:
                    need[1].add(b)
        L += table_code(w, need)
        A, B = need
        for acc, a, b in ups:
            if j == 0:  # first column initialises the accumulators
                if a and b:
                    L.append(f"v_xor_b32 v{acc}, v{A[a]}, v{B[b]}")
                elif a or b:
                    L.append(f"v_mov_b32 v{acc}, v{A[a] if a else B[b]}")
                else:
                    L.append(f"v_mov_b32 v{acc}, 0")
            elif a and b:
                L.append(f"v_bitop3_b32 v{acc}, v{acc}, v{A[a]}, v{B[b]} bitop3:0x96")
            elif a:
                L.append(f"v_xor_b32 v{acc}, v{A[a]}, v{acc}")
            elif b:
                L.append(f"v_xor_b32 v{acc}, v{B[b]}, v{acc}")
        if j + NSLOT < k:
            L += loads(j + NSLOT)
            issued = j + NSLOT
    # epilogue: planes back to bytes, optional accumulate, store
    mk_epi = epi_temps()
    for r in range(rows):
        w = [acc_reg(r, i) for i in range(8)]
        L += transpose(w, mk_epi)
        L.append(f"s_mul_i32 s{S_ROW}, %[ss], {k + r0 + r}")
        tmp = slot_regs(0)
        L.append("s_cmp_eq_u32 %[acc], 0")
        L.append(f"s_cbranch_scc1 Lnoacc_{r}_%=")
        for q in range(4):
            L.append(f"buffer_load_dwordx2 v[{tmp[2 * q]}:{tmp[2 * q + 1]}], {soffs[q]}, s[{S_SRS}:{S_SRS + 3}], s{S_ROW} offen")
        L.append("s_waitcnt vmcnt(0)")
        for q in range(4):
            L.append(f"v_xor_b32 v{w[2 * q]}, v{tmp[2 * q]}, v{w[2 * q]}")
            L.append(f"v_xor_b32 v{w[2 * q + 1]}, v{tmp[2 * q + 1]}, v{w[2 * q + 1]}")
        L.append(f"Lnoacc_{r}_%=:")
        for q in range(4):
            if "nostore" not in flags:
                L.append(f"buffer_store_dwordx2 v[{w[2 * q]}:{w[2 * q + 1]}], {soffs[q]}, s[{S_SRS}:{S_SRS + 3}], s{S_ROW} offen{spol}")
    return L


def clobbers():
    v = [f'"v{i}"' for i in range(256) if i not in IN_REGS]
    s = [f'"s{i}"' for i in range(S_LRS, S_ROW + 1)]
    return ", ".join(v + s + ['"scc"', '"memory"'])


def mdp_matrix(k, m):
    """m x k block map of the MDP LFSR encoder for a full block of k source symbols: the same
    linear map as norm_amd/csrc/gf_host.cpp mdp_encode_matrix (reference
    normEncoderMDP.cpp:102-170 generator polynomial, :178-211 in-order Encode steps)."""
    g = [1] + [0] * m
    for n in range(1, m + 1):
        a = EXP[n]
        for i in range(n, 0, -1):
            g[i] = g[i - 1] ^ mul(g[i], a)
        g[0] = mul(g[0], a)
    st = [0] * m

    def step(d):
        fb = d ^ st[0]
        st[:] = [st[i + 1] ^ mul(g[m - 1 - i], fb) for i in range(m - 1)] + [mul(g[0], fb)]

    out = [[0] * k for _ in range(m)]
    step(1)
    for j in range(k - 1, -1, -1):
        for i in range(m):
            out[i][j] = st[i]
        if j:
            step(0)
    return out


def gen_kernel(k, m, probe=None, suffix="", G=None, prefix="rs8_asm_enc"):
    G = G if G is not None else generator(k, m)
    roles = [(r0, min(ROWS, m - r0)) for r0 in range(0, m, ROWS)]
    nroles = len(roles)
    groups = max(1, 4 // nroles)
    threads = 64 * nroles * groups
    K = f"{prefix}{suffix}_k{k}_m{m}"
    out = []
    for ri, (r0, rows) in enumerate(roles):
        body = role_asm(G, k, m, r0, rows, probe)
        s = "\\n\"\n        \"".join(body)
        out.append(f"""__device__ __forceinline__ void {K}_role{ri}(const bs::EncArgs& a, const bs::Items& it, const uint32_t so[4])
{{
    asm volatile(
        "{s}\\n"
        :
        : [ib] "s"(it.wbase), [ob] "s"(it.obase), [ss] "s"(a.seg_stride), [acc] "s"(a.accumulate),
          [o0] "v"(it.off[0]), [o1] "v"(it.off[1]), [o2] "v"(it.off[2]), [o3] "v"(it.off[3]),
          [s0] "v"(so[0]), [s1] "v"(so[1]), [s2] "v"(so[2]), [s3] "v"(so[3])
        : {clobbers()});
}}""")
    body = [f"__global__ __launch_bounds__({threads}, 2) void {K}(bs::EncArgs a)", "{"]
    body.append("    const uint32_t lane = threadIdx.x & 63;")
    body.append("    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);")
    body.append(f"    const uint32_t role = wave % {nroles};")
    body.append(f"    const uint64_t group = (uint64_t)bs::wg_index(a.xcd_remap) * {groups} + wave / {nroles};")
    body.append("    bs::Items it;")
    body.append("    bs::make_items(a, (uint32_t)group * 256u, lane, it);")
    body.append("    uint32_t so[4];")
    body.append("    // stores of out-of-range items land past the store descriptor's 2^31 records")
    body.append("#pragma unroll")
    body.append("    for (int i = 0; i < 4; ++i) so[i] = it.nbytes[i] == 8 ? it.off[i] : 0x80000000u;")
    for ri in range(nroles):
        kw = "if" if ri == 0 else "else if"
        body.append(f"    {kw} (role == {ri}) {K}_role{ri}(a, it, so);")
    body.append("}")
    out.append("\n".join(body))
    out.append(f"""
static int launch_{K}(const bs::EncArgs& a, hipStream_t s)
{{
    const uint64_t items = (uint64_t)a.nblocks * ((a.vec + 7) / 8);
    if (a.num_data || (a.vec & 7u) || a.nt_store || items >= (1ull << 31) ||
        !bs::offsets_fit(a.block_stride, a.seg_stride))
        return NFEC_ENOTSUP;
    const uint64_t groups = (items + 255) / 256;
    const uint64_t wgs = (groups + {groups} - 1) / {groups};
    hipLaunchKernelGGL({K}, dim3((uint32_t)wgs), dim3({threads}), 0, s, a);
    return hipGetLastError() == hipSuccess ? NFEC_OK : NFEC_EDEVICE;
}}""")
    return "\n\n".join(out)


def main():
    # the round-1 2-role encode is an A/B alternative to the q4 kernels: it is built into the
    # diagnostic library only (make -C norm_amd diag), always with its probes
    argv = [a for a in sys.argv if a != "--diag"]
    path = argv[1]
    shapes = DEFAULT_SHAPES
    if len(argv) > 2:
        shapes = [tuple(int(v) for v in s.split(",")) for s in argv[2:]]
    parts = [
        "// GENERATED by tools/codegen/gen_rs8_asm.py -- do not edit by hand.",
        "// Bit-sliced RS8 encode kernels with hand-allocated gfx950 assembly role bodies for",
        "// (k, m) in: " + ", ".join(f"({k},{m})" for k, m in shapes),
        '#include <cstdlib>',
        '#include "bitslice.hpp"',
        "",
        "namespace nfec {",
        "namespace {",
    ]
    for k, m in shapes:
        parts.append(gen_kernel(k, m))
        if (k, m) == (64, 32):
            for v, (probe, suffix) in PROBES.items():
                parts.append(gen_kernel(k, m, probe, suffix))
    # MDP full blocks: the LFSR encoder is a fixed linear map too, so the same bodies apply
    for k, m in MDP_SHAPES:
        parts.append(gen_kernel(k, m, G=mdp_matrix(k, m), prefix="mdp_asm_enc"))
    parts.append("}  // namespace")
    parts.append("")
    parts.append("static int asm_variant()")
    parts.append("{")
    parts.append("    static const int v = [] { const char* e = std::getenv(\"NFEC_ASM_VARIANT\"); return e ? std::atoi(e) : 0; }();")
    parts.append("    return v;")
    parts.append("}")
    parts.append("")
    parts.append("// NFEC_ENOTSUP when no assembly kernel covers (k, m) or the batch (tails, shortened blocks)")
    parts.append("int launch_rs8_asm_encode(uint32_t k, uint32_t m, const bs::EncArgs& a, hipStream_t s)")
    parts.append("{")
    for k, m in shapes:
        if (k, m) == (64, 32):
            for v, (probe, suffix) in PROBES.items():
                parts.append(f"    if (k == {k} && m == {m} && asm_variant() == {v}) return launch_rs8_asm_enc{suffix}_k{k}_m{m}(a, s);")
        parts.append(f"    if (k == {k} && m == {m}) return launch_rs8_asm_enc_k{k}_m{m}(a, s);")
    parts.append("    return NFEC_ENOTSUP;")
    parts.append("}")
    parts.append("")
    parts.append("// MDP encode of full blocks (num_data == NULL); NFEC_ENOTSUP otherwise")
    parts.append("int launch_mdp_asm_encode(uint32_t k, uint32_t m, const bs::EncArgs& a, hipStream_t s)")
    parts.append("{")
    for k, m in MDP_SHAPES:
        parts.append(f"    if (k == {k} && m == {m}) return launch_mdp_asm_enc_k{k}_m{m}(a, s);")
    parts.append("    return NFEC_ENOTSUP;")
    parts.append("}")
    parts.append("")
    parts.append("}  // namespace nfec")
    open(path, "w").write("\n".join(parts) + "\n")


if __name__ == "__main__":
    main()
