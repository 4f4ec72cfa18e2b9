"""Generate callchain.hip: what does a snippet call of the tower kernel cost, and would chaining
calls (each snippet jumping straight to the next instead of returning) pay?

The tower kernel (tools/codegen/gen_gf16_tw.py) applies a coefficient by jumping into one of 256
GF(2^8) snippets (<= 8 v_bitop3 on M0-indexed accumulators) and back: per call an s_pack (the
target), an s_mov to M0 (the accumulator group), s_swappc and the snippet's s_setpc, two taken
branches.  The chained form runs two rows (four calls) per jump from the caller: every snippet
ends with
    s_add_u32 m0, m0, 8                       ; the next call's accumulators
    s_lshr_b64 CE, CE, 16                     ; the next 16-bit entry into CE's low half
    s_pack_lh_b32_b16 TGT, CE, SNIP           ; its address
    s_setpc_b64 TGT
and the fifth (exhausted, zero) entry lands on slot 0, a trampoline back to the caller; a zero
coefficient would take slot 256.  One taken branch per call plus one per chain instead of two
per call, for 21 instead of 16 SALU per four calls.

Kernels, R rows per sweep (2R calls), the snippet bodies and the register map of the real kernel
(--rows R layout; R = 7 without the prefetch: 3 waves per SIMD; R = 4: 4 waves per SIMD):
  k_plain_r{R}        the kernel's calls (gpr-index mode on SRC0 and DST, M0 per call)
  k_chain_r{R}        the chained calls above
  k_empty_r{R}        the kernel's calls into empty snippets (the calls' own cost)
  k_noidx_r{R}        the calls with the snippets outside gpr-index mode (fixed accumulators)
  k_inline_idx_r{R}   no calls: the bodies inline in gpr-index mode, M0 per call (_once: per sweep)
  k_inline_reg_r{R}   no calls: the bodies inline on explicit registers (_mov: plus an M0 write)
Each wave runs `reps` sweeps over fixed random coefficients.  Prints one JSON line per kernel:
ms, ns per call per SIMD.  Results: profiles/r05/callchain/ (DESIGN.md section 9, item 3).

    python3 tools/ubench/gen_callchain.py /tmp/callchain.hip
    hipcc --offload-arch=gfx950 -O3 /tmp/callchain.hip -o tools/callchain_bin   (tools/ubench is
    not sent to the GPU box)
"""
import os
import random
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "codegen"))
import gen_gf16_tw as g  # noqa: E402

S_SNIP, S_TGT, S_RET = 56, 58, 60
S_CE = 66                  # 2: the chain's entry pair
S_E = 72                   # 8: entries of the sweep's rows (row r: dword S_E + r, out0 low, out1 high)
S_CNT = 64
GPR_MODE = 0x9000


MODE = ""   # "" (real bodies), "empty" (no VALU in the snippets)


def body(c):
    return [] if MODE == "empty" else g.snippet_body(c)   # noidx: the same, outside gpr-index mode


IDX_MODE = "SRC0,DST"


def inline_sweep(rows, entries, idx, mov=True):
    """no calls: each call's body inline (idx: behind an s_mov to M0 in gpr-index mode, else on
    explicit accumulator registers; mov=False: M0 set once per sweep (idx) / no M0 write (reg);
    mov=True with explicit registers: a dummy M0 write per call)"""
    L = []
    if idx:
        L += [f"s_mov_b32 s{S_CNT + 1}, 0", f"s_set_gpr_idx_on s{S_CNT + 1}, gpr_idx({IDX_MODE})"]
    for r in range(rows):
        for j in range(2):
            c = entries[r][j]
            b = g.snippet_body(c)
            if idx:
                if mov or (r == 0 and j == 0):
                    L.append(f"s_mov_b32 m0, 0x{GPR_MODE | (16 * r + 8 * j):x}")
                L += b
            elif mov == "dummy":
                L.append(f"s_mov_b32 m0, 0x{16 * r + 8 * j:x}")
                L += _explicit(b, 16 * r + 8 * j)
            else:
                L += _explicit(b, 16 * r + 8 * j)
    if idx:
        L += ["s_set_gpr_idx_off", "s_nop 1"]
    return L


def _explicit(b, off):
    """a snippet body with its M0-relative destination made explicit (+off)"""
    out = []
    for op in b:
        parts = op.split(" ", 1)
        regs = parts[1].split(", ")
        d = int(regs[0][1:]) + off
        regs[0] = f"v{d}"
        regs[1] = f"v{d}"
        out.append(parts[0] + " " + ", ".join(regs))
    return out


ALIGN = 7   # snippet slot alignment (log2 bytes)


def table(chain):
    out = [".p2align 16", "Lsnip0_%=:"]
    for c in range(257 if chain else 256):
        if c:
            out.append(f".p2align {ALIGN}")
        if chain and c == 0:
            out.append(f"s_setpc_b64 s[{S_RET}:{S_RET + 1}]")   # slot 0: back to the caller
            continue
        out += body(c % 256)
        if chain:
            out += ["s_add_u32 m0, m0, 8", f"s_lshr_b64 s[{S_CE}:{S_CE + 1}], s[{S_CE}:{S_CE + 1}], 16",
                    f"s_pack_lh_b32_b16 s{S_TGT}, s{S_CE}, s{S_SNIP}", f"s_setpc_b64 s[{S_TGT}:{S_TGT + 1}]"]
        else:
            out.append(f"s_setpc_b64 s[{S_RET}:{S_RET + 1}]")
    return out


def sweep(rows, chain):
    if MODE == "noidx":   # calls into snippets on fixed accumulators (ACC0..7), no gpr-index mode
        L = []
        for r in range(rows):
            for j in range(2):
                op = "s_pack_lh_b32_b16" if j == 0 else "s_pack_hh_b32_b16"
                L += [f"{op} s{S_TGT}, s{S_E + r}, s{S_SNIP}", f"s_mov_b32 m0, 0x{16 * r + 8 * j:x}",
                      f"s_swappc_b64 s[{S_RET}:{S_RET + 1}], s[{S_TGT}:{S_TGT + 1}]"]
        return L
    L = [f"s_mov_b32 s{S_CNT + 1}, 0", f"s_set_gpr_idx_on s{S_CNT + 1}, gpr_idx(SRC0,DST)"]
    if chain:
        for r in range(0, rows, 2):
            L.append(f"s_mov_b64 s[{S_CE}:{S_CE + 1}], s[{S_E + r}:{S_E + r + 1}]")
            if r + 1 == rows:
                L.append(f"s_mov_b32 s{S_CE + 1}, 0")
            L += [f"s_mov_b32 m0, 0x{GPR_MODE | (16 * r):x}",
                  f"s_pack_lh_b32_b16 s{S_TGT}, s{S_CE}, s{S_SNIP}",
                  f"s_swappc_b64 s[{S_RET}:{S_RET + 1}], s[{S_TGT}:{S_TGT + 1}]"]
    else:
        for r in range(rows):
            for j in range(2):
                op = "s_pack_lh_b32_b16" if j == 0 else "s_pack_hh_b32_b16"
                # movk: a 4-byte SOPK (M0's upper half gets the sign copies of bit 15)
                mv = (f"s_movk_i32 m0, 0x{GPR_MODE | (16 * r + 8 * j):x}" if MODE == "movk"
                      else f"s_mov_b32 m0, 0x{GPR_MODE | (16 * r + 8 * j):x}")
                L += [f"{op} s{S_TGT}, s{S_E + r}, s{S_SNIP}", mv,
                      f"s_swappc_b64 s[{S_RET}:{S_RET + 1}], s[{S_TGT}:{S_TGT + 1}]"]
    L += ["s_set_gpr_idx_off", "s_nop 1"]
    return L


def kernel(name, rows, chain, inline=None, entries=None):
    g.set_prefetch(rows != 7)
    g.set_rows(rows)
    waves = 512 // ((g.V_LAST + 1 + 7) // 8 * 8)
    L = [f"s_getpc_b64 s[{S_SNIP}:{S_SNIP + 1}]", "Lpc_%=:",
         f"s_add_u32 s{S_SNIP}, s{S_SNIP}, Lsnip0_%=-Lpc_%=", f"s_addc_u32 s{S_SNIP + 1}, s{S_SNIP + 1}, 0",
         f"s_mov_b32 s{S_TGT + 1}, s{S_SNIP + 1}",
         f"s_load_dwordx8 s[{S_E}:{S_E + 7}], %[tab], 0x0", "s_waitcnt lgkmcnt(0)",
         f"s_and_b32 s{S_CNT}, s{S_SNIP}, 0xffff", f"s_cmp_lg_u32 s{S_CNT}, 0", "s_cbranch_scc1 Lbad_%=",
         f"s_mov_b32 s{S_CNT}, %[reps]"]
    for v in range(g.V_SLOT, g.V_LAST + 1):
        L.append(f"v_mov_b32 v{v}, {v}")
    L.append("Lloop_%=:")
    if inline is None:
        L += sweep(rows, chain)
    else:
        L += inline_sweep(rows, entries, inline.startswith("idx"),
                          {"idx": True, "idx_once": False, "reg": False, "reg_mov": "dummy"}[inline])
    L += [f"s_sub_u32 s{S_CNT}, s{S_CNT}, 1", f"s_cmp_lg_u32 s{S_CNT}, 0", "s_cbranch_scc1 Lloop_%=",
          f"v_mov_b32 %[res], v{g.ACC0}", "s_branch Lend_%=",
          "Lbad_%=:", "v_mov_b32 %[res], -1", "s_branch Lend_%="]
    L += table(chain)
    L.append("Lend_%=:")
    text = "\\n\"\n        \"".join(L)
    clob = ", ".join([f'"v{i}"' for i in range(g.V_SLOT, g.V_LAST + 1)] +
                     [f'"s{i}"' for i in range(S_SNIP, S_E + 8)] + ['"m0"', '"scc"', '"memory"'])
    g.set_prefetch(True)
    g.set_rows(6)
    return waves, f"""extern "C" __global__ __launch_bounds__(256, {waves}) void {name}(unsigned* out, const unsigned* tab, int reps)
{{
    unsigned res;
    asm volatile(
        "{text}\\n"
        : [res] "=v"(res)
        : [tab] "s"(tab), [reps] "s"(reps)
        : {clob});
    out[blockIdx.x * 256 + threadIdx.x] = res;
}}"""


def main(path):
    rnd = random.Random(5)
    parts = ["#include <hip/hip_runtime.h>", "#include <cstdio>", "#include <vector>"]
    runs = []
    global MODE, ALIGN
    coef = [(rnd.randrange(1, 256), rnd.randrange(1, 256)) for _ in range(8)]
    entries = [(c0 << 7) | ((c1 << 7) << 16) for c0, c1 in coef]
    for rows in (7, 4):
        global IDX_MODE
        for kind in ("plain", "movk", "movk256", "chain", "empty", "noidx", "inline_idx", "inline_idx_once",
                     "inline_reg", "inline_reg_mov"):
            MODE = "movk" if kind == "movk256" else kind if kind in ("empty", "noidx", "movk") else ""
            ALIGN = 8 if kind == "movk256" else 7
            name = f"k_{kind}_r{rows}"
            IDX_MODE = {"inline_idxdst_once": "DST", "inline_idxsrc0_once": "SRC0"}.get(kind, "SRC0,DST")
            inline = kind[len("inline_"):] if kind.startswith("inline_") else None
            inline = {"idxdst_once": "idx_once", "idxsrc0_once": "idx_once"}.get(inline, inline)
            waves, src = kernel(name, rows, kind == "chain", inline, coef)
            parts.append(src)
            runs.append(f'    run("{name}", {name}, {rows}, {waves}, {"tab2" if kind == "movk256" else "tab"});')
    MODE, ALIGN = "", 7
    ent = ", ".join(f"0x{e:08x}u" for e in entries)
    parts.append(r'''
typedef void (*kfn)(unsigned*, const unsigned*, int);
static void run(const char* name, kfn k, int rows, int waves, const unsigned* tab)
{
    const int cus = 256, reps = 20000;
    const int grid = cus * waves;   // one workgroup of 4 waves per SIMD-set: waves per SIMD resident
    unsigned* out;
    hipMalloc(&out, (size_t)grid * 256 * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, out, tab, 100);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, out, tab, reps);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    unsigned first;
    hipMemcpy(&first, out, 4, hipMemcpyDeviceToHost);
    const double calls = (double)grid * 4 * reps * 2 * rows;   // all waves
    const double per_simd = calls / 1024.0;
    printf("{\"kernel\": \"%s\", \"rows\": %d, \"waves_per_simd\": %d, \"ms\": %.3f, \"ns_per_call_per_simd\": %.4f, \"aligned\": %s}\n",
           name, rows, waves, ms, ms * 1e6 / per_simd, first == 0xFFFFFFFFu ? "false" : "true");
    hipFree(out);
}

int main()
{
    const unsigned h[8] = {''' + ent + r'''};
    unsigned* tab;
    hipMalloc(&tab, 64);
    hipMemcpy(tab, h, 32, hipMemcpyHostToDevice);
    unsigned h2[8];   // the same coefficients at 256-byte slots
    for (int i = 0; i < 8; ++i) h2[i] = ((h[i] & 0xFFFFu) << 1) | (((h[i] >> 16) << 1) << 16);
    unsigned* tab2;
    hipMalloc(&tab2, 64);
    hipMemcpy(tab2, h2, 32, hipMemcpyHostToDevice);
''' + "\n".join(runs) + r'''
    return 0;
}
''')
    open(path, "w").write("\n\n".join(parts))


if __name__ == "__main__":
    main(sys.argv[1])
