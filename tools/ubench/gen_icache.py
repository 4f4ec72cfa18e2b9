"""Generate icache.hip: does instruction-stream diversity or VGPR bank pattern limit the VALU
rate of long straight-line bit-sliced code?

The generated RS8 kernels run R distinct straight-line streams (one per role) on the same CU
at the same time.  This bench runs v_bitop3_b32 streams of L instructions with explicit VGPRs:
  * roles R in {1, 2, 4}: wave w executes copy (w % R) of the stream (different bytes);
  * bank pattern: operands in 3 distinct VGPR banks (reg % 4), all in one bank, or random.
It reports lane-ops/s against the 7.86e13 nominal peak.
"""
import random
import sys

L = 12288           # instructions per stream (96 KiB of VOP3 code)
NREG = 64           # v8 .. v71
BASE = 8


def stream(seed, pattern):
    rnd = random.Random(seed)
    out = []
    for _ in range(L):
        if pattern == "distinct":
            banks = rnd.sample(range(4), 3)
            regs = [BASE + 4 * rnd.randrange(NREG // 4) + b for b in banks]
        elif pattern == "same":
            b = rnd.randrange(4)
            regs = rnd.sample([BASE + 4 * i + b for i in range(NREG // 4)], 3)
        else:
            regs = rnd.sample(range(BASE, BASE + NREG), 3)
        a, x, y = regs
        out.append(f"v_bitop3_b32 v{a}, v{a}, v{x}, v{y} bitop3:0x96")
    return out


def clobbers():
    return ", ".join(f'"v{r}"' for r in range(BASE, BASE + NREG))


def asm_block(lines):
    # split into chunks so no single asm string is huge
    parts = []
    for i in range(0, len(lines), 512):
        body = "\\n".join(lines[i:i + 512])
        parts.append(f'      asm volatile("{body}" ::: {clobbers()});')
    return "\n".join(parts)


def kernel(name, pattern, roles):
    k = [f'extern "C" __global__ __launch_bounds__(256) void {name}(unsigned* out, unsigned seed, int reps) {{']
    k.append("  const unsigned gw = blockIdx.x * 4 + (threadIdx.x >> 6);")
    k.append(f"  const unsigned role = __builtin_amdgcn_readfirstlane(gw % {roles});")
    init = "\\n".join(f"v_xor_b32 v{r}, {r * 2654435761 % (1 << 31)}, %0" for r in range(BASE, BASE + NREG))
    k.append(f'  asm volatile("{init}" :: "v"(seed ^ threadIdx.x) : {clobbers()});')
    k.append("  for (int it = 0; it < reps; ++it) {")
    for r in range(roles):
        kw = "if" if r == 0 else "else if"
        k.append(f"    {kw} (role == {r}) {{")
        k.append(asm_block(stream(1000 * r + len(pattern), pattern)))
        k.append("    }")
    k.append("  }")
    k.append("  unsigned res;")
    k.append('  asm volatile("v_mov_b32 %0, v8" : "=v"(res));')
    k.append("  out[blockIdx.x * 256 + threadIdx.x] = res;")
    k.append("}")
    return "\n".join(k)


def main(path):
    cases = [("rnd", "random", 1), ("rnd", "random", 2), ("rnd", "random", 4),
             ("dst", "distinct", 1), ("same", "same", 1), ("dst", "distinct", 2)]
    parts = ["#include <hip/hip_runtime.h>", "#include <cstdio>"]
    names = []
    for tag, pat, roles in cases:
        n = f"k_{tag}_r{roles}"
        names.append((n, pat, roles))
        parts.append(kernel(n, pat, roles))
    runs = "\n".join(
        f'  for (int w : occ) run("{n}", "{pat}", {roles}, {n}, w);' for n, pat, roles in names)
    parts.append(r'''
typedef void (*kfn)(unsigned*, unsigned, int);
static void run(const char* name, const char* pat, int roles, kfn k, int waves_per_cu) {
  const int cus = 256, reps = 8;
  int grid = cus * waves_per_cu / 4;
  unsigned* out; hipMalloc(&out, (size_t)grid * 256 * 4);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, out, 1u, reps);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, out, 1u, reps);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1); ms /= 3;
  double lane_ops = (double)grid * 256 * ''' + str(L) + r''' * reps;
  printf("{\"kernel\": \"%s\", \"pattern\": \"%s\", \"roles\": %d, \"waves_per_cu\": %d, \"ms\": %.4f, \"lane_ops_per_s\": %.4e, \"frac_of_7.86e13\": %.3f}\n",
         name, pat, roles, waves_per_cu, ms, lane_ops / (ms * 1e-3), lane_ops / (ms * 1e-3) / 7.86e13);
  hipFree(out);
}
int main() {
  int occ[] = {8, 16};
''' + runs + r'''
  return 0;
}
''')
    open(path, "w").write("\n\n".join(parts))


if __name__ == "__main__":
    main(sys.argv[1])
