"""Generate ubench.hip: VALU issue-rate microbenchmarks for the FEC kernel design.

Measures lane-ops/s of v_perm_b32, v_bitop3_b32 and v_xor_b32 loops, and of long
straight-line bitop3 streams (to see whether code larger than the 64 KiB instruction cache
costs throughput) at low and high VGPR counts.
"""
import sys

L_SMALL, L_BIG = 4096, 32768


def straight(name, nreg, length):
    lines = [f'extern "C" __global__ __launch_bounds__(256) void {name}(unsigned* out, unsigned seed, int reps) {{']
    lines.append("  unsigned lane = threadIdx.x + blockIdx.x * 256;")
    for r in range(nreg):
        lines.append(f"  unsigned r{r} = seed * {2 * r + 1}u + lane;")
    lines.append("  for (int it = 0; it < reps; ++it) {")
    for i in range(length):
        a = i % nreg
        b = (i * 7 + 3) % nreg
        c = (i * 13 + 5) % nreg
        if b == a:
            b = (b + 1) % nreg
        if c == a or c == b:
            c = (c + 2) % nreg
        lines.append(f'    asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(r{a}) : "v"(r{b}), "v"(r{c}));')
    lines.append("  }")
    acc = " ^ ".join(f"r{r}" for r in range(nreg))
    lines.append(f"  out[lane] = {acc};")
    lines.append("}")
    return "\n".join(lines)


def loop_kernel(name, body):
    return f'''extern "C" __global__ __launch_bounds__(256) void {name}(unsigned* out, unsigned seed, int reps) {{
  unsigned lane = threadIdx.x + blockIdx.x * 256;
  unsigned a[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) a[i] = seed * (2 * i + 1) + lane;
  unsigned s = (lane * 0x01010101u) & 0x07070707u;
  for (int it = 0; it < reps; ++it) {{
#pragma unroll
    for (int i = 0; i < 16; ++i) {{ {body} }}
  }}
  unsigned r = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) r ^= a[i];
  out[lane] = r;
}}'''


def main(path):
    parts = ['#include <hip/hip_runtime.h>', '#include <cstdio>', '#include <vector>']
    parts.append(loop_kernel("k_perm", 'asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(a[(i + 1) & 15]), "v"(s));'))
    parts.append(loop_kernel("k_bitop3", 'asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a[i]) : "v"(a[(i + 1) & 15]), "v"(a[(i + 2) & 15]));'))
    parts.append(loop_kernel("k_xor", 'asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[i]) : "v"(a[(i + 1) & 15]));'))
    parts.append(straight("k_line_small_lo", 40, L_SMALL))
    parts.append(straight("k_line_big_lo", 40, L_BIG))
    parts.append(straight("k_line_small_hi", 280, L_SMALL))
    parts.append(straight("k_line_big_hi", 280, L_BIG))
    parts.append(r'''
typedef void (*kfn)(unsigned*, unsigned, int);
static void run(const char* name, kfn k, long ops_per_rep, int reps, int waves_per_cu) {
  int cus = 256;
  int grid = cus * waves_per_cu / 4;
  unsigned* out; hipMalloc(&out, (size_t)grid * 256 * 4);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, out, 1u, reps);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, out, 1u, reps);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1); ms /= 3;
  double lane_ops = (double)grid * 256 * ops_per_rep * reps;
  printf("{\"kernel\": \"%s\", \"waves_per_cu\": %d, \"ms\": %.4f, \"lane_ops_per_s\": %.4e, \"frac_of_7.86e13\": %.3f}\n",
         name, waves_per_cu, ms, lane_ops / (ms * 1e-3), lane_ops / (ms * 1e-3) / 7.86e13);
  hipFree(out);
}
int main() {
  int occ[] = {4, 8, 16, 32};
  for (int w : occ) {
    run("perm", k_perm, 16, 4000, w);
    run("bitop3", k_bitop3, 16, 4000, w);
    run("xor", k_xor, 16, 4000, w);
  }
  for (int w : occ) {
    run("line_small_lo(40 regs, 4k instr=32KB)", k_line_small_lo, ''' + str(L_SMALL) + r''', 16, w);
    run("line_big_lo(40 regs, 32k instr=256KB)", k_line_big_lo, ''' + str(L_BIG) + r''', 2, w);
  }
  int occ_hi[] = {4, 8};
  for (int w : occ_hi) {
    run("line_small_hi(280 regs, 32KB)", k_line_small_hi, ''' + str(L_SMALL) + r''', 16, w);
    run("line_big_hi(280 regs, 256KB)", k_line_big_hi, ''' + str(L_BIG) + r''', 2, w);
  }
  return 0;
}
''')
    open(path, "w").write("\n\n".join(parts))


if __name__ == "__main__":
    main(sys.argv[1])
