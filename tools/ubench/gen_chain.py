"""Generate chain microbenchmarks: one wave runs N dependent complex subtracts
(the forward-sweep op shape) under several variants; s_memtime brackets."""
import sys

N = 122
VARIANTS = {
    "full": dict(load=True, store=True),     # as generated: lookahead load + store per op
    "noload": dict(load=False, store=True),  # drop operands from registers
    "nostore": dict(load=True, store=False),
    "regs": dict(load=False, store=False),   # pure f64 add chain
    "regs1": dict(load=False, store=False, one=True),   # one real chain only
    "f32": dict(load=False, store=False, f32=True),     # f32 complex chain
}


def kernel(name, load, store, ahead=6, one=False, f32=False):
    o = [f'extern "C" __global__ __launch_bounds__(64) void k_{name}(double *out, unsigned long long *t, double seed) {{',
         "  extern __shared__ double2 L[];",
         "  const int ln = threadIdx.x & 63, wv = threadIdx.x >> 6;",
         f"  double2 *B = L + wv * {(N + 2) * 64} + ln;",
         f"  for (int i = 0; i < {N + 2}; ++i) B[i * 64] = make_double2(seed * i, -seed * i);",
         "  __syncthreads();",
         "  double dr[8], di[8];",
         "  for (int i = 0; i < 8; ++i) { dr[i] = seed * (i + 1); di[i] = seed * (i + 2); }",
         "  double vr = seed, vi = -seed;",
         "  float fr = (float)seed, fi = -(float)seed;",
         "  unsigned long long t0;",
         '  __asm__ volatile("s_waitcnt lgkmcnt(0)\\n s_memtime %0\\n s_waitcnt lgkmcnt(0)" : "=s"(t0) : : "memory");',
         '  __asm__ volatile("" : "+v"(vr), "+v"(vi), "+v"(fr), "+v"(fi));']
    if load:
        for i in range(min(ahead, N)):
            o.append(f"  const double2 d{i} = B[{(i + 1) * 64}];")
    for i in range(N):
        if load and i + ahead < N:
            o.append(f"  const double2 d{i + ahead} = B[{(i + ahead + 1) * 64}];")
        if load:
            o.append(f"  vr = vr - d{i}.x; vi = vi - d{i}.y;")
        elif one:
            o.append(f"  vr = vr - dr[{i % 8}];")
        elif f32:
            o.append(f"  fr = fr - (float)dr[{i % 8}]; fi = fi - (float)di[{i % 8}];")
        else:
            o.append(f"  vr = vr - dr[{i % 8}]; vi = vi - di[{i % 8}];")
        if store:
            o.append(f"  B[{(i + 1) * 64}] = make_double2(vr, vi);")
    o += ['  __asm__ volatile("" : "+v"(vr), "+v"(vi), "+v"(fr), "+v"(fi));',
          "  B[0] = make_double2(vr + fr, vi + fi);",
          "  unsigned long long t1;",
          '  __asm__ volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\\n s_memtime %0\\n s_waitcnt lgkmcnt(0)" : "=s"(t1) : : "memory");',
          "  out[threadIdx.x] = vr + vi;",
          "  if (ln == 0) t[wv] = t1 - t0;",
          "}"]
    return "\n".join(o)


src = ["#include <hip/hip_runtime.h>", "#pragma clang fp contract(off)"]
for n, v in VARIANTS.items():
    src.append(kernel(n, **v))
src.append(r'''
#include <cstdio>
int main() {
  double *out; unsigned long long *t;
  hipMalloc(&out, 1024 * sizeof(double)); hipMalloc(&t, 16 * 8);
  const char *names[] = {"full", "noload", "nostore", "regs", "regs1", "f32"};
  void (*ks[])(double *, unsigned long long *, double) = {k_full, k_noload, k_nostore, k_regs, k_regs1, k_f32};
  for (int v = 0; v < 6; ++v) hipFuncSetAttribute((const void *)ks[v], hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  for (int v = 0; v < 6; ++v) for (int waves : {1, 2, 4}) {
    unsigned long long best = ~0ull, h[16];
    for (int r = 0; r < 20; ++r) {
      hipLaunchKernelGGL(ks[v], dim3(1), dim3(64 * waves), (size_t)waves * 64 * 124 * 16, 0, out, t, 1.0 + r);
      hipMemcpy(h, t, 8 * waves, hipMemcpyDeviceToHost);
      unsigned long long m = 0;
      for (int w = 0; w < waves; ++w) m = h[w] > m ? h[w] : m;
      if (m < best) best = m;
    }
    printf("%-8s waves=%d  %6llu cycles  %.1f cycles/op\n", names[v], waves, best, best / 122.0);
  }
  return 0;
}
''')
open(sys.argv[1], "w").write("\n".join(src))
