"""Sequential-stage step microbenchmark (gfx950): W waves (one per SIMD), each
runs S dependent steps  x = x + LDS[off(s)]; LDS[off(s)] = x  on 48 lanes with
the comb layout of the specialised kernel; variants differ in lookahead A,
masked stores (idle tracks) and store batching.  s_memtime-bracketed; prints
cycles per step (best of 10)."""
import sys

S = 60
SL = 52 * 16          # slot bytes (T=4, NS=4, tile 16 layout)
VARIANTS = []
for A in (2, 4, 8, 12):
    for mask in (0, 1):
        for batch in (1, 4, 8):
            VARIANTS.append((A, mask, batch))


def kernel(name, A, mask, batch):
    o = [f'extern "C" __global__ __launch_bounds__(256) void k_{name}(double *out, unsigned long long *t, double seed, unsigned act) {{',
         "  extern __shared__ char L[];",
         "  const int ln = threadIdx.x & 63, wv = threadIdx.x >> 6;",
         "  const int qp = ln / 16, qt = (ln / 4) % 4, qs = wv * 4 + ln % 4;",
         "  const bool on = ln < 48;",
         f"  for (int i = threadIdx.x; i < {(2 * S + 12) * SL // 16}; i += blockDim.x) ((double2 *)L)[i] = make_double2(seed * i, -seed);",
         "  __syncthreads();",
         f"  double2 *B = (double2 *)(L + qp * 256 + qs * 16 + qt * {SL});",
         "  const bool st_ok = (act >> qt) & 1u;",
         "  double xr = seed, xi = -seed;",
         "  unsigned long long t0;",
         '  __asm__ volatile("s_waitcnt lgkmcnt(0)\\n s_memtime %0\\n s_waitcnt lgkmcnt(0)" : "=s"(t0) : : "memory");',
         "  if (on) {"]
    off = lambda s: (4 + s * 2) * SL // 16  # noqa: E731  (comb bases 2 slots apart, as packed)
    for s in range(min(A, S)):
        o.append(f"    const double2 d{s} = B[{off(s)}];")
    pend = []
    for s in range(S):
        if s + A < S:
            o.append(f"    const double2 d{s + A} = B[{off(s + A)}];")
        o.append(f"    xr = xr + d{s}.x; xi = xi + d{s}.y; const double2 r{s} = make_double2(xr, xi);")
        pend.append(s)
        if len(pend) == batch or s == S - 1:
            for q in pend:
                if mask:
                    o.append(f"    if (st_ok) B[{off(q)}] = r{q};")
                else:
                    o.append(f"    B[{off(q)}] = r{q};")
            pend = []
        o.append("    __builtin_amdgcn_sched_barrier(0);")
    o += ["  }",
          "  unsigned long long t1;",
          '  __asm__ volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\\n s_memtime %0\\n s_waitcnt lgkmcnt(0)" : "=s"(t1) : : "memory");',
          "  out[threadIdx.x] = xr + xi;",
          "  if (ln == 0) t[wv] = t1 - t0;",
          "}"]
    return "\n".join(o)


src = ["#include <hip/hip_runtime.h>", "#include <cstdio>", "#pragma clang fp contract(off)"]
names = []
for A, mask, batch in VARIANTS:
    n = f"a{A}_m{mask}_b{batch}"
    names.append(n)
    src.append(kernel(n, A, mask, batch))
src.append("int main() {\n  double *out; unsigned long long *t;\n  (void)hipMalloc(&out, 1024 * sizeof(double)); (void)hipMalloc(&t, 64);")
src.append("  const char *names[] = {" + ", ".join(f'"{n}"' for n in names) + "};")
src.append("  void (*ks[])(double *, unsigned long long *, double, unsigned) = {" + ", ".join(f"k_{n}" for n in names) + "};")
src.append(f"""  const size_t lds = {(2 * S + 12) * SL};
  for (int v = 0; v < {len(names)}; ++v) {{
    (void)hipFuncSetAttribute((const void *)ks[v], hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    for (int waves : {{1, 4}}) {{
      unsigned long long best = ~0ull, h[4];
      for (int r = 0; r < 10; ++r) {{
        hipLaunchKernelGGL(ks[v], dim3(1), dim3(64 * waves), lds, 0, out, t, 1.0 + r, 0x7u);
        (void)hipMemcpy(h, t, 8 * waves, hipMemcpyDeviceToHost);
        unsigned long long m = 0;
        for (int w = 0; w < waves; ++w) m = h[w] > m ? h[w] : m;
        if (m < best) best = m;
      }}
      printf("%-12s waves=%d %7.1f cycles/step\\n", names[v], waves, best / {S}.0);
    }}
  }}
  return 0;
}}""")
open(sys.argv[1], "w").write("\n".join(src))
