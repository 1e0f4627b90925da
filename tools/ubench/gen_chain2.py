"""Chain-op cost breakdown on one wave (gfx950): what does each LDS instruction
add to a dependent f64 chain?  s_memtime-bracketed, best of 20."""
import sys

N = 122


def kernel(name, body, pre=()):
    o = [f'extern "C" __global__ __launch_bounds__(64) void k_{name}(double *out, unsigned long long *t, double seed) {{',
         "  extern __shared__ double2 L[];",
         "  const int ln = threadIdx.x;",
         "  double2 *B = L + ln;",
         "  double *Bd = (double *)L + ln;",
         f"  for (int i = 0; i < {N + 16}; ++i) B[i * 64] = make_double2(seed * i, -seed * i);",
         "  __syncthreads();",
         "  double dr[8], di[8];",
         "  for (int i = 0; i < 8; ++i) { dr[i] = seed * (i + 1); di[i] = seed * (i + 2); }",
         "  double vr = seed, vi = -seed, cr = seed * 3, ci = seed * 5;",
         "  unsigned long long t0;",
         '  __asm__ volatile("s_waitcnt lgkmcnt(0)\\n s_memtime %0\\n s_waitcnt lgkmcnt(0)" : "=s"(t0) : : "memory");',
         '  __asm__ volatile("" : "+v"(vr), "+v"(vi), "+v"(cr), "+v"(ci));']
    o += list(pre)
    for i in range(N):
        o.append(body(i))
    o += ['  __asm__ volatile("" : "+v"(vr), "+v"(vi));',
          "  B[0] = make_double2(vr, vi);",
          "  unsigned long long t1;",
          '  __asm__ volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\\n s_memtime %0\\n s_waitcnt lgkmcnt(0)" : "=s"(t1) : : "memory");',
          "  out[ln] = vr + vi;",
          "  if (ln == 0) t[0] = t1 - t0;",
          "}"]
    return "\n".join(o)


def ahead_loads(k):
    pre = [f"  const double2 d{i} = B[{(i + 1) * 64}];" for i in range(k)]

    def body(i):
        s = f"  const double2 d{i + k} = B[{(i + k + 1) * 64}];" if i + k < N else ""
        return s + f" vr = vr - d{i}.x; vi = vi - d{i}.y; B[{(i + 1) * 64}] = make_double2(vr, vi);"
    return body, pre


V = {
    "regs": (lambda i: f"  vr = vr - dr[{i % 8}]; vi = vi - di[{i % 8}];", ()),
    "st128_chain": (lambda i: f"  vr = vr - dr[{i % 8}]; vi = vi - di[{i % 8}]; B[{(i + 1) * 64}] = make_double2(vr, vi);", ()),
    "st128_const": (lambda i: f"  vr = vr - dr[{i % 8}]; vi = vi - di[{i % 8}]; B[{(i + 1) * 64}] = make_double2(cr, ci);", ()),
    "st64x2_chain": (lambda i: f"  vr = vr - dr[{i % 8}]; vi = vi - di[{i % 8}]; Bd[{(i + 1) * 128}] = vr; Bd[{(i + 1) * 128 + 64}] = vi;", ()),
    "st_every4": (lambda i: f"  vr = vr - dr[{i % 8}]; vi = vi - di[{i % 8}];" + (f" B[{(i + 1) * 64}] = make_double2(vr, vi);" if i % 4 == 0 else ""), ()),
    "full_a6": ahead_loads(6),
    "full_a3": ahead_loads(3),
    "full_a10": ahead_loads(10),
}

src = ["#include <hip/hip_runtime.h>", "#include <cstdio>", "#pragma clang fp contract(off)"]
for n, (b, pre) in V.items():
    src.append(kernel(n, b, pre))
names = list(V)
src.append("int main() {\n  double *out; unsigned long long *t;\n  (void)hipMalloc(&out, 64 * sizeof(double)); (void)hipMalloc(&t, 8);")
src.append("  const char *names[] = {" + ", ".join(f'"{n}"' for n in names) + "};")
src.append("  void (*ks[])(double *, unsigned long long *, double) = {" + ", ".join(f"k_{n}" for n in names) + "};")
src.append(f"""  for (int v = 0; v < {len(names)}; ++v) {{
    unsigned long long best = ~0ull, h;
    for (int r = 0; r < 20; ++r) {{
      hipLaunchKernelGGL(ks[v], dim3(1), dim3(64), 64 * 140 * 16, 0, out, t, 1.0 + r);
      (void)hipMemcpy(&h, t, 8, hipMemcpyDeviceToHost);
      if (h < best) best = h;
    }}
    printf("%-14s %6llu cycles  %.1f cycles/op\\n", names[v], best, best / {N}.0);
  }}
  return 0;
}}""")
open(sys.argv[1], "w").write("\n".join(src))
