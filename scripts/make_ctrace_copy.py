"""Generate x2-gnn_amd/build/ab_src/attention_center_ab.hip (untracked) from csrc/attention_center.hip with the phase stamps of the
center backward (scripts/trace_center_bwd.py reads them): thread 0 of each workgroup stamps the 100 MHz wall
clock at kernel start, after staging, after its pass 1, after the fence barrier, after rho, after pass 2 and
at the end (CTR(0..6), compiled only with -DX2G_TRACE).  Then:
    make -C x2-gnn_amd ab AB_UNIT=attention_center AB_NAME=ctrace AB_FLAGS=-DX2G_TRACE"""
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = open(os.path.join(ROOT, "x2-gnn_amd", "csrc", "attention_center.hip")).read()
head = '''#include "common.hpp"

// A/B trace build (-DX2G_TRACE): thread 0 of every backward workgroup stamps the 100 MHz wall clock at its
// phase boundaries into x2g_ctrace[block][8] (x2g_ctrace_fetch copies them out)
#ifdef X2G_TRACE
__device__ unsigned long long x2g_ctrace[8192 * 8];
#define CTR(k)                                                                                          \\
  do {                                                                                                  \\
    if (threadIdx.x == 0 && blockIdx.x < 8192) x2g_ctrace[blockIdx.x * 8 + (k)] = wall_clock64();     \\
  } while (0)
// the fused-projection forward's: start, tables, staging, P products, end (x2g_ftrace_fetch)
__device__ unsigned long long x2g_ftrace[8192 * 8];
#define FTR(k)                                                                                          \\
  do {                                                                                                  \\
    if (threadIdx.x == 0 && blockIdx.x < 8192) x2g_ftrace[blockIdx.x * 8 + (k)] = wall_clock64();     \\
  } while (0)
#else
#define FTR(k) \\
  do {         \\
  } while (0)
#define CTR(k) \\
  do {         \\
  } while (0)
#endif
'''
s = src.replace('#include "common.hpp"\n', head, 1)
i = s.index("attn_bwd_center_kernel(const BwdCenterArgs a) {")
s = s[:i] + s[i:].replace("{", "{\n  CTR(0);", 1)


def after(s, start, marker, text):
    j = s.index(marker, start) + len(marker)
    return s[:j] + text + s[j:]


s = after(s, i, "  __syncthreads();\n  const int nt = n - 1;  // triplets per destination (and per source)\n",
          "  CTR(1);\n")
j = s.index("  // the scratch written by every owner is read by others below", i)
s = s[:j] + "  CTR(2);\n" + s[j:]
s = after(s, i, "  __threadfence_block();\n  __syncthreads();\n", "  CTR(3);\n")
s = after(s, i, "    if (leader) RHO[i * H + head] = rho;\n  }\n  __syncthreads();\n", "  CTR(4);\n")
j = s.index("  if (a.d_edge) {  // d_edge[b] = sum_j (dv_j + dk_j), j ascending", i)
s = s[:j] + "  CTR(5);\n" + s[j:]
s = after(s, i, "      st4(a.d_edge + b * kCD + c0, s);\n    }\n  }\n", "  CTR(6);\n")
# the fused-projection forward
i = s.index("attn_fwd_center_sf_kernel(const FwdSfArgs a) {")
s = s[:i] + s[i:].replace("{", "{\n  FTR(0);", 1)
s = after(s, i, "  if (n_rows <= 0) return;  // (workgroup-uniform)\n", "  FTR(1);\n")
j = s.index("  __syncthreads();\n  {\n    if (pthr) {", i) + len("  __syncthreads();\n")
s = s[:j] + "  FTR(2);\n" + s[j:]
j = s.index("  __syncthreads();\n  for (; g < n_rows; g += 2 * WAVES) {", i) + len("  __syncthreads();\n")
s = s[:j] + "  FTR(3);\n" + s[j:]
j = s.index("\nconstexpr size_t fwd_sf_lds(int rows)", i)
j = s.rindex("}\n", i, j)
s = s[:j] + "  __syncthreads();  // (trace build only: the workgroup's end)\n  FTR(4);\n" + s[j:]
s += '''
#ifdef X2G_TRACE
X2G_API int x2g_ftrace_fetch(unsigned long long* host, int n) {
  return static_cast<int>(hipMemcpyFromSymbol(host, HIP_SYMBOL(x2g_ftrace), sizeof(unsigned long long) * n));
}
#endif
'''
s += '''
#ifdef X2G_TRACE
X2G_API int x2g_ctrace_fetch(unsigned long long* host, int n) {
  return static_cast<int>(hipMemcpyFromSymbol(host, HIP_SYMBOL(x2g_ctrace), sizeof(unsigned long long) * n));
}
#endif
'''
assert s.count("CTR(") == 9 and s.count("FTR(") == 7, (s.count("CTR("), s.count("FTR("))
dst = os.path.join(ROOT, "x2-gnn_amd", "build", "ab_src", "attention_center_ab.hip")
os.makedirs(os.path.dirname(dst), exist_ok=True)
open(dst, "w").write(s)
print("ok")
