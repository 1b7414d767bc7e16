// Small-table chains: the Linear layers X2-GNN applies to its per-element edge table.
//
// Every triplet into line node e = (a -> b) carries edge_attr = emb(Z_b) (xgnn.py:57-58), so the
// embedding Linear (atom_embedding.py:22-25), edgenn (model.py:39) and each conv layer's lin_edge
// (sbftransformer_conv.py:144) run on the element table: <= 16 rows, D = 128.  As separate GEMM
// launches each of those layers is pure latency (one workgroup loads a 64 KB weight, does 0.3
// MFLOP, writes 5 KB): 7 launches forward and 7 backward at 7-12 us each.  Here the whole tree of
// stages runs in ONE workgroup per direction: the rows stay in LDS from stage to stage, the next
// stage's weight is prefetched into registers while the current one computes, and the backward
// accumulates every stage's output gradient in LDS (children before parents), so the weight and
// data gradients of all stages come out of one launch.  Deterministic: one workgroup, fixed order.
#include "common.hpp"

namespace x2g {
namespace {

constexpr int kTD = 128;        // feature width
constexpr int kTRows = 16;      // table rows (X2-GNN: 10 element types)
constexpr int kTThreads = 512;  // 8 waves: wave w owns the 16 features 16w..16w+15 of every product
constexpr int kTS = 132;        // LDS row stride (floats): conflict-free 16-byte operand reads
constexpr int kTMax = X2G_TABLE_MAX_STAGES;

typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float silu_(float z) { return z / (1.0f + expf(-z)); }
__device__ __forceinline__ float silu_grad_(float z) {
  const float s = 1.0f / (1.0f + expf(-z));
  return s * (1.0f + z * (1.0f - s));
}

__device__ __forceinline__ f4 mfma4(float a, float b, f4 acc) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
}

// Every product is a 16-row v_mfma_f32_16x16x4_f32 sweep: lane l = (i = l & 15, g = l >> 4), and
// the contraction index of k-step s in 16-group q is 16q + 4g + s, so one 16-byte read per lane
// and group feeds four MFMAs (the order of a sum's terms is free).  D lane l holds rows 4g + e,
// column i of the wave's 16-column block.

// rows [R, D] -> LDS [16][kTS] (rows >= R zero)
__device__ __forceinline__ void rows_to_lds(float* __restrict__ dst, const float* __restrict__ src, int R) {
  const int tid = threadIdx.x, r = tid >> 5, c4 = 4 * (tid & 31);
  *reinterpret_cast<f4*>(dst + r * kTS + c4) = r < R ? *reinterpret_cast<const f4*>(src + r * kTD + c4)
                                                     : f4{0.f, 0.f, 0.f, 0.f};
}

// Stages run by one workgroup (bit s of mask: stage s); own: the stages whose outputs it writes.
// A tree with several leaves (X2-GNN: emb -> edgenn -> edgenn -> 4 x lin_edge) runs as one
// workgroup per leaf, each computing the path from the root to its leaf (the shared prefix
// redundantly: a 16-row stage is latency, not work), so the chain is as deep as the longest path
// (4 stages) instead of the stage count (7).
struct TableFwdArgs {
  const float* x;
  x2g_table_stage st[kTMax];
  int n;
  int R;
  uint32_t mask[kTMax];
  uint32_t own[kTMax];
};

// the next stage after s in mask (n when none; s = -1: the first)
__device__ __forceinline__ int next_in(uint32_t mask, int s, int n) {
  const uint32_t rest = s + 1 < 32 ? (mask >> (s + 1)) : 0u;
  return (s >= n || rest == 0) ? n : s + 1 + __builtin_ctz(rest);
}
// the stage before s in mask (-1 when none)
__device__ __forceinline__ int prev_in(uint32_t mask, int s) {
  const uint32_t below = s > 0 ? (mask & ((1u << s) - 1u)) : 0u;
  return below == 0 ? -1 : 31 - __builtin_clz(below);
}

// Stage s + 1's weight slice (the wave's 16 rows of W, 32 VGPRs) and bias are in flight while
// stage s computes; two register sets alternate (loop unrolled by two, no copies).
struct FwdPre {
  f4 w[8];
  float b;
};

__device__ __forceinline__ void fwd_prefetch(const TableFwdArgs& a, int s, FwdPre& p) {
  if (s < 0 || s >= a.n) return;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = 16 * w + (lane & 15), g = lane >> 4;
  const float* W = a.st[s].w + c * kTD + 4 * g;
#pragma unroll
  for (int q = 0; q < 8; ++q) p.w[q] = *reinterpret_cast<const f4*>(W + 16 * q);
  p.b = a.st[s].b ? a.st[s].b[c] : 0.0f;
}

// stage s of this workgroup's path; pf: the stage after it on the path (prefetched into nxt)
__device__ __forceinline__ void fwd_stage(const TableFwdArgs& a, int s, int pf, bool own, FwdPre& cur, FwdPre& nxt,
                                          float (*Y)[kTRows * kTS]) {
  const x2g_table_stage& S = a.st[s];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int i = lane & 15, g = lane >> 4, c = 16 * w + i;
  __syncthreads();  // Y[parent] is complete
  fwd_prefetch(a, pf, nxt);
  const float* in = Y[S.parent + 1] + i * kTS + 4 * g;
  f4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const f4 av = *reinterpret_cast<const f4*>(in + 16 * q);
#pragma unroll
    for (int e = 0; e < 4; ++e) acc = mfma4(av[e], cur.w[q][e], acc);
  }
  const int R = a.R;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int r = 4 * g + e;
    const float z = acc[e] + cur.b;
    const float y = S.act ? silu_(z) : z;
    Y[s + 1][r * kTS + c] = y;
    if (r < R && own) {
      if (S.z) S.z[r * kTD + c] = z;
      S.y[r * kTD + c] = y;
    }
  }
}

__global__ void __launch_bounds__(kTThreads) table_chain_fwd_kernel(const TableFwdArgs a) {
  __shared__ __attribute__((aligned(16))) float Y[kTMax + 1][kTRows * kTS];  // x, then each stage's output
  const uint32_t mask = a.mask[blockIdx.x], own = a.own[blockIdx.x];
  const int n = a.n;
  FwdPre p0, p1;
  int s = next_in(mask, -1, n);
  fwd_prefetch(a, s, p0);
  rows_to_lds(Y[0], a.x, a.R);
  while (s < n) {  // two register sets alternate (unrolled by two, no copies)
    const int s1 = next_in(mask, s, n);
    fwd_stage(a, s, s1, (own >> s) & 1u, p0, p1, Y);
    if (s1 >= n) break;
    const int s2 = next_in(mask, s1, n);
    fwd_stage(a, s1, s2, (own >> s1) & 1u, p1, p0, Y);
    s = s2;
  }
}

// Backward with several leaves: launch 1 (leaf pass) runs each leaf stage in its own workgroup and
// leaves its input-gradient share dy_leaf W_leaf in the workspace (part[leaf]); launch 2 runs the
// other stages in one workgroup, adding the shares into their parents' gradients in leaf order.
struct TableBwdArgs {
  x2g_table_bwd_stage st[kTMax];
  float* dx;
  int n;
  int R;
  uint32_t mask;          // launch 2: the stages it runs (the rest are leaves done by launch 1)
  int leaf[kTMax];        // launch 1: workgroup b runs stage leaf[b]
  float* part;            // [n][16][128] the leaves' input-gradient shares (or NULL: one launch)
};

// Stage s's weight (read transposed: column block 16w, rows 16q + 4g + e), forward input and
// pre-activation are loaded during stage s + 1; the old gradient-bucket values it adds to fly
// during its own products.
struct BwdPre {
  f4 w[8];     // W[16q + 4g + e][16w + i]
  f4 in;       // row tid >> 5, columns 4 (tid & 31) ..
  float z[4];  // pre-activation at (rows 4g + e, column 16w + i)
};

__device__ __forceinline__ void bwd_prefetch(const TableBwdArgs& a, int s, BwdPre& p) {
  if (s < 0) return;
  const x2g_table_bwd_stage& S = a.st[s];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int i = lane & 15, g = lane >> 4, c = 16 * w + i;
  const int R = a.R;
#pragma unroll
  for (int q = 0; q < 8; ++q)
#pragma unroll
    for (int e = 0; e < 4; ++e) p.w[q][e] = S.w[(16 * q + 4 * g + e) * kTD + c];
  {
    const int r = tid >> 5;
    p.in = r < R ? *reinterpret_cast<const f4*>(S.in + r * kTD + 4 * (tid & 31)) : f4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int r = 4 * g + e;
    p.z[e] = (S.act && r < R) ? S.z[r * kTD + c] : 0.0f;
  }
}

// old values of stage s's dW / db when it accumulates into a gradient bucket (zero otherwise), in
// the MFMA D layout of the dW product: old[t][e] = dw[16w + 4g + e][16t + i]
__device__ __forceinline__ void load_old(const TableBwdArgs& a, int s, f4 (&old)[8]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, i = lane & 15, g = lane >> 4;
  const bool on = s >= 0 && a.st[s >= 0 ? s : 0].accum;
  const float* dw = a.st[s >= 0 ? s : 0].dw;
#pragma unroll
  for (int t = 0; t < 8; ++t)
#pragma unroll
    for (int e = 0; e < 4; ++e) old[t][e] = on ? dw[(16 * w + 4 * g + e) * kTD + 16 * t + i] : 0.0f;
}

template <bool LEAF>
__device__ __forceinline__ void bwd_stage(const TableBwdArgs& a, int s, int pf, BwdPre& cur, BwdPre& nxt,
                                          float (*G)[kTRows * kTS], float* dZ, float* In, f4 (&old)[8]) {
  const x2g_table_bwd_stage& S = a.st[s];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int i = lane & 15, g = lane >> 4, c = 16 * w + i;
  __syncthreads();  // G[s + 1] is complete (every child has added its share); dZ, In are free
  *reinterpret_cast<f4*>(In + (tid >> 5) * kTS + 4 * (tid & 31)) = cur.in;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int r = 4 * g + e;
    const float gv = G[s + 1][r * kTS + c];
    dZ[r * kTS + c] = S.act ? gv * silu_grad_(cur.z[e]) : gv;
  }
  __syncthreads();
  bwd_prefetch(a, pf, nxt);
  // dW[n][k] = sum_r dz[r][n] in[r][k]: wave w owns rows n = 16w + ..., all 8 column blocks; the
  // old bucket values (old, loaded at the end of the previous stage) are added at the store
  float ad[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) ad[e] = dZ[(4 * g + e) * kTS + c];  // A: (n = c, r = 4g + e)
  f4 dwv[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    dwv[t] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int e = 0; e < 4; ++e) dwv[t] = mfma4(ad[e], In[(4 * g + e) * kTS + 16 * t + i], dwv[t]);
  }
#pragma unroll
  for (int t = 0; t < 8; ++t)
#pragma unroll
    for (int e = 0; e < 4; ++e) S.dw[(16 * w + 4 * g + e) * kTD + 16 * t + i] = old[t][e] + dwv[t][e];
  load_old(a, pf, old);  // the next stage's, in flight through its barriers and dz
  if (S.db && tid < kTD) {
    float acc = 0.0f;
    for (int r = 0; r < a.R; ++r) acc += dZ[r * kTS + tid];
    S.db[tid] = S.accum ? S.db[tid] + acc : acc;
  }
  // dL/d in[r][k] += sum_n dz[r][n] W[n][k]: wave w owns columns k = 16w + ...
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  const float* dzr = dZ + i * kTS + 4 * g;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const f4 av = *reinterpret_cast<const f4*>(dzr + 16 * q);
#pragma unroll
    for (int e = 0; e < 4; ++e) acc = mfma4(av[e], cur.w[q][e], acc);
  }
  if (LEAF) {  // the share goes to the parent's gradient through the workspace
    float* pp = a.part + static_cast<int64_t>(s) * kTRows * kTD;
#pragma unroll
    for (int e = 0; e < 4; ++e) pp[(4 * g + e) * kTD + c] = acc[e];
    return;
  }
  float* gp = G[S.parent + 1];
#pragma unroll
  for (int e = 0; e < 4; ++e) gp[(4 * g + e) * kTS + c] += acc[e];
}

template <bool LEAF>
__global__ void __launch_bounds__(kTThreads) table_chain_bwd_kernel(const TableBwdArgs a) {
  __shared__ __attribute__((aligned(16))) float G[kTMax + 1][kTRows * kTS];  // dL/d(x), dL/d(y_s)
  __shared__ __attribute__((aligned(16))) float dZ[kTRows * kTS];
  __shared__ __attribute__((aligned(16))) float In[kTRows * kTS];
  const int tid = threadIdx.x;
  const int R = a.R;
  BwdPre p0, p1;
  f4 old[8];
  if (LEAF) {  // launch 1: this workgroup's leaf stage alone
    const int s = a.leaf[blockIdx.x];
    bwd_prefetch(a, s, p0);
    load_old(a, s, old);
    const float* dy = a.st[s].dy;
    if (dy)
      rows_to_lds(G[s + 1], dy, R);
    else
      *reinterpret_cast<f4*>(G[s + 1] + (tid >> 5) * kTS + 4 * (tid & 31)) = f4{0.f, 0.f, 0.f, 0.f};
    bwd_stage<true>(a, s, -1, p0, p1, G, dZ, In, old);
    return;
  }
  const uint32_t mask = a.mask;
  int s = prev_in(mask, a.n);
  for (int t = -1; t < a.n; ++t) {
    const float* dy = t >= 0 ? a.st[t].dy : nullptr;
    if (dy)
      rows_to_lds(G[t + 1], dy, R);
    else
      *reinterpret_cast<f4*>(G[t + 1] + (tid >> 5) * kTS + 4 * (tid & 31)) = f4{0.f, 0.f, 0.f, 0.f};
  }
  if (a.part) {  // the leaves' shares, added in stage order (each thread its own elements: no race)
    const int r = tid >> 5, c4 = 4 * (tid & 31);
    for (int t = 0; t < a.n; ++t) {
      if ((mask >> t) & 1u) continue;
      float* gp = G[a.st[t].parent + 1] + r * kTS + c4;
      const f4 v = r < R ? *reinterpret_cast<const f4*>(a.part + (static_cast<int64_t>(t) * kTRows + r) * kTD + c4)
                         : f4{0.f, 0.f, 0.f, 0.f};
      *reinterpret_cast<f4*>(gp) = *reinterpret_cast<const f4*>(gp) + v;
    }
  }
  bwd_prefetch(a, s, p0);
  load_old(a, s, old);
  while (s >= 0) {  // two register sets alternate (unrolled by two, no copies)
    const int s1 = prev_in(mask, s);
    bwd_stage<false>(a, s, s1, p0, p1, G, dZ, In, old);
    if (s1 < 0) break;
    const int s2 = prev_in(mask, s1);
    bwd_stage<false>(a, s1, s2, p1, p0, G, dZ, In, old);
    s = s2;
  }
  if (a.dx) {
    __syncthreads();
    const int r = tid >> 5, c4 = 4 * (tid & 31);
    if (r < R) *reinterpret_cast<f4*>(a.dx + r * kTD + c4) = *reinterpret_cast<const f4*>(G[0] + r * kTS + c4);
  }
}

inline bool al16(const void* p) { return reinterpret_cast<uintptr_t>(p) % 16 == 0; }

}  // namespace
}  // namespace x2g

using namespace x2g;

X2G_API int x2g_table_chain_fwd(const float* x, int64_t rows, int32_t dim, const x2g_table_stage* stages,
                                int32_t n_stages, void* stream) {
  if (!stages || n_stages < 1 || n_stages > kTMax || rows < 0 || dim <= 0) return X2G_EINVAL;
  if (dim != kTD || rows > kTRows) return X2G_EUNSUPPORTED;
  TableFwdArgs a{};
  for (int s = 0; s < n_stages; ++s) {
    const x2g_table_stage& S = stages[s];
    if (!S.w || !S.y || S.parent < -1 || S.parent >= s || (S.act != 0 && S.act != 1) || (S.act && !S.z))
      return X2G_EINVAL;
    if (!al16(S.w)) return X2G_EUNSUPPORTED;
    a.st[s] = S;
  }
  if (rows == 0) return X2G_OK;
  if (!x) return X2G_EINVAL;
  if (!al16(x)) return X2G_EUNSUPPORTED;
  a.x = x;
  a.n = n_stages;
  a.R = static_cast<int>(rows);
  // one workgroup per leaf, each running the path root -> leaf; a stage's outputs are written by the
  // first workgroup whose path holds it
  uint32_t has_child = 0, owned = 0;
  for (int s = 0; s < n_stages; ++s)
    if (stages[s].parent >= 0) has_child |= 1u << stages[s].parent;
  int nwg = 0;
  for (int s = 0; s < n_stages; ++s) {
    if ((has_child >> s) & 1u) continue;
    uint32_t m = 0;
    for (int t = s; t >= 0; t = stages[t].parent) m |= 1u << t;
    a.mask[nwg] = m;
    a.own[nwg] = m & ~owned;
    owned |= m;
    ++nwg;
  }
  table_chain_fwd_kernel<<<static_cast<unsigned>(nwg), kTThreads, 0, as_stream(stream)>>>(a);
  return last_launch_status();
}

// the one-workgroup chain (a tree with one leaf)
static int table_chain_bwd_1wg(const x2g_table_bwd_stage* stages, int32_t n_stages, int64_t rows, float* dx,
                               hipStream_t st) {
  TableBwdArgs a{};
  for (int s = 0; s < n_stages; ++s) {
    const x2g_table_bwd_stage& S = stages[s];
    if (!S.w || !S.in || !S.dw || S.parent < -1 || S.parent >= s || (S.act != 0 && S.act != 1) || (S.act && !S.z))
      return X2G_EINVAL;
    if (!al16(S.w) || !al16(S.in) || !al16(S.dy)) return X2G_EUNSUPPORTED;
    a.st[s] = S;
  }
  // rows == 0 still launches: the weight gradients are zero, not left unwritten
  a.dx = dx;
  a.n = n_stages;
  a.R = static_cast<int>(rows);
  a.mask = n_stages >= 32 ? ~0u : (1u << n_stages) - 1u;
  table_chain_bwd_kernel<false><<<1, kTThreads, 0, st>>>(a);
  return last_launch_status();
}

X2G_API size_t x2g_table_chain_bwd_workspace(int32_t n_stages) {
  return n_stages > 0 ? static_cast<size_t>(n_stages) * kTRows * kTD * sizeof(float) : 0;
}

X2G_API int x2g_table_chain_bwd_ex(const x2g_table_bwd_stage* stages, int32_t n_stages, int64_t rows, int32_t dim,
                                   float* dx, void* workspace, size_t workspace_bytes, void* stream) {
  if (!stages || n_stages < 1 || n_stages > kTMax || rows < 0 || dim <= 0) return X2G_EINVAL;
  if (dim != kTD || rows > kTRows) return X2G_EUNSUPPORTED;
  uint32_t has_child = 0;
  for (int s = 0; s < n_stages; ++s)
    if (stages[s].parent >= 0 && stages[s].parent < s) has_child |= 1u << stages[s].parent;
  int nleaf = 0;
  for (int s = 0; s < n_stages; ++s) nleaf += ((has_child >> s) & 1u) ? 0 : 1;
  if (nleaf < 2) return table_chain_bwd_1wg(stages, n_stages, rows, dx, as_stream(stream));
  if (!workspace || workspace_bytes < x2g_table_chain_bwd_workspace(n_stages)) return X2G_EWORKSPACE;
  if (!al16(workspace)) return X2G_EUNSUPPORTED;
  TableBwdArgs a{};
  for (int s = 0; s < n_stages; ++s) {
    const x2g_table_bwd_stage& S = stages[s];
    if (!S.w || !S.in || !S.dw || S.parent < -1 || S.parent >= s || (S.act != 0 && S.act != 1) || (S.act && !S.z))
      return X2G_EINVAL;
    if (!al16(S.w) || !al16(S.in) || !al16(S.dy)) return X2G_EUNSUPPORTED;
    a.st[s] = S;
  }
  a.dx = dx;
  a.n = n_stages;
  a.R = static_cast<int>(rows);
  a.part = static_cast<float*>(workspace);
  int nl = 0;
  for (int s = 0; s < n_stages; ++s)
    if (!((has_child >> s) & 1u)) a.leaf[nl++] = s;
  hipStream_t st = as_stream(stream);
  // launch 1: the leaves side by side (their dW / db, and their input-gradient shares)
  table_chain_bwd_kernel<true><<<static_cast<unsigned>(nl), kTThreads, 0, st>>>(a);
  if (int rc = last_launch_status()) return rc;
  // launch 2: the inner stages in one workgroup, the shares added into their parents' gradients
  a.mask = has_child;
  table_chain_bwd_kernel<false><<<1, kTThreads, 0, st>>>(a);
  return last_launch_status();
}
