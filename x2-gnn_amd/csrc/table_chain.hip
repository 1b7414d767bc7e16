// Small-table chains: the Linear layers X2-GNN applies to its per-element edge table.
//
// Every triplet into line node e = (a -> b) carries edge_attr = emb(Z_b) (xgnn.py:57-58), so the
// embedding Linear (atom_embedding.py:22-25), edgenn (model.py:39) and each conv layer's lin_edge
// (sbftransformer_conv.py:144) run on the element table: <= 16 rows, D = 128.  As separate GEMM
// launches each of those layers is pure latency (one workgroup loads a 64 KB weight, does 0.3
// MFLOP, writes 5 KB): 7 launches forward and 7 backward at 7-12 us each.  Here the whole tree of
// stages runs in ONE workgroup per path: the rows stay in LDS from stage to stage, the next stage's
// weight is prefetched into registers while the current one computes, and the backward accumulates
// every stage's output gradient in LDS (children before parents) in one workgroup, then forms all
// weight gradients side by side in a second launch.  Deterministic: fixed orders throughout.
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

// Backward: the tree's stage arguments (launch 1 reads every stage's w / z / dy, launch 2 one stage each).
struct TableBwdArgs {
  x2g_table_bwd_stage st[kTMax];
  float* dx;
  int n;
  int R;
  float* part;  // [n][16][128] every stage's dz (launch 1 -> launch 2)
};

// ---- backward in two launches without a serial weight-gradient chain (round 6).  Round 5's form ran, per
// stage, the dz / dx chain AND the stage's dW / db in one workgroup (32 strided stores per lane, the old
// bucket values loaded behind them; the leaves side by side in a first launch), so every stage of the
// serial chain also waited on its weight-gradient traffic: 38 us per step for 7 stages of 16 rows
// (profiles/r5_step_work.json).  Now launch 1 (one
// workgroup) runs only the chain — per stage dz = dL/dy_s SiLU'(z_s) into LDS and out to the workspace,
// and dL/d in_s = dz W_s added into the parent's gradient — and launch 2 (one workgroup per stage, side by
// side) forms every dW / db from the workspace's dz and the stage input: dW^T = in^T dz as v_mfma_f32_16x16x4
// with the input as the A operand, so each lane ends with 4 consecutive columns of a dW row (16-byte loads of
// the old bucket values and 16-byte stores).
struct DzPre {
  f4 w[8];     // W[16q + 4g + e][16w + i]
  float z[4];  // pre-activation at (rows 4g + e, column 16w + i)
};

__device__ __forceinline__ void dz_prefetch(const TableBwdArgs& a, int s, DzPre& p) {
  if (s < 0) return;
  const x2g_table_bwd_stage& S = a.st[s];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int i = lane & 15, g = lane >> 4, c = 16 * w + i;
#pragma unroll
  for (int q = 0; q < 8; ++q)
#pragma unroll
    for (int e = 0; e < 4; ++e) p.w[q][e] = S.w[(16 * q + 4 * g + e) * kTD + c];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int r = 4 * g + e;
    p.z[e] = (S.act && r < a.R) ? S.z[r * kTD + c] : 0.0f;
  }
}

__device__ __forceinline__ void dz_stage(const TableBwdArgs& a, int s, int pf, DzPre& cur, DzPre& nxt,
                                         float (*G)[kTRows * kTS], float* dZ) {
  const x2g_table_bwd_stage& S = a.st[s];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int i = lane & 15, g = lane >> 4, c = 16 * w + i;
  __syncthreads();  // G[s + 1] is complete (every child has added its share); dZ is free
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int r = 4 * g + e;
    const float gv = G[s + 1][r * kTS + c];
    dZ[r * kTS + c] = S.act ? gv * silu_grad_(cur.z[e]) : gv;
  }
  __syncthreads();
  dz_prefetch(a, pf, nxt);
  {  // dz rows to the workspace (rows >= R are zero: their gradients and pre-activations are)
    const int r = tid >> 5, c4 = 4 * (tid & 31);
    *reinterpret_cast<f4*>(a.part + (static_cast<int64_t>(s) * kTRows + r) * kTD + c4) =
        *reinterpret_cast<const f4*>(dZ + r * kTS + c4);
  }
  // dL/d in[r][k] = sum_n dz[r][n] W[n][k]: wave w owns columns k = 16w + ...
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  const float* dzr = dZ + i * kTS + 4 * g;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const f4 av = *reinterpret_cast<const f4*>(dzr + 16 * q);
#pragma unroll
    for (int e = 0; e < 4; ++e) acc = mfma4(av[e], cur.w[q][e], acc);
  }
  float* gp = G[S.parent + 1];
#pragma unroll
  for (int e = 0; e < 4; ++e) gp[(4 * g + e) * kTS + c] += acc[e];
}

__global__ void __launch_bounds__(kTThreads) table_bwd_dz_kernel(const TableBwdArgs a) {
  __shared__ __attribute__((aligned(16))) float G[kTMax + 1][kTRows * kTS];  // dL/d(x), dL/d(y_s)
  __shared__ __attribute__((aligned(16))) float dZ[kTRows * kTS];
  const int tid = threadIdx.x;
  const int R = a.R;
  for (int t = -1; t < a.n; ++t) {
    const float* dy = t >= 0 ? a.st[t].dy : nullptr;
    if (dy)
      rows_to_lds(G[t + 1], dy, R);
    else
      *reinterpret_cast<f4*>(G[t + 1] + (tid >> 5) * kTS + 4 * (tid & 31)) = f4{0.f, 0.f, 0.f, 0.f};
  }
  DzPre p0, p1;
  int s = a.n - 1;  // children before parents: a stage's parent is an earlier stage
  dz_prefetch(a, s, p0);
  while (s >= 0) {  // two register sets alternate (unrolled by two, no copies)
    dz_stage(a, s, s - 1, p0, p1, G, dZ);
    if (s - 1 < 0) break;
    dz_stage(a, s - 1, s - 2, p1, p0, G, dZ);
    s -= 2;
  }
  if (a.dx) {
    __syncthreads();
    const int r = tid >> 5, c4 = 4 * (tid & 31);
    if (r < R) *reinterpret_cast<f4*>(a.dx + r * kTD + c4) = *reinterpret_cast<const f4*>(G[0] + r * kTS + c4);
  }
}

// workgroup s: dW_s (+)= dz_s^T in_s, db_s (+)= column sums of dz_s (rows ascending)
__global__ void __launch_bounds__(kTThreads) table_bwd_wgrad_kernel(const TableBwdArgs a) {
  __shared__ __attribute__((aligned(16))) float Dz[kTRows * kTS];
  __shared__ __attribute__((aligned(16))) float In[kTRows * kTS];
  const int s = blockIdx.x;
  const x2g_table_bwd_stage& S = a.st[s];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int i = lane & 15, g = lane >> 4;
  rows_to_lds(Dz, a.part + static_cast<int64_t>(s) * kTRows * kTD, kTRows);
  rows_to_lds(In, S.in, a.R);
  float* dwrow = S.dw + (16 * w + i) * kTD + 4 * g;  // dW row 16w + i, columns 16t + 4g .. + 3
  f4 old[8];
#pragma unroll
  for (int t = 0; t < 8; ++t)
    old[t] = S.accum ? *reinterpret_cast<const f4*>(dwrow + 16 * t) : f4{0.f, 0.f, 0.f, 0.f};
  __syncthreads();
  // D = dW^T block t: D[16t + m][16w + n] = sum_r in[r][16t + m] dz[r][16w + n]; lane (i, g) ends with
  // D[16t + 4g + e][16w + i] = dW[16w + i][16t + 4g + e]
  float bv[4];
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) bv[kk] = Dz[(4 * kk + g) * kTS + 16 * w + i];
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    f4 d = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) d = mfma4(In[(4 * kk + g) * kTS + 16 * t + i], bv[kk], d);
    *reinterpret_cast<f4*>(dwrow + 16 * t) = old[t] + d;
  }
  if (S.db && tid < kTD) {
    float acc = 0.0f;
    for (int r = 0; r < a.R; ++r) acc += Dz[r * kTS + tid];
    S.db[tid] = S.accum ? S.db[tid] + acc : acc;
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

X2G_API size_t x2g_table_chain_bwd_workspace(int32_t n_stages) {
  return n_stages > 0 ? static_cast<size_t>(n_stages) * kTRows * kTD * sizeof(float) : 0;
}

X2G_API int x2g_table_chain_bwd_ex(const x2g_table_bwd_stage* stages, int32_t n_stages, int64_t rows, int32_t dim,
                                   float* dx, void* workspace, size_t workspace_bytes, void* stream) {
  if (!stages || n_stages < 1 || n_stages > kTMax || rows < 0 || dim <= 0) return X2G_EINVAL;
  if (dim != kTD || rows > kTRows) return X2G_EUNSUPPORTED;
  if (!workspace || workspace_bytes < x2g_table_chain_bwd_workspace(n_stages)) return X2G_EWORKSPACE;
  if (!al16(workspace) || !al16(dx)) return X2G_EUNSUPPORTED;
  TableBwdArgs a{};
  for (int s = 0; s < n_stages; ++s) {
    const x2g_table_bwd_stage& S = stages[s];
    if (!S.w || !S.in || !S.dw || S.parent < -1 || S.parent >= s || (S.act != 0 && S.act != 1) || (S.act && !S.z))
      return X2G_EINVAL;
    if (!al16(S.w) || !al16(S.in) || !al16(S.dy) || !al16(S.dw)) return X2G_EUNSUPPORTED;
    a.st[s] = S;
  }
  // rows == 0 still launches: the weight gradients are zero, not left unwritten
  a.dx = dx;
  a.n = n_stages;
  a.R = static_cast<int>(rows);
  a.part = static_cast<float*>(workspace);  // dz of every stage [n][16][128]
  hipStream_t st = as_stream(stream);
  // launch 1: the dz / dx chain in one workgroup; launch 2: every stage's dW / db side by side
  table_bwd_dz_kernel<<<1, kTThreads, 0, st>>>(a);
  if (int rc = last_launch_status()) return rc;
  table_bwd_wgrad_kernel<<<static_cast<unsigned>(n_stages), kTThreads, 0, st>>>(a);
  return last_launch_status();
}
