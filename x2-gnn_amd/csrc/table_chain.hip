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

struct TableFwdArgs {
  const float* x;
  x2g_table_stage st[kTMax];
  int n;
  int R;
};

// Stage s + 1's weight slice (the wave's 16 rows of W, 32 VGPRs) and bias are in flight while
// stage s computes; two register sets alternate (loop unrolled by two, no copies).
struct FwdPre {
  f4 w[8];
  float b;
};

__device__ __forceinline__ void fwd_prefetch(const TableFwdArgs& a, int s, FwdPre& p) {
  if (s >= a.n) return;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = 16 * w + (lane & 15), g = lane >> 4;
  const float* W = a.st[s].w + c * kTD + 4 * g;
#pragma unroll
  for (int q = 0; q < 8; ++q) p.w[q] = *reinterpret_cast<const f4*>(W + 16 * q);
  p.b = a.st[s].b ? a.st[s].b[c] : 0.0f;
}

__device__ __forceinline__ void fwd_stage(const TableFwdArgs& a, int s, FwdPre& cur, FwdPre& nxt,
                                          float (*Y)[kTRows * kTS]) {
  const x2g_table_stage& S = a.st[s];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int i = lane & 15, g = lane >> 4, c = 16 * w + i;
  __syncthreads();  // Y[parent] is complete
  fwd_prefetch(a, s + 1, nxt);
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
    if (r < R) {
      if (S.z) S.z[r * kTD + c] = z;
      S.y[r * kTD + c] = y;
    }
  }
}

__global__ void __launch_bounds__(kTThreads) table_chain_fwd_kernel(const TableFwdArgs a) {
  __shared__ __attribute__((aligned(16))) float Y[kTMax + 1][kTRows * kTS];  // x, then each stage's output
  FwdPre p0, p1;
  fwd_prefetch(a, 0, p0);
  rows_to_lds(Y[0], a.x, a.R);
  for (int s = 0; s < a.n; s += 2) {
    fwd_stage(a, s, p0, p1, Y);
    if (s + 1 < a.n) fwd_stage(a, s + 1, p1, p0, Y);
  }
}

struct TableBwdArgs {
  x2g_table_bwd_stage st[kTMax];
  float* dx;
  int n;
  int R;
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

__device__ __forceinline__ void bwd_stage(const TableBwdArgs& a, int s, BwdPre& cur, BwdPre& nxt,
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
  bwd_prefetch(a, s - 1, nxt);
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
  load_old(a, s - 1, old);  // the next stage's, in flight through its barriers and dz
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
  float* gp = G[S.parent + 1];
#pragma unroll
  for (int e = 0; e < 4; ++e) gp[(4 * g + e) * kTS + c] += acc[e];
}

__global__ void __launch_bounds__(kTThreads) table_chain_bwd_kernel(const TableBwdArgs a) {
  __shared__ __attribute__((aligned(16))) float G[kTMax + 1][kTRows * kTS];  // dL/d(x), dL/d(y_s)
  __shared__ __attribute__((aligned(16))) float dZ[kTRows * kTS];
  __shared__ __attribute__((aligned(16))) float In[kTRows * kTS];
  const int tid = threadIdx.x;
  const int R = a.R;
  BwdPre p0, p1;
  bwd_prefetch(a, a.n - 1, p0);
  f4 old[8];
  load_old(a, a.n - 1, old);
  for (int s = -1; s < a.n; ++s) {
    const float* dy = s >= 0 ? a.st[s].dy : nullptr;
    if (dy)
      rows_to_lds(G[s + 1], dy, R);
    else
      *reinterpret_cast<f4*>(G[s + 1] + (tid >> 5) * kTS + 4 * (tid & 31)) = f4{0.f, 0.f, 0.f, 0.f};
  }
  for (int s = a.n - 1; s >= 0; s -= 2) {
    bwd_stage(a, s, p0, p1, G, dZ, In, old);
    if (s - 1 >= 0) bwd_stage(a, s - 1, p1, p0, G, dZ, In, old);
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
  table_chain_fwd_kernel<<<1, kTThreads, 0, as_stream(stream)>>>(a);
  return last_launch_status();
}

X2G_API int x2g_table_chain_bwd(const x2g_table_bwd_stage* stages, int32_t n_stages, int64_t rows, int32_t dim,
                                float* dx, void* stream) {
  if (!stages || n_stages < 1 || n_stages > kTMax || rows < 0 || dim <= 0) return X2G_EINVAL;
  if (dim != kTD || rows > kTRows) return X2G_EUNSUPPORTED;
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
  table_chain_bwd_kernel<<<1, kTThreads, 0, as_stream(stream)>>>(a);
  return last_launch_status();
}
