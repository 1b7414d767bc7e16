// The readouts' final Linear(D, 1), all readouts at once (readout.py:25-31,42 and 55-62,76; the
// per-layer results summed in model.py:41,50-53).  Forward: out[r] = sum_g (h_g[r] . w_g + b_g),
// 64 / LPR rows per wave, one 16-byte chunk of each row per lane, group dot products reduced
// over the row's lanes.  Backward: dh_g[r] = dout[r] w_g (row-parallel) and dw_g / db_g as
// per-workgroup partials (one accumulator set per row slot in LDS, folded in a fixed order) +
// the batched fixed-order slab sum.
#include "common.hpp"

namespace x2g {

constexpr int kHeadSplits = 256;

struct HeadBatch {
  x2g_head_group g[X2G_MAX_GROUPS];
};

typedef float f4h __attribute__((ext_vector_type(4)));

template <int LPR>
__global__ void __launch_bounds__(256) readout_head_fwd_kernel(const HeadBatch b, int G, int64_t R,
                                                               float* __restrict__ out) {
  constexpr int RPW = 64 / LPR;
  const int lane = threadIdx.x & 63, sub = lane % LPR;
  const int64_t nw = static_cast<int64_t>(gridDim.x) * 4;
  for (int64_t r = (static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6)) * RPW + lane / LPR; r < R;
       r += nw * RPW) {
    float acc = 0.f;
    for (int g = 0; g < G; ++g) {
      const f4h hv = reinterpret_cast<const f4h*>(b.g[g].h)[r * LPR + sub];
      const f4h wv = reinterpret_cast<const f4h*>(b.g[g].w)[sub];
      float d = hv.x * wv.x + hv.y * wv.y + hv.z * wv.z + hv.w * wv.w;
      d = group_sum<LPR>(d);
      acc += d + (b.g[g].b ? b.g[g].b[0] : 0.f);
    }
    if (sub == 0) out[r] = acc;
  }
}

// The heads with the per-molecule sum fused (model.py:53, the global add pool after AtomWise): one
// workgroup per segment of rows; wave w takes the segment's rows w*RPW .. in turns, each row's heads
// summed in job order, then the waves' sums in wave order (fixed order: deterministic).  Replaces the
// head launch + the pooling launch.
template <int LPR>
__global__ void __launch_bounds__(256) readout_head_pool_fwd_kernel(const HeadBatch b, int G,
                                                                    const int32_t* __restrict__ seg_rowptr,
                                                                    int64_t n_seg, float* __restrict__ out) {
  constexpr int RPW = 64 / LPR;
  __shared__ float red[4];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, sub = lane % LPR;
  for (int64_t m = blockIdx.x; m < n_seg; m += gridDim.x) {
    const int r0 = seg_rowptr[m], r1 = seg_rowptr[m + 1];
    float acc = 0.f;
    for (int r = r0 + wv * RPW + lane / LPR; r < r1; r += 4 * RPW) {
      float rowv = 0.f;
      for (int g = 0; g < G; ++g) {
        const f4h hv = reinterpret_cast<const f4h*>(b.g[g].h)[static_cast<int64_t>(r) * LPR + sub];
        const f4h wv4 = reinterpret_cast<const f4h*>(b.g[g].w)[sub];
        float d = hv.x * wv4.x + hv.y * wv4.y + hv.z * wv4.z + hv.w * wv4.w;
        d = group_sum<LPR>(d);
        rowv += d + (b.g[g].b ? b.g[g].b[0] : 0.f);
      }
      acc += sub == 0 ? rowv : 0.f;
    }
    acc = wave64_sum(acc);
    if (lane == 0) red[wv] = acc;
    __syncthreads();
    if (threadIdx.x == 0) out[m] = ((red[0] + red[1]) + red[2]) + red[3];
    __syncthreads();
  }
}

// the segment of row r: the last s with seg_rowptr[s] <= r (segments cover every row)
__device__ __forceinline__ int64_t seg_of_row(const int32_t* __restrict__ seg_rowptr, int64_t n_seg, int64_t r) {
  int64_t lo = 0, hi = n_seg;  // seg_rowptr[lo] <= r < seg_rowptr[hi]
  while (hi - lo > 1) {
    const int64_t mid = (lo + hi) >> 1;
    if (seg_rowptr[mid] <= r) lo = mid; else hi = mid;
  }
  return lo;
}

// block k owns rows [k * per, (k + 1) * per); partial slabs: part[g][k][D] and part[g][splits*D + k].
// seg_rowptr (or NULL): dout is per segment of rows (the fused pool's gradient, broadcast here)
template <int LPR>
__global__ void __launch_bounds__(256) readout_head_bwd_kernel(const float* __restrict__ dout, const HeadBatch b, int G,
                                                               int64_t R, float* __restrict__ part,
                                                               const int32_t* __restrict__ seg_rowptr,
                                                               int64_t n_seg) {
  constexpr int RPB = 256 / LPR;
  constexpr int D = 4 * LPR;
  __shared__ f4h red[RPB * LPR];
  __shared__ float redb[RPB];
  const int sub = threadIdx.x % LPR, slot = threadIdx.x / LPR;
  const int64_t per = (R + gridDim.x - 1) / gridDim.x;
  const int64_t lo = per * blockIdx.x, hi = lo + per < R ? lo + per : R;
  const int splits = gridDim.x;
  {  // job g = blockIdx.y (r2 looped over the jobs in every block: 5 x its row loop's round trips)
    const int g = blockIdx.y;
    const f4h wv = reinterpret_cast<const f4h*>(b.g[g].w)[sub];
    f4h aw = {0.f, 0.f, 0.f, 0.f};
    float ab = 0.f;
    constexpr int U = 4;  // rows per slot issued together
    for (int64_t r0 = lo + slot; r0 < hi; r0 += static_cast<int64_t>(RPB) * U) {
      float dv[U];
      f4h hv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t r = r0 + static_cast<int64_t>(u) * RPB;
        const int64_t rc = r < hi ? r : lo;
        dv[u] = dout[seg_rowptr ? seg_of_row(seg_rowptr, n_seg, rc) : rc];
        hv[u] = reinterpret_cast<const f4h*>(b.g[g].h)[rc * LPR + sub];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t r = r0 + static_cast<int64_t>(u) * RPB;
        if (r < hi) {
          aw += hv[u] * dv[u];
          ab += dv[u];
          if (b.g[g].dh) reinterpret_cast<f4h*>(b.g[g].dh)[r * LPR + sub] = wv * dv[u];
        }
      }
    }
    red[slot * LPR + sub] = aw;
    if (sub == 0) redb[slot] = ab;
    __syncthreads();
    float* pg = part + static_cast<int64_t>(g) * splits * (D + 1);
    if (threadIdx.x < LPR) {
      f4h s = {0.f, 0.f, 0.f, 0.f};
      for (int sl = 0; sl < RPB; ++sl) s += red[sl * LPR + threadIdx.x];
      reinterpret_cast<f4h*>(pg + static_cast<int64_t>(blockIdx.x) * D)[threadIdx.x] = s;
    }
    if (threadIdx.x == 0) {
      float s = 0.f;
      for (int sl = 0; sl < RPB; ++sl) s += redb[sl];
      pg[static_cast<int64_t>(splits) * D + blockIdx.x] = s;
    }
    __syncthreads();
  }
}

inline int head_splits(int64_t R) {
  const int64_t want = (R + 31) / 32;
  return static_cast<int>(want < kHeadSplits ? (want < 1 ? 1 : want) : kHeadSplits);
}

inline bool head_ok(const x2g_head_group* groups, int G, int D) {
  if (G < 1 || G > X2G_MAX_GROUPS || D % 4 || D < 4 || D > 256 || ((D / 4) & (D / 4 - 1))) return false;
  for (int g = 0; g < G; ++g)
    if (!groups[g].h || !groups[g].w || reinterpret_cast<uintptr_t>(groups[g].h) % 16 ||
        reinterpret_cast<uintptr_t>(groups[g].w) % 16 || reinterpret_cast<uintptr_t>(groups[g].dh) % 16)
      return false;
  return true;
}

}  // namespace x2g

using namespace x2g;

#define X2G_HEAD_DISPATCH(KERNEL, GRID, ...)                                     \
  switch (D / 4) {                                                               \
    case 1: KERNEL<1><<<GRID, 256, 0, st>>>(__VA_ARGS__); break;                 \
    case 2: KERNEL<2><<<GRID, 256, 0, st>>>(__VA_ARGS__); break;                 \
    case 4: KERNEL<4><<<GRID, 256, 0, st>>>(__VA_ARGS__); break;                 \
    case 8: KERNEL<8><<<GRID, 256, 0, st>>>(__VA_ARGS__); break;                 \
    case 16: KERNEL<16><<<GRID, 256, 0, st>>>(__VA_ARGS__); break;               \
    case 32: KERNEL<32><<<GRID, 256, 0, st>>>(__VA_ARGS__); break;               \
    default: KERNEL<64><<<GRID, 256, 0, st>>>(__VA_ARGS__); break;               \
  }

X2G_API int x2g_readout_head_fwd(const x2g_head_group* groups, int32_t G, int64_t R, int32_t D, float* out,
                                 void* stream) {
  if (R < 0 || !groups || !out) return X2G_EINVAL;
  if (!head_ok(groups, G, D)) return X2G_EUNSUPPORTED;
  if (R == 0) return X2G_OK;
  HeadBatch b{};
  for (int g = 0; g < G; ++g) b.g[g] = groups[g];
  hipStream_t st = as_stream(stream);
  const int64_t waves = (R * (D / 4) + 63) / 64;
  const unsigned grid = static_cast<unsigned>((waves + 3) / 4 < 2048 ? (waves + 3) / 4 : 2048);
  X2G_HEAD_DISPATCH(readout_head_fwd_kernel, grid, b, G, R, out)
  return last_launch_status();
}

X2G_API int32_t x2g_readout_head_bwd_splits(int64_t R) { return R > 0 ? head_splits(R) : 0; }

X2G_API size_t x2g_readout_head_bwd_workspace(int64_t R, int32_t D, int32_t G) {
  if (R <= 0 || D <= 0 || G <= 0) return 0;
  return static_cast<size_t>(G) * head_splits(R) * (D + 1) * sizeof(float);
}

static int head_bwd(const float* dout, const int32_t* seg_rowptr, int64_t n_seg, const x2g_head_group* groups,
                    int32_t G, int64_t R, int32_t D, int flags, void* ws, size_t wsb, void* stream) {
  if (R < 0 || !groups) return X2G_EINVAL;
  if (!head_ok(groups, G, D)) return X2G_EUNSUPPORTED;
  for (int g = 0; g < G; ++g)
    if (!groups[g].dw) return X2G_EINVAL;
  const bool accum = flags & X2G_ACCUM_WGRAD;
  hipStream_t st = as_stream(stream);
  if (R == 0) {
    if (flags & X2G_DEFER_SLAB_SUM) return X2G_EINVAL;
    if (accum) return X2G_OK;
    for (int g = 0; g < G; ++g) {
      hipError_t e = hipMemsetAsync(groups[g].dw, 0, sizeof(float) * D, st);
      if (e == hipSuccess && groups[g].db) e = hipMemsetAsync(groups[g].db, 0, sizeof(float), st);
      if (e != hipSuccess) return static_cast<int>(e);
    }
    return X2G_OK;
  }
  if (!dout) return X2G_EINVAL;
  if (!ws || wsb < x2g_readout_head_bwd_workspace(R, D, G)) return X2G_EWORKSPACE;
  HeadBatch b{};
  for (int g = 0; g < G; ++g) b.g[g] = groups[g];
  const int splits = head_splits(R);
  float* part = static_cast<float*>(ws);
  X2G_HEAD_DISPATCH(readout_head_bwd_kernel, dim3(splits, G), dout, b, G, R, part, seg_rowptr, n_seg)
  if (int rc = last_launch_status()) return rc;
  if (flags & X2G_DEFER_SLAB_SUM) return X2G_OK;
  x2g_slab_job jobs[X2G_MAX_GROUPS];
  for (int g = 0; g < G; ++g) {
    float* pg = part + static_cast<int64_t>(g) * splits * (D + 1);
    jobs[g] = x2g_slab_job{pg, groups[g].db ? pg + static_cast<int64_t>(splits) * D : nullptr, groups[g].dw,
                           groups[g].db, D, groups[g].db ? 1 : 0, splits};
  }
  return x2g_slab_sum_batch(jobs, G, accum ? 1 : 0, stream);
}

X2G_API int x2g_readout_head_bwd(const float* dout, const x2g_head_group* groups, int32_t G, int64_t R, int32_t D,
                                 int flags, void* ws, size_t wsb, void* stream) {
  return head_bwd(dout, nullptr, 0, groups, G, R, D, flags, ws, wsb, stream);
}

X2G_API int x2g_readout_head_pool_fwd(const x2g_head_group* groups, int32_t G, int64_t R, int32_t D,
                                      const int32_t* seg_rowptr, int64_t n_seg, float* out_seg, void* stream) {
  if (R < 0 || n_seg < 0 || !groups || !out_seg || (n_seg > 0 && !seg_rowptr)) return X2G_EINVAL;
  if (!head_ok(groups, G, D)) return X2G_EUNSUPPORTED;
  if (n_seg == 0) return X2G_OK;
  HeadBatch b{};
  for (int g = 0; g < G; ++g) b.g[g] = groups[g];
  hipStream_t st = as_stream(stream);
  const unsigned grid = static_cast<unsigned>(n_seg < 65535 ? n_seg : 65535);
  X2G_HEAD_DISPATCH(readout_head_pool_fwd_kernel, grid, b, G, seg_rowptr, n_seg, out_seg)
  return last_launch_status();
}

X2G_API int x2g_readout_head_pool_bwd(const float* dout_seg, const int32_t* seg_rowptr, int64_t n_seg,
                                      const x2g_head_group* groups, int32_t G, int64_t R, int32_t D, int flags,
                                      void* ws, size_t wsb, void* stream) {
  if (n_seg < 0 || (R > 0 && (n_seg < 1 || !seg_rowptr))) return X2G_EINVAL;
  return head_bwd(dout_seg, seg_rowptr, n_seg, groups, G, R, D, flags, ws, wsb, stream);
}

// ---------------------------------------------------------------- loss (trainer.py:41)
// F.smooth_l1_loss(pred, target) (reduction 'mean', beta) as one launch each way instead of
// torch's elementwise + mean (forward) and fill + fill + elementwise (backward): one 256-thread
// workgroup, per-thread sums then a fixed-order reduction (deterministic).
namespace x2g {
namespace {
constexpr int kLossThreads = 256;

// dpred (optional): the gradient for d loss = 1 (the backward kernel's values for gout = 1, same
// expression), written by the same pass
__global__ void __launch_bounds__(kLossThreads) smooth_l1_mean_fwd_kernel(const float* __restrict__ pred,
                                                                          const float* __restrict__ target, int64_t n,
                                                                          float beta, float* __restrict__ out,
                                                                          float* __restrict__ dpred) {
  __shared__ float red[kLossThreads / 64];
  float s = 0.f;
  const float g = 1.0f / static_cast<float>(n);
  for (int64_t i = threadIdx.x; i < n; i += kLossThreads) {
    const float d = pred[i] - target[i], a = fabsf(d);
    s += a < beta ? 0.5f * d * d / beta : a - 0.5f * beta;
    if (dpred) dpred[i] = g * (d < -beta ? -1.f : (d > beta ? 1.f : d / beta));
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = red[0];
#pragma unroll
    for (int w = 1; w < kLossThreads / 64; ++w) t += red[w];
    out[0] = t / static_cast<float>(n);
  }
}

__global__ void __launch_bounds__(kLossThreads) smooth_l1_mean_bwd_kernel(const float* __restrict__ pred,
                                                                          const float* __restrict__ target, int64_t n,
                                                                          float beta, const float* __restrict__ gout,
                                                                          float* __restrict__ dpred) {
  const float g = gout[0] / static_cast<float>(n);
  for (int64_t i = blockIdx.x * static_cast<int64_t>(kLossThreads) + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * kLossThreads) {
    const float d = pred[i] - target[i];
    dpred[i] = g * (d < -beta ? -1.f : (d > beta ? 1.f : d / beta));
  }
}
}  // namespace
}  // namespace x2g

X2G_API int x2g_smooth_l1_mean_fwd(const float* pred, const float* target, int64_t n, float beta, float* out,
                                   void* stream) {
  if (n <= 0 || !pred || !target || !out || !(beta > 0.f)) return X2G_EINVAL;
  x2g::smooth_l1_mean_fwd_kernel<<<1, x2g::kLossThreads, 0, as_stream(stream)>>>(pred, target, n, beta, out,
                                                                                 nullptr);
  return last_launch_status();
}

X2G_API int x2g_smooth_l1_mean_fwd_grad(const float* pred, const float* target, int64_t n, float beta, float* out,
                                        float* dpred_unit, void* stream) {
  if (n <= 0 || !pred || !target || !out || !dpred_unit || !(beta > 0.f)) return X2G_EINVAL;
  x2g::smooth_l1_mean_fwd_kernel<<<1, x2g::kLossThreads, 0, as_stream(stream)>>>(pred, target, n, beta, out,
                                                                                 dpred_unit);
  return last_launch_status();
}

X2G_API int x2g_smooth_l1_mean_bwd(const float* pred, const float* target, int64_t n, float beta, const float* gout,
                                   float* dpred, void* stream) {
  if (n <= 0 || !pred || !target || !gout || !dpred || !(beta > 0.f)) return X2G_EINVAL;
  const int64_t want = (n + x2g::kLossThreads - 1) / x2g::kLossThreads;
  x2g::smooth_l1_mean_bwd_kernel<<<static_cast<unsigned>(want < 1024 ? want : 1024), x2g::kLossThreads, 0,
                                   as_stream(stream)>>>(pred, target, n, beta, gout, dpred);
  return last_launch_status();
}
