// CSR segmented reductions: scatter-add, its adjoint broadcast, segment softmax, graph LayerNorm.
//
// These replace the torch_scatter 2.1.0 / PyG 2.1.0 operators X2-GNN reaches with sorted
// indices: scatter_add over edges by source atom (readout.py:37, AtomWise) and over atoms by
// molecule (model.py:190, the global add pool), scatter_mean (readout.py:69, MolWise),
// utils.softmax and nn.LayerNorm(mode='graph') (model.py:183).  Because every index here is
// sorted, each destination row is a contiguous segment [rowptr[g], rowptr[g+1]) and the sum
// is a fixed-order in-register reduction: no atomics, bitwise reproducible.
#include <math.h>

#include "common.hpp"

namespace x2g {

constexpr int kSegWaves = 4;
constexpr unsigned kSegMaxBlocks = 16384;

__device__ __forceinline__ float4 f4_fma(float4 a, float4 b, float4 c) {
  return make_float4(fmaf(a.x, b.x, c.x), fmaf(a.y, b.y, c.y), fmaf(a.z, b.z, c.z), fmaf(a.w, b.w, c.w));
}
__device__ __forceinline__ float4 f4_add(float4 a, float4 b) {
  return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}
__device__ __forceinline__ float4 f4_mul(float4 a, float4 b) {
  return make_float4(a.x * b.x, a.y * b.y, a.z * b.z, a.w * b.w);
}
__device__ __forceinline__ float4 f4_shfl_xor(float4 v, int off) {
  return make_float4(__shfl_xor(v.x, off, 64), __shfl_xor(v.y, off, 64), __shfl_xor(v.z, off, 64),
                     __shfl_xor(v.w, off, 64));
}

// ------------------------------------------------------------------------------ segment sum
// One wave per segment (grid-stride).  LPR = D/4 lanes cover a row with 16-byte loads, so a
// wave-instruction reads RPI = 64/LPR whole rows (D=128: two 512 B rows = 1 KiB).  Each lane
// issues UNROLL loads per batch unconditionally — rows past the segment end read a clamped row
// of the same segment and are zeroed by keep() — so a typical segment (T/E ~ 9 rows at S160)
// is one batch of 8 loads in flight per lane, one memory round trip.  The RPI partial rows are
// then folded with xor shuffles.  (A non-finite row stays non-finite in the sum, but a masked
// duplicate of an inf row contributes NaN instead of 0: both give a non-finite segment.)
template <int LPR, bool MUL>
__global__ void __launch_bounds__(256) seg_sum_vec(const float4* __restrict__ x, const float4* __restrict__ mul,
                                                   const int32_t* __restrict__ rowptr, int64_t G,
                                                   float4* __restrict__ out) {
  constexpr int RPI = 64 / LPR;
  constexpr int UNROLL = 8;
  const int lane = threadIdx.x & 63;
  const int sub = lane % LPR, slot = lane / LPR;
  const int nwaves = gridDim.x * kSegWaves;
  for (int64_t g = uniform(blockIdx.x * kSegWaves + (threadIdx.x >> 6)); g < G; g += nwaves) {
    const int r0 = uniform(rowptr[g]), r1 = uniform(rowptr[g + 1]);
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int rb = r0; rb < r1; rb += UNROLL * RPI) {
      float4 v[UNROLL], w[UNROLL];
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) {
        const int r = rb + u * RPI + slot;
        const int64_t idx = static_cast<int64_t>(r < r1 ? r : r1 - 1) * LPR + sub;
        v[u] = x[idx];
        if (MUL) w[u] = mul[idx];
      }
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) {
        const bool ok = rb + u * RPI + slot < r1;
        const float4 t = MUL ? f4_mul(v[u], w[u]) : v[u];
        acc.x += keep(t.x, ok);
        acc.y += keep(t.y, ok);
        acc.z += keep(t.z, ok);
        acc.w += keep(t.w, ok);
      }
    }
#pragma unroll
    for (int off = LPR; off < 64; off <<= 1) acc = f4_add(acc, f4_shfl_xor(acc, off));
    if (slot == 0) out[g * LPR + sub] = acc;
  }
}

// Any width: one thread per (segment, column), sequential over the segment's rows.
template <bool MUL>
__global__ void seg_sum_scalar(const float* __restrict__ x, const float* __restrict__ mul,
                               const int32_t* __restrict__ rowptr, int64_t G, int64_t D, float* __restrict__ out) {
  const int64_t gid = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (gid >= G * D) return;
  const int64_t g = gid / D, c = gid - g * D;
  float acc = 0.f;
  for (int64_t r = rowptr[g]; r < rowptr[g + 1]; ++r)
    acc = MUL ? fmaf(x[r * D + c], mul[r * D + c], acc) : acc + x[r * D + c];
  out[gid] = acc;
}

// ------------------------------------------------------------------------------ broadcast (adjoint)
template <int LPR, bool MUL>
__global__ void __launch_bounds__(256) seg_bcast_vec(const float4* __restrict__ g_in, const float4* __restrict__ mul,
                                                     const int32_t* __restrict__ rowptr, int64_t G,
                                                     float4* __restrict__ out) {
  constexpr int RPI = 64 / LPR;
  const int lane = threadIdx.x & 63;
  const int sub = lane % LPR, slot = lane / LPR;
  const int nwaves = gridDim.x * kSegWaves;
  for (int64_t g = uniform(blockIdx.x * kSegWaves + (threadIdx.x >> 6)); g < G; g += nwaves) {
    const int r0 = rowptr[g], r1 = rowptr[g + 1];
    if (r0 == r1) continue;
    const float4 gv = g_in[g * LPR + sub];
    for (int r = r0 + slot; r < r1; r += RPI) {
      const int64_t idx = static_cast<int64_t>(r) * LPR + sub;
      out[idx] = MUL ? f4_mul(gv, mul[idx]) : gv;
    }
  }
}

template <bool MUL>
__global__ void seg_bcast_scalar(const float* __restrict__ g_in, const float* __restrict__ mul,
                                 const int32_t* __restrict__ rowptr, int64_t G, int64_t D, float* __restrict__ out) {
  const int64_t gid = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (gid >= G * D) return;
  const int64_t g = gid / D, c = gid - g * D;
  const float gv = g_in[gid];
  for (int64_t r = rowptr[g]; r < rowptr[g + 1]; ++r) out[r * D + c] = MUL ? gv * mul[r * D + c] : gv;
}

unsigned seg_grid(int64_t G) {
  const int64_t want = (G + kSegWaves - 1) / kSegWaves;
  return static_cast<unsigned>(want < kSegMaxBlocks ? want : kSegMaxBlocks);
}

template <bool MUL>
int seg_sum_launch(const float* x, const float* mul, const int32_t* rowptr, int64_t G, int64_t D, float* out,
                   hipStream_t st) {
  const auto* xv = reinterpret_cast<const float4*>(x);
  const auto* mv = reinterpret_cast<const float4*>(mul);
  auto* ov = reinterpret_cast<float4*>(out);
  const unsigned grid = seg_grid(G);
  const bool aligned = (reinterpret_cast<uintptr_t>(x) % 16 == 0) && (reinterpret_cast<uintptr_t>(out) % 16 == 0) &&
                       (!MUL || reinterpret_cast<uintptr_t>(mul) % 16 == 0);
  switch (aligned ? D : -1) {
    case 4: seg_sum_vec<1, MUL><<<grid, 256, 0, st>>>(xv, mv, rowptr, G, ov); break;
    case 8: seg_sum_vec<2, MUL><<<grid, 256, 0, st>>>(xv, mv, rowptr, G, ov); break;
    case 16: seg_sum_vec<4, MUL><<<grid, 256, 0, st>>>(xv, mv, rowptr, G, ov); break;
    case 32: seg_sum_vec<8, MUL><<<grid, 256, 0, st>>>(xv, mv, rowptr, G, ov); break;
    case 64: seg_sum_vec<16, MUL><<<grid, 256, 0, st>>>(xv, mv, rowptr, G, ov); break;
    case 128: seg_sum_vec<32, MUL><<<grid, 256, 0, st>>>(xv, mv, rowptr, G, ov); break;
    case 256: seg_sum_vec<64, MUL><<<grid, 256, 0, st>>>(xv, mv, rowptr, G, ov); break;
    default: seg_sum_scalar<MUL><<<blocks_for(G * D, 256), 256, 0, st>>>(x, mul, rowptr, G, D, out); break;
  }
  return last_launch_status();
}

template <bool MUL>
int seg_bcast_launch(const float* g, const float* mul, const int32_t* rowptr, int64_t G, int64_t D, float* out,
                     hipStream_t st) {
  const auto* gv = reinterpret_cast<const float4*>(g);
  const auto* mv = reinterpret_cast<const float4*>(mul);
  auto* ov = reinterpret_cast<float4*>(out);
  const unsigned grid = seg_grid(G);
  const bool aligned = (reinterpret_cast<uintptr_t>(g) % 16 == 0) && (reinterpret_cast<uintptr_t>(out) % 16 == 0) &&
                       (!MUL || reinterpret_cast<uintptr_t>(mul) % 16 == 0);
  switch (aligned ? D : -1) {
    case 4: seg_bcast_vec<1, MUL><<<grid, 256, 0, st>>>(gv, mv, rowptr, G, ov); break;
    case 8: seg_bcast_vec<2, MUL><<<grid, 256, 0, st>>>(gv, mv, rowptr, G, ov); break;
    case 16: seg_bcast_vec<4, MUL><<<grid, 256, 0, st>>>(gv, mv, rowptr, G, ov); break;
    case 32: seg_bcast_vec<8, MUL><<<grid, 256, 0, st>>>(gv, mv, rowptr, G, ov); break;
    case 64: seg_bcast_vec<16, MUL><<<grid, 256, 0, st>>>(gv, mv, rowptr, G, ov); break;
    case 128: seg_bcast_vec<32, MUL><<<grid, 256, 0, st>>>(gv, mv, rowptr, G, ov); break;
    case 256: seg_bcast_vec<64, MUL><<<grid, 256, 0, st>>>(gv, mv, rowptr, G, ov); break;
    default: seg_bcast_scalar<MUL><<<blocks_for(G * D, 256), 256, 0, st>>>(g, mul, rowptr, G, D, out); break;
  }
  return last_launch_status();
}

// ------------------------------------------------------------------------------ permuted reductions
// The same segment walk for an index in ANY order: the caller sorts the keys (a stable sort on the
// device, no host read) and hands over the permutation; segment g's rows are x[perm[r]] for r in
// [rowptr[g], rowptr[g+1]), so a [R, D] source is read once in place instead of being gathered
// into sorted order first.  MEAN divides by max(count, 1) (torch_scatter scatter_mean: empty
// segments give 0).  The stable sort keeps each segment's rows in the caller's order: the sum is
// the fixed left-to-right order of a sorted index, bitwise reproducible.
template <int LPR, bool MEAN>
__global__ void __launch_bounds__(256) seg_reduce_perm_vec(const float4* __restrict__ x,
                                                           const int32_t* __restrict__ perm,
                                                           const int32_t* __restrict__ rowptr, int64_t G,
                                                           float4* __restrict__ out) {
  constexpr int RPI = 64 / LPR;
  constexpr int UNROLL = 8;
  const int lane = threadIdx.x & 63;
  const int sub = lane % LPR, slot = lane / LPR;
  const int nwaves = gridDim.x * kSegWaves;
  for (int64_t g = uniform(blockIdx.x * kSegWaves + (threadIdx.x >> 6)); g < G; g += nwaves) {
    const int r0 = uniform(rowptr[g]), r1 = uniform(rowptr[g + 1]);
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int rb = r0; rb < r1; rb += UNROLL * RPI) {
      int src[UNROLL];
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) {
        const int r = rb + u * RPI + slot;
        src[u] = perm[r < r1 ? r : r1 - 1];
      }
      float4 v[UNROLL];
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) v[u] = x[static_cast<int64_t>(src[u]) * LPR + sub];
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) {
        const bool ok = rb + u * RPI + slot < r1;
        acc.x += keep(v[u].x, ok);
        acc.y += keep(v[u].y, ok);
        acc.z += keep(v[u].z, ok);
        acc.w += keep(v[u].w, ok);
      }
    }
#pragma unroll
    for (int off = LPR; off < 64; off <<= 1) acc = f4_add(acc, f4_shfl_xor(acc, off));
    if (MEAN) {
      const float inv = 1.0f / static_cast<float>(r1 - r0 > 1 ? r1 - r0 : 1);
      acc = make_float4(acc.x * inv, acc.y * inv, acc.z * inv, acc.w * inv);
    }
    if (slot == 0) out[g * LPR + sub] = acc;
  }
}

template <bool MEAN>
__global__ void seg_reduce_perm_scalar(const float* __restrict__ x, const int32_t* __restrict__ perm,
                                       const int32_t* __restrict__ rowptr, int64_t G, int64_t D,
                                       float* __restrict__ out) {
  const int64_t gid = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (gid >= G * D) return;
  const int64_t g = gid / D, c = gid - g * D;
  const int64_t r0 = rowptr[g], r1 = rowptr[g + 1];
  float acc = 0.f;
  for (int64_t r = r0; r < r1; ++r) acc += x[static_cast<int64_t>(perm[r]) * D + c];
  out[gid] = MEAN ? acc / static_cast<float>(r1 - r0 > 1 ? r1 - r0 : 1) : acc;
}

// Adjoint: out[perm[r], :] = g[seg(r), :] (/ count for MEAN).  perm is a permutation, so no output
// row is written twice; rows outside every segment (keys outside [0, G)) are left as they are.
template <int LPR, bool MEAN>
__global__ void __launch_bounds__(256) seg_bcast_perm_vec(const float4* __restrict__ g_in,
                                                          const int32_t* __restrict__ perm,
                                                          const int32_t* __restrict__ rowptr, int64_t G,
                                                          float4* __restrict__ out) {
  constexpr int RPI = 64 / LPR;
  const int lane = threadIdx.x & 63;
  const int sub = lane % LPR, slot = lane / LPR;
  const int nwaves = gridDim.x * kSegWaves;
  for (int64_t g = uniform(blockIdx.x * kSegWaves + (threadIdx.x >> 6)); g < G; g += nwaves) {
    const int r0 = rowptr[g], r1 = rowptr[g + 1];
    if (r0 >= r1) continue;
    float4 gv = g_in[g * LPR + sub];
    if (MEAN) {
      const float inv = 1.0f / static_cast<float>(r1 - r0);
      gv = make_float4(gv.x * inv, gv.y * inv, gv.z * inv, gv.w * inv);
    }
    for (int r = r0 + slot; r < r1; r += RPI) out[static_cast<int64_t>(perm[r]) * LPR + sub] = gv;
  }
}

template <bool MEAN>
__global__ void seg_bcast_perm_scalar(const float* __restrict__ g_in, const int32_t* __restrict__ perm,
                                      const int32_t* __restrict__ rowptr, int64_t G, int64_t D,
                                      float* __restrict__ out) {
  const int64_t gid = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (gid >= G * D) return;
  const int64_t g = gid / D, c = gid - g * D;
  const int64_t r0 = rowptr[g], r1 = rowptr[g + 1];
  if (r0 >= r1) return;
  const float gv = MEAN ? g_in[gid] / static_cast<float>(r1 - r0) : g_in[gid];
  for (int64_t r = r0; r < r1; ++r) out[static_cast<int64_t>(perm[r]) * D + c] = gv;
}

template <bool MEAN, bool BCAST>
int seg_perm_launch(const float* in, const int32_t* perm, const int32_t* rowptr, int64_t G, int64_t D, float* out,
                    hipStream_t st) {
  const auto* iv = reinterpret_cast<const float4*>(in);
  auto* ov = reinterpret_cast<float4*>(out);
  const unsigned grid = seg_grid(G);
  const bool aligned = (reinterpret_cast<uintptr_t>(in) % 16 == 0) && (reinterpret_cast<uintptr_t>(out) % 16 == 0);
#define X2G_PERM_CASE(W, L)                                                                  \
  case W:                                                                                    \
    if (BCAST) seg_bcast_perm_vec<L, MEAN><<<grid, 256, 0, st>>>(iv, perm, rowptr, G, ov);  \
    else seg_reduce_perm_vec<L, MEAN><<<grid, 256, 0, st>>>(iv, perm, rowptr, G, ov);       \
    break;
  switch (aligned ? D : -1) {
    X2G_PERM_CASE(4, 1)
    X2G_PERM_CASE(8, 2)
    X2G_PERM_CASE(16, 4)
    X2G_PERM_CASE(32, 8)
    X2G_PERM_CASE(64, 16)
    X2G_PERM_CASE(128, 32)
    X2G_PERM_CASE(256, 64)
    default:
      if (BCAST) seg_bcast_perm_scalar<MEAN><<<blocks_for(G * D, 256), 256, 0, st>>>(in, perm, rowptr, G, D, out);
      else seg_reduce_perm_scalar<MEAN><<<blocks_for(G * D, 256), 256, 0, st>>>(in, perm, rowptr, G, D, out);
      break;
  }
#undef X2G_PERM_CASE
  return last_launch_status();
}

// ------------------------------------------------------------------------------ segment softmax
// perm == NULL: rows of segment g are [rowptr[g], rowptr[g+1]); otherwise perm[r] over that range.
__device__ __forceinline__ int64_t seg_row(const int32_t* perm, int64_t r) { return perm ? perm[r] : r; }

__global__ void seg_softmax_fwd_kernel(const float* __restrict__ src, const int32_t* __restrict__ perm,
                                       const int32_t* __restrict__ rowptr, int64_t G, int64_t H,
                                       float* __restrict__ out) {
  const int64_t gid = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (gid >= G * H) return;
  const int64_t g = gid / H, h = gid - g * H;
  const int64_t r0 = rowptr[g], r1 = rowptr[g + 1];
  float mx = -INFINITY;
  for (int64_t r = r0; r < r1; ++r) mx = fmaxf(mx, src[seg_row(perm, r) * H + h]);
  float sum = 0.f;
  for (int64_t r = r0; r < r1; ++r) sum += expf(src[seg_row(perm, r) * H + h] - mx);
  const float den = sum + 1e-16f;
  for (int64_t r = r0; r < r1; ++r) {
    const int64_t i = seg_row(perm, r) * H + h;
    out[i] = expf(src[i] - mx) / den;
  }
}

__global__ void seg_softmax_bwd_kernel(const float* __restrict__ out, const float* __restrict__ dout,
                                       const int32_t* __restrict__ perm, const int32_t* __restrict__ rowptr,
                                       int64_t G, int64_t H, float* __restrict__ dsrc) {
  const int64_t gid = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (gid >= G * H) return;
  const int64_t g = gid / H, h = gid - g * H;
  const int64_t r0 = rowptr[g], r1 = rowptr[g + 1];
  float dot = 0.f;
  for (int64_t r = r0; r < r1; ++r) {
    const int64_t i = seg_row(perm, r) * H + h;
    dot = fmaf(out[i], dout[i], dot);
  }
  for (int64_t r = r0; r < r1; ++r) {
    const int64_t i = seg_row(perm, r) * H + h;
    dsrc[i] = out[i] * (dout[i] - dot);
  }
}

// ------------------------------------------------------------------------------ graph LayerNorm
constexpr int kLnThreads = 256;

__device__ __forceinline__ float block_sum(float v, float* lds) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  if (lane == 0) lds[wave] = v;
  __syncthreads();
  float s = 0.f;
#pragma unroll
  for (int w = 0; w < kLnThreads / 64; ++w) s += lds[w];
  __syncthreads();
  return s;
}

// One 256-thread block per segment (molecule); the segment is swept three times (sum,
// centred sum of squares, write), re-reads served by L2.
__global__ void __launch_bounds__(kLnThreads) graph_ln_fwd_kernel(const float* __restrict__ x,
                                                                 const int32_t* __restrict__ rowptr, int64_t D,
                                                                 float eps, float* __restrict__ out,
                                                                 float* __restrict__ mean_out,
                                                                 float* __restrict__ rstd_out) {
  __shared__ float lds[kLnThreads / 64];
  const int64_t g = blockIdx.x;
  const int64_t r0 = rowptr[g], r1 = rowptr[g + 1];
  const int64_t n = r1 - r0, M = n * D;
  const float norm = static_cast<float>((n > 0 ? n : 1) * D);
  const float* xs = x + r0 * D;
  float* os = out + r0 * D;
  const bool vec = (D % 4 == 0) && (reinterpret_cast<uintptr_t>(xs) % 16 == 0) &&
                   (reinterpret_cast<uintptr_t>(os) % 16 == 0);
  float s = 0.f;
  if (vec) {
    for (int64_t i = threadIdx.x; i < M / 4; i += kLnThreads) {
      const float4 v = reinterpret_cast<const float4*>(xs)[i];
      s += (v.x + v.y) + (v.z + v.w);
    }
  } else {
    for (int64_t i = threadIdx.x; i < M; i += kLnThreads) s += xs[i];
  }
  const float mu = block_sum(s, lds) / norm;
  float q = 0.f;
  if (vec) {
    for (int64_t i = threadIdx.x; i < M / 4; i += kLnThreads) {
      const float4 v = reinterpret_cast<const float4*>(xs)[i];
      const float a = v.x - mu, b = v.y - mu, c = v.z - mu, d = v.w - mu;
      q += (a * a + b * b) + (c * c + d * d);
    }
  } else {
    for (int64_t i = threadIdx.x; i < M; i += kLnThreads) {
      const float a = xs[i] - mu;
      q += a * a;
    }
  }
  const float var = block_sum(q, lds) / norm;
  const float denom = sqrtf(var + eps);
  if (vec) {
    for (int64_t i = threadIdx.x; i < M / 4; i += kLnThreads) {
      const float4 v = reinterpret_cast<const float4*>(xs)[i];
      reinterpret_cast<float4*>(os)[i] =
          make_float4((v.x - mu) / denom, (v.y - mu) / denom, (v.z - mu) / denom, (v.w - mu) / denom);
    }
  } else {
    for (int64_t i = threadIdx.x; i < M; i += kLnThreads) os[i] = (xs[i] - mu) / denom;
  }
  if (threadIdx.x == 0) {
    mean_out[g] = mu;
    rstd_out[g] = 1.0f / denom;
  }
}

// dx = rstd * (dy - mean(dy) - y * mean(dy * y)), means over the segment's n*D elements.
__global__ void __launch_bounds__(kLnThreads) graph_ln_bwd_kernel(const float* __restrict__ y,
                                                                 const float* __restrict__ dy,
                                                                 const float* __restrict__ rstd,
                                                                 const int32_t* __restrict__ rowptr, int64_t D,
                                                                 float* __restrict__ dx) {
  __shared__ float lds[kLnThreads / 64];
  const int64_t g = blockIdx.x;
  const int64_t r0 = rowptr[g], r1 = rowptr[g + 1];
  const int64_t n = r1 - r0, M = n * D;
  if (n == 0) return;
  const float norm = static_cast<float>(n * D);
  const float* ys = y + r0 * D;
  const float* gs = dy + r0 * D;
  float* xs = dx + r0 * D;
  float s1 = 0.f, s2 = 0.f;
  for (int64_t i = threadIdx.x; i < M; i += kLnThreads) {
    const float gv = gs[i];
    s1 += gv;
    s2 = fmaf(gv, ys[i], s2);
  }
  const float m1 = block_sum(s1, lds) / norm;
  const float m2 = block_sum(s2, lds) / norm;
  const float r = rstd[g];
  for (int64_t i = threadIdx.x; i < M; i += kLnThreads) xs[i] = r * (gs[i] - m1 - ys[i] * m2);
}

// Register-resident graph LayerNorm for segments of up to 1024 * CAP float4 (a QM9 molecule:
// ~165 line nodes x 128 = 5.3k float4, CAP = 8): one 1024-thread block per molecule reads its
// rows ONCE into registers (16-byte loads, all in flight together), then the mean, the centred
// variance and the output come from registers — same two-pass arithmetic as graph_ln_fwd_kernel.
// Larger segments take the looping kernels above.
constexpr int kLnBig = 1024;

__device__ __forceinline__ float block_sum_big(float v, float* lds) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  if (lane == 0) lds[wave] = v;
  __syncthreads();
  float s = 0.f;
#pragma unroll
  for (int w = 0; w < kLnBig / 64; ++w) s += lds[w];
  __syncthreads();
  return s;
}

template <int CAP>
__global__ void __launch_bounds__(kLnBig) graph_ln_fwd_reg(const float4* __restrict__ x, const int32_t* __restrict__ rowptr,
                                                           int64_t D4, float eps, float4* __restrict__ out,
                                                           float* __restrict__ mean_out, float* __restrict__ rstd_out) {
  __shared__ float lds[kLnBig / 64];
  const int64_t g = blockIdx.x;
  const int64_t r0 = rowptr[g], r1 = rowptr[g + 1];
  const int64_t M4 = (r1 - r0) * D4;
  const float norm = static_cast<float>((r1 > r0 ? r1 - r0 : 1) * D4 * 4);
  const float4* xs = x + r0 * D4;
  float4* os = out + r0 * D4;
  if (M4 > static_cast<int64_t>(kLnBig) * CAP) {  // too big for registers: three sweeps
    float s = 0.f;
    for (int64_t i = threadIdx.x; i < M4; i += kLnBig) s += (xs[i].x + xs[i].y) + (xs[i].z + xs[i].w);
    const float mu = block_sum_big(s, lds) / norm;
    float q = 0.f;
    for (int64_t i = threadIdx.x; i < M4; i += kLnBig) {
      const float4 t = xs[i];
      const float a = t.x - mu, b = t.y - mu, c = t.z - mu, d = t.w - mu;
      q += (a * a + b * b) + (c * c + d * d);
    }
    const float denom = sqrtf(block_sum_big(q, lds) / norm + eps);
    for (int64_t i = threadIdx.x; i < M4; i += kLnBig) {
      const float4 t = xs[i];
      os[i] = make_float4((t.x - mu) / denom, (t.y - mu) / denom, (t.z - mu) / denom, (t.w - mu) / denom);
    }
    if (threadIdx.x == 0) {
      if (mean_out) mean_out[g] = mu;
      rstd_out[g] = 1.0f / denom;
    }
    return;
  }
  float4 v[CAP];
  float sum = 0.f;
#pragma unroll
  for (int u = 0; u < CAP; ++u) {
    const int64_t i = threadIdx.x + static_cast<int64_t>(kLnBig) * u;
    const bool ok = i < M4;
    const float4 t = xs[ok ? i : 0];
    v[u] = ok ? t : make_float4(0.f, 0.f, 0.f, 0.f);
  }
#pragma unroll
  for (int u = 0; u < CAP; ++u) sum += (v[u].x + v[u].y) + (v[u].z + v[u].w);
  const float mu = block_sum_big(sum, lds) / norm;
  float q = 0.f;
#pragma unroll
  for (int u = 0; u < CAP; ++u) {
    const int64_t i = threadIdx.x + static_cast<int64_t>(kLnBig) * u;
    if (i < M4) {
      const float a = v[u].x - mu, b = v[u].y - mu, c = v[u].z - mu, d = v[u].w - mu;
      q += (a * a + b * b) + (c * c + d * d);
    }
  }
  const float var = block_sum_big(q, lds) / norm;
  const float denom = sqrtf(var + eps);
#pragma unroll
  for (int u = 0; u < CAP; ++u) {
    const int64_t i = threadIdx.x + static_cast<int64_t>(kLnBig) * u;
    if (i < M4)
      os[i] = make_float4((v[u].x - mu) / denom, (v[u].y - mu) / denom, (v[u].z - mu) / denom, (v[u].w - mu) / denom);
  }
  if (threadIdx.x == 0) {
    if (mean_out) mean_out[g] = mu;
    rstd_out[g] = 1.0f / denom;
  }
}

template <int CAP>
__global__ void __launch_bounds__(kLnBig) graph_ln_bwd_reg(const float4* __restrict__ y, const float4* __restrict__ dy,
                                                           const float* __restrict__ rstd,
                                                           const int32_t* __restrict__ rowptr, int64_t D4,
                                                           float4* __restrict__ dx) {
  __shared__ float lds[kLnBig / 64];
  const int64_t g = blockIdx.x;
  const int64_t r0 = rowptr[g], r1 = rowptr[g + 1];
  if (r1 == r0) return;
  const int64_t M4 = (r1 - r0) * D4;
  const float norm = static_cast<float>((r1 - r0) * D4 * 4);
  const float4* ys = y + r0 * D4;
  const float4* gs = dy + r0 * D4;
  float4* xs = dx + r0 * D4;
  if (M4 > static_cast<int64_t>(kLnBig) * CAP) {  // too big for registers: two sweeps
    float a1 = 0.f, a2 = 0.f;
    for (int64_t i = threadIdx.x; i < M4; i += kLnBig) {
      const float4 gg = gs[i], yy = ys[i];
      a1 += (gg.x + gg.y) + (gg.z + gg.w);
      a2 = fmaf(gg.x, yy.x, a2);
      a2 = fmaf(gg.y, yy.y, a2);
      a2 = fmaf(gg.z, yy.z, a2);
      a2 = fmaf(gg.w, yy.w, a2);
    }
    const float m1 = block_sum_big(a1, lds) / norm;
    const float m2 = block_sum_big(a2, lds) / norm;
    const float r = rstd[g];
    for (int64_t i = threadIdx.x; i < M4; i += kLnBig) {
      const float4 gg = gs[i], yy = ys[i];
      xs[i] = make_float4(r * (gg.x - m1 - yy.x * m2), r * (gg.y - m1 - yy.y * m2), r * (gg.z - m1 - yy.z * m2),
                          r * (gg.w - m1 - yy.w * m2));
    }
    return;
  }
  float4 yv[CAP], gv[CAP];
#pragma unroll
  for (int u = 0; u < CAP; ++u) {
    const int64_t i = threadIdx.x + static_cast<int64_t>(kLnBig) * u;
    const bool ok = i < M4;
    const float4 a = ys[ok ? i : 0], b = gs[ok ? i : 0];
    const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
    yv[u] = ok ? a : z;
    gv[u] = ok ? b : z;
  }
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int u = 0; u < CAP; ++u) {
    s1 += (gv[u].x + gv[u].y) + (gv[u].z + gv[u].w);
    s2 = fmaf(gv[u].x, yv[u].x, s2);
    s2 = fmaf(gv[u].y, yv[u].y, s2);
    s2 = fmaf(gv[u].z, yv[u].z, s2);
    s2 = fmaf(gv[u].w, yv[u].w, s2);
  }
  const float m1 = block_sum_big(s1, lds) / norm;
  const float m2 = block_sum_big(s2, lds) / norm;
  const float r = rstd[g];
#pragma unroll
  for (int u = 0; u < CAP; ++u) {
    const int64_t i = threadIdx.x + static_cast<int64_t>(kLnBig) * u;
    if (i < M4)
      xs[i] = make_float4(r * (gv[u].x - m1 - yv[u].x * m2), r * (gv[u].y - m1 - yv[u].y * m2),
                          r * (gv[u].z - m1 - yv[u].z * m2), r * (gv[u].w - m1 - yv[u].w * m2));
  }
}

// Split backward (the default with a workspace): the one-block-per-molecule form runs 128 blocks
// at config 2 — half the CUs idle and each block's loads, two block reductions and stores in
// series (~23 us for 32 MB).  Here kLnSplit blocks share a molecule: a stats pass writes each
// block's (sum dy, sum dy*y) over its row range, an apply pass re-reads its range (MALL-hot) and
// sums the molecule's kLnSplit partials in block order (fixed order: deterministic).
constexpr int kLnSplit = 4;
constexpr int kLnSplitThreads = 256;
constexpr int kLnSplitUnroll = 4;
constexpr int kLnRowsUnroll = 8;  // graph_ln_bwd_apply_rows: a config-2 split (~41 rows x 32 float4) in one batch

__device__ __forceinline__ void ln_split_range(const int32_t* __restrict__ rowptr, int64_t D4, int64_t& g, int64_t& lo,
                                               int64_t& hi, int64_t& n) {
  g = blockIdx.x / kLnSplit;
  const int64_t s = blockIdx.x % kLnSplit;
  const int64_t r0 = rowptr[g], r1 = rowptr[g + 1];
  n = r1 - r0;
  lo = (r0 + n * s / kLnSplit) * D4;
  hi = (r0 + n * (s + 1) / kLnSplit) * D4;
}

__global__ void __launch_bounds__(kLnSplitThreads) graph_ln_bwd_stats(const float4* __restrict__ y,
                                                                      const float4* __restrict__ dy,
                                                                      const int32_t* __restrict__ rowptr, int64_t D4,
                                                                      float2* __restrict__ part) {
  __shared__ float2 lds[kLnSplitThreads / 64];
  int64_t g, lo, hi, n;
  ln_split_range(rowptr, D4, g, lo, hi, n);
  float s1 = 0.f, s2 = 0.f;
  for (int64_t i0 = lo + threadIdx.x; i0 < hi; i0 += kLnSplitThreads * kLnSplitUnroll) {
    float4 gv[kLnSplitUnroll], yv[kLnSplitUnroll];
#pragma unroll
    for (int u = 0; u < kLnSplitUnroll; ++u) {  // every load of the batch first (clamped, masked)
      const int64_t i = i0 + u * kLnSplitThreads;
      const int64_t ic = i < hi ? i : lo;
      gv[u] = dy[ic];
      yv[u] = y[ic];
    }
#pragma unroll
    for (int u = 0; u < kLnSplitUnroll; ++u) {
      if (i0 + u * kLnSplitThreads < hi) {
        s1 += (gv[u].x + gv[u].y) + (gv[u].z + gv[u].w);
        s2 = fmaf(gv[u].x, yv[u].x, s2);
        s2 = fmaf(gv[u].y, yv[u].y, s2);
        s2 = fmaf(gv[u].z, yv[u].z, s2);
        s2 = fmaf(gv[u].w, yv[u].w, s2);
      }
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    s1 += __shfl_xor(s1, off, 64);
    s2 += __shfl_xor(s2, off, 64);
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) lds[wave] = make_float2(s1, s2);
  __syncthreads();
  if (threadIdx.x == 0) {
    float2 t = lds[0];
#pragma unroll
    for (int w = 1; w < kLnSplitThreads / 64; ++w) {
      t.x += lds[w].x;
      t.y += lds[w].y;
    }
    part[blockIdx.x] = t;
  }
}

__global__ void __launch_bounds__(kLnSplitThreads) graph_ln_bwd_apply(const float4* __restrict__ y,
                                                                      const float4* __restrict__ dy,
                                                                      const float* __restrict__ rstd,
                                                                      const int32_t* __restrict__ rowptr, int64_t D4,
                                                                      const float2* __restrict__ part,
                                                                      float4* __restrict__ dx) {
  int64_t g, lo, hi, n;
  ln_split_range(rowptr, D4, g, lo, hi, n);
  if (n == 0) return;
  const float norm = static_cast<float>(n * D4 * 4);
  float2 t = part[g * kLnSplit];
#pragma unroll
  for (int s = 1; s < kLnSplit; ++s) {
    t.x += part[g * kLnSplit + s].x;
    t.y += part[g * kLnSplit + s].y;
  }
  const float m1 = t.x / norm, m2 = t.y / norm, r = rstd[g];
  for (int64_t i0 = lo + threadIdx.x; i0 < hi; i0 += kLnSplitThreads * kLnSplitUnroll) {
    float4 gv[kLnSplitUnroll], yv[kLnSplitUnroll];
#pragma unroll
    for (int u = 0; u < kLnSplitUnroll; ++u) {
      const int64_t i = i0 + u * kLnSplitThreads;
      const int64_t ic = i < hi ? i : lo;
      gv[u] = dy[ic];
      yv[u] = y[ic];
    }
#pragma unroll
    for (int u = 0; u < kLnSplitUnroll; ++u) {
      const int64_t i = i0 + u * kLnSplitThreads;
      if (i < hi)
        dx[i] = make_float4(r * (gv[u].x - m1 - yv[u].x * m2), r * (gv[u].y - m1 - yv[u].y * m2),
                            r * (gv[u].z - m1 - yv[u].z * m2), r * (gv[u].w - m1 - yv[u].w * m2));
    }
  }
}

// The apply pass from per-row sums (x2g_chain_bwd_ln's row_gstats: (sum_c dy, sum_c dy y) per row)
// instead of a stats pass over dy and y: each of the segment's kLnSplit blocks sums the segment's
// row pairs in the same fixed order (so every block holds identical molecule totals), then applies.
__global__ void __launch_bounds__(kLnSplitThreads) graph_ln_bwd_apply_rows(const float4* __restrict__ y,
                                                                           const float4* __restrict__ dy,
                                                                           const float* __restrict__ rstd,
                                                                           const int32_t* __restrict__ rowptr, int64_t D4,
                                                                           const float2* __restrict__ rows,
                                                                           float4* __restrict__ dx) {
  __shared__ float2 lds[kLnSplitThreads / 64];
  int64_t g, lo, hi, n;
  ln_split_range(rowptr, D4, g, lo, hi, n);
  if (n == 0) return;
  // the first batch of dy / y rows goes out before the molecule sums (it does not depend on them),
  // so the sums' round trip and barrier hide under its loads
  constexpr int U = kLnRowsUnroll;
  float4 gv[U], yv[U];
  int64_t i0 = lo + threadIdx.x;
  auto load_batch = [&](int64_t b) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = b + u * kLnSplitThreads;
      const int64_t ic = i < hi ? i : lo;  // b < hi, so lo < hi: a valid row of this split
      gv[u] = dy[ic];
      yv[u] = y[ic];
    }
  };
  if (i0 < hi) load_batch(i0);
  const int64_t r0 = rowptr[g];
  float s1 = 0.f, s2 = 0.f;
  for (int64_t r = threadIdx.x; r < n; r += kLnSplitThreads) {
    const float2 t = rows[r0 + r];
    s1 += t.x;
    s2 += t.y;
  }
  s1 = wave64_sum(s1);
  s2 = wave64_sum(s2);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) lds[wave] = make_float2(s1, s2);
  __syncthreads();
  float2 t = lds[0];
#pragma unroll
  for (int w = 1; w < kLnSplitThreads / 64; ++w) {
    t.x += lds[w].x;
    t.y += lds[w].y;
  }
  const float norm = static_cast<float>(n * D4 * 4);
  const float m1 = t.x / norm, m2 = t.y / norm, r = rstd[g];
  while (i0 < hi) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + u * kLnSplitThreads;
      if (i < hi)
        dx[i] = make_float4(r * (gv[u].x - m1 - yv[u].x * m2), r * (gv[u].y - m1 - yv[u].y * m2),
                            r * (gv[u].z - m1 - yv[u].z * m2), r * (gv[u].w - m1 - yv[u].w * m2));
    }
    i0 += kLnSplitThreads * U;
    if (i0 < hi) load_batch(i0);
  }
}

}  // namespace x2g

using namespace x2g;

X2G_API int x2g_segment_sum(const float* x, const float* mul, const int32_t* rowptr, int64_t G, int64_t D,
                            float* out, void* stream) {
  if (G < 0 || D <= 0 || (G > 0 && (!rowptr || !out || !x))) return X2G_EINVAL;
  if (G == 0) return X2G_OK;
  hipStream_t st = as_stream(stream);
  return mul ? seg_sum_launch<true>(x, mul, rowptr, G, D, out, st) : seg_sum_launch<false>(x, mul, rowptr, G, D, out, st);
}

X2G_API int x2g_segment_broadcast(const float* g, const float* mul, const int32_t* rowptr, int64_t G, int64_t D,
                                  float* out, void* stream) {
  if (G < 0 || D <= 0 || (G > 0 && (!rowptr || !out || !g))) return X2G_EINVAL;
  if (G == 0) return X2G_OK;
  hipStream_t st = as_stream(stream);
  return mul ? seg_bcast_launch<true>(g, mul, rowptr, G, D, out, st)
             : seg_bcast_launch<false>(g, mul, rowptr, G, D, out, st);
}

X2G_API int x2g_segment_softmax_fwd(const float* src, const int32_t* rowptr, int64_t G, int64_t H, float* out,
                                    void* stream) {
  if (G < 0 || H <= 0 || (G > 0 && (!src || !rowptr || !out))) return X2G_EINVAL;
  if (G == 0) return X2G_OK;
  seg_softmax_fwd_kernel<<<blocks_for(G * H, 256), 256, 0, as_stream(stream)>>>(src, nullptr, rowptr, G, H, out);
  return last_launch_status();
}

X2G_API int x2g_segment_softmax_bwd(const float* out, const float* dout, const int32_t* rowptr, int64_t G,
                                    int64_t H, float* dsrc, void* stream) {
  if (G < 0 || H <= 0 || (G > 0 && (!out || !dout || !rowptr || !dsrc))) return X2G_EINVAL;
  if (G == 0) return X2G_OK;
  seg_softmax_bwd_kernel<<<blocks_for(G * H, 256), 256, 0, as_stream(stream)>>>(out, dout, nullptr, rowptr, G, H,
                                                                                 dsrc);
  return last_launch_status();
}

X2G_API int x2g_segment_reduce_perm(const float* x, const int32_t* perm, const int32_t* rowptr, int64_t G, int64_t D,
                                    int mode, float* out, void* stream) {
  if (G < 0 || D <= 0 || (mode != X2G_REDUCE_SUM && mode != X2G_REDUCE_MEAN)) return X2G_EINVAL;
  if (G > 0 && (!rowptr || !out || !x || !perm)) return X2G_EINVAL;
  if (G == 0) return X2G_OK;
  hipStream_t st = as_stream(stream);
  return mode == X2G_REDUCE_MEAN ? seg_perm_launch<true, false>(x, perm, rowptr, G, D, out, st)
                                 : seg_perm_launch<false, false>(x, perm, rowptr, G, D, out, st);
}

X2G_API int x2g_segment_reduce_perm_bwd(const float* g, const int32_t* perm, const int32_t* rowptr, int64_t G,
                                        int64_t D, int mode, float* out, void* stream) {
  if (G < 0 || D <= 0 || (mode != X2G_REDUCE_SUM && mode != X2G_REDUCE_MEAN)) return X2G_EINVAL;
  if (G > 0 && (!rowptr || !out || !g || !perm)) return X2G_EINVAL;
  if (G == 0) return X2G_OK;
  hipStream_t st = as_stream(stream);
  return mode == X2G_REDUCE_MEAN ? seg_perm_launch<true, true>(g, perm, rowptr, G, D, out, st)
                                 : seg_perm_launch<false, true>(g, perm, rowptr, G, D, out, st);
}

X2G_API int x2g_segment_softmax_perm_fwd(const float* src, const int32_t* perm, const int32_t* rowptr, int64_t G,
                                         int64_t H, float* out, void* stream) {
  if (G < 0 || H <= 0 || (G > 0 && (!src || !perm || !rowptr || !out))) return X2G_EINVAL;
  if (G == 0) return X2G_OK;
  seg_softmax_fwd_kernel<<<blocks_for(G * H, 256), 256, 0, as_stream(stream)>>>(src, perm, rowptr, G, H, out);
  return last_launch_status();
}

X2G_API int x2g_segment_softmax_perm_bwd(const float* out, const float* dout, const int32_t* perm,
                                         const int32_t* rowptr, int64_t G, int64_t H, float* dsrc, void* stream) {
  if (G < 0 || H <= 0 || (G > 0 && (!out || !dout || !perm || !rowptr || !dsrc))) return X2G_EINVAL;
  if (G == 0) return X2G_OK;
  seg_softmax_bwd_kernel<<<blocks_for(G * H, 256), 256, 0, as_stream(stream)>>>(out, dout, perm, rowptr, G, H, dsrc);
  return last_launch_status();
}

namespace x2g {

constexpr int kKeyedMaxKeys = 16;
constexpr int kKeyedSplits = 256;

// block b sums rows [b * per, (b + 1) * per): row slot s (of 256 / LPR) adds its rows into its own
// LDS accumulator set acc[s][key][:] (lanes own disjoint 16-byte column chunks: no races), then the
// slots are folded in a fixed order into part[b][key][:]
constexpr int kKeyedMaxJobs = X2G_KEYED_MAX_JOBS;
struct KeyedJobs {  // job blockIdx.y: rows of src[j] summed by key into its slabs part[j]
  const float4* src[kKeyedMaxJobs];
  float4* part[kKeyedMaxJobs];
};

template <int LPR>
__global__ void __launch_bounds__(256) keyed_row_sum_partial(const KeyedJobs J, const int32_t* __restrict__ key,
                                                             int64_t rows, int nkeys) {
  const float4* __restrict__ src = J.src[blockIdx.y];
  float4* __restrict__ part = J.part[blockIdx.y];
  constexpr int RPB = 256 / LPR;
  __shared__ float4 acc[RPB * kKeyedMaxKeys * LPR];
  const int sub = threadIdx.x % LPR, slot = threadIdx.x / LPR;
  const int64_t per = (rows + gridDim.x - 1) / gridDim.x;
  const int64_t lo = per * blockIdx.x, hi = lo + per < rows ? lo + per : rows;
  constexpr int U = 4;
  float4 v[U];
  int k[U];
  auto load = [&](int64_t r0) {  // r0 < hi
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t r = r0 + u * RPB, rc = r < hi ? r : hi - 1;
      v[u] = src[rc * LPR + sub];
      k[u] = key[rc];
    }
  };
  int64_t r0 = lo + slot;
  if (r0 < hi) load(r0);  // the first rows fly while the accumulators are cleared
  for (int i = threadIdx.x; i < RPB * kKeyedMaxKeys * LPR; i += 256) acc[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  __syncthreads();
  float4* mine = acc + slot * kKeyedMaxKeys * LPR + sub;
  while (r0 < hi) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (r0 + u * RPB < hi) {
        float4& a = mine[k[u] * LPR];
        a.x += v[u].x;
        a.y += v[u].y;
        a.z += v[u].z;
        a.w += v[u].w;
      }
    }
    r0 += RPB * U;
    if (r0 < hi) load(r0);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < nkeys * LPR; i += 256) {
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int sl = 0; sl < RPB; ++sl) {
      const float4 a = acc[sl * kKeyedMaxKeys * LPR + i];
      s.x += a.x;
      s.y += a.y;
      s.z += a.z;
      s.w += a.w;
    }
    part[static_cast<int64_t>(blockIdx.x) * nkeys * LPR + i] = s;
  }
}

inline int keyed_splits(int64_t rows) {
  const int64_t want = (rows + 63) / 64;
  return static_cast<int>(want < kKeyedSplits ? (want < 1 ? 1 : want) : kKeyedSplits);
}

}  // namespace x2g

static int keyed_partial_launch(const KeyedJobs& J, int n_jobs, const int32_t* key, int64_t rows, int dim, int nkeys,
                                int splits, hipStream_t st) {
  const dim3 grid(static_cast<unsigned>(splits), static_cast<unsigned>(n_jobs));
  switch (dim / 4) {
    case 1: keyed_row_sum_partial<1><<<grid, 256, 0, st>>>(J, key, rows, nkeys); break;
    case 2: keyed_row_sum_partial<2><<<grid, 256, 0, st>>>(J, key, rows, nkeys); break;
    case 4: keyed_row_sum_partial<4><<<grid, 256, 0, st>>>(J, key, rows, nkeys); break;
    case 8: keyed_row_sum_partial<8><<<grid, 256, 0, st>>>(J, key, rows, nkeys); break;
    case 16: keyed_row_sum_partial<16><<<grid, 256, 0, st>>>(J, key, rows, nkeys); break;
    case 32: keyed_row_sum_partial<32><<<grid, 256, 0, st>>>(J, key, rows, nkeys); break;
    case 64: keyed_row_sum_partial<64><<<grid, 256, 0, st>>>(J, key, rows, nkeys); break;
    default: return X2G_EUNSUPPORTED;
  }
  return last_launch_status();
}

X2G_API size_t x2g_keyed_row_sum_workspace(int64_t rows, int32_t dim, int32_t nkeys) {
  if (rows <= 0 || dim <= 0 || nkeys <= 0) return 0;
  return static_cast<size_t>(keyed_splits(rows)) * dim * nkeys * sizeof(float);
}

X2G_API int x2g_keyed_row_sum(const float* src, const int32_t* key, int64_t rows, int32_t dim, int32_t nkeys,
                              float* out, int flags, void* ws, size_t wsb, void* stream) {
  if (rows < 0 || dim <= 0 || nkeys <= 0 || !out) return X2G_EINVAL;
  if (nkeys > kKeyedMaxKeys || dim % 4 != 0 || dim > 256) return X2G_EUNSUPPORTED;
  const bool accum = flags & X2G_ACCUM_WGRAD;
  hipStream_t st = as_stream(stream);
  if (rows == 0) {
    if (accum) return X2G_OK;
    const hipError_t e = hipMemsetAsync(out, 0, sizeof(float) * dim * nkeys, st);
    return e == hipSuccess ? X2G_OK : static_cast<int>(e);
  }
  if (!src || !key) return X2G_EINVAL;
  if (reinterpret_cast<uintptr_t>(src) % 16) return X2G_EINVAL;
  if (!ws || wsb < x2g_keyed_row_sum_workspace(rows, dim, nkeys)) return X2G_EWORKSPACE;
  const int splits = keyed_splits(rows);
  KeyedJobs J{};
  J.src[0] = reinterpret_cast<const float4*>(src);
  J.part[0] = static_cast<float4*>(ws);
  if (int rc = keyed_partial_launch(J, 1, key, rows, dim, nkeys, splits, st)) return rc;
  return sum_slabs_launch(static_cast<const float*>(ws), static_cast<int64_t>(dim) * nkeys, nullptr, 0, splits, out,
                          nullptr, accum, st);
}

X2G_API size_t x2g_keyed_row_sum_batch_workspace(int64_t rows, int32_t dim, int32_t nkeys, int32_t n_jobs) {
  return n_jobs > 0 ? static_cast<size_t>(n_jobs) * x2g_keyed_row_sum_workspace(rows, dim, nkeys) : 0;
}

X2G_API int x2g_keyed_row_sum_batch(const float* const* srcs, float* const* outs, int32_t n_jobs, const int32_t* key,
                                    int64_t rows, int32_t dim, int32_t nkeys, int flags, void* ws, size_t wsb,
                                    void* stream) {
  if (!srcs || !outs || n_jobs < 1 || n_jobs > kKeyedMaxJobs || rows <= 0 || dim <= 0 || nkeys <= 0 || !key)
    return X2G_EINVAL;
  if (nkeys > kKeyedMaxKeys || dim % 4 != 0 || dim > 256) return X2G_EUNSUPPORTED;
  if (!ws || wsb < x2g_keyed_row_sum_batch_workspace(rows, dim, nkeys, n_jobs)) return X2G_EWORKSPACE;
  hipStream_t st = as_stream(stream);
  const int splits = keyed_splits(rows);
  const int64_t per = static_cast<int64_t>(splits) * dim * nkeys;
  KeyedJobs J{};
  x2g_slab_job sj[kKeyedMaxJobs];
  for (int j = 0; j < n_jobs; ++j) {
    if (!srcs[j] || !outs[j] || reinterpret_cast<uintptr_t>(srcs[j]) % 16) return X2G_EINVAL;
    J.src[j] = reinterpret_cast<const float4*>(srcs[j]);
    float* part = static_cast<float*>(ws) + j * per;
    J.part[j] = reinterpret_cast<float4*>(part);
    sj[j] = x2g_slab_job{part, nullptr, outs[j], nullptr, static_cast<int64_t>(dim) * nkeys, 0, splits, 0, 0};
  }
  if (int rc = keyed_partial_launch(J, n_jobs, key, rows, dim, nkeys, splits, st)) return rc;
  return x2g_slab_sum_batch(sj, n_jobs, (flags & X2G_ACCUM_WGRAD) ? 1 : 0, stream);
}

X2G_API int x2g_graph_layernorm_fwd(const float* x, const int32_t* rowptr, int64_t G, int64_t D, float eps,
                                    float* out, float* mean, float* rstd, void* stream) {
  if (G < 0 || D <= 0 || (G > 0 && (!x || !rowptr || !out || !mean || !rstd))) return X2G_EINVAL;
  if (G == 0) return X2G_OK;
  if (D % 4 == 0 && reinterpret_cast<uintptr_t>(x) % 16 == 0 && reinterpret_cast<uintptr_t>(out) % 16 == 0)
    graph_ln_fwd_reg<8><<<static_cast<unsigned>(G), kLnBig, 0, as_stream(stream)>>>(
        reinterpret_cast<const float4*>(x), rowptr, D / 4, eps, reinterpret_cast<float4*>(out), mean, rstd);
  else
    graph_ln_fwd_kernel<<<static_cast<unsigned>(G), kLnThreads, 0, as_stream(stream)>>>(x, rowptr, D, eps, out, mean,
                                                                                       rstd);
  return last_launch_status();
}

X2G_API int x2g_graph_layernorm_bwd(const float* out, const float* dout, const float* rstd, const int32_t* rowptr,
                                    int64_t G, int64_t D, float* dx, void* stream) {
  if (G < 0 || D <= 0 || (G > 0 && (!out || !dout || !rstd || !rowptr || !dx))) return X2G_EINVAL;
  if (G == 0) return X2G_OK;
  if (D % 4 == 0 && reinterpret_cast<uintptr_t>(out) % 16 == 0 && reinterpret_cast<uintptr_t>(dout) % 16 == 0 &&
      reinterpret_cast<uintptr_t>(dx) % 16 == 0)
    graph_ln_bwd_reg<8><<<static_cast<unsigned>(G), kLnBig, 0, as_stream(stream)>>>(
        reinterpret_cast<const float4*>(out), reinterpret_cast<const float4*>(dout), rstd, rowptr, D / 4,
        reinterpret_cast<float4*>(dx));
  else
    graph_ln_bwd_kernel<<<static_cast<unsigned>(G), kLnThreads, 0, as_stream(stream)>>>(out, dout, rstd, rowptr, D,
                                                                                       dx);
  return last_launch_status();
}

X2G_API size_t x2g_graph_layernorm_bwd_workspace(int64_t G) {
  return G > 0 ? static_cast<size_t>(G) * kLnSplit * sizeof(float2) : 0;
}

X2G_API int x2g_graph_layernorm_bwd_ex(const float* out, const float* dout, const float* rstd, const int32_t* rowptr,
                                       int64_t G, int64_t D, float* dx, void* ws, size_t wsb, void* stream) {
  if (G < 0 || D <= 0 || (G > 0 && (!out || !dout || !rstd || !rowptr || !dx))) return X2G_EINVAL;
  if (G == 0) return X2G_OK;
  const bool vec = D % 4 == 0 && reinterpret_cast<uintptr_t>(out) % 16 == 0 &&
                   reinterpret_cast<uintptr_t>(dout) % 16 == 0 && reinterpret_cast<uintptr_t>(dx) % 16 == 0;
  if (!vec || !ws || wsb < x2g_graph_layernorm_bwd_workspace(G))
    return x2g_graph_layernorm_bwd(out, dout, rstd, rowptr, G, D, dx, stream);
  hipStream_t st = as_stream(stream);
  const unsigned grid = static_cast<unsigned>(G * kLnSplit);
  auto* part = static_cast<float2*>(ws);
  graph_ln_bwd_stats<<<grid, kLnSplitThreads, 0, st>>>(reinterpret_cast<const float4*>(out),
                                                       reinterpret_cast<const float4*>(dout), rowptr, D / 4, part);
  graph_ln_bwd_apply<<<grid, kLnSplitThreads, 0, st>>>(reinterpret_cast<const float4*>(out),
                                                       reinterpret_cast<const float4*>(dout), rstd, rowptr, D / 4, part,
                                                       reinterpret_cast<float4*>(dx));
  return last_launch_status();
}

X2G_API int x2g_graph_layernorm_bwd_rows(const float* out, const float* dout, const float* rstd, const int32_t* rowptr,
                                         int64_t G, int64_t D, const float* row_gstats, float* dx, void* stream) {
  if (G < 0 || D <= 0) return X2G_EINVAL;
  if (G == 0) return X2G_OK;
  if (!out || !dout || !rstd || !rowptr || !row_gstats || !dx) return X2G_EINVAL;
  if (D % 4 || reinterpret_cast<uintptr_t>(out) % 16 || reinterpret_cast<uintptr_t>(dout) % 16 ||
      reinterpret_cast<uintptr_t>(dx) % 16 || reinterpret_cast<uintptr_t>(row_gstats) % 8)
    return X2G_EUNSUPPORTED;
  const unsigned grid = static_cast<unsigned>(G * kLnSplit);
  graph_ln_bwd_apply_rows<<<grid, kLnSplitThreads, 0, as_stream(stream)>>>(
      reinterpret_cast<const float4*>(out), reinterpret_cast<const float4*>(dout), rstd, rowptr, D / 4,
      reinterpret_cast<const float2*>(row_gstats), reinterpret_cast<float4*>(dx));
  return last_launch_status();
}
