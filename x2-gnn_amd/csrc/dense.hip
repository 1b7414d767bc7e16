// Row-wise dense layers with fused epilogues (f32 MFMA).
//
// X2-GNN's trunk is a chain of small Linear layers applied row-wise to E line nodes (or N atoms):
// q/k/v/skip projections, ResidualLayer = x + SiLU(W1 SiLU(W0 x + b0) + b1), SiLU(dense) + residual,
// readout MLPs (residual_layer.py:21-27, model.py:39-50, readout.py:38-42,
// sbftransformer_conv.py:99-107,127).  Through PyTorch each is a hipBLASLt GEMM followed by
// separate bias / SiLU / add kernels (and the same again in the backward); here one kernel does
//      Y = act(X W^T + b) (+ res),   Z = X W^T + b saved for the backward when act != none,
// and the backward's data gradient is one kernel too:
//      dZ = dY * act'(Z) (written out for the weight gradient),   dX = dZ W.
//
// Tiling: a 256-thread workgroup owns 64 rows x 128 output columns; wave w computes columns
// 32w..32w+31 for two 32-row MFMA tiles (v_mfma_f32_32x32x2_f32, exact fp32).  K is streamed in
// 32-wide chunks through LDS with the next chunk prefetched into registers during the MFMAs.
#include <math.h>

#include "common.hpp"

namespace x2g {

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int kDenseRows = 64;
constexpr int kDenseCols = 128;
constexpr int kDenseK = 32;
constexpr int kAStride = kDenseK + 1;     // A tile [64][33]: conflict-free column reads
constexpr int kBStride = kDenseCols + 1;  // B tile [32][129]: conflict-free transposed stores

enum Act { kActNone = 0, kActSilu = 1 };

__device__ __forceinline__ float sigmoidf_(float z) { return 1.0f / (1.0f + expf(-z)); }

// B operand element (k, n): BT -> stored as Bm[n][k] (a torch Linear weight [N, K]),
// else Bm[k][n] (the same weight read as [K', N'] for the data gradient).
template <bool BT, int ACT_IN>
__global__ void __launch_bounds__(256) dense_rows(const float* __restrict__ A, const float* __restrict__ Bm,
                                                  const float* __restrict__ bias, const float* __restrict__ res,
                                                  const float* __restrict__ zin, int64_t R, int K, int N, int act,
                                                  float* __restrict__ Y, float* __restrict__ zout,
                                                  float* __restrict__ aout) {
  __shared__ float As[kDenseRows][kAStride];
  __shared__ float Bs[kDenseK][kBStride];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t m0 = static_cast<int64_t>(blockIdx.x) * kDenseRows;
  const int n0 = blockIdx.y * kDenseCols;
  const bool write_a = aout != nullptr && blockIdx.y == 0;
  floatx16 acc0, acc1;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    acc0[j] = 0.f;
    acc1[j] = 0.f;
  }
  float ra[8], rb[16];
  auto load = [&](int k0) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {  // A chunk: 64 rows x 32 k, row-contiguous reads
      const int q = tid + 256 * u, rr = q >> 5, kk = q & 31;
      const int64_t r = m0 + rr;
      const int k = k0 + kk;
      const int64_t o = (r < R ? r : R - 1) * K + (k < K ? k : K - 1);
      float v = ld_pin(A + o);
      if (ACT_IN == kActSilu) {  // dZ = dY * silu'(Z)
        const float z = ld_pin(zin + o);
        const float s = sigmoidf_(z);
        v = v * (s * (1.0f + z * (1.0f - s)));
      }
      ra[u] = keep(v, r < R && k < K);
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) {  // B chunk: 32 k x 128 n
      const int q = tid + 256 * u;
      int kk, nn;
      if (BT) {
        nn = q >> 5;
        kk = q & 31;
      } else {
        kk = q >> 7;
        nn = q & 127;
      }
      const int k = k0 + kk, n = n0 + nn;
      const int kc = k < K ? k : K - 1, nc = n < N ? n : N - 1;
      const float v = ld_pin(BT ? Bm + static_cast<int64_t>(nc) * K + kc : Bm + static_cast<int64_t>(kc) * N + nc);
      rb[u] = keep(v, k < K && n < N);
    }
  };
  auto store = [&](int k0) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int q = tid + 256 * u, rr = q >> 5, kk = q & 31;
      As[rr][kk] = ra[u];
      if (write_a) {
        const int64_t r = m0 + rr;
        const int k = k0 + kk;
        if (r < R && k < K) aout[r * K + k] = ra[u];
      }
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int q = tid + 256 * u;
      if (BT) Bs[q & 31][q >> 5] = rb[u];
      else Bs[q >> 7][q & 127] = rb[u];
    }
  };
  load(0);
  for (int k0 = 0; k0 < K; k0 += kDenseK) {
    store(k0);
    __syncthreads();
    if (k0 + kDenseK < K) load(k0 + kDenseK);
#pragma unroll 4
    for (int ks = 0; ks < kDenseK / 2; ++ks) {
      const int kr = 2 * ks + (lane >> 5);
      const float b = Bs[kr][wave * 32 + (lane & 31)];
      const float a0 = As[lane & 31][kr];
      const float a1 = As[32 + (lane & 31)][kr];
      acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b, acc1, 0, 0, 0);
    }
    __syncthreads();
  }
  // epilogue: accumulator (j) -> row (j&3) + 8(j>>2) + 4(lane>>5) of the tile, column lane&31
  const int n = n0 + wave * 32 + (lane & 31);
  if (n >= N) return;
  const float bn = bias ? bias[n] : 0.f;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int64_t r = m0 + 32 * t + (j & 3) + 8 * (j >> 2) + 4 * (lane >> 5);
      if (r >= R) continue;
      float v = (t == 0 ? acc0[j] : acc1[j]) + bn;
      const int64_t o = r * N + n;
      if (zout) zout[o] = v;
      if (act == kActSilu) v = v / (1.0f + expf(-v));
      if (res) v += res[o];
      Y[o] = v;
    }
  }
}


// ------------------------------------------------------------------------------------------------
// Persistent forms for the common case K <= 128 and N <= 128 (every 128x128 layer, lin_rbf with
// K = 6, the readout head with N = 1): the weight is staged into LDS ONCE per workgroup (one
// 8-wave workgroup per CU) and the waves walk row tiles with the next tile's loads in flight.
//
// MFMA v_mfma_f32_32x32x2_f32, step s: lane l = (h = l >> 5, i = l & 31) supplies A[i][c] and
// B[c][i'] for contraction index c = cmap(s, h).  Any bijection works as long as A and B agree:
//   STEPS = 64 (c < 128): c = 64 h + s  -> a lane's A values are 64 CONTIGUOUS floats of one row;
//   STEPS = 4  (c < 8)  : c = 2 s + h.
// The weight lives in LDS in "slot" layout: B[cmap(s, h)][j] at (s * 128 + j) * 2 + h, so a B
// fragment is 64 consecutive floats (no bank conflicts, no padding).
template <int STEPS>
__device__ __forceinline__ int cmap(int s, int h) { return STEPS == 64 ? 64 * h + s : 2 * s + h; }

// Weight -> slot layout.  FWD: B[c][j] = w[j][c] (x w^T);  else B[c][j] = w[c][j] (dz w).
// Thread (j = idx & 127, s = idx >> 7) writes its two h values as one 8-byte LDS word; all loads
// are issued before the first LDS write.
template <int STEPS, bool FWD, int NT>
__device__ __forceinline__ void wslot_load(const float* __restrict__ W, int N, int K, float (&v)[16384 / NT]) {
#pragma unroll
  for (int u = 0; u < 8192 / NT; ++u) {
    const int idx = threadIdx.x + NT * u, j = idx & 127, sl = idx >> 7;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int c = cmap<STEPS>(sl, h);
      const int n = FWD ? j : c, k = FWD ? c : j;
      const float x = ld_pin(W + static_cast<int64_t>(n < N ? n : N - 1) * K + (k < K ? k : K - 1));
      v[2 * u + h] = (n < N && k < K) ? x : 0.f;
    }
  }
}

template <int NT>
__device__ __forceinline__ void wslot_store(float* __restrict__ ws, const float (&v)[16384 / NT]) {
#pragma unroll
  for (int u = 0; u < 8192 / NT; ++u) {
    const int idx = threadIdx.x + NT * u, j = idx & 127, sl = idx >> 7;
    *reinterpret_cast<float2*>(ws + (sl * 128 + j) * 2) = make_float2(v[2 * u], v[2 * u + 1]);
  }
}

// 16 values of a row-major [R, N] matrix in the MFMA C/D layout of rows [r0, r0+32), column n
// (rows clamped, so the loads are unconditional).
__device__ __forceinline__ void cfrag_load(const float* __restrict__ m, int64_t r0, int64_t R, int N, int n,
                                           float (&v)[16]) {
  const int lane = threadIdx.x & 63;
  // 32-bit offsets (the host guarantees R * max(K, N) < 2^31): 64-bit addresses hoisted out of
  // the tile loop would not fit in the register budget
  const int nc = n < N ? n : N - 1;
  const int rb = static_cast<int>(r0) + 4 * (lane >> 5), rmax = static_cast<int>(R) - 1;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int r = rb + (j & 3) + 8 * (j >> 2);
    v[j] = ld_pin(m + ((r < rmax ? r : rmax) * N + nc));
  }
}

// ---------------------------------------------------------------------------------- forward
constexpr int kPTile = 32;     // forward rows per tile
constexpr int kPFwdGrid = 256;  // one 8-wave workgroup per CU

// A fragment of rows [r0, r0+32) straight from global memory into registers: a[s] = X[row][cmap(s,h)]
// (rows and columns clamped: a clamped column meets a zero weight, a clamped row is not stored).
template <int STEPS, bool VEC>
__device__ __forceinline__ void afrag_load(const float* __restrict__ X, int64_t r0, int64_t R, int K,
                                           float (&a)[STEPS]) {
  const int lane = threadIdx.x & 63, h = lane >> 5;
  const int r = static_cast<int>(r0) + (lane & 31), rmax = static_cast<int>(R) - 1;
  const float* row = X + (r < rmax ? r : rmax) * K;
  if (STEPS == 64 && VEC) {  // 16 float4 per lane (K % 4 == 0, 16-byte aligned rows)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int c = 64 * h + 4 * i;
      const float4 v = *reinterpret_cast<const float4*>(row + (c + 4 <= K ? c : K - 4));
      a[4 * i] = v.x;
      a[4 * i + 1] = v.y;
      a[4 * i + 2] = v.z;
      a[4 * i + 3] = v.w;
    }
  } else {
#pragma unroll
    for (int s = 0; s < STEPS; ++s) {
      const int c = cmap<STEPS>(s, h);
      a[s] = ld_pin(row + (c < K ? c : K - 1));
    }
  }
}

template <int STEPS, bool VEC>
__device__ __forceinline__ void fwd_tile(const float* __restrict__ Ws, const float* __restrict__ X,
                                         const float* __restrict__ res, int64_t t, int64_t R, int K, int N, int act,
                                         int n, float bn, float* __restrict__ Y, float* __restrict__ Z) {
  const int lane = threadIdx.x & 63, h = lane >> 5;
  float a[STEPS], rv[16];
  afrag_load<STEPS, VEC>(X, t * kPTile, R, K, a);
  if (res) cfrag_load(res, t * kPTile, R, N, n, rv);
  floatx16 acc0, acc1;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    acc0[j] = 0.f;
    acc1[j] = 0.f;
  }
  const float* wb = Ws + n * 2 + h;
#pragma unroll
  for (int s = 0; s < STEPS; s += 2) {
    acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s], wb[s * 256], acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s + 1], wb[(s + 1) * 256], acc1, 0, 0, 0);
  }
  const int rbase = static_cast<int>(t) * kPTile + 4 * h;
  if (n < N) {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int r = rbase + (j & 3) + 8 * (j >> 2);
      const float zv = acc0[j] + acc1[j] + bn;
      float v = act == kActSilu ? zv / (1.0f + expf(-zv)) : zv;
      if (res) v += rv[j];
      if (r < R) {
        if (Z) Z[r * N + n] = zv;
        Y[r * N + n] = v;
      }
    }
  }
}

// y = act(x w^T + b) (+ res), z = x w^T + b.  8 waves: wave w computes output columns
// 32 (w & 3).. of every other 32-row tile (tile slot w >> 2), its A operand loaded from global
// memory straight into registers, its B operand read from the LDS weight.  After the weight is
// staged the waves never synchronise: with two waves per SIMD one multiplies while the other
// waits for its tile.
template <int STEPS, bool VEC>
__global__ void __launch_bounds__(512) dense_fwd_persist(const float* __restrict__ X, const float* __restrict__ W,
                                                         const float* __restrict__ bias,
                                                         const float* __restrict__ res, int64_t R, int K, int N,
                                                         int act, float* __restrict__ Y, float* __restrict__ Z) {
  __shared__ __attribute__((aligned(16))) float Ws[64 * 128 * 2];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n = 32 * (wave & 3) + (lane & 31);
  const int64_t ntiles = (R + kPTile - 1) / kPTile;
  const int64_t step = 2 * static_cast<int64_t>(gridDim.x);
  const float bn = (bias && n < N) ? bias[n] : 0.f;
  {
    float wv[32];
    wslot_load<STEPS, true, 512>(W, N, K, wv);
    wslot_store<512>(Ws, wv);
    __syncthreads();
  }
  for (int64_t t = 2 * static_cast<int64_t>(blockIdx.x) + (wave >> 2); t < ntiles; t += step)
    fwd_tile<STEPS, VEC>(Ws, X, res, t, R, K, N, act, n, bn, Y, Z);
}

// ---------------------------------------------------------------------------------- backward
// Backward of dense_fwd_persist, fused: dz = dy * act'(z); dx = dz w (if dx != NULL); partial
// weight / bias gradients dz^T x and colsum(dz) over the workgroup's tiles, written to slab
// blockIdx.x (summed afterwards in a fixed order).  8 waves, 64-row tiles staged through LDS
// with row stride 130 (32 rows at columns c, c+1: 64 distinct banks; rows r and r+16 over 32
// consecutive columns: 64 distinct banks):
//   dx: wave w -> rows 32 (w >> 2).., k columns 32 (w & 3)..   (cmap c = 2s + h)
//   dW: wave w -> n rows 32 (w & 3).., k columns 64 (w >> 2).. (rows paired r, r+16)
// NSTEPS: N <= 2*NSTEPS.  LDS: weight 64 KB + dz and x tiles 33 KB each.
constexpr int kBTile = 64;
constexpr int kBwdStride = 130;
constexpr int kPBwdGrid = 256;
constexpr int kBPer = kBTile * 128 / 512;  // tile values per thread

// 64 rows x 128 columns of a row-major [R, cols] matrix, 16 raw (clamped) loads per thread.
__device__ __forceinline__ void btile_load(const float* __restrict__ m, int64_t r0, int64_t R, int cols,
                                           float (&v)[kBPer]) {
#pragma unroll
  for (int u = 0; u < kBPer; ++u) {
    const int idx = threadIdx.x + 512 * u, rr = idx >> 7, cc = idx & 127;
    const int r = static_cast<int>(r0) + rr, rmax = static_cast<int>(R) - 1;
    v[u] = ld_pin(m + ((r < rmax ? r : rmax) * cols + (cc < cols ? cc : cols - 1)));
  }
}

// ... and into LDS, rows >= R and columns >= cols zeroed (a select, no branch)
__device__ __forceinline__ void btile_store(float* __restrict__ lds, const float (&v)[kBPer], int64_t r0, int64_t R,
                                            int cols) {
  const bool col_ok = static_cast<int>(threadIdx.x & 127) < cols;
#pragma unroll
  for (int u = 0; u < kBPer; ++u) {
    const int idx = threadIdx.x + 512 * u, rr = idx >> 7, cc = idx & 127;
    lds[rr * kBwdStride + cc] = (col_ok && r0 + rr < R) ? v[u] : 0.f;
  }
}

struct BwdRegs {
  float d[kBPer];
  float z[kBPer];
  float x[kBPer];
};

__device__ __forceinline__ void bwd_regs_load(BwdRegs& S, const float* __restrict__ dY, const float* __restrict__ Zin,
                                              const float* __restrict__ X, int64_t t, int64_t R, int K, int N,
                                              int act) {
  btile_load(dY, t * kBTile, R, N, S.d);
  if (act == kActSilu) btile_load(Zin, t * kBTile, R, N, S.z);
  btile_load(X, t * kBTile, R, K, S.x);
}

template <int NSTEPS>
__device__ __forceinline__ void bwd_tile(float* __restrict__ Ds, float* __restrict__ Xs, const float* __restrict__ Ws,
                                         BwdRegs& cur, BwdRegs& nxt, const float* __restrict__ dY,
                                         const float* __restrict__ Zin, const float* __restrict__ X, int64_t t,
                                         int64_t G, int64_t ntiles, int64_t R, int K, int N, int act,
                                         float* __restrict__ dX, floatx16 (&accw)[2], float& bsum, bool do_bias) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5, i = lane & 31;
  if (act == kActSilu) {
#pragma unroll
    for (int u = 0; u < kBPer; ++u) {
      const float s = 1.0f / (1.0f + expf(-cur.z[u]));
      cur.d[u] = cur.d[u] * (s * (1.0f + cur.z[u] * (1.0f - s)));
    }
  }
  btile_store(Ds, cur.d, t * kBTile, R, N);
  btile_store(Xs, cur.x, t * kBTile, R, K);
  __syncthreads();
  if (t + G < ntiles) bwd_regs_load(nxt, dY, Zin, X, t + G, R, K, N, act);
  if (dX) {  // dx tile: rows rt.., k columns 32 cb..; contraction over n = 2s + h
    const int rt = 32 * (wave >> 2), k = 32 * (wave & 3) + i;
    floatx16 acc0, acc1;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      acc0[j] = 0.f;
      acc1[j] = 0.f;
    }
    const float* ab = Ds + (rt + i) * kBwdStride + h;
    const float* wb = Ws + k * 2 + h;
#pragma unroll
    for (int s = 0; s < NSTEPS; s += 2) {
      acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(ab[2 * s], wb[s * 256], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(ab[2 * s + 2], wb[(s + 1) * 256], acc1, 0, 0, 0);
    }
    if (k < K) {
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int r = static_cast<int>(t) * kBTile + rt + (j & 3) + 8 * (j >> 2) + 4 * h;
        if (r < R) dX[r * K + k] = acc0[j] + acc1[j];
      }
    }
  }
  // dW[n][k] += sum_r dz[r][n] x[r][k]; step s covers rows (s & 15) + 32 (s >> 4) and +16
  const int nb = 32 * (wave & 3), kb = 64 * (wave >> 2);
  const float* db_ = Ds + 16 * h * kBwdStride + nb + i;
  const float* xb_ = Xs + 16 * h * kBwdStride + kb + i;
#pragma unroll 8
  for (int s = 0; s < kBTile / 2; ++s) {
    const int ro = ((s & 15) + 32 * (s >> 4)) * kBwdStride;
    const float a = db_[ro];
    accw[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, xb_[ro], accw[0], 0, 0, 0);
    accw[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, xb_[ro + 32], accw[1], 0, 0, 0);
  }
  if (do_bias && tid < 128) {
#pragma unroll 8
    for (int rr = 0; rr < kBTile; ++rr) bsum += Ds[rr * kBwdStride + tid];
  }
  __syncthreads();  // Ds / Xs are rewritten by the next tile
}

template <int NSTEPS>
__global__ void __launch_bounds__(512) dense_bwd_persist(const float* __restrict__ dY, const float* __restrict__ Zin,
                                                         const float* __restrict__ X, const float* __restrict__ W,
                                                         int64_t R, int K, int N, int act, float* __restrict__ dX,
                                                         float* __restrict__ part_w, float* __restrict__ part_b) {
  __shared__ __attribute__((aligned(16))) float Ws[64 * 128 * 2];
  __shared__ float Ds[kBTile * kBwdStride];
  __shared__ float Xs[kBTile * kBwdStride];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t ntiles = (R + kBTile - 1) / kBTile;
  const int64_t G = gridDim.x;
  floatx16 accw[2];
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int j = 0; j < 16; ++j) accw[q][j] = 0.f;
  float bsum = 0.f;
  int64_t t = blockIdx.x;
  BwdRegs A, B;
  {
    float wv[32];
    if (dX) wslot_load<4, false, 512>(W, N, K, wv);  // cmap<4>: c = 2s + h, for any s < 64
    bwd_regs_load(A, dY, Zin, X, t, R, K, N, act);
    if (dX) wslot_store<512>(Ws, wv);
  }
  const bool do_bias = part_b != nullptr;
  for (; t < ntiles; t += 2 * G) {
    bwd_tile<NSTEPS>(Ds, Xs, Ws, A, B, dY, Zin, X, t, G, ntiles, R, K, N, act, dX, accw, bsum, do_bias);
    if (t + G >= ntiles) break;
    bwd_tile<NSTEPS>(Ds, Xs, Ws, B, A, dY, Zin, X, t + G, G, ntiles, R, K, N, act, dX, accw, bsum, do_bias);
  }
  float* slab = part_w + static_cast<int64_t>(blockIdx.x) * N * K;
  const int nb = 32 * (wave & 3), kb = 64 * (wave >> 2);
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int k = kb + 32 * q + (lane & 31);
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int nn = nb + (j & 3) + 8 * (j >> 2) + 4 * (lane >> 5);
      if (nn < N && k < K) slab[static_cast<int64_t>(nn) * K + k] = accw[q][j];
    }
  }
  if (part_b && tid < N) part_b[static_cast<int64_t>(blockIdx.x) * N + tid] = bsum;
}

}  // namespace x2g

using namespace x2g;

X2G_API int x2g_dense_fwd(const float* x, const float* w, const float* b, int64_t R, int32_t K, int32_t N, int act,
                          const float* res, float* y, float* z, void* stream) {
  if (R < 0 || K <= 0 || N <= 0 || (act != kActNone && act != kActSilu)) return X2G_EINVAL;
  if (R == 0) return X2G_OK;
  if (!x || !w || !y) return X2G_EINVAL;
  hipStream_t st = as_stream(stream);
  const int variant = tuning(kTuneDenseFwd);  // 0: persistent (default), other: tiled
  if (K <= 128 && N <= 128 && variant == 0 && R * 128 < (int64_t(1) << 31)) {
    const int64_t ntiles = (R + kPTile - 1) / kPTile;
    const int64_t want = (ntiles + 1) / 2;
    const unsigned grid = static_cast<unsigned>(want < kPFwdGrid ? want : kPFwdGrid);
    const bool vec = K % 4 == 0 && reinterpret_cast<uintptr_t>(x) % 16 == 0;
    if (K <= 8)
      dense_fwd_persist<4, false><<<grid, 512, 0, st>>>(x, w, b, res, R, K, N, act, y, z);
    else if (vec)
      dense_fwd_persist<64, true><<<grid, 512, 0, st>>>(x, w, b, res, R, K, N, act, y, z);
    else
      dense_fwd_persist<64, false><<<grid, 512, 0, st>>>(x, w, b, res, R, K, N, act, y, z);
    return last_launch_status();
  }
  dim3 grid(static_cast<unsigned>((R + kDenseRows - 1) / kDenseRows), (N + kDenseCols - 1) / kDenseCols);
  dense_rows<true, kActNone><<<grid, 256, 0, st>>>(x, w, b, res, nullptr, R, K, N, act, y, z, nullptr);
  return last_launch_status();
}

X2G_API int x2g_dense_bwd_data(const float* dy, const float* z, int act, const float* w, int64_t R, int32_t K,
                               int32_t N, float* dx, float* dz, void* stream) {
  // dy, z: [R, N]; w: [N, K]; dx: [R, K]; dz (optional, [R, N]) receives dy * act'(z)
  if (R < 0 || K <= 0 || N <= 0 || (act != kActNone && act != kActSilu)) return X2G_EINVAL;
  if (R == 0) return X2G_OK;
  if (!dy || !w || !dx || (act == kActSilu && !z)) return X2G_EINVAL;
  // as a row GEMM: A = dY' [R, N] (contraction over N), B[k'=n][n'=k] = w[n][k] (row-major, no transpose)
  dim3 grid(static_cast<unsigned>((R + kDenseRows - 1) / kDenseRows), (K + kDenseCols - 1) / kDenseCols);
  if (act == kActSilu)
    dense_rows<false, kActSilu><<<grid, 256, 0, as_stream(stream)>>>(dy, w, nullptr, nullptr, z, R, N, K, kActNone,
                                                                      dx, nullptr, dz);
  else
    dense_rows<false, kActNone><<<grid, 256, 0, as_stream(stream)>>>(dy, w, nullptr, nullptr, nullptr, R, N, K,
                                                                      kActNone, dx, nullptr, dz);
  return last_launch_status();
}

namespace x2g {  // slab sums come from linear.hip
int sum_slabs_launch(const float* part_w, int64_t nw, const float* part_b, int64_t nb, int splits, float* dw,
                     float* db, hipStream_t st);
}  // namespace x2g

X2G_API size_t x2g_linear_wgrad_workspace(int64_t R, int32_t O, int32_t I);
X2G_API int x2g_linear_wgrad(const float* dy, const float* x, int64_t R, int32_t O, int32_t I, float* dw, float* db,
                             void* workspace, size_t workspace_bytes, void* stream);

static inline bool dense_persistent_bwd(int64_t R, int32_t K, int32_t N) {
  return K <= 128 && N <= 128 && R > 0 && R * 128 < (int64_t(1) << 31);  // 32-bit offsets inside
}

X2G_API size_t x2g_dense_bwd_workspace(int64_t R, int32_t K, int32_t N) {
  if (R <= 0 || K <= 0 || N <= 0) return 0;
  if (dense_persistent_bwd(R, K, N)) {
    const int64_t ntiles = (R + kBTile - 1) / kBTile;
    const int64_t g = ntiles < kPBwdGrid ? ntiles : kPBwdGrid;
    return static_cast<size_t>(g) * (static_cast<int64_t>(N) * K + N) * sizeof(float);
  }
  // general path: dz [R, N] + the row-split weight-gradient slabs
  const size_t dz = ((static_cast<size_t>(R) * N * sizeof(float)) + 255) / 256 * 256;
  return dz + x2g_linear_wgrad_workspace(R, N, K);
}

X2G_API int x2g_dense_bwd(const float* dy, const float* z, int act, const float* x, const float* w, int64_t R,
                          int32_t K, int32_t N, float* dx, float* dw, float* db, void* workspace,
                          size_t workspace_bytes, void* stream) {
  if (R < 0 || K <= 0 || N <= 0 || (act != kActNone && act != kActSilu) || !dw) return X2G_EINVAL;
  hipStream_t st = as_stream(stream);
  if (R == 0) {
    hipError_t e = hipMemsetAsync(dw, 0, sizeof(float) * N * K, st);
    if (e == hipSuccess && db) e = hipMemsetAsync(db, 0, sizeof(float) * N, st);
    return e == hipSuccess ? X2G_OK : static_cast<int>(e);
  }
  if (!dy || !x || !w || (act == kActSilu && !z)) return X2G_EINVAL;
  if (!workspace || workspace_bytes < x2g_dense_bwd_workspace(R, K, N)) return X2G_EWORKSPACE;
  if (dense_persistent_bwd(R, K, N)) {
    const int64_t ntiles = (R + kBTile - 1) / kBTile;
    const int grid = static_cast<int>(ntiles < kPBwdGrid ? ntiles : kPBwdGrid);
    float* part_w = static_cast<float*>(workspace);
    float* part_b = db ? part_w + static_cast<int64_t>(grid) * N * K : nullptr;
    if (N <= 8)
      dense_bwd_persist<4><<<grid, 512, 0, st>>>(dy, z, x, w, R, K, N, act, dx, part_w, part_b);
    else
      dense_bwd_persist<64><<<grid, 512, 0, st>>>(dy, z, x, w, R, K, N, act, dx, part_w, part_b);
    int rc = last_launch_status();
    if (rc) return rc;
    return sum_slabs_launch(part_w, static_cast<int64_t>(N) * K, part_b, N, grid, dw, db, st);
  }
  // general shapes: dz = dy * act'(z) and dx = dz w in one kernel, then the weight gradient
  float* dzbuf = static_cast<float*>(workspace);
  const size_t dz_bytes = ((static_cast<size_t>(R) * N * sizeof(float)) + 255) / 256 * 256;
  const float* dzp = dy;
  int rc;
  if (act != kActNone || dx) {
    float* dx_tmp = dx;
    if (!dx_tmp) return X2G_EUNSUPPORTED;  // general path needs a dx buffer when an activation is fused
    if ((rc = x2g_dense_bwd_data(dy, z, act, w, R, K, N, dx_tmp, act != kActNone ? dzbuf : nullptr, stream))) return rc;
    if (act != kActNone) dzp = dzbuf;
  }
  return x2g_linear_wgrad(dzp, x, R, N, K, dw, db, static_cast<char*>(workspace) + dz_bytes,
                          workspace_bytes - dz_bytes, stream);
}
