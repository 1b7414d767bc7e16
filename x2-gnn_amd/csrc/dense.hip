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

// ---------------------------------------------------------------- forward, LDS-staged x tiles
// The same product for K % 4 == 0 (every trunk layer), with x staged through LDS in full
// 512-byte rows instead of fragment-shaped loads (lane-per-row 16-byte loads touch 64 cache
// lines per instruction and load the tile once per column wave: texture-address bound).
//   * 8 waves, two 32-row tiles per iteration (slot = wave >> 2), wave w -> columns 32 (w & 3)..;
//   * the next tile pair is loaded into registers (4 x 16 B per thread, coalesced rows) while the
//     current pair is multiplied, then written to the other LDS buffer (double buffered);
//   * LDS x tile: row r, 16-byte chunk q at chunk position q ^ (r & 15) — writes of 16
//     consecutive chunks and the A-fragment reads (lane = row, chunk 16h + g) are both
//     conflict-free; a lane's ds_read_b128 yields A values for 4 consecutive MFMA steps
//     (c = 64h + 4g .. 64h + 4g + 3, the cmap<64> order of the slot-layout weight);
//   * residual fragments for the current pair are loaded before the next pair's tile loads, so
//     waiting for them never drains the prefetch.

__device__ __forceinline__ void xpair_load(const float* __restrict__ X, int64_t tp, int64_t R, int K,
                                           float4 (&v)[4]) {
  const int kc = K >> 2;  // valid chunks per row
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int idx = threadIdx.x + 512 * u, row = idx >> 5, q = idx & 31;
    const int r = static_cast<int>(tp) * 64 + row, rmax = static_cast<int>(R) - 1;
    v[u] = *reinterpret_cast<const float4*>(X + (r < rmax ? r : rmax) * K + 4 * (q < kc ? q : kc - 1));
  }
}

__device__ __forceinline__ void xpair_store(float* __restrict__ buf, const float4 (&v)[4]) {
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int idx = threadIdx.x + 512 * u, row = idx >> 5, q = idx & 31;
    *reinterpret_cast<float4*>(buf + row * 128 + 4 * (q ^ (row & 15))) = v[u];
  }
}

__global__ void __launch_bounds__(512) dense_fwd_staged(const float* __restrict__ X, const float* __restrict__ W,
                                                        const float* __restrict__ bias,
                                                        const float* __restrict__ res, int64_t R, int K, int N,
                                                        int act, float* __restrict__ Y, float* __restrict__ Z) {
  __shared__ __attribute__((aligned(16))) float Ws[64 * 128 * 2];
  __shared__ __attribute__((aligned(16))) float Xs[2][64 * 128];  // [buffer][slot*32 + row][128]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5, i = lane & 31;
  const int slot = wave >> 2;
  const int n = 32 * (wave & 3) + i;
  const int64_t npairs = (R + 63) / 64;
  const int64_t G = gridDim.x;
  const float bn = (bias && n < N) ? bias[n] : 0.f;
  int64_t tp = blockIdx.x;
  float4 stage[4];
  {
    float wv[32];
    wslot_load<64, true, 512>(W, N, K, wv);
    xpair_load(X, tp, R, K, stage);
    wslot_store<512>(Ws, wv);
    xpair_store(Xs[0], stage);
    if (tp + G < npairs) xpair_load(X, tp + G, R, K, stage);
    __syncthreads();
  }
  const float* wb = Ws + n * 2 + h;
  for (int it = 0; tp < npairs; tp += G, ++it) {
    const float* xs = Xs[it & 1] + (slot * 32 + i) * 128;
    const int t = static_cast<int>(tp) * 2 + slot;  // this wave's 32-row tile
    float rv[16];
    if (res) cfrag_load(res, static_cast<int64_t>(t) * kPTile, R, N, n, rv);
    // the pair after next: write the staged pair to the other buffer, then refill the registers
    const bool more = tp + G < npairs;
    if (more) xpair_store(Xs[(it + 1) & 1], stage);
    if (tp + 2 * G < npairs) xpair_load(X, tp + 2 * G, R, K, stage);
    floatx16 acc0, acc1;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      acc0[j] = 0.f;
      acc1[j] = 0.f;
    }
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      const float4 a = *reinterpret_cast<const float4*>(xs + 4 * ((16 * h + g) ^ (i & 15)));
      const int s = 4 * g;
      acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, wb[s * 256], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, wb[(s + 1) * 256], acc1, 0, 0, 0);
      acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, wb[(s + 2) * 256], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, wb[(s + 3) * 256], acc1, 0, 0, 0);
    }
    const int rbase = t * kPTile + 4 * h;
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
    __syncthreads();  // the next buffer is complete; this one is free for the pair after next
  }
}

// ---------------------------------------------------------------- forward helpers (v5 design, used by v6)
// dense_fwd_staged plus the two fixes its phase measurements called for (R = 21k rows: weight
// staging 5.6 us, epilogue stores 6.3 us of 40 us):
//   * the weight is read row-contiguous (coalesced) and written to a slot layout padded to 258
//     floats per slot: 2-way bank conflicts on the staging writes, conflict-free B reads;
//   * the epilogue goes through LDS: the C fragments (one column, 16 rows per lane) are written
//     into the consumed x buffer, then every thread handles whole 16-byte row chunks: bias,
//     activation, residual (loaded row-wise and early), and 16-byte stores of z and y
//     (4x fewer store instructions than per-lane dword stores, which are issue-bound).
constexpr int kSlotStride = 258;

__device__ __forceinline__ void wpad_load(const float* __restrict__ W, int N, int K, float (&v)[32]) {
#pragma unroll
  for (int u = 0; u < 32; ++u) {
    const int idx = threadIdx.x + 512 * u, n = idx >> 7, k = idx & 127;
    const float x = ld_pin(W + (n < N ? n : N - 1) * K + (k < K ? k : K - 1));
    v[u] = (n < N && k < K) ? x : 0.f;
  }
}

__device__ __forceinline__ void wpad_store(float* __restrict__ ws, const float (&v)[32]) {
#pragma unroll
  for (int u = 0; u < 32; ++u) {
    const int idx = threadIdx.x + 512 * u, n = idx >> 7, k = idx & 127;
    ws[(k & 63) * kSlotStride + 2 * n + (k >> 6)] = v[u];  // B[c=k][j=n], cmap<64>: c = 64h + s
  }
}

// 64 rows x 128 columns of a row-major [R, N] matrix (N % 4 == 0) in the x-pair thread mapping.
__device__ __forceinline__ void rows_load(const float* __restrict__ m, int64_t tp, int64_t R, int N,
                                          float4 (&v)[4]) {
  const int nc = N >> 2;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int idx = threadIdx.x + 512 * u, row = idx >> 5, q = idx & 31;
    const int r = static_cast<int>(tp) * 64 + row, rmax = static_cast<int>(R) - 1;
    v[u] = *reinterpret_cast<const float4*>(m + (r < rmax ? r : rmax) * N + 4 * (q < nc ? q : nc - 1));
  }
}

typedef float f4 __attribute__((ext_vector_type(4)));  // native vector: loads/stores stay in registers

struct Stage4 {
  f4 v0, v1, v2, v3;
};

// The tile-pair staging on named registers: a float4[4] carried across the tile loop with a
// conditional refill stayed a private (scratch) array.  Chunk u of this thread: row
// (tid >> 5) + 16 u of the pair, 16-byte column chunk tid & 31.
template <int U>
__device__ __forceinline__ f4 st_get(const Stage4& st) {
  if constexpr (U == 0) return st.v0;
  else if constexpr (U == 1) return st.v1;
  else if constexpr (U == 2) return st.v2;
  else return st.v3;
}

__device__ __forceinline__ void xpair_load4(const float* __restrict__ X, int64_t tp, int64_t R, int K, Stage4& st) {
  const int kc = K >> 2, q = threadIdx.x & 31, qc = 4 * (q < kc ? q : kc - 1);
  const int rmax = static_cast<int>(R) - 1, r0 = static_cast<int>(tp) * 64 + (threadIdx.x >> 5);
  const int ra = r0 < rmax ? r0 : rmax, rb = r0 + 16 < rmax ? r0 + 16 : rmax;
  const int rc = r0 + 32 < rmax ? r0 + 32 : rmax, rd = r0 + 48 < rmax ? r0 + 48 : rmax;
  st.v0 = *reinterpret_cast<const f4*>(X + ra * K + qc);
  st.v1 = *reinterpret_cast<const f4*>(X + rb * K + qc);
  st.v2 = *reinterpret_cast<const f4*>(X + rc * K + qc);
  st.v3 = *reinterpret_cast<const f4*>(X + rd * K + qc);
}

__device__ __forceinline__ void xpair_store4(float* __restrict__ buf, const Stage4& st) {
  const int q = threadIdx.x & 31, row = threadIdx.x >> 5;  // rows row, +16, +32, +48 share (row & 15)
  float* p = buf + row * 128 + 4 * (q ^ (row & 15));
  *reinterpret_cast<f4*>(p) = st.v0;
  *reinterpret_cast<f4*>(p + 16 * 128) = st.v1;
  *reinterpret_cast<f4*>(p + 32 * 128) = st.v2;
  *reinterpret_cast<f4*>(p + 48 * 128) = st.v3;
}

__device__ __forceinline__ float act_apply(float z, int act) { return act == kActSilu ? z / (1.0f + expf(-z)) : z; }

// Row-wise epilogue of one 16-byte chunk (row (tid >> 5) + 16 U of the pair): bias, activation,
// residual, 16-byte stores of z and y.
template <int U>
__device__ __forceinline__ void epi_chunk(const float* __restrict__ buf, const Stage4& rres, f4 b4, int64_t tp,
                                          int64_t R, int N, int act, float* __restrict__ Y, float* __restrict__ Z) {
  const int q = threadIdx.x & 31, row = (threadIdx.x >> 5) + 16 * U;
  const int r = static_cast<int>(tp) * 64 + row;
  const f4 zc = *reinterpret_cast<const f4*>(buf + row * 128 + 4 * (q ^ (row & 15))) + b4;
  const f4 rr = st_get<U>(rres);
  f4 yv;
  yv.x = act_apply(zc.x, act) + rr.x;
  yv.y = act_apply(zc.y, act) + rr.y;
  yv.z = act_apply(zc.z, act) + rr.z;
  yv.w = act_apply(zc.w, act) + rr.w;
  if (r < R && 4 * q < N) {
    if (Z) *reinterpret_cast<f4*>(Z + r * N + 4 * q) = zc;
    *reinterpret_cast<f4*>(Y + r * N + 4 * q) = yv;
  }
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
                                         float* __restrict__ dX, const float* __restrict__ dXadd,
                                         floatx16 (&accw)[2], float& bsum, bool do_bias) {
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
        if (r < R) dX[r * K + k] = acc0[j] + acc1[j] + (dXadd ? dXadd[r * K + k] : 0.f);
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
                                                         const float* __restrict__ dXadd, float* __restrict__ part_w,
                                                         float* __restrict__ part_b) {
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
    bwd_tile<NSTEPS>(Ds, Xs, Ws, A, B, dY, Zin, X, t, G, ntiles, R, K, N, act, dX, dXadd, accw, bsum, do_bias);
    if (t + G >= ntiles) break;
    bwd_tile<NSTEPS>(Ds, Xs, Ws, B, A, dY, Zin, X, t + G, G, ntiles, R, K, N, act, dX, dXadd, accw, bsum,
                     do_bias);
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

// ---------------------------------------------------------------- forward, v6: two workgroups per CU
// 4 waves and 80 KB of LDS per workgroup (weight 64 KB + one 32-row x tile 16 KB), so two
// workgroups share a CU and one multiplies while the other loads / stores: at 21k rows the
// busiest CU then holds 3 tiles of 32 rows instead of 2 pairs of 64 (v5).  The weight slot
// layout is unpadded with an XOR swizzle instead: B[c(s,h)][j] at s*256 + 2 (j ^ (s & 31)) + h
// (staging writes 2-way, B reads conflict-free).
__device__ __forceinline__ int wswz(int s, int j, int h) { return s * 256 + 2 * (j ^ (s & 31)) + h; }

__device__ __forceinline__ void xtile_load(const float* __restrict__ X, int64_t t, int64_t R, int K, Stage4& st) {
  const int kc = K >> 2, q = threadIdx.x & 31, qc = 4 * (q < kc ? q : kc - 1);
  const int rmax = static_cast<int>(R) - 1, r0 = static_cast<int>(t) * 32 + (threadIdx.x >> 5);
  const int ra = r0 < rmax ? r0 : rmax, rb = r0 + 8 < rmax ? r0 + 8 : rmax;
  const int rc = r0 + 16 < rmax ? r0 + 16 : rmax, rd = r0 + 24 < rmax ? r0 + 24 : rmax;
  st.v0 = *reinterpret_cast<const f4*>(X + ra * K + qc);
  st.v1 = *reinterpret_cast<const f4*>(X + rb * K + qc);
  st.v2 = *reinterpret_cast<const f4*>(X + rc * K + qc);
  st.v3 = *reinterpret_cast<const f4*>(X + rd * K + qc);
}

__device__ __forceinline__ void xtile_store(float* __restrict__ buf, const Stage4& st) {
  const int q = threadIdx.x & 31, row = threadIdx.x >> 5;  // rows row, +8, +16, +24 (row & 15 differs by 8)
  *reinterpret_cast<f4*>(buf + row * 128 + 4 * (q ^ (row & 15))) = st.v0;
  *reinterpret_cast<f4*>(buf + (row + 8) * 128 + 4 * (q ^ ((row + 8) & 15))) = st.v1;
  *reinterpret_cast<f4*>(buf + (row + 16) * 128 + 4 * (q ^ ((row + 16) & 15))) = st.v2;
  *reinterpret_cast<f4*>(buf + (row + 24) * 128 + 4 * (q ^ ((row + 24) & 15))) = st.v3;
}

template <int U>
__device__ __forceinline__ void epi_tile(const float* __restrict__ buf, const Stage4& rres, f4 b4, int64_t t,
                                         int64_t R, int N, int act, float* __restrict__ Y, float* __restrict__ Z) {
  const int q = threadIdx.x & 31, row = (threadIdx.x >> 5) + 8 * U;
  const int r = static_cast<int>(t) * 32 + row;
  const f4 zc = *reinterpret_cast<const f4*>(buf + row * 128 + 4 * (q ^ (row & 15))) + b4;
  const f4 rr = st_get<U>(rres);
  f4 yv;
  yv.x = act_apply(zc.x, act) + rr.x;
  yv.y = act_apply(zc.y, act) + rr.y;
  yv.z = act_apply(zc.z, act) + rr.z;
  yv.w = act_apply(zc.w, act) + rr.w;
  if (r < R && 4 * q < N) {
    if (Z) *reinterpret_cast<f4*>(Z + r * N + 4 * q) = zc;
    *reinterpret_cast<f4*>(Y + r * N + 4 * q) = yv;
  }
}

__device__ __forceinline__ void dense_fwd_v6_body(const float* __restrict__ X, const float* __restrict__ W,
                                                  const float* __restrict__ bias, const float* __restrict__ res,
                                                  int64_t R, int K, int N, int act, float* __restrict__ Y,
                                                  float* __restrict__ Z, float* __restrict__ Ws,
                                                  float* __restrict__ Xs /* x tile, then the output tile */) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5, i = lane & 31;
  const int n = 32 * wave + i;
  const int q = tid & 31;
  const int64_t ntiles = (R + 31) / 32;
  const int64_t G = gridDim.x;
  f4 b4 = {0.f, 0.f, 0.f, 0.f};
  if (bias && 4 * q < N) b4 = f4{bias[4 * q], bias[4 * q + 1], bias[4 * q + 2], bias[4 * q + 3]};
  int64_t t = blockIdx.x;
  {
    Stage4 first;
    xtile_load(X, t, R, K, first);
#pragma unroll
    for (int half = 0; half < 2; ++half) {  // weight in two halves of 32 loads per thread
      float v[32];
#pragma unroll
      for (int u = 0; u < 32; ++u) {
        const int idx = tid + 256 * (32 * half + u), nn = idx >> 7, k = idx & 127;
        const float x = ld_pin(W + (nn < N ? nn : N - 1) * K + (k < K ? k : K - 1));
        v[u] = (nn < N && k < K) ? x : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 32; ++u) {
        const int idx = tid + 256 * (32 * half + u), nn = idx >> 7, k = idx & 127;
        Ws[wswz(k & 63, nn, k >> 6)] = v[u];
      }
    }
    xtile_store(Xs, first);
    __syncthreads();
  }
  for (; t < ntiles; t += G) {
    const bool more = t + G < ntiles;
    Stage4 rres{}, nxt;
    if (res) xtile_load(res, t, R, N, rres);  // first: waiting for it never drains the prefetch
    if (more) xtile_load(X, t + G, R, K, nxt);
    floatx16 acc0, acc1;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      acc0[j] = 0.f;
      acc1[j] = 0.f;
    }
    const float* xs = Xs + i * 128;
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      const f4 a = *reinterpret_cast<const f4*>(xs + 4 * ((16 * h + g) ^ (i & 15)));
      const int s = 4 * g;
      acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, Ws[wswz(s, n, h)], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, Ws[wswz(s + 1, n, h)], acc1, 0, 0, 0);
      acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, Ws[wswz(s + 2, n, h)], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, Ws[wswz(s + 3, n, h)], acc1, 0, 0, 0);
    }
    __syncthreads();  // the x tile is consumed: the buffer stages the output
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int r = (j & 3) + 8 * (j >> 2) + 4 * h;
      Xs[r * 128 + 4 * ((n >> 2) ^ (r & 15)) + (n & 3)] = acc0[j] + acc1[j];
    }
    __syncthreads();
    epi_tile<0>(Xs, rres, b4, t, R, N, act, Y, Z);
    epi_tile<1>(Xs, rres, b4, t, R, N, act, Y, Z);
    epi_tile<2>(Xs, rres, b4, t, R, N, act, Y, Z);
    epi_tile<3>(Xs, rres, b4, t, R, N, act, Y, Z);
    __syncthreads();
    if (more) xtile_store(Xs, nxt);
    __syncthreads();
  }
}

__global__ void __launch_bounds__(256, 2) dense_fwd_v6(const float* __restrict__ X, const float* __restrict__ W,
                                                       const float* __restrict__ bias, const float* __restrict__ res,
                                                       int64_t R, int K, int N, int act, float* __restrict__ Y,
                                                       float* __restrict__ Z) {
  __shared__ __attribute__((aligned(16))) float Ws[64 * 256];
  __shared__ __attribute__((aligned(16))) float Xs[32 * 128];
  dense_fwd_v6_body(X, W, bias, res, R, K, N, act, Y, Z, Ws, Xs);
}

// G independent layers of one shape in one launch (blockIdx.y = layer): the readout MLPs
struct DenseFwdBatch {
  x2g_dense_fwd_group g[X2G_MAX_GROUPS];
};

__global__ void __launch_bounds__(256, 2) dense_fwd_v6_batched(const DenseFwdBatch b, int64_t R, int K, int N,
                                                               int act) {
  __shared__ __attribute__((aligned(16))) float Ws[64 * 256];
  __shared__ __attribute__((aligned(16))) float Xs[32 * 128];
  const x2g_dense_fwd_group& p = b.g[blockIdx.y];
  dense_fwd_v6_body(p.x, p.w, p.b, p.res, R, K, N, act, p.y, p.z, Ws, Xs);
}

// ---------------------------------------------------------------- ResidualLayer forward, fused
// y = x + SiLU(W1 SiLU(W0 x + b0) + b1) (residual_layer.py:21-27) for D <= 128 in ONE persistent
// kernel: both weights staged once per CU (2 x 64 KB, the v6 swizzled slot layout), and per
// 32-row tile: GEMM 1 from the x tile, its C fragments transposed into the h tile (16 KB), bias +
// SiLU applied in place (z0 and h stored for the backward), GEMM 2 from the h tile, and the
// epilogue adds the residual straight from the x tile still in LDS.  160 KB of LDS: one
// workgroup per CU.  Versus two v6 launches: no second weight staging / launch ramp and no
// re-read of h and x from HBM.
__device__ __forceinline__ void stage_w_swz(const float* __restrict__ W, int N, int K, float* __restrict__ Ws) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    float v[32];
#pragma unroll
    for (int u = 0; u < 32; ++u) {
      const int idx = tid + 256 * (32 * half + u), nn = idx >> 7, k = idx & 127;
      const float x = ld_pin(W + (nn < N ? nn : N - 1) * K + (k < K ? k : K - 1));
      v[u] = (nn < N && k < K) ? x : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 32; ++u) {
      const int idx = tid + 256 * (32 * half + u), nn = idx >> 7, k = idx & 127;
      Ws[wswz(k & 63, nn, k >> 6)] = v[u];
    }
  }
}

// acc = A tile (rows swizzled, [32][128]) x B (slot layout): this wave's 32 output columns
__device__ __forceinline__ void tile_mfma(const float* __restrict__ As, const float* __restrict__ Ws, int n, int h,
                                          int i, floatx16& acc0, floatx16& acc1) {
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    acc0[j] = 0.f;
    acc1[j] = 0.f;
  }
  const float* xs = As + i * 128;
#pragma unroll
  for (int g = 0; g < 16; ++g) {
    const f4 a = *reinterpret_cast<const f4*>(xs + 4 * ((16 * h + g) ^ (i & 15)));
    const int s = 4 * g;
    acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, Ws[wswz(s, n, h)], acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, Ws[wswz(s + 1, n, h)], acc1, 0, 0, 0);
    acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, Ws[wswz(s + 2, n, h)], acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, Ws[wswz(s + 3, n, h)], acc1, 0, 0, 0);
  }
}

__device__ __forceinline__ void acc_to_rows(float* __restrict__ buf, const floatx16& acc0, const floatx16& acc1, int n,
                                            int h) {
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int r = (j & 3) + 8 * (j >> 2) + 4 * h;
    buf[r * 128 + 4 * ((n >> 2) ^ (r & 15)) + (n & 3)] = acc0[j] + acc1[j];
  }
}

__global__ void __launch_bounds__(256, 1) residual_fwd_kernel(const float* __restrict__ X, const float* __restrict__ W0,
                                                              const float* __restrict__ B0,
                                                              const float* __restrict__ W1,
                                                              const float* __restrict__ B1, int64_t R, int D,
                                                              float* __restrict__ H, float* __restrict__ Z0,
                                                              float* __restrict__ Z1, float* __restrict__ Y) {
  __shared__ __attribute__((aligned(16))) float Ws0[64 * 256];
  __shared__ __attribute__((aligned(16))) float Ws1[64 * 256];
  __shared__ __attribute__((aligned(16))) float Xs[32 * 128];
  __shared__ __attribute__((aligned(16))) float Hs[32 * 128];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5, i = lane & 31;
  const int n = 32 * wave + i;
  const int q = tid & 31;
  const int64_t ntiles = (R + 31) / 32;
  const int64_t G = gridDim.x;
  const bool colok = 4 * q < D;
  f4 b0 = {0.f, 0.f, 0.f, 0.f}, b1 = {0.f, 0.f, 0.f, 0.f};
  if (B0 && colok) b0 = f4{B0[4 * q], B0[4 * q + 1], B0[4 * q + 2], B0[4 * q + 3]};
  if (B1 && colok) b1 = f4{B1[4 * q], B1[4 * q + 1], B1[4 * q + 2], B1[4 * q + 3]};
  int64_t t = blockIdx.x;
  {
    Stage4 first;
    xtile_load(X, t, R, D, first);
    stage_w_swz(W0, D, D, Ws0);
    stage_w_swz(W1, D, D, Ws1);
    xtile_store(Xs, first);
    __syncthreads();
  }
  for (; t < ntiles; t += G) {
    const bool more = t + G < ntiles;
    Stage4 nxt;
    if (more) xtile_load(X, t + G, R, D, nxt);
    floatx16 acc0, acc1;
    tile_mfma(Xs, Ws0, n, h, i, acc0, acc1);
    acc_to_rows(Hs, acc0, acc1, n, h);
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 4; ++u) {  // z0 = . + b0 -> Z0; h = SiLU(z0) -> H and in place
      const int row = (tid >> 5) + 8 * u, r = static_cast<int>(t) * 32 + row;
      f4* hp = reinterpret_cast<f4*>(Hs + row * 128 + 4 * (q ^ (row & 15)));
      const f4 z = *hp + b0;
      f4 hv;
      hv.x = act_apply(z.x, kActSilu);
      hv.y = act_apply(z.y, kActSilu);
      hv.z = act_apply(z.z, kActSilu);
      hv.w = act_apply(z.w, kActSilu);
      *hp = hv;
      if (r < R && colok) {
        *reinterpret_cast<f4*>(Z0 + r * D + 4 * q) = z;
        *reinterpret_cast<f4*>(H + r * D + 4 * q) = hv;
      }
    }
    __syncthreads();
    tile_mfma(Hs, Ws1, n, h, i, acc0, acc1);
    __syncthreads();  // h consumed: Hs stages the second output
    acc_to_rows(Hs, acc0, acc1, n, h);
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 4; ++u) {  // z1 = . + b1 -> Z1; y = SiLU(z1) + x -> Y
      const int row = (tid >> 5) + 8 * u, r = static_cast<int>(t) * 32 + row;
      const int off = row * 128 + 4 * (q ^ (row & 15));
      const f4 z = *reinterpret_cast<const f4*>(Hs + off) + b1;
      const f4 xv = *reinterpret_cast<const f4*>(Xs + off);
      f4 yv;
      yv.x = act_apply(z.x, kActSilu) + xv.x;
      yv.y = act_apply(z.y, kActSilu) + xv.y;
      yv.z = act_apply(z.z, kActSilu) + xv.z;
      yv.w = act_apply(z.w, kActSilu) + xv.w;
      if (r < R && colok) {
        *reinterpret_cast<f4*>(Z1 + r * D + 4 * q) = z;
        *reinterpret_cast<f4*>(Y + r * D + 4 * q) = yv;
      }
    }
    __syncthreads();
    if (more) xtile_store(Xs, nxt);
    __syncthreads();
  }
}

// ---------------------------------------------------------------- forward, narrow K (K % 4 != 0)
// For rows too narrow / odd for 16-byte row chunks (lin_sbf: K = 42): a 64-row tile pair is one
// contiguous span of 64*K floats, read with 16-byte loads regardless of K and scattered into
// LDS unchanged (row stride K, 16-byte writes); the MFMA operand read strides by K.  Contraction order
// c(s, h) = 4 (s >> 1) + 2h + (s & 1): a lane's two consecutive steps read one 8-byte pair.
// Weight in the padded slot layout with the same order; epilogue as dense_fwd_v5.
__device__ __forceinline__ int cmap_n(int s, int h) { return 4 * (s >> 1) + 2 * h + (s & 1); }

template <int STEPS>
__global__ void __launch_bounds__(512) dense_fwd_narrow(const float* __restrict__ X, const float* __restrict__ W,
                                                        const float* __restrict__ bias,
                                                        const float* __restrict__ res, int64_t R, int K, int N,
                                                        int act, float* __restrict__ Y, float* __restrict__ Z) {
  constexpr int KP = 2 * STEPS;  // padded row length (>= K, multiple of 4)
  __shared__ __attribute__((aligned(16))) float Ws[STEPS * kSlotStride];
  __shared__ __attribute__((aligned(16))) float Xs[64 * 128];  // x tile [64][KP], then the output tile
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5, i = lane & 31;
  const int slot = wave >> 2;
  const int n = 32 * (wave & 3) + i;
  const int q = tid & 31;
  const int64_t npairs = (R + 63) / 64;
  const int64_t G = gridDim.x;
  f4 b4 = {0.f, 0.f, 0.f, 0.f};
  if (bias && 4 * q < N) b4 = f4{bias[4 * q], bias[4 * q + 1], bias[4 * q + 2], bias[4 * q + 3]};
  // weight: B[c][j] = w[j][c] for c < K, zero beyond
  for (int idx = tid; idx < STEPS * 2 * 128; idx += 512) {
    const int j = idx / (2 * STEPS), r = idx - j * 2 * STEPS;  // r = contraction index c
    const int sl = 2 * (r >> 2) + (r & 1), hh = (r >> 1) & 1;
    const float wv = (j < N && r < K) ? W[j * K + r] : 0.f;
    Ws[sl * kSlotStride + 2 * j + hh] = wv;
  }
  const float* wb = Ws + 2 * n + h;
  const int nq = (64 * K) >> 2;
  // register double buffer: the next pair's x span is in flight while this pair's MFMAs and
  // epilogue run (NQI 16-byte chunks per thread cover 64 rows x KP floats)
  constexpr int NQI = (16 * KP + 511) / 512;
  f4 pre[NQI];
  auto prefetch = [&](int64_t tpn) {
    const int64_t bn = tpn * 64 * K;
    const int64_t nv = ((R - tpn * 64) < 64 ? (R - tpn * 64) : 64) * K;
#pragma unroll
    for (int u = 0; u < NQI; ++u) {
      const int qi = tid + 512 * u;
      // whole 16-byte chunks load as one vector; the span's last partial chunk (64*K or the
      // ragged tail's length need not be a multiple of 4) element-wise, never past the end of X
      if (qi < nq && 4 * qi + 4 <= nv) {
        pre[u] = *reinterpret_cast<const f4*>(X + bn + 4 * qi);
      } else {
        pre[u] = f4{0.f, 0.f, 0.f, 0.f};
        if (qi < nq && 4 * qi < nv)
          for (int e = 0; e < 4; ++e)
            if (4 * qi + e < nv) pre[u][e] = X[bn + 4 * qi + e];
      }
    }
  };
  if (blockIdx.x < npairs) prefetch(blockIdx.x);
  for (int64_t tp = blockIdx.x; tp < npairs; tp += G) {
    // stage the pair: rows [64 tp, 64 tp + 64) are floats [64 tp K, 64 tp K + 64 K)
    const int64_t nvalid = ((R - tp * 64) < 64 ? (R - tp * 64) : 64) * K;
    __syncthreads();  // previous pair's output tile fully stored
#pragma unroll
    for (int u = 0; u < NQI; ++u) {  // the span lands as-is (row stride K): one 16-byte LDS write
      const int qi = tid + 512 * u;
      if (qi < nq) {
        f4 v = pre[u];
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (4 * qi + e >= nvalid) v[e] = 0.f;
        *reinterpret_cast<f4*>(Xs + 4 * qi) = v;
      }
    }
    // contraction columns K..KP-1 of a row fall on the next row's first floats: the operand read
    // below masks them (a zero weight alone would turn a neighbour's Inf/NaN into NaN here)
    if (tid < KP - K) Xs[64 * K + tid] = 0.f;
    __syncthreads();
    if (tp + G < npairs) prefetch(tp + G);
    floatx16 acc0, acc1;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      acc0[j] = 0.f;
      acc1[j] = 0.f;
    }
    const float* xs = Xs + (slot * 32 + i) * K + 2 * h;
    const int klim = K - 2 * h;  // contraction index 4g + 2h (+1) must stay below K
#pragma unroll
    for (int g = 0; g < STEPS / 2; ++g) {
      const float a0 = 4 * g < klim ? xs[4 * g] : 0.f, a1 = 4 * g + 1 < klim ? xs[4 * g + 1] : 0.f;
      acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, wb[(2 * g) * kSlotStride], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, wb[(2 * g + 1) * kSlotStride], acc1, 0, 0, 0);
    }
    __syncthreads();  // x tile consumed: the buffer stages the output
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int r = slot * 32 + (j & 3) + 8 * (j >> 2) + 4 * h;
      Xs[r * 128 + 4 * ((n >> 2) ^ (r & 15)) + (n & 3)] = acc0[j] + acc1[j];
    }
    __syncthreads();
    Stage4 rres{};
    if (res) xpair_load4(res, tp, R, N, rres);
    epi_chunk<0>(Xs, rres, b4, tp, R, N, act, Y, Z);
    epi_chunk<1>(Xs, rres, b4, tp, R, N, act, Y, Z);
    epi_chunk<2>(Xs, rres, b4, tp, R, N, act, Y, Z);
    epi_chunk<3>(Xs, rres, b4, tp, R, N, act, Y, Z);
  }
}

int dense_fwd_narrow_launch(const float* x, const float* w, const float* b, const float* res, int64_t R, int K, int N,
                            int act, float* y, float* z, hipStream_t st) {
  // the kernel covers N <= 128 columns and K <= 2*64; row offsets are 32-bit
  if (N > 128 || K > 128 || R * 128 * 4 >= (int64_t(1) << 31)) return X2G_EUNSUPPORTED;
  const int64_t npairs = (R + 63) / 64;
  const unsigned grid = static_cast<unsigned>(npairs < 512 ? npairs : 512);
  if (K <= 44)
    dense_fwd_narrow<22><<<grid, 512, 0, st>>>(x, w, b, res, R, K, N, act, y, z);
  else
    dense_fwd_narrow<64><<<grid, 512, 0, st>>>(x, w, b, res, R, K, N, act, y, z);
  return last_launch_status();
}

// ---------------------------------------------------------------- backward, narrow input (K <= 8)
// The radial-basis layers (lin_rbf: 6 -> 128, sbftransformer_conv.py:99, readout.py:38) have
// almost no data gradient to compute: dx[r, 0:K] = dz[r, :] w[:, 0:K] is K dot products of
// length N per row.  One wave per row (grid-stride): lane holds CPL = N/64 channels of dz,
// forms its K partial products, and a 64-lane xor reduction leaves dx[r, k] in every lane;
// dW[n, k] += dz[r, n] x[r, k] accumulates in registers (x row wave-uniform: scalar loads),
// db[n] += dz[r, n].  Waves fold their partials through LDS into one slab per workgroup.
template <int CPL, int KMAX>
__global__ void __launch_bounds__(256) dense_bwd_narrow(const float* __restrict__ dY, const float* __restrict__ Zin,
                                                        const float* __restrict__ X, const float* __restrict__ W,
                                                        int64_t R, int K, int N, int act, float* __restrict__ dX,
                                                        const float* __restrict__ dXadd, float* __restrict__ part_w,
                                                        float* __restrict__ part_b) {
  __shared__ float red[4][64 * CPL * (KMAX + 1)];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c0 = lane * CPL;
  float wr[CPL][KMAX];
#pragma unroll
  for (int j = 0; j < CPL; ++j)
#pragma unroll
    for (int k = 0; k < KMAX; ++k) wr[j][k] = (c0 + j < N && k < K) ? W[(c0 + j) * K + k] : 0.f;
  float gw[CPL][KMAX], gb[CPL];
#pragma unroll
  for (int j = 0; j < CPL; ++j) {
    gb[j] = 0.f;
#pragma unroll
    for (int k = 0; k < KMAX; ++k) gw[j][k] = 0.f;
  }
  // four rows per iteration (rows r, r + nw, r + 2nw, r + 3nw) so their loads are in flight together
  constexpr int ROWS = 4;
  const int64_t nw = static_cast<int64_t>(gridDim.x) * 4;
  for (int64_t r0 = uniform(blockIdx.x * 4 + wave); r0 < R; r0 += ROWS * nw) {
    float d[ROWS][CPL], xr[ROWS][KMAX];
#pragma unroll
    for (int u = 0; u < ROWS; ++u) {
      const int64_t r = r0 + u * nw;
      const bool rok = r < R;
      const int64_t rc = rok ? r : R - 1;
#pragma unroll
      for (int j = 0; j < CPL; ++j) {
        const bool ok = rok && c0 + j < N;
        float v = dY[rc * N + (c0 + j < N ? c0 + j : N - 1)];
        if (act == kActSilu) {
          const float z = Zin[rc * N + (c0 + j < N ? c0 + j : N - 1)];
          const float sg = 1.0f / (1.0f + expf(-z));
          v *= sg * (1.0f + z * (1.0f - sg));
        }
        d[u][j] = ok ? v : 0.f;
      }
#pragma unroll
      for (int k = 0; k < KMAX; ++k) xr[u][k] = (k < K) ? keep(X[rc * K + (k < K ? k : 0)], rok) : 0.f;
    }
#pragma unroll
    for (int u = 0; u < ROWS; ++u) {
      const int64_t r = r0 + u * nw;
      float px[KMAX];
#pragma unroll
      for (int k = 0; k < KMAX; ++k) {
        float acc = 0.f;
#pragma unroll
        for (int j = 0; j < CPL; ++j) {
          acc = fmaf(d[u][j], wr[j][k], acc);
          gw[j][k] = fmaf(d[u][j], xr[u][k], gw[j][k]);
        }
        px[k] = group_sum<64>(acc);
      }
#pragma unroll
      for (int j = 0; j < CPL; ++j) gb[j] += d[u][j];
      if (dX && lane < K && r < R) {
        float v = 0.f;
#pragma unroll
        for (int k = 0; k < KMAX; ++k) v = lane == k ? px[k] : v;
        if (dXadd) v += dXadd[r * K + lane];
        dX[r * K + lane] = v;
      }
    }
  }
  // fold the 4 waves (fixed order) and write this workgroup's slab
#pragma unroll
  for (int j = 0; j < CPL; ++j) {
#pragma unroll
    for (int k = 0; k < KMAX; ++k) red[wave][(c0 + j) * (KMAX + 1) + k] = gw[j][k];
    red[wave][(c0 + j) * (KMAX + 1) + KMAX] = gb[j];
  }
  __syncthreads();
  if (wave == 0) {
#pragma unroll
    for (int j = 0; j < CPL; ++j) {
      const int n = c0 + j;
      if (n >= N) continue;
#pragma unroll
      for (int k = 0; k < KMAX; ++k) {
        const int o = n * (KMAX + 1) + k;
        if (k < K) part_w[static_cast<int64_t>(blockIdx.x) * N * K + n * K + k] =
            ((red[0][o] + red[1][o]) + red[2][o]) + red[3][o];
      }
      const int o = n * (KMAX + 1) + KMAX;
      if (part_b) part_b[static_cast<int64_t>(blockIdx.x) * N + n] = ((red[0][o] + red[1][o]) + red[2][o]) + red[3][o];
    }
  }
}

constexpr int kNarrowBwdGrid = 512;

static inline bool dense_narrow_bwd(int64_t R, int32_t K, int32_t N) {
  return R > 0 && K <= 8 && N <= 128 && N > 64 && N % 64 == 0;
}

// ---------------------------------------------------------------- backward helpers (v5 design, used by v8)
// dense_bwd_persist restructured like the v5 forward (K % 4 == 0, N % 4 == 0, 16-byte aligned):
//   * dy, z, x tiles (64 rows) are read with 16-byte loads (4 per thread per matrix instead of
//     16 dword loads) into registers, the next tile's loads fly during the MFMAs;
//   * LDS: weight in the padded slot layout (cmap<64>, B[c = n][j = k] = w[n][k], staged from
//     coalesced rows), dz and x tiles in the chunk-swizzled [64][128] layout: dx's A fragments
//     are ds_read_b128 (4 MFMA steps each) and dW's row pairs (r, r ^ 8) hit disjoint banks;
//   * dx leaves through LDS (transposed into the consumed x tile) as 16-byte row stores.
// 8 waves: dx wave w -> rows 32 (w >> 2).., k columns 32 (w & 3)..;
//          dW wave w -> n rows 32 (w & 3).., k columns 64 (w >> 2)...
__device__ __forceinline__ int swz(int r, int c) { return r * 128 + 4 * ((c >> 2) ^ (r & 15)) + (c & 3); }

__device__ __forceinline__ void wpad_load_bwd(const float* __restrict__ W, int N, int K, float (&v)[32]) {
#pragma unroll
  for (int u = 0; u < 32; ++u) {  // row n = idx >> 7 of w, k = idx & 127: coalesced
    const int idx = threadIdx.x + 512 * u, n = idx >> 7, k = idx & 127;
    const float x = ld_pin(W + (n < N ? n : N - 1) * K + (k < K ? k : K - 1));
    v[u] = (n < N && k < K) ? x : 0.f;
  }
}

__device__ __forceinline__ void wpad_store_bwd(float* __restrict__ ws, const float (&v)[32]) {
#pragma unroll
  for (int u = 0; u < 32; ++u) {
    const int idx = threadIdx.x + 512 * u, n = idx >> 7, k = idx & 127;
    ws[(n & 63) * kSlotStride + 2 * k + (n >> 6)] = v[u];  // B[c=n][j=k], c = 64h + s
  }
}

template <int U>
__device__ __forceinline__ f4 silu_grad4(f4 d, f4 z) {
  f4 o;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float sg = 1.0f / (1.0f + expf(-z[e]));
    o[e] = d[e] * (sg * (1.0f + z[e] * (1.0f - sg)));
  }
  return o;
}

// rows >= R and columns >= cols of a staged tile are zeroed on the way into LDS
__device__ __forceinline__ f4 mask4(f4 v, int64_t tp, int U, int64_t R, int cols) {
  const int q = threadIdx.x & 31, row = (threadIdx.x >> 5) + 16 * U;
  const bool ok = tp * 64 + row < R && 4 * q < cols;
  return ok ? v : f4{0.f, 0.f, 0.f, 0.f};
}

struct DenseBwdBatch {
  x2g_dense_bwd_group g[X2G_MAX_GROUPS];
  float* part_w[X2G_MAX_GROUPS];
  float* part_b[X2G_MAX_GROUPS];
};

// ---------------------------------------------------------------- backward, v8: 32-row tiles
// As v5 (weight in the padded slot layout, dz and x tiles chunk-swizzled in LDS, next tile
// prefetched into registers during the MFMAs, dx through LDS as 16-byte row stores), but on
// 32-row tiles with the work split by wave role: waves 0-3 compute the tile's dx (32 rows x 32
// columns each, K = N), waves 4-7 its dW contribution (32 n-rows x all K columns each, over the
// tile's 32 rows).  Each SIMD then holds one dx wave and one dW wave (64 MFMAs each per tile), and
// the 32-row granularity balances the chip: at 21k rows 658 tiles over 220 workgroups (<= 3
// tiles each, 10.2 us of MFMA per CU) instead of 330 64-row tiles over 165 (2 x 6.8 us).
struct Stage2 {
  f4 v0, v1;
};

__device__ __forceinline__ void xt32_load(const float* __restrict__ X, int64_t t, int64_t R, int K, Stage2& st) {
  const int kc = K >> 2, q = threadIdx.x & 31, qc = 4 * (q < kc ? q : kc - 1);
  const int rmax = static_cast<int>(R) - 1, r0 = static_cast<int>(t) * 32 + (threadIdx.x >> 5);
  const int ra = r0 < rmax ? r0 : rmax, rb = r0 + 16 < rmax ? r0 + 16 : rmax;
  st.v0 = *reinterpret_cast<const f4*>(X + ra * K + qc);
  st.v1 = *reinterpret_cast<const f4*>(X + rb * K + qc);
}

__device__ __forceinline__ f4 mask32(f4 v, int64_t t, int U, int64_t R, int cols) {
  const int q = threadIdx.x & 31, row = (threadIdx.x >> 5) + 16 * U;
  const bool ok = t * 32 + row < R && 4 * q < cols;
  return ok ? v : f4{0.f, 0.f, 0.f, 0.f};
}

__device__ __forceinline__ void xt32_store(float* __restrict__ buf, f4 v0, f4 v1) {
  const int q = threadIdx.x & 31, row = threadIdx.x >> 5;  // rows row and row + 16 share (row & 15)
  float* p = buf + row * 128 + 4 * (q ^ (row & 15));
  *reinterpret_cast<f4*>(p) = v0;
  *reinterpret_cast<f4*>(p + 16 * 128) = v1;
}

__device__ __forceinline__ void dense_bwd_v8_body(const float* __restrict__ dY, const float* __restrict__ Zin,
                                                  const float* __restrict__ X, const float* __restrict__ W, int64_t R,
                                                  int K, int N, int act, float* __restrict__ dX,
                                                  const float* __restrict__ dXadd, float* __restrict__ part_w,
                                                  float* __restrict__ part_b, float* __restrict__ Ws,
                                                  float* __restrict__ Ds, float* __restrict__ Xs,
                                                  float* __restrict__ Os) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5, i = lane & 31;
  const int64_t ntiles = (R + 31) / 32;
  const int64_t G = gridDim.x;
  const bool silu = act == kActSilu;
  const bool dw_wave = wave >= 4;
  floatx16 accw[4];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int j = 0; j < 16; ++j) accw[m][j] = 0.f;
  float bsum = 0.f;
  int64_t t = blockIdx.x;
  Stage2 sd, sz, sx;
  {
    float wv[32];
    if (dX) wpad_load_bwd(W, N, K, wv);
    xt32_load(dY, t, R, N, sd);
    if (silu) xt32_load(Zin, t, R, N, sz);
    xt32_load(X, t, R, K, sx);
    if (dX) wpad_store_bwd(Ws, wv);
  }
  const int kcol = 32 * (wave & 3) + i;  // dx waves: output columns
  const int nb = 32 * (wave & 3);        // dW waves: n rows
  for (; t < ntiles; t += G) {
    {
      f4 d0 = sd.v0, d1 = sd.v1;
      if (silu) {
        d0 = silu_grad4<0>(d0, sz.v0);
        d1 = silu_grad4<1>(d1, sz.v1);
      }
      xt32_store(Ds, mask32(d0, t, 0, R, N), mask32(d1, t, 1, R, N));
      xt32_store(Xs, mask32(sx.v0, t, 0, R, K), mask32(sx.v1, t, 1, R, K));
    }
    __syncthreads();
    if (t + G < ntiles) {  // the next tile's loads fly during the MFMAs below
      xt32_load(dY, t + G, R, N, sd);
      if (silu) xt32_load(Zin, t + G, R, N, sz);
      xt32_load(X, t + G, R, K, sx);
    }
    if (!dw_wave) {
      if (dX) {  // dx[i][kcol] = sum_n dz[i][n] w[n][kcol], n = 64h + 4g + e
        floatx16 acc0, acc1;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          acc0[j] = 0.f;
          acc1[j] = 0.f;
        }
        const float* ds = Ds + i * 128;
        const float* wb = Ws + 2 * kcol + h;
#pragma unroll
        for (int g = 0; g < 16; ++g) {
          const f4 a = *reinterpret_cast<const f4*>(ds + 4 * ((16 * h + g) ^ (i & 15)));
          const int sb = 4 * g * kSlotStride;
          acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, wb[sb], acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, wb[sb + kSlotStride], acc1, 0, 0, 0);
          acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, wb[sb + 2 * kSlotStride], acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, wb[sb + 3 * kSlotStride], acc1, 0, 0, 0);
        }
#pragma unroll
        for (int j = 0; j < 16; ++j) Os[swz((j & 3) + 8 * (j >> 2) + 4 * h, kcol)] = acc0[j] + acc1[j];
      }
    } else {
      // dW[n][k] += sum_r dz[r][n] x[r][k]; step (sg, s): rows r = 16 sg + s + 8h
#pragma unroll
      for (int sg = 0; sg < 2; ++sg) {
#pragma unroll
        for (int s = 0; s < 8; ++s) {
          const int r = 16 * sg + s + 8 * h;
          const float a = Ds[swz(r, nb + i)];
#pragma unroll
          for (int m = 0; m < 4; ++m)
            accw[m] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, Xs[swz(r, 32 * m + i)], accw[m], 0, 0, 0);
        }
      }
      if (part_b && tid - 256 < 128) {
#pragma unroll 8
        for (int rr = 0; rr < 32; ++rr) bsum += Ds[swz(rr, tid - 256)];
      }
    }
    __syncthreads();  // Ds / Xs consumed, the dx tile is in Os
    if (dX) {
      const int q = tid & 31;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int row = (tid >> 5) + 16 * u;
        const int r = static_cast<int>(t) * 32 + row;
        f4 v = *reinterpret_cast<const f4*>(Os + row * 128 + 4 * (q ^ (row & 15)));
        if (r < R && 4 * q < K) {
          if (dXadd) v += *reinterpret_cast<const f4*>(dXadd + r * K + 4 * q);
          *reinterpret_cast<f4*>(dX + r * K + 4 * q) = v;
        }
      }
    }
  }
  if (dw_wave) {
    float* slab = part_w + static_cast<int64_t>(blockIdx.x) * N * K;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int nn = nb + (j & 3) + 8 * (j >> 2) + 4 * h;
        const int k = 32 * m + i;
        if (nn < N && k < K) slab[nn * K + k] = accw[m][j];
      }
    }
    if (part_b && tid - 256 < N && tid - 256 < 128) part_b[static_cast<int64_t>(blockIdx.x) * N + tid - 256] = bsum;
  }
}

__global__ void __launch_bounds__(512) dense_bwd_v8(const float* __restrict__ dY, const float* __restrict__ Zin,
                                                    const float* __restrict__ X, const float* __restrict__ W,
                                                    int64_t R, int K, int N, int act, float* __restrict__ dX,
                                                    const float* __restrict__ dXadd, float* __restrict__ part_w,
                                                    float* __restrict__ part_b) {
  __shared__ __attribute__((aligned(16))) float Ws[64 * kSlotStride];
  __shared__ __attribute__((aligned(16))) float Ds[32 * 128];
  __shared__ __attribute__((aligned(16))) float Xs[32 * 128];
  __shared__ __attribute__((aligned(16))) float Os[32 * 128];
  dense_bwd_v8_body(dY, Zin, X, W, R, K, N, act, dX, dXadd, part_w, part_b, Ws, Ds, Xs, Os);
}

__global__ void __launch_bounds__(512) dense_bwd_v8_batched(const DenseBwdBatch b, int64_t R, int K, int N, int act) {
  __shared__ __attribute__((aligned(16))) float Ws[64 * kSlotStride];
  __shared__ __attribute__((aligned(16))) float Ds[32 * 128];
  __shared__ __attribute__((aligned(16))) float Xs[32 * 128];
  __shared__ __attribute__((aligned(16))) float Os[32 * 128];
  const int gi = blockIdx.y;
  const x2g_dense_bwd_group& p = b.g[gi];
  dense_bwd_v8_body(p.dy, p.z, p.x, p.w, R, K, N, act, p.dx, p.dx_add, b.part_w[gi], b.part_b[gi], Ws, Ds, Xs, Os);
}

}  // namespace x2g

using namespace x2g;

static inline bool aligned16(const void* p) { return reinterpret_cast<uintptr_t>(p) % 16 == 0; }

X2G_API int x2g_dense_fwd(const float* x, const float* w, const float* b, int64_t R, int32_t K, int32_t N, int act,
                          const float* res, float* y, float* z, void* stream) {
  if (R < 0 || K <= 0 || N <= 0 || (act != kActNone && act != kActSilu)) return X2G_EINVAL;
  if (R == 0) return X2G_OK;
  if (!x || !w || !y) return X2G_EINVAL;
  hipStream_t st = as_stream(stream);
  if (K <= 128 && N <= 128 && R * 128 * 4 < (int64_t(1) << 31)) {
    const int64_t ntiles = (R + kPTile - 1) / kPTile;
    const int64_t want = (ntiles + 1) / 2;
    const unsigned grid = static_cast<unsigned>(want < kPFwdGrid ? want : kPFwdGrid);
    const bool vec = K % 4 == 0 && reinterpret_cast<uintptr_t>(x) % 16 == 0;
    if (K <= 8)
      dense_fwd_persist<4, false><<<grid, 512, 0, st>>>(x, w, b, res, R, K, N, act, y, z);
    else if (!vec && K % 4 != 0 && N % 4 == 0 && aligned16(x) && aligned16(y) && aligned16(z) && aligned16(res))
      return dense_fwd_narrow_launch(x, w, b, res, R, K, N, act, y, z, st);
    else if (vec && N % 4 == 0 && aligned16(y) && aligned16(z) && aligned16(res)) {
      // v6: two 256-thread workgroups per CU.  (A register-resident-weight variant with one tile
      // per workgroup measured no faster: at 21k rows the layer is bound by its 43 MB of
      // x / res / y / z traffic plus the launch ramp, not by the weight staging.)
      const unsigned g6 = static_cast<unsigned>(ntiles < 512 ? ntiles : 512);
      dense_fwd_v6<<<g6, 256, 0, st>>>(x, w, b, res, R, K, N, act, y, z);
    } else if (vec)
      dense_fwd_staged<<<grid, 512, 0, st>>>(x, w, b, res, R, K, N, act, y, z);
    else
      dense_fwd_persist<64, false><<<grid, 512, 0, st>>>(x, w, b, res, R, K, N, act, y, z);
    return last_launch_status();
  }
  dim3 grid(static_cast<unsigned>((R + kDenseRows - 1) / kDenseRows), (N + kDenseCols - 1) / kDenseCols);
  dense_rows<true, kActNone><<<grid, 256, 0, st>>>(x, w, b, res, nullptr, R, K, N, act, y, z, nullptr);
  return last_launch_status();
}

// dz = dy * SiLU'(z) alone (grid-stride, float4 where aligned)
__global__ void __launch_bounds__(256) silu_grad_elementwise(const float* __restrict__ dy, const float* __restrict__ z,
                                                              int64_t n, float* __restrict__ dz) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
    const float zz = z[i];
    const float s = 1.0f / (1.0f + expf(-zz));
    dz[i] = dy[i] * (s * (1.0f + zz * (1.0f - s)));
  }
}

// dx (+)= (dy * act'(z)) w for any shape; dx_add (optional, may alias dx) is added in the epilogue,
// where every element is read and then written by the same thread
static int dense_bwd_data_impl(const float* dy, const float* z, int act, const float* w, int64_t R, int32_t K,
                               int32_t N, float* dx, const float* dx_add, float* dz, hipStream_t st) {
  // as a row GEMM: A = dY' [R, N] (contraction over N), B[k'=n][n'=k] = w[n][k] (row-major, no transpose)
  dim3 grid(static_cast<unsigned>((R + kDenseRows - 1) / kDenseRows), (K + kDenseCols - 1) / kDenseCols);
  if (act == kActSilu)
    dense_rows<false, kActSilu><<<grid, 256, 0, st>>>(dy, w, nullptr, dx_add, z, R, N, K, kActNone, dx, nullptr, dz);
  else
    dense_rows<false, kActNone><<<grid, 256, 0, st>>>(dy, w, nullptr, dx_add, nullptr, R, N, K, kActNone, dx, nullptr,
                                                       dz);
  return last_launch_status();
}

namespace x2g {  // slab sums come from linear.hip
int sum_slabs_launch(const float* part_w, int64_t nw, const float* part_b, int64_t nb, int splits, float* dw,
                     float* db, bool accum, hipStream_t st);
}  // namespace x2g

X2G_API size_t x2g_linear_wgrad_workspace(int64_t R, int32_t O, int32_t I);

// Backward grid: the fewest workgroups that keep the busiest one at ceil(tiles / 256) tiles —
// every workgroup writes a full weight-gradient slab, so idle-making extra workgroups would only
// add slab traffic (330 tiles at config 2: 165 workgroups x 2 tiles instead of 256).
// (32-row tiles: dense_bwd_v8; the register-fragment persistent kernel strides over the same grid)
static inline int64_t bwd_grid(int64_t R) {
  const int64_t ntiles = (R + 31) / 32;
  const int64_t per = (ntiles + kPBwdGrid - 1) / kPBwdGrid;
  return (ntiles + per - 1) / per;
}

static inline bool dense_persistent_bwd(int64_t R, int32_t K, int32_t N) {
  return K <= 128 && N <= 128 && R > 0 && R * 128 * 4 < (int64_t(1) << 31);  // 32-bit offsets inside
}

static inline int64_t narrow_bwd_grid(int64_t R) {
  const int64_t want = (R + 15) / 16;  // >= 4 rows per wave
  return want < kNarrowBwdGrid ? (want > 0 ? want : 1) : kNarrowBwdGrid;
}

X2G_API size_t x2g_dense_bwd_workspace(int64_t R, int32_t K, int32_t N) {
  if (R <= 0 || K <= 0 || N <= 0) return 0;
  if (dense_narrow_bwd(R, K, N))
    return static_cast<size_t>(narrow_bwd_grid(R)) * (static_cast<int64_t>(N) * K + N) * sizeof(float);
  if (dense_persistent_bwd(R, K, N)) {
    const int64_t g = bwd_grid(R);
    return static_cast<size_t>(g) * (static_cast<int64_t>(N) * K + N) * sizeof(float);
  }
  // general path: dz [R, N] + the row-split weight-gradient slabs
  const size_t dz = ((static_cast<size_t>(R) * N * sizeof(float)) + 255) / 256 * 256;
  return dz + x2g_linear_wgrad_workspace(R, N, K);
}

X2G_API int x2g_linear_wgrad_ex(const float* dy, const float* x, int64_t R, int32_t O, int32_t I, float* dw,
                                float* db, int flags, void* workspace, size_t workspace_bytes, void* stream);

X2G_API int x2g_dense_bwd_ex(const float* dy, const float* z, int act, const float* x, const float* w, int64_t R,
                             int32_t K, int32_t N, float* dx, const float* dx_add, float* dw, float* db, int flags,
                             void* workspace, size_t workspace_bytes, void* stream) {
  if (R < 0 || K <= 0 || N <= 0 || (act != kActNone && act != kActSilu) || !dw ||
      (flags & ~(X2G_ACCUM_WGRAD | X2G_DEFER_SLAB_SUM)))
    return X2G_EINVAL;
  if ((flags & X2G_DEFER_SLAB_SUM) && R == 0) return X2G_EINVAL;
  if (dx_add && !dx) return X2G_EINVAL;
  const bool accum = flags & X2G_ACCUM_WGRAD;
  hipStream_t st = as_stream(stream);
  if (R == 0) {
    if (accum) return X2G_OK;
    hipError_t e = hipMemsetAsync(dw, 0, sizeof(float) * N * K, st);
    if (e == hipSuccess && db) e = hipMemsetAsync(db, 0, sizeof(float) * N, st);
    return e == hipSuccess ? X2G_OK : static_cast<int>(e);
  }
  if (!dy || !x || !w || (act == kActSilu && !z)) return X2G_EINVAL;
  if (!workspace || workspace_bytes < x2g_dense_bwd_workspace(R, K, N)) return X2G_EWORKSPACE;
  if (dense_narrow_bwd(R, K, N)) {
    const int grid = static_cast<int>(narrow_bwd_grid(R));
    float* part_w = static_cast<float*>(workspace);
    float* part_b = db ? part_w + static_cast<int64_t>(grid) * N * K : nullptr;
    if (N == 128)
      dense_bwd_narrow<2, 8><<<grid, 256, 0, st>>>(dy, z, x, w, R, K, N, act, dx, dx_add, part_w, part_b);
    else
      dense_bwd_narrow<1, 8><<<grid, 256, 0, st>>>(dy, z, x, w, R, K, N, act, dx, dx_add, part_w, part_b);
    int rc = last_launch_status();
    if (rc) return rc;
    if (flags & X2G_DEFER_SLAB_SUM) return X2G_OK;
    return sum_slabs_launch(part_w, static_cast<int64_t>(N) * K, part_b, N, grid, dw, db, accum, st);
  }
  if (dense_persistent_bwd(R, K, N)) {
    const int grid = static_cast<int>(bwd_grid(R));
    float* part_w = static_cast<float*>(workspace);
    float* part_b = db ? part_w + static_cast<int64_t>(grid) * N * K : nullptr;
    const bool vec = K % 4 == 0 && N % 4 == 0 && N > 8 && aligned16(dy) && aligned16(z) && aligned16(x) &&
                     aligned16(dx) && aligned16(dx_add);
    if (vec)
      dense_bwd_v8<<<grid, 512, 0, st>>>(dy, z, x, w, R, K, N, act, dx, dx_add, part_w, part_b);
    else if (N <= 8)
      dense_bwd_persist<4><<<grid, 512, 0, st>>>(dy, z, x, w, R, K, N, act, dx, dx_add, part_w, part_b);
    else
      dense_bwd_persist<64><<<grid, 512, 0, st>>>(dy, z, x, w, R, K, N, act, dx, dx_add, part_w, part_b);
    int rc = last_launch_status();
    if (rc) return rc;
    if (flags & X2G_DEFER_SLAB_SUM) return X2G_OK;
    return sum_slabs_launch(part_w, static_cast<int64_t>(N) * K, part_b, N, grid, dw, db, accum, st);
  }
  // general shapes: dz = dy * act'(z) and dx = dz w (+ dx_add) in one kernel, then the weight gradient
  float* dzbuf = static_cast<float*>(workspace);
  const size_t dz_bytes = ((static_cast<size_t>(R) * N * sizeof(float)) + 255) / 256 * 256;
  const float* dzp = dy;
  int rc;
  if (dx) {
    if ((rc = dense_bwd_data_impl(dy, z, act, w, R, K, N, dx, dx_add, act != kActNone ? dzbuf : nullptr, st)))
      return rc;
    if (act != kActNone) dzp = dzbuf;
  } else if (act != kActNone) {  // no data gradient wanted (e.g. a layer on non-differentiable input): dz only
    const int64_t n = R * static_cast<int64_t>(N);
    const int64_t blocks = (n + 1023) / 1024;
    silu_grad_elementwise<<<static_cast<unsigned>(blocks < 65535 ? blocks : 65535), 256, 0, st>>>(dy, z, n, dzbuf);
    if ((rc = last_launch_status())) return rc;
    dzp = dzbuf;
  }
  return x2g_linear_wgrad_ex(dzp, x, R, N, K, dw, db, flags, static_cast<char*>(workspace) + dz_bytes,
                             workspace_bytes - dz_bytes, stream);
}

X2G_API int32_t x2g_linear_wgrad_splits(int64_t R, int32_t O, int32_t I);

// slab count of a deferred x2g_dense_bwd_ex; the general path's slabs follow its dz buffer
X2G_API int32_t x2g_dense_bwd_splits(int64_t R, int32_t K, int32_t N) {
  if (R <= 0 || K <= 0 || N <= 0) return 0;
  if (dense_narrow_bwd(R, K, N)) return static_cast<int32_t>(narrow_bwd_grid(R));
  if (dense_persistent_bwd(R, K, N)) return static_cast<int32_t>(bwd_grid(R));
  return x2g_linear_wgrad_splits(R, N, K);
}

// byte offset of the weight-gradient slabs inside x2g_dense_bwd_ex's workspace
X2G_API int64_t x2g_dense_bwd_slab_offset(int64_t R, int32_t K, int32_t N) {
  if (R <= 0 || K <= 0 || N <= 0 || dense_persistent_bwd(R, K, N)) return 0;
  return static_cast<int64_t>(((static_cast<size_t>(R) * N * sizeof(float)) + 255) / 256 * 256);
}

X2G_API int x2g_dense_bwd(const float* dy, const float* z, int act, const float* x, const float* w, int64_t R,
                          int32_t K, int32_t N, float* dx, float* dw, float* db, void* workspace,
                          size_t workspace_bytes, void* stream) {
  return x2g_dense_bwd_ex(dy, z, act, x, w, R, K, N, dx, nullptr, dw, db, 0, workspace, workspace_bytes, stream);
}

// ------------------------------------------------------------------------------- fused ResidualLayer
X2G_API int x2g_residual_fwd(const float* x, const float* w0, const float* b0, const float* w1, const float* b1,
                             int64_t R, int32_t D, float* h, float* z0, float* z1, float* y, void* stream) {
  if (R < 0 || D <= 0) return X2G_EINVAL;
  if (R == 0) return X2G_OK;
  if (!x || !w0 || !w1 || !h || !z0 || !z1 || !y) return X2G_EINVAL;
  if (D > 128 || D % 4 || D <= 8 || R * 128 * 4 >= (int64_t(1) << 31)) return X2G_EUNSUPPORTED;
  if (!aligned16(x) || !aligned16(h) || !aligned16(z0) || !aligned16(z1) || !aligned16(y)) return X2G_EUNSUPPORTED;
  const int64_t ntiles = (R + 31) / 32;
  const unsigned grid = static_cast<unsigned>(ntiles < 256 ? ntiles : 256);
  residual_fwd_kernel<<<grid, 256, 0, as_stream(stream)>>>(x, w0, b0, w1, b1, R, D, h, z0, z1, y);
  return last_launch_status();
}

// ------------------------------------------------------------------------------- batched layers
X2G_API int x2g_dense_fwd_batched(const x2g_dense_fwd_group* groups, int32_t G, int64_t R, int32_t K, int32_t N,
                                  int act, void* stream) {
  if (!groups || G < 1 || G > X2G_MAX_GROUPS || R < 0 || K <= 0 || N <= 0 || (act != kActNone && act != kActSilu))
    return X2G_EINVAL;
  if (R == 0) return X2G_OK;
  if (K > 128 || N > 128 || K % 4 || N % 4 || K <= 8 || R * 128 * 4 >= (int64_t(1) << 31)) return X2G_EUNSUPPORTED;
  DenseFwdBatch b{};
  for (int g = 0; g < G; ++g) {
    const x2g_dense_fwd_group& p = groups[g];
    if (!p.x || !p.w || !p.y) return X2G_EINVAL;
    if (!aligned16(p.x) || !aligned16(p.y) || !aligned16(p.z) || !aligned16(p.res)) return X2G_EUNSUPPORTED;
    b.g[g] = p;
  }
  const int64_t ntiles = (R + 31) / 32;
  const dim3 grid(static_cast<unsigned>(ntiles < 512 ? ntiles : 512), G);
  dense_fwd_v6_batched<<<grid, 256, 0, as_stream(stream)>>>(b, R, K, N, act);
  return last_launch_status();
}

X2G_API int x2g_dense_bwd_batched(const x2g_dense_bwd_group* groups, int32_t G, int64_t R, int32_t K, int32_t N,
                                  int act, int flags, void* workspace, size_t workspace_bytes, void* stream) {
  if (!groups || G < 1 || G > X2G_MAX_GROUPS || R <= 0 || K <= 0 || N <= 0 ||
      (act != kActNone && act != kActSilu) || (flags & ~(X2G_ACCUM_WGRAD | X2G_DEFER_SLAB_SUM)))
    return X2G_EINVAL;
  if (!dense_persistent_bwd(R, K, N) || K % 4 || N % 4 || N <= 8) return X2G_EUNSUPPORTED;
  const size_t wsz = x2g_dense_bwd_workspace(R, K, N);
  if (!workspace || workspace_bytes < wsz * G) return X2G_EWORKSPACE;
  const int grid = static_cast<int>(bwd_grid(R));
  DenseBwdBatch b{};
  x2g_slab_job jobs[X2G_MAX_GROUPS];
  for (int g = 0; g < G; ++g) {
    const x2g_dense_bwd_group& p = groups[g];
    if (!p.dy || !p.x || !p.w || !p.dw || (act == kActSilu && !p.z) || (p.dx_add && !p.dx)) return X2G_EINVAL;
    if (!aligned16(p.dy) || !aligned16(p.z) || !aligned16(p.x) || !aligned16(p.dx) || !aligned16(p.dx_add))
      return X2G_EUNSUPPORTED;
    b.g[g] = p;
    b.part_w[g] = reinterpret_cast<float*>(static_cast<char*>(workspace) + wsz * g);
    b.part_b[g] = p.db ? b.part_w[g] + static_cast<int64_t>(grid) * N * K : nullptr;
    jobs[g] = x2g_slab_job{b.part_w[g], b.part_b[g], p.dw, p.db, static_cast<int64_t>(N) * K, p.db ? N : 0, grid};
  }
  hipStream_t st = as_stream(stream);
  dense_bwd_v8_batched<<<dim3(grid, G), 512, 0, st>>>(b, R, K, N, act);
  if (int rc = last_launch_status()) return rc;
  if (flags & X2G_DEFER_SLAB_SUM) return X2G_OK;
  return x2g_slab_sum_batch(jobs, G, (flags & X2G_ACCUM_WGRAD) ? 1 : 0, stream);
}
