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
// K = 6, the readout head with N = 1): the weight is staged into LDS ONCE per workgroup and the
// workgroup walks 32-row tiles, prefetching the next tile into registers while the MFMAs run.
// One workgroup per CU (grid <= 256), 4 waves, wave w owns output columns 32w..32w+31.
constexpr int kPTile = 32;       // rows per tile
constexpr int kPStride = 129;    // LDS row stride (floats): conflict-free row and column access
constexpr int kPGrid = 256;      // workgroups (one per CU)


// 32 rows x 128 columns of a row-major [R, cols] matrix -> 16 floats per thread (coalesced).
// Branch-free: addresses are clamped into the matrix and out-of-range values masked to 0, so
// all 16 loads issue back to back.
__device__ __forceinline__ void tile_load(const float* __restrict__ m, int64_t r0, int64_t R, int cols, float (&v)[16]) {
#pragma unroll
  for (int u = 0; u < 16; ++u) {
    const int idx = threadIdx.x + 256 * u, rr = idx >> 7, cc = idx & 127;
    const int64_t r = r0 + rr;
    const int64_t rc = r < R ? r : R - 1;
    const int ccc = cc < cols ? cc : cols - 1;
    const float x = ld_pin(m + rc * cols + ccc);
    v[u] = keep(x, r < R && cc < cols);
  }
}

// Stage a [N, K] weight (N, K <= 128, zero padded) into LDS, transposed ([k][n]) or not ([n][k]).
// Loads go out 16 at a time so their latencies overlap (the weight is L2-resident after the
// first workgroup touches it).
template <bool TRANSPOSE>
__device__ __forceinline__ void stage_weight(float (*ws)[kPStride], const float* __restrict__ W, int N, int K) {
#pragma unroll 1
  for (int round = 0; round < 4; ++round) {
    float v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int idx = threadIdx.x + 256 * (16 * round + u), n = idx >> 7, k = idx & 127;
      const float x = ld_pin(W + static_cast<int64_t>(n < N ? n : N - 1) * K + (k < K ? k : K - 1));
      v[u] = keep(x, n < N && k < K);
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int idx = threadIdx.x + 256 * (16 * round + u), n = idx >> 7, k = idx & 127;
      if (TRANSPOSE) ws[k][n] = v[u];
      else ws[n][k] = v[u];
    }
  }
}

__device__ __forceinline__ void tile_store(float (*lds)[kPStride], const float (&v)[16]) {
#pragma unroll
  for (int u = 0; u < 16; ++u) {
    const int idx = threadIdx.x + 256 * u;
    lds[idx >> 7][idx & 127] = v[u];
  }
}

// y = act(x w^T + b) (+ res), z = x w^T + b.  KSTEPS = 2-row k steps compiled (K <= 2*KSTEPS).
template <int KSTEPS>
__global__ void __launch_bounds__(256) dense_fwd_persist(const float* __restrict__ X, const float* __restrict__ W,
                                                         const float* __restrict__ bias,
                                                         const float* __restrict__ res, int64_t R, int K, int N,
                                                         int act, float* __restrict__ Y, float* __restrict__ Z) {
  __shared__ float Ws[128][kPStride];          // B operand [k][n] = w[n][k]
  __shared__ float As[2][kPTile][kPStride];    // x tile [r][k], double buffered
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  stage_weight<true>(Ws, W, N, K);
  const int64_t ntiles = (R + kPTile - 1) / kPTile;
  const int n = wave * 32 + (lane & 31);
  const float bn = (bias && n < N) ? bias[n] : 0.f;
  float va[16];
  int64_t t = blockIdx.x;
  if (t < ntiles) tile_load(X, t * kPTile, R, K, va);
  for (int it = 0; t < ntiles; t += gridDim.x, ++it) {
    const int buf = it & 1;
    tile_store(As[buf], va);
    __syncthreads();
    if (t + gridDim.x < ntiles) tile_load(X, (t + gridDim.x) * kPTile, R, K, va);
    // two independent accumulator chains (k steps [0, KSTEPS/2) and [KSTEPS/2, KSTEPS)) so
    // consecutive MFMAs never wait on each other's result
    floatx16 acc0, acc1;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      acc0[j] = 0.f;
      acc1[j] = 0.f;
    }
    constexpr int HALF = KSTEPS / 2;
#pragma unroll
    for (int ks = 0; ks < HALF; ++ks) {
      const int k0 = 2 * ks + (lane >> 5), k1 = 2 * (ks + HALF) + (lane >> 5);
      acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(As[buf][lane & 31][k0], Ws[k0][wave * 32 + (lane & 31)], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(As[buf][lane & 31][k1], Ws[k1][wave * 32 + (lane & 31)], acc1, 0, 0, 0);
    }
    // epilogue: all residual loads first (clamped rows), then bias / activation / stores
    const int64_t rbase = t * kPTile + 4 * (lane >> 5);
    float rv[16];
    if (res) {
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int64_t r = rbase + (j & 3) + 8 * (j >> 2);
        rv[j] = res[(r < R ? r : R - 1) * N + (n < N ? n : N - 1)];
      }
    }
    if (n < N) {
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int64_t r = rbase + (j & 3) + 8 * (j >> 2);
        float v = acc0[j] + acc1[j] + bn;
        const int64_t o = r * N + n;
        if (r < R) {
          if (Z) Z[o] = v;
          if (act == kActSilu) v = v / (1.0f + expf(-v));
          if (res) v += rv[j];
          Y[o] = v;
        }
      }
    }
  }
}

// Backward of dense_fwd_persist, fused: dz = dy * act'(z); dx = dz w (if dx != NULL);
// per-workgroup partial weight / bias gradients dz^T x and colsum(dz) over the workgroup's
// tiles, written to slab blockIdx.x (summed afterwards in a fixed order).  NSTEPS: N <= 2*NSTEPS.
template <int NSTEPS>
__global__ void __launch_bounds__(256) dense_bwd_persist(const float* __restrict__ dY, const float* __restrict__ Zin,
                                                         const float* __restrict__ X, const float* __restrict__ W,
                                                         int64_t R, int K, int N, int act, float* __restrict__ dX,
                                                         float* __restrict__ part_w, float* __restrict__ part_b) {
  __shared__ float Ws[128][kPStride];          // B operand of dx = dz w: [n][k] = w[n][k]
  __shared__ float Ds[2][kPTile][kPStride];    // dz tile [r][n]
  __shared__ float Xs[2][kPTile][kPStride];    // x tile [r][k]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  stage_weight<false>(Ws, W, N, K);
  const int64_t ntiles = (R + kPTile - 1) / kPTile;
  floatx16 accw[4];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int j = 0; j < 16; ++j) accw[q][j] = 0.f;
  float bsum = 0.f;
  float vd[16], vz[16], vx[16];
  int64_t t = blockIdx.x;
  auto load = [&](int64_t tt) {
    tile_load(dY, tt * kPTile, R, N, vd);
    if (act == kActSilu) tile_load(Zin, tt * kPTile, R, N, vz);
    tile_load(X, tt * kPTile, R, K, vx);
  };
  if (t < ntiles) load(t);
  for (int it = 0; t < ntiles; t += gridDim.x, ++it) {
    const int buf = it & 1;
    if (act == kActSilu) {
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const float s = 1.0f / (1.0f + expf(-vz[u]));
        vd[u] = vd[u] * (s * (1.0f + vz[u] * (1.0f - s)));
      }
    }
    tile_store(Ds[buf], vd);
    tile_store(Xs[buf], vx);
    __syncthreads();
    if (t + gridDim.x < ntiles) load(t + gridDim.x);
    if (dX) {  // dx tile = dz (32 x N) . w (N x K): wave w owns k columns 32w..
      floatx16 acc0, acc1;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        acc0[j] = 0.f;
        acc1[j] = 0.f;
      }
      constexpr int HALF = NSTEPS / 2;
#pragma unroll
      for (int ks = 0; ks < HALF; ++ks) {
        const int k0 = 2 * ks + (lane >> 5), k1 = 2 * (ks + HALF) + (lane >> 5);
        acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(Ds[buf][lane & 31][k0], Ws[k0][wave * 32 + (lane & 31)], acc0, 0,
                                                    0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(Ds[buf][lane & 31][k1], Ws[k1][wave * 32 + (lane & 31)], acc1, 0,
                                                    0, 0);
      }
      const int k = wave * 32 + (lane & 31);
      if (k < K) {
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          const int64_t r = t * kPTile + (j & 3) + 8 * (j >> 2) + 4 * (lane >> 5);
          if (r < R) dX[r * K + k] = acc0[j] + acc1[j];
        }
      }
    }
    // dW[n][k] += sum_r dz[r][n] x[r][k]: wave w owns n rows 32w..32w+31, four 32-wide k blocks
#pragma unroll 4
    for (int ks = 0; ks < kPTile / 2; ++ks) {
      const int rr = 2 * ks + (lane >> 5);
      const float a = Ds[buf][rr][wave * 32 + (lane & 31)];
#pragma unroll
      for (int q = 0; q < 4; ++q)
        accw[q] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, Xs[buf][rr][q * 32 + (lane & 31)], accw[q], 0, 0, 0);
    }
    if (part_b && tid < 128) {
#pragma unroll 8
      for (int rr = 0; rr < kPTile; ++rr) bsum += Ds[buf][rr][tid];
    }
  }
  float* slab = part_w + static_cast<int64_t>(blockIdx.x) * N * K;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int k = q * 32 + (lane & 31);
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int nn = wave * 32 + (j & 3) + 8 * (j >> 2) + 4 * (lane >> 5);
      if (nn < N && k < K) slab[static_cast<int64_t>(nn) * K + k] = accw[q][j];
    }
  }
  if (part_b && tid < N) part_b[static_cast<int64_t>(blockIdx.x) * N + tid] = bsum;
}


// ------------------------------------------------------------------------------------------------
// Weight-in-registers form (K, N <= 128).  A workgroup (4 waves) walks 64-row blocks; wave w owns
// rows 32*(w>>1).. and output columns 64*(w&1).. (two 32x32 MFMA tiles), and keeps the MFMA B
// fragments of its 64 weight columns in VGPRs for the whole kernel, so the inner loop is ONE
// LDS read (the A fragment) feeding two independent MFMAs.  LDS holds the weight only during the
// prologue and is then reused as the double-buffered 64-row A block (66 KB: two workgroups per CU).
//   DGRAD = false: y = act(x w^T + b) (+ res), z = x w^T + b           (B[k][n] = w[n][k])
//   DGRAD = true : a = dy * act'(z) -> dz (optional), dx = a w         (B[k][n] = w[k][n])
constexpr int kWBlock = 64;
constexpr int kWGrid = 512;
constexpr int kWPer = kWBlock * 128 / 256;  // A elements staged per thread per block

template <bool DGRAD>
__device__ __forceinline__ void wreg_load_block(const float* __restrict__ A, const float* __restrict__ zin,
                                                int64_t blk, int64_t R, int Kin, int act, float (&xa)[kWPer]) {
#pragma unroll
  for (int u = 0; u < kWPer; ++u) {
    const int idx = threadIdx.x + 256 * u, rr = idx >> 7, cc = idx & 127;
    const int64_t r = blk * kWBlock + rr;
    const int64_t rc = r < R ? r : R - 1;
    const int ccc = cc < Kin ? cc : Kin - 1;
    float v = ld_pin(A + rc * Kin + ccc);
    if (DGRAD && act == kActSilu) {
      const float z = ld_pin(zin + rc * Kin + ccc);
      const float sg = 1.0f / (1.0f + expf(-z));
      v = v * (sg * (1.0f + z * (1.0f - sg)));
    }
    xa[u] = keep(v, r < R && cc < Kin);
  }
}

template <int KSTEPS, bool DGRAD>
__global__ void __launch_bounds__(256) dense_wreg(const float* __restrict__ A, const float* __restrict__ W,
                                                     const float* __restrict__ bias, const float* __restrict__ res,
                                                     const float* __restrict__ zin, int64_t R, int Kin, int Nout,
                                                     int Nw, int Kw, int act, float* __restrict__ Y,
                                                     float* __restrict__ zout, float* __restrict__ aout) {
  // Kin: contraction length (columns of A); Nout: output columns; W is [Nw, Kw] row-major.
  // prologue: the weight image [128][129]; afterwards the same bytes hold the A blocks [2][64][129]
  __shared__ union {
    float w[128][kPStride];
    float a[2][kWBlock][kPStride];
  } sh;
  auto& Ws = sh.w;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int rt = wave >> 1, ch = wave & 1;
  stage_weight<false>(Ws, W, Nw, Kw);
  __syncthreads();
  float wr[2][KSTEPS];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int s2 = 0; s2 < KSTEPS; ++s2) {
      const int kk = 2 * s2 + (lane >> 5), nn = 64 * ch + 32 * t + (lane & 31);
      wr[t][s2] = DGRAD ? Ws[kk][nn] : Ws[nn][kk];
    }
  float bn[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int n = 64 * ch + 32 * t + (lane & 31);
    bn[t] = (bias && n < Nout) ? bias[n] : 0.f;
  }
  __syncthreads();  // the weight image is dead from here on; the space becomes the A blocks
  const int64_t nblocks = (R + kWBlock - 1) / kWBlock;
  constexpr int PER = kWPer;
  float xa[PER];
  int64_t blk = blockIdx.x;
  if (blk < nblocks) wreg_load_block<DGRAD>(A, zin, blk, R, Kin, act, xa);
  for (int it = 0; blk < nblocks; blk += gridDim.x, ++it) {
    auto& As = sh.a[it & 1];
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int idx = tid + 256 * u;
      As[idx >> 7][idx & 127] = xa[u];
    }
    if (DGRAD && aout) {  // dz = dy * act'(z), kept for the weight gradient
#pragma unroll
      for (int u = 0; u < PER; ++u) {
        const int idx = tid + 256 * u, rr = idx >> 7, cc = idx & 127;
        const int64_t r = blk * kWBlock + rr;
        if (r < R && cc < Kin) aout[r * Kin + cc] = xa[u];
      }
    }
    __syncthreads();
    if (blk + gridDim.x < nblocks) wreg_load_block<DGRAD>(A, zin, blk + gridDim.x, R, Kin, act, xa);
    floatx16 acc0, acc1;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      acc0[j] = 0.f;
      acc1[j] = 0.f;
    }
#pragma unroll
    for (int s2 = 0; s2 < KSTEPS; ++s2) {
      const float a = As[32 * rt + (lane & 31)][2 * s2 + (lane >> 5)];
      acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, wr[0][s2], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, wr[1][s2], acc1, 0, 0, 0);
    }
    const int64_t rbase = blk * kWBlock + 32 * rt + 4 * (lane >> 5);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int n = 64 * ch + 32 * t + (lane & 31);
      float rv[16];
      if (res) {
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          const int64_t r = rbase + (j & 3) + 8 * (j >> 2);
          rv[j] = ld_pin(res + (r < R ? r : R - 1) * Nout + (n < Nout ? n : Nout - 1));
        }
      }
      if (n < Nout) {
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          const int64_t r = rbase + (j & 3) + 8 * (j >> 2);
          if (r < R) {
            float v = (t == 0 ? acc0[j] : acc1[j]) + bn[t];
            const int64_t o = r * Nout + n;
            if (zout) zout[o] = v;
            if (!DGRAD && act == kActSilu) v = v / (1.0f + expf(-v));
            if (res) v += rv[j];
            Y[o] = v;
          }
        }
      }
    }
  }
}

}  // namespace x2g

using namespace x2g;

X2G_API int x2g_dense_fwd(const float* x, const float* w, const float* b, int64_t R, int32_t K, int32_t N, int act,
                          const float* res, float* y, float* z, void* stream) {
  if (R < 0 || K <= 0 || N <= 0 || (act != kActNone && act != kActSilu)) return X2G_EINVAL;
  if (R == 0) return X2G_OK;
  if (!x || !w || !y) return X2G_EINVAL;
  hipStream_t st = as_stream(stream);
  const int variant = tuning(kTuneDenseFwd);  // 0: LDS-persistent, 1: weight-in-registers, 2: tiled
  if (K <= 128 && N <= 128 && variant == 0) {
    const int64_t ntiles = (R + kPTile - 1) / kPTile;
    const unsigned grid = static_cast<unsigned>(ntiles < kPGrid ? ntiles : kPGrid);
    if (K <= 8)
      dense_fwd_persist<4><<<grid, 256, 0, st>>>(x, w, b, res, R, K, N, act, y, z);
    else
      dense_fwd_persist<64><<<grid, 256, 0, st>>>(x, w, b, res, R, K, N, act, y, z);
    return last_launch_status();
  }
  if (K <= 128 && N <= 128 && variant == 1) {
    const int64_t nblk = (R + kWBlock - 1) / kWBlock;
    const unsigned grid = static_cast<unsigned>(nblk < kWGrid ? nblk : kWGrid);
    if (K <= 8)
      dense_wreg<4, false><<<grid, 256, 0, st>>>(x, w, b, res, nullptr, R, K, N, N, K, act, y, z, nullptr);
    else
      dense_wreg<64, false><<<grid, 256, 0, st>>>(x, w, b, res, nullptr, R, K, N, N, K, act, y, z, nullptr);
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
int sum_slabs_launch(const float* part, int64_t n, int splits, float* out, hipStream_t st);
}  // namespace x2g

X2G_API size_t x2g_linear_wgrad_workspace(int64_t R, int32_t O, int32_t I);
X2G_API int x2g_linear_wgrad(const float* dy, const float* x, int64_t R, int32_t O, int32_t I, float* dw, float* db,
                             void* workspace, size_t workspace_bytes, void* stream);

static inline bool dense_persistent_bwd(int64_t R, int32_t K, int32_t N) { return K <= 128 && N <= 128 && R > 0; }

X2G_API size_t x2g_dense_bwd_workspace(int64_t R, int32_t K, int32_t N) {
  if (R <= 0 || K <= 0 || N <= 0) return 0;
  if (dense_persistent_bwd(R, K, N)) {
    const int64_t ntiles = (R + kPTile - 1) / kPTile;
    const int64_t g = ntiles < kPGrid ? ntiles : kPGrid;
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
    const int64_t ntiles = (R + kPTile - 1) / kPTile;
    const int grid = static_cast<int>(ntiles < kPGrid ? ntiles : kPGrid);
    float* part_w = static_cast<float*>(workspace);
    float* part_b = db ? part_w + static_cast<int64_t>(grid) * N * K : nullptr;
    if (N <= 8)
      dense_bwd_persist<4><<<grid, 256, 0, st>>>(dy, z, x, w, R, K, N, act, dx, part_w, part_b);
    else
      dense_bwd_persist<64><<<grid, 256, 0, st>>>(dy, z, x, w, R, K, N, act, dx, part_w, part_b);
    int rc = last_launch_status();
    if (rc) return rc;
    if ((rc = sum_slabs_launch(part_w, static_cast<int64_t>(N) * K, grid, dw, st))) return rc;
    if (db && (rc = sum_slabs_launch(part_b, N, grid, db, st))) return rc;
    return X2G_OK;
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
