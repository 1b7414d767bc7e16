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
      float v = 0.f;
      if (r < R && k < K) {
        v = A[r * K + k];
        if (ACT_IN == kActSilu) {  // dZ = dY * silu'(Z)
          const float z = zin[r * K + k];
          const float s = sigmoidf_(z);
          v = v * (s * (1.0f + z * (1.0f - s)));
        }
      }
      ra[u] = v;
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
      float v = 0.f;
      if (k < K && n < N) v = BT ? Bm[static_cast<int64_t>(n) * K + k] : Bm[static_cast<int64_t>(k) * N + n];
      rb[u] = v;
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

}  // namespace x2g

using namespace x2g;

X2G_API int x2g_dense_fwd(const float* x, const float* w, const float* b, int64_t R, int32_t K, int32_t N, int act,
                          const float* res, float* y, float* z, void* stream) {
  if (R < 0 || K <= 0 || N <= 0 || (act != kActNone && act != kActSilu)) return X2G_EINVAL;
  if (R == 0) return X2G_OK;
  if (!x || !w || !y) return X2G_EINVAL;
  dim3 grid(static_cast<unsigned>((R + kDenseRows - 1) / kDenseRows), (N + kDenseCols - 1) / kDenseCols);
  dense_rows<true, kActNone><<<grid, 256, 0, as_stream(stream)>>>(x, w, b, res, nullptr, R, K, N, act, y, z,
                                                                   nullptr);
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
