// Diagnostic probe (not part of libx2g.so): sustained rate of the chain kernels' inner product
// (v_mfma_f32_16x16x4_f32, A from registers, B from an LDS image via ds_read_b128) with no
// epilogue and no barriers, to separate the product's own efficiency from the stage overheads.
#include <hip/hip_runtime.h>
#include <stdint.h>
typedef float f4 __attribute__((ext_vector_type(4)));

template <int RB, bool LDSB>
__global__ void __launch_bounds__(512, 1) probe(const float* __restrict__ src, float* __restrict__ out, int iters) {
  __shared__ f4 img[96 * 32];
  const int tid = threadIdx.x, lane = tid & 63, rl = lane & 15, g = lane >> 4;
  for (int q = tid; q < 96 * 32; q += 512) img[q] = f4{src[q & 127], 1.f, 2.f, 3.f};
  __syncthreads();
  f4 A[8];
  for (int b = 0; b < 8; ++b) A[b] = f4{src[b], src[b + 1], src[b + 2], src[b + 3]};
  f4 acc[RB];
  for (int rb = 0; rb < RB; ++rb) acc[rb] = f4{0.f, 0.f, 0.f, 0.f};
  f4 breg[RB];
  for (int rb = 0; rb < RB; ++rb) breg[rb] = f4{src[rb], 0.5f, 0.25f, 0.125f};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      f4 bo[RB];
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) bo[rb] = LDSB ? img[(16 * rb + rl) * 32 + ((4 * b + g) ^ rl)] : breg[rb];
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) acc[rb] = __builtin_amdgcn_mfma_f32_16x16x4f32(A[b][e], bo[rb][e], acc[rb], 0, 0, 0);
    }
  }
  f4 s = acc[0];
  for (int rb = 1; rb < RB; ++rb) s += acc[rb];
  reinterpret_cast<f4*>(out)[blockIdx.x * 512 + tid] = s;
}

extern "C" int probe_run(int variant, const float* src, float* out, int iters, int grid, void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  switch (variant) {
    case 0: probe<6, true><<<grid, 512, 0, st>>>(src, out, iters); break;
    case 1: probe<6, false><<<grid, 512, 0, st>>>(src, out, iters); break;
    case 2: probe<8, true><<<grid, 512, 0, st>>>(src, out, iters); break;
    case 3: probe<4, true><<<grid, 512, 0, st>>>(src, out, iters); break;
    default: return 1;
  }
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
