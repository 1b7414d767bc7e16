// Shared helpers for the gfx950 kernels of libx2g.so.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/x2g.h"

#define X2G_API extern "C" __attribute__((visibility("default")))

namespace x2g {

constexpr int kWave = 64;  // CDNA wavefront

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

inline int last_launch_status() {
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? X2G_OK : static_cast<int>(e);
}

inline unsigned blocks_for(int64_t n, int per_block) {
  return static_cast<unsigned>((n + per_block - 1) / per_block);
}

// Wave-uniform value (forces the compiler to treat it as scalar).
__device__ __forceinline__ int uniform(int v) { return __builtin_amdgcn_readfirstlane(v); }

// Sum over aligned groups of `G` consecutive lanes (G power of two, <= 64); every lane of a
// group ends with the group total.
template <int G>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int off = 1; off < G; off <<= 1) v += __shfl_xor(v, off, kWave);
  return v;
}

template <int G>
__device__ __forceinline__ float group_max(float v) {
#pragma unroll
  for (int off = 1; off < G; off <<= 1) v = fmaxf(v, __shfl_xor(v, off, kWave));
  return v;
}

}  // namespace x2g
