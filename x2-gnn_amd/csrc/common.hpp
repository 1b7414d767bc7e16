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


// Fixed-order sum of `splits` per-workgroup partial slabs (linear.hip): dw[i] (+)= sum_s part_w[s][i]
// and, when part_b and db are given, db likewise.
int sum_slabs_launch(const float* part_w, int64_t nw, const float* part_b, int64_t nb, int splits, float* dw,
                     float* db, bool accum, hipStream_t st);

// Masked loads without control flow.  Written as `ok ? load : 0`, the compiler sinks each load
// into a conditional block and then waits for it (s_waitcnt vmcnt(0)) before issuing the next:
// a batch of independent loads becomes a serial chain.  Loading from a clamped (always valid)
// address and multiplying by a 0/1 mask keeps every load unconditional and in flight together.
__device__ __forceinline__ float ld_pin(const float* p) { return *p; }
__device__ __forceinline__ float2 ld_pin2(const float* p) { return *reinterpret_cast<const float2*>(p); }
__device__ __forceinline__ float4 ld_pin4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ float keep(float v, bool ok) { return v * (ok ? 1.0f : 0.0f); }

// Wave-uniform value (forces the compiler to treat it as scalar).
__device__ __forceinline__ int uniform(int v) { return __builtin_amdgcn_readfirstlane(v); }

// Sum over aligned groups of `G` consecutive lanes (G power of two, <= 64); every lane of a
// group ends with the group total.
// Value of lane `lane` (wave-uniform index) in every lane: v_readlane into a scalar register.
__device__ __forceinline__ int lane_bcast(int v, int lane) { return __builtin_amdgcn_readlane(v, lane); }
__device__ __forceinline__ float lane_bcast(float v, int lane) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}

template <int CTL>
__device__ __forceinline__ float dpp_mov(float v);

template <int G>
__device__ __forceinline__ float group_sum(float v) {
  // groups of up to 16 lanes on DPP (quad permutes, then row_half_mirror / row_mirror: after the quad
  // steps every lane of a quad holds the same value, so the partner lane the mirrors pick gives the
  // same sums, bitwise, as xor 4 / xor 8); wider groups through ds_bpermute
  if (G >= 2) v += dpp_mov<0xB1>(v);   // quad_perm [1, 0, 3, 2]
  if (G >= 4) v += dpp_mov<0x4E>(v);   // quad_perm [2, 3, 0, 1]
  if (G >= 8) v += dpp_mov<0x141>(v);  // row_half_mirror
  if (G >= 16) v += dpp_mov<0x140>(v); // row_mirror
#pragma unroll
  for (int off = 16; off < G; off <<= 1) v += __shfl_xor(v, off, kWave);
  return v;
}

// Cross-lane sums on DPP (no LDS round trips, unlike __shfl_xor's ds_bpermute / ds_swizzle chains).
template <int CTL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTL, 0xF, 0xF, false));
}
// sum over each 16-lane DPP row, in every lane of the row
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp_mov<0xB1>(v);   // quad_perm [1, 0, 3, 2]
  v += dpp_mov<0x4E>(v);   // quad_perm [2, 3, 0, 1]
  v += dpp_mov<0x141>(v);  // row_half_mirror
  v += dpp_mov<0x140>(v);  // row_mirror
  return v;
}
// sum over each aligned 32-lane half of the wave, valid in its upper 16 lanes (16..31, 48..63):
// row_bcast15 adds lane 15 of rows 0 / 2 to rows 1 / 3
__device__ __forceinline__ float half32_sum_hi(float v) {
  v = row16_sum(v);
  return v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x142, 0xA, 0xF, false));
}
// sum over the whole wave, wave-uniform
__device__ __forceinline__ float wave64_sum(float v) {
  v = row16_sum(v);
  return (lane_bcast(v, 0) + lane_bcast(v, 16)) + (lane_bcast(v, 32) + lane_bcast(v, 48));
}

// A partner exchange for butterflies over lane bit log2(OFF): xor OFF for OFF 1, 2 and >= 16 (the
// last through ds_bpermute); OFF 4 / 8 take row_half_mirror / row_mirror, i.e. xor 7 / xor 15 inside
// a DPP row - the partner still has bit OFF flipped and every higher bit kept, and the masks stay
// triangular, so a butterfly that visits each bit once still sums every lane exactly once.
template <int OFF>
__device__ __forceinline__ float xor_xchg(float v) {
  if constexpr (OFF == 1) return dpp_mov<0xB1>(v);
  else if constexpr (OFF == 2) return dpp_mov<0x4E>(v);
  else if constexpr (OFF == 4) return dpp_mov<0x141>(v);
  else if constexpr (OFF == 8) return dpp_mov<0x140>(v);
  else return __shfl_xor(v, OFF, kWave);
}

template <int G>
__device__ __forceinline__ float group_max(float v) {
  if (G >= 2) v = fmaxf(v, xor_xchg<1>(v));
  if (G >= 4) v = fmaxf(v, xor_xchg<2>(v));
  if (G >= 8) v = fmaxf(v, xor_xchg<4>(v));
  if (G >= 16) v = fmaxf(v, xor_xchg<8>(v));
#pragma unroll
  for (int off = 16; off < G; off <<= 1) v = fmaxf(v, __shfl_xor(v, off, kWave));
  return v;
}

}  // namespace x2g
