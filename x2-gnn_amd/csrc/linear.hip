// Weight gradients of the row-wise dense layers: dW[o,i] = sum_r dY[r,o] X[r,i], db[o] = sum_r dY[r,o].
//
// Every dense layer of X2-GNN runs on E (line nodes), N (atoms) or T (triplets) rows with tiny
// weights (128x128, 128x42, 256x338, ...).  Their weight gradient is a GEMM with a huge K
// (the row count, 2e4..2e5) and a tiny M x N output; the vendor GEMMs pick a handful of
// output tiles and no K split for that shape (hipBLASLt: 90 us for 128x128 over 21k rows,
// 440 us for lin_sbf's 128x42 over 194k rows on MI355X).  Here the rows are split over many
// workgroups (<= 160 slices of >= 64 rows), every workgroup computes its slice's full 128x128 output
// block with f32 MFMA (v_mfma_f32_32x32x2_f32: exact fp32 FMA chains), writes it to a partial
// slab, and a second pass sums the slabs in a fixed order: deterministic, no atomics.
#include "common.hpp"

namespace x2g {

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int kWgTile = 128;       // output block (o) x (i) per workgroup
constexpr int kWgChunk = 32;       // rows staged in LDS per iteration
constexpr int kWgMinSplits = 160;        // row splits for a full 128x128 output block
constexpr int kWgMaxSplits = 1024;       // ... and for narrow outputs (cheap slabs)
constexpr int64_t kWgSlabBudget = 16 << 20;  // bytes of partial slabs one call may write
constexpr int kLdsStride = kWgTile + 4;  // keeps 16-byte row alignment for the float4 stores

// Chunk of 32 rows x 128 columns of one operand, held in registers between global and LDS.
// Load modes: kScalar = 16 scalars per thread; kVec = 4 float4 per thread (columns a multiple of
// 4); kFlat = the chunk's 32 full rows are one contiguous span of 32*cols floats (cols <= 128),
// read as float4 whatever cols is (32*cols is a multiple of 4 and the span starts 16-byte
// aligned): lin_sbf's 42-wide sbf rows take this path.
enum { kScalar = 0, kVec = 1, kFlat = 2 };

template <int MODE>
struct ChunkRegs {
  float v[16];
};

template <int MODE>
__device__ __forceinline__ void load_chunk(const float* __restrict__ m, int cols, int c0, int64_t r0,
                                           int64_t r_end, ChunkRegs<MODE>& reg) {
  const int tid = threadIdx.x;
  if (MODE == kFlat) {
    const int64_t nval = (r_end - r0 < kWgChunk ? r_end - r0 : kWgChunk) * cols;  // valid floats
    const int nq = (kWgChunk * cols) >> 2;
    const float* base = m + r0 * cols;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int qi = tid + 256 * u;
      const bool ok = qi < nq && 4 * qi < nval;
      const float4 f = ld_pin4(base + (ok ? 4 * qi : 0));
      reg.v[4 * u] = keep(f.x, ok && 4 * qi < nval);
      reg.v[4 * u + 1] = keep(f.y, ok && 4 * qi + 1 < nval);
      reg.v[4 * u + 2] = keep(f.z, ok && 4 * qi + 2 < nval);
      reg.v[4 * u + 3] = keep(f.w, ok && 4 * qi + 3 < nval);
    }
  } else if (MODE == kVec) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int q = tid + 256 * u, rr = q >> 5, c = c0 + 4 * (q & 31);
      const int64_t r = r0 + rr;
      const bool ok = r < r_end && c < cols;
      const float4 f = ld_pin4(m + (ok ? r * cols + c : 0));
      reg.v[4 * u] = keep(f.x, ok);
      reg.v[4 * u + 1] = keep(f.y, ok);
      reg.v[4 * u + 2] = keep(f.z, ok);
      reg.v[4 * u + 3] = keep(f.w, ok);
    }
  } else {
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int q = tid + 256 * u, rr = q >> 7, c = c0 + (q & 127);
      const int64_t r = r0 + rr;
      const bool ok = r < r_end && c < cols;
      const float x = ld_pin(m + (ok ? r * cols + c : 0));
      reg.v[u] = keep(x, ok);
    }
  }
}

template <int MODE>
__device__ __forceinline__ void store_chunk(float (*lds)[kLdsStride], const ChunkRegs<MODE>& reg, int cols) {
  const int tid = threadIdx.x;
  if (MODE == kFlat) {
    const int nq = (kWgChunk * cols) >> 2;
    const unsigned magic = 0xFFFFFFFFu / static_cast<unsigned>(cols) + 1u;  // wraps to 0 for cols == 1
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int qi = tid + 256 * u;
      if (qi < nq) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {  // f / cols by a multiply-high (exact for f < 2^16)
          const unsigned f = 4 * qi + e, rr = cols == 1 ? f : __umulhi(f, magic), c = f - rr * cols;
          lds[rr][c] = reg.v[4 * u + e];
        }
      }
    }
    // columns cols..127 of the chunk stay as they are: they only meet output columns >= cols,
    // which are never written back
  } else if (MODE == kVec) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int q = tid + 256 * u;
      *reinterpret_cast<float4*>(&lds[q >> 5][4 * (q & 31)]) =
          make_float4(reg.v[4 * u], reg.v[4 * u + 1], reg.v[4 * u + 2], reg.v[4 * u + 3]);
    }
  } else {
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int q = tid + 256 * u;
      lds[q >> 7][q & 127] = reg.v[u];
    }
  }
}

// One workgroup = one 128x128 output block x one row slice.  The next 32-row chunk is loaded
// into registers while the MFMAs consume the current one from LDS.
template <int MA, int MB>
__global__ void __launch_bounds__(256) wgrad_partial(const float* __restrict__ dy, const float* __restrict__ x,
                                                     int64_t R, int O, int I, int tiles_i, int64_t rows_per_split,
                                                     float* __restrict__ part, float* __restrict__ part_b) {
  __shared__ __attribute__((aligned(16))) float As[kWgChunk][kLdsStride];
  __shared__ __attribute__((aligned(16))) float Bs[kWgChunk][kLdsStride];
  const int ob = blockIdx.x / tiles_i, ib = blockIdx.x % tiles_i;
  const int split = blockIdx.y;
  const int64_t r_begin = static_cast<int64_t>(split) * rows_per_split;
  const int64_t r_end = r_begin + rows_per_split < R ? r_begin + rows_per_split : R;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int o0 = ob * kWgTile, i0 = ib * kWgTile;
  const bool do_bias = part_b && ib == 0;
  const int nt = uniform((I - i0 + 31) / 32 < 4 ? (I - i0 + 31) / 32 : 4);  // live 32-wide column blocks
  floatx16 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[t][j] = 0.f;
  float bsum = 0.f;
  ChunkRegs<MA> ra;
  ChunkRegs<MB> rb;
  load_chunk<MA>(dy, O, o0, r_begin, r_end, ra);
  load_chunk<MB>(x, I, i0, r_begin, r_end, rb);
  for (int64_t r0 = r_begin; r0 < r_end; r0 += kWgChunk) {
    store_chunk<MA>(As, ra, O);
    store_chunk<MB>(Bs, rb, I);
    __syncthreads();
    if (r0 + kWgChunk < r_end) {  // prefetch the next chunk; it lands while the MFMAs run
      load_chunk<MA>(dy, O, o0, r0 + kWgChunk, r_end, ra);
      load_chunk<MB>(x, I, i0, r0 + kWgChunk, r_end, rb);
    }
#pragma unroll 4
    for (int ks = 0; ks < kWgChunk / 2; ++ks) {
      const int kr = 2 * ks + (lane >> 5);
      const float a = As[kr][wave * 32 + (lane & 31)];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        if (t < nt) {  // column blocks past I (e.g. lin_sbf's 42 columns: 2 of 4) are skipped
          const float b = Bs[kr][t * 32 + (lane & 31)];
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[t], 0, 0, 0);
        }
      }
    }
    if (do_bias && tid < kWgTile) {
#pragma unroll 8
      for (int rr = 0; rr < kWgChunk; ++rr) bsum += As[rr][tid];
    }
    __syncthreads();
  }
  // C/D layout of the 32x32 f32 accumulator: col = lane&31, row = (j&3) + 8*(j>>2) + 4*(lane>>5)
  float* slab = part + static_cast<int64_t>(split) * O * I;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int i = i0 + t * 32 + (lane & 31);
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int o = o0 + wave * 32 + (j & 3) + 8 * (j >> 2) + 4 * (lane >> 5);
      if (o < O && i < I) slab[static_cast<int64_t>(o) * I + i] = acc[t][j];
    }
  }
  if (do_bias && tid < kWgTile && o0 + tid < O) part_b[static_cast<int64_t>(split) * O + o0 + tid] = bsum;
}

// out[e] = sum_s part[s][e] in a fixed order: a block owns 256 consecutive elements (4 per lane,
// one 16-byte load per slab when the slabs allow it), each of its 4 waves sums a quarter of the
// slabs, then the quarters are added in wave order.  The slabs are read once at 16 B per lane
// (a wave keeps 8 KB in flight), so the pass runs at stream bandwidth instead of 256-byte requests.
constexpr int kSlabElems = 256;  // elements per block

// ld > 0: element e is (row e / 128, column e % 128) of a block written at out + row * ld + column,
// columns < cols only (a 128-wide slab of a larger weight).
__device__ __forceinline__ void sum_slabs_block(const float* __restrict__ part, int64_t n, int splits, int64_t blk,
                                                bool accum, float* __restrict__ out, float4 (*red)[64], int ld = 0,
                                                int cols = 0) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t e = blk * kSlabElems + 4 * lane;
  const int per = (splits + 3) / 4;
  const int k0 = wave * per, k1 = k0 + per < splits ? k0 + per : splits;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  const bool vec = (n & 3) == 0 && (reinterpret_cast<uintptr_t>(part) & 15) == 0;  // block-uniform
  if (vec) {
    if (e < n) {
      const float4* p = reinterpret_cast<const float4*>(part + e);
      const int64_t stride = n / 4;
#pragma unroll 8
      for (int k = k0; k < k1; ++k) {
        const float4 v = p[static_cast<int64_t>(k) * stride];
        s.x += v.x;
        s.y += v.y;
        s.z += v.z;
        s.w += v.w;
      }
    }
  } else {
    float t[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < 4; ++c)
      if (e + c < n) {
#pragma unroll 4
        for (int k = k0; k < k1; ++k) t[c] += part[static_cast<int64_t>(k) * n + e + c];
      }
    s = make_float4(t[0], t[1], t[2], t[3]);
  }
  red[wave][lane] = s;
  __syncthreads();
  if (wave == 0 && e < n) {
    const float4 a = red[0][lane], b = red[1][lane], c = red[2][lane], d = red[3][lane];
    const float v[4] = {((a.x + b.x) + c.x) + d.x, ((a.y + b.y) + c.y) + d.y, ((a.z + b.z) + c.z) + d.z,
                        ((a.w + b.w) + c.w) + d.w};
    if (ld > 0) {  // the 4 elements share a row (128 % 4 == 0)
      const int64_t row = e >> 7;
      const int c0 = static_cast<int>(e & 127);
      float* o = out + row * ld + c0;
#pragma unroll
      for (int c4 = 0; c4 < 4; ++c4)
        if (c0 + c4 < cols) o[c4] = accum ? o[c4] + v[c4] : v[c4];
    } else {
#pragma unroll
      for (int c4 = 0; c4 < 4; ++c4)
        if (e + c4 < n) out[e + c4] = accum ? out[e + c4] + v[c4] : v[c4];
    }
  }
}

// Many slabs (the per-workgroup partials of the gate, radial and conv weight gradients: up to 256
// of a few thousand elements): the block above would walk splits / 4 slabs per wave, one memory
// round trip per 8, and its few blocks became the batch launch's tail.  Here a block takes 64
// elements and 16 split phases (lane l: float4 l & 15, phase 4 wave + l / 16), so a phase walks
// splits / 16 slabs and there are 4x as many blocks; the 16 phase sums are added in phase order.
// Used when the slabs allow 16-byte loads (block-uniform; the host counts blocks by the same rule).
constexpr int kSlabNarrowElems = 64;
constexpr int kSlabNarrowMin = 33;  // splits from which a slab set takes the narrow form

__host__ __device__ __forceinline__ bool slab_narrow(const float* part, int64_t n, int splits) {
  return splits >= kSlabNarrowMin && (n & 3) == 0 && (reinterpret_cast<uintptr_t>(part) & 15) == 0;
}

__device__ __forceinline__ void sum_slabs_block_narrow(const float* __restrict__ part, int64_t n, int splits,
                                                       int64_t blk, bool accum, float* __restrict__ out,
                                                       float4 (*red)[64], int ld, int cols) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int q = lane & 15, ph = 4 * wave + (lane >> 4);
  const int64_t e = blk * kSlabNarrowElems + 4 * q;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (e < n) {
    const float4* p = reinterpret_cast<const float4*>(part + e);
    const int64_t stride = n / 4;
#pragma unroll 8
    for (int k = ph; k < splits; k += 16) {
      const float4 v = p[static_cast<int64_t>(k) * stride];
      s.x += v.x;
      s.y += v.y;
      s.z += v.z;
      s.w += v.w;
    }
  }
  float4* r = &red[0][0];  // [16 phases][16 float4]
  r[ph * 16 + q] = s;
  __syncthreads();
  if (threadIdx.x < 16 && e < n) {
    float v[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int h = 0; h < 16; ++h) {
      const float4 a = r[h * 16 + q];
      v[0] += a.x;
      v[1] += a.y;
      v[2] += a.z;
      v[3] += a.w;
    }
    if (ld > 0) {
      const int64_t row = e >> 7;
      const int c0 = static_cast<int>(e & 127);
      float* o = out + row * ld + c0;
#pragma unroll
      for (int c4 = 0; c4 < 4; ++c4)
        if (c0 + c4 < cols) o[c4] = accum ? o[c4] + v[c4] : v[c4];
    } else {
#pragma unroll
      for (int c4 = 0; c4 < 4; ++c4)
        if (e + c4 < n) out[e + c4] = accum ? out[e + c4] + v[c4] : v[c4];
    }
  }
}

// blocks of one slab set, and the block body, in the form slab_narrow picks
__host__ __device__ __forceinline__ int64_t slab_blocks(const float* part, int64_t n, int splits) {
  const int64_t per = slab_narrow(part, n, splits) ? kSlabNarrowElems : kSlabElems;
  return n > 0 ? (n + per - 1) / per : 0;
}
__device__ __forceinline__ void sum_slabs_any(const float* __restrict__ part, int64_t n, int splits, int64_t blk,
                                              bool accum, float* __restrict__ out, float4 (*red)[64], int ld = 0,
                                              int cols = 0) {
  if (slab_narrow(part, n, splits))
    sum_slabs_block_narrow(part, n, splits, blk, accum, out, red, ld, cols);
  else
    sum_slabs_block(part, n, splits, blk, accum, out, red, ld, cols);
}

__global__ void __launch_bounds__(256) sum_slabs(const float* __restrict__ part, int64_t n, int splits, int accum,
                                                 float* __restrict__ out) {
  __shared__ float4 red[4][64];
  sum_slabs_any(part, n, splits, blockIdx.x, accum != 0, out, red);
}

// Two slab sets (weight and bias partials) in one launch: blocks [0, nblk_a) take the first.
__global__ void __launch_bounds__(256) sum_slabs2(const float* __restrict__ part_a, int64_t na,
                                                  const float* __restrict__ part_b, int64_t nb, int splits, int accum,
                                                  float* __restrict__ out_a, float* __restrict__ out_b) {
  __shared__ float4 red[4][64];
  const int64_t nblk_a = slab_blocks(part_a, na, splits);
  if (static_cast<int64_t>(blockIdx.x) < nblk_a)
    sum_slabs_any(part_a, na, splits, blockIdx.x, accum != 0, out_a, red);
  else
    sum_slabs_any(part_b, nb, splits, blockIdx.x - nblk_a, accum != 0, out_b, red);
}

// dw (and db when part_b != NULL) from their slabs, one launch; accum: dw += ..., db += ...
int sum_slabs_launch(const float* part_w, int64_t nw, const float* part_b, int64_t nb, int splits, float* dw,
                     float* db, bool accum, hipStream_t st) {
  if (part_b && db)
    sum_slabs2<<<static_cast<unsigned>(slab_blocks(part_w, nw, splits) + slab_blocks(part_b, nb, splits)), 256, 0, st>>>(
        part_w, nw, part_b, nb, splits, accum, dw, db);
  else
    sum_slabs<<<static_cast<unsigned>(slab_blocks(part_w, nw, splits)), 256, 0, st>>>(part_w, nw, splits, accum, dw);
  return last_launch_status();
}

// Row splits: as many workgroups as the slab budget allows (a 128x128 output: 160 x 64 KB; lin_sbf's
// 128x42: 512+, so the 194k-row reduction fills the chip), rows per split a multiple of the
// 32-row chunk and at least 64.
inline int max_splits(int O, int I) {
  const int64_t per = (static_cast<int64_t>(O) * I + O) * static_cast<int64_t>(sizeof(float));
  int64_t m = kWgSlabBudget / per;
  m = m < kWgMinSplits ? kWgMinSplits : m;
  return static_cast<int>(m > kWgMaxSplits ? kWgMaxSplits : m);
}
inline int64_t wgrad_rows_per_split(int64_t R, int O, int I) {
  const int ms = max_splits(O, I);
  int64_t rps = (R + ms - 1) / ms;
  rps = (rps + kWgChunk - 1) / kWgChunk * kWgChunk;
  return rps < 64 ? 64 : rps;
}
inline int wgrad_splits(int64_t R, int O, int I) {
  const int64_t rps = wgrad_rows_per_split(R, O, I);
  return static_cast<int>((R + rps - 1) / rps);
}

}  // namespace x2g

using namespace x2g;

X2G_API size_t x2g_linear_wgrad_workspace(int64_t R, int32_t O, int32_t I) {
  if (R <= 0 || O <= 0 || I <= 0) return 0;
  const int64_t s = wgrad_splits(R, O, I);
  return static_cast<size_t>(s) * (static_cast<int64_t>(O) * I + O) * sizeof(float);
}

X2G_API int x2g_linear_wgrad_ex(const float* dy, const float* x, int64_t R, int32_t O, int32_t I, float* dw,
                                float* db, int flags, void* workspace, size_t workspace_bytes, void* stream) {
  if (R < 0 || O <= 0 || I <= 0 || !dw || (flags & ~(X2G_ACCUM_WGRAD | X2G_DEFER_SLAB_SUM))) return X2G_EINVAL;
  const bool accum = flags & X2G_ACCUM_WGRAD;
  if ((flags & X2G_DEFER_SLAB_SUM) && R == 0) return X2G_EINVAL;  // nothing to defer: caller's bug
  hipStream_t st = as_stream(stream);
  if (R == 0) {
    if (accum) return X2G_OK;
    hipError_t e = hipMemsetAsync(dw, 0, sizeof(float) * O * I, st);
    if (e == hipSuccess && db) e = hipMemsetAsync(db, 0, sizeof(float) * O, st);
    return e == hipSuccess ? X2G_OK : static_cast<int>(e);
  }
  if (!dy || !x) return X2G_EINVAL;
  if (!workspace || workspace_bytes < x2g_linear_wgrad_workspace(R, O, I)) return X2G_EWORKSPACE;
  const int splits = wgrad_splits(R, O, I);
  float* part = static_cast<float*>(workspace);
  float* part_b = db ? part + static_cast<int64_t>(splits) * O * I : nullptr;
  const int tiles_o = (O + kWgTile - 1) / kWgTile, tiles_i = (I + kWgTile - 1) / kWgTile;
  dim3 grid(tiles_o * tiles_i, splits);
  auto mode = [](int cols, const float* p) {
    if (reinterpret_cast<uintptr_t>(p) % 16 != 0) return static_cast<int>(kScalar);
    if (cols % 4 == 0) return static_cast<int>(kVec);
    return cols <= kWgTile ? static_cast<int>(kFlat) : static_cast<int>(kScalar);
  };
  const int ma = mode(O, dy), mb = mode(I, x);
  const int64_t rps = wgrad_rows_per_split(R, O, I);
#define X2G_WGRAD(A, B) wgrad_partial<A, B><<<grid, 256, 0, st>>>(dy, x, R, O, I, tiles_i, rps, part, part_b)
  if (ma == kVec && mb == kVec) X2G_WGRAD(kVec, kVec);
  else if (ma == kVec && mb == kFlat) X2G_WGRAD(kVec, kFlat);
  else if (ma == kFlat && mb == kVec) X2G_WGRAD(kFlat, kVec);
  else if (ma == kFlat && mb == kFlat) X2G_WGRAD(kFlat, kFlat);
  else X2G_WGRAD(kScalar, kScalar);
#undef X2G_WGRAD
  int rc = last_launch_status();
  if (rc) return rc;
  if (flags & X2G_DEFER_SLAB_SUM) return X2G_OK;
  return sum_slabs_launch(part, static_cast<int64_t>(O) * I, part_b, O, splits, dw, db, accum, st);
}

X2G_API int32_t x2g_linear_wgrad_splits(int64_t R, int32_t O, int32_t I) {
  return (R > 0 && O > 0 && I > 0) ? wgrad_splits(R, O, I) : 0;
}

// ------------------------------------------------------------------------------ batched slab sums
constexpr int kBatchJobs = 60;  // jobs per launch (kernel arguments: 60 B per job, < 4 KB): a training
                                // step's ~90 deferred reductions in two launches

struct SlabBatch {
  const float* part[2 * kBatchJobs];  // job j: entry 2j = weight slabs, 2j+1 = bias slabs
  float* out[2 * kBatchJobs];
  int32_t n[2 * kBatchJobs];
  int splits[kBatchJobs];
  int block_end[2 * kBatchJobs];  // exclusive prefix of the entries' blocks (slab_blocks)
  int ld[kBatchJobs];             // weight entries: strided destination (x2g_slab_job.ld / cols)
  int cols[kBatchJobs];
  int nent;
  int accum;
};

__global__ void __launch_bounds__(256) sum_slabs_batch(const SlabBatch b) {
  __shared__ float4 red[4][64];
  // the entry owning this block: first ent with block_end[ent] > blockIdx.x (binary search over the
  // kernel-argument table, block-uniform)
  int lo = 0, hi = b.nent - 1;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (static_cast<int>(blockIdx.x) >= b.block_end[mid]) lo = mid + 1;
    else hi = mid;
  }
  const int ent = lo;
  const int first = ent ? b.block_end[ent - 1] : 0;
  const bool wgt = (ent & 1) == 0;
  sum_slabs_any(b.part[ent], b.n[ent], b.splits[ent >> 1], blockIdx.x - first, b.accum != 0, b.out[ent], red,
                wgt ? b.ld[ent >> 1] : 0, wgt ? b.cols[ent >> 1] : 0);
}

X2G_API int x2g_slab_sum_batch(const x2g_slab_job* jobs, int32_t njobs, int32_t accum, void* stream) {
  if (njobs < 0 || (njobs > 0 && !jobs)) return X2G_EINVAL;
  hipStream_t st = as_stream(stream);
  for (int j0 = 0; j0 < njobs; j0 += kBatchJobs) {
    SlabBatch b{};
    b.accum = accum;
    int blocks = 0;
    for (int j = j0; j < njobs && j < j0 + kBatchJobs; ++j) {
      const x2g_slab_job& jb = jobs[j];
      if (!jb.part_w || !jb.dw || jb.n_w <= 0 || jb.splits <= 0 || (jb.part_b && !jb.db)) return X2G_EINVAL;
      if (jb.n_w >= (int64_t(1) << 31)) return X2G_EUNSUPPORTED;
      if (jb.ld < 0 || (jb.ld > 0 && (jb.n_w % 128 || jb.cols < 0 || jb.cols > 128 || jb.cols > jb.ld)))
        return X2G_EINVAL;
      const int k = j - j0;
      b.splits[k] = jb.splits;
      b.ld[k] = jb.ld;
      b.cols[k] = jb.cols;
      const int e0 = 2 * k, e1 = 2 * k + 1;
      b.part[e0] = jb.part_w;
      b.out[e0] = jb.dw;
      b.n[e0] = static_cast<int32_t>(jb.n_w);
      blocks += static_cast<int>(slab_blocks(jb.part_w, jb.n_w, jb.splits));
      b.block_end[e0] = blocks;
      b.part[e1] = jb.part_b;
      b.out[e1] = jb.db;
      b.n[e1] = (jb.part_b && jb.db) ? jb.n_b : 0;
      blocks += static_cast<int>(slab_blocks(jb.part_b, b.n[e1], jb.splits));
      b.block_end[e1] = blocks;
      b.nent = e1 + 1;
    }
    if (blocks == 0) continue;
    sum_slabs_batch<<<blocks, 256, 0, st>>>(b);
    const int rc = last_launch_status();
    if (rc) return rc;
  }
  return X2G_OK;
}


