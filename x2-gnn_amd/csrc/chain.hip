// Row chains: a sequence of D x D Linear stages (bias, SiLU, residual) applied to the same rows in
// ONE kernel, every 16-row tile held in registers from the first stage to the last.
//
// X2-GNN's trunk ends each conv layer with seven such layers on the E line-node rows
// (model.py:47-50: bf_skip = ResidualLayer, SiLU(dense_bf_skip(.)) + the conv input, af_skip =
// 2 x ResidualLayer; residual_layer.py:21-27).  At QM9 batch sizes (E ~ 21k rows) one Linear is
// ~5 us of f32 MFMA work spread over the chip, so as separate launches each pays its own
// ramp (weight staging, first tile's load latency) and drain; here the chain pays them once.
//
// Row layout of a tile: lane l = (r = l & 15, g = l >> 4) of the owning wave holds row r's
// features 16b + 4g + e (b = 0..7, e = 0..3) as eight float4 x[b].  A stage computes the
// transposed product D = M X^T with v_mfma_f32_16x16x4_f32 (exact f32 FMA chains): A operand =
// rows of M from LDS, B operand = the tile itself — lane (r, g) supplies X[r][k] for the k of
// MFMA step (b, e) in its lane group g, k = 16b + 4g + e, which is its own register x[b][e] —
// and output block bp comes back as lane (r, g) holding out[r][16bp + 4g + e]: the same row
// layout, so the next stage takes it as its B operand with no data movement.
// M = W for the forward (y = x W^T), W^T for the backward (dx = dz W).
//
// M sits in LDS as 128 rows of 32 16-byte chunks, chunk c of row n at position c ^ (n & 15).
// The A-operand read of lane (n, g) is chunk 4b + g of row 16bp + n; within every ds_read_b128
// lane group the 16 chunks then fall on distinct bank quads (lanes 0-3/12-15 of group g and
// lanes 4-11 of group g+1 differ in the chunk's low bit after the XOR).  Two weight images are
// double-buffered (128 KB): the next stage's weight is loaded into registers while this stage's
// MFMAs run and written to LDS after them.
#include <math.h>

#include <type_traits>

#include "common.hpp"

namespace x2g {
namespace {

typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int kCD = 128;                // compiled width
constexpr int kCWaves = 8;              // 512 threads: two waves per SIMD, one 16-row tile each
constexpr int kCThreads = kCWaves * 64;

struct ChainFwdArgs {
  const float* x;
  const float* res;
  float* in_t;    // T-layout stage inputs for the weight gradient (or NULL)
  int64_t tf;     // floats per T-layout tensor
  int64_t R;
  int n;
  x2g_chain_stage st[X2G_CHAIN_MAX_STAGES];
};

struct ChainBwdArgs {
  const float* dy;
  const float* dy_add;
  float* dx;
  float* dres;
  float* dz_t;    // T-layout dz per stage (or NULL)
  const float* ln_y;   // the LayerNorm output the chain read (x2g_chain_fwd_ln's x_norm), or NULL
  float2* ln_gstats;   // with ln_y: per row (sum_c dx, sum_c dx * ln_y) for the LayerNorm backward
  int64_t tf;
  int64_t R;
  int n;
  x2g_chain_bwd_stage st[X2G_CHAIN_MAX_STAGES];
};

__device__ __forceinline__ f4 zero4() { return f4{0.f, 0.f, 0.f, 0.f}; }

// The epilogues use the hardware exp2 / reciprocal (v_exp_f32, v_rcp_f32: ~1 ulp each) instead
// of libm expf and IEEE division (~25 VALU instructions per element): the epilogue runs between
// barriers with no MFMA to hide behind, and the exact forms cost ~1.7 us per stage at config 2.
// sigmoid(z) = rcp(1 + 2^(-z log2 e)); z -> -inf gives 0, z -> +inf gives 1, NaN stays NaN.
__device__ __forceinline__ float sigmoid_fast(float z) {
  return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-1.4426950408889634f * z));
}
__device__ __forceinline__ float silu_fast(float z) { return z * sigmoid_fast(z); }
__device__ __forceinline__ float silu_grad_fast(float z) {
  const float s = sigmoid_fast(z);
  return s * (1.0f + z * (1.0f - s));
}

// ------------------------------------------------------------------------- rows in LDS
// A register-tile design (every wave a whole 16-row tile: at E ~ 21k rows 1317 tiles on 165 CUs,
// two per SIMD, a third of the chip idle, stores and SiLU in lock-step between barriers; round 1)
// was replaced by this one: each workgroup (one per CU,
// 8 waves) a contiguous range of <= 96 rows (E / 256 ~ 82 rows at config 2: every CU busy, at most
// 6 16-row blocks each) held in LDS as a swizzled [96][128] image, and each wave a 16-feature
// slice of every stage's output: wave w computes out[:, 16w .. 16w+15] for all of the range's row
// blocks, with its slice of the weight in registers (buffer loads from L2, the next stage's while
// this one runs; no LDS weight image).  MFMA v_mfma_f32_16x16x4_f32 with A = the weight slice,
// B = image rows (ds_read_b128, conflict-free with the chunk swizzle c ^ (row & 15)), so lane
// (r, g) of wave w ends with out[row 16rb + r][16w + 4g + e] — written to the other image (the
// next stage's input) and, for z, straight to global memory; y leaves coalesced, 512-byte rows
// at a time, from the LDS image after the stage's barrier.  A third image holds the external
// residual rows.  Backward likewise with the weight slice read transposed (dx = dz W) and dz
// formed in LDS before the product.
constexpr int kV2RB = 6;                 // row blocks (16 rows) per workgroup chunk

__device__ __forceinline__ int ipos(int r, int c) { return r * 32 + (c ^ (r & 15)); }

typedef __amdgpu_buffer_rsrc_t rsrc_t;

// buffer descriptor of a wave-uniform base pointer (32-bit per-lane offsets, immediate offsets
// folded: fewer address registers than 64-bit flat addresses)
__device__ __forceinline__ rsrc_t rsrc(const float* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), static_cast<short>(0), 0x7fffffff, 0x00020000);
}

__device__ __forceinline__ f4 bload4(rsrc_t r, int voff_bytes, int soff_bytes) {
  return __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(r, voff_bytes, soff_bytes, 0));
}

__device__ __forceinline__ float bload1(rsrc_t r, int voff_bytes, int soff_bytes) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, voff_bytes, soff_bytes, 0));
}

// rows [r0, r0 + nrows) of a row-major [R, 128] tensor (+ a second one) -> image (rows >= nrows zero);
// RB row blocks of 16 rows (the image's height)
template <int RB = kV2RB>
__device__ __forceinline__ void stage_rows(f4* __restrict__ img, const float* __restrict__ P,
                                           const float* __restrict__ P2, int r0, int nrows) {
  const int tid = threadIdx.x;
  f4 v[RB];
#pragma unroll
  for (int u = 0; u < RB; ++u) {
    const int q = tid + kCThreads * u, r = q >> 5, c = q & 31;
    const bool ok = r < nrows;
    const int rr = r0 + (ok ? r : 0);
    v[u] = *reinterpret_cast<const f4*>(P + rr * kCD + 4 * c) * (ok ? 1.0f : 0.0f);
    if (P2) v[u] += *reinterpret_cast<const f4*>(P2 + rr * kCD + 4 * c) * (ok ? 1.0f : 0.0f);
  }
#pragma unroll
  for (int u = 0; u < RB; ++u) {
    const int q = tid + kCThreads * u;
    img[ipos(q >> 5, q & 31)] = v[u];
  }
}

// image rows < nrows -> global rows [r0, r0 + nrows), full 512-byte rows per half-wave
template <int RB = kV2RB>
__device__ __forceinline__ void store_img(float* __restrict__ P, const f4* __restrict__ img, int r0, int nrows) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int u = 0; u < RB; ++u) {
    const int q = tid + kCThreads * u, r = q >> 5, c = q & 31;
    if (r < nrows) *reinterpret_cast<f4*>(P + (r0 + r) * kCD + 4 * c) = img[ipos(r, c)];
  }
}

// rows [r0, r0 + RB * 16) of a row-major [R, 128] tensor -> image, through buffer_load ... lds (no
// registers; the copies stay in flight while the caller computes): wave w's instruction u lands
// 1 KB (64 lanes x 16 B) at image chunks 64 (8 u + w) + lane, the swizzle applied to the
// SOURCE offset (chunk position p = 32 r + cs holds chunk cs ^ (r & 15) of row r).  One 32-bit lane
// offset; instruction u's row step (16 rows: the swizzle repeats) rides in the scalar offset.  Rows past the range are
// whatever the tensor holds there (the next range's rows: callers mask those rows' results), rows
// past R read as zero (buffer range check).  The caller waits (s_waitcnt vmcnt) and barriers
// before reading the image.
template <int RB>
__device__ __forceinline__ void stage_rows_async(f4* __restrict__ img, const float* __restrict__ P, int64_t R,
                                                 int r0, bool on = true) {
  static_assert(kCWaves == 8, "the swizzle repeats every 16 rows = one instruction's step");
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  // !on: an empty descriptor (the copies are issued but fetch nothing and land zeros), which keeps
  // the caller's instruction stream, and so its vmcnt arithmetic, branch-free
  const rsrc_t pr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(P), static_cast<short>(0),
                                                      on ? static_cast<int>(R * kCD * 4) : 0, 0x00020000);
  const int r = (64 * w + lane) >> 5, c = (lane & 31) ^ (r & 15);
  const int vo = 4 * ((r0 + r) * kCD + 4 * c);
#pragma unroll
  for (int u = 0; u < RB; ++u)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(pr, (__attribute__((address_space(3))) void*)(img + 64 * (8 * u + w)), 16,
                                             vo, u * 16 * kCD * 4, 0, 0);
}

// 4 x 4 transpose inside each lane quad (lanes 4m..4m+3 of a 16-lane row group, DPP quad
// permutes, no LDS): lane 4m + j holding (row 4m + j, features 0..3) ends with (feature j, rows
// 4m..4m+3) — a 16-byte run of the tiled-transposed layout.
__device__ __forceinline__ float dpp_xor1(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));
}
__device__ __forceinline__ float dpp_xor2(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false));
}

// sum over the 16 lanes of each row (lanes 16k .. 16k + 15), in every lane of the row: DPP quad
// swaps, then row_half_mirror (lane i <-> 7 - i) and row_mirror (i <-> 15 - i); no LDS round trips
template <int CTL>
__device__ __forceinline__ float dpp_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTL, 0xF, 0xF, false));
}
__device__ __forceinline__ float row_sum16(float v) {
  v += dpp_f<0xB1>(v);   // quad_perm [1, 0, 3, 2]
  v += dpp_f<0x4E>(v);   // quad_perm [2, 3, 0, 1]
  v += dpp_f<0x141>(v);  // row_half_mirror
  v += dpp_f<0x140>(v);  // row_mirror
  return v;
}
__device__ __forceinline__ f4 quad_transpose(f4 v, int j) {
  f4 b, c;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float t = dpp_xor1(v[k ^ 1]);
    b[k] = ((k ^ j) & 1) ? t : v[k];
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float t = dpp_xor2(b[k ^ 2]);
    c[k] = ((k ^ j) & 2) ? t : b[k];
  }
  return c;
}

// The wave's row-layout slice v[rb] (lane (rl, g): rows 16rb + rl, features 16w + 4g + e) -> the
// T layout (tile t of the chunk at dst + (r0/16 + t) * 2048, element (r, f) at f * 16 + r % 16),
// rows >= nrows written as zero; a wave's store is 1 KB contiguous (16 features x 16 rows).
template <int RB>
__device__ __forceinline__ void store_t_slice(float* __restrict__ dst, const f4 (&v)[RB], int r0, int nrows, int w,
                                              int rl, int g) {
  const int j = rl & 3, m = rl >> 2, f = 16 * w + 4 * g + j;
  const int ntile = (nrows + 15) >> 4;
  // buffer stores: one 32-bit lane offset, the tile step in the scalar offset (T tensors < 2^31 B);
  // tiles past the range (and every tile when dst is NULL: an empty descriptor) are dropped by the
  // buffer unit, so the sequence has no branches
  const rsrc_t dr = __builtin_amdgcn_make_buffer_rsrc(dst, static_cast<short>(0), dst ? 0x7fffffff : 0, 0x00020000);
  const int vo = 4 * ((r0 >> 4) * (16 * kCD) + f * 16 + 4 * m);
#pragma unroll
  for (int rb = 0; rb < RB; ++rb) {
    f4 t = quad_transpose(v[rb], j);
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (16 * rb + 4 * m + e >= nrows) t[e] = 0.0f;
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, t), dr,
                                           rb < ntile ? vo + rb * 4 * 16 * kCD : static_cast<int>(0x80000000u), 0, 0);
  }
}

// the wave's weight slice as MFMA A operands: fwd A[b][e] = W[16w + rl][16b + 4g + e];
// transposed (dx = dz W) A[b][e] = W[16b + 4g + e][16w + rl]
template <bool TRANS>
__device__ __forceinline__ void load_slice(const float* W, int w, int rl, int g, f4 (&A)[8]) {
  const rsrc_t r = rsrc(W);
  if (!TRANS) {
    const int vo = 4 * ((16 * w + rl) * kCD + 4 * g);
#pragma unroll
    for (int b = 0; b < 8; ++b) A[b] = bload4(r, vo, 64 * b);
  } else {
    const int vo = 4 * (4 * g * kCD + 16 * w + rl);
#pragma unroll
    for (int b = 0; b < 8; ++b)
#pragma unroll
      for (int e = 0; e < 4; ++e) A[b][e] = bload1(r, vo, 4 * (16 * b + e) * kCD);
  }
}

// acc[rb] (+)= the wave's 16 output features of row block rb: sum over k of A (weight slice) and
// the image rows (ZERO: acc starts at zero, else the chain continues from acc); the image chunks of step group b + 1 are read before group b's MFMAs
template <int RB, bool ZERO = true>
__device__ __forceinline__ void slice_gemm(const f4* __restrict__ img, const f4 (&A)[8], f4 (&acc)[RB], int rl,
                                           int g) {
  if (ZERO) {
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) acc[rb] = zero4();
  }
  f4 bo[2][RB];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb) bo[0][rb] = img[(16 * rb + rl) * 32 + (g ^ rl)];
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    const int cur = b & 1;
    if (b + 1 < 8) {
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) bo[cur ^ 1][rb] = img[(16 * rb + rl) * 32 + ((4 * (b + 1) + g) ^ rl)];
    }
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int rb = 0; rb < RB; ++rb)
        acc[rb] = __builtin_amdgcn_mfma_f32_16x16x4f32(A[b][e], bo[cur][rb][e], acc[rb], 0, 0, 0);
  }
}

// Pin prefetched registers: the compiler otherwise sinks the next stage's weight-slice (and z)
// loads across the stage loop's back edge to their first use, i.e. to the start of the next
// stage, where their L2 latency is exposed before the first MFMA.  An empty asm that "modifies"
// the registers at the END of this stage keeps the loads issued here, ahead of this stage's
// product, and retires them by then.
template <int N>
__device__ __forceinline__ void pin(f4 (&v)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) asm volatile("" : "+v"(v[i]));
}

// chunk ch of nch: row blocks [ch * nblk / nch, (ch + 1) * nblk / nch)
__device__ __forceinline__ void chunk_rows(int64_t ch, int64_t nch, int64_t nblk, int64_t R, int& r0, int& nrows) {
  const int64_t b0 = ch * nblk / nch, b1 = (ch + 1) * nblk / nch;
  const int64_t e = b1 * 16 < R ? b1 * 16 : R;
  r0 = static_cast<int>(b0 * 16);
  nrows = static_cast<int>(e - b0 * 16);
}

// ---- forward building blocks (the v3 design, kept as v4's parts): a branch-free epilogue
// interleaved with the MFMAs.  The 6 row blocks are computed in thirds; third t's product is
// scheduled together with third t-1's epilogue (SiLU, residual, LDS write, z and T-layout stores)
// through sched_group_barrier, so the transcendental / store work runs in the MFMA shadow instead
// of after the whole product with both waves of the SIMD idle on the matrix pipe (7-stage forward
// 73 -> 69 us at config 2, scripts/chain_bench.py).  Conditional stores become buffer stores at an
// out-of-range offset (dropped by the buffer unit, as composable_kernel's OOB-offset stores).
// a store at byte offset kOOB is out of range of every descriptor below (num_records <= 2^31 - 1)
// and dropped by the buffer unit
constexpr int kOOB = static_cast<int>(0x80000000u);


// descriptor over `bytes` bytes at p (0 when off: every store dropped)
__device__ __forceinline__ rsrc_t rsrc_n(const float* p, int64_t bytes, bool on) {
  const int64_t nr = on ? (bytes < 0x7fffffff ? bytes : 0x7fffffff) : 0;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), static_cast<short>(0), static_cast<int>(nr),
                                           0x00020000);
}
__device__ __forceinline__ void bstore4(rsrc_t r, f4 v, int voff_bytes) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, v), r,
                                         voff_bytes, 0, 0);
}

template <int RB0, int RB1, int N>
__device__ __forceinline__ void half_gemm(const f4* __restrict__ img, const f4 (&A)[8], f4 (&acc)[N], int rl,
                                          int g) {
#pragma unroll
  for (int rb = RB0; rb < RB1; ++rb) acc[rb] = zero4();
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    f4 bo[RB1 - RB0];
#pragma unroll
    for (int rb = RB0; rb < RB1; ++rb) bo[rb - RB0] = img[(16 * rb + rl) * 32 + ((4 * b + g) ^ rl)];
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int rb = RB0; rb < RB1; ++rb)
        acc[rb] = __builtin_amdgcn_mfma_f32_16x16x4f32(A[b][e], bo[rb - RB0][e], acc[rb], 0, 0, 0);
  }
}

// epilogue of blocks [RB0, RB1): z = acc + bias (stored), y = act(z) (+ residual) -> out image and
// the T-layout copy; acc[rb] := y
template <int RB0, int RB1, int N, bool TC = true>
__device__ __forceinline__ void half_epi(f4 (&acc)[N], const f4 (&held)[N], f4 bias, float silu_m, float res_m,
                                         rsrc_t zr, rsrc_t tr, f4* __restrict__ out, int r0, int nrows, int w,
                                         int rl, int g) {
  const int j = rl & 3, m = rl >> 2, f = 16 * w + 4 * g + j;
  const int ntile = (nrows + 15) >> 4;
#pragma unroll
  for (int rb = RB0; rb < RB1; ++rb) {
    const int r = 16 * rb + rl;
    const f4 z = acc[rb] + bias;
    if constexpr (TC) bstore4(zr, z, r < nrows ? 4 * ((r0 + r) * kCD + 16 * w + 4 * g) : kOOB);
    f4 y;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float sv = silu_fast(z[e]);
      y[e] = silu_m * sv + (1.0f - silu_m) * z[e] + res_m * held[rb][e];
    }
    out[ipos(r, 4 * w + g)] = y;
    acc[rb] = y;
    if constexpr (TC) {  // (inference: no weight gradient, no T-layout copy — not even dropped stores)
      f4 t = quad_transpose(y, j);
#pragma unroll
      for (int e = 0; e < 4; ++e) t[e] = 16 * rb + 4 * m + e < nrows ? t[e] : 0.0f;
      bstore4(tr, t, rb < ntile ? 4 * static_cast<int>((static_cast<int64_t>(r0 >> 4) + rb) * (16 * kCD) + f * 16 + 4 * m)
                                : kOOB);
    }
  }
}

// scheduling pattern for one two-block product (8 k-groups x (2 LDS reads + 8 MFMAs)) with an
// epilogue's instructions threaded between the MFMAs
template <int BPT = 2>  // blocks per third
__device__ __forceinline__ void interleave_epi_sched() {
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    __builtin_amdgcn_sched_group_barrier(0x100, BPT, 0);  // DS read
#pragma unroll
    for (int k = 0; k < 4 * BPT; ++k) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
      __builtin_amdgcn_sched_group_barrier(0x006, 3, 0);  // VALU / SALU
      __builtin_amdgcn_sched_group_barrier(0x400, 1, 0);  // transcendental
      __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);  // DS write
      __builtin_amdgcn_sched_group_barrier(0x040, 1, 0);  // VMEM write
    }
  }
}

// ---- forward v4 (the shipped kernel): the v3 design with the product's LDS reads
// software-pipelined.  PMC on v3 (SQ_VALU_MFMA_BUSY_CYCLES: the matrix pipe busy 46 % of the kernel
// at 2.3 GHz) and its ISA showed
// each k-group's two B fragments read right before that group's 8 MFMAs, so every group waited out
// the LDS latency, and the two waves of a SIMD, in lockstep, waited together.  Here group g + 1's
// fragments (across third boundaries too) are read before group g's MFMAs; the two stage images
// are separate __shared__ arrays (stages unrolled by two) so the compiler knows the epilogue's
// image writes never alias the product's reads and may interleave them freely.  A/B (bitwise
// equal outputs, scripts/chain_ab.py): 66.5 -> 64.3 us alone, +0.3 % molecules/s in the step.
// (The same change to the backward measured 73.7 -> 72.6 us alone but -0.2 % in the step, and a
// forward with two 256-thread workgroups per CU, so that one workgroup's stage tail overlaps the
// other's product, measured the same as v4 alone: neither is kept.)
template <int T, int BPT = 2>
__device__ __forceinline__ void frag_load(const f4* __restrict__ img, int b, int rl, int g, f4 (&bo)[BPT]) {
#pragma unroll
  for (int j = 0; j < BPT; ++j) bo[j] = img[(16 * (BPT * T + j) + rl) * 32 + ((4 * b + g) ^ rl)];
}

// third T's product (blocks 2T, 2T + 1); on entry bo[0] holds its group 0, on exit (T < 2) bo[0]
// holds third T + 1's group 0
template <int T, int BPT, int N>
__device__ __forceinline__ void third_gemm(const f4* __restrict__ img, const f4 (&A)[8], f4 (&acc)[N],
                                           f4 (&bo)[2][BPT], int rl, int g) {
#pragma unroll
  for (int j = 0; j < BPT; ++j) acc[BPT * T + j] = zero4();
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    const int cur = b & 1;
    if (b + 1 < 8)
      frag_load<T, BPT>(img, b + 1, rl, g, bo[cur ^ 1]);
    else if (T < 2)
      frag_load<(T < 2 ? T + 1 : T), BPT>(img, 0, rl, g, bo[cur ^ 1]);
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int j = 0; j < BPT; ++j)
        acc[BPT * T + j] = __builtin_amdgcn_mfma_f32_16x16x4f32(A[b][e], bo[cur][j][e], acc[BPT * T + j], 0, 0, 0);
  }
}

// a third's product alone: per group its 2 (next-group) LDS reads, then 8 MFMAs
template <int BPT = 2>
__device__ __forceinline__ void pipe_sched() {
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    __builtin_amdgcn_sched_group_barrier(0x100, BPT, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, 4 * BPT, 0);
  }
}

// one stage of the v4 forward: in -> out (distinct arrays after inlining); RB row blocks per chunk (6,
// or 3 for the small-row batched chains), computed in thirds of RB / 3 blocks
template <int RB, bool TC = true>
__device__ __forceinline__ void fwd4_stage(const ChainFwdArgs& a, int s, const f4* __restrict__ in,
                                           f4* __restrict__ out, const f4* __restrict__ rimg, f4 (&A)[8],
                                           f4 (&held)[RB], int r0, int nrows,
                                           int w, int rl, int g) {
  constexpr int BPT = RB / 3;
  const int n = a.n;
  const x2g_chain_stage& S = a.st[s];
  const int fl = S.flags;
  f4 An[8];
  load_slice<false>(a.st[s + 1 < n ? s + 1 : 0].w, w, rl, g, An);
  const f4 bias = bload4(rsrc(S.b ? S.b : S.w), 4 * (16 * w + 4 * g), 0) * (S.b ? 1.0f : 0.0f);
  if (fl & (X2G_CHAIN_HOLD | X2G_CHAIN_RES_EXT)) {
    const f4* src = (fl & X2G_CHAIN_HOLD) ? in : rimg;
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) held[rb] = src[ipos(16 * rb + rl, 4 * w + g)];
  }
  const float silu_m = (fl & X2G_CHAIN_SILU) ? 1.0f : 0.0f;
  const float res_m = (fl & (X2G_CHAIN_RES_HELD | X2G_CHAIN_RES_EXT)) ? 1.0f : 0.0f;
  const rsrc_t zr = rsrc_n(S.z ? S.z : S.w, a.R * kCD * 4, S.z != nullptr);
  const bool t_on = a.in_t && s + 1 < n;
  const rsrc_t tr = rsrc_n(t_on ? a.in_t + (s + 1) * a.tf : S.w, a.tf * 4, t_on);
  f4 acc[RB];
  f4 bo[2][BPT];
  frag_load<0, BPT>(in, 0, rl, g, bo[0]);
  __builtin_amdgcn_sched_barrier(0);  // the region below: third 0's MFMAs and its next-group reads only
  third_gemm<0, BPT>(in, A, acc, bo, rl, g);
  pipe_sched<BPT>();
  __builtin_amdgcn_sched_barrier(0);
  third_gemm<1, BPT>(in, A, acc, bo, rl, g);
  half_epi<0, BPT, RB, TC>(acc, held, bias, silu_m, res_m, zr, tr, out, r0, nrows, w, rl, g);
  interleave_epi_sched<BPT>();
  __builtin_amdgcn_sched_barrier(0);
  third_gemm<2, BPT>(in, A, acc, bo, rl, g);
  half_epi<BPT, 2 * BPT, RB, TC>(acc, held, bias, silu_m, res_m, zr, tr, out, r0, nrows, w, rl, g);
  interleave_epi_sched<BPT>();
  __builtin_amdgcn_sched_barrier(0);
  half_epi<2 * BPT, 3 * BPT, RB, TC>(acc, held, bias, silu_m, res_m, zr, tr, out, r0, nrows, w, rl, g);
  pin(An);
  __syncthreads();
  if (S.y) store_img<RB>(S.y, out, r0, nrows);
#pragma unroll
  for (int b = 0; b < 8; ++b) A[b] = An[b];
}

// Graph LayerNorm (model.py:46, PyG LayerNorm(mode='graph'): per molecule, mean and biased
// variance over all its rows and features, out = (x - mean) / sqrt(var + eps)) applied while the
// chain's first input is staged, from per-row statistics the producing kernel left
// (x2g_sbf_attention_fwd_stats: (mean_r, M2_r) per row): the molecule's statistics are the exact
// Chan combination mean = sum_r mean_r / n, M2 = sum_r (M2_r + D (mean_r - mean)^2), so the
// LayerNorm needs no pass of its own over the rows.
struct ChainLn {
  const float2* stats;   // [R] (mean_r, M2_r) or NULL: no LayerNorm
  const int32_t* ptr;    // [G + 1] rows per molecule (CSR)
  float* out;            // [R, D] the normalised rows (the LayerNorm backward's input), or NULL
  float* mean;           // [G] or NULL
  float* rstd;           // [G] or NULL
  int64_t G;
  float eps;
};

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// stage_rows for the chain's first input with the graph LayerNorm applied; lnrow: LDS scratch of
// RB * 16 (mean, denominator) pairs.  The x rows go to LDS by buffer_load ... lds first (no
// registers held across the rest), so their latency hides under the statistics; each wave
// combines the statistics of every 8th molecule that has rows in the chunk (every workgroup that
// holds rows of a molecule computes the same values, in the same order); the workgroup holding a
// molecule's first row writes its mean / rstd; then every image element is normalised in place.
// A molecule of more than kLongMol rows (AID's ~2,000-row molecules) is combined by the whole workgroup
// instead, each thread summing every 512th row: a chunk inside such a molecule then takes two short
// passes, not one wave's serial walk over the molecule twice (config 5: 533 -> ~400 us per chain launch,
// the other 7 waves had waited at the staging barrier; +6.5 % molecules/s).  Up to kLongMol rows the
// one-wave form (at most 4 loop trips past its register window; S5A's ~300-row molecules: one) stays.
// red: 2 x 8 floats of LDS.
constexpr int kLongMol = 512;
template <int RB = kV2RB>
__device__ __forceinline__ void stage_rows_ln(f4* __restrict__ img, const float* __restrict__ P, int64_t R,
                                              const ChainLn& ln, float2* __restrict__ lnrow,
                                              float* __restrict__ red, int r0, int nrows) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  stage_rows_async<RB>(img, P, R, r0);
  // the segment row pointers ptr[k], k = lane + 64 j < 256, in registers (one round of independent
  // loads); the first molecule with rows here is (#k with ptr[k] <= r0) - 1
  constexpr int kPW = 4;
  int pk[kPW];
#pragma unroll
  for (int j = 0; j < kPW; ++j) {
    const int64_t k = lane + 64 * j;
    pk[j] = ln.ptr[k <= ln.G ? k : ln.G];
  }
  float cnt = 0.f;
#pragma unroll
  for (int j = 0; j < kPW; ++j) cnt += (lane + 64 * j <= ln.G && pk[j] <= r0) ? 1.f : 0.f;
  for (int64_t k = lane + 64 * kPW; k <= ln.G; k += 64) cnt += ln.ptr[k] <= r0 ? 1.f : 0.f;  // G >= 256
  const int64_t m0 = static_cast<int64_t>(wave64_sum(cnt)) - 1;
  auto ptr_at = [&](int64_t k) -> int {  // wave-uniform k
    if (k >= 64 * kPW) return uniform(ln.ptr[k]);
    const int l = static_cast<int>(k & 63);
    switch (k >> 6) {
      case 0: return lane_bcast(pk[0], l);
      case 1: return lane_bcast(pk[1], l);
      case 2: return lane_bcast(pk[2], l);
      default: return lane_bcast(pk[3], l);
    }
  };
  constexpr int kSW = 4;  // molecules of up to 256 rows: their statistics stay in registers
  // the long molecules with rows here (workgroup-uniform loop; none at QM9 sizes)
  for (int64_t m = m0 > 0 ? m0 : 0; m < ln.G; ++m) {
    const int p0 = ptr_at(m), p1 = ptr_at(m + 1);
    if (p0 >= r0 + nrows) break;
    if (p1 - p0 <= kLongMol) continue;
    const float n = static_cast<float>(p1 - p0);
    constexpr int kU = 4;  // loads in flight per thread and pass
    float s = 0.f;
    for (int base = p0 + tid; base < p1; base += kU * kCThreads) {
      float v[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int r = base + u * kCThreads;
        v[u] = r < p1 ? ln.stats[r].x : 0.f;
      }
#pragma unroll
      for (int u = 0; u < kU; ++u) s += v[u];
    }
    s = wave64_sum(s);
    if (lane == 0) red[w] = s;
    __syncthreads();
    float st = 0.f;
#pragma unroll
    for (int ww = 0; ww < kCWaves; ++ww) st += red[ww];
    const float mu = st / n;
    float q = 0.f;
    for (int base = p0 + tid; base < p1; base += kU * kCThreads) {
      float2 v[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int r = base + u * kCThreads;
        v[u] = r < p1 ? ln.stats[r] : make_float2(mu, 0.f);
      }
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const float d = v[u].x - mu;
        q += fmaf(static_cast<float>(kCD) * d, d, v[u].y);
      }
    }
    q = wave64_sum(q);
    if (lane == 0) red[kCWaves + w] = q;
    __syncthreads();
    float qt = 0.f;
#pragma unroll
    for (int ww = 0; ww < kCWaves; ++ww) qt += red[kCWaves + ww];
    const float denom = sqrtf(qt / (n * static_cast<float>(kCD)) + ln.eps);
    const int lo = p0 > r0 ? p0 : r0, hi = p1 < r0 + nrows ? p1 : r0 + nrows;
    for (int r = lo + tid; r < hi; r += kCThreads) lnrow[r - r0] = make_float2(mu, denom);
    if (tid == 0 && p0 >= r0) {
      if (ln.mean) ln.mean[m] = mu;
      if (ln.rstd) ln.rstd[m] = 1.0f / denom;
    }
    __syncthreads();  // red is reused by the next long molecule
  }
  for (int64_t m = (m0 > 0 ? m0 : 0) + w; m < ln.G; m += kCWaves) {
    const int p0 = ptr_at(m), p1 = ptr_at(m + 1);
    if (p0 >= r0 + nrows) break;
    if (p1 <= p0 || p1 - p0 > kLongMol) continue;
    const float n = static_cast<float>(p1 - p0);
    float2 sv[kSW];
#pragma unroll
    for (int j = 0; j < kSW; ++j) {
      const int r = p0 + lane + 64 * j;
      sv[j] = ln.stats[r < p1 ? r : p0];
    }
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < kSW; ++j) s += p0 + lane + 64 * j < p1 ? sv[j].x : 0.f;
    for (int r = p0 + lane + 64 * kSW; r < p1; r += 64) s += ln.stats[r].x;
    const float mu = wave64_sum(s) / n;
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < kSW; ++j) {
      const float d = sv[j].x - mu;
      q += p0 + lane + 64 * j < p1 ? fmaf(static_cast<float>(kCD) * d, d, sv[j].y) : 0.f;
    }
    for (int r = p0 + lane + 64 * kSW; r < p1; r += 64) {
      const float2 st = ln.stats[r];
      const float d = st.x - mu;
      q += fmaf(static_cast<float>(kCD) * d, d, st.y);
    }
    const float denom = sqrtf(wave64_sum(q) / (n * static_cast<float>(kCD)) + ln.eps);
    const int lo = p0 > r0 ? p0 : r0, hi = p1 < r0 + nrows ? p1 : r0 + nrows;
    for (int r = lo + lane; r < hi; r += 64) lnrow[r - r0] = make_float2(mu, denom);
    if (lane == 0 && p0 >= r0) {
      if (ln.mean) ln.mean[m] = mu;
      if (ln.rstd) ln.rstd[m] = 1.0f / denom;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the image copies
  __syncthreads();
#pragma unroll
  for (int u = 0; u < RB; ++u) {
    const int q = tid + kCThreads * u, r = q >> 5, c = q & 31;
    const bool ok = r < nrows;
    const float2 st = lnrow[ok ? r : 0];
    const f4 v = img[ipos(r, c)];
    f4 y;
#pragma unroll
    for (int e = 0; e < 4; ++e) y[e] = ok ? (v[e] - st.x) / st.y : 0.0f;
    img[ipos(r, c)] = y;
    if (ln.out && ok) *reinterpret_cast<f4*>(ln.out + (r0 + r) * kCD + 4 * c) = y;
  }
}

template <bool LN, int RB = kV2RB, bool TC = true>
__device__ __forceinline__ void chain_fwd_v4_run(const ChainFwdArgs& a, const ChainLn& ln) {
  static_assert(RB == 6 || RB == 3, "thirds of 2 or 1 row blocks");
  __shared__ f4 img0[RB * 16 * 32];
  __shared__ f4 img1[RB * 16 * 32];
  __shared__ f4 imgr[RB * 16 * 32];
  __shared__ float2 lnrow[LN ? RB * 16 : 1];
  __shared__ float lnred[LN ? 2 * kCWaves : 1];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int rl = lane & 15, g = lane >> 4;
  const int64_t nblk = (a.R + 15) / 16, G = gridDim.x;
  const int64_t nch = (nblk + RB * G - 1) / (RB * G) * G;
  const int n = a.n;
  // W^T of every stage for the backward (x2g_chain_stage.wt): each workgroup writes its share, one
  // element per thread (written by the first 8 chunks, it made those workgroups the launch's tail)
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kCThreads + tid; i < static_cast<int64_t>(n) * kCD * kCD;
       i += G * kCThreads) {
    const int s = static_cast<int>(i / (kCD * kCD)), e = static_cast<int>(i % (kCD * kCD));
    if (a.st[s].wt) a.st[s].wt[e] = a.st[s].w[(e % kCD) * kCD + e / kCD];
  }
  for (int64_t ch = blockIdx.x; ch < nch; ch += G) {
    int r0, nrows;
    chunk_rows(ch, nch, nblk, a.R, r0, nrows);
    __syncthreads();
    if (LN)
      stage_rows_ln<RB>(img0, a.x, a.R, ln, lnrow, lnred, r0, nrows);
    else
      stage_rows<RB>(img0, a.x, nullptr, r0, nrows);
    if (a.res) stage_rows<RB>(imgr, a.res, nullptr, r0, nrows);
    f4 A[8], held[RB];
    load_slice<false>(a.st[0].w, w, rl, g, A);
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) held[rb] = zero4();
    __syncthreads();
    if (a.in_t) {
      f4 xs[RB];
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) xs[rb] = img0[ipos(16 * rb + rl, 4 * w + g)];
      store_t_slice(a.in_t, xs, r0, nrows, w, rl, g);
    }
    for (int s = 0; s < n; s += 2) {
      fwd4_stage<RB, TC>(a, s, img0, img1, imgr, A, held, r0, nrows, w, rl, g);
      if (s + 1 < n) fwd4_stage<RB, TC>(a, s + 1, img1, img0, imgr, A, held, r0, nrows, w, rl, g);
    }
  }
}

__global__ void __launch_bounds__(kCThreads, 1) chain_fwd_v4(const ChainFwdArgs a) { chain_fwd_v4_run<false>(a, {}); }

// the chain with the graph LayerNorm of its input fused into the staging (x2g_chain_fwd_ln)
struct ChainFwdLnArgs {
  ChainFwdArgs a;
  ChainLn ln;
};
__global__ void __launch_bounds__(kCThreads, 1) chain_fwd_v4_ln(const ChainFwdLnArgs b) {
  chain_fwd_v4_run<true>(b.a, b.ln);
}
// the same without the backward's T-layout copies and pre-activation stores (inference: in_t and every
// stage's z NULL)
__global__ void __launch_bounds__(kCThreads, 1) chain_fwd_v4_ln_infer(const ChainFwdLnArgs b) {
  chain_fwd_v4_run<true, kV2RB, false>(b.a, b.ln);
}

// several independent chains over the same row count in one launch (job = blockIdx.y): the
// readouts' MLPs, whose 2304 atom rows alone would fill a tenth of the chip
constexpr int kChainMaxJobs = X2G_CHAIN_MAX_JOBS;
struct ChainFwdBatch {
  ChainFwdArgs a[kChainMaxJobs];
};
// RB = 3 when one chunk of 3 row blocks per workgroup covers a job (the readouts' 2304 rows on 51
// workgroups each): the products of 6 blocks, half of them padding, would set the stage time
template <int RB>
__global__ void __launch_bounds__(kCThreads, 1) chain_fwd_v4_batch(const ChainFwdBatch b) {
  chain_fwd_v4_run<false, RB>(b.a[blockIdx.y], {});
}

// ---- backward v3 (the shipped kernel): the v2 design with stage s-1's elementwise
// part (residual gradients, dz = g SiLU'(z), the dz stores, the T-layout copy) computed per third of
// the row blocks and scheduled into the next third's MFMAs, branch-free as the forward v3.
// A stage that adds its external residual gradient into d_res_ext (X2G_CHAIN_RES_ACCUM): the read
// of the old value waits (vmcnt) for every older memory operation of the wave — the next stage's
// weight / z prefetches and all T-layout stores so far — so it is issued, behind a wave-uniform
// branch, only in the accumulating stage's elementwise part (1 of the trunk's 7; r2 issued it in
// every stage as a dropped out-of-range load and waited on it there: removing every external access
// measured +1.3 % in the step, profiles/r3d_ab_chain_noext.log, the bound for this change)
template <int RB0, int RB1, int N>
__device__ __forceinline__ void bwd_elem(f4 (&gs)[N], f4 (&dh)[N], const f4 (&zc)[N], const f4 (&acc)[N],
                                         float hold_m, float held_m, float silu_m, float dres_acc_m, rsrc_t dres_r,
                                         rsrc_t dz_r, rsrc_t t_r, f4* __restrict__ out, int r0, int nrows, int w,
                                         int rl, int g) {
  const int col = 16 * w + 4 * g;
  const int j = rl & 3, m = rl >> 2, f = 16 * w + 4 * g + j;
  const int ntile = (nrows + 15) >> 4;
#pragma unroll
  for (int rb = RB0; rb < RB1; ++rb) {
    const int r = 16 * rb + rl;
    const int off = r < nrows ? 4 * ((r0 + r) * kCD + col) : kOOB;
    const f4 gv = acc[rb] + dh[rb] * hold_m;  // in_s was also the held residual (stage s HOLD)
    dh[rb] = dh[rb] * (1.0f - hold_m) + gv * held_m;  // stage s-1 adds the held residual
    if (dres_acc_m != 0.0f) {  // wave-uniform: only the accumulating stage reads (and waits)
      bstore4(dres_r, gv + bload4(dres_r, off, 0), off);
    } else {
      bstore4(dres_r, gv, off);
    }
    f4 dz;
#pragma unroll
    for (int e = 0; e < 4; ++e) dz[e] = gv[e] * (silu_m * silu_grad_fast(zc[rb][e]) + (1.0f - silu_m));
    bstore4(dz_r, dz, off);
    out[ipos(r, 4 * w + g)] = dz;
    gs[rb] = dz;
    f4 t = quad_transpose(dz, j);
#pragma unroll
    for (int e = 0; e < 4; ++e) t[e] = 16 * rb + 4 * m + e < nrows ? t[e] : 0.0f;
    bstore4(t_r, t, rb < ntile ? 4 * static_cast<int>((static_cast<int64_t>(r0 >> 4) + rb) * (16 * kCD) + f * 16 + 4 * m)
                               : kOOB);
  }
}

// store_img of the chain's input gradient g, plus the per-row sums the graph LayerNorm backward needs
// (sum_c g, sum_c g y with y the LayerNorm output: PyG LayerNorm(mode='graph') backward,
// dx = rstd (g - mean(g) - y mean(g y)) per molecule): a row's 32 chunks sit in 32 consecutive
// lanes, reduced by xor shuffles; the molecule sums are then a pass over these [R, 2] (no second
// pass over g and y)
// yimg: the chain input's rows (x2g_chain_fwd_ln's x_norm), copied into LDS by stage_rows_async at the
// start of the last stage (landed by its barrier)
template <int RB = kV2RB>
__device__ __forceinline__ void store_img_lnstats(float* __restrict__ P, const f4* __restrict__ img,
                                                  const f4* __restrict__ yimg, float2* __restrict__ gs, int r0,
                                                  int nrows) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int u = 0; u < RB; ++u) {
    const int q = tid + kCThreads * u, r = q >> 5, c = q & 31;
    const f4 g = img[ipos(r, c)], y = yimg[ipos(r, c)];
    if (r < nrows) *reinterpret_cast<f4*>(P + (r0 + r) * kCD + 4 * c) = g;
    // a row's 32 chunks are one aligned half-wave: DPP sums, valid in its upper 16 lanes
    const float s1 = half32_sum_hi((g[0] + g[1]) + (g[2] + g[3]));
    const float s2 = half32_sum_hi(fmaf(g[0], y[0], fmaf(g[1], y[1], fmaf(g[2], y[2], g[3] * y[3]))));
    if (c == 16 && r < nrows) gs[r0 + r] = make_float2(s1, s2);
  }
}

template <int RB = kV2RB>
__device__ __forceinline__ void chain_bwd_v3_run(const ChainBwdArgs& a) {
  static_assert(RB == 6 || RB == 3, "thirds of 2 or 1 row blocks");
  constexpr int BPT = RB / 3;
  __shared__ f4 img[2][RB * 16 * 32];
  __shared__ f4 yimg[RB * 16 * 32];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int rl = lane & 15, g = lane >> 4;
  const int64_t nblk = (a.R + 15) / 16, G = gridDim.x;
  const int64_t nch = (nblk + RB * G - 1) / (RB * G) * G;
  const int n = a.n;
  const int col = 16 * w + 4 * g;
  for (int64_t ch = blockIdx.x; ch < nch; ch += G) {
    int r0, nrows;
    chunk_rows(ch, nch, nblk, a.R, r0, nrows);
    f4 A[8], dh[RB], zc[RB], gs[RB];
    auto load_z = [&](int s) {
      const rsrc_t zr = rsrc((a.st[s].flags & X2G_CHAIN_SILU) ? a.st[s].z : a.dy);
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) {
        const int r = 16 * rb + rl;
        zc[rb] = bload4(zr, 4 * ((r0 + (r < nrows ? r : 0)) * kCD + col), 0);
      }
    };
    auto load_wslice = [&](int s, f4 (&dst)[8]) {
      if (a.st[s].wt)
        load_slice<false>(a.st[s].wt, w, rl, g, dst);
      else
        load_slice<true>(a.st[s].w, w, rl, g, dst);
    };
    // the elementwise part's per-stage descriptors and masks
    auto elem_args = [&](int s, float& held_m, float& silu_m, float& dres_acc_m, rsrc_t& dres_r, rsrc_t& dz_r,
                         rsrc_t& t_r) {
      const x2g_chain_bwd_stage& S = a.st[s];
      const int fl = S.flags;
      held_m = (fl & X2G_CHAIN_RES_HELD) ? 1.0f : 0.0f;
      silu_m = (fl & X2G_CHAIN_SILU) ? 1.0f : 0.0f;
      const bool dres_on = (fl & X2G_CHAIN_RES_EXT) && a.dres;
      dres_acc_m = (fl & X2G_CHAIN_RES_ACCUM) ? 1.0f : 0.0f;
      dres_r = rsrc_n(dres_on ? a.dres : a.dy, a.R * kCD * 4, dres_on);
      dz_r = rsrc_n(S.dz ? S.dz : a.dy, a.R * kCD * 4, S.dz != nullptr);
      t_r = rsrc_n(a.dz_t ? a.dz_t + s * a.tf : a.dy, a.tf * 4, a.dz_t != nullptr);
    };
    // whether stage s's elementwise part stores anything but dz in the T layout (wave-uniform)
    // the LayerNorm backward's y rows for the final store: an LDS copy in flight with the first loads
    // (yimg is read only after the last stage's barrier; the first waits below cover it)
    if (a.ln_y) stage_rows_async<RB>(yimg, a.ln_y, a.R, r0);
    load_wslice(n - 1, A);
    load_z(n - 1);
    f4 acc0[RB];
    {
      const rsrc_t yr = rsrc(a.dy), ar = rsrc(a.dy_add ? a.dy_add : a.dy);
      const float am = a.dy_add ? 1.0f : 0.0f;
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) {
        const int r = 16 * rb + rl;
        const int vo = 4 * ((r0 + (r < nrows ? r : 0)) * kCD + col);
        acc0[rb] = bload4(yr, vo, 0) + bload4(ar, vo, 0) * am;
        dh[rb] = zero4();
      }
    }
    int p = 0;
    __syncthreads();  // the previous chunk's images are no longer read
    {
      float held_m, silu_m, dres_acc_m;
      rsrc_t dres_r, dz_r, t_r;
      elem_args(n - 1, held_m, silu_m, dres_acc_m, dres_r, dz_r, t_r);
      bwd_elem<0, RB>(gs, dh, zc, acc0, 0.0f, held_m, silu_m, dres_acc_m, dres_r, dz_r, t_r, img[p], r0, nrows,
                              w, rl, g);
    }
    __syncthreads();
    for (int s = n - 1; s >= 0; --s) {
      f4 An[8];
      load_wslice(s > 0 ? s - 1 : n - 1, An);
      load_z(s > 0 ? s - 1 : 0);
      const float hold_m = (a.st[s].flags & X2G_CHAIN_HOLD) ? 1.0f : 0.0f;
      const f4* in = img[p];
      f4* out = img[p ^ 1];
      f4 acc[RB];
      if (s > 0) {
        float held_m, silu_m, dres_acc_m;
        rsrc_t dres_r, dz_r, t_r;
        elem_args(s - 1, held_m, silu_m, dres_acc_m, dres_r, dz_r, t_r);
        {
          half_gemm<0, BPT>(in, A, acc, rl, g);
          __builtin_amdgcn_sched_barrier(0);
          half_gemm<BPT, 2 * BPT>(in, A, acc, rl, g);
          bwd_elem<0, BPT>(gs, dh, zc, acc, hold_m, held_m, silu_m, dres_acc_m, dres_r, dz_r, t_r, out, r0, nrows,
                            w, rl, g);
          interleave_epi_sched<BPT>();
          __builtin_amdgcn_sched_barrier(0);
          half_gemm<2 * BPT, 3 * BPT>(in, A, acc, rl, g);
          bwd_elem<BPT, 2 * BPT>(gs, dh, zc, acc, hold_m, held_m, silu_m, dres_acc_m, dres_r, dz_r, t_r, out, r0, nrows,
                            w, rl, g);
          interleave_epi_sched<BPT>();
          __builtin_amdgcn_sched_barrier(0);
          bwd_elem<2 * BPT, 3 * BPT>(gs, dh, zc, acc, hold_m, held_m, silu_m, dres_acc_m, dres_r, dz_r, t_r, out, r0, nrows,
                            w, rl, g);
        }
      } else {
        slice_gemm<RB>(in, A, acc, rl, g);
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) out[ipos(16 * rb + rl, 4 * w + g)] = acc[rb] + dh[rb] * hold_m;
      }
      p ^= 1;
      pin(An);
      __syncthreads();
#pragma unroll
      for (int b = 0; b < 8; ++b) A[b] = An[b];
    }
    if (a.ln_y)
      store_img_lnstats<RB>(a.dx, img[p], yimg, a.ln_gstats, r0, nrows);
    else
      store_img<RB>(a.dx, img[p], r0, nrows);
  }
}

struct ChainBwdBatch {
  ChainBwdArgs a[kChainMaxJobs];
};
template <int RB>
__global__ void __launch_bounds__(kCThreads, 1) chain_bwd_v3_batch(const ChainBwdBatch b) {
  chain_bwd_v3_run<RB>(b.a[blockIdx.y]);
}


// ------------------------------------------------------------------------- batched weight gradients
// dW_j[n][k] = sum_r dy_j[r][n] x_j[r][k] for up to 8 layers: workgroup (chunk, j) owns a fixed
// range of rows of layer j; 32-row tiles of dy and x are staged through LDS (double-buffered,
// next tile in registers during the MFMAs) and wave w accumulates dW rows 32w..32w+31 x all 128
// columns (4 x v_mfma_f32_32x32x2_f32 accumulators) over the chunk; the chunk's partial goes to
// its slab, summed later in a fixed order (x2g_slab_sum_batch).
constexpr int kWThreads = 256;
typedef float floatx16 __attribute__((ext_vector_type(16)));

struct WgradArgs {
  x2g_wgrad_job job[X2G_CHAIN_MAX_STAGES];
  float* part_w[X2G_CHAIN_MAX_STAGES];
  float* part_b[X2G_CHAIN_MAX_STAGES];
  int64_t R;
  int chunk_rows;
};

__device__ __forceinline__ int wswz(int r, int c) { return r * 128 + 4 * ((c >> 2) ^ (r & 15)) + (c & 3); }

__device__ __forceinline__ void wtile_load(const float* __restrict__ P, int64_t r0, int64_t r1, f4 (&v)[4]) {
  const int tid = threadIdx.x, q = tid & 31;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int64_t r = r0 + (tid >> 5) + 8 * u;
    const bool ok = r < r1;
    const int64_t rc = ok ? r : r0;
    v[u] = *reinterpret_cast<const f4*>(P + rc * kCD + 4 * q) * (ok ? 1.0f : 0.0f);
  }
}

__device__ __forceinline__ void wtile_store(float* __restrict__ T, const f4 (&v)[4]) {
  const int tid = threadIdx.x, q = tid & 31;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int r = (tid >> 5) + 8 * u;
    *reinterpret_cast<f4*>(T + r * 128 + 4 * (q ^ (r & 15))) = v[u];
  }
}

__global__ void __launch_bounds__(kWThreads, 2) wgrad_batched_kernel(const WgradArgs a) {
  __shared__ __attribute__((aligned(16))) float Ds[2][32 * 128];
  __shared__ __attribute__((aligned(16))) float Xs[2][32 * 128];
  const int j = blockIdx.y;
  const x2g_wgrad_job& J = a.job[j];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5, i = lane & 31;
  const int nb = 32 * wave;
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * a.chunk_rows;
  const int64_t r1 = r0 + a.chunk_rows < a.R ? r0 + a.chunk_rows : a.R;
  floatx16 acc[4];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[m][e] = 0.f;
  float bsum = 0.f;
  f4 vd[4], vx[4];
  int buf = 0;
  if (r0 < r1) {
    wtile_load(J.dy, r0, r1, vd);
    wtile_load(J.x, r0, r1, vx);
  }
  for (int64_t t = r0; t < r1; t += 32) {
    wtile_store(Ds[buf], vd);
    wtile_store(Xs[buf], vx);
    __syncthreads();
    if (t + 32 < r1) {  // the next tile's loads fly during the MFMAs
      wtile_load(J.dy, t + 32, r1, vd);
      wtile_load(J.x, t + 32, r1, vx);
    }
    const float* D = Ds[buf];
    const float* X = Xs[buf];
#pragma unroll
    for (int sg = 0; sg < 2; ++sg) {
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        const int r = 16 * sg + s + 8 * h;
        const float av = D[wswz(r, nb + i)];
#pragma unroll
        for (int m = 0; m < 4; ++m) acc[m] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, X[wswz(r, 32 * m + i)], acc[m], 0, 0, 0);
      }
    }
    if (J.db && tid < 128) {
#pragma unroll 8
      for (int rr = 0; rr < 32; ++rr) bsum += D[wswz(rr, tid)];
    }
    buf ^= 1;  // the other buffer was last read before this tile's barrier
  }
  float* slab = a.part_w[j] + static_cast<int64_t>(blockIdx.x) * kCD * kCD;
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int e = 0; e < 16; ++e) slab[(nb + (e & 3) + 8 * (e >> 2) + 4 * h) * kCD + 32 * m + i] = acc[m][e];
  if (J.db && tid < 128) a.part_b[j][static_cast<int64_t>(blockIdx.x) * kCD + tid] = bsum;
}

// ---------------------------------------------------------------- chain weight gradients (T layout)
// dW_s = dz_s^T in_s over all rows: workgroup (c, s) owns a fixed range of 16-row tiles of stage s.
// Two T tiles (32 rows) per step are copied into LDS as-is (8 KB each, double-buffered, the next
// pair in registers during the MFMAs), so both MFMA operands come as ds_read_b128 of 4 consecutive
// rows of one feature: wave w accumulates dW rows 16w..16w+15 x all 128 columns (8 blocks of
// v_mfma_f32_16x16x4_f32).  Image position of (feature f, row quad q): f * 4 + (q ^ sigma(f)),
// sigma(f) = 3 * ((f >> 3) & 1): conflict-free in every ds_read_b128 lane group.
constexpr int kWTiles = 2;  // T tiles per step

__device__ __forceinline__ int tpos(int f, int q) { return f * 4 + (q ^ (((f >> 3) & 1) * 3)); }

struct ChainWgradArgs {
  const float* in_t[X2G_CHAIN_MAX_STAGES];  // per job: the layer input and dz, T layout
  const float* dz_t[X2G_CHAIN_MAX_STAGES];
  int64_t ntiles;
  float* part_w[X2G_CHAIN_MAX_STAGES];
  float* part_b[X2G_CHAIN_MAX_STAGES];
  int has_b[X2G_CHAIN_MAX_STAGES];
  int splits;
};

// Three LDS buffers, filled by global_load_lds (no registers: each wave's instruction lands 1 KB
// lane-linearly, the swizzle applied to the source addresses), two steps in flight ahead of the
// product; raw s_barrier with counted vmcnt waits so the in-flight copies survive the barriers.
// One call reduces tiles [t0, t1) of one job into a slab (dW rows 16w + 4g + e, columns 16bk + rl).
template <int NB, bool SPREAD = true, int WT = kWTiles>  // NB LDS buffers: NB - 1 steps in flight ahead of the product;
// SPREAD: the bias column sums over all eight waves (else waves 0-1 only)
__device__ __forceinline__ void tiled_segment(const float* __restrict__ dz, const float* __restrict__ xin, int64_t t0,
                                              int64_t t1, bool has_b, float* __restrict__ slab,
                                              float* __restrict__ slab_b, f4 (*Ds)[WT][512],
                                              f4 (*Xs)[WT][512]) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int rl = lane & 15, g = lane >> 4;
  const int nsteps = static_cast<int>((t1 - t0 + WT - 1) / WT);
  // LDS position P = 64w + lane of a tile image holds source chunk (P >> 2) * 4 + ((P & 3) ^ sigma)
  const int P = 64 * w + lane;
  const int src_chunk = (P >> 2) * 4 + ((P & 3) ^ (((P >> 5) & 1) * 3));
  auto issue = [&](int step) {  // the step's tiles into buffer step % NB (tiles past t1: tile t0)
    const int b = step % NB;
#pragma unroll
    for (int k = 0; k < WT; ++k) {
      int64_t t = t0 + static_cast<int64_t>(step) * WT + k;
      t = t < t1 ? t : t0;
      __builtin_amdgcn_global_load_lds(dz + t * 2048 + 4 * src_chunk, &Ds[b][k][64 * w], 16, 0, 0);
      __builtin_amdgcn_global_load_lds(xin + t * 2048 + 4 * src_chunk, &Xs[b][k][64 * w], 16, 0, 0);
    }
  };
  f4 acc[8];
#pragma unroll
  for (int bk = 0; bk < 8; ++bk) acc[bk] = zero4();
  float bsum = 0.f;
#pragma unroll
  for (int p = 0; p < NB - 1; ++p)
    if (p < nsteps) issue(p);
  for (int i = 0; i < nsteps; ++i) {
    // this step's copies are done when at most the later issued steps' 2 * WT each remain
    const int ahead = nsteps - 1 - i < NB - 2 ? nsteps - 1 - i : NB - 2;
    if (ahead >= 2)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * WT) : "memory");
    else if (ahead == 1)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * WT) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave's copies of this step have landed; step i-1 is read
    if (i + NB - 1 < nsteps) issue(i + NB - 1);
    const int b = i % NB;
#pragma unroll
    for (int k = 0; k < WT; ++k) {
      if (t0 + static_cast<int64_t>(i) * WT + k >= t1) break;  // wave-uniform
      const f4 av = Ds[b][k][tpos(16 * w + rl, g)];
      f4 bv[8];
#pragma unroll
      for (int bk = 0; bk < 8; ++bk) bv[bk] = Xs[b][k][tpos(16 * bk + rl, g)];
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int bk = 0; bk < 8; ++bk) acc[bk] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[e], bv[bk][e], acc[bk], 0, 0, 0);
      if (SPREAD && has_b) {  // bias: thread (q, f) sums feature f's row quad q (every wave takes a share)
        const f4 v = Ds[b][k][tpos(tid & (kCD - 1), tid >> 7)];
        bsum += (v[0] + v[1]) + (v[2] + v[3]);
      }
      if (!SPREAD && tid < 128) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const f4 v = Ds[b][k][tpos(tid, q)];
          bsum += (v[0] + v[1]) + (v[2] + v[3]);
        }
      }
    }
  }
#pragma unroll
  for (int bk = 0; bk < 8; ++bk)
#pragma unroll
    for (int e = 0; e < 4; ++e) slab[(16 * w + 4 * g + e) * kCD + 16 * bk + rl] = acc[bk][e];
  if (!SPREAD && has_b && tid < 128) slab_b[tid] = bsum;
  if (SPREAD && has_b) {  // the four row-quad partials of each feature, in quad order
    __shared__ float bred[4 * kCD];
    bred[tid] = bsum;
    __syncthreads();
    if (tid < kCD) slab_b[tid] = ((bred[tid] + bred[kCD + tid]) + bred[2 * kCD + tid]) + bred[3 * kCD + tid];
  }
}

// NB = 2 with the two buffers as distinct NAMED LDS arrays and the step loop unrolled by two, so every
// buffer index is static.  With one dynamically indexed [NB] array the compiler could not tell the
// buffer a step reads from the one the next step's copies are filling, and waited for those copies
// (vmcnt(0)) before the step's first LDS read: step i + 1's copy never ran under step i's MFMAs.  The
// next step's copy is issued unconditionally (past the segment's end it re-reads tile t0 into the idle
// buffer, drained at the end), since a branch around it would merge two wait histories into vmcnt(0).
template <bool SPREAD, int WT>
__device__ __forceinline__ void tiled_segment2(const float* __restrict__ dz, const float* __restrict__ xin, int64_t t0,
                                               int64_t t1, bool has_b, float* __restrict__ slab,
                                               float* __restrict__ slab_b, f4 (*D0)[512], f4 (*X0)[512],
                                               f4 (*D1)[512], f4 (*X1)[512]) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int rl = lane & 15, g = lane >> 4;
  const int nsteps = static_cast<int>((t1 - t0 + WT - 1) / WT);
  const int P = 64 * w + lane;
  const int src_chunk = (P >> 2) * 4 + ((P & 3) ^ (((P >> 5) & 1) * 3));
  // buffer_load ... lds over the segment's tiles (global_load_lds carried no LDS memory operand the
  // compiler could tell apart, so it waited on it before any LDS read even with separate buffers)
  const int64_t nt = t1 - t0;
  const int nbytes = static_cast<int>(nt * 8192 < 0x7fffffff ? nt * 8192 : 0x7fffffff);
  const rsrc_t dr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(dz + t0 * 2048), static_cast<short>(0), nbytes,
                                                      0x00020000);
  const rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(xin + t0 * 2048), static_cast<short>(0), nbytes,
                                                      0x00020000);
  auto issue = [&](int step, f4 (*Dd)[512], f4 (*Xd)[512]) {  // tiles past t1: tile t0
#pragma unroll
    for (int k = 0; k < WT; ++k) {
      int tt = step * WT + k;
      tt = tt < nt ? tt : 0;
      const int vo = tt * 8192 + 16 * src_chunk;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(dr, (__attribute__((address_space(3))) void*)(&Dd[k][64 * w]), 16, vo, 0,
                                               0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (__attribute__((address_space(3))) void*)(&Xd[k][64 * w]), 16, vo, 0,
                                               0, 0);
    }
  };
  f4 acc[8];
#pragma unroll
  for (int bk = 0; bk < 8; ++bk) acc[bk] = zero4();
  float bsum = 0.f;
  auto body = [&](int i, f4 (*Dc)[512], f4 (*Xc)[512], f4 (*Dn)[512], f4 (*Xn)[512]) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this step's copies (the only ones in flight)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave's copies of this step have landed; step i - 1 is read
    issue(i + 1, Dn, Xn);
#pragma unroll
    for (int k = 0; k < WT; ++k) {
      if (t0 + static_cast<int64_t>(i) * WT + k >= t1) break;  // wave-uniform
      const f4 av = Dc[k][tpos(16 * w + rl, g)];
      f4 bv[8];
#pragma unroll
      for (int bk = 0; bk < 8; ++bk) bv[bk] = Xc[k][tpos(16 * bk + rl, g)];
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int bk = 0; bk < 8; ++bk) acc[bk] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[e], bv[bk][e], acc[bk], 0, 0, 0);
      if (SPREAD && has_b) {
        const f4 v = Dc[k][tpos(tid & (kCD - 1), tid >> 7)];
        bsum += (v[0] + v[1]) + (v[2] + v[3]);
      }
      if (!SPREAD && tid < 128) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const f4 v = Dc[k][tpos(tid, q)];
          bsum += (v[0] + v[1]) + (v[2] + v[3]);
        }
      }
    }
  };
  if (nsteps > 0) issue(0, D0, X0);
  for (int i = 0; i < nsteps; i += 2) {
    body(i, D0, X0, D1, X1);
    if (i + 1 >= nsteps) break;
    body(i + 1, D1, X1, D0, X0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the copy issued past the end lands before reuse
#pragma unroll
  for (int bk = 0; bk < 8; ++bk)
#pragma unroll
    for (int e = 0; e < 4; ++e) slab[(16 * w + 4 * g + e) * kCD + 16 * bk + rl] = acc[bk][e];
  if (!SPREAD && has_b && tid < 128) slab_b[tid] = bsum;
  if (SPREAD && has_b) {  // the four row-quad partials of each feature, in quad order
    __shared__ float bred[4 * kCD];
    bred[tid] = bsum;
    __syncthreads();
    if (tid < kCD) slab_b[tid] = ((bred[tid] + bred[kCD + tid]) + bred[2 * kCD + tid]) + bred[3 * kCD + tid];
  }
}

__global__ void __launch_bounds__(kCThreads, 1) chain_wgrad_kernel(const ChainWgradArgs a) {
  __shared__ f4 Ds[3][kWTiles][512];
  __shared__ f4 Xs[3][kWTiles][512];
  const int s = blockIdx.y, c = blockIdx.x;
  const int64_t t0 = c * a.ntiles / a.splits, t1 = (c + 1) * a.ntiles / a.splits;
  tiled_segment<3>(a.dz_t[s], a.in_t[s], t0, t1, a.has_b[s] != 0, a.part_w[s] + static_cast<int64_t>(c) * kCD * kCD,
                a.part_b[s] + static_cast<int64_t>(c) * kCD, Ds, Xs);
}

// Every T-layout weight gradient of a backward in ONE launch: the jobs' tiles are concatenated
// (job j owns [tile0[j], tile0[j + 1]): jobs may differ in row count) and workgroup i takes the equal share
// [i * total / G, (i + 1) * total / G), i.e. at most a few job segments; each segment leaves one
// slab, job j's slabs contiguous from workgroup wg_lo[j] on.  Versus one launch per layer with
// 256 / jobs splits per job: the same MFMA work, ~256 + jobs slabs in all instead of 256 per
// launch, and one launch tail.
struct TiledFlatArgs {
  const float* in_t[X2G_TILED_MAX_JOBS];
  const float* dz_t[X2G_TILED_MAX_JOBS];
  float* slab_w[X2G_TILED_MAX_JOBS];  // job j's slab k (k = workgroup - wg_lo[j]) at + k * D * D
  float* slab_b[X2G_TILED_MAX_JOBS];  // ... and its bias slab at + k * D
  int wg_lo[X2G_TILED_MAX_JOBS];
  int has_b[X2G_TILED_MAX_JOBS];
  int64_t tile0[X2G_TILED_MAX_JOBS + 1];  // job j: tiles [tile0[j], tile0[j + 1]) of the concatenation
  int64_t total;
  int njobs;
};

// NB LDS buffers of 2 x WT tiles (NB x WT x 16 KB; NB - 1 steps in flight); WPC workgroups per CU
template <int NB, bool SPREAD = true, int WT = kWTiles, int WPC = 1>
__global__ void __launch_bounds__(kCThreads, 2 * WPC) tiled_flat_kernel(const TiledFlatArgs a) {
  static_assert(NB == 2, "the flat launch's two named buffers (tiled_segment2)");
  __shared__ f4 D0[WT][512];
  __shared__ f4 X0[WT][512];
  __shared__ f4 D1[WT][512];
  __shared__ f4 X1[WT][512];
  const int64_t G = gridDim.x, i = blockIdx.x;
  const int64_t lo = i * a.total / G, hi = (i + 1) * a.total / G;
  int j0 = 0;
  while (j0 < a.njobs && a.tile0[j0 + 1] <= lo) ++j0;  // (uniform; <= 64 jobs)
  for (int j = j0; j < a.njobs && a.tile0[j] < hi; ++j) {
    const int64_t s0 = lo > a.tile0[j] ? lo : a.tile0[j];
    const int64_t s1 = hi < a.tile0[j + 1] ? hi : a.tile0[j + 1];
    if (s0 >= s1) continue;
    __syncthreads();  // a previous segment's last buffers are no longer read
    const int64_t k = i - a.wg_lo[j];
    tiled_segment2<SPREAD, WT>(a.dz_t[j], a.in_t[j], s0 - a.tile0[j], s1 - a.tile0[j], a.has_b[j] != 0,
                               a.slab_w[j] + k * kCD * kCD, a.slab_b[j] + k * kCD, D0, X0, D1, X1);
  }
}

inline int chain_wgrad_splits_of(int64_t ntiles, int stages) {
  // at most one workgroup per CU over all stages (96 KB of LDS each: a 257th would run alone in a
  // second round), >= 4 tiles each
  int64_t per = 256 / stages;
  const int64_t cap = (ntiles + 3) / 4;
  if (per > cap) per = cap;
  return static_cast<int>(per < 1 ? 1 : per);
}

// ---------------------------------------------------------------- conv projections
// SBFTransformerConv's five projections (sbftransformer_conv.py:99-107,127) with the row-chain
// v2 structure: a workgroup's <= 96 rows of x, and of x_src = x * (rbf W_rbf^T) formed in
// registers, sit in LDS; each wave computes its 16-feature slice of q, k, v and skip.
constexpr int kRbfMax = 8;
constexpr int kGateRB = 3;  // row blocks per chunk of the pipelined projection kernels

struct ProjFwdArgs {
  const float* x;
  const float* rbf;
  const float* wr;
  int RR;
  x2g_proj p[4];
  float* x_t;
  float* xs_t;
  int64_t R;
};

template <int RB>
__device__ __forceinline__ void load_rows_slice(const float* P, int r0, int nrows, int w, int rl, int g,
                                                f4 (&v)[RB]) {
  const rsrc_t pr = rsrc(P);
#pragma unroll
  for (int rb = 0; rb < RB; ++rb) {
    const int r = 16 * rb + rl;
    const bool ok = r < nrows;
    v[rb] = bload4(pr, 4 * ((r0 + (ok ? r : 0)) * kCD + 16 * w + 4 * g), 0) * (ok ? 1.0f : 0.0f);
  }
}

// rows of rbf [R, RR] -> srbf[row * NJ + j] (zero beyond RR / nrows); W_rbf [D, RR] -> swr[c * NJ + j]
template <int NJ, int RB = kV2RB, int NT = kCThreads>
__device__ __forceinline__ void stage_rbf(float* __restrict__ srbf, const float* __restrict__ rbf, int RR, int r0,
                                          int nrows) {
  for (int i = threadIdx.x; i < RB * 16 * NJ; i += NT) {
    const int r = i / NJ, j = i % NJ;
    srbf[i] = (r < nrows && j < RR) ? rbf[static_cast<int64_t>(r0 + r) * RR + j] : 0.0f;
  }
}

// the gate filter f = rbf W_rbf^T at (row r, features c0..c0+3), the rbf_gate kernels' order
template <int NJ>
__device__ __forceinline__ f4 gate_filter(const float* __restrict__ srbf, const float* __restrict__ swr, int r, int c0) {
  f4 f;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    float acc = 0.0f;
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc = fmaf(swr[(c0 + e) * NJ + j], srbf[r * NJ + j], acc);
    f[e] = acc;
  }
  return f;
}

// (A two-chunk software pipeline as in the gate backward below measured slower here, 51.5 vs
// 39.6 us at config 2: the products are already most of the launch, and 48-row chunks add a
// barrier skew per chunk; phase stamps, scripts/trace_proj_fwd.py.)
template <int NJ>
__global__ void __launch_bounds__(kCThreads, 2) conv_proj_fwd_kernel(const ProjFwdArgs a) {
  constexpr int RB = kV2RB;
  __shared__ f4 img[2][RB * 16 * 32];  // x, x_src
  __shared__ float srbf[RB * 16 * NJ];
  __shared__ float swr[kCD * NJ];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int rl = lane & 15, g = lane >> 4;
  const int64_t nblk = (a.R + 15) / 16, G = gridDim.x;
  const int64_t nch = (nblk + RB * G - 1) / (RB * G) * G;
  for (int i = tid; i < kCD * NJ; i += kCThreads) {
    const int c = i / NJ, j = i % NJ;
    swr[i] = j < a.RR ? a.wr[c * a.RR + j] : 0.0f;
  }
  // W^T for the backward (x2g_proj.wt): every workgroup writes its share, one element per thread
  // (the first 8 chunks writing it all made those workgroups the launch's tail)
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kCThreads + tid; i < 4 * kCD * kCD; i += G * kCThreads) {
    const int p = static_cast<int>(i / (kCD * kCD)), e = static_cast<int>(i % (kCD * kCD));
    if (a.p[p].wt) a.p[p].wt[e] = a.p[p].w[(e % kCD) * kCD + e / kCD];
  }
  for (int64_t ch = blockIdx.x; ch < nch; ch += G) {
    int r0, nrows;
    chunk_rows(ch, nch, nblk, a.R, r0, nrows);
    __syncthreads();
    stage_rows<RB>(img[0], a.x, nullptr, r0, nrows);
    stage_rbf<NJ, RB>(srbf, a.rbf, a.RR, r0, nrows);
    f4 A[8];
    load_slice<false>(a.p[0].w, w, rl, g, A);
    __syncthreads();
    {
      f4 xv[RB], xs[RB];
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) {
        const int r = 16 * rb + rl;
        xv[rb] = img[0][ipos(r, 4 * w + g)];
        xs[rb] = xv[rb] * gate_filter<NJ>(srbf, swr, r, 16 * w + 4 * g);
        img[1][ipos(r, 4 * w + g)] = xs[rb];
      }
      if (a.x_t) store_t_slice(a.x_t, xv, r0, nrows, w, rl, g);
      if (a.xs_t) store_t_slice(a.xs_t, xs, r0, nrows, w, rl, g);
    }
    __syncthreads();
#pragma unroll 1
    for (int p = 0; p < 4; ++p) {  // q (x), k (x_src), v (x_src), skip (x)
      const x2g_proj& P = a.p[p];
      f4 An[8];
      load_slice<false>(a.p[p + 1 < 4 ? p + 1 : 0].w, w, rl, g, An);
      const f4 bias = bload4(rsrc(P.b ? P.b : P.w), 4 * (16 * w + 4 * g), 0) * (P.b ? 1.0f : 0.0f);
      f4 acc[RB];
      slice_gemm(img[(p == 1 || p == 2) ? 1 : 0], A, acc, rl, g);
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) {
        const int r = 16 * rb + rl;
        if (r < nrows) *reinterpret_cast<f4*>(P.out + (r0 + r) * kCD + 16 * w + 4 * g) = acc[rb] + bias;
      }
      pin(An);
#pragma unroll
      for (int b = 0; b < 8; ++b) A[b] = An[b];
    }
  }
}

// The projections' backward with the rbf gate's backward folded into the dxs epilogue (what
// x2g_rbf_gate_bwd did as a separate pass over dxs, x, rbf and dx): dxs never leaves registers.
//   dx   = (dx_add + dxs * f) + (dq Wq + dskip Ws)       f = rbf W_rbf^T (the forward's filter)
//   (dx_add is read only when given: an uninitialised dx never meets a 0 * NaN)
//   drbf = (dxs * x) W_rbf   (+= with drbf_acc)          per row: MFMA over the wave's features, then waves in order
//   dW_rbf slab of this workgroup = sum over its rows of (dxs * x)^T rbf   (fixed-order slab sum after)
//
// Software pipeline.  A workgroup walks its chunks (<= 48 rows each, kGateRB row blocks) as a
// sequence of operand PAIRS, (dk, dv) then (dq, dskip) per chunk, through two LDS pair buffers:
// pair q + 1's copies (buffer_load ... lds, no registers) fly while pair q's products run, so the
// HBM traffic (operands in, T-layout copies and dx out) overlaps the matrix pipe instead of
// alternating with it (the one-pass-per-chunk form kept the HBM busy during only ~40 % of the
// launch: phase stamps, scripts/trace_gate.py).  The next pair's weight slices are read after this
// pair's products, the next chunk's x rows one pair ahead, dx_add's under the (dq, dskip) products;
// dx leaves once per row (dxs * f held in registers until then).  Each pair's two products are one
// K = 256 accumulation chain.  Nothing between a pair's copies and its products may wait on vmcnt
// for a load issued after those copies (a spill reload would: the kernel must not spill).
struct ProjBwdGateArgs {
  x2g_proj_grad gr[4];
  const float* dx_add;
  float* dx;
  const float* x;
  const float* rbf;
  const float* wr;
  float* drbf;
  float* part_w;
  int RR;
  int drbf_acc;
  int64_t R;
};


template <int NJ, bool TW>  // TW: every projection's W^T given (else W read transposed)
__global__ void __launch_bounds__(kCThreads, 2) conv_proj_bwd_gate_kernel(const ProjBwdGateArgs a) {
  constexpr int RB = kGateRB;
  constexpr int kImg = RB * 16 * 32;
  // the two pair buffers as four distinct arrays (24 KB each): the compiler then sees that a pair's
  // products never read what the other pair's in-flight copies write, and adds no vmcnt wait
  __shared__ f4 img_k[kImg], img_v[kImg];  // (dk, dv)
  __shared__ f4 img_q[kImg], img_s[kImg];  // (dq, dskip)
  __shared__ float srbf[RB * 16 * NJ];
  __shared__ float swr[kCD * NJ];
  __shared__ float red[kCWaves * RB * 16 * 16];  // drbf partials: [wave][row][16 columns, j < NJ used]
  __shared__ float sdw[kCD * NJ];                 // this workgroup's dW_rbf
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int rl = lane & 15, g = lane >> 4;
  const int64_t nblk = (a.R + 15) / 16, G = gridDim.x;
  const int64_t nch = (nblk + RB * G - 1) / (RB * G) * G;  // a multiple of G: every workgroup nk chunks
  const int nk = static_cast<int>(nch / G);
  const int c0 = 16 * w + 4 * g;
  for (int i = tid; i < kCD * NJ; i += kCThreads) {
    const int c = i / NJ, j = i % NJ;
    swr[i] = j < a.RR ? a.wr[c * a.RR + j] : 0.0f;
    sdw[i] = 0.0f;
  }
  auto load_ws = [&](int p, f4 (&dst)[8]) {
    if (TW)
      load_slice<false>(a.gr[p].wt, w, rl, g, dst);
    else
      load_slice<true>(a.gr[p].w, w, rl, g, dst);
  };
  auto t_copy = [&](int p, const f4* im, int r0, int nrows) {  // the weight gradient's dy operand
    f4 v[RB];
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) v[rb] = im[ipos(16 * rb + rl, 4 * w + g)];
    store_t_slice(a.gr[p].g_t, v, r0, nrows, w, rl, g);
  };
  auto chunk = [&](int k, int& r0, int& nrows) { chunk_rows(blockIdx.x + k * G, nch, nblk, a.R, r0, nrows); };
  // Every global access of the chunk loop is unconditional (a disabled one goes through an empty
  // descriptor or to an out-of-range offset): the compiler's vmcnt waits then count exactly instead
  // of falling back to vmcnt(0), which would wait for the next pair's copies.
  const int64_t bytes = a.R * kCD * 4;
  const rsrc_t ar = rsrc_n(a.dx_add, bytes, a.dx_add != nullptr);  // dx_add absent: reads 0
  const rsrc_t dr = rsrc_n(a.dx, bytes, true);
  const rsrc_t xr = rsrc_n(a.x, bytes, true);
  const rsrc_t rr = rsrc_n(a.rbf, a.R * a.RR * 4, true);
  const rsrc_t br = rsrc_n(a.drbf, a.R * a.RR * 4, a.drbf != nullptr);
  const rsrc_t bo = rsrc_n(a.drbf, a.R * a.RR * 4, a.drbf != nullptr && a.drbf_acc);
  static_assert(RB * 16 * NJ <= kCThreads && RB * 16 * kRbfMax <= kCThreads, "one srbf / drbf element per thread");
  // outstanding operations a pair's top wait may leave (issued after the pair's copies): 2 RB
  // T-layout stores, the next weight slices (kWL loads each) and, at a (dk, dv) top, RB dx stores
  constexpr int kWL = TW ? 8 : 32;
  constexpr int kKVWait = 3 * RB + 2 * kWL < 63 ? 3 * RB + 2 * kWL : 63;
  constexpr int kQSWait = 2 * RB + 2 * kWL < 63 ? 2 * RB + 2 * kWL : 63;
  if (nk > 0) {
    int r0, nrows;
    chunk(0, r0, nrows);
    stage_rows_async<RB>(img_k, a.gr[1].g, a.R, r0);
    stage_rows_async<RB>(img_v, a.gr[2].g, a.R, r0);
  }
  f4 A[8], An[8];  // this pair's two weight slices
  load_ws(1, A);
  load_ws(2, An);
  __syncthreads();  // swr
  float dold = 0.0f;
  int doff = kOOB;
  auto drbf_out = [&]() {  // the last chunk's drbf (partials in red, written before the last barrier)
    const int i = doff == kOOB ? 0 : tid, r = i / a.RR, j = i % a.RR;
    float sum = 0.0f;
#pragma unroll
    for (int ww = 0; ww < kCWaves; ++ww) sum += red[(ww * RB * 16 + r) * 16 + j];
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, dold + sum), br, doff, 0, 0);
  };
  for (int k = 0; k < nk; ++k) {
    int r0, nrows;
    chunk(k, r0, nrows);
    // ---- (dk, dv): acc1 = dxs = [dk | dv] [Wk ; Wv]
    if (k > 0)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kKVWait) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // every wave's copies landed; the previous chunk's (dq, dskip), srbf and red read
    drbf_out();
    stage_rows_async<RB>(img_q, a.gr[0].g, a.R, r0);
    stage_rows_async<RB>(img_s, a.gr[3].g, a.R, r0);
    asm volatile("" ::: "memory");  // every later memory operation issues after the copies (the top waits count on it)
    f4 xv[RB];  // this chunk's x slice and rbf element, for the epilogue under the second pair
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {
      const int r = 16 * rb + rl;
      xv[rb] = bload4(xr, 4 * ((r0 + (r < nrows ? r : 0)) * kCD + c0), 0);  // rows past the chunk: its first
    }
    float rbv;
    {
      const int r = tid / NJ, j = tid % NJ;
      rbv = bload1(rr, (tid < RB * 16 * NJ && r < nrows && j < a.RR) ? 4 * ((r0 + r) * a.RR + j) : kOOB, 0);
    }
    t_copy(1, img_k, r0, nrows);
    t_copy(2, img_v, r0, nrows);
    f4 acc1[RB];
    slice_gemm(img_k, A, acc1, rl, g);
    load_ws(0, A);  // Wq under the second product
    slice_gemm<RB, false>(img_v, An, acc1, rl, g);
    load_ws(3, An);  // Ws under the next pair's wait
    if (tid < RB * 16 * NJ) srbf[tid] = rbv;  // read after the next barrier
    // ---- (dq, dskip): dx = (dx_add + dxs * f) + [dq | dskip] [Wq ; Ws]; the gate epilogue of
    // acc1 runs under these products
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kQSWait) : "memory");
    __syncthreads();  // every wave's copies landed; (dk, dv) no longer read; srbf written
    // reads that must not wait behind the next chunk's copies go out before them
    doff = tid < nrows * a.RR ? 4 * (r0 * a.RR + tid) : kOOB;
    dold = bload1(bo, doff, 0);  // drbf += : 0 when not accumulating
    f4 xa[RB];
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {
      const int r = 16 * rb + rl;
      xa[rb] = bload4(ar, 4 * ((r0 + (r < nrows ? r : 0)) * kCD + c0), 0);
    }
    {
      const bool more = k + 1 < nk;
      int r1, n1;
      chunk(more ? k + 1 : k, r1, n1);
      stage_rows_async<RB>(img_k, a.gr[1].g, a.R, r1, more);
      stage_rows_async<RB>(img_v, a.gr[2].g, a.R, r1, more);
      asm volatile("" ::: "memory");
    }
    t_copy(0, img_q, r0, nrows);
    t_copy(3, img_s, r0, nrows);
    f4 acc[RB], d1[RB];  // d1 = dx_add + dxs * f
    slice_gemm(img_q, A, acc, rl, g);
    load_ws(1, A);  // the next chunk's Wk under the second product (once more after the last chunk)
    f4 wrv;  // drbf's MFMA B operand: lane (j, g) of step e holds W_rbf[c0 + e][j] (zero for j >= NJ)
#pragma unroll
    for (int e = 0; e < 4; ++e) wrv[e] = swr[(c0 + e) * NJ + (rl < NJ ? rl : 0)] * (rl < NJ ? 1.0f : 0.0f);
    float aw[4][NJ];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) aw[i][j] = 0.0f;
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {
      const int r = 16 * rb + rl;
      d1[rb] = xa[rb] + acc1[rb] * gate_filter<NJ>(srbf, swr, r, c0);
      const f4 df = r < nrows ? acc1[rb] * xv[rb] : zero4();
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) aw[i][j] = fmaf(df[i], srbf[r * NJ + j], aw[i][j]);
      // the wave's drbf partial of row block rb = df (16 rows x its 16 features) W_rbf slice, on the
      // matrix pipe: lane (j, g) ends with rows 16 rb + 4 g + i, column j (zero for j >= NJ)
      f4 pd = zero4();
#pragma unroll
      for (int e = 0; e < 4; ++e) pd = __builtin_amdgcn_mfma_f32_16x16x4f32(df[e], wrv[e], pd, 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 4; ++i) red[(w * RB * 16 + 16 * rb + 4 * g + i) * 16 + rl] = pd[i];
    }
    // this chunk's dW_rbf partial: the 16 row lanes' sum (in every lane of the row group), added by
    // all 16 lanes at once (same address, same value: one wave instruction, no branch)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) sdw[(c0 + i) * NJ + j] += row_sum16(aw[i][j]);
    slice_gemm<RB, false>(img_s, An, acc, rl, g);
    load_ws(2, An);
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {
      const int r = 16 * rb + rl;
      bstore4(dr, d1[rb] + acc[rb], r < nrows ? 4 * ((r0 + r) * kCD + c0) : kOOB);
    }
  }
  __syncthreads();  // red of the last chunk
  drbf_out();
  float* slab = a.part_w + static_cast<int64_t>(blockIdx.x) * kCD * a.RR;  // this workgroup's dW_rbf slab
  for (int i = tid; i < kCD * a.RR; i += kCThreads) slab[i] = sdw[(i / a.RR) * NJ + i % a.RR];
}

inline bool al16(const void* p) { return reinterpret_cast<uintptr_t>(p) % 16 == 0; }

// rows per weight-gradient chunk: about two workgroups per CU over all jobs, >= 64 rows
inline int wgrad_chunk_rows(int64_t R, int jobs) {
  const int64_t target = 512;
  const int64_t per_job = (target + jobs - 1) / jobs;
  int64_t cr = (R + per_job - 1) / per_job;
  cr = (cr + 31) / 32 * 32;
  return static_cast<int>(cr < 64 ? 64 : cr);
}

}  // namespace
}  // namespace x2g

using namespace x2g;

X2G_API int64_t x2g_chain_t_floats(int64_t rows, int32_t dim) {
  return rows > 0 && dim > 0 ? (rows + 15) / 16 * 16 * dim : 0;
}

// validate one chain's forward and fill its kernel arguments; empty = no rows (nothing to launch)
static int chain_fwd_prepare(const float* x, const float* res_ext, const x2g_chain_stage* stages, int32_t n_stages,
                             int64_t rows, int32_t dim, float* in_t, ChainFwdArgs& a, bool& empty) {
  empty = false;
  if (!stages || n_stages < 1 || n_stages > X2G_CHAIN_MAX_STAGES || rows < 0 || dim <= 0) return X2G_EINVAL;
  if (dim != kCD || rows * kCD * 4 >= (int64_t(1) << 31)) return X2G_EUNSUPPORTED;
  a = ChainFwdArgs{};
  a.x = x;
  a.res = res_ext;
  a.in_t = in_t;
  a.tf = x2g_chain_t_floats(rows, dim);
  a.R = rows;
  a.n = n_stages;
  int n_ext = 0, held = 0;
  for (int s = 0; s < n_stages; ++s) {
    const x2g_chain_stage& S = stages[s];
    if (!S.w || (s == n_stages - 1 && !S.y)) return X2G_EINVAL;
    if (S.flags & ~(X2G_CHAIN_SILU | X2G_CHAIN_HOLD | X2G_CHAIN_RES_HELD | X2G_CHAIN_RES_EXT)) return X2G_EINVAL;
    // one register set holds the residual: a ResidualLayer input (HOLD .. RES_HELD) must not span
    // the RES_EXT stage, and a stage adds at most one residual
    if ((S.flags & X2G_CHAIN_RES_EXT) && (S.flags & (X2G_CHAIN_HOLD | X2G_CHAIN_RES_HELD))) return X2G_EINVAL;
    if (S.flags & X2G_CHAIN_RES_EXT) held = 0;
    if (S.flags & X2G_CHAIN_HOLD) held = 1;
    if ((S.flags & X2G_CHAIN_RES_HELD) && !held) return X2G_EINVAL;
    if (S.flags & X2G_CHAIN_RES_EXT) ++n_ext;
    if (!al16(S.w) || !al16(S.b) || !al16(S.z) || !al16(S.y) || !al16(S.wt)) return X2G_EUNSUPPORTED;
    a.st[s] = S;
  }
  if (n_ext > 1 || (n_ext && !res_ext)) return X2G_EINVAL;
  if (rows == 0) {
    empty = true;
    return X2G_OK;
  }
  if (!x) return X2G_EINVAL;
  if (!al16(x) || !al16(res_ext) || !al16(in_t)) return X2G_EUNSUPPORTED;
  return X2G_OK;
}

X2G_API int x2g_chain_fwd(const float* x, const float* res_ext, const x2g_chain_stage* stages, int32_t n_stages,
                          int64_t rows, int32_t dim, float* in_t, void* stream) {
  ChainFwdArgs a{};
  bool empty;
  if (int rc = chain_fwd_prepare(x, res_ext, stages, n_stages, rows, dim, in_t, a, empty)) return rc;
  if (empty) return X2G_OK;
  hipStream_t st = as_stream(stream);
  const int64_t nblk = (rows + 15) / 16;  // one workgroup per CU, <= 96 rows each
  chain_fwd_v4<<<static_cast<unsigned>(nblk < 256 ? nblk : 256), kCThreads, 0, st>>>(a);
  return last_launch_status();
}

X2G_API int x2g_chain_fwd_ln(const float* x, const float* row_stats, const int32_t* seg_rowptr, int64_t num_segments,
                             float eps, float* x_norm, float* seg_mean, float* seg_rstd, const float* res_ext,
                             const x2g_chain_stage* stages, int32_t n_stages, int64_t rows, int32_t dim, float* in_t,
                             void* stream) {
  ChainFwdArgs a{};
  bool empty;
  if (int rc = chain_fwd_prepare(x, res_ext, stages, n_stages, rows, dim, in_t, a, empty)) return rc;
  if (num_segments < 0 || (rows > 0 && (!row_stats || !seg_rowptr || num_segments < 1))) return X2G_EINVAL;
  if (reinterpret_cast<uintptr_t>(row_stats) % 8 || !al16(x_norm)) return X2G_EUNSUPPORTED;
  if (empty) return X2G_OK;
  const ChainFwdLnArgs b{a, {reinterpret_cast<const float2*>(row_stats), seg_rowptr, x_norm, seg_mean, seg_rstd,
                             num_segments, eps}};
  const int64_t nblk = (rows + 15) / 16;
  // inference (no T-layout inputs and no pre-activations asked for): the instance without those stores
  bool infer = b.a.in_t == nullptr;
  for (int s = 0; s < b.a.n; ++s) infer = infer && b.a.st[s].z == nullptr;
  if (infer)
    chain_fwd_v4_ln_infer<<<static_cast<unsigned>(nblk < 256 ? nblk : 256), kCThreads, 0, as_stream(stream)>>>(b);
  else
    chain_fwd_v4_ln<<<static_cast<unsigned>(nblk < 256 ? nblk : 256), kCThreads, 0, as_stream(stream)>>>(b);
  return last_launch_status();
}

static int chain_bwd_prepare(const float* dy, const float* dy_add, const x2g_chain_bwd_stage* stages, int32_t n_stages,
                             int64_t rows, int32_t dim, float* dx, float* d_res_ext, float* dz_t, ChainBwdArgs& a,
                             bool& empty, bool& res_accum) {
  empty = false;
  res_accum = false;
  if (!stages || n_stages < 1 || n_stages > X2G_CHAIN_MAX_STAGES || rows < 0 || dim <= 0) return X2G_EINVAL;
  if (dim != kCD || rows * kCD * 4 >= (int64_t(1) << 31)) return X2G_EUNSUPPORTED;
  a = ChainBwdArgs{};
  a.dy = dy;
  a.dy_add = dy_add;
  a.dx = dx;
  a.dres = d_res_ext;
  a.dz_t = dz_t;
  a.tf = x2g_chain_t_floats(rows, dim);
  a.R = rows;
  a.n = n_stages;
  int n_ext = 0, held = 0;
  for (int s = 0; s < n_stages; ++s) {
    const x2g_chain_bwd_stage& S = stages[s];
    if (!S.w || ((S.flags & X2G_CHAIN_SILU) && !S.z)) return X2G_EINVAL;
    if (S.flags & ~(X2G_CHAIN_SILU | X2G_CHAIN_HOLD | X2G_CHAIN_RES_HELD | X2G_CHAIN_RES_EXT | X2G_CHAIN_RES_ACCUM))
      return X2G_EINVAL;
    if ((S.flags & X2G_CHAIN_RES_ACCUM) && !(S.flags & X2G_CHAIN_RES_EXT)) return X2G_EINVAL;
    if ((S.flags & X2G_CHAIN_RES_EXT) && (S.flags & (X2G_CHAIN_HOLD | X2G_CHAIN_RES_HELD))) return X2G_EINVAL;
    if (S.flags & X2G_CHAIN_RES_EXT) held = 0;
    if (S.flags & X2G_CHAIN_HOLD) held = 1;
    if ((S.flags & X2G_CHAIN_RES_HELD) && !held) return X2G_EINVAL;
    if (S.flags & X2G_CHAIN_RES_EXT) ++n_ext;
    if (S.flags & X2G_CHAIN_RES_ACCUM) res_accum = true;
    if (!al16(S.w) || !al16(S.wt) || !al16(S.z) || !al16(S.dz)) return X2G_EUNSUPPORTED;
    a.st[s] = S;
  }
  if (n_ext > 1) return X2G_EINVAL;
  if (rows == 0) {
    empty = true;
    return X2G_OK;
  }
  if (!dy || !dx) return X2G_EINVAL;
  if (!al16(dy) || !al16(dy_add) || !al16(dx) || !al16(d_res_ext) || !al16(dz_t)) return X2G_EUNSUPPORTED;
  return X2G_OK;
}

static int chain_bwd_launch(const ChainBwdArgs& a, int64_t rows, void* stream) {
  hipStream_t st = as_stream(stream);
  {  // through the batched kernel: a by-value ChainBwdArgs handed to the shared body by reference is
     // copied to scratch (392 B, 79 -> 121 us); a batch entry is not
    const int64_t nblk = (rows + 15) / 16;
    ChainBwdBatch b{};
    b.a[0] = a;
    const dim3 grid(static_cast<unsigned>(nblk < 256 ? nblk : 256), 1);
    chain_bwd_v3_batch<kV2RB><<<grid, kCThreads, 0, st>>>(b);
  }
  return last_launch_status();
}

X2G_API int x2g_chain_bwd_ln(const float* dy, const float* dy_add, const x2g_chain_bwd_stage* stages,
                             int32_t n_stages, int64_t rows, int32_t dim, float* dx, float* d_res_ext, float* dz_t,
                             const float* x_norm, float* row_gstats, void* stream) {
  ChainBwdArgs a{};
  bool empty, res_accum;
  if (int rc = chain_bwd_prepare(dy, dy_add, stages, n_stages, rows, dim, dx, d_res_ext, dz_t, a, empty, res_accum))
    return rc;
  if (rows > 0 && (!x_norm || !row_gstats)) return X2G_EINVAL;
  if (!al16(x_norm) || reinterpret_cast<uintptr_t>(row_gstats) % 8) return X2G_EUNSUPPORTED;
  if (empty) return X2G_OK;
  a.ln_y = x_norm;
  a.ln_gstats = reinterpret_cast<float2*>(row_gstats);
  return chain_bwd_launch(a, rows, stream);
}

X2G_API int x2g_chain_bwd(const float* dy, const float* dy_add, const x2g_chain_bwd_stage* stages, int32_t n_stages,
                          int64_t rows, int32_t dim, float* dx, float* d_res_ext, float* dz_t, void* stream) {
  ChainBwdArgs a{};
  bool empty, res_accum;
  if (int rc = chain_bwd_prepare(dy, dy_add, stages, n_stages, rows, dim, dx, d_res_ext, dz_t, a, empty, res_accum))
    return rc;
  if (empty) return X2G_OK;
  return chain_bwd_launch(a, rows, stream);
}

// grid of a batched chain launch: about one workgroup per CU over all jobs, each job's row blocks
// split evenly over its share (the kernels' chunking follows gridDim.x)
static inline unsigned chain_batch_grid(int64_t rows, int n_jobs) {
  const int64_t nblk = (rows + 15) / 16, per = 256 / n_jobs;
  return static_cast<unsigned>(nblk < per ? nblk : (per < 1 ? 1 : per));
}

// one chunk of <= 3 row blocks per workgroup covers the job: the 3-block form (products of 3 blocks
// instead of 6, half of them padding; at config 2 the readouts' 144 blocks on 51 workgroups)
static inline bool chain_batch_rb3(int64_t rows, unsigned grid_x) {
  const int64_t nblk = (rows + 15) / 16;
  return nblk <= 3 * static_cast<int64_t>(grid_x);
}

X2G_API int x2g_chain_fwd_batch(const x2g_chain_fwd_job* jobs, int32_t n_jobs, int32_t n_stages, int64_t rows,
                                int32_t dim, void* stream) {
  if (!jobs || n_jobs < 1 || n_jobs > kChainMaxJobs) return X2G_EINVAL;
  ChainFwdBatch b{};
  bool empty = false;
  for (int j = 0; j < n_jobs; ++j) {
    const x2g_chain_fwd_job& J = jobs[j];
    if (int rc = chain_fwd_prepare(J.x, J.res_ext, J.stages, n_stages, rows, dim, J.in_t, b.a[j], empty)) return rc;
  }
  if (empty) return X2G_OK;
  const dim3 grid(chain_batch_grid(rows, n_jobs), static_cast<unsigned>(n_jobs));
  if (chain_batch_rb3(rows, grid.x))
    chain_fwd_v4_batch<3><<<grid, kCThreads, 0, as_stream(stream)>>>(b);
  else
    chain_fwd_v4_batch<kV2RB><<<grid, kCThreads, 0, as_stream(stream)>>>(b);
  return last_launch_status();
}

X2G_API int x2g_chain_bwd_batch(const x2g_chain_bwd_job* jobs, int32_t n_jobs, int32_t n_stages, int64_t rows,
                                int32_t dim, void* stream) {
  if (!jobs || n_jobs < 1 || n_jobs > kChainMaxJobs) return X2G_EINVAL;
  ChainBwdBatch b{};
  bool empty = false, res_accum;
  for (int j = 0; j < n_jobs; ++j) {
    const x2g_chain_bwd_job& J = jobs[j];
    if (int rc = chain_bwd_prepare(J.dy, J.dy_add, J.stages, n_stages, rows, dim, J.dx, J.d_res_ext, J.dz_t, b.a[j],
                                   empty, res_accum))
      return rc;
  }
  if (empty) return X2G_OK;
  const dim3 grid(chain_batch_grid(rows, n_jobs), static_cast<unsigned>(n_jobs));
  if (chain_batch_rb3(rows, grid.x))
    chain_bwd_v3_batch<3><<<grid, kCThreads, 0, as_stream(stream)>>>(b);
  else
    chain_bwd_v3_batch<kV2RB><<<grid, kCThreads, 0, as_stream(stream)>>>(b);
  return last_launch_status();
}

X2G_API int32_t x2g_wgrad_batched_splits(int64_t rows, int32_t dim, int32_t num_jobs) {
  if (rows <= 0 || dim != kCD || num_jobs < 1 || num_jobs > X2G_CHAIN_MAX_STAGES) return 0;
  const int cr = wgrad_chunk_rows(rows, num_jobs);
  return static_cast<int32_t>((rows + cr - 1) / cr);
}

X2G_API size_t x2g_wgrad_batched_workspace(int64_t rows, int32_t dim, int32_t num_jobs) {
  const int32_t splits = x2g_wgrad_batched_splits(rows, dim, num_jobs);
  return static_cast<size_t>(num_jobs > 0 ? num_jobs : 0) * splits * (kCD * kCD + kCD) * sizeof(float);
}

X2G_API int x2g_wgrad_batched(const x2g_wgrad_job* jobs, int32_t num_jobs, int64_t rows, int32_t dim, int flags,
                              void* workspace, size_t workspace_bytes, void* stream) {
  if (!jobs || num_jobs < 1 || num_jobs > X2G_CHAIN_MAX_STAGES || rows <= 0 || dim <= 0 ||
      (flags & ~(X2G_ACCUM_WGRAD | X2G_DEFER_SLAB_SUM)))
    return X2G_EINVAL;
  if (dim != kCD || rows * kCD * 4 >= (int64_t(1) << 31)) return X2G_EUNSUPPORTED;
  const size_t need = x2g_wgrad_batched_workspace(rows, dim, num_jobs);
  if (!workspace || workspace_bytes < need) return X2G_EWORKSPACE;
  WgradArgs a{};
  a.R = rows;
  a.chunk_rows = wgrad_chunk_rows(rows, num_jobs);
  const int splits = x2g_wgrad_batched_splits(rows, dim, num_jobs);
  const size_t per_job = need / num_jobs;
  x2g_slab_job sj[X2G_CHAIN_MAX_STAGES];
  for (int j = 0; j < num_jobs; ++j) {
    const x2g_wgrad_job& J = jobs[j];
    if (!J.dy || !J.x || !J.dw) return X2G_EINVAL;
    if (!al16(J.dy) || !al16(J.x)) return X2G_EUNSUPPORTED;
    a.job[j] = J;
    a.part_w[j] = reinterpret_cast<float*>(static_cast<char*>(workspace) + per_job * j);
    a.part_b[j] = a.part_w[j] + static_cast<int64_t>(splits) * kCD * kCD;
    sj[j] = x2g_slab_job{a.part_w[j], J.db ? a.part_b[j] : nullptr, J.dw, J.db, kCD * kCD, J.db ? kCD : 0, splits};
  }
  hipStream_t st = as_stream(stream);
  wgrad_batched_kernel<<<dim3(static_cast<unsigned>(splits), static_cast<unsigned>(num_jobs)), kWThreads, 0, st>>>(a);
  const int rc = last_launch_status();
  if (rc || (flags & X2G_DEFER_SLAB_SUM)) return rc;
  return x2g_slab_sum_batch(sj, num_jobs, (flags & X2G_ACCUM_WGRAD) ? 1 : 0, stream);
}

static int32_t chain_wgrad_splits(int64_t rows, int32_t dim, int32_t n_stages) {
  if (rows <= 0 || dim != kCD || n_stages < 1 || n_stages > X2G_CHAIN_MAX_STAGES) return 0;
  return chain_wgrad_splits_of((rows + 15) / 16, n_stages);
}

X2G_API size_t x2g_chain_wgrad_workspace(int64_t rows, int32_t dim, int32_t n_stages) {
  const int32_t splits = chain_wgrad_splits(rows, dim, n_stages);
  return static_cast<size_t>(splits > 0 ? n_stages : 0) * splits * (kCD * kCD + kCD) * sizeof(float);
}

X2G_API int x2g_chain_wgrad(const float* in_t, const float* dz_t, int32_t n_stages, int64_t rows, int32_t dim,
                            float* const* dw, float* const* db, int flags, void* workspace, size_t workspace_bytes,
                            void* stream) {
  if (!in_t || !dz_t || !dw || n_stages < 1 || n_stages > X2G_CHAIN_MAX_STAGES || rows <= 0 || dim <= 0 ||
      (flags & ~(X2G_ACCUM_WGRAD | X2G_DEFER_SLAB_SUM)))
    return X2G_EINVAL;
  if (dim != kCD || rows * kCD * 4 >= (int64_t(1) << 31)) return X2G_EUNSUPPORTED;
  if (!al16(in_t) || !al16(dz_t)) return X2G_EUNSUPPORTED;
  const size_t need = x2g_chain_wgrad_workspace(rows, dim, n_stages);
  if (!workspace || workspace_bytes < need) return X2G_EWORKSPACE;
  ChainWgradArgs a{};
  const int64_t tf = x2g_chain_t_floats(rows, dim);
  for (int j = 0; j < n_stages; ++j) {
    a.in_t[j] = in_t + j * tf;
    a.dz_t[j] = dz_t + j * tf;
  }
  a.ntiles = (rows + 15) / 16;
  a.splits = chain_wgrad_splits(rows, dim, n_stages);
  const size_t per = need / n_stages;
  x2g_slab_job sj[X2G_CHAIN_MAX_STAGES];
  for (int j = 0; j < n_stages; ++j) {
    if (!dw[j]) return X2G_EINVAL;
    const bool hb = db && db[j];
    a.part_w[j] = reinterpret_cast<float*>(static_cast<char*>(workspace) + per * j);
    a.part_b[j] = a.part_w[j] + static_cast<int64_t>(a.splits) * kCD * kCD;
    a.has_b[j] = hb;
    sj[j] = x2g_slab_job{a.part_w[j], hb ? a.part_b[j] : nullptr, dw[j], hb ? db[j] : nullptr, kCD * kCD,
                         hb ? kCD : 0, a.splits};
  }
  chain_wgrad_kernel<<<dim3(static_cast<unsigned>(a.splits), static_cast<unsigned>(n_stages)), kCThreads, 0,
                       as_stream(stream)>>>(a);
  const int rc = last_launch_status();
  if (rc || (flags & X2G_DEFER_SLAB_SUM)) return rc;
  return x2g_slab_sum_batch(sj, n_stages, (flags & X2G_ACCUM_WGRAD) ? 1 : 0, stream);
}

static inline unsigned v2_grid(int64_t rows) {
  const int64_t nblk = (rows + 15) / 16;
  return static_cast<unsigned>(nblk < 256 ? nblk : 256);
}

// the projection kernels: one 512-thread workgroup per CU (two waves per SIMD at 256 VGPRs)
static inline unsigned proj_grid(int64_t rows) {
  const int64_t nblk = (rows + 15) / 16, cap = 256;
  return static_cast<unsigned>(nblk < cap ? nblk : cap);
}

X2G_API int x2g_conv_proj_fwd(const float* x, const float* rbf, int32_t rbf_dim, const float* w_rbf,
                              const x2g_proj* proj, int64_t rows, int32_t dim, float* x_t, float* xs_t, void* stream) {
  if (!proj || rows < 0 || dim <= 0 || rbf_dim <= 0) return X2G_EINVAL;
  if (dim != kCD || rbf_dim > kRbfMax || rows * kCD * 4 >= (int64_t(1) << 31)) return X2G_EUNSUPPORTED;
  if (rows == 0) return X2G_OK;
  if (!x || !rbf || !w_rbf) return X2G_EINVAL;
  ProjFwdArgs a{};
  a.x = x;
  a.rbf = rbf;
  a.wr = w_rbf;
  a.RR = rbf_dim;
  a.x_t = x_t;
  a.xs_t = xs_t;
  a.R = rows;
  for (int p = 0; p < 4; ++p) {
    if (!proj[p].w || !proj[p].out) return X2G_EINVAL;
    if (!al16(proj[p].w) || !al16(proj[p].b) || !al16(proj[p].out) || !al16(proj[p].wt)) return X2G_EUNSUPPORTED;
    a.p[p] = proj[p];
  }
  if (!al16(x) || !al16(x_t) || !al16(xs_t)) return X2G_EUNSUPPORTED;
  if (rbf_dim <= 6)
    conv_proj_fwd_kernel<6><<<proj_grid(rows), kCThreads, 0, as_stream(stream)>>>(a);
  else
    conv_proj_fwd_kernel<8><<<proj_grid(rows), kCThreads, 0, as_stream(stream)>>>(a);
  return last_launch_status();
}

X2G_API int32_t x2g_conv_proj_bwd_gate_splits(int64_t rows) { return rows > 0 ? static_cast<int32_t>(proj_grid(rows)) : 0; }

X2G_API size_t x2g_conv_proj_bwd_gate_workspace(int64_t rows, int32_t rbf_dim) {
  if (rows <= 0 || rbf_dim <= 0) return 0;
  return static_cast<size_t>(proj_grid(rows)) * kCD * rbf_dim * sizeof(float);
}

X2G_API int x2g_conv_proj_bwd_gate(const x2g_proj_grad* grads, int64_t rows, int32_t dim, const float* x,
                                   const float* rbf, int32_t rbf_dim, const float* w_rbf, float* dx,
                                   const float* dx_add, float* drbf, float* dw_rbf, int flags, void* ws, size_t wsb,
                                   void* stream) {
  if (!grads || rows < 0 || dim <= 0 || rbf_dim <= 0 || !dw_rbf) return X2G_EINVAL;
  if (flags & ~(X2G_ACCUM_WGRAD | X2G_DEFER_SLAB_SUM | X2G_GATE_DRBF_ACCUM)) return X2G_EINVAL;
  if (dim != kCD || rbf_dim > kRbfMax || rows * kCD * 4 >= (int64_t(1) << 31)) return X2G_EUNSUPPORTED;
  hipStream_t st = as_stream(stream);
  if (rows == 0) {
    if (flags & X2G_DEFER_SLAB_SUM) return X2G_EINVAL;
    if (flags & X2G_ACCUM_WGRAD) return X2G_OK;
    const hipError_t e = hipMemsetAsync(dw_rbf, 0, sizeof(float) * kCD * rbf_dim, st);
    return e == hipSuccess ? X2G_OK : static_cast<int>(e);
  }
  if (!dx || !x || !rbf || !w_rbf) return X2G_EINVAL;
  if (!ws || wsb < x2g_conv_proj_bwd_gate_workspace(rows, rbf_dim)) return X2G_EWORKSPACE;
  ProjBwdGateArgs a{};
  for (int p = 0; p < 4; ++p) {
    if (!grads[p].g || !grads[p].w) return X2G_EINVAL;
    if (!al16(grads[p].g) || !al16(grads[p].w) || !al16(grads[p].wt) || !al16(grads[p].g_t)) return X2G_EUNSUPPORTED;
    a.gr[p] = grads[p];
  }
  if (!al16(dx) || !al16(dx_add) || !al16(x)) return X2G_EUNSUPPORTED;
  a.dx_add = dx_add;
  a.dx = dx;
  a.x = x;
  a.rbf = rbf;
  a.wr = w_rbf;
  a.drbf = drbf;
  a.part_w = static_cast<float*>(ws);
  a.RR = rbf_dim;
  a.drbf_acc = (flags & X2G_GATE_DRBF_ACCUM) ? 1 : 0;
  a.R = rows;
  const unsigned grid = proj_grid(rows);
  const bool tw = grads[0].wt && grads[1].wt && grads[2].wt && grads[3].wt;
  if (rbf_dim <= 6) {
    if (tw)
      conv_proj_bwd_gate_kernel<6, true><<<grid, kCThreads, 0, st>>>(a);
    else
      conv_proj_bwd_gate_kernel<6, false><<<grid, kCThreads, 0, st>>>(a);
  } else if (tw) {
    conv_proj_bwd_gate_kernel<8, true><<<grid, kCThreads, 0, st>>>(a);
  } else {
    conv_proj_bwd_gate_kernel<8, false><<<grid, kCThreads, 0, st>>>(a);
  }
  const int rc = last_launch_status();
  if (rc || (flags & X2G_DEFER_SLAB_SUM)) return rc;
  x2g_slab_job sj{a.part_w, nullptr, dw_rbf, nullptr, static_cast<int64_t>(kCD) * rbf_dim, 0,
                  static_cast<int32_t>(grid), 0, 0};
  return x2g_slab_sum_batch(&sj, 1, (flags & X2G_ACCUM_WGRAD) ? 1 : 0, stream);
}

// ---- one launch for many jobs (x2g_tiled_wgrad_flat)
// two 512-thread workgroups per CU (66 KB of LDS and 100 VGPRs each: 4 waves per SIMD)
constexpr int kFlatWPC = 2;
static inline unsigned flat_grid(int64_t total) {
  const int64_t cap = 256 * kFlatWPC;
  return static_cast<unsigned>(total < cap ? (total < 1 ? 1 : total) : cap);
}

// slabs of job j (tiles [t0, t1) of the concatenation): the workgroups overlapping them
static inline void flat_span(int64_t t0, int64_t t1, int64_t total, int64_t G, int& lo, int& n) {
  // workgroup i covers [i * total / G, (i + 1) * total / G): the one holding tile t is the largest i
  // with i * total / G <= t
  auto owner = [&](int64_t t) {
    int64_t i = (t * G) / total;  // close; adjust for the integer floors
    while (i + 1 < G && (i + 1) * total / G <= t) ++i;
    while (i > 0 && i * total / G > t) --i;
    return static_cast<int>(i);
  };
  lo = owner(t0);
  n = owner(t1 - 1) - lo + 1;
}

// the concatenation's tile offsets of jobs with rows[j] rows each (0 on a bad row count)
static inline bool flat_tiles(const int64_t* rows, int num_jobs, int64_t* tile0) {
  tile0[0] = 0;
  for (int j = 0; j < num_jobs; ++j) {
    if (rows[j] <= 0 || rows[j] * kCD * 4 >= (int64_t(1) << 31)) return false;
    tile0[j + 1] = tile0[j] + (rows[j] + 15) / 16;
  }
  return true;
}

static size_t flat_workspace(const int64_t* rows, int32_t num_jobs, int32_t dim) {
  if (!rows || dim != kCD || num_jobs < 1 || num_jobs > X2G_TILED_MAX_JOBS) return 0;
  int64_t tile0[X2G_TILED_MAX_JOBS + 1];
  if (!flat_tiles(rows, num_jobs, tile0)) return 0;
  const int64_t total = tile0[num_jobs], G = flat_grid(total);
  int64_t slabs = 0;
  for (int j = 0; j < num_jobs; ++j) {
    int lo, n;
    flat_span(tile0[j], tile0[j + 1], total, G, lo, n);
    slabs += n;
  }
  return static_cast<size_t>(slabs) * (kCD * kCD + kCD) * sizeof(float);
}

static int flat_launch(const x2g_tiled_job* jobs, const int64_t* rows, int32_t num_jobs, int32_t dim, int flags,
                       x2g_slab_job* slab_jobs, void* workspace, size_t workspace_bytes, void* stream) {
  if (!jobs || !rows || num_jobs < 1 || num_jobs > X2G_TILED_MAX_JOBS || dim <= 0 ||
      (flags & ~(X2G_ACCUM_WGRAD | X2G_DEFER_SLAB_SUM)))
    return X2G_EINVAL;
  for (int j = 0; j < num_jobs; ++j)
    if (rows[j] <= 0) return X2G_EINVAL;
  if (dim != kCD) return X2G_EUNSUPPORTED;
  if ((flags & X2G_DEFER_SLAB_SUM) && !slab_jobs) return X2G_EINVAL;
  TiledFlatArgs a{};
  if (!flat_tiles(rows, num_jobs, a.tile0)) return X2G_EUNSUPPORTED;
  const size_t need = flat_workspace(rows, num_jobs, dim);
  if (!workspace || workspace_bytes < need) return X2G_EWORKSPACE;
  a.total = a.tile0[num_jobs];
  a.njobs = num_jobs;
  const int64_t G = flat_grid(a.total);
  x2g_slab_job sj[X2G_TILED_MAX_JOBS];
  float* base = static_cast<float*>(workspace);
  for (int j = 0; j < num_jobs; ++j) {
    const x2g_tiled_job& J = jobs[j];
    if (!J.dy_t || !J.x_t || !J.dw) return X2G_EINVAL;
    if (!al16(J.dy_t) || !al16(J.x_t)) return X2G_EUNSUPPORTED;
    if (J.ld < 0 || (J.ld > 0 && (J.cols < 1 || J.cols > kCD || J.cols > J.ld))) return X2G_EINVAL;
    int lo, n;
    flat_span(a.tile0[j], a.tile0[j + 1], a.total, G, lo, n);
    a.in_t[j] = J.x_t;
    a.dz_t[j] = J.dy_t;
    a.wg_lo[j] = lo;
    a.has_b[j] = J.db != nullptr;
    a.slab_w[j] = base;
    a.slab_b[j] = base + static_cast<int64_t>(n) * kCD * kCD;
    base += static_cast<int64_t>(n) * (kCD * kCD + kCD);
    sj[j] = x2g_slab_job{a.slab_w[j], J.db ? a.slab_b[j] : nullptr, J.dw, J.db, kCD * kCD, J.db ? kCD : 0, n,
                         J.ld, J.cols};
  }
  // two independent workgroups per CU, each with two 2-tile buffers: one workgroup's copy waits and
  // barriers run under the other's MFMAs (+1.4 % in the step A/B over one workgroup per CU with two
  // 4-tile buffers, which was +0.7 % over r2's one workgroup with four 2-tile buffers; three 3-tile
  // buffers: -0.3 %).  Twice the slabs (512 + jobs), summed by the deferred slab pass.
  tiled_flat_kernel<2, true, 2, kFlatWPC><<<static_cast<unsigned>(G), kCThreads, 0, as_stream(stream)>>>(a);
  const int rc = last_launch_status();
  if (rc) return rc;
  if (flags & X2G_DEFER_SLAB_SUM) {
    for (int j = 0; j < num_jobs; ++j) slab_jobs[j] = sj[j];
    return X2G_OK;
  }
  return x2g_slab_sum_batch(sj, num_jobs, (flags & X2G_ACCUM_WGRAD) ? 1 : 0, stream);
}

X2G_API size_t x2g_tiled_wgrad_flat_workspace(int64_t rows, int32_t dim, int32_t num_jobs) {
  if (rows <= 0 || num_jobs < 1 || num_jobs > X2G_TILED_MAX_JOBS) return 0;
  int64_t r[X2G_TILED_MAX_JOBS];
  for (int j = 0; j < num_jobs; ++j) r[j] = rows;
  return flat_workspace(r, num_jobs, dim);
}

X2G_API int x2g_tiled_wgrad_flat(const x2g_tiled_job* jobs, int32_t num_jobs, int64_t rows, int32_t dim, int flags,
                                 x2g_slab_job* slab_jobs, void* workspace, size_t workspace_bytes, void* stream) {
  if (rows <= 0 || num_jobs < 1 || num_jobs > X2G_TILED_MAX_JOBS) return X2G_EINVAL;
  int64_t r[X2G_TILED_MAX_JOBS];
  for (int j = 0; j < num_jobs; ++j) r[j] = rows;
  return flat_launch(jobs, r, num_jobs, dim, flags, slab_jobs, workspace, workspace_bytes, stream);
}

X2G_API size_t x2g_tiled_wgrad_flat_rows_workspace(const int64_t* job_rows, int32_t num_jobs, int32_t dim) {
  return flat_workspace(job_rows, num_jobs, dim);
}

X2G_API int x2g_tiled_wgrad_flat_rows(const x2g_tiled_job* jobs, const int64_t* job_rows, int32_t num_jobs,
                                      int32_t dim, int flags, x2g_slab_job* slab_jobs, void* workspace,
                                      size_t workspace_bytes, void* stream) {
  return flat_launch(jobs, job_rows, num_jobs, dim, flags, slab_jobs, workspace, workspace_bytes, stream);
}

X2G_API size_t x2g_tiled_wgrad_workspace(int64_t rows, int32_t dim, int32_t num_jobs) {
  return x2g_chain_wgrad_workspace(rows, dim, num_jobs);
}

X2G_API int x2g_tiled_wgrad(const x2g_tiled_job* jobs, int32_t num_jobs, int64_t rows, int32_t dim, int flags,
                            void* workspace, size_t workspace_bytes, void* stream) {
  if (!jobs || num_jobs < 1 || num_jobs > X2G_CHAIN_MAX_STAGES || rows <= 0 || dim <= 0 ||
      (flags & ~(X2G_ACCUM_WGRAD | X2G_DEFER_SLAB_SUM)))
    return X2G_EINVAL;
  if (dim != kCD || rows * kCD * 4 >= (int64_t(1) << 31)) return X2G_EUNSUPPORTED;
  const size_t need = x2g_tiled_wgrad_workspace(rows, dim, num_jobs);
  if (!workspace || workspace_bytes < need) return X2G_EWORKSPACE;
  ChainWgradArgs a{};
  a.ntiles = (rows + 15) / 16;
  a.splits = chain_wgrad_splits(rows, dim, num_jobs);
  const size_t per = need / num_jobs;
  x2g_slab_job sj[X2G_CHAIN_MAX_STAGES];
  for (int j = 0; j < num_jobs; ++j) {
    const x2g_tiled_job& J = jobs[j];
    if (!J.dy_t || !J.x_t || !J.dw) return X2G_EINVAL;
    if (!al16(J.dy_t) || !al16(J.x_t)) return X2G_EUNSUPPORTED;
    a.in_t[j] = J.x_t;
    a.dz_t[j] = J.dy_t;
    a.part_w[j] = reinterpret_cast<float*>(static_cast<char*>(workspace) + per * j);
    a.part_b[j] = a.part_w[j] + static_cast<int64_t>(a.splits) * kCD * kCD;
    a.has_b[j] = J.db != nullptr;
    if (J.ld < 0 || (J.ld > 0 && (J.cols < 1 || J.cols > kCD || J.cols > J.ld))) return X2G_EINVAL;
    sj[j] = x2g_slab_job{a.part_w[j], J.db ? a.part_b[j] : nullptr, J.dw, J.db, kCD * kCD, J.db ? kCD : 0,
                         a.splits, J.ld, J.cols};
  }
  chain_wgrad_kernel<<<dim3(static_cast<unsigned>(a.splits), static_cast<unsigned>(num_jobs)), kCThreads, 0,
                       as_stream(stream)>>>(a);
  const int rc = last_launch_status();
  if (rc || (flags & X2G_DEFER_SLAB_SUM)) return rc;
  return x2g_slab_sum_batch(sj, num_jobs, (flags & X2G_ACCUM_WGRAD) ? 1 : 0, stream);
}
