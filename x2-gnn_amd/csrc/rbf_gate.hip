// rbf gates: x * lin_rbf(rbf) without the [E, D] filter tensor.
//
// SBFTransformerConv scales its source features by a filter of the 6-wide radial basis
// (x_src = x * lin_rbf(rbf), sbftransformer_conv.py:99-101) and both readouts pool
// lin_rbf(rbf) * x from edges to atoms (readout.py:39-41,66-67).  As torch ops that is a
// K = 6 GEMM writing an [E, D] filter, an elementwise product (or a segment sum with a multiply)
// reading it back, and in the backward two more elementwise products plus the K = 6 weight /
// input gradients.  Here the filter row is recomputed in registers from the row's R <= 8 basis
// values (each lane owns 4 channels and their 4 x R weights), so a gate is one streaming pass:
//   forward: read x and rbf, write out (gate) or the segment sums (pool);
//   backward: read g (per row, or per owning segment for the pool), x and rbf; write dx and
//             drbf; dW / db partials per workgroup, summed in a fixed order (deterministic).
#include "common.hpp"

namespace x2g {

constexpr int kGateRMax = 8;
// workgroups per job of the pool / gate backward: 128 (about 165 rows each at config 2) amortise each
// workgroup's weight staging, LDS reduction and slab over 4x the rows of r2's 512 and leave a quarter
// of the slabs to sum (+0.45 % in the step A/B, profiles/r3e_ab_small_kernels.log)
constexpr int kGateBwdSplits = 128;

typedef float f4v __attribute__((ext_vector_type(4)));

// W [D, R] and b [D] staged once per workgroup with coalesced loads (reading them per lane
// straight from global memory is a 24-byte-strided gather per lane and per weight: at one
// row per lane that gather, not HBM, bounded the kernel)
template <int D>
__device__ __forceinline__ void stage_gate_weights(const float* __restrict__ W, const float* __restrict__ B, int R,
                                                   float* __restrict__ sw) {
  for (int i = threadIdx.x; i < D * R; i += blockDim.x) sw[i] = W[i];
  for (int i = threadIdx.x; i < D; i += blockDim.x) sw[D * kGateRMax + i] = B ? B[i] : 0.f;
  __syncthreads();
}

template <int LPR>
struct GateW {  // the lane's 4 channels: w[c][j] (zero beyond R) and b[c]
  float w[4][kGateRMax];
  float b[4];
  __device__ __forceinline__ void load(const float* __restrict__ sw, int R, int sub) {
    constexpr int D = 4 * LPR;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = 4 * sub + i;
#pragma unroll
      for (int j = 0; j < kGateRMax; ++j) w[i][j] = j < R ? sw[c * R + j] : 0.f;
      b[i] = sw[D * kGateRMax + c];
    }
  }
  __device__ __forceinline__ f4v filter(const float (&rb)[kGateRMax]) const {
    f4v f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float a = b[i];
#pragma unroll
      for (int j = 0; j < kGateRMax; ++j) a = fmaf(w[i][j], rb[j], a);
      f[i] = a;
    }
    return f;
  }
};

// the row's basis values (a clamped index beyond R: those weights are zero)
__device__ __forceinline__ void load_rbf(const float* __restrict__ rbf, int64_t r, int R, float (&rb)[kGateRMax]) {
#pragma unroll
  for (int j = 0; j < kGateRMax; ++j) rb[j] = rbf[r * R + (j < R ? j : R - 1)];
}

template <int LPR>
__global__ void __launch_bounds__(256) rbf_gate_fwd_kernel(const f4v* __restrict__ x, const float* __restrict__ rbf,
                                                           const float* __restrict__ W, const float* __restrict__ B,
                                                           int64_t rows, int R, f4v* __restrict__ out) {
  constexpr int RPB = 256 / LPR;
  constexpr int UNROLL = 4;
  __shared__ float sw[4 * LPR * (kGateRMax + 1)];
  stage_gate_weights<4 * LPR>(W, B, R, sw);
  const int sub = threadIdx.x % LPR, slot = threadIdx.x / LPR;
  GateW<LPR> gw;
  gw.load(sw, R, sub);
  const int64_t stride = static_cast<int64_t>(gridDim.x) * RPB * UNROLL;
  for (int64_t r0 = static_cast<int64_t>(blockIdx.x) * RPB * UNROLL + slot; r0 < rows; r0 += stride) {
    float rb[UNROLL][kGateRMax];
    f4v xv[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const int64_t r = r0 + u * RPB, rc = r < rows ? r : rows - 1;
      load_rbf(rbf, rc, R, rb[u]);
      xv[u] = x[rc * LPR + sub];
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const int64_t r = r0 + u * RPB;
      if (r < rows) out[r * LPR + sub] = xv[u] * gw.filter(rb[u]);
    }
  }
}

// pool: one wave per segment, 64 / LPR rows per load, 8 loads in flight per lane (a QM9 atom's
// ~9 edges are one round trip)
// up to kGateMaxJobs pools over the same rows / segments / basis in one launch: job blockIdx.y
constexpr int kGateMaxJobs = X2G_GATE_MAX_JOBS;
struct PoolJobs {
  const f4v* x[kGateMaxJobs];
  const float* w[kGateMaxJobs];
  const float* b[kGateMaxJobs];
  f4v* out[kGateMaxJobs];
};

template <int LPR>
__global__ void __launch_bounds__(256) rbf_pool_fwd_kernel(const PoolJobs J, const float* __restrict__ rbf,
                                                           const int32_t* __restrict__ rowptr, int64_t G, int R) {
  constexpr int RPI = 64 / LPR;
  constexpr int UNROLL = 8;
  __shared__ float sw[4 * LPR * (kGateRMax + 1)];
  const int job = blockIdx.y;
  const f4v* __restrict__ x = J.x[job];
  f4v* __restrict__ out = J.out[job];
  stage_gate_weights<4 * LPR>(J.w[job], J.b[job], R, sw);
  const int lane = threadIdx.x & 63;
  const int sub = lane % LPR, slot = lane / LPR;
  GateW<LPR> gw;
  gw.load(sw, R, sub);
  const int nwaves = gridDim.x * 4;
  // a row's basis values: lane j of each 16-lane DPP row (LPR >= 16, so a data row spans whole DPP
  // rows) loads value j and row_newbcast hands value j to the row — one load and one register per row
  // slot instead of kGateRMax of each (occupancy 4 -> 8 waves per SIMD)
  const int jl = (lane & 15) < R ? (lane & 15) : R - 1;
  for (int64_t g = uniform(blockIdx.x * 4 + (threadIdx.x >> 6)); g < G; g += nwaves) {
    const int r0 = uniform(rowptr[g]), r1 = uniform(rowptr[g + 1]);
    f4v acc = {0.f, 0.f, 0.f, 0.f};
    for (int rb0 = r0; rb0 < r1; rb0 += UNROLL * RPI) {
      f4v v[UNROLL];
      float rv[UNROLL];
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) {
        const int r = rb0 + u * RPI + slot;
        const int rc = r < r1 ? r : r1 - 1;
        v[u] = x[static_cast<int64_t>(rc) * LPR + sub];
        rv[u] = rbf[static_cast<int64_t>(rc) * R + jl];
      }
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) {
        const float ok = rb0 + u * RPI + slot < r1 ? 1.f : 0.f;
        float rb[kGateRMax];
        rb[0] = dpp_mov<0x150>(rv[u]);
        rb[1] = dpp_mov<0x151>(rv[u]);
        rb[2] = dpp_mov<0x152>(rv[u]);
        rb[3] = dpp_mov<0x153>(rv[u]);
        rb[4] = dpp_mov<0x154>(rv[u]);
        rb[5] = dpp_mov<0x155>(rv[u]);
        rb[6] = dpp_mov<0x156>(rv[u]);
        rb[7] = dpp_mov<0x157>(rv[u]);
        acc += (v[u] * gw.filter(rb)) * ok;
      }
    }
#pragma unroll
    for (int off = LPR; off < 64; off <<= 1) {
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i] += __shfl_xor(acc[i], off, kWave);
    }
    if (slot == 0) out[g * LPR + sub] = acc;
  }
}

// Sum of 8 per-lane values over an aligned group of LPR lanes (LPR in 16..64), as a butterfly
// that halves the vector at each of the top three levels (4 + 2 + 1 exchanges instead of 8 x 3),
// then plain sums over the remaining lane bits (partners per xor_xchg: DPP below 16 lanes, so for
// LPR = 32 only the first level goes through LDS): lane `sub` ends with the group total of
// element j = 4 [sub & LPR/2] + 2 [sub & LPR/4] + [sub & LPR/8] (returned in j).
template <int LPR>
__device__ __forceinline__ float transpose_sum(const float (&p)[kGateRMax], int sub, int& j) {
  constexpr int o1 = LPR / 2, o2 = LPR / 4, o3 = LPR / 8;
  const bool h1 = sub & o1, h2 = sub & o2, h3 = sub & o3;
  float q[4], r[2];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float send = h1 ? p[k] : p[k + 4];
    const float recv = xor_xchg<o1>(send);
    q[k] = (h1 ? p[k + 4] : p[k]) + recv;
  }
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const float send = h2 ? q[k] : q[k + 2];
    const float recv = xor_xchg<o2>(send);
    r[k] = (h2 ? q[k + 2] : q[k]) + recv;
  }
  float t;
  {
    const float send = h3 ? r[0] : r[1];
    const float recv = xor_xchg<o3>(send);
    t = (h3 ? r[1] : r[0]) + recv;
  }
  if constexpr (o3 >= 8) t += xor_xchg<4>(t);
  if constexpr (o3 >= 4) t += xor_xchg<2>(t);
  if constexpr (o3 >= 2) t += xor_xchg<1>(t);
  j = 4 * h1 + 2 * h2 + h3;
  return t;
}

// backward: block b owns rows [b * per, (b + 1) * per); slot s of the block takes every RPB-th
// row; partial dW / db per block through LDS (fixed order over slots)
// backward jobs: job blockIdx.y (drbf: the job's own buffer; a batch gives each job a partial)
struct GateBwdJobs {
  const f4v* g[kGateMaxJobs];
  const f4v* x[kGateMaxJobs];
  const float* w[kGateMaxJobs];
  const float* b[kGateMaxJobs];
  f4v* dx[kGateMaxJobs];
  const f4v* dx_add[kGateMaxJobs];
  float* drbf[kGateMaxJobs];
  float* part_w[kGateMaxJobs];
  float* part_b[kGateMaxJobs];
};

template <int LPR>
__global__ void __launch_bounds__(256) rbf_gate_bwd_kernel(const GateBwdJobs J, const int32_t* __restrict__ owner,
                                                           const float* __restrict__ rbf, int64_t rows, int R,
                                                           int drbf_acc) {
  constexpr int RPB = 256 / LPR;
  constexpr int D = 4 * LPR;
  __shared__ float red[RPB * D * (kGateRMax + 1)];
  __shared__ float sw[D * (kGateRMax + 1)];
  const int job = blockIdx.y;
  const f4v* __restrict__ g = J.g[job];
  const f4v* __restrict__ x = J.x[job];
  f4v* __restrict__ dx = J.dx[job];
  const f4v* __restrict__ dx_add = J.dx_add[job];
  float* __restrict__ drbf = J.drbf[job];
  float* __restrict__ part_w = J.part_w[job];
  float* __restrict__ part_b = J.part_b[job];
  stage_gate_weights<D>(J.w[job], J.b[job], R, sw);
  const int sub = threadIdx.x % LPR, slot = threadIdx.x / LPR;
  GateW<LPR> gw;
  gw.load(sw, R, sub);
  float aw[4][kGateRMax], ab[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    ab[i] = 0.f;
#pragma unroll
    for (int j = 0; j < kGateRMax; ++j) aw[i][j] = 0.f;
  }
  constexpr int UNROLL = 3;
  // the drbf element this lane writes (transpose_sum's j); its old value is loaded with the rows
  const int jd = 4 * ((sub & (LPR / 2)) != 0) + 2 * ((sub & (LPR / 4)) != 0) + ((sub & (LPR / 8)) != 0);
  const bool acc_drbf = drbf && drbf_acc && jd < R;
  const int64_t per = (rows + gridDim.x - 1) / gridDim.x;
  const int64_t lo = per * blockIdx.x, hi = lo + per < rows ? lo + per : rows;
  // a row's basis values: lane j of each 16-lane DPP row loads value j (a data row spans whole DPP
  // rows, LPR >= 16) and row_newbcast hands value j to the row's lanes — one load per row, not R
  const int jl = (threadIdx.x & 15) < R ? (threadIdx.x & 15) : R - 1;
  // the optional operands (owner, the accumulated drbf, dx_add) through descriptors that are empty when
  // absent: every load is unconditional (a lane that must not read goes out of range and gets zero),
  // so no branch merges two wait histories into a vmcnt(0) between the owner load and its gather
  auto desc = [](const void* p, int64_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), static_cast<short>(0),
                                             static_cast<int>(bytes < 0x7fffffff ? bytes : 0x7fffffff), 0x00020000);
  };
  const __amdgpu_buffer_rsrc_t own_r = desc(owner, owner ? rows * 4 : 0);
  const __amdgpu_buffer_rsrc_t od_r = desc(drbf, (drbf && drbf_acc) ? rows * R * 4 : 0);
  const __amdgpu_buffer_rsrc_t add_r = desc(dx_add, dx_add ? rows * LPR * 16 : 0);
  const bool has_owner = owner != nullptr;
  for (int64_t r0 = lo + slot; r0 < hi; r0 += RPB * UNROLL) {
    float rv[UNROLL];
    f4v gv[UNROLL], xv[UNROLL], av[UNROLL];
    float od[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {  // every load of the UNROLL rows first
      const int64_t r = r0 + u * RPB, rc = r < hi ? r : hi - 1;
      rv[u] = rbf[rc * R + jl];
      od[u] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                            od_r, acc_drbf ? static_cast<int>((rc * R + jd) * 4) : 0x7ffffff0, 0, 0));
      const int ow = static_cast<int>(__builtin_amdgcn_raw_buffer_load_b32(own_r, static_cast<int>(rc * 4), 0, 0));
      const int64_t o = has_owner ? ow : rc;
      gv[u] = g[o * LPR + sub];
      xv[u] = x[rc * LPR + sub];
      av[u] = __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(
                                         add_r, static_cast<int>((rc * LPR + sub) * 16), 0, 0));
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const int64_t r = r0 + u * RPB;
      const bool ok = r < hi;
      const float m = ok ? 1.f : 0.f;
      float rb[kGateRMax];
      rb[0] = dpp_mov<0x150>(rv[u]);
      rb[1] = dpp_mov<0x151>(rv[u]);
      rb[2] = dpp_mov<0x152>(rv[u]);
      rb[3] = dpp_mov<0x153>(rv[u]);
      rb[4] = dpp_mov<0x154>(rv[u]);
      rb[5] = dpp_mov<0x155>(rv[u]);
      rb[6] = dpp_mov<0x156>(rv[u]);
      rb[7] = dpp_mov<0x157>(rv[u]);
      if (dx && ok) {
        f4v d = gv[u] * gw.filter(rb);
        if (dx_add) d += av[u];
        dx[r * LPR + sub] = d;
      }
      const f4v df = gv[u] * xv[u] * m;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        ab[i] += df[i];
#pragma unroll
        for (int j = 0; j < kGateRMax; ++j) aw[i][j] = fmaf(df[i], rb[j], aw[i][j]);
      }
      if (drbf) {
        float p[kGateRMax];
#pragma unroll
        for (int j = 0; j < kGateRMax; ++j) {
          float a = 0.f;
#pragma unroll
          for (int i = 0; i < 4; ++i) a = fmaf(df[i], gw.w[i][j], a);
          p[j] = a;
        }
        int j;
        const float tot = transpose_sum<LPR>(p, sub, j);
        if ((sub & (LPR / 8 - 1)) == 0 && ok && j < R) drbf[r * R + j] = tot + od[u];  // od = 0 unless accumulating
      }
    }
  }
  // slot-major partials: red[slot][c * R + j] (weights) and red[slot][D * R + c] (bias)
  const int per_slot = D * (R + 1);
  float* mine = red + slot * per_slot;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = 4 * sub + i;
    for (int j = 0; j < R; ++j) mine[c * R + j] = aw[i][j];
    mine[D * R + c] = ab[i];
  }
  __syncthreads();
  for (int idx = threadIdx.x; idx < per_slot; idx += 256) {
    float s = 0.f;
    for (int sl = 0; sl < RPB; ++sl) s += red[sl * per_slot + idx];
    if (idx < D * R)
      part_w[static_cast<int64_t>(blockIdx.x) * D * R + idx] = s;
    else if (part_b)
      part_b[static_cast<int64_t>(blockIdx.x) * D + idx - D * R] = s;
  }
}

inline bool gate_shape_ok(int D, int R) { return R >= 1 && R <= kGateRMax && (D == 64 || D == 128 || D == 256); }

inline int gate_bwd_splits(int64_t rows) {
  const int64_t want = (rows + 7) / 8;  // >= 8 rows per workgroup: one or two per slot
  return static_cast<int>(want < kGateBwdSplits ? (want < 1 ? 1 : want) : kGateBwdSplits);
}

}  // namespace x2g

using namespace x2g;

static inline bool al16(const void* p) { return reinterpret_cast<uintptr_t>(p) % 16 == 0; }

X2G_API int x2g_rbf_gate_fwd(const float* x, const float* rbf, const float* w, const float* b, int64_t rows, int32_t D,
                             int32_t R, float* out, void* stream) {
  if (rows < 0 || !gate_shape_ok(D, R)) return rows < 0 ? X2G_EINVAL : X2G_EUNSUPPORTED;
  if (rows == 0) return X2G_OK;
  if (!x || !rbf || !w || !out) return X2G_EINVAL;
  if (!al16(x) || !al16(out)) return X2G_EINVAL;
  const auto* xv = reinterpret_cast<const f4v*>(x);
  auto* ov = reinterpret_cast<f4v*>(out);
  const int64_t want = (rows * D / 4 + 1023) / 1024;  // 4 rows per lane
  const unsigned grid = static_cast<unsigned>(want < 2048 ? want : 2048);
  hipStream_t st = as_stream(stream);
  switch (D) {
    case 64: rbf_gate_fwd_kernel<16><<<grid, 256, 0, st>>>(xv, rbf, w, b, rows, R, ov); break;
    case 128: rbf_gate_fwd_kernel<32><<<grid, 256, 0, st>>>(xv, rbf, w, b, rows, R, ov); break;
    default: rbf_gate_fwd_kernel<64><<<grid, 256, 0, st>>>(xv, rbf, w, b, rows, R, ov); break;
  }
  return last_launch_status();
}

static int pool_launch(const PoolJobs& J, int n_jobs, const float* rbf, const int32_t* rowptr, int64_t G, int D, int R,
                       hipStream_t st) {
  const int64_t want = (G + 3) / 4;
  const dim3 grid(static_cast<unsigned>(want < 2048 ? want : 2048), static_cast<unsigned>(n_jobs));
  switch (D) {
    case 64: rbf_pool_fwd_kernel<16><<<grid, 256, 0, st>>>(J, rbf, rowptr, G, R); break;
    case 128: rbf_pool_fwd_kernel<32><<<grid, 256, 0, st>>>(J, rbf, rowptr, G, R); break;
    default: rbf_pool_fwd_kernel<64><<<grid, 256, 0, st>>>(J, rbf, rowptr, G, R); break;
  }
  return last_launch_status();
}

X2G_API int x2g_rbf_pool_fwd(const float* x, const float* rbf, const float* w, const float* b, const int32_t* rowptr,
                             int64_t G, int32_t D, int32_t R, float* out, void* stream) {
  if (G < 0 || !gate_shape_ok(D, R)) return G < 0 ? X2G_EINVAL : X2G_EUNSUPPORTED;
  if (G == 0) return X2G_OK;
  if (!x || !rbf || !w || !rowptr || !out) return X2G_EINVAL;
  if (!al16(x) || !al16(out)) return X2G_EINVAL;
  PoolJobs J{};
  J.x[0] = reinterpret_cast<const f4v*>(x);
  J.w[0] = w;
  J.b[0] = b;
  J.out[0] = reinterpret_cast<f4v*>(out);
  return pool_launch(J, 1, rbf, rowptr, G, D, R, as_stream(stream));
}

X2G_API int x2g_rbf_pool_fwd_batch(const x2g_gate_job* jobs, int32_t n_jobs, const float* rbf, const int32_t* rowptr,
                                   int64_t G, int32_t D, int32_t R, void* stream) {
  if (!jobs || n_jobs < 1 || n_jobs > kGateMaxJobs || G < 0) return X2G_EINVAL;
  if (!gate_shape_ok(D, R)) return X2G_EUNSUPPORTED;
  if (G == 0) return X2G_OK;
  if (!rbf || !rowptr) return X2G_EINVAL;
  PoolJobs J{};
  for (int j = 0; j < n_jobs; ++j) {
    const x2g_gate_job& q = jobs[j];
    if (!q.x || !q.w || !q.out) return X2G_EINVAL;
    if (!al16(q.x) || !al16(q.out)) return X2G_EINVAL;
    J.x[j] = reinterpret_cast<const f4v*>(q.x);
    J.w[j] = q.w;
    J.b[j] = q.b;
    J.out[j] = reinterpret_cast<f4v*>(q.out);
  }
  return pool_launch(J, n_jobs, rbf, rowptr, G, D, R, as_stream(stream));
}

static int gate_bwd_launch(const GateBwdJobs& J, int n_jobs, const int32_t* owner, const float* rbf, int64_t rows,
                           int D, int R, int drbf_acc, int splits, hipStream_t st) {
  // the optional operands go through 32-bit buffer offsets, so each one PRESENT bounds the rows (an
  // absent one's descriptor is empty: every offset reads zero); g, x, dx, drbf use 64-bit pointers
  constexpr int64_t kLim = int64_t(1) << 31;
  bool add = false;
  for (int j = 0; j < n_jobs; ++j) add = add || J.dx_add[j] != nullptr;
  if ((owner && rows * 4 >= kLim) || (drbf_acc && rows * static_cast<int64_t>(R) * 4 >= kLim) ||
      (add && rows * static_cast<int64_t>(D) * 4 >= kLim))
    return X2G_EUNSUPPORTED;
  const dim3 grid(static_cast<unsigned>(splits), static_cast<unsigned>(n_jobs));
  switch (D) {
    case 64: rbf_gate_bwd_kernel<16><<<grid, 256, 0, st>>>(J, owner, rbf, rows, R, drbf_acc); break;
    case 128: rbf_gate_bwd_kernel<32><<<grid, 256, 0, st>>>(J, owner, rbf, rows, R, drbf_acc); break;
    default: rbf_gate_bwd_kernel<64><<<grid, 256, 0, st>>>(J, owner, rbf, rows, R, drbf_acc); break;
  }
  return last_launch_status();
}

X2G_API int32_t x2g_rbf_gate_bwd_splits(int64_t rows) { return rows > 0 ? gate_bwd_splits(rows) : 0; }

X2G_API size_t x2g_rbf_gate_bwd_workspace(int64_t rows, int32_t D, int32_t R) {
  if (rows <= 0 || D <= 0 || R <= 0) return 0;
  return static_cast<size_t>(gate_bwd_splits(rows)) * D * (R + 1) * sizeof(float);
}

X2G_API int x2g_rbf_gate_bwd(const float* g, const int32_t* owner, const float* x, const float* rbf, const float* w,
                             const float* b, int64_t rows, int32_t D, int32_t R, float* dx, const float* dx_add,
                             float* drbf, float* dw, float* db, int flags, void* ws, size_t wsb, void* stream) {
  if (rows < 0 || !dw) return X2G_EINVAL;
  if (!gate_shape_ok(D, R)) return X2G_EUNSUPPORTED;
  if (dx_add && !dx) return X2G_EINVAL;
  if (flags & ~(X2G_ACCUM_WGRAD | X2G_DEFER_SLAB_SUM | X2G_GATE_DRBF_ACCUM)) return X2G_EINVAL;
  const bool accum = flags & X2G_ACCUM_WGRAD;
  const int drbf_acc = (flags & X2G_GATE_DRBF_ACCUM) ? 1 : 0;
  hipStream_t st = as_stream(stream);
  if (rows == 0) {
    if (flags & X2G_DEFER_SLAB_SUM) return X2G_EINVAL;
    if (accum) return X2G_OK;
    hipError_t e = hipMemsetAsync(dw, 0, sizeof(float) * D * R, st);
    if (e == hipSuccess && db) e = hipMemsetAsync(db, 0, sizeof(float) * D, st);
    return e == hipSuccess ? X2G_OK : static_cast<int>(e);
  }
  if (!g || !x || !rbf || !w) return X2G_EINVAL;
  if (!al16(g) || !al16(x) || (dx && !al16(dx)) || (dx_add && !al16(dx_add))) return X2G_EINVAL;
  if (!ws || wsb < x2g_rbf_gate_bwd_workspace(rows, D, R)) return X2G_EWORKSPACE;
  const int splits = gate_bwd_splits(rows);
  GateBwdJobs J{};
  J.g[0] = reinterpret_cast<const f4v*>(g);
  J.x[0] = reinterpret_cast<const f4v*>(x);
  J.w[0] = w;
  J.b[0] = b;
  J.dx[0] = reinterpret_cast<f4v*>(dx);
  J.dx_add[0] = reinterpret_cast<const f4v*>(dx_add);
  J.drbf[0] = drbf;
  J.part_w[0] = static_cast<float*>(ws);
  J.part_b[0] = db ? J.part_w[0] + static_cast<int64_t>(splits) * D * R : nullptr;
  if (int rc = gate_bwd_launch(J, 1, owner, rbf, rows, D, R, drbf_acc, splits, st)) return rc;
  if (flags & X2G_DEFER_SLAB_SUM) return X2G_OK;
  return sum_slabs_launch(J.part_w[0], static_cast<int64_t>(D) * R, J.part_b[0], D, splits, dw, db, accum, st);
}

X2G_API size_t x2g_rbf_gate_bwd_batch_workspace(int64_t rows, int32_t D, int32_t R, int32_t n_jobs) {
  if (rows <= 0 || D <= 0 || R <= 0 || n_jobs < 1) return 0;
  return static_cast<size_t>(n_jobs) * (static_cast<size_t>(gate_bwd_splits(rows)) * D * (R + 1) + rows * R) *
         sizeof(float);
}

X2G_API int x2g_rbf_gate_bwd_batch(const x2g_gate_job* jobs, int32_t n_jobs, const int32_t* owner, const float* rbf,
                                   int64_t rows, int32_t D, int32_t R, float* drbf, int flags,
                                   x2g_slab_job* slab_jobs, void* ws, size_t wsb, void* stream) {
  if (!jobs || n_jobs < 1 || n_jobs > kGateMaxJobs || rows <= 0) return X2G_EINVAL;
  if (!gate_shape_ok(D, R)) return X2G_EUNSUPPORTED;
  if (flags & ~(X2G_ACCUM_WGRAD | X2G_DEFER_SLAB_SUM | X2G_GATE_DRBF_ACCUM)) return X2G_EINVAL;
  if ((flags & X2G_DEFER_SLAB_SUM) && !slab_jobs) return X2G_EINVAL;
  if (!rbf) return X2G_EINVAL;
  if (!ws || wsb < x2g_rbf_gate_bwd_batch_workspace(rows, D, R, n_jobs)) return X2G_EWORKSPACE;
  hipStream_t st = as_stream(stream);
  const int splits = gate_bwd_splits(rows);
  const int64_t per_w = static_cast<int64_t>(splits) * D * R, per_b = static_cast<int64_t>(splits) * D;
  float* base = static_cast<float*>(ws);
  float* scratch = base + n_jobs * (per_w + per_b);  // per-job drbf partials [n_jobs][rows][R]
  GateBwdJobs J{};
  x2g_slab_job sj[kGateMaxJobs];
  for (int j = 0; j < n_jobs; ++j) {
    const x2g_gate_job& q = jobs[j];
    if (!q.g || !q.x || !q.w || !q.dw || (q.dx_add && !q.dx)) return X2G_EINVAL;
    if (!al16(q.g) || !al16(q.x) || (q.dx && !al16(q.dx)) || (q.dx_add && !al16(q.dx_add))) return X2G_EINVAL;
    J.g[j] = reinterpret_cast<const f4v*>(q.g);
    J.x[j] = reinterpret_cast<const f4v*>(q.x);
    J.w[j] = q.w;
    J.b[j] = q.b;
    J.dx[j] = reinterpret_cast<f4v*>(q.dx);
    J.dx_add[j] = reinterpret_cast<const f4v*>(q.dx_add);
    J.drbf[j] = drbf ? scratch + static_cast<int64_t>(j) * rows * R : nullptr;
    J.part_w[j] = base + j * per_w;
    J.part_b[j] = q.db ? base + n_jobs * per_w + j * per_b : nullptr;
    sj[j] = x2g_slab_job{J.part_w[j], J.part_b[j], q.dw, q.db, static_cast<int64_t>(D) * R, q.db ? D : 0, splits, 0,
                         0};
  }
  if (int rc = gate_bwd_launch(J, n_jobs, owner, rbf, rows, D, R, 0, splits, st)) return rc;
  if (drbf) {  // the jobs' basis gradients summed in job order (+ the old value)
    const bool acc = flags & X2G_GATE_DRBF_ACCUM;
    if (int rc = sum_slabs_launch(scratch, rows * R, nullptr, 0, n_jobs, drbf, nullptr, acc, st)) return rc;
  }
  if (flags & X2G_DEFER_SLAB_SUM) {
    for (int j = 0; j < n_jobs; ++j) slab_jobs[j] = sj[j];
    return X2G_OK;
  }
  return x2g_slab_sum_batch(sj, n_jobs, (flags & X2G_ACCUM_WGRAD) ? 1 : 0, stream);
}
