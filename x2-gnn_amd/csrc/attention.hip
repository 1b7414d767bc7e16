// Fused SBF-transformer attention over the line graph (the hot loop of X2-GNN).
//
// Reference: SBFTransformerConv (sbftransformer_conv.py:93-162) through PyG 2.1's
// MessagePassing.propagate: q_i = q[edge_index[1]], k_j/v_j = k/v[edge_index[0]] lifted to
// [T,H,C] by index_select, the per-triplet message, torch_geometric.utils.softmax over each
// destination, torch_scatter 'add' aggregation to [E,H,C], + lin_skip(x).  The reference
// materialises ~10 [T,128] fp32 tensors per layer for this; here nothing T x 128 is written in
// the forward.
//
// Layout: triplets are CSR by destination (trip_rowptr / trip_src, the order vertex_to_edge_2
// produces).  One 64-lane wave owns one destination line node at a time and walks its
// triplets in order (deterministic); each lane owns CPL consecutive channels, so a head of C
// channels spans LPH = C/CPL lanes and the q.k dot product is a LPH-lane xor-shuffle reduction.
// The neighbour rows k[src], v[src] are read as one coalesced 512 B row per wave (D=128), the
// 42-float sbf row of the triplet is wave-uniform (scalar loads), and the lin_sbf weight lives
// in registers (S=42 floats per channel), so the [T,42]x[42,128] projection is computed on the
// fly instead of being materialised.  Softmax is the online (running max / rescale) form; the
// per-(destination, head) max and denominator are saved for the backward.
//
// Backward is two passes with no float atomics:
//  * destination-major (bwd_dst): dq, the edge-term gradient, the softmax-logit gradient
//    dlogit[T,H], and d_sbfproj[T,HC] (for dW_sbf = d_sbfproj^T sbf);
//  * source-major (bwd_src) over the transposed triplet lists: dk and dv, each a fixed-order
//    segmented sum (the adjoint of the k_j / v_j gathers).
#include <type_traits>
#include <math.h>

#include "common.hpp"

namespace x2g {

constexpr int kS = 42;           // sbf_dim compiled in (7 spherical x 6 radial)
constexpr int kSph = 7;
constexpr int kAttnWaves = 4;    // waves per 256-thread block
// persistent-ish grid: waves grid-stride over line nodes (round 4 A/B of 1024 / 2048 / 4096 / 8192: 2048)
constexpr int kMaxBlocks = 2048;
constexpr float kSoftmaxEps = 1e-16f;

struct AttnArgs {
  const float* q;
  const float* k;
  const float* v;
  const float* skip;
  const float* edge;
  const int32_t* edge_row;
  int edge_mode;
  const float* sbf;
  const float* w;
  const float* b;
  const int32_t* rowptr;   // fwd/bwd_dst: trip_rowptr; bwd_src: src_rowptr
  const int32_t* tidx;     // fwd/bwd_dst: trip_src;    bwd_src: src_perm
  const int32_t* tdst;     // bwd_src: trip_dst
  const float* alpha;
  const float* smax;
  const float* sden;
  const float* dlogit_in;
  const float* dout;
  int64_t E;
  int64_t T;
  int D;
  int H;
  float sqrt_c;
  float* out;
  float* alpha_out;
  float* smax_out;
  float* sden_out;
  float2* row_stats;  // fwd: per output row (mean, sum of squared deviations) for a fused graph LayerNorm, or NULL
  float* dq;
  float* d_edge;
  float* dlogit;
  float* dproj;
  float* dk;
  float* dv;
};

// Inactive lanes (D < 64 * CPL) read the row's first element instead of being branched around,
// so consecutive row loads stay independent (see ld_pin in common.hpp).
template <int CPL>
__device__ __forceinline__ void load_row(const float* __restrict__ p, bool act, float (&r)[CPL]) {
  if (CPL == 2) {
    const float2 x = ld_pin2(p);
    r[0] = keep(x.x, act);
    r[1] = keep(x.y, act);
  } else if (CPL == 4) {
    const float4 x = ld_pin4(p);
    r[0] = keep(x.x, act);
    r[1] = keep(x.y, act);
    r[2] = keep(x.z, act);
    r[3] = keep(x.w, act);
  } else {
#pragma unroll
    for (int j = 0; j < CPL; ++j) {
      const float x = ld_pin(p + j);
      r[j] = keep(x, act);
    }
  }
}

template <int CPL>
__device__ __forceinline__ void store_row(float* __restrict__ p, bool act, const float (&r)[CPL]) {
  if (!act) return;
  if (CPL == 2) {
    *reinterpret_cast<float2*>(p) = make_float2(r[0], r[1]);
  } else if (CPL == 4) {
    *reinterpret_cast<float4*>(p) = make_float4(r[0], r[1], r[2], r[3]);
  } else {
#pragma unroll
    for (int j = 0; j < CPL; ++j) p[j] = r[j];
  }
}

// sp[j] = b[j] + sum_s W[c0+j][s] * sbf_t[s]; the sbf row pointer is wave-uniform (scalar loads).
template <int CPL>
__device__ __forceinline__ void sbf_project(const float (&wr)[CPL][kS], const float (&br)[CPL],
                                            const float* __restrict__ srow, float (&sp)[CPL]) {
  float acc[CPL];
#pragma unroll
  for (int j = 0; j < CPL; ++j) acc[j] = 0.f;
#pragma unroll
  for (int s = 0; s < kS; ++s) {
    const float x = srow[s];
#pragma unroll
    for (int j = 0; j < CPL; ++j) acc[j] = fmaf(wr[j][s], x, acc[j]);
  }
#pragma unroll
  for (int j = 0; j < CPL; ++j) sp[j] = acc[j] + br[j];
}

template <int CPL>
__device__ __forceinline__ void load_weights(const float* __restrict__ w, const float* __restrict__ b, int c0,
                                             bool act, float (&wr)[CPL][kS], float (&br)[CPL]) {
#pragma unroll
  for (int j = 0; j < CPL; ++j) {
    const float* wrow = w + static_cast<int64_t>(c0 + j) * kS;
#pragma unroll
    for (int s = 0; s < kS; ++s) wr[j][s] = keep(wrow[s], act);
    br[j] = keep(b[c0 + j], act);
  }
}

// XCD-aware work split.  Workgroups are dispatched round-robin over the 8 XCDs (block b runs on
// XCD b % 8) and each XCD has its own 4 MiB L2.  Triplets never leave a molecule and molecules
// are contiguous ranges of line nodes, so giving XCD x the contiguous range [E x/8, E (x+1)/8)
// keeps the k/v/q rows its triplets gather (1 KiB per line node) inside ITS L2 instead of every
// XCD streaming every molecule through its cache.  Within an XCD the waves grid-stride.
// The grid is a multiple of 8 (dispatch rounds it up).
struct WaveRange {
  int64_t first, end, stride;
};

__device__ __forceinline__ WaveRange xcd_wave_range(int64_t n) {
  const int b = blockIdx.x, nb = gridDim.x;
  const int xcd = b & 7, per_xcd = nb >> 3;
  const int w = uniform((b >> 3) * kAttnWaves + static_cast<int>(threadIdx.x >> 6));
  const int64_t lo = n * xcd / 8, hi = n * (xcd + 1) / 8;
  return {lo + w, hi, static_cast<int64_t>(per_xcd) * kAttnWaves};
}

template <int CPL>
__device__ __forceinline__ void zero_row(float (&r)[CPL]) {
#pragma unroll
  for (int j = 0; j < CPL; ++j) r[j] = 0.f;
}

// Per-row statistics of an output row for the graph LayerNorm that follows the conv (model.py:46):
// rs[e] = (mean over the row's D values, sum of their squared deviations from it).  The consumer
// (x2g_chain_fwd_ln) combines a molecule's rows exactly (Chan: M2 = sum M2_r + D sum (mean_r -
// mean)^2), so the LayerNorm needs no pass of its own over the rows.
template <int CPL>
__device__ __forceinline__ void store_row_stats(float2* __restrict__ rs, int64_t e, const float (&o)[CPL], bool act,
                                                int D, int lane) {
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < CPL; ++j) s += act ? o[j] : 0.f;
  const float mu = wave64_sum(s) / static_cast<float>(D);
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < CPL; ++j) {
    const float d = o[j] - mu;
    q = act ? fmaf(d, d, q) : q;
  }
  q = wave64_sum(q);
  if (lane == 0) rs[e] = make_float2(mu, q);
}

// Every kernel below takes its pointers as __restrict__ parameters: with them the compiler may
// serve wave-uniform reads (row pointers, triplet indices, the sbf row) from the scalar cache.

// The sbf projection S_t = W sbf_t + b either comes precomputed (PRE: S[T, D] from
// x2g_sbf_project, read as one coalesced row per triplet) or is computed on the fly from the
// 42-float sbf row with W held in registers (84 VGPRs at CPL = 2).
template <int CPL, bool PRE>
struct Proj {
  float wr[CPL][kS];
  float br[CPL];
  __device__ __forceinline__ void init(const float* __restrict__ w, const float* __restrict__ b, int c0, bool act) {
    load_weights<CPL>(w, b, c0, act, wr, br);
  }
};

template <int CPL>
struct Proj<CPL, true> {
  __device__ __forceinline__ void init(const float*, const float*, int, bool) {}
};

template <int CPL, bool PRE>
__device__ __forceinline__ void proj_row(const Proj<CPL, PRE>& P, const float* __restrict__ sbf, int64_t t,
                                         const float (&pre)[CPL], float (&sp)[CPL]) {
  if constexpr (PRE) {
#pragma unroll
    for (int j = 0; j < CPL; ++j) sp[j] = pre[j];
  } else {
    sbf_project<CPL>(P.wr, P.br, sbf + t * kS, sp);
  }
}

// Triplet loops keep three register sets in flight and rotate their ROLES by unrolling the loop
// three times, never their contents: copying a set whose loads are still in flight would wait
// for them (a v_mov of a pending VGPR), shrinking the prefetch distance to nothing.

// ------------------------------------------------------------------------------ forward
template <int CPL>
struct FwdSet {
  float k[CPL], v[CPL], s[CPL];
};

template <int CPL, bool PRE>
__device__ __forceinline__ void fwd_load(FwdSet<CPL>& S, const float* __restrict__ k, const float* __restrict__ v,
                                         const float* __restrict__ sbf, const int32_t* __restrict__ tsrc, int t,
                                         int D, int c0, bool act) {
  const int64_t src = uniform(tsrc[t]);
  load_row<CPL>(k + src * D + c0, act, S.k);
  load_row<CPL>(v + src * D + c0, act, S.v);
  if (PRE) load_row<CPL>(sbf + static_cast<int64_t>(t) * D + c0, act, S.s);
}

template <int CPL>
struct FwdState {
  float qv[CPL], ed[CPL], acc[CPL];
  float m, den;
};

template <int CPL, int LPH, int MODE, bool PRE>
__device__ __forceinline__ void fwd_step(FwdSet<CPL>& S, int t, int t1, FwdState<CPL>& st, const Proj<CPL, PRE>& P,
                                         const float* __restrict__ k, const float* __restrict__ v,
                                         const float* __restrict__ edge, const float* __restrict__ sbf,
                                         const int32_t* __restrict__ tsrc, int D, int H, int c0, int head, bool act,
                                         bool leader, float sqrt_c, float* __restrict__ alpha_out) {
  float et[CPL];
  if (MODE == X2G_EDGE_PER_TRIPLET) {
    load_row<CPL>(edge + static_cast<int64_t>(t) * D + c0, act, et);
  } else {
#pragma unroll
    for (int j = 0; j < CPL; ++j) et[j] = st.ed[j];
  }
  float dot = 0.f;
#pragma unroll
  for (int j = 0; j < CPL; ++j) dot = fmaf(st.qv[j], S.k[j] + et[j], dot);
  const float logit = group_sum<LPH>(dot) / sqrt_c;
  float sp[CPL];
  proj_row<CPL, PRE>(P, sbf, t, S.s, sp);
  const float m_new = fmaxf(st.m, logit);
  const float corr = expf(st.m - m_new);
  const float p = expf(logit - m_new);
  st.den = st.den * corr + p;
#pragma unroll
  for (int j = 0; j < CPL; ++j) st.acc[j] = st.acc[j] * corr + p * ((S.v[j] + et[j]) * sp[j]);
  st.m = m_new;
  if (leader) alpha_out[static_cast<int64_t>(t) * H + head] = logit;
  if (t + 3 < t1) fwd_load<CPL, PRE>(S, k, v, sbf, tsrc, t + 3, D, c0, act);  // this set's next triplet
}

template <int CPL, int LPH, int MODE, bool PRE>
__global__ void __launch_bounds__(256) attn_fwd_kernel(
    const float* __restrict__ q, const float* __restrict__ k, const float* __restrict__ v,
    const float* __restrict__ skip, const float* __restrict__ edge, const int32_t* __restrict__ edge_row,
    const float* __restrict__ sbf, const float* __restrict__ w, const float* __restrict__ b,
    const int32_t* __restrict__ rowptr, const int32_t* __restrict__ tsrc, int64_t E, int D, int H, float sqrt_c,
    float* __restrict__ out, float* __restrict__ alpha_out, float* __restrict__ smax_out,
    float* __restrict__ sden_out, float2* __restrict__ row_stats) {
  const int lane = threadIdx.x & 63;
  const bool act = lane * CPL < D;
  const int c0 = act ? lane * CPL : 0;
  const int head = lane / LPH;
  const bool leader = act && (lane % LPH) == 0;
  Proj<CPL, PRE> P;
  P.init(w, b, c0, act);
  const WaveRange wr_ = xcd_wave_range(E);
  for (int64_t e = wr_.first; e < wr_.end; e += wr_.stride) {
    const int t0 = uniform(rowptr[e]), t1 = uniform(rowptr[e + 1]);
    FwdState<CPL> st;
    load_row<CPL>(q + e * D + c0, act, st.qv);
    if (MODE == X2G_EDGE_PER_DST) {
      const int64_t r = edge_row ? uniform(edge_row[e]) : e;
      load_row<CPL>(edge + r * D + c0, act, st.ed);
    } else {
      zero_row<CPL>(st.ed);
    }
    zero_row<CPL>(st.acc);
    st.m = -INFINITY;
    st.den = 0.f;
    FwdSet<CPL> A{}, B{}, C{};
    if (t0 < t1) fwd_load<CPL, PRE>(A, k, v, sbf, tsrc, t0, D, c0, act);
    if (t0 + 1 < t1) fwd_load<CPL, PRE>(B, k, v, sbf, tsrc, t0 + 1, D, c0, act);
    if (t0 + 2 < t1) fwd_load<CPL, PRE>(C, k, v, sbf, tsrc, t0 + 2, D, c0, act);
    for (int t = t0; t < t1; t += 3) {
      fwd_step<CPL, LPH, MODE, PRE>(A, t, t1, st, P, k, v, edge, sbf, tsrc, D, H, c0, head, act, leader, sqrt_c,
                                    alpha_out);
      if (t + 1 >= t1) break;
      fwd_step<CPL, LPH, MODE, PRE>(B, t + 1, t1, st, P, k, v, edge, sbf, tsrc, D, H, c0, head, act, leader, sqrt_c,
                                    alpha_out);
      if (t + 2 >= t1) break;
      fwd_step<CPL, LPH, MODE, PRE>(C, t + 2, t1, st, P, k, v, edge, sbf, tsrc, D, H, c0, head, act, leader, sqrt_c,
                                    alpha_out);
    }
    float sk[CPL], o[CPL];
    load_row<CPL>(skip + e * D + c0, act, sk);
    const float inv = 1.0f / (st.den + kSoftmaxEps);
#pragma unroll
    for (int j = 0; j < CPL; ++j) o[j] = st.acc[j] * inv + sk[j];
    store_row<CPL>(out + e * D + c0, act, o);
    if (row_stats) store_row_stats<CPL>(row_stats, e, o, act, D, lane);
    if (leader) {
      smax_out[e * H + head] = st.m;
      sden_out[e * H + head] = st.den;
    }
  }
}

// Batched forward (the default for precomputed S): the destination's triplets are contiguous, so
// their source ids arrive as one coalesced load (lane i <-> triplet t0 + i, broadcast with
// v_readlane) and the k/v/S rows of up to B triplets are issued back to back (clamped to the
// segment, masked in the arithmetic) — one memory round trip per batch instead of a dependent
// scalar index chain per triplet.  Same online softmax, same order: bitwise equal results.
template <int CPL, int LPH, int MODE, int B>
__device__ __forceinline__ void fwd_batch(int k0, int n, int tb, int sl, FwdState<CPL>& st,
                                          const float* __restrict__ k, const float* __restrict__ v,
                                          const float* __restrict__ sp, int D, int H, int c0, int head, bool act,
                                          bool leader, float sqrt_c, float* __restrict__ alpha_out) {
  float kv[B][CPL], vv[B][CPL], sv[B][CPL];
#pragma unroll
  for (int j = 0; j < B; ++j) {
    const int idx = k0 + j < n ? k0 + j : n - 1;
    const int64_t src = lane_bcast(sl, idx);
    load_row<CPL>(k + src * D + c0, act, kv[j]);
    load_row<CPL>(v + src * D + c0, act, vv[j]);
    load_row<CPL>(sp + static_cast<int64_t>(tb + idx) * D + c0, act, sv[j]);
  }
#pragma unroll
  for (int j = 0; j < B; ++j) {
    if (k0 + j >= n) break;  // wave-uniform
    float dot = 0.f;
#pragma unroll
    for (int c = 0; c < CPL; ++c) dot = fmaf(st.qv[c], kv[j][c] + st.ed[c], dot);
    const float logit = group_sum<LPH>(dot) / sqrt_c;
    const float m_new = fmaxf(st.m, logit);
    const float corr = expf(st.m - m_new);
    const float p = expf(logit - m_new);
    st.den = st.den * corr + p;
#pragma unroll
    for (int c = 0; c < CPL; ++c) st.acc[c] = st.acc[c] * corr + p * ((vv[j][c] + st.ed[c]) * sv[j][c]);
    st.m = m_new;
    if (leader) alpha_out[static_cast<int64_t>(tb + k0 + j) * H + head] = logit;
  }
}


// Software-pipelined over the wave's destinations: the row pointer two segments ahead, the next
// segment's source ids and this segment's skip row are requested at the top of the segment, so the
// dependent index chain (rowptr -> trip_src -> the k / v / S gathers) of the next segment is in flight
// under this one's gathers and math instead of costing two serial round trips per segment.
template <int CPL, int LPH, int MODE>
__global__ void __launch_bounds__(256) attn_fwd_batched(
    const float* __restrict__ q, const float* __restrict__ k, const float* __restrict__ v,
    const float* __restrict__ skip, const float* __restrict__ edge, const int32_t* __restrict__ edge_row,
    const float* __restrict__ sp, const int32_t* __restrict__ rowptr, const int32_t* __restrict__ tsrc, int64_t E,
    int64_t T, int D, int H, float sqrt_c, float* __restrict__ out, float* __restrict__ alpha_out,
    float* __restrict__ smax_out, float* __restrict__ sden_out, float2* __restrict__ row_stats) {
  const int lane = threadIdx.x & 63;
  const bool act = lane * CPL < D;
  const int c0 = act ? lane * CPL : 0;
  const int head = lane / LPH;
  const bool leader = act && (lane % LPH) == 0;
  // source ids through a descriptor: unconditional loads (see attn_bwd_dst_g_batched)
  const int tbytes = static_cast<int>(T * 4 < 0x7fffffff ? T * 4 : 0x7fffffff);
  const __amdgpu_buffer_rsrc_t ts_r =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<int32_t*>(tsrc), static_cast<short>(0), tbytes, 0x00020000);
  auto chunk_src = [&](int t, int n) {
    const int idx = t + (lane < n ? lane : (n > 0 ? n - 1 : 0));
    return static_cast<int>(__builtin_amdgcn_raw_buffer_load_b32(ts_r, n > 0 ? idx * 4 : 0x7ffffff0, 0, 0));
  };
  const WaveRange wr_ = xcd_wave_range(E);
  int64_t e = wr_.first;
  if (e >= wr_.end) return;
  const int64_t last = wr_.end - 1;
  int t0 = uniform(rowptr[e]), t1 = uniform(rowptr[e + 1]);
  const int64_t e1 = e + wr_.stride < wr_.end ? e + wr_.stride : last;
  int q0 = uniform(rowptr[e1]), q1 = uniform(rowptr[e1 + 1]);
  int sl = chunk_src(t0, t1 - t0 < 64 ? t1 - t0 : 64);
  // the edge-table row of the current / next destination (one segment ahead, like the source ids)
  int er = (MODE == X2G_EDGE_PER_DST && edge_row) ? uniform(edge_row[e]) : static_cast<int>(e);
  int ern = (MODE == X2G_EDGE_PER_DST && edge_row) ? uniform(edge_row[e1]) : static_cast<int>(e1);
  for (; e < wr_.end; e += wr_.stride) {
    FwdState<CPL> st;
    float sk[CPL];
    load_row<CPL>(q + e * D + c0, act, st.qv);
    load_row<CPL>(skip + e * D + c0, act, sk);
    if (MODE == X2G_EDGE_PER_DST) {
      load_row<CPL>(edge + static_cast<int64_t>(er) * D + c0, act, st.ed);
    } else {
      zero_row<CPL>(st.ed);
    }
    zero_row<CPL>(st.acc);
    st.m = -INFINITY;
    st.den = 0.f;
    const int64_t e2r = e + 2 * wr_.stride;
    const int64_t e2 = e2r < wr_.end ? e2r : last;
    const int r0 = uniform(rowptr[e2]), r1 = uniform(rowptr[e2 + 1]);
    const int er2 = (MODE == X2G_EDGE_PER_DST && edge_row) ? uniform(edge_row[e2]) : static_cast<int>(e2);
    const int sln = chunk_src(q0, q1 - q0 < 64 ? q1 - q0 : 64);
    for (int tb = t0; tb < t1; tb += 64) {
      const int n = t1 - tb < 64 ? t1 - tb : 64;
      if (tb != t0) sl = chunk_src(tb, n);  // segments longer than 64 triplets
      int k0 = 0;
      for (; n - k0 > 4; k0 += 8)
        fwd_batch<CPL, LPH, MODE, 8>(k0, n, tb, sl, st, k, v, sp, D, H, c0, head, act, leader, sqrt_c, alpha_out);
      if (k0 < n)
        fwd_batch<CPL, LPH, MODE, 4>(k0, n, tb, sl, st, k, v, sp, D, H, c0, head, act, leader, sqrt_c, alpha_out);
    }
    float o[CPL];
    const float inv = 1.0f / (st.den + kSoftmaxEps);
#pragma unroll
    for (int c = 0; c < CPL; ++c) o[c] = st.acc[c] * inv + sk[c];
    store_row<CPL>(out + e * D + c0, act, o);
    if (row_stats) store_row_stats<CPL>(row_stats, e, o, act, D, lane);
    if (leader) {
      smax_out[e * H + head] = st.m;
      sden_out[e * H + head] = st.den;
    }
    t0 = q0;
    t1 = q1;
    q0 = r0;
    q1 = r1;
    sl = sln;
    er = ern;
    ern = er2;
  }
}

// ------------------------------------------------------------------------------ backward (dst)
// pass 1 (per triplet): g = d loss / d a_t per head (sum over the head's channels of
// go (v + e) S), rho = sum_t a_t g_t, d_sbfproj = go (v + e) a, the value part of d_edge.
// pass 2: dlogit = a (g - rho), dq, the key part of d_edge.
template <int CPL>
struct DstSet1 {
  float v[CPL], s[CPL];
  float al;  // raw logit of the triplet (this lane's head)
};

template <int CPL>
struct DstSet2 {
  float k[CPL];
  float al, g;
};

template <int CPL>
struct DstState {
  float go[CPL], qv[CPL], ed[CPL], edacc[CPL], dqa[CPL];
  float mx, inv, rho;
};

template <int CPL, bool PRE>
__device__ __forceinline__ void dst_load1(DstSet1<CPL>& S, const float* __restrict__ v,
                                          const float* __restrict__ sbf, const float* __restrict__ alpha,
                                          const int32_t* __restrict__ tsrc, int t, int D, int H, int c0, int head,
                                          bool act) {
  const int64_t src = uniform(tsrc[t]);
  load_row<CPL>(v + src * D + c0, act, S.v);
  if (PRE) load_row<CPL>(sbf + static_cast<int64_t>(t) * D + c0, act, S.s);
  S.al = alpha[static_cast<int64_t>(t) * H + (act ? head : 0)];
}

template <int CPL, int LPH, int MODE, bool PRE>
__device__ __forceinline__ void dst_step1(DstSet1<CPL>& S, int t, int t1, DstState<CPL>& st,
                                          const Proj<CPL, PRE>& P, const float* __restrict__ v,
                                          const float* __restrict__ edge, const float* __restrict__ sbf,
                                          const float* __restrict__ alpha, const int32_t* __restrict__ tsrc, int D,
                                          int H, int c0, int head, bool act, bool leader,
                                          float* __restrict__ d_edge, float* __restrict__ dlogit,
                                          float* __restrict__ dproj) {
  constexpr bool per_trip = MODE == X2G_EDGE_PER_TRIPLET;
  float et[CPL], sp[CPL];
  if (per_trip) {
    load_row<CPL>(edge + static_cast<int64_t>(t) * D + c0, act, et);
  } else {
#pragma unroll
    for (int j = 0; j < CPL; ++j) et[j] = st.ed[j];
  }
  proj_row<CPL, PRE>(P, sbf, t, S.s, sp);
  const float at = act ? expf(S.al - st.mx) * st.inv : 0.f;
  float gpart = 0.f, dp[CPL], du[CPL];
#pragma unroll
  for (int j = 0; j < CPL; ++j) {
    const float u = S.v[j] + et[j];
    gpart = fmaf(st.go[j] * u, sp[j], gpart);
    dp[j] = st.go[j] * u * at;
    du[j] = st.go[j] * sp[j] * at;
  }
  const float g = group_sum<LPH>(gpart);
  st.rho = fmaf(at, g, st.rho);
  store_row<CPL>(dproj + static_cast<int64_t>(t) * D + c0, act, dp);
  if (per_trip) {
    store_row<CPL>(d_edge + static_cast<int64_t>(t) * D + c0, act, du);
  } else {
#pragma unroll
    for (int j = 0; j < CPL; ++j) st.edacc[j] += du[j];
  }
  if (leader) dlogit[static_cast<int64_t>(t) * H + head] = g;
  if (t + 3 < t1) dst_load1<CPL, PRE>(S, v, sbf, alpha, tsrc, t + 3, D, H, c0, head, act);
}

template <int CPL>
__device__ __forceinline__ void dst_load2(DstSet2<CPL>& S, const float* __restrict__ k,
                                          const float* __restrict__ alpha, const float* __restrict__ dlogit,
                                          const int32_t* __restrict__ tsrc, int t, int D, int H, int c0, int head,
                                          bool act, bool leader) {
  const int64_t src = uniform(tsrc[t]);
  load_row<CPL>(k + src * D + c0, act, S.k);
  const int64_t ah = static_cast<int64_t>(t) * H + (act ? head : 0);
  S.al = alpha[ah];
  // pass 1's g of this (triplet, head) was written by the head's leader lane: only that lane
  // reads it back (its own earlier store), the others get it by a shuffle at use
  S.g = leader ? dlogit[ah] : 0.f;
}

template <int CPL, int LPH, int MODE>
__device__ __forceinline__ void dst_step2(DstSet2<CPL>& S, int t, int t1, DstState<CPL>& st,
                                          const float* __restrict__ k, const float* __restrict__ edge,
                                          const float* __restrict__ alpha, const int32_t* __restrict__ tsrc, int D,
                                          int H, int c0, int head, bool act, bool leader, float sqrt_c,
                                          float* __restrict__ d_edge, float* __restrict__ dlogit) {
  constexpr bool per_trip = MODE == X2G_EDGE_PER_TRIPLET;
  float et[CPL];
  if (per_trip) {
    load_row<CPL>(edge + static_cast<int64_t>(t) * D + c0, act, et);
  } else {
#pragma unroll
    for (int j = 0; j < CPL; ++j) et[j] = st.ed[j];
  }
  const float at = act ? expf(S.al - st.mx) * st.inv : 0.f;
  const float dl = at * (group_sum<LPH>(S.g) - st.rho);
  const float ds = dl / sqrt_c;
  float dk[CPL];
#pragma unroll
  for (int j = 0; j < CPL; ++j) {
    st.dqa[j] = fmaf(ds, S.k[j] + et[j], st.dqa[j]);
    dk[j] = ds * st.qv[j];
  }
  if (per_trip) {
    float cur[CPL];
    load_row<CPL>(d_edge + static_cast<int64_t>(t) * D + c0, act, cur);
#pragma unroll
    for (int j = 0; j < CPL; ++j) cur[j] += dk[j];
    store_row<CPL>(d_edge + static_cast<int64_t>(t) * D + c0, act, cur);
  } else {
#pragma unroll
    for (int j = 0; j < CPL; ++j) st.edacc[j] += dk[j];
  }
  if (t + 3 < t1) dst_load2<CPL>(S, k, alpha, dlogit, tsrc, t + 3, D, H, c0, head, act, leader);
  if (leader) dlogit[static_cast<int64_t>(t) * H + head] = dl;  // after the prefetch read t + 3, not t
}

template <int CPL, int LPH, int MODE, bool PRE>
__global__ void __launch_bounds__(256) attn_bwd_dst_kernel(
    const float* __restrict__ q, const float* __restrict__ k, const float* __restrict__ v,
    const float* __restrict__ edge, const int32_t* __restrict__ edge_row, const float* __restrict__ sbf,
    const float* __restrict__ w, const float* __restrict__ b, const int32_t* __restrict__ rowptr,
    const int32_t* __restrict__ tsrc, const float* __restrict__ alpha, const float* __restrict__ smax,
    const float* __restrict__ sden, const float* __restrict__ dout, int64_t E, int D, int H, float sqrt_c,
    float* __restrict__ dq, float* __restrict__ d_edge, float* __restrict__ dlogit, float* __restrict__ dproj) {
  const int lane = threadIdx.x & 63;
  const bool act = lane * CPL < D;
  const int c0 = act ? lane * CPL : 0;
  const int head = lane / LPH;
  const bool leader = act && (lane % LPH) == 0;
  constexpr bool per_dst = MODE == X2G_EDGE_PER_DST;
  Proj<CPL, PRE> P;
  P.init(w, b, c0, act);
  const WaveRange wr_ = xcd_wave_range(E);
  for (int64_t e = wr_.first; e < wr_.end; e += wr_.stride) {
    const int t0 = uniform(rowptr[e]), t1 = uniform(rowptr[e + 1]);
    DstState<CPL> st;
    load_row<CPL>(dout + e * D + c0, act, st.go);
    load_row<CPL>(q + e * D + c0, act, st.qv);
    if (per_dst) {
      const int64_t r = edge_row ? uniform(edge_row[e]) : e;
      load_row<CPL>(edge + r * D + c0, act, st.ed);
    } else {
      zero_row<CPL>(st.ed);
    }
    zero_row<CPL>(st.edacc);
    zero_row<CPL>(st.dqa);
    st.mx = keep(smax[e * H + head], act);
    st.inv = act ? 1.0f / (sden[e * H + head] + kSoftmaxEps) : 0.f;
    st.rho = 0.f;
    {
      DstSet1<CPL> A{}, B{}, C{};
      if (t0 < t1) dst_load1<CPL, PRE>(A, v, sbf, alpha, tsrc, t0, D, H, c0, head, act);
      if (t0 + 1 < t1) dst_load1<CPL, PRE>(B, v, sbf, alpha, tsrc, t0 + 1, D, H, c0, head, act);
      if (t0 + 2 < t1) dst_load1<CPL, PRE>(C, v, sbf, alpha, tsrc, t0 + 2, D, H, c0, head, act);
      for (int t = t0; t < t1; t += 3) {
        dst_step1<CPL, LPH, MODE, PRE>(A, t, t1, st, P, v, edge, sbf, alpha, tsrc, D, H, c0, head, act, leader,
                                       d_edge, dlogit, dproj);
        if (t + 1 >= t1) break;
        dst_step1<CPL, LPH, MODE, PRE>(B, t + 1, t1, st, P, v, edge, sbf, alpha, tsrc, D, H, c0, head, act, leader,
                                       d_edge, dlogit, dproj);
        if (t + 2 >= t1) break;
        dst_step1<CPL, LPH, MODE, PRE>(C, t + 2, t1, st, P, v, edge, sbf, alpha, tsrc, D, H, c0, head, act, leader,
                                       d_edge, dlogit, dproj);
      }
    }
    {
      DstSet2<CPL> A{}, B{}, C{};
      if (t0 < t1) dst_load2<CPL>(A, k, alpha, dlogit, tsrc, t0, D, H, c0, head, act, leader);
      if (t0 + 1 < t1) dst_load2<CPL>(B, k, alpha, dlogit, tsrc, t0 + 1, D, H, c0, head, act, leader);
      if (t0 + 2 < t1) dst_load2<CPL>(C, k, alpha, dlogit, tsrc, t0 + 2, D, H, c0, head, act, leader);
      for (int t = t0; t < t1; t += 3) {
        dst_step2<CPL, LPH, MODE>(A, t, t1, st, k, edge, alpha, tsrc, D, H, c0, head, act, leader, sqrt_c, d_edge, dlogit);
        if (t + 1 >= t1) break;
        dst_step2<CPL, LPH, MODE>(B, t + 1, t1, st, k, edge, alpha, tsrc, D, H, c0, head, act, leader, sqrt_c, d_edge,
                             dlogit);
        if (t + 2 >= t1) break;
        dst_step2<CPL, LPH, MODE>(C, t + 2, t1, st, k, edge, alpha, tsrc, D, H, c0, head, act, leader, sqrt_c, d_edge,
                             dlogit);
      }
    }
    store_row<CPL>(dq + e * D + c0, act, st.dqa);
    if (per_dst) store_row<CPL>(d_edge + e * D + c0, act, st.edacc);
  }
}

// ------------------------------------------------------------------------------ backward (src)
template <int CPL>
struct SrcSet {
  float go[CPL], qv[CPL], s[CPL];
  float al, mx, den, dl;
  int64_t t;
};

template <int CPL, bool PRE>
__device__ __forceinline__ void src_load(SrcSet<CPL>& S, const float* __restrict__ q, const float* __restrict__ sbf,
                                         const int32_t* __restrict__ perm, const int32_t* __restrict__ tdst,
                                         const float* __restrict__ alpha, const float* __restrict__ smax,
                                         const float* __restrict__ sden, const float* __restrict__ dlogit_in,
                                         const float* __restrict__ dout, int p, int D, int H, int c0, int head,
                                         bool act) {
  const int64_t t = uniform(perm[p]);
  const int64_t e = uniform(tdst[t]);
  S.t = t;
  load_row<CPL>(dout + e * D + c0, act, S.go);
  load_row<CPL>(q + e * D + c0, act, S.qv);
  if (PRE) load_row<CPL>(sbf + t * D + c0, act, S.s);
  const int hh = act ? head : 0;
  S.al = alpha[t * H + hh];
  S.dl = dlogit_in[t * H + hh];
  S.mx = smax[e * H + hh];
  S.den = sden[e * H + hh];
}

template <int CPL, bool PRE>
__device__ __forceinline__ void src_step(SrcSet<CPL>& S, int p, int p1, const Proj<CPL, PRE>& P,
                                         float (&dka)[CPL], float (&dva)[CPL], const float* __restrict__ q,
                                         const float* __restrict__ sbf, const int32_t* __restrict__ perm,
                                         const int32_t* __restrict__ tdst, const float* __restrict__ alpha,
                                         const float* __restrict__ smax, const float* __restrict__ sden,
                                         const float* __restrict__ dlogit_in, const float* __restrict__ dout, int D,
                                         int H, int c0, int head, bool act, float sqrt_c) {
  float sp[CPL];
  proj_row<CPL, PRE>(P, sbf, S.t, S.s, sp);
  const float at = act ? expf(S.al - S.mx) / (S.den + kSoftmaxEps) : 0.f;
  const float ds = act ? S.dl / sqrt_c : 0.f;
#pragma unroll
  for (int j = 0; j < CPL; ++j) {
    dva[j] = fmaf(S.go[j] * sp[j], at, dva[j]);
    dka[j] = fmaf(ds, S.qv[j], dka[j]);
  }
  if (p + 3 < p1) src_load<CPL, PRE>(S, q, sbf, perm, tdst, alpha, smax, sden, dlogit_in, dout, p + 3, D, H, c0, head,
                                     act);
}

template <int CPL, int LPH, bool PRE>
__global__ void __launch_bounds__(256) attn_bwd_src_kernel(
    const float* __restrict__ q, const float* __restrict__ sbf, const float* __restrict__ w,
    const float* __restrict__ b, const int32_t* __restrict__ rowptr, const int32_t* __restrict__ perm,
    const int32_t* __restrict__ tdst, const float* __restrict__ alpha, const float* __restrict__ smax,
    const float* __restrict__ sden, const float* __restrict__ dlogit_in, const float* __restrict__ dout,
    int64_t E, int D, int H, float sqrt_c, float* __restrict__ dk, float* __restrict__ dv) {
  const int lane = threadIdx.x & 63;
  const bool act = lane * CPL < D;
  const int c0 = act ? lane * CPL : 0;
  const int head = lane / LPH;
  Proj<CPL, PRE> P;
  P.init(w, b, c0, act);
  const WaveRange wr_ = xcd_wave_range(E);
  for (int64_t s = wr_.first; s < wr_.end; s += wr_.stride) {
    const int p0 = uniform(rowptr[s]), p1 = uniform(rowptr[s + 1]);
    float dka[CPL], dva[CPL];
    zero_row<CPL>(dka);
    zero_row<CPL>(dva);
    SrcSet<CPL> A{}, B{}, C{};
    if (p0 < p1) src_load<CPL, PRE>(A, q, sbf, perm, tdst, alpha, smax, sden, dlogit_in, dout, p0, D, H, c0, head, act);
    if (p0 + 1 < p1)
      src_load<CPL, PRE>(B, q, sbf, perm, tdst, alpha, smax, sden, dlogit_in, dout, p0 + 1, D, H, c0, head, act);
    if (p0 + 2 < p1)
      src_load<CPL, PRE>(C, q, sbf, perm, tdst, alpha, smax, sden, dlogit_in, dout, p0 + 2, D, H, c0, head, act);
    for (int p = p0; p < p1; p += 3) {
      src_step<CPL, PRE>(A, p, p1, P, dka, dva, q, sbf, perm, tdst, alpha, smax, sden, dlogit_in, dout, D, H, c0, head,
                         act, sqrt_c);
      if (p + 1 >= p1) break;
      src_step<CPL, PRE>(B, p + 1, p1, P, dka, dva, q, sbf, perm, tdst, alpha, smax, sden, dlogit_in, dout, D, H, c0,
                         head, act, sqrt_c);
      if (p + 2 >= p1) break;
      src_step<CPL, PRE>(C, p + 2, p1, P, dka, dva, q, sbf, perm, tdst, alpha, smax, sden, dlogit_in, dout, D, H, c0,
                         head, act, sqrt_c);
    }
    store_row<CPL>(dk + s * D + c0, act, dka);
    store_row<CPL>(dv + s * D + c0, act, dva);
  }
}

#include "attention_fold.inc"

// ------------------------------------------------------------------------------ sbf projection
// S[t, :] = W sbf_t + b for all triplets (x2g_sbf_project): one wave per triplet row (grid-
// stride), CPL channels per lane with W in registers, the 42-float sbf row wave-uniform (scalar
// loads), one coalesced row store.  Every attention kernel then reads S rows instead of
// re-projecting (3 x 84 FMAs per triplet and lane, and 84 weight VGPRs, saved per layer).
template <int CPL>
__global__ void __launch_bounds__(256) sbf_project_kernel(const float* __restrict__ sbf, const float* __restrict__ w,
                                                          const float* __restrict__ b, int64_t T, int D,
                                                          float* __restrict__ S) {
  const int lane = threadIdx.x & 63;
  const bool act = lane * CPL < D;
  const int c0 = act ? lane * CPL : 0;
  float wr[CPL][kS], br[CPL];
  load_weights<CPL>(w, b, c0, act, wr, br);
  const int64_t nw = static_cast<int64_t>(gridDim.x) * kAttnWaves;
  for (int64_t t = uniform(blockIdx.x * kAttnWaves + (threadIdx.x >> 6)); t < T; t += nw) {
    float sp[CPL];
    sbf_project<CPL>(wr, br, sbf + t * kS, sp);
    store_row<CPL>(S + t * D + c0, act, sp);
  }
}

// ------------------------------------------------------------------------------ dispatch
enum class Pass { kFwd, kBwdDst, kBwdSrc };

template <int CPL, int LPH, int MODE, bool PRE>
void launch_pre(Pass pass, const AttnArgs& a, unsigned blocks, hipStream_t st) {
  switch (pass) {
    case Pass::kFwd:
      if (PRE && MODE != X2G_EDGE_PER_TRIPLET) {  // batched: up to 8 triplets' rows in flight per wave
        attn_fwd_batched<CPL, LPH, MODE><<<blocks, 256, 0, st>>>(a.q, a.k, a.v, a.skip, a.edge, a.edge_row, a.sbf,
                                                                 a.rowptr, a.tidx, a.E, a.T, a.D, a.H, a.sqrt_c, a.out,
                                                                 a.alpha_out, a.smax_out, a.sden_out, a.row_stats);
        break;
      }
      attn_fwd_kernel<CPL, LPH, MODE, PRE><<<blocks, 256, 0, st>>>(
          a.q, a.k, a.v, a.skip, a.edge, a.edge_row, a.sbf, a.w, a.b, a.rowptr, a.tidx, a.E, a.D, a.H, a.sqrt_c, a.out,
          a.alpha_out, a.smax_out, a.sden_out, a.row_stats);
      break;
    case Pass::kBwdDst:
      attn_bwd_dst_kernel<CPL, LPH, MODE, PRE><<<blocks, 256, 0, st>>>(
          a.q, a.k, a.v, a.edge, a.edge_row, a.sbf, a.w, a.b, a.rowptr, a.tidx, a.alpha, a.smax, a.sden, a.dout,
          a.E, a.D, a.H, a.sqrt_c, a.dq, a.d_edge, a.dlogit, a.dproj);
      break;
    case Pass::kBwdSrc:
      attn_bwd_src_kernel<CPL, LPH, PRE><<<blocks, 256, 0, st>>>(a.q, a.sbf, a.w, a.b, a.rowptr, a.tidx, a.tdst,
                                                                 a.alpha, a.smax, a.sden, a.dlogit_in, a.dout, a.E,
                                                                 a.D, a.H, a.sqrt_c, a.dk, a.dv);
      break;
  }
}

// w == NULL: `sbf` is the precomputed projection S[T, D] (x2g_sbf_project)
template <int CPL, int LPH, int MODE>
void launch_mode(Pass pass, const AttnArgs& a, unsigned blocks, hipStream_t st) {
  if (a.w == nullptr)
    launch_pre<CPL, LPH, MODE, true>(pass, a, blocks, st);
  else
    launch_pre<CPL, LPH, MODE, false>(pass, a, blocks, st);
}

template <int CPL, int LPH>
void launch_one(Pass pass, const AttnArgs& a, unsigned blocks, hipStream_t st) {
  if (pass == Pass::kBwdSrc) {
    launch_mode<CPL, LPH, X2G_EDGE_NONE>(pass, a, blocks, st);
    return;
  }
  switch (a.edge_mode) {
    case X2G_EDGE_PER_TRIPLET: launch_mode<CPL, LPH, X2G_EDGE_PER_TRIPLET>(pass, a, blocks, st); break;
    case X2G_EDGE_PER_DST: launch_mode<CPL, LPH, X2G_EDGE_PER_DST>(pass, a, blocks, st); break;
    default: launch_mode<CPL, LPH, X2G_EDGE_NONE>(pass, a, blocks, st); break;
  }
}

template <int CPL>
int launch_cpl(Pass pass, const AttnArgs& a, int lph, unsigned blocks, hipStream_t st) {
  switch (lph) {
    case 1: if (CPL >= 4) { launch_one<CPL, 1>(pass, a, blocks, st); return X2G_OK; } break;
    case 2: launch_one<CPL, 2>(pass, a, blocks, st); return X2G_OK;
    case 4: launch_one<CPL, 4>(pass, a, blocks, st); return X2G_OK;
    case 8: launch_one<CPL, 8>(pass, a, blocks, st); return X2G_OK;
    case 16: if (CPL == 1) { launch_one<CPL, 16>(pass, a, blocks, st); return X2G_OK; } break;
    default: break;
  }
  return X2G_EUNSUPPORTED;
}

int dispatch(Pass pass, AttnArgs a, int heads, int channels, int sbf_dim, hipStream_t st) {
  if (a.E < 0 || heads <= 0 || channels <= 0) return X2G_EINVAL;
  if (a.w ? sbf_dim != kS : sbf_dim != heads * channels) return X2G_EUNSUPPORTED;
  if (a.edge_mode != X2G_EDGE_NONE && a.edge_mode != X2G_EDGE_PER_TRIPLET && a.edge_mode != X2G_EDGE_PER_DST)
    return X2G_EINVAL;
  const int D = heads * channels;
  int cpl;
  if (D == 32 || D == 64) cpl = 1;
  else if (D == 128) cpl = 2;
  else if (D == 256) cpl = 4;
  else return X2G_EUNSUPPORTED;
  if (channels % cpl) return X2G_EUNSUPPORTED;
  const int lph = channels / cpl;
  if (lph > 64 || (lph & (lph - 1))) return X2G_EUNSUPPORTED;
  a.D = D;
  a.H = heads;
  a.sqrt_c = static_cast<float>(sqrt(static_cast<double>(channels)));
  if (a.E == 0) return X2G_OK;
  int64_t want = (a.E + kAttnWaves - 1) / kAttnWaves;
  want = want < kMaxBlocks ? want : kMaxBlocks;
  const unsigned blocks = static_cast<unsigned>((want + 7) / 8 * 8);  // a multiple of the 8 XCDs
  int rc;
  switch (cpl) {
    case 1: rc = launch_cpl<1>(pass, a, lph, blocks, st); break;
    case 2: rc = launch_cpl<2>(pass, a, lph, blocks, st); break;
    default: rc = launch_cpl<4>(pass, a, lph, blocks, st); break;
  }
  if (rc) return rc;
  return last_launch_status();
}

}  // namespace x2g

using namespace x2g;

X2G_API int x2g_sbf_attention_fwd(const float* q, const float* k, const float* v, const float* skip,
                                  const float* edge, const int32_t* edge_row, int edge_mode, const float* sbf,
                                  const float* w_sbf, const float* b_sbf, const int32_t* trip_rowptr,
                                  const int32_t* trip_src, int64_t E, int64_t T, int32_t heads,
                                  int32_t channels, int32_t sbf_dim, float* out, float* alpha_raw,
                                  float* seg_max, float* seg_den, void* stream) {
  if (E > 0 && (!q || !k || !v || !skip || !sbf || (w_sbf && !b_sbf) || !trip_rowptr || !out || !seg_max ||
                !seg_den))
    return X2G_EINVAL;
  if (T > 0 && (!trip_src || !alpha_raw)) return X2G_EINVAL;
  if (edge_mode != X2G_EDGE_NONE && !edge) return X2G_EINVAL;
  AttnArgs a{};
  a.q = q; a.k = k; a.v = v; a.skip = skip; a.edge = edge; a.edge_row = edge_row; a.edge_mode = edge_mode;
  a.sbf = sbf; a.w = w_sbf; a.b = b_sbf; a.rowptr = trip_rowptr; a.tidx = trip_src; a.E = E; a.T = T;
  a.out = out; a.alpha_out = alpha_raw; a.smax_out = seg_max; a.sden_out = seg_den;
  return dispatch(Pass::kFwd, a, heads, channels, sbf_dim, as_stream(stream));
}

X2G_API int x2g_sbf_attention_fwd_stats(const float* q, const float* k, const float* v, const float* skip,
                                        const float* edge, const int32_t* edge_row, int edge_mode, const float* sbf,
                                        const float* w_sbf, const float* b_sbf, const int32_t* trip_rowptr,
                                        const int32_t* trip_src, int64_t E, int64_t T, int32_t heads,
                                        int32_t channels, int32_t sbf_dim, float* out, float* alpha_raw,
                                        float* seg_max, float* seg_den, float* row_stats, void* stream) {
  if (E > 0 && (!q || !k || !v || !skip || !sbf || (w_sbf && !b_sbf) || !trip_rowptr || !out || !seg_max ||
                !seg_den || !row_stats))
    return X2G_EINVAL;
  if (T > 0 && (!trip_src || !alpha_raw)) return X2G_EINVAL;
  if (edge_mode != X2G_EDGE_NONE && !edge) return X2G_EINVAL;
  if (reinterpret_cast<uintptr_t>(row_stats) % 8) return X2G_EUNSUPPORTED;
  AttnArgs a{};
  a.q = q; a.k = k; a.v = v; a.skip = skip; a.edge = edge; a.edge_row = edge_row; a.edge_mode = edge_mode;
  a.sbf = sbf; a.w = w_sbf; a.b = b_sbf; a.rowptr = trip_rowptr; a.tidx = trip_src; a.E = E; a.T = T;
  a.out = out; a.alpha_out = alpha_raw; a.smax_out = seg_max; a.sden_out = seg_den;
  a.row_stats = reinterpret_cast<float2*>(row_stats);
  return dispatch(Pass::kFwd, a, heads, channels, sbf_dim, as_stream(stream));
}

X2G_API int x2g_sbf_attention_bwd_dst(const float* q, const float* k, const float* v, const float* edge,
                                      const int32_t* edge_row, int edge_mode, const float* sbf,
                                      const float* w_sbf, const float* b_sbf, const int32_t* trip_rowptr,
                                      const int32_t* trip_src, const float* alpha_raw, const float* seg_max,
                                      const float* seg_den, const float* dout, int64_t E, int64_t T,
                                      int32_t heads, int32_t channels, int32_t sbf_dim, float* dq,
                                      float* d_edge, float* dlogit, float* d_sbfproj, void* stream) {
  if (E > 0 && (!q || !k || !v || !sbf || (w_sbf && !b_sbf) || !trip_rowptr || !seg_max || !seg_den || !dout ||
                !dq))
    return X2G_EINVAL;
  if (T > 0 && (!trip_src || !alpha_raw || !dlogit || !d_sbfproj)) return X2G_EINVAL;
  if (edge_mode != X2G_EDGE_NONE && (!edge || !d_edge)) return X2G_EINVAL;
  AttnArgs a{};
  a.q = q; a.k = k; a.v = v; a.edge = edge; a.edge_row = edge_row; a.edge_mode = edge_mode;
  a.sbf = sbf; a.w = w_sbf; a.b = b_sbf; a.rowptr = trip_rowptr; a.tidx = trip_src; a.alpha = alpha_raw;
  a.smax = seg_max; a.sden = seg_den; a.dout = dout; a.E = E;
  a.dq = dq; a.d_edge = d_edge; a.dlogit = dlogit; a.dproj = d_sbfproj;
  return dispatch(Pass::kBwdDst, a, heads, channels, sbf_dim, as_stream(stream));
}

X2G_API int x2g_sbf_attention_bwd_src(const float* q, const float* sbf, const float* w_sbf, const float* b_sbf,
                                      const int32_t* src_rowptr, const int32_t* src_perm, const int32_t* trip_dst,
                                      const float* alpha_raw, const float* seg_max, const float* seg_den,
                                      const float* dlogit, const float* dout, int64_t E, int64_t T,
                                      int32_t heads, int32_t channels, int32_t sbf_dim, float* dk, float* dv,
                                      void* stream) {
  if (E > 0 && (!q || !sbf || (w_sbf && !b_sbf) || !src_rowptr || !seg_max || !seg_den || !dout || !dk || !dv))
    return X2G_EINVAL;
  if (T > 0 && (!src_perm || !trip_dst || !alpha_raw || !dlogit)) return X2G_EINVAL;
  AttnArgs a{};
  a.q = q; a.sbf = sbf; a.w = w_sbf; a.b = b_sbf; a.rowptr = src_rowptr; a.tidx = src_perm; a.tdst = trip_dst;
  a.alpha = alpha_raw; a.smax = seg_max; a.sden = seg_den; a.dlogit_in = dlogit; a.dout = dout; a.E = E;
  a.dk = dk; a.dv = dv;
  return dispatch(Pass::kBwdSrc, a, heads, channels, sbf_dim, as_stream(stream));
}

namespace x2g {  // csrc/dense.hip: the narrow-K MFMA dense forward
int dense_fwd_narrow_launch(const float* x, const float* w, const float* b, const float* res, int64_t R, int K, int N,
                            int act, float* y, float* z, hipStream_t st);
}  // namespace x2g

namespace x2g {
// S = sbf W^T + b for the 42-wide sbf rows, wave-independent: a wave takes 16-row blocks of sbf
// (held as the MFMA B operand, lane (i, g) = row i, k = 16q + 4g + e as two 8-byte loads: the
// 168-byte rows are 8-byte aligned) and produces all 16 NOB output columns with
// v_mfma_f32_16x16x4_f32 against W^T fragments staged once per workgroup in LDS (the A operand,
// read as one conflict-free 16-byte chunk per lane and group); D lane (i, g) holds the block's
// row i, columns 16 ob + 4g .. +3: one 16-byte store each.  No barriers after the staging, the next
// block's rows in flight during the MFMAs: the loads, MFMAs and stores of the 4-5 resident waves
// per SIMD overlap (the tile-staged dense_fwd_narrow serialised them per workgroup: 3.1 TB/s).
constexpr int kSPQ = 3;  // 16-wide contraction groups (K = 42 -> 48, zero-padded)

// Round 3: the same wave-independent MFMA product with both HBM streams made line-coalesced (the
// per-lane form read each 168-byte sbf row as 8-byte pieces and wrote every output row as 64-byte
// pieces, 3.2 TB/s).  A wave's 16-row sbf block is 2688 contiguous bytes: three buffer_load ... lds
// instructions land it in the wave's own LDS slot (double-buffered: the next block's copy flies
// during this block's MFMAs), and each half of the output block goes out through the same slot
// (the block's rows are in registers by then), swizzled, as 256-byte row runs, 1 KB per store
// instruction.  No workgroup barrier after the W staging: every LDS slot is private to its wave (LDS
// operations of a wave execute in order).  16-wave workgroups share one W image: 16 waves per CU
// (153 KB of LDS), where 8-wave workgroups with private output tiles fitted only 8.
typedef __amdgpu_buffer_rsrc_t sp_rsrc_t;
__device__ __forceinline__ sp_rsrc_t sp_rsrc(const float* p, int64_t bytes) {
  const int64_t nr = bytes <= 0 ? 0 : (bytes < 0x7fffffff ? bytes : 0x7fffffff);
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), static_cast<short>(0), static_cast<int>(nr),
                                           0x00020000);
}

constexpr int kSPWaves = 16;           // 1024-thread workgroups, one per CU
constexpr int kSPChunks = 16 * kS / 4;  // 16-byte chunks per 16-row sbf block (168)

// The two LDS slots of a wave are two NAMED arrays and the loop is unrolled by two, so every slot
// index is static: with one dynamically indexed array the compiler could not tell the slot a ds_read
// reads from the slot the next block's buffer_load ... lds is filling and waited for every copy in
// flight (vmcnt(0)) before the B reads — the prefetch then bought nothing.  The wave index is read
// through readfirstlane, so block bases and buffer descriptors live in SGPRs (a descriptor the
// compiler thinks divergent costs a readfirstlane loop around every buffer instruction).
template <int NOB>
__device__ __forceinline__ void sbf_project_body(const float* __restrict__ sbf, const float* __restrict__ w,
                                                 const float* __restrict__ b, int64_t T, float* __restrict__ out) {
  typedef float f4t __attribute__((ext_vector_type(4)));
  __shared__ f4t Wl[NOB * kSPQ * 64];         // [ob][q][lane]: W[16ob + i][16q + 4g .. +3]
  __shared__ f4t Bl[NOB * 4];                 // [ob][g]: b[16ob + 4g .. +3]
  __shared__ f4t XsA[kSPWaves][16 * 16];      // per wave, slot A / slot B: a 16-row sbf block (168
  __shared__ f4t XsB[kSPWaves][16 * 16];      // chunks), then 16 rows x 64 output columns, swizzled
  constexpr int N = 16 * NOB;
  constexpr int HB = NOB < 4 ? NOB : 4;       // output blocks per half (64 columns)
  constexpr int kStores = NOB;                // store instructions per block (NOB / HB halves x HB)
  for (int idx = threadIdx.x; idx < NOB * kSPQ * 64; idx += blockDim.x) {
    const int l = idx & 63, q = (idx >> 6) % kSPQ, ob = (idx >> 6) / kSPQ;
    const int c = 16 * ob + (l & 15), k = 16 * q + (l >> 4);  // element e: contraction index k + 4e
    f4t v;
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = k + 4 * e < kS ? w[c * kS + k + 4 * e] : 0.0f;
    Wl[idx] = v;
  }
  for (int idx = threadIdx.x; idx < NOB * 4; idx += blockDim.x) {
    f4t v;
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = b ? b[4 * idx + e] : 0.0f;
    Bl[idx] = v;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
  const int wv = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
  const int64_t nblk = (T + 15) / 16;
  const int64_t nw = static_cast<int64_t>(gridDim.x) * kSPWaves;
  f4t* const slotA = &XsA[wv][0];
  f4t* const slotB = &XsB[wv][0];
  // a block's rows are 2688 contiguous bytes: chunk u * 64 + lane of the block (chunks >= 168 and rows
  // >= T read as zero through the range check)
  auto issue = [&](int64_t bk, f4t* slot) {
    const float* base = sbf + bk * (16 * kS);
    const sp_rsrc_t r = sp_rsrc(base, (T - bk * 16) * kS * 4);
#pragma unroll
    for (int u = 0; u < 3; ++u)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)(slot + 64 * u), 16,
                                               (64 * u + lane) < kSPChunks ? 16 * (64 * u + lane) : 0x7fffff00, 0, 0,
                                               0);
  };
  // block bk from `cur` (its copy issued one block earlier); the next block's copy goes to `nxt`
  auto block = [&](int64_t bk, f4t* cur, f4t* nxt, auto first) {
    // the next block's copy, unconditionally (past the end its descriptor has no records: zeros land
    // in the idle slot) — no branch, so the compiler's wait counts stay exact
    issue(bk + nw, nxt);
    asm volatile("" ::: "memory");
    // this block's copy is done when at most what was issued after it remains: the previous block's
    // stores and the next block's 3 copies (the stores read registers: nothing waits for them)
    if constexpr (decltype(first)::value)  // nothing was stored before the first block
      asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kStores + 3) : "memory");
    // B operand: lane (i, g) = row i, k = 16q + 4e + g (row i's floats at 42 i).  MFMA (q, e) then
    // contracts the 4 consecutive indices 16q + 4e .. +3, so the all-padding group k = 44..47 is
    // skipped: 11 MFMAs per output block instead of 12
    const float* xr = reinterpret_cast<const float*>(cur) + i * kS + g;
    f4t B[kSPQ];
#pragma unroll
    for (int q = 0; q < kSPQ; ++q)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int k0 = 16 * q + 4 * e;  // + g: padding when >= kS (the read stays inside the slot)
        if (k0 >= kS) continue;          // (the skipped group)
        const float xv = xr[k0];
        B[q][e] = k0 + g < kS ? xv : 0.0f;
      }
    float* ob = out + bk * 16 * N;
    const sp_rsrc_t orr = sp_rsrc(ob, (T - bk * 16) * N * 4);
    float* ys = reinterpret_cast<float*>(cur);  // B is in registers: the slot is free
#pragma unroll
    for (int h0 = 0; h0 < NOB; h0 += HB) {
      f4t acc[HB];
#pragma unroll
      for (int j = 0; j < HB; ++j) acc[j] = Bl[(h0 + j) * 4 + g];
#pragma unroll
      for (int q = 0; q < kSPQ; ++q) {
        f4t a[HB];
#pragma unroll
        for (int j = 0; j < HB; ++j) a[j] = Wl[((h0 + j) * kSPQ + q) * 64 + lane];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if (16 * q + 4 * e >= kS) continue;  // an all-padding contraction group
#pragma unroll
          for (int j = 0; j < HB; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j][e], B[q][e], acc[j], 0, 0, 0);
        }
      }
      // D lane (i, g): row i, local columns 16 j + 4 g .. +3 = chunk 4 j + g of the row's 16
#pragma unroll
      for (int j = 0; j < HB; ++j) *reinterpret_cast<f4t*>(ys + i * 64 + 4 * ((4 * j + g) ^ i)) = acc[j];
      // row-major out: instruction u covers rows 4u .. 4u + 3, lane = (row 4u + (lane >> 4), chunk lane & 15)
#pragma unroll
      for (int u = 0; u < 16 * HB / 16; ++u) {
        const int r = 4 * u + (lane >> 4), c = lane & 15;
        const f4t v = *reinterpret_cast<const f4t*>(ys + r * 64 + 4 * (c ^ r));
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, v), orr,
                                               4 * (r * N + 16 * h0 + 4 * c), 0, 0);
      }
    }
  };
  // the first block peeled (nothing stored before it), then pairs: every block's wait then sees the
  // same history on all paths into it and the compiler's own count for the slot reads stays exact
  int64_t blk = static_cast<int64_t>(blockIdx.x) * kSPWaves + wv;
  if (blk < nblk) {
    issue(blk, slotA);
    block(blk, slotA, slotB, std::true_type{});
    for (blk += nw; blk < nblk; blk += nw) {
      block(blk, slotB, slotA, std::false_type{});
      blk += nw;
      if (blk >= nblk) break;
      block(blk, slotA, slotB, std::false_type{});
    }
  }
}

template <int NOB>
__global__ void __launch_bounds__(kSPWaves * 64) sbf_project_waves(const float* __restrict__ sbf,
                                                                  const float* __restrict__ w,
                                                                  const float* __restrict__ b, int64_t T,
                                                                  float* __restrict__ out) {
  sbf_project_body<NOB>(sbf, w, b, T, out);
}

// Every layer's S = lin_sbf_l(sbf) in ONE launch (layer = blockIdx.y): one ramp and drain instead of
// one per layer, and the layers after the first read sbf (33 MB at config 2) from the MALL, which the
// first layer's pass has just filled, instead of from HBM.
constexpr int kSPMaxLayers = X2G_SBF_PROJECT_MAX_LAYERS;
struct SPBatch {
  const float* w[kSPMaxLayers];
  const float* b[kSPMaxLayers];
  float* out[kSPMaxLayers];
};
template <int NOB>
__global__ void __launch_bounds__(kSPWaves * 64) sbf_project_waves_batch(const float* __restrict__ sbf,
                                                                        const SPBatch a, int64_t T) {
  const int l = blockIdx.y;
  sbf_project_body<NOB>(sbf, a.w[l], a.b[l], T, a.out[l]);
}
}  // namespace x2g

X2G_API int x2g_sbf_project(const float* sbf, int64_t T, int32_t sbf_dim, const float* w_sbf, const float* b_sbf,
                            int32_t out_dim, float* sbfproj, void* stream) {
  if (T < 0 || out_dim <= 0 || sbf_dim <= 0) return X2G_EINVAL;
  // other basis sizes (e.g. the reference's default F_B_2D(7, 16): sbf_dim 112) take the generic
  // fused dense kernels (x2g_dense_fwd: any K, N; no activation, no residual)
  if (sbf_dim != kS) return x2g_dense_fwd(sbf, w_sbf, b_sbf, T, sbf_dim, out_dim, 0, nullptr, sbfproj, nullptr, stream);
  if (T == 0) return X2G_OK;
  if (!sbf || !w_sbf || !b_sbf || !sbfproj) return X2G_EINVAL;
  hipStream_t st = as_stream(stream);
  // wave-independent f32 MFMA kernel (out_dim 128 or 64, 16-byte aligned sbf and output)
  if ((out_dim == 128 || out_dim == 64) && reinterpret_cast<uintptr_t>(sbf) % 16 == 0 &&
      reinterpret_cast<uintptr_t>(sbfproj) % 16 == 0) {
    const int64_t nblk = (T + 15) / 16;
    int64_t want = (nblk + kSPWaves - 1) / kSPWaves;
    want = want < 256 ? want : 256;  // one 1024-thread workgroup per CU, each wave looping over its blocks
    if (out_dim == 128)
      sbf_project_waves<8><<<static_cast<unsigned>(want), kSPWaves * 64, 0, st>>>(sbf, w_sbf, b_sbf, T, sbfproj);
    else
      sbf_project_waves<4><<<static_cast<unsigned>(want), kSPWaves * 64, 0, st>>>(sbf, w_sbf, b_sbf, T, sbfproj);
    return last_launch_status();
  }
  // f32 MFMA, tiles staged through LDS (dense.hip): that kernel covers N <= 128 output columns
  // and addresses rows with 32-bit offsets; wider projections take the per-row kernel below
  if (out_dim % 4 == 0 && out_dim <= 128 && T * 128 * 4 < (int64_t(1) << 31) &&
      reinterpret_cast<uintptr_t>(sbf) % 16 == 0 && reinterpret_cast<uintptr_t>(sbfproj) % 16 == 0)
    return dense_fwd_narrow_launch(sbf, w_sbf, b_sbf, nullptr, T, kS, out_dim, 0, sbfproj, nullptr, st);
  int64_t want = (T + kAttnWaves - 1) / kAttnWaves;
  const unsigned blocks = static_cast<unsigned>(want < 4096 ? want : 4096);
  switch (out_dim) {
    case 32: case 64: sbf_project_kernel<1><<<blocks, 256, 0, st>>>(sbf, w_sbf, b_sbf, T, out_dim, sbfproj); break;
    case 128: sbf_project_kernel<2><<<blocks, 256, 0, st>>>(sbf, w_sbf, b_sbf, T, out_dim, sbfproj); break;
    case 256: sbf_project_kernel<4><<<blocks, 256, 0, st>>>(sbf, w_sbf, b_sbf, T, out_dim, sbfproj); break;
    default: return X2G_EUNSUPPORTED;
  }
  return last_launch_status();
}

X2G_API int x2g_sbf_project_batch(const float* sbf, int64_t T, int32_t sbf_dim, const float* const* w_sbf,
                                  const float* const* b_sbf, int32_t n_layers, int32_t out_dim, float* const* sbfproj,
                                  void* stream) {
  if (T < 0 || out_dim <= 0 || sbf_dim <= 0 || n_layers < 1 || n_layers > kSPMaxLayers || !w_sbf || !b_sbf ||
      !sbfproj)
    return X2G_EINVAL;
  if (T == 0) return X2G_OK;
  bool fused = sbf_dim == kS && out_dim == 128 && sbf && reinterpret_cast<uintptr_t>(sbf) % 16 == 0;
  SPBatch a{};
  for (int l = 0; l < n_layers; ++l) {
    if (!w_sbf[l] || !b_sbf[l] || !sbfproj[l]) return X2G_EINVAL;
    fused = fused && reinterpret_cast<uintptr_t>(sbfproj[l]) % 16 == 0;
    a.w[l] = w_sbf[l];
    a.b[l] = b_sbf[l];
    a.out[l] = sbfproj[l];
  }
  if (!fused) {  // other shapes / alignments: the single-layer entry per layer (same arithmetic)
    for (int l = 0; l < n_layers; ++l)
      if (int rc = x2g_sbf_project(sbf, T, sbf_dim, w_sbf[l], b_sbf[l], out_dim, sbfproj[l], stream)) return rc;
    return X2G_OK;
  }
  const int64_t nblk = (T + 15) / 16;
  int64_t want = (nblk + kSPWaves - 1) / kSPWaves;
  want = want < 256 ? want : 256;
  sbf_project_waves_batch<8><<<dim3(static_cast<unsigned>(want), static_cast<unsigned>(n_layers)), kSPWaves * 64, 0,
                                as_stream(stream)>>>(sbf, a, T);
  return last_launch_status();
}

// ------------------------------------------------------------------------------ factorised backward
namespace x2g {

struct FoldArgs {
  const float *q, *k, *v, *edge;
  const int32_t* edge_row;
  int edge_rows;
  int mode;
  const float *sp, *y;
  const int32_t *rowptr, *tidx, *tdst;
  const int32_t *sdst, *src_row;  // source pass: destination per source-major position / edge row per source
  const float *alpha, *smax, *sden, *prob, *rho_in, *g_in, *dout;
  int64_t E, T;
  int D, H;
  float sqrt_c;
  float *dq, *d_edge, *g_out, *prob_out, *rho_out, *dk, *dv, *gfold;
};

template <int CPL, int LPH>
void fold_launch_mode(bool dst, const FoldArgs& a, unsigned blocks, hipStream_t st) {
  if (dst) {  // destination-major pass
    if (a.mode == X2G_EDGE_PER_DST)
      attn_bwd_dst_g_batched<CPL, LPH, X2G_EDGE_PER_DST><<<blocks, 256, 0, st>>>(
          a.q, a.k, a.v, a.edge, a.edge_row, a.sp, a.rowptr, a.tidx, a.alpha, a.smax, a.sden, a.dout, a.E, a.T, a.D,
          a.H, a.sqrt_c, a.dq, a.d_edge, a.g_out, a.prob_out, a.rho_out);
    else
      attn_bwd_dst_g_batched<CPL, LPH, X2G_EDGE_NONE><<<blocks, 256, 0, st>>>(
          a.q, a.k, a.v, a.edge, a.edge_row, a.sp, a.rowptr, a.tidx, a.alpha, a.smax, a.sden, a.dout, a.E, a.T, a.D,
          a.H, a.sqrt_c, a.dq, a.d_edge, a.g_out, a.prob_out, a.rho_out);
  } else {  // source-major pass
    const int C = a.D / a.H;
#define X2G_SRC_FOLD(TABLE, SROW, GIN)                                                                           \
  attn_bwd_src_fold_batched<CPL, LPH, TABLE, SROW, GIN><<<blocks, 256, 0, st>>>(                                 \
      a.q, a.v, a.edge, a.edge_row, a.src_row, a.edge_rows, a.sp, a.y, a.rowptr, a.tidx, a.sdst, a.tdst, a.prob,   \
      a.rho_in, a.g_in, a.dout, a.E, a.D, a.H, C, a.dk, a.dv, a.gfold)
    const bool gin = a.g_in != nullptr;
    if (a.mode == X2G_EDGE_PER_DST) {
      if (a.src_row) {
        if (gin) X2G_SRC_FOLD(true, true, true); else X2G_SRC_FOLD(true, true, false);
      } else {
        if (gin) X2G_SRC_FOLD(true, false, true); else X2G_SRC_FOLD(true, false, false);
      }
    } else {
      if (gin) X2G_SRC_FOLD(false, false, true); else X2G_SRC_FOLD(false, false, false);
    }
#undef X2G_SRC_FOLD
  }
}

int fold_dispatch(bool dst, FoldArgs a, int heads, int channels, hipStream_t st) {
  if (a.E < 0 || heads <= 0 || channels <= 0) return X2G_EINVAL;
  if (a.mode != X2G_EDGE_NONE && a.mode != X2G_EDGE_PER_DST) return X2G_EUNSUPPORTED;
  const int D = heads * channels;
  int cpl;
  if (D == 32 || D == 64) cpl = 1;
  else if (D == 128) cpl = 2;
  else if (D == 256) cpl = 4;
  else return X2G_EUNSUPPORTED;
  if (channels % cpl) return X2G_EUNSUPPORTED;
  const int lph = channels / cpl;
  a.D = D;
  a.H = heads;
  a.sqrt_c = static_cast<float>(sqrt(static_cast<double>(channels)));
  if (a.E == 0) return X2G_OK;
  int64_t want = (a.E + kAttnWaves - 1) / kAttnWaves;
  want = want < kMaxBlocks ? want : kMaxBlocks;
  const unsigned blocks = static_cast<unsigned>((want + 7) / 8 * 8);
  const int key = cpl * 100 + lph;
  switch (key) {
    case 102: fold_launch_mode<1, 2>(dst, a, blocks, st); break;
    case 104: fold_launch_mode<1, 4>(dst, a, blocks, st); break;
    case 108: fold_launch_mode<1, 8>(dst, a, blocks, st); break;
    case 116: fold_launch_mode<1, 16>(dst, a, blocks, st); break;
    case 202: fold_launch_mode<2, 2>(dst, a, blocks, st); break;
    case 204: fold_launch_mode<2, 4>(dst, a, blocks, st); break;
    case 208: fold_launch_mode<2, 8>(dst, a, blocks, st); break;
    case 401: fold_launch_mode<4, 1>(dst, a, blocks, st); break;
    case 402: fold_launch_mode<4, 2>(dst, a, blocks, st); break;
    case 404: fold_launch_mode<4, 4>(dst, a, blocks, st); break;
    case 408: fold_launch_mode<4, 8>(dst, a, blocks, st); break;
    default: return X2G_EUNSUPPORTED;
  }
  return last_launch_status();
}

}  // namespace x2g

X2G_API int x2g_sbf_attention_bwd_dst_g(const float* q, const float* k, const float* v, const float* edge,
                                        const int32_t* edge_row, int edge_mode, const float* sbfproj,
                                        const int32_t* trip_rowptr, const int32_t* trip_src, const float* alpha_raw,
                                        const float* seg_max, const float* seg_den, const float* dout, int64_t E,
                                        int64_t T, int32_t heads, int32_t channels, float* dq, float* d_edge,
                                        float* g_out, float* prob_out, float* seg_rho, void* stream) {
  if (E > 0 && (!q || !k || !v || !sbfproj || !trip_rowptr || !seg_max || !seg_den || !dout || !dq || !seg_rho))
    return X2G_EINVAL;
  if (T > 0 && (!trip_src || !alpha_raw || !prob_out)) return X2G_EINVAL;  // g_out may be NULL
  if (edge_mode != X2G_EDGE_NONE && (!edge || !d_edge)) return X2G_EINVAL;
  FoldArgs a{};
  a.q = q; a.k = k; a.v = v; a.edge = edge; a.edge_row = edge_row; a.mode = edge_mode; a.sp = sbfproj;
  a.rowptr = trip_rowptr; a.tidx = trip_src; a.alpha = alpha_raw; a.smax = seg_max; a.sden = seg_den; a.dout = dout;
  a.E = E; a.T = T; a.dq = dq; a.d_edge = d_edge; a.g_out = g_out; a.prob_out = prob_out; a.rho_out = seg_rho;
  return fold_dispatch(true, a, heads, channels, as_stream(stream));
}

X2G_API int x2g_sbf_attention_bwd_src_fold(const float* q, const float* v, const float* edge, const int32_t* edge_row,
                                           const int32_t* src_row, int32_t edge_rows, int edge_mode,
                                           const float* sbfproj, const float* sph_y, const int32_t* src_rowptr,
                                           const int32_t* src_perm, const int32_t* src_dst, const int32_t* trip_dst,
                                           const float* prob, const float* g_in, const float* seg_rho,
                                           const float* dout, int64_t E, int64_t T, int32_t heads, int32_t channels,
                                           float* dk, float* dv, float* radial_grad, void* stream) {
  if (E > 0 && (!q || !v || !sbfproj || !src_rowptr || !seg_rho || !dout || !dk || !dv || !radial_grad))
    return X2G_EINVAL;
  if (T > 0 && (!src_perm || (!trip_dst && !src_dst) || !prob || !sph_y)) return X2G_EINVAL;  // g_in may be NULL
  // the source pass reads the edge term from a small table staged in LDS (X2-GNN's element table)
  if (edge_mode == X2G_EDGE_PER_DST && (!edge || !edge_row || edge_rows < 1 || edge_rows > kFoldTableRows))
    return X2G_EUNSUPPORTED;
  if (T > 0x7fffffff || E > 0x7fffffff) return X2G_EUNSUPPORTED;  // int32 triplet ids in the prefetch sets
  FoldArgs a{};
  a.q = q; a.v = v; a.edge = edge; a.edge_row = edge_row; a.edge_rows = edge_rows; a.mode = edge_mode;
  a.sp = sbfproj; a.y = sph_y; a.rowptr = src_rowptr; a.tidx = src_perm; a.tdst = trip_dst; a.prob = prob;
  a.sdst = src_dst; a.src_row = edge_mode == X2G_EDGE_PER_DST ? src_row : nullptr;
  a.rho_in = seg_rho; a.g_in = g_in; a.dout = dout; a.E = E; a.dk = dk; a.dv = dv; a.gfold = radial_grad;
  return fold_dispatch(false, a, heads, channels, as_stream(stream));
}

X2G_API int32_t x2g_sbf_radial_wgrad_splits(int64_t E) { return radial_splits(E); }

X2G_API size_t x2g_sbf_radial_wgrad_workspace(int64_t E, int32_t D) {
  if (E <= 0 || D <= 0) return 0;
  return static_cast<size_t>(radial_splits(E)) * (static_cast<int64_t>(D) * kS + D) * sizeof(float);
}

X2G_API int x2g_sbf_radial_wgrad(const float* radial_grad, const float* radial, int64_t E, int32_t D, float* dw,
                                 float* db, int flags, void* workspace, size_t workspace_bytes, void* stream) {
  if (E < 0 || !dw || !db || (flags & ~(X2G_ACCUM_WGRAD | X2G_DEFER_SLAB_SUM))) return X2G_EINVAL;
  if (D != 32 && D != 64 && D != 128) return X2G_EUNSUPPORTED;  // blockDim = 2 D threads
  const bool accum = flags & X2G_ACCUM_WGRAD;
  if ((flags & X2G_DEFER_SLAB_SUM) && E == 0) return X2G_EINVAL;
  hipStream_t st = as_stream(stream);
  if (E == 0) {
    if (accum) return X2G_OK;
    hipError_t e = hipMemsetAsync(dw, 0, sizeof(float) * D * kS, st);
    if (e == hipSuccess) e = hipMemsetAsync(db, 0, sizeof(float) * D, st);
    return e == hipSuccess ? X2G_OK : static_cast<int>(e);
  }
  if (!radial_grad || !radial) return X2G_EINVAL;
  if (!workspace || workspace_bytes < x2g_sbf_radial_wgrad_workspace(E, D)) return X2G_EWORKSPACE;
  const int splits = radial_splits(E);
  const int64_t rps = radial_rows_per_split(E);
  float* part_w = static_cast<float*>(workspace);
  float* part_b = part_w + static_cast<int64_t>(splits) * D * kS;
  sbf_radial_wgrad_kernel<kRadialVpt>
      <<<splits, 8 * D / kRadialVpt * kRadialGroups, 0, st>>>(radial_grad, radial, E, D, rps, part_w, part_b);
  if (int rc = last_launch_status()) return rc;
  if (flags & X2G_DEFER_SLAB_SUM) return X2G_OK;
  return sum_slabs_launch(part_w, static_cast<int64_t>(D) * kS, part_b, D, splits, dw, db, accum, st);
}
