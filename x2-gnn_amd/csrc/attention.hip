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
#include <math.h>

#include "common.hpp"

namespace x2g {

constexpr int kS = 42;           // sbf_dim compiled in (7 spherical x 6 radial)
constexpr int kAttnWaves = 4;    // waves per 256-thread block
constexpr int kMaxBlocks = 2048; // persistent-ish grid: waves grid-stride over line nodes
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
  int D;
  int H;
  float sqrt_c;
  float* out;
  float* alpha_out;
  float* smax_out;
  float* sden_out;
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

// Every kernel below takes its pointers as __restrict__ parameters: with them the compiler may
// serve wave-uniform reads (row pointers, triplet indices, the sbf row) from the scalar cache.

// ------------------------------------------------------------------------------ forward
template <int CPL, int LPH, int MODE>
__global__ void __launch_bounds__(256) attn_fwd_kernel(
    const float* __restrict__ q, const float* __restrict__ k, const float* __restrict__ v,
    const float* __restrict__ skip, const float* __restrict__ edge, const int32_t* __restrict__ edge_row,
    const float* __restrict__ sbf, const float* __restrict__ w, const float* __restrict__ b,
    const int32_t* __restrict__ rowptr, const int32_t* __restrict__ tsrc, int64_t E, int D, int H, float sqrt_c,
    float* __restrict__ out, float* __restrict__ alpha_out, float* __restrict__ smax_out,
    float* __restrict__ sden_out) {
  const int lane = threadIdx.x & 63;
  const bool act = lane * CPL < D;
  const int c0 = act ? lane * CPL : 0;
  const int head = lane / LPH;
  const bool leader = act && (lane % LPH) == 0;
  float wr[CPL][kS], br[CPL];
  load_weights<CPL>(w, b, c0, act, wr, br);
  const WaveRange wr_ = xcd_wave_range(E);
  for (int64_t e = wr_.first; e < wr_.end; e += wr_.stride) {
    const int t0 = uniform(rowptr[e]), t1 = uniform(rowptr[e + 1]);
    float qv[CPL], ed[CPL], acc[CPL];
    load_row<CPL>(q + e * D + c0, act, qv);
    if (MODE == X2G_EDGE_PER_DST) {
      const int64_t r = edge_row ? uniform(edge_row[e]) : e;
      load_row<CPL>(edge + r * D + c0, act, ed);
    } else {
      zero_row<CPL>(ed);
    }
    zero_row<CPL>(acc);
    float m = -INFINITY, den = 0.f;
    // two triplets' neighbour rows in flight ahead of the one being consumed
    float k0[CPL], v0[CPL], k1[CPL], v1[CPL];
    zero_row<CPL>(k0); zero_row<CPL>(v0); zero_row<CPL>(k1); zero_row<CPL>(v1);
    if (t0 < t1) {
      const int64_t s = uniform(tsrc[t0]);
      load_row<CPL>(k + s * D + c0, act, k0);
      load_row<CPL>(v + s * D + c0, act, v0);
    }
    if (t0 + 1 < t1) {
      const int64_t s = uniform(tsrc[t0 + 1]);
      load_row<CPL>(k + s * D + c0, act, k1);
      load_row<CPL>(v + s * D + c0, act, v1);
    }
    for (int t = t0; t < t1; ++t) {
      float k2[CPL], v2[CPL];
      zero_row<CPL>(k2); zero_row<CPL>(v2);
      if (t + 2 < t1) {
        const int64_t s = uniform(tsrc[t + 2]);
        load_row<CPL>(k + s * D + c0, act, k2);
        load_row<CPL>(v + s * D + c0, act, v2);
      }
      float et[CPL];
      if (MODE == X2G_EDGE_PER_TRIPLET) {
        load_row<CPL>(edge + static_cast<int64_t>(t) * D + c0, act, et);
      } else {
#pragma unroll
        for (int j = 0; j < CPL; ++j) et[j] = ed[j];
      }
      float dot = 0.f;
#pragma unroll
      for (int j = 0; j < CPL; ++j) dot = fmaf(qv[j], k0[j] + et[j], dot);
      const float logit = group_sum<LPH>(dot) / sqrt_c;
      float sp[CPL];
      sbf_project<CPL>(wr, br, sbf + static_cast<int64_t>(t) * kS, sp);
      const float m_new = fmaxf(m, logit);
      const float corr = expf(m - m_new);
      const float p = expf(logit - m_new);
      den = den * corr + p;
#pragma unroll
      for (int j = 0; j < CPL; ++j) acc[j] = acc[j] * corr + p * ((v0[j] + et[j]) * sp[j]);
      m = m_new;
      if (leader) alpha_out[static_cast<int64_t>(t) * H + head] = logit;
#pragma unroll
      for (int j = 0; j < CPL; ++j) {
        k0[j] = k1[j]; v0[j] = v1[j];
        k1[j] = k2[j]; v1[j] = v2[j];
      }
    }
    float sk[CPL], o[CPL];
    load_row<CPL>(skip + e * D + c0, act, sk);
    const float inv = 1.0f / (den + kSoftmaxEps);
#pragma unroll
    for (int j = 0; j < CPL; ++j) o[j] = acc[j] * inv + sk[j];
    store_row<CPL>(out + e * D + c0, act, o);
    if (leader) {
      smax_out[e * H + head] = m;
      sden_out[e * H + head] = den;
    }
  }
}

// ------------------------------------------------------------------------------ backward (dst)
template <int CPL, int LPH, int MODE>
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
  constexpr bool per_trip = MODE == X2G_EDGE_PER_TRIPLET;
  constexpr bool per_dst = MODE == X2G_EDGE_PER_DST;
  float wr[CPL][kS], br[CPL];
  load_weights<CPL>(w, b, c0, act, wr, br);
  const WaveRange wr_ = xcd_wave_range(E);
  for (int64_t e = wr_.first; e < wr_.end; e += wr_.stride) {
    const int t0 = uniform(rowptr[e]), t1 = uniform(rowptr[e + 1]);
    float go[CPL], qv[CPL], ed[CPL], edacc[CPL], dqa[CPL];
    load_row<CPL>(dout + e * D + c0, act, go);
    load_row<CPL>(q + e * D + c0, act, qv);
    if (per_dst) {
      const int64_t r = edge_row ? uniform(edge_row[e]) : e;
      load_row<CPL>(edge + r * D + c0, act, ed);
    } else {
      zero_row<CPL>(ed);
    }
    zero_row<CPL>(edacc);
    zero_row<CPL>(dqa);
    const float mx = keep(smax[e * H + head], act);
    const float inv = act ? 1.0f / (sden[e * H + head] + kSoftmaxEps) : 0.f;
    // pass 1: g_t = d(loss)/d(a_t) per head, rho = sum_t a_t g_t; d_sbfproj and the value part
    float rho = 0.f;
    float vn[CPL];
    zero_row<CPL>(vn);
    if (t0 < t1) load_row<CPL>(v + static_cast<int64_t>(uniform(tsrc[t0])) * D + c0, act, vn);
    for (int t = t0; t < t1; ++t) {
      float vv[CPL], et[CPL], sp[CPL];
#pragma unroll
      for (int j = 0; j < CPL; ++j) vv[j] = vn[j];
      if (t + 1 < t1) load_row<CPL>(v + static_cast<int64_t>(uniform(tsrc[t + 1])) * D + c0, act, vn);
      if (per_trip) {
        load_row<CPL>(edge + static_cast<int64_t>(t) * D + c0, act, et);
      } else {
#pragma unroll
        for (int j = 0; j < CPL; ++j) et[j] = ed[j];
      }
      sbf_project<CPL>(wr, br, sbf + static_cast<int64_t>(t) * kS, sp);
      const float at = act ? expf(alpha[static_cast<int64_t>(t) * H + head] - mx) * inv : 0.f;
      float gpart = 0.f, dp[CPL], du[CPL];
#pragma unroll
      for (int j = 0; j < CPL; ++j) {
        const float u = vv[j] + et[j];
        gpart = fmaf(go[j] * u, sp[j], gpart);
        dp[j] = go[j] * u * at;
        du[j] = go[j] * sp[j] * at;
      }
      const float g = group_sum<LPH>(gpart);
      rho = fmaf(at, g, rho);
      store_row<CPL>(dproj + static_cast<int64_t>(t) * D + c0, act, dp);
      if (per_trip) {
        store_row<CPL>(d_edge + static_cast<int64_t>(t) * D + c0, act, du);
      } else {
#pragma unroll
        for (int j = 0; j < CPL; ++j) edacc[j] += du[j];
      }
      if (leader) dlogit[static_cast<int64_t>(t) * H + head] = g;
    }
    // pass 2: dlogit = a (g - rho); dq, and the key part of the edge gradient
    float kn[CPL];
    zero_row<CPL>(kn);
    if (t0 < t1) load_row<CPL>(k + static_cast<int64_t>(uniform(tsrc[t0])) * D + c0, act, kn);
    for (int t = t0; t < t1; ++t) {
      float kk[CPL], et[CPL];
#pragma unroll
      for (int j = 0; j < CPL; ++j) kk[j] = kn[j];
      if (t + 1 < t1) load_row<CPL>(k + static_cast<int64_t>(uniform(tsrc[t + 1])) * D + c0, act, kn);
      if (per_trip) {
        load_row<CPL>(edge + static_cast<int64_t>(t) * D + c0, act, et);
      } else {
#pragma unroll
        for (int j = 0; j < CPL; ++j) et[j] = ed[j];
      }
      const float at = act ? expf(alpha[static_cast<int64_t>(t) * H + head] - mx) * inv : 0.f;
      // only the leader lane wrote g for this head: read it back in that lane, then broadcast
      const float g = group_sum<LPH>(leader ? dlogit[static_cast<int64_t>(t) * H + head] : 0.f);
      const float dl = at * (g - rho);
      const float ds = dl / sqrt_c;
      float dk[CPL];
#pragma unroll
      for (int j = 0; j < CPL; ++j) {
        dqa[j] = fmaf(ds, kk[j] + et[j], dqa[j]);
        dk[j] = ds * qv[j];
      }
      if (per_trip) {
        float cur[CPL];
        load_row<CPL>(d_edge + static_cast<int64_t>(t) * D + c0, act, cur);
#pragma unroll
        for (int j = 0; j < CPL; ++j) cur[j] += dk[j];
        store_row<CPL>(d_edge + static_cast<int64_t>(t) * D + c0, act, cur);
      } else {
#pragma unroll
        for (int j = 0; j < CPL; ++j) edacc[j] += dk[j];
      }
      if (leader) dlogit[static_cast<int64_t>(t) * H + head] = dl;
    }
    store_row<CPL>(dq + e * D + c0, act, dqa);
    if (per_dst) store_row<CPL>(d_edge + e * D + c0, act, edacc);
  }
}

// ------------------------------------------------------------------------------ backward (src)
template <int CPL, int LPH>
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
  float wr[CPL][kS], br[CPL];
  load_weights<CPL>(w, b, c0, act, wr, br);
  const WaveRange wr_ = xcd_wave_range(E);
  for (int64_t s = wr_.first; s < wr_.end; s += wr_.stride) {
    const int p0 = uniform(rowptr[s]), p1 = uniform(rowptr[s + 1]);
    float dka[CPL], dva[CPL];
    zero_row<CPL>(dka);
    zero_row<CPL>(dva);
    // next triplet's gathered rows (dout, q of its destination) in flight
    float gn[CPL], qn[CPL];
    zero_row<CPL>(gn);
    zero_row<CPL>(qn);
    int64_t tn = 0, en = 0;
    if (p0 < p1) {
      tn = uniform(perm[p0]);
      en = uniform(tdst[tn]);
      load_row<CPL>(dout + en * D + c0, act, gn);
      load_row<CPL>(q + en * D + c0, act, qn);
    }
    for (int p = p0; p < p1; ++p) {
      const int64_t t = tn, e = en;
      float go[CPL], qv[CPL], sp[CPL];
#pragma unroll
      for (int j = 0; j < CPL; ++j) {
        go[j] = gn[j];
        qv[j] = qn[j];
      }
      if (p + 1 < p1) {
        tn = uniform(perm[p + 1]);
        en = uniform(tdst[tn]);
        load_row<CPL>(dout + en * D + c0, act, gn);
        load_row<CPL>(q + en * D + c0, act, qn);
      }
      float at = 0.f, dl = 0.f;
      if (act) {
        const float mx = smax[e * H + head];
        const float inv = 1.0f / (sden[e * H + head] + kSoftmaxEps);
        at = expf(alpha[t * H + head] - mx) * inv;
        dl = dlogit_in[t * H + head];
      }
      sbf_project<CPL>(wr, br, sbf + t * kS, sp);
      const float ds = dl / sqrt_c;
#pragma unroll
      for (int j = 0; j < CPL; ++j) {
        dva[j] = fmaf(go[j] * sp[j], at, dva[j]);
        dka[j] = fmaf(ds, qv[j], dka[j]);
      }
    }
    store_row<CPL>(dk + s * D + c0, act, dka);
    store_row<CPL>(dv + s * D + c0, act, dva);
  }
}

// ------------------------------------------------------------------------------ dispatch
enum class Pass { kFwd, kBwdDst, kBwdSrc };

template <int CPL, int LPH, int MODE>
void launch_mode(Pass pass, const AttnArgs& a, unsigned blocks, hipStream_t st) {
  switch (pass) {
    case Pass::kFwd:
      attn_fwd_kernel<CPL, LPH, MODE><<<blocks, 256, 0, st>>>(a.q, a.k, a.v, a.skip, a.edge, a.edge_row, a.sbf, a.w,
                                                              a.b, a.rowptr, a.tidx, a.E, a.D, a.H, a.sqrt_c, a.out,
                                                              a.alpha_out, a.smax_out, a.sden_out);
      break;
    case Pass::kBwdDst:
      attn_bwd_dst_kernel<CPL, LPH, MODE><<<blocks, 256, 0, st>>>(
          a.q, a.k, a.v, a.edge, a.edge_row, a.sbf, a.w, a.b, a.rowptr, a.tidx, a.alpha, a.smax, a.sden, a.dout,
          a.E, a.D, a.H, a.sqrt_c, a.dq, a.d_edge, a.dlogit, a.dproj);
      break;
    case Pass::kBwdSrc:
      attn_bwd_src_kernel<CPL, LPH><<<blocks, 256, 0, st>>>(a.q, a.sbf, a.w, a.b, a.rowptr, a.tidx, a.tdst, a.alpha,
                                                            a.smax, a.sden, a.dlogit_in, a.dout, a.E, a.D, a.H,
                                                            a.sqrt_c, a.dk, a.dv);
      break;
  }
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
  if (sbf_dim != kS) return X2G_EUNSUPPORTED;
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
  if (E > 0 && (!q || !k || !v || !skip || !sbf || !w_sbf || !b_sbf || !trip_rowptr || !out || !seg_max ||
                !seg_den))
    return X2G_EINVAL;
  if (T > 0 && (!trip_src || !alpha_raw)) return X2G_EINVAL;
  if (edge_mode != X2G_EDGE_NONE && !edge) return X2G_EINVAL;
  AttnArgs a{};
  a.q = q; a.k = k; a.v = v; a.skip = skip; a.edge = edge; a.edge_row = edge_row; a.edge_mode = edge_mode;
  a.sbf = sbf; a.w = w_sbf; a.b = b_sbf; a.rowptr = trip_rowptr; a.tidx = trip_src; a.E = E;
  a.out = out; a.alpha_out = alpha_raw; a.smax_out = seg_max; a.sden_out = seg_den;
  return dispatch(Pass::kFwd, a, heads, channels, sbf_dim, as_stream(stream));
}

X2G_API int x2g_sbf_attention_bwd_dst(const float* q, const float* k, const float* v, const float* edge,
                                      const int32_t* edge_row, int edge_mode, const float* sbf,
                                      const float* w_sbf, const float* b_sbf, const int32_t* trip_rowptr,
                                      const int32_t* trip_src, const float* alpha_raw, const float* seg_max,
                                      const float* seg_den, const float* dout, int64_t E, int64_t T,
                                      int32_t heads, int32_t channels, int32_t sbf_dim, float* dq,
                                      float* d_edge, float* dlogit, float* d_sbfproj, void* stream) {
  if (E > 0 && (!q || !k || !v || !sbf || !w_sbf || !b_sbf || !trip_rowptr || !seg_max || !seg_den || !dout ||
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
  if (E > 0 && (!q || !sbf || !w_sbf || !b_sbf || !src_rowptr || !seg_max || !seg_den || !dout || !dk || !dv))
    return X2G_EINVAL;
  if (T > 0 && (!src_perm || !trip_dst || !alpha_raw || !dlogit)) return X2G_EINVAL;
  AttnArgs a{};
  a.q = q; a.sbf = sbf; a.w = w_sbf; a.b = b_sbf; a.rowptr = src_rowptr; a.tidx = src_perm; a.tdst = trip_dst;
  a.alpha = alpha_raw; a.smax = seg_max; a.sden = seg_den; a.dlogit_in = dlogit; a.dout = dout; a.E = E;
  a.dk = dk; a.dv = dv;
  return dispatch(Pass::kBwdSrc, a, heads, channels, sbf_dim, as_stream(stream));
}
