// Center-atom SBF-transformer attention (symmetric line graphs: every molecular batch).
//
// Reference: SBFTransformerConv.forward / message (sbftransformer_conv.py:93-162) over the triplets
// vertex_to_edge_2 emits (edge_graph.py:12-30).  A triplet (s -> d) joins destination d = (a -> b) and
// source s = (b -> k), k != a: every triplet has a middle ("center") atom b, and the triplets through b
// are the complete bipartite block {(b -> k_j) -> (k_i -> b) : i != j} over b's n = deg(b) neighbours.
// Grouped by center atom instead of by destination, a workgroup owns one atom b and all of its n (n - 1)
// triplets:
//   * the n source rows of k and v are b's out-edges, CONTIGUOUS line nodes atom_rowptr[b] .. +n: loaded
//     once, coalesced, into LDS (k + e and v + e: X2-GNN's edge term is the element-table row of the
//     center atom, xgnn.py:57-58, uniform over the block), instead of being gathered from L2 once per
//     triplet (8 times each at config 2) by one-destination-per-wave kernels;
//   * destination i = rev(b -> k_i) owns the contiguous triplet rows rev_trip[b -> k_i] + 0 .. n - 2
//     (vertex_to_edge_2's order: sources ascending, the reverse edge skipped), read as one S stream.
// A destination is owned by a HALF wave (32 lanes x 4 channels = D = 128, LPH lanes per head), so a
// 16-byte load moves two destinations' rows per instruction and the per-head softmax arithmetic runs on
// 2 lanes per head instead of 4.  Both halves walk j = 0 .. n-1 in lockstep (each masks its own j == i),
// so their LDS row reads are the same address (broadcast).  Online softmax per batch of B triplets (one
// running-max rescale per batch); fixed order (j ascending), no atomics.
//
// Needs x2g_vertex_to_edge_sym's / x2g_line_graph_sym_build's edge_rev and rev_trip.
#include <math.h>

#include <type_traits>

#include "common.hpp"

namespace x2g {
namespace {

constexpr int kCD = 128;  // D compiled (H * C)
constexpr float kCEps = 1e-16f;
typedef float cf4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ cf4 ld4(const float* p) { return *reinterpret_cast<const cf4*>(p); }
__device__ __forceinline__ void st4(float* p, cf4 v) { *reinterpret_cast<cf4*>(p) = v; }

// sum over the LPH lanes of a head (aligned groups inside a half wave)
template <int LPH>
__device__ __forceinline__ float head_sum(float v) {
  return group_sum<LPH>(v);
}

// a head's logit q . kr / sqrt C over its LPH lanes, in one fixed arithmetic (explicitly rounded product and
// fmas: no contraction choice left to the compiler), so that every forward and the backward that recomputes
// it (x2g_sbf_attention_bwd_center from P rows) produce the same bits
template <int LPH>
__device__ __forceinline__ float qk_logit(cf4 qv, cf4 kr, float sqrt_c) {
  float dot = __fmul_rn(qv[0], kr[0]);
  dot = __fmaf_rn(qv[1], kr[1], dot);
  dot = __fmaf_rn(qv[2], kr[2], dot);
  dot = __fmaf_rn(qv[3], kr[3], dot);
  return __fdiv_rn(head_sum<LPH>(dot), sqrt_c);
}

// sum over each aligned 32-lane half, in every lane of that half
__device__ __forceinline__ float half_sum(float v, int half) {
  v = half32_sum_hi(v);
  const float lo = lane_bcast(v, 31), hi = lane_bcast(v, 63);
  return half ? hi : lo;
}

// triplets per round trip of the backward's pass 1 when it rebuilds S_t from the P rows (their 28 VGPRs
// live through the source's batches: 8 spills 21 VGPRs, 6 spills 7; 4 spills none and measured best,
// r5q: 55.66k vs 55.46k mol/s at 6)
constexpr int kFactBatch = 4;
constexpr int kSfL = 7;                  // angular orders (sbf_dim 42 = 7 x 6)
constexpr int kSfR = 6;                  // radial functions per order
constexpr int kSfK = kSfL * kSfR;        // 42

// ------------------------------------------------------------------------------ workgroup rows
// A workgroup runs one UNIT: one center atom, or (pack_ptr given) a PACK of center atoms
// order[pack_ptr[u]] .. order[pack_ptr[u + 1] - 1] whose blocks it processes side by side.  A block has
// n = deg(b) rows (b's out-edges, the sources; their reverses, the destinations), and a workgroup has 2 x
// WAVES half-wave owners, so one atom per workgroup leaves owners idle whenever deg(b) is not a multiple
// of the owner count (config 2: degrees 2-17 on 16 owners, 57 % busy); packs of total degree <= 16
// (the host's best-fit decreasing, data.center_packs) keep 90 % of them busy.  Row g of the workgroup
// is line node LN[g] = r0_m + (g - base_m) of member m, whose block is rows base_m .. base_m + n_m - 1:
// RI[g] = base_m | n_m << 16, ER[g] = the member's edge-table row (src_row of its first out-edge: the center
// atom's element).  Every sum keeps its order (sources / destinations ascending within a block), so packed
// and unpacked launches give the same bits.
constexpr int kMaxMembers = 32;  // atoms per pack (wave 0 builds the tables, one lane per member)

struct UnitRows {
  int* LN;   // [rows] line node
  int* RI;   // [rows] base | n << 16
  int* ER;   // [rows] edge-table row
  int* MA;   // [kMaxMembers] member atom
  int* MI;   // [kMaxMembers] member base | n << 16
  int* NRS;  // [2] rows, members
};

__host__ __device__ constexpr size_t unit_rows_lds(int rows) {  // (a multiple of 16 bytes)
  return ((static_cast<size_t>(3) * rows + 2 * kMaxMembers + 4) * 4 + 15) / 16 * 16;
}

__device__ __forceinline__ UnitRows unit_rows_carve(int* p, int max_rows) {
  UnitRows u;
  u.NRS = p;
  u.MA = p + 4;
  u.MI = u.MA + kMaxMembers;
  u.LN = u.MI + kMaxMembers;
  u.RI = u.LN + max_rows;
  u.ER = u.RI + max_rows;
  return u;
}

// wave 0 fills the tables (the caller synchronises before reading them); src_row may be NULL (ER = 0).
// With info (int32 [.., 4] per atom in the order's positions: atom, first out-edge, degree, edge-table
// row; the host's, data.center_packs) a member's row range is one load instead of three dependent ones
// (order -> rowptr -> src_row).
// A unit of more than max_rows rows (a device-made schedule lists the atoms beyond the LDS image among the
// packs: x2g_sbf_attention_fwd_center_sf_tiled takes them) writes no table entry and reports 0 rows, so
// the workgroup leaves.
__device__ __forceinline__ void unit_rows_build(const UnitRows& u, const int32_t* __restrict__ order,
                                                const int32_t* __restrict__ packs, int64_t unit,
                                                const int32_t* __restrict__ rowptr,
                                                const int32_t* __restrict__ src_row,
                                                const int4* __restrict__ info, int max_rows) {
  if (threadIdx.x >= 64) return;
  const int lane = threadIdx.x;
  int64_t m0 = unit, m1 = unit + 1;
  if (packs) {
    m0 = packs[unit];
    m1 = packs[unit + 1];
  }
  const int M = static_cast<int>(m1 - m0);  // <= kMaxMembers (host contract)
  int b = 0, r0 = 0, n = 0, er = 0;
  if (info) {
    if (lane < M) {
      const int4 v = info[m0 + lane];
      b = v.x;
      r0 = v.y;
      n = v.z;
      er = src_row ? v.w : 0;
    }
  } else {
    if (lane < M) {
      b = order ? order[m0 + lane] : static_cast<int>(m0 + lane);
      r0 = rowptr[b];
      n = rowptr[b + 1] - r0;
    }
    er = (src_row && n > 0) ? src_row[r0] : 0;
  }
  int inc = n;  // inclusive prefix over the members
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int v = __shfl_up(inc, o);
    if (lane >= o) inc += v;
  }
  const int base = inc - n;
  const int total = __shfl(inc, 63);
  if (total > max_rows) {  // (wave-uniform)
    if (lane == 63) {
      u.NRS[0] = 0;
      u.NRS[1] = 0;
    }
    return;
  }
  if (lane < M) {
    u.MA[lane] = b;
    u.MI[lane] = base | n << 16;
    for (int r = 0; r < n; ++r) {
      u.LN[base + r] = r0 + r;
      u.RI[base + r] = base | n << 16;
      u.ER[base + r] = er;
    }
  }
  if (lane == 63) {
    u.NRS[0] = inc;
    u.NRS[1] = M;
  }
}

struct FwdCenterArgs {
  const float *q, *k, *v, *skip, *edge;
  const int32_t* src_row;  // per source line node: its edge-table row (the center atom's element)
  const float* sp;         // S rows, row t - t_base
  int64_t t_base;
  const int32_t *atom_rowptr, *edge_rev, *rev_trip;
  const int32_t* order;  // workgroup -> center atom (NULL: atom0 + blockIdx.x)
  int64_t atom0, n_atoms;
  int H;
  float sqrt_c;
  float *out, *alpha, *smax, *sden;
  float2* row_stats;
};

template <int LPH, int WAVES, int B, bool EDGE>
__global__ void __launch_bounds__(64 * WAVES) attn_fwd_center_kernel(const FwdCenterArgs a) {
  extern __shared__ cf4 lds[];  // [n][32] (k + e), then [n][32] (v + e)
  // (the host orders the atoms by decreasing degree: the longest blocks start first, the short ones fill the
  // tail of the launch)
  const int64_t b = a.order ? static_cast<int64_t>(a.order[a.atom0 + blockIdx.x]) : a.atom0 + blockIdx.x;
  const int r0 = uniform(a.atom_rowptr[b]);
  const int n = uniform(a.atom_rowptr[b + 1]) - r0;
  if (n <= 0) return;  // (workgroup-uniform: no barrier is skipped by a part of it)
  cf4* ke = lds;
  cf4* ve = lds + n * 32;
  const int tid = threadIdx.x;
  const int l32 = tid & 31, half = (tid >> 5) & 1, wave = tid >> 6;
  const int owner = 2 * wave + half;
  const int head = l32 / LPH;
  const bool leader = (l32 % LPH) == 0;
  const int c0 = 4 * l32;
  // this owner's first destination: its id and triplet block (in flight under the staging)
  int i = owner;
  int d = 0, tb = 0;
  if (i < n) {
    d = a.edge_rev[r0 + i];
    tb = a.rev_trip[r0 + i];
  }
  // stage k + e, v + e of the n source rows (contiguous line nodes r0 .. r0 + n - 1)
  cf4 e4 = {0.f, 0.f, 0.f, 0.f};
  for (int idx = tid; idx < n * 32; idx += 64 * WAVES) {
    const int j = idx >> 5, c = idx & 31;
    if (EDGE) e4 = ld4(a.edge + static_cast<int64_t>(uniform(a.src_row[r0])) * kCD + 4 * c);
    const int64_t row = static_cast<int64_t>(r0 + j) * kCD + 4 * c;
    ke[idx] = ld4(a.k + row) + e4;
    ve[idx] = ld4(a.v + row) + e4;
  }
  __syncthreads();
  const int nt = n - 1;  // triplets per destination
  for (; i < n; i += 2 * WAVES) {
    if (i != owner) {
      d = a.edge_rev[r0 + i];
      tb = a.rev_trip[r0 + i];
    }
    const int64_t drow = static_cast<int64_t>(d) * kCD + c0;
    const cf4 qv = ld4(a.q + drow);
    const cf4 sk = ld4(a.skip + drow);
    cf4 acc = {0.f, 0.f, 0.f, 0.f};
    float m = -INFINITY, den = 0.f;
    const float* sbase = a.sp + (static_cast<int64_t>(tb) - a.t_base) * kCD + c0;
    // one batch of BB consecutive sources j0 .. j0 + BB - 1 (those >= n or == i masked): every S row
    // of the batch in flight together, then the logits, one rescale, the weighted values
    auto batch = [&](int j0, auto bb) {
      constexpr int BB = decltype(bb)::value;
      cf4 sv[BB];
#pragma unroll
      for (int u = 0; u < BB; ++u) {
        const int j = j0 + u;
        int jj = j - (j > i ? 1 : 0);
        jj = jj < nt ? jj : nt - 1;  // clamped (nt >= 1 here): every load unconditional
        sv[u] = ld4(sbase + static_cast<int64_t>(jj) * kCD);
      }
      float lg[BB];
      float mb = -INFINITY;
#pragma unroll
      for (int u = 0; u < BB; ++u) {
        const int j = j0 + u;
        const bool ok = j < n && j != i;
        const cf4 kr = ke[(j < n ? j : n - 1) * 32 + l32];
        const float logit = qk_logit<LPH>(qv, kr, a.sqrt_c);
        lg[u] = ok ? logit : -INFINITY;
        mb = fmaxf(mb, lg[u]);
        if (a.alpha && ok && leader) a.alpha[(static_cast<int64_t>(tb) + (j - (j > i ? 1 : 0))) * a.H + head] = logit;
      }
      const float m_new = fmaxf(m, mb);
      const float corr = m_new == -INFINITY ? 1.f : expf(m - m_new);
      den *= corr;
      acc *= corr;
#pragma unroll
      for (int u = 0; u < BB; ++u) {
        const int j = j0 + u;
        const float p = lg[u] == -INFINITY ? 0.f : expf(lg[u] - m_new);
        const cf4 vr = ve[(j < n ? j : n - 1) * 32 + l32];
        den += p;
        acc += p * (vr * sv[u]);
      }
      m = m_new;
    };
    if (nt > 0) {  // (workgroup-uniform)
      int j0 = 0;
      for (; n - j0 > B / 2; j0 += B) batch(j0, std::integral_constant<int, B>{});
      if (j0 < n) batch(j0, std::integral_constant<int, B / 2>{});
    }
    const float inv = 1.0f / (den + kCEps);
    const cf4 o = acc * inv + sk;
    st4(a.out + drow, o);
    if (a.row_stats) {
      const float mu = half_sum(o[0] + o[1] + o[2] + o[3], half) / static_cast<float>(kCD);
      const cf4 dv = o - mu;
      const float q2 = half_sum(dv[0] * dv[0] + dv[1] * dv[1] + dv[2] * dv[2] + dv[3] * dv[3], half);
      if (l32 == 0) a.row_stats[d] = make_float2(mu, q2);
    }
    if (leader) {
      a.smax[static_cast<int64_t>(d) * a.H + head] = m;
      a.sden[static_cast<int64_t>(d) * a.H + head] = den;
    }
  }
}

// ------------------------------------------------------------------------------ forward, fused projection
// The same forward without a materialised S = lin_sbf(sbf) to read: X2-GNN's sbf row is the per-SOURCE
// radial factor times the per-triplet angular one (angular_basis_layer.py:87-91: sbf[t, 6l+n] =
// R[s, 6l+n] Y_l(t)), so
//     S_t[c] = b[c] + sum_l Y_l(t) P_s[l][c],   P_s[l][c] = sum_n W[c][6l+n] R[s, 6l+n],
// and a center atom's block needs P only for its n sources (7 rows of 128 per source, staged in LDS with
// k + e and v + e: 4.5 KB per source), then 7 FMAs per channel per triplet from the triplet's 8-float
// Y row instead of a 512-byte S row.  The separate projection launch (which read sbf [T, 42] and wrote S
// [T, 128]) and this kernel's S reads disappear; when a backward will need S (training), each triplet's
// S row is stored as it is formed (the same 512-byte writes the projection made).
struct FwdSfArgs {
  const float *q, *k, *v, *skip, *edge;
  const int32_t* src_row;
  const float *radial, *y, *w, *bias;  // rbf_env [E, 42], Y [T, 8], lin_sbf weight [128, 42] and bias [128]
  const int32_t *atom_rowptr, *edge_rev, *rev_trip;
  const int32_t* order;  // unit -> center atom(s) (NULL: the identity)
  const int32_t* packs;  // unit u = atoms order[packs[u]] .. order[packs[u + 1] - 1] (NULL: one atom per unit)
  const int4* info;      // per order position: atom, first out-edge, degree, edge-table row (NULL: derived)
  int64_t atom0, n_atoms;  // units atom0 .. atom0 + n_atoms - 1
  int max_rows;            // rows of the largest unit (the LDS image is sized for it)
  int skip_rows;           // source-tiled form: units whose (first) atom has at most this many rows are left out
  int H;
  float sqrt_c;
  float *out, *alpha, *smax, *sden, *sp;  // sp: S [T, 128] out (NULL: not stored)
  float* pp;  // P [E, 7, 128] out (NULL: not stored): the backward's S_t = b + sum_l Y_l(t) P_s[l]
  float2* row_stats;
};

// (4 waves per SIMD, two 8-wave workgroups per CU: at most 128 VGPRs)
template <int LPH, int WAVES, int B, bool EDGE>
__global__ void __launch_bounds__(64 * WAVES, 4) attn_fwd_center_sf_kernel(const FwdSfArgs a) {
  // [tables] then [rows][32] (k + e), [rows][32] (v + e), [rows][7][32] P, [rows][42] R
  extern __shared__ cf4 lds[];
  const UnitRows u = unit_rows_carve(reinterpret_cast<int*>(lds), a.max_rows);
  // (the host orders the units by decreasing work: the longest start first, the short ones fill the tail)
  unit_rows_build(u, a.order, a.packs, a.atom0 + blockIdx.x, a.atom_rowptr, EDGE ? a.src_row : nullptr, a.info,
                  a.max_rows);
  __syncthreads();
  const int n_rows = uniform(u.NRS[0]);
  if (n_rows <= 0) return;  // (workgroup-uniform)
  cf4* KE = lds + unit_rows_lds(a.max_rows) / 16;
  cf4* VE = KE + n_rows * 32;
  cf4* P = VE + n_rows * 32;
  float* RS = reinterpret_cast<float*>(P + n_rows * kSfL * 32);
  constexpr int NT = 64 * WAVES;
  const int tid = threadIdx.x;
  const int l32 = tid & 31, half = (tid >> 5) & 1, wave = tid >> 6;
  const int owner = 2 * wave + half;
  const int head = l32 / LPH;
  const bool leader = (l32 % LPH) == 0;
  const int c0 = 4 * l32;
  // this owner's first destination row: its id and triplet block (in flight under the staging)
  int g = owner;
  int d = 0, tb = 0;
  if (g < n_rows) {
    d = a.edge_rev[u.LN[g]];
    tb = a.rev_trip[u.LN[g]];
  }
  for (int idx = tid; idx < n_rows * 32; idx += NT) {
    const int r = idx >> 5, c = idx & 31;
    const int64_t ln = u.LN[r];
    const cf4 e4 = EDGE ? ld4(a.edge + static_cast<int64_t>(u.ER[r]) * kCD + 4 * c) : cf4{0.f, 0.f, 0.f, 0.f};
    const int64_t row = ln * kCD + 4 * c;
    KE[idx] = ld4(a.k + row) + e4;
    VE[idx] = ld4(a.v + row) + e4;
  }
  // the rows' radial factors (42 floats each) staged too: the P loop below then reads LDS instead of one
  // dependent global round trip per source
  for (int idx = tid; idx < n_rows * kSfK; idx += NT) {
    const int r = idx / kSfK;
    RS[idx] = a.radial[static_cast<int64_t>(u.LN[r]) * kSfK + (idx - r * kSfK)];
  }
  // P[r][l][c] for the unit's sources: thread (group g, order l, channels 4 c4 .. +3) keeps its 4 x 6
  // weights in registers (loaded before the barrier) and walks rows r = pg, pg + NG, ...
  constexpr int NG = NT / 256;  // thread groups of 7 x 32 (the last 32 threads of each 256 idle)
  const int pg = tid / 256, prest = tid % 256;
  const bool pthr = prest < kSfL * 32;
  const int pl = pthr ? prest >> 5 : 0, pc4 = prest & 31;
  float wv[4][kSfR];
#pragma unroll
  for (int cc = 0; cc < 4; ++cc)
#pragma unroll
    for (int r = 0; r < kSfR; ++r) wv[cc][r] = a.w[(4 * pc4 + cc) * kSfK + kSfR * pl + r];
  __syncthreads();
  {
    if (pthr) {
      const int l = pl, c4 = pc4;
      for (int j = pg; j < n_rows; j += NG) {
        const float* rr = RS + j * kSfK + kSfR * l;
        float rv[kSfR];
#pragma unroll
        for (int r = 0; r < kSfR; ++r) rv[r] = rr[r];
        cf4 p;
#pragma unroll
        for (int cc = 0; cc < 4; ++cc) {
          float acc = wv[cc][0] * rv[0];
#pragma unroll
          for (int r = 1; r < kSfR; ++r) acc = fmaf(wv[cc][r], rv[r], acc);
          p[cc] = acc;
        }
        P[(j * kSfL + l) * 32 + c4] = p;
      }
    }
  }
  const cf4 bias4 = ld4(a.bias + c0);
  // the first destination row's q and skip rows in flight under the P products
  cf4 qv = {0.f, 0.f, 0.f, 0.f}, sk = {0.f, 0.f, 0.f, 0.f};
  if (g < n_rows) {
    qv = ld4(a.q + static_cast<int64_t>(d) * kCD + c0);
    sk = ld4(a.skip + static_cast<int64_t>(d) * kCD + c0);
  }
  __syncthreads();
  for (; g < n_rows; g += 2 * WAVES) {
    const int ri = u.RI[g];
    const int base = ri & 0xffff, n = ri >> 16;  // this destination's block: rows base .. base + n - 1
    const int i = g - base;
    if (g != owner) {
      d = a.edge_rev[u.LN[g]];
      tb = a.rev_trip[u.LN[g]];
      qv = ld4(a.q + static_cast<int64_t>(d) * kCD + c0);
      sk = ld4(a.skip + static_cast<int64_t>(d) * kCD + c0);
    }
    const int nt = n - 1;  // triplets per destination
    const int64_t drow = static_cast<int64_t>(d) * kCD + c0;
    cf4 acc = {0.f, 0.f, 0.f, 0.f};
    float m = -INFINITY, den = 0.f;
    auto batch = [&](int j0, auto bb) {
      constexpr int BB = decltype(bb)::value;
      float yv[BB];
      int tt[BB];
#pragma unroll
      for (int uu = 0; uu < BB; ++uu) {
        const int j = j0 + uu;
        int jj = j - (j > i ? 1 : 0);
        jj = jj < nt ? jj : nt - 1;  // clamped (nt >= 1 here): every load unconditional
        tt[uu] = tb + jj;
        yv[uu] = a.y[static_cast<int64_t>(tt[uu]) * 8 + (l32 & 7)];
      }
      cf4 sv[BB];
      float lg[BB];
      float mb = -INFINITY;
#pragma unroll
      for (int uu = 0; uu < BB; ++uu) {
        const int j = j0 + uu;
        const bool ok = j < n && j != i;
        const int jr = base + (j < n ? j : n - 1);  // the source's row
        // S_t = b + sum_l Y_l(t) P_j[l]: Y_l handed to the half's lanes by row_newbcast (both 16-lane rows
        // of a half loaded the same triplet's Y row, one value per lane)
        float yl[kSfL];
        yl[0] = dpp_mov<0x150>(yv[uu]);
        yl[1] = dpp_mov<0x151>(yv[uu]);
        yl[2] = dpp_mov<0x152>(yv[uu]);
        yl[3] = dpp_mov<0x153>(yv[uu]);
        yl[4] = dpp_mov<0x154>(yv[uu]);
        yl[5] = dpp_mov<0x155>(yv[uu]);
        yl[6] = dpp_mov<0x156>(yv[uu]);
        cf4 s4 = bias4;
#pragma unroll
        for (int l = 0; l < kSfL; ++l) s4 += yl[l] * P[(jr * kSfL + l) * 32 + l32];
        sv[uu] = s4;
        if (a.sp && ok) st4(a.sp + static_cast<int64_t>(tt[uu]) * kCD + c0, s4);
        const cf4 kr = KE[jr * 32 + l32];
        const float logit = qk_logit<LPH>(qv, kr, a.sqrt_c);
        lg[uu] = ok ? logit : -INFINITY;
        mb = fmaxf(mb, lg[uu]);
        if (a.alpha && ok && leader) a.alpha[static_cast<int64_t>(tt[uu]) * a.H + head] = logit;
      }
      const float m_new = fmaxf(m, mb);
      const float corr = m_new == -INFINITY ? 1.f : expf(m - m_new);
      den *= corr;
      acc *= corr;
#pragma unroll
      for (int uu = 0; uu < BB; ++uu) {
        const int j = j0 + uu;
        const float p = lg[uu] == -INFINITY ? 0.f : expf(lg[uu] - m_new);
        const cf4 vr = VE[(base + (j < n ? j : n - 1)) * 32 + l32];
        den += p;
        acc += p * (vr * sv[uu]);
      }
      m = m_new;
    };
    if (nt > 0) {  // (per owner: the two halves of a wave may hold blocks of different atoms)
      int j0 = 0;
      for (; n - j0 > B / 2; j0 += B) batch(j0, std::integral_constant<int, B>{});
      if (j0 < n) batch(j0, std::integral_constant<int, B / 2>{});
    }
    const float inv = 1.0f / (den + kCEps);
    const cf4 o = acc * inv + sk;
    st4(a.out + drow, o);
    if (a.row_stats) {
      const float mu = half_sum(o[0] + o[1] + o[2] + o[3], half) / static_cast<float>(kCD);
      const cf4 dv = o - mu;
      const float q2 = half_sum(dv[0] * dv[0] + dv[1] * dv[1] + dv[2] * dv[2] + dv[3] * dv[3], half);
      if (l32 == 0) a.row_stats[d] = make_float2(mu, q2);
    }
    if (leader) {
      a.smax[static_cast<int64_t>(d) * a.H + head] = m;
      a.sden[static_cast<int64_t>(d) * a.H + head] = den;
    }
  }
  // P rows out for the backward (instead of every S row: 3.5 KB per source line node against 512 B per
  // triplet), issued last so that no load above waits behind these stores
  if (a.pp) {
    cf4* pout = reinterpret_cast<cf4*>(a.pp);
    for (int idx = tid; idx < n_rows * kSfL * 32; idx += NT) {
      const int r = idx / (kSfL * 32);
      pout[static_cast<int64_t>(u.LN[r]) * (kSfL * 32) + (idx - r * (kSfL * 32))] = P[idx];
    }
  }
}

constexpr size_t fwd_sf_lds(int rows) {
  return unit_rows_lds(rows) + static_cast<size_t>(rows) * ((2 + kSfL) * kCD + kSfK) * 4;
}

template <int LPH>
int fwd_sf_launch(const FwdSfArgs& a, bool edge, hipStream_t st) {
  constexpr int W = 8, B = 8;
  const size_t lds = fwd_sf_lds(a.max_rows);
  const unsigned grid = static_cast<unsigned>(a.n_atoms);
  auto go = [&](auto kern) -> int {
    if (lds > 64 * 1024) {
      const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
      if (e != hipSuccess) return static_cast<int>(e);
    }
    kern<<<grid, 64 * W, lds, st>>>(a);
    return last_launch_status();
  };
  return edge ? go(attn_fwd_center_sf_kernel<LPH, W, B, true>) : go(attn_fwd_center_sf_kernel<LPH, W, B, false>);
}

// ------------------------------------------------------------------------------ forward, fused, source tiles
// Center atoms whose block does not fit the fused forward's LDS image (4.7 KB per source row: degree > 17 at
// two workgroups per CU; config 5's AID atoms have median degree 24 and reach 61): the same forward with the
// atom's SOURCES staged kTileRows at a time.  One workgroup per atom; its 16 half-wave owners take the
// destination rows g = owner + 16 r (r < RMAX), whose online-softmax state (acc, max, den) lives in registers
// across the tiles; per tile the sources' k + e, v + e, radial rows and P rows are formed in LDS exactly as the
// untiled kernel forms them, and every owner runs its destinations' batches over the tile's sources, in the
// untiled kernel's order of sources; batches of 4 sources per memory round trip (the state of RMAX
// destinations takes the registers the untiled kernel's batches of 8 use), so the online softmax rescales
// at other points: equal to fp32 rounding.
constexpr int kTileRows = 16;

template <int LPH, int WAVES, int B, bool EDGE, int RMAX, bool STORE>
__global__ void __launch_bounds__(64 * WAVES, 4) attn_fwd_center_sf_tiled_kernel(const FwdSfArgs a) {
  static_assert(kTileRows % B == 0, "batches never cross a tile");
  // [TS][32] (k + e), [TS][32] (v + e), [TS][7][32] P, [TS][42] R, then per destination row its id and
  // triplet block [X2G_CENTER_MAX_DEGREE] x 2
  extern __shared__ cf4 lds[];
  constexpr int TS = kTileRows, NT = 64 * WAVES, NO = 2 * WAVES;
  cf4* KE = lds;
  cf4* VE = KE + TS * 32;
  cf4* P = VE + TS * 32;
  float* RS = reinterpret_cast<float*>(P + TS * kSfL * 32);
  int* DDs = reinterpret_cast<int*>(RS + TS * kSfK);
  int* TBs = DDs + X2G_CENTER_MAX_DEGREE;
  // the unit: one atom (the host routes the units of more than max_rows rows here, each a single atom)
  const int64_t unit = a.atom0 + blockIdx.x;
  int64_t pos = unit;
  if (a.packs) {
    pos = a.packs[unit];
    if (a.packs[unit + 1] <= pos) return;  // an empty unit slot (x2g_center_schedule's layout)
  }
  int r0, n, er = 0;
  if (a.info) {
    const int4 v = a.info[pos];
    r0 = uniform(v.y);
    n = uniform(v.z);
    if (EDGE) er = uniform(v.w);
  } else {
    const int b = a.order ? a.order[pos] : static_cast<int>(pos);
    r0 = uniform(a.atom_rowptr[b]);
    n = uniform(a.atom_rowptr[b + 1]) - r0;
    if (EDGE && n > 0) er = uniform(a.src_row[r0]);
  }
  // (workgroup-uniform; skip_rows: a device-made schedule's list mixes the packs of small atoms, which the
  // untiled form takes, with the single atoms beyond its LDS image)
  if (n <= 0 || n <= a.skip_rows) return;
  const int tid = threadIdx.x;
  const int l32 = tid & 31, half = (tid >> 5) & 1, wave = tid >> 6;
  const int owner = 2 * wave + half;
  const int head = l32 / LPH;
  const bool leader = (l32 % LPH) == 0;
  const int c0 = 4 * l32;
  const int nt = n - 1;
  cf4 acc[RMAX];
  float m[RMAX], den[RMAX];
#pragma unroll
  for (int r = 0; r < RMAX; ++r) {
    acc[r] = cf4{0.f, 0.f, 0.f, 0.f};
    m[r] = -INFINITY;
    den[r] = 0.f;
  }
  const cf4 bias4 = ld4(a.bias + c0);
  constexpr int NG = NT / 256;  // P thread groups of 7 x 32 (as the untiled kernel)
  const int pg = tid / 256, prest = tid % 256;
  const bool pthr = prest < kSfL * 32;
  const int pl = pthr ? prest >> 5 : 0, pc4 = prest & 31;
  // the destinations' ids and triplet blocks, once (each (destination, tile) pair then starts its q / Y
  // loads from LDS instead of behind two dependent global round trips; read after the first tile's barrier)
  for (int idx = tid; idx < n; idx += NT) {
    DDs[idx] = a.edge_rev[r0 + idx];
    TBs[idx] = a.rev_trip[r0 + idx];
  }
  for (int t0 = 0; t0 < n; t0 += TS) {
    const int ts = n - t0 < TS ? n - t0 : TS;
    __syncthreads();  // the previous tile's rows are no longer read
    const cf4 e4 = EDGE ? ld4(a.edge + static_cast<int64_t>(er) * kCD + 4 * (tid & 31)) : cf4{0.f, 0.f, 0.f, 0.f};
    for (int idx = tid; idx < ts * 32; idx += NT) {
      const int64_t row = static_cast<int64_t>(r0 + t0 + (idx >> 5)) * kCD + 4 * (idx & 31);
      KE[idx] = ld4(a.k + row) + e4;
      VE[idx] = ld4(a.v + row) + e4;
    }
    for (int idx = tid; idx < ts * kSfK; idx += NT) RS[idx] = a.radial[static_cast<int64_t>(r0 + t0) * kSfK + idx];
    float wv[4][kSfR];
#pragma unroll
    for (int cc = 0; cc < 4; ++cc)
#pragma unroll
      for (int r = 0; r < kSfR; ++r) wv[cc][r] = a.w[(4 * pc4 + cc) * kSfK + kSfR * pl + r];
    __syncthreads();
    if (pthr) {
      for (int j = pg; j < ts; j += NG) {
        const float* rr = RS + j * kSfK + kSfR * pl;
        float rv[kSfR];
#pragma unroll
        for (int r = 0; r < kSfR; ++r) rv[r] = rr[r];
        cf4 p;
#pragma unroll
        for (int cc = 0; cc < 4; ++cc) {
          float s = wv[cc][0] * rv[0];
#pragma unroll
          for (int r = 1; r < kSfR; ++r) s = fmaf(wv[cc][r], rv[r], s);
          p[cc] = s;
        }
        P[(j * kSfL + pl) * 32 + pc4] = p;
        // P rows out for the backward (each source row is in exactly one tile)
        if (a.pp) st4(a.pp + (static_cast<int64_t>(r0 + t0 + j) * kSfL + pl) * kCD + 4 * pc4, p);
      }
    }
    __syncthreads();
    const int t1 = t0 + ts;
#pragma unroll
    for (int r = 0; r < RMAX; ++r) {
      const int i = owner + NO * r;  // this destination's row in the block
      if (i >= n) continue;          // (per owner)
      const int dd = DDs[i], tb = TBs[i];
      const cf4 qv = ld4(a.q + static_cast<int64_t>(dd) * kCD + c0);
      if (nt > 0) {  // (n = 1: an empty softmax, out = skip)
        // batches of B sources, software-pipelined: batch j0 + B's Y values are loaded before batch j0's
        // arithmetic (clamped indices: every load unconditional), so a destination waits out one load
        // latency per tile instead of one per batch; the last batch of the atom masked
        float yv[B];
        int tt[B];
        auto load = [&](int j0, float (&y_)[B], int (&t_)[B]) {
#pragma unroll
          for (int uu = 0; uu < B; ++uu) {
            const int j = j0 + uu;
            int jj = j - (j > i ? 1 : 0);
            jj = jj < nt ? jj : nt - 1;
            t_[uu] = tb + jj;
            y_[uu] = a.y[static_cast<int64_t>(t_[uu]) * 8 + (l32 & 7)];
          }
        };
        load(t0, yv, tt);
        for (int j0 = t0; j0 < t1; j0 += B) {
          float yn[B];
          int tn[B];
          load(j0 + B, yn, tn);
          cf4 sv[B];
          float lg[B];
          float mb = -INFINITY;
#pragma unroll
          for (int uu = 0; uu < B; ++uu) {
            const int j = j0 + uu;
            const bool ok = j < n && j != i;
            const int jr = (j < t1 ? j : t1 - 1) - t0;  // the source's row in the tile
            float yl[kSfL];
            yl[0] = dpp_mov<0x150>(yv[uu]);
            yl[1] = dpp_mov<0x151>(yv[uu]);
            yl[2] = dpp_mov<0x152>(yv[uu]);
            yl[3] = dpp_mov<0x153>(yv[uu]);
            yl[4] = dpp_mov<0x154>(yv[uu]);
            yl[5] = dpp_mov<0x155>(yv[uu]);
            yl[6] = dpp_mov<0x156>(yv[uu]);
            cf4 s4 = bias4;
#pragma unroll
            for (int l = 0; l < kSfL; ++l) s4 += yl[l] * P[(jr * kSfL + l) * 32 + l32];
            sv[uu] = s4;
            if constexpr (STORE) {
              if (a.sp && ok) st4(a.sp + static_cast<int64_t>(tt[uu]) * kCD + c0, s4);
            }
            const cf4 kr = KE[jr * 32 + l32];
            const float logit = qk_logit<LPH>(qv, kr, a.sqrt_c);
            lg[uu] = ok ? logit : -INFINITY;
            mb = fmaxf(mb, lg[uu]);
            if constexpr (STORE) {
              if (a.alpha && ok && leader) a.alpha[static_cast<int64_t>(tt[uu]) * a.H + head] = logit;
            }
          }
          const float m_new = fmaxf(m[r], mb);
          const float corr = m_new == -INFINITY ? 1.f : expf(m[r] - m_new);
          den[r] *= corr;
          acc[r] *= corr;
#pragma unroll
          for (int uu = 0; uu < B; ++uu) {
            const int j = j0 + uu;
            const float p = lg[uu] == -INFINITY ? 0.f : expf(lg[uu] - m_new);
            const cf4 vr = VE[((j < t1 ? j : t1 - 1) - t0) * 32 + l32];
            den[r] += p;
            acc[r] += p * (vr * sv[uu]);
          }
          m[r] = m_new;
#pragma unroll
          for (int uu = 0; uu < B; ++uu) {
            yv[uu] = yn[uu];
            tt[uu] = tn[uu];
          }
        }
      }
    }
  }
#pragma unroll
  for (int r = 0; r < RMAX; ++r) {
    if (owner + NO * r >= n) continue;
    const int dd = DDs[owner + NO * r];
    const int64_t drow = static_cast<int64_t>(dd) * kCD + c0;
    const float inv = 1.0f / (den[r] + kCEps);
    const cf4 o = acc[r] * inv + ld4(a.skip + drow);
    st4(a.out + drow, o);
    if (a.row_stats) {
      const float mu = half_sum(o[0] + o[1] + o[2] + o[3], half) / static_cast<float>(kCD);
      const cf4 dv = o - mu;
      const float q2 = half_sum(dv[0] * dv[0] + dv[1] * dv[1] + dv[2] * dv[2] + dv[3] * dv[3], half);
      if (l32 == 0) a.row_stats[dd] = make_float2(mu, q2);
    }
    if (leader) {
      a.smax[static_cast<int64_t>(dd) * a.H + head] = m[r];
      a.sden[static_cast<int64_t>(dd) * a.H + head] = den[r];
    }
  }
}

constexpr size_t fwd_sf_tiled_lds() {
  return static_cast<size_t>(kTileRows) * ((2 + kSfL) * kCD + kSfK) * 4 + 2 * X2G_CENTER_MAX_DEGREE * 4;
}

template <int LPH>
int fwd_sf_tiled_launch(const FwdSfArgs& a, bool edge, int max_degree, hipStream_t st) {
  // batches of 4 sources: with 8 the RMAX destinations' state spills (4-6 VGPRs at RMAX 2, 15-17 at 4)
  constexpr int W = 8, B = 4;
  const size_t lds = fwd_sf_tiled_lds();
  const unsigned grid = static_cast<unsigned>(a.n_atoms);
  auto go = [&](auto kern) -> int {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
    if (e != hipSuccess) return static_cast<int>(e);
    kern<<<grid, 64 * W, lds, st>>>(a);
    return last_launch_status();
  };
  constexpr int NO = 2 * W;
  // STORE: logits / S rows / P rows for a backward or the attention weights (inference stores none: no store
  // in the pipelined batch loop, whose load waits then stay counted)
  const bool store = a.alpha || a.sp || a.pp;
  auto pick = [&](auto rmax) -> int {
    constexpr int R = decltype(rmax)::value;
    if (store)
      return edge ? go(attn_fwd_center_sf_tiled_kernel<LPH, W, B, true, R, true>)
                  : go(attn_fwd_center_sf_tiled_kernel<LPH, W, B, false, R, true>);
    return edge ? go(attn_fwd_center_sf_tiled_kernel<LPH, W, B, true, R, false>)
                : go(attn_fwd_center_sf_tiled_kernel<LPH, W, B, false, R, false>);
  };
  if (max_degree <= 2 * NO) return pick(std::integral_constant<int, 2>{});
  if (max_degree <= 4 * NO) return pick(std::integral_constant<int, 4>{});
  return pick(std::integral_constant<int, 8>{});
}

template <int LPH>
int fwd_center_launch(const FwdCenterArgs& a, bool edge, int max_degree, hipStream_t st) {
  constexpr int W = 4, B = 8;
  const size_t lds = static_cast<size_t>(2) * max_degree * kCD * sizeof(float);
  const unsigned grid = static_cast<unsigned>(a.n_atoms);
  auto go = [&](auto kern) -> int {
    if (lds > 64 * 1024) {  // above the default dynamic-LDS limit (degrees > 64)
      const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
      if (e != hipSuccess) return static_cast<int>(e);
    }
    kern<<<grid, 64 * W, lds, st>>>(a);
    return last_launch_status();
  };
  return edge ? go(attn_fwd_center_kernel<LPH, W, B, true>) : go(attn_fwd_center_kernel<LPH, W, B, false>);
}

// ------------------------------------------------------------------------------ fused backward
// One workgroup per center atom b does BOTH backward passes of the destination-major kernels
// (attention_fold.inc) over b's triplet block, from LDS images of the block's rows:
//   KE[j] = k_j + e, GO[i] = dout[d_i], QI[i] = q[d_i], per-destination max / 1 / (den + eps);
// pass 1, one owner per SOURCE j (its S rows t(i, j) = TB[i] + j - [j > i], one 512-byte row each):
//   at = exp(alpha_t - max_i) / (den_i + eps),  g_t = sum over the head of go_i (v_j + e) S_t,
//   dv_j += at go_i S_t,  and (g_t, at) pairs into a [T, H] scratch (L2-resident until the same workgroup
//   reads it back);
// then rho_i = sum_j at g (j ascending: the destination pass's order) over destination i's contiguous
// block, and pass 2 (at, g from the scratch, Y_t, rows from LDS), per owner both roles:
//   w = at (g - rho_i) / sqrt(C),  dk_j = sum_i w q_i,  G_j[l] = sum_i at go_i (v_j + e) Y_l(t)  (source j:
//   the folded lin_sbf gradient),  dq_i = sum_j w (k_j + e)  (destination i),
// and, for the element-table gradient, d_edge[b] = sum_j (dk_j + dv_j) (X2-GNN's edge term enters as
// k_j + e and v_j + e with e the center atom's row: its gradient is the block's sum).  S is read once per
// backward (the two destination-major passes read S twice and gather k / v / q / dout rows per triplet
// from L2), only pass 1 holds S rows and only pass 2 the 32 G accumulators, so both take 8 triplets per
// memory round trip within 128 VGPRs.
struct BwdCenterArgs {
  const float *q, *k, *v, *edge;
  const int32_t* src_row;
  const float *sp, *alpha, *smax, *sden, *dout, *y;
  const float *pp, *bias;  // FACT: S_t = bias + sum_l Y_l(t) P_s[l] from pp [E, 7, 128] instead of sp rows
  const int32_t *atom_rowptr, *edge_rev, *rev_trip;
  const int32_t* order;  // workgroup -> center atom (NULL: blockIdx.x)
  int64_t n_atoms, T;
  int H;
  float inv_sqrt_c;
  float sqrt_c;  // FACT: the logits are recomputed as the forward formed them (q . (k + e) / sqrt C)
  float *dq, *dk, *dv, *gfold, *d_edge, *gw;  // gw: [T, H] (g, a) pairs of scratch
};

template <int H>
__host__ __device__ constexpr size_t bwd_center_lds(int n) {
  return static_cast<size_t>(n) * 4 * kCD * 4  // KE, GO, QI, DE
         + static_cast<size_t>(n) * H * 4 * 3  // MX, IV, RHO
         + static_cast<size_t>(n) * 4 * 2;     // TB, DI
}

template <int LPH, int WAVES, int B, bool EDGE, bool FACT>
__global__ void __launch_bounds__(64 * WAVES, 4) attn_bwd_center_kernel(const BwdCenterArgs a) {
  constexpr int H = 32 / LPH;
  extern __shared__ cf4 lds[];
  const int64_t b = a.order ? static_cast<int64_t>(a.order[blockIdx.x]) : static_cast<int64_t>(blockIdx.x);
  const int r0 = uniform(a.atom_rowptr[b]);
  const int n = uniform(a.atom_rowptr[b + 1]) - r0;
  const int tid = threadIdx.x;
  const int l32 = tid & 31, half = (tid >> 5) & 1, wave = tid >> 6;
  const int owner = 2 * wave + half;
  constexpr int NO = 2 * WAVES;  // owners
  const int head = l32 / LPH;
  const bool leader = (l32 % LPH) == 0;
  const int c0 = 4 * l32;
  if (n <= 0) {  // an atom without edges: its element-table gradient row is zero
    if (a.d_edge && tid < 32) st4(a.d_edge + b * kCD + c0, cf4{0.f, 0.f, 0.f, 0.f});
    return;
  }
  cf4* KE = lds;
  cf4* GO = KE + n * 32;
  cf4* QI = GO + n * 32;
  cf4* DE = QI + n * 32;
  float* MX = reinterpret_cast<float*>(DE + n * 32);
  float* IV = MX + n * H;
  float* RHO = IV + n * H;
  int* TB = reinterpret_cast<int*>(RHO + n * H);
  int* DI = TB + n;
  const int64_t e_row = EDGE ? static_cast<int64_t>(uniform(a.src_row[r0])) * kCD : 0;
  // ---- staging: the destinations and triplet blocks first, then every row load from addresses in LDS
  // (two dependent round trips instead of an index load in front of each row load)
  for (int idx = tid; idx < n; idx += 64 * WAVES) {
    TB[idx] = a.rev_trip[r0 + idx];
    DI[idx] = a.edge_rev[r0 + idx];
  }
  __syncthreads();
  constexpr int NT = 64 * WAVES;
  if (n * 32 <= 2 * NT && n * H <= NT) {  // (workgroup-uniform) every staging load in flight together
    cf4 kk[2], gg[2], qq[2];
    const int c = tid & 31;  // (the same column in both slots: NT is a multiple of 32)
    const cf4 e4 = EDGE ? ld4(a.edge + e_row + 4 * c) : cf4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      int j = (tid + u * NT) >> 5;
      j = j < n ? j : n - 1;  // clamped: loads unconditional, stores masked below
      const int64_t d = DI[j];
      kk[u] = ld4(a.k + static_cast<int64_t>(r0 + j) * kCD + 4 * c);
      gg[u] = ld4(a.dout + d * kCD + 4 * c);
      qq[u] = ld4(a.q + d * kCD + 4 * c);
    }
    const int sidx = tid < n * H ? tid : 0;
    const int si = sidx / H, sh = sidx - si * H;
    const int64_t sd = DI[si];
    const float mx = a.smax[sd * H + sh], dn = a.sden[sd * H + sh];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int idx = tid + u * NT;
      if (idx < n * 32) {
        KE[idx] = kk[u] + e4;
        GO[idx] = gg[u];
        QI[idx] = qq[u];
      }
    }
    if (tid < n * H) {
      MX[tid] = mx;
      IV[tid] = 1.0f / (dn + kCEps);
    }
  } else {
    for (int idx = tid; idx < n * 32; idx += NT) {
      const int j = idx >> 5, c = idx & 31;
      const int64_t d = DI[j];
      const cf4 e4 = EDGE ? ld4(a.edge + e_row + 4 * c) : cf4{0.f, 0.f, 0.f, 0.f};
      KE[idx] = ld4(a.k + static_cast<int64_t>(r0 + j) * kCD + 4 * c) + e4;
      GO[idx] = ld4(a.dout + d * kCD + 4 * c);
      QI[idx] = ld4(a.q + d * kCD + 4 * c);
    }
    for (int idx = tid; idx < n * H; idx += NT) {
      const int i = idx / H, h = idx - i * H;
      const int64_t d = DI[i];
      MX[idx] = a.smax[d * H + h];
      IV[idx] = 1.0f / (a.sden[d * H + h] + kCEps);
    }
  }
  __syncthreads();
  const int nt = n - 1;  // triplets per destination (and per source)
  auto rsrc = [](const void* p, int64_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), static_cast<short>(0),
                                             static_cast<int>(bytes < 0x7fffffff ? bytes : 0x7fffffff), 0x00020000);
  };
  const __amdgpu_buffer_rsrc_t sp_r = rsrc(a.sp, a.T * kCD * 4);
  const __amdgpu_buffer_rsrc_t al_r = rsrc(a.alpha, a.T * H * 4);
  const __amdgpu_buffer_rsrc_t y_r = rsrc(a.y, a.T * 8 * 4);
  // the scratch holds (g_t, a_t) pairs per (triplet, head): one 8-byte store in pass 1, one 8-byte load
  // per use below
  const __amdgpu_buffer_rsrc_t ag_r = rsrc(a.gw, a.T * H * 8);
  auto ldf = [](__amdgpu_buffer_rsrc_t r, int off) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
  };
  auto ldag = [&](int t) {  // (g, a) of triplet t, this lane's head
    return __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(ag_r, (t * H + head) * 8, 0, 0));
  };
  // the triplet of destination i and source j (i != j; i == j gives some row of i's block, unused)
  auto trip = [&](int i, int j) {
    int pos = j - (j > i ? 1 : 0);
    pos = pos < nt ? pos : nt - 1;
    return TB[i] + pos;  // (32-bit offsets below: T * 512 < 2^31, checked)
  };
  // ---- pass 1: one owner per source j: at, g (to the scratch), dv
  for (int j = owner; j < n; j += NO) {
    const int64_t srow = static_cast<int64_t>(r0 + j) * kCD + c0;
    cf4 ue = ld4(a.v + srow);
    if (EDGE) ue += ld4(a.edge + e_row + c0);
    cf4 dv = {0.f, 0.f, 0.f, 0.f};
    // FACT: this source's 7 P rows (the forward's own, so S_t below is the forward's S_t bit for bit)
    cf4 pj[FACT ? kSfL : 1], bias4 = {0.f, 0.f, 0.f, 0.f};
    if constexpr (FACT) {
#pragma unroll
      for (int l = 0; l < kSfL; ++l) pj[l] = ld4(a.pp + (static_cast<int64_t>(r0 + j) * kSfL + l) * kCD + c0);
      bias4 = ld4(a.bias + c0);
    }
    auto batch = [&](int i0, auto bb) {
      constexpr int BB = decltype(bb)::value;
      cf4 sv[FACT ? 1 : BB];
      float yv[FACT ? BB : 1];
      float al[BB];
      int tt[BB];
#pragma unroll
      for (int u = 0; u < BB; ++u) {
        const int i = i0 + u < n ? i0 + u : n - 1;  // clamped: loads unconditional, masked below
        tt[u] = trip(i, j);
        if constexpr (FACT)
          yv[u] = ldf(y_r, (tt[u] * 8 + (l32 & 7)) * 4);
        else
          sv[u] = __builtin_bit_cast(cf4, __builtin_amdgcn_raw_buffer_load_b128(sp_r, tt[u] * (kCD * 4) + c0 * 4, 0, 0));
        al[u] = ldf(al_r, (tt[u] * H + head) * 4);
      }
#pragma unroll
      for (int u = 0; u < BB; ++u) {
        const int i = i0 + u < n ? i0 + u : n - 1;
        const bool ok = i0 + u < n && i != j;
        cf4 st;
        if constexpr (FACT) {  // S_t = b + sum_l Y_l(t) P_j[l], the forward's arithmetic in its order
          float yl[kSfL];
          yl[0] = dpp_mov<0x150>(yv[u]);
          yl[1] = dpp_mov<0x151>(yv[u]);
          yl[2] = dpp_mov<0x152>(yv[u]);
          yl[3] = dpp_mov<0x153>(yv[u]);
          yl[4] = dpp_mov<0x154>(yv[u]);
          yl[5] = dpp_mov<0x155>(yv[u]);
          yl[6] = dpp_mov<0x156>(yv[u]);
          st = bias4;
#pragma unroll
          for (int l = 0; l < kSfL; ++l) st += yl[l] * pj[l];
        } else {
          st = sv[u];
        }
        const float at = ok ? expf(al[u] - MX[i * H + head]) * IV[i * H + head] : 0.f;
        const cf4 go = GO[i * 32 + l32];
        const cf4 gu = go * ue;
        float gp = gu[0] * st[0];
        gp = fmaf(gu[1], st[1], gp);
        gp = fmaf(gu[2], st[2], gp);
        gp = fmaf(gu[3], st[3], gp);
        const float g = head_sum<LPH>(gp);
        if (ok && leader) *reinterpret_cast<float2*>(a.gw + (static_cast<int64_t>(tt[u]) * H + head) * 2) = make_float2(g, at);
        dv += at * (go * st);
      }
    };
    if constexpr (FACT) {
      // software-pipelined: batch i0 + 4's Y and logit loads are issued before batch i0's arithmetic, so
      // only the first batch of a source waits out the load latency (every batch full, the last masked;
      // every load and store unconditional — clamped indices, the (g, a) store of a masked triplet to an
      // out-of-range offset — so the compiler's vmcnt waits stay counted)
      // The logits are not read back: a_t's logit is q_i . (k_j + e) / sqrt C over the head's lanes, from the
      // QI / KE rows already in LDS, in the forward's own arithmetic (the same products, fma order and head
      // sum: the same bits), so the forward stores no [T, H] logits for this backward (x2gnn passes none).
      constexpr int BB = kFactBatch;
      if (nt > 0) {  // (workgroup-uniform)
        const cf4 kj = KE[j * 32 + l32];
        float yv[BB];
        int tt[BB];
        auto load = [&](int i0, float (&y_)[BB], int (&t_)[BB]) {
#pragma unroll
          for (int u = 0; u < BB; ++u) {
            const int i = i0 + u < n ? i0 + u : n - 1;
            t_[u] = trip(i, j);
            y_[u] = ldf(y_r, (t_[u] * 8 + (l32 & 7)) * 4);
          }
        };
        load(0, yv, tt);
        for (int i0 = 0; i0 < n; i0 += BB) {
          float yn[BB];
          int tn[BB];
          load(i0 + BB, yn, tn);
#pragma unroll
          for (int u = 0; u < BB; ++u) {
            const int i = i0 + u < n ? i0 + u : n - 1;
            const bool ok = i0 + u < n && i != j;
            float yl[kSfL];
            yl[0] = dpp_mov<0x150>(yv[u]);
            yl[1] = dpp_mov<0x151>(yv[u]);
            yl[2] = dpp_mov<0x152>(yv[u]);
            yl[3] = dpp_mov<0x153>(yv[u]);
            yl[4] = dpp_mov<0x154>(yv[u]);
            yl[5] = dpp_mov<0x155>(yv[u]);
            yl[6] = dpp_mov<0x156>(yv[u]);
            cf4 st = bias4;  // S_t = b + sum_l Y_l(t) P_j[l], the forward's arithmetic in its order
#pragma unroll
            for (int l = 0; l < kSfL; ++l) st += yl[l] * pj[l];
            const float logit = qk_logit<LPH>(QI[i * 32 + l32], kj, a.sqrt_c);
            const float at = ok ? expf(logit - MX[i * H + head]) * IV[i * H + head] : 0.f;
            const cf4 go = GO[i * 32 + l32];
            const cf4 gu = go * ue;
            float gp = gu[0] * st[0];
            gp = fmaf(gu[1], st[1], gp);
            gp = fmaf(gu[2], st[2], gp);
            gp = fmaf(gu[3], st[3], gp);
            const float g = head_sum<LPH>(gp);
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned,
                                                                     make_float2(g, at)),
                                                  ag_r, (ok && leader) ? (tt[u] * H + head) * 8 : static_cast<int>(0x80000000u),
                                                  0, 0);
            dv += at * (go * st);
          }
#pragma unroll
          for (int u = 0; u < BB; ++u) {
            yv[u] = yn[u];
            tt[u] = tn[u];
          }
        }
      }
    } else if (nt > 0) {  // (workgroup-uniform)
      int i0 = 0;
      for (; n - i0 > B / 2; i0 += B) batch(i0, std::integral_constant<int, B>{});
      if (i0 < n) batch(i0, std::integral_constant<int, B / 2>{});
    }
    st4(a.dv + srow, dv);
    DE[j * 32 + l32] = dv;  // (the edge term's gradient: dk added in pass 2)
  }
  // the scratch written by every owner is read by others below: workgroup-scope release / acquire
  __threadfence_block();
  __syncthreads();
  // ---- rho_i = sum_{j != i} at g over i's contiguous block, j ascending (one owner per destination)
  for (int i = owner; i < n; i += NO) {
    float rho = 0.f;
    for (int p0 = 0; p0 < nt; p0 += 8) {
      float at[8], g[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const float2 ag = ldag(TB[i] + (p0 + u < nt ? p0 + u : nt - 1));
        g[u] = ag.x;
        at[u] = ag.y;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (p0 + u < nt) rho = fmaf(at[u], g[u], rho);
    }
    if (leader) RHO[i * H + head] = rho;
  }
  __syncthreads();
  // ---- pass 2, owner o in both roles, x over the other n - 1:
  //   source j = o (destinations i = x): dk_o, G_o;  destination i = o (sources j = x): dq_o
  for (int o = owner; o < n; o += NO) {
    const int64_t srow = static_cast<int64_t>(r0 + o) * kCD + c0;
    cf4 ue = ld4(a.v + srow);
    if (EDGE) ue += ld4(a.edge + e_row + c0);
    cf4 dk = {0.f, 0.f, 0.f, 0.f}, dq = {0.f, 0.f, 0.f, 0.f};
    cf4 G[8];
#pragma unroll
    for (int l = 0; l < 8; ++l) G[l] = cf4{0.f, 0.f, 0.f, 0.f};
    const float rho_o = RHO[o * H + head];
    auto batch = [&](int x0, auto bb) {
      constexpr int BB = decltype(bb)::value;
      float ats[BB], gs[BB], yv[BB], atd[BB], gd[BB];
#pragma unroll
      for (int u = 0; u < BB; ++u) {
        const int x = x0 + u < n ? x0 + u : n - 1;
        const int ts = trip(x, o), td = trip(o, x);
        const float2 ags = ldag(ts), agd = ldag(td);
        gs[u] = ags.x;
        ats[u] = ags.y;
        yv[u] = ldf(y_r, (ts * 8 + (l32 & 7)) * 4);
        gd[u] = agd.x;
        atd[u] = agd.y;
      }
#pragma unroll
      for (int u = 0; u < BB; ++u) {
        const int x = x0 + u < n ? x0 + u : n - 1;
        const bool ok = x0 + u < n && x != o;
        const float as = ok ? ats[u] : 0.f, ad = ok ? atd[u] : 0.f;
        const float ws = as * (gs[u] - RHO[x * H + head]) * a.inv_sqrt_c;
        dk += ws * QI[x * 32 + l32];
        const float wd = ad * (gd[u] - rho_o) * a.inv_sqrt_c;
        dq += wd * KE[x * 32 + l32];
        const cf4 ds = (GO[x * 32 + l32] * ue) * as;
        float yl[8];
        yl[0] = dpp_mov<0x150>(yv[u]);
        yl[1] = dpp_mov<0x151>(yv[u]);
        yl[2] = dpp_mov<0x152>(yv[u]);
        yl[3] = dpp_mov<0x153>(yv[u]);
        yl[4] = dpp_mov<0x154>(yv[u]);
        yl[5] = dpp_mov<0x155>(yv[u]);
        yl[6] = dpp_mov<0x156>(yv[u]);
        yl[7] = dpp_mov<0x157>(yv[u]);
#pragma unroll
        for (int l = 0; l < 8; ++l) G[l] += ds * yl[l];
      }
    };
    if (nt > 0) {
      int x0 = 0;
      for (; n - x0 > B / 2; x0 += B) batch(x0, std::integral_constant<int, B>{});
      if (x0 < n) batch(x0, std::integral_constant<int, B / 2>{});
    }
    st4(a.dk + srow, dk);
    st4(a.dq + static_cast<int64_t>(DI[o]) * kCD + c0, dq);
    float* gf = a.gfold + static_cast<int64_t>(r0 + o) * 8 * kCD + c0;
#pragma unroll
    for (int l = 0; l < 8; ++l) st4(gf + l * kCD, G[l]);
    DE[o * 32 + l32] += dk;  // (this owner's own dv row of pass 1)
  }
  if (a.d_edge) {  // d_edge[b] = sum_j (dv_j + dk_j), j ascending
    __syncthreads();
    if (tid < 32) {
      cf4 s = DE[l32];
      for (int j = 1; j < n; ++j) s += DE[j * 32 + l32];
      st4(a.d_edge + b * kCD + c0, s);
    }
  }
}

template <int LPH>
int bwd_center_launch(const BwdCenterArgs& a, bool edge, int max_degree, hipStream_t st) {
  constexpr int W = 4, B = 8;
  constexpr int H = 32 / LPH;
  const size_t lds = bwd_center_lds<H>(max_degree);
  if (lds > 160 * 1024) return X2G_EUNSUPPORTED;
  const unsigned grid = static_cast<unsigned>(a.n_atoms);
  auto go = [&](auto kern) -> int {
    if (lds > 64 * 1024) {  // above the default dynamic-LDS limit
      const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
      if (e != hipSuccess) return static_cast<int>(e);
    }
    kern<<<grid, 64 * W, lds, st>>>(a);
    return last_launch_status();
  };
  if (a.pp)
    return edge ? go(attn_bwd_center_kernel<LPH, W, B, true, true>) : go(attn_bwd_center_kernel<LPH, W, B, false, true>);
  return edge ? go(attn_bwd_center_kernel<LPH, W, B, true, false>) : go(attn_bwd_center_kernel<LPH, W, B, false, false>);
}

}  // namespace
}  // namespace x2g

using namespace x2g;

X2G_API size_t x2g_sbf_attention_bwd_center_lds(int32_t max_degree, int32_t heads) {
  if (max_degree < 0 || heads <= 0) return 0;
  const int n = max_degree > 0 ? max_degree : 1;
  return static_cast<size_t>(n) * 4 * kCD * 4 + static_cast<size_t>(n) * heads * 12 + static_cast<size_t>(n) * 8;
}

X2G_API int x2g_sbf_attention_bwd_center(const float* q, const float* k, const float* v, const float* edge,
                                         const int32_t* src_row, int edge_mode, const float* sbfproj,
                                         const float* sbf_p, const float* b_sbf,
                                         const float* sph_y, const int32_t* atom_rowptr, const int32_t* edge_rev,
                                         const int32_t* rev_trip, const int32_t* atom_order, const float* alpha_raw,
                                         const float* seg_max,
                                         const float* seg_den, const float* dout, int64_t num_atoms,
                                         int32_t max_degree, int64_t num_edges, int64_t num_triplets, int32_t heads,
                                         int32_t channels, float* dq, float* dk, float* dv, float* radial_grad,
                                         float* d_edge_atom, float* g_work, void* stream) {
  if (num_atoms < 0 || num_edges < 0 || num_triplets < 0 || heads <= 0 || channels <= 0) return X2G_EINVAL;
  if (edge_mode != X2G_EDGE_NONE && edge_mode != X2G_EDGE_PER_DST) return X2G_EUNSUPPORTED;
  if (heads * channels != kCD || channels % 4 || max_degree < 0 || max_degree > X2G_CENTER_MAX_DEGREE)
    return X2G_EUNSUPPORTED;
  if (x2g_sbf_attention_bwd_center_lds(max_degree, heads) > 160 * 1024) return X2G_EUNSUPPORTED;
  // 32-bit buffer offsets: the S rows (T x 512 B), or with P rows the (g, a) scratch (T x H x 8 B, the
  // largest T-row array then: logits T x H x 4, Y rows T x 32)
  if (num_triplets * (sbf_p ? int64_t(heads) * 8 : int64_t(kCD) * 4) >= (int64_t(1) << 31)) return X2G_EUNSUPPORTED;
  if (num_atoms == 0) return X2G_OK;
  if (!sbfproj == !sbf_p || (sbf_p && !b_sbf)) return X2G_EINVAL;  // S rows, or the P rows and the bias
  if (num_edges > 0 && (!q || !k || !v || !sph_y || !atom_rowptr || !edge_rev || !rev_trip ||
                        (!alpha_raw && !sbf_p) || !seg_max || !seg_den || !dout || !dq || !dk || !dv ||
                        !radial_grad || (num_triplets > 0 && !g_work)))
    return X2G_EINVAL;
  if (!atom_rowptr) return X2G_EINVAL;
  if (edge_mode == X2G_EDGE_PER_DST && (!edge || !src_row)) return X2G_EINVAL;
  const auto al = [](const void* p, int m) { return p == nullptr || reinterpret_cast<uintptr_t>(p) % m == 0; };
  if (!al(q, 16) || !al(k, 16) || !al(v, 16) || !al(edge, 16) || !al(sbfproj, 16) || !al(dout, 16) || !al(dq, 16) ||
      !al(dk, 16) || !al(dv, 16) || !al(radial_grad, 16) || !al(d_edge_atom, 16) || !al(sbf_p, 16) || !al(b_sbf, 16))
    return X2G_EUNSUPPORTED;
  BwdCenterArgs a{};
  a.pp = sbf_p; a.bias = b_sbf;
  a.q = q; a.k = k; a.v = v; a.edge = edge; a.src_row = src_row; a.sp = sbfproj; a.alpha = alpha_raw;
  a.smax = seg_max; a.sden = seg_den; a.dout = dout; a.y = sph_y; a.atom_rowptr = atom_rowptr; a.edge_rev = edge_rev;
  a.rev_trip = rev_trip; a.order = atom_order; a.n_atoms = num_atoms; a.T = num_triplets; a.H = heads;
  a.inv_sqrt_c = static_cast<float>(1.0 / sqrt(static_cast<double>(channels)));
  a.sqrt_c = static_cast<float>(sqrt(static_cast<double>(channels)));
  a.dq = dq; a.dk = dk; a.dv = dv; a.gfold = radial_grad; a.d_edge = d_edge_atom; a.gw = g_work;
  const int md = max_degree > 0 ? max_degree : 1;
  const bool edge_on = edge_mode == X2G_EDGE_PER_DST;
  hipStream_t st = as_stream(stream);
  switch (channels / 4) {
    case 1: return bwd_center_launch<1>(a, edge_on, md, st);
    case 2: return bwd_center_launch<2>(a, edge_on, md, st);
    case 4: return bwd_center_launch<4>(a, edge_on, md, st);
    case 8: return bwd_center_launch<8>(a, edge_on, md, st);
    default: return X2G_EUNSUPPORTED;
  }
}

X2G_API int x2g_sbf_attention_fwd_center(const float* q, const float* k, const float* v, const float* skip,
                                         const float* edge, const int32_t* src_row, int edge_mode,
                                         const float* sbfproj, int64_t t_base, const int32_t* atom_rowptr,
                                         const int32_t* edge_rev, const int32_t* rev_trip, const int32_t* atom_order,
                                         int64_t atom0,
                                         int64_t n_atoms, int32_t max_degree, int64_t num_edges,
                                         int64_t num_triplets, int32_t heads, int32_t channels, float* out,
                                         float* alpha_raw, float* seg_max, float* seg_den, float* row_stats,
                                         void* stream) {
  if (n_atoms < 0 || atom0 < 0 || num_edges < 0 || num_triplets < 0 || heads <= 0 || channels <= 0)
    return X2G_EINVAL;
  if (edge_mode != X2G_EDGE_NONE && edge_mode != X2G_EDGE_PER_DST) return X2G_EUNSUPPORTED;
  if (heads * channels != kCD || channels % 4 || max_degree < 0 || max_degree > X2G_CENTER_MAX_DEGREE)
    return X2G_EUNSUPPORTED;
  if (n_atoms == 0 || num_edges == 0) return X2G_OK;
  if (!q || !k || !v || !skip || !sbfproj || !atom_rowptr || !edge_rev || !rev_trip || !out || !seg_max || !seg_den)
    return X2G_EINVAL;
  // (alpha_raw NULL: the logits are not stored — inference)
  if (edge_mode == X2G_EDGE_PER_DST && (!edge || !src_row)) return X2G_EINVAL;
  // 16-byte rows (float4 per lane), 8-byte row statistics
  const auto al = [](const void* p, int m) { return p == nullptr || reinterpret_cast<uintptr_t>(p) % m == 0; };
  if (!al(q, 16) || !al(k, 16) || !al(v, 16) || !al(skip, 16) || !al(edge, 16) || !al(sbfproj, 16) || !al(out, 16) ||
      !al(row_stats, 8))
    return X2G_EUNSUPPORTED;
  FwdCenterArgs a{};
  a.q = q; a.k = k; a.v = v; a.skip = skip; a.edge = edge; a.src_row = src_row; a.sp = sbfproj; a.t_base = t_base;
  a.atom_rowptr = atom_rowptr; a.edge_rev = edge_rev; a.rev_trip = rev_trip; a.order = atom_order; a.atom0 = atom0;
  a.n_atoms = n_atoms; a.H = heads; a.sqrt_c = static_cast<float>(sqrt(static_cast<double>(channels)));
  a.out = out; a.alpha = alpha_raw; a.smax = seg_max; a.sden = seg_den;
  a.row_stats = reinterpret_cast<float2*>(row_stats);
  const int md = max_degree > 0 ? max_degree : 1;
  const bool edge_on = edge_mode == X2G_EDGE_PER_DST;
  hipStream_t st = as_stream(stream);
  switch (channels / 4) {
    case 1: return fwd_center_launch<1>(a, edge_on, md, st);
    case 2: return fwd_center_launch<2>(a, edge_on, md, st);
    case 4: return fwd_center_launch<4>(a, edge_on, md, st);
    case 8: return fwd_center_launch<8>(a, edge_on, md, st);
    default: return X2G_EUNSUPPORTED;
  }
}

X2G_API int x2g_sbf_attention_fwd_center_sf(const float* q, const float* k, const float* v, const float* skip,
                                            const float* edge, const int32_t* src_row, int edge_mode,
                                            const float* radial, const float* sph_y, const float* w_sbf,
                                            const float* b_sbf, const int32_t* atom_rowptr, const int32_t* edge_rev,
                                            const int32_t* rev_trip, const int32_t* atom_order,
                                            const int32_t* pack_ptr, const int32_t* atom_info, int64_t unit0,
                                            int64_t n_units,
                                            int32_t max_rows, int64_t num_edges, int64_t num_triplets, int32_t heads,
                                            int32_t channels, float* out, float* alpha_raw, float* seg_max,
                                            float* seg_den, float* row_stats, float* sbfproj_out, float* sbf_p_out,
                                            void* stream) {
  if (n_units < 0 || unit0 < 0 || num_edges < 0 || num_triplets < 0 || heads <= 0 || channels <= 0)
    return X2G_EINVAL;
  if (edge_mode != X2G_EDGE_NONE && edge_mode != X2G_EDGE_PER_DST) return X2G_EUNSUPPORTED;
  if (heads * channels != kCD || channels % 4 || max_rows < 0 || max_rows > X2G_CENTER_MAX_DEGREE ||
      fwd_sf_lds(max_rows > 0 ? max_rows : 1) > 160 * 1024)
    return X2G_EUNSUPPORTED;
  if (n_units == 0 || num_edges == 0) return X2G_OK;
  if (!q || !k || !v || !skip || !radial || !sph_y || !w_sbf || !b_sbf || !atom_rowptr || !edge_rev || !rev_trip ||
      !out || !seg_max || !seg_den || (pack_ptr && !atom_order))
    return X2G_EINVAL;
  // (alpha_raw NULL: the logits are not stored — inference)
  if (edge_mode == X2G_EDGE_PER_DST && (!edge || !src_row)) return X2G_EINVAL;
  const auto al = [](const void* p, int m) { return p == nullptr || reinterpret_cast<uintptr_t>(p) % m == 0; };
  if (!al(q, 16) || !al(k, 16) || !al(v, 16) || !al(skip, 16) || !al(edge, 16) || !al(out, 16) || !al(b_sbf, 16) ||
      !al(sbfproj_out, 16) || !al(sbf_p_out, 16) || !al(row_stats, 8) || !al(atom_info, 16))
    return X2G_EUNSUPPORTED;
  FwdSfArgs a{};
  a.info = reinterpret_cast<const int4*>(atom_info);
  a.pp = sbf_p_out;
  a.q = q; a.k = k; a.v = v; a.skip = skip; a.edge = edge; a.src_row = src_row; a.radial = radial; a.y = sph_y;
  a.w = w_sbf; a.bias = b_sbf; a.atom_rowptr = atom_rowptr; a.edge_rev = edge_rev; a.rev_trip = rev_trip;
  a.order = atom_order; a.packs = pack_ptr; a.atom0 = unit0; a.n_atoms = n_units;
  a.max_rows = max_rows > 0 ? max_rows : 1; a.H = heads;
  a.sqrt_c = static_cast<float>(sqrt(static_cast<double>(channels)));
  a.out = out; a.alpha = alpha_raw; a.smax = seg_max; a.sden = seg_den; a.sp = sbfproj_out;
  a.row_stats = reinterpret_cast<float2*>(row_stats);
  const bool edge_on = edge_mode == X2G_EDGE_PER_DST;
  hipStream_t st = as_stream(stream);
  switch (channels / 4) {
    case 1: return fwd_sf_launch<1>(a, edge_on, st);
    case 2: return fwd_sf_launch<2>(a, edge_on, st);
    case 4: return fwd_sf_launch<4>(a, edge_on, st);
    case 8: return fwd_sf_launch<8>(a, edge_on, st);
    default: return X2G_EUNSUPPORTED;
  }
}

X2G_API size_t x2g_sbf_attention_fwd_center_sf_tiled_lds(void) { return fwd_sf_tiled_lds(); }

X2G_API int x2g_sbf_attention_fwd_center_sf_tiled(const float* q, const float* k, const float* v, const float* skip,
                                                  const float* edge, const int32_t* src_row, int edge_mode,
                                                  const float* radial, const float* sph_y, const float* w_sbf,
                                                  const float* b_sbf, const int32_t* atom_rowptr,
                                                  const int32_t* edge_rev, const int32_t* rev_trip,
                                                  const int32_t* atom_order, const int32_t* pack_ptr,
                                                  const int32_t* atom_info, int64_t unit0, int64_t n_units,
                                                  int32_t max_degree, int32_t skip_rows, int64_t num_edges,
                                                  int64_t num_triplets,
                                                  int32_t heads, int32_t channels, float* out, float* alpha_raw,
                                                  float* seg_max, float* seg_den, float* row_stats,
                                                  float* sbfproj_out, float* sbf_p_out, void* stream) {
  if (n_units < 0 || unit0 < 0 || num_edges < 0 || num_triplets < 0 || heads <= 0 || channels <= 0)
    return X2G_EINVAL;
  if (edge_mode != X2G_EDGE_NONE && edge_mode != X2G_EDGE_PER_DST) return X2G_EUNSUPPORTED;
  if (heads * channels != kCD || channels % 4 || max_degree < 0 || max_degree > X2G_CENTER_MAX_DEGREE)
    return X2G_EUNSUPPORTED;
  if (n_units == 0 || num_edges == 0) return X2G_OK;
  if (!q || !k || !v || !skip || !radial || !sph_y || !w_sbf || !b_sbf || !atom_rowptr || !edge_rev || !rev_trip ||
      !out || !seg_max || !seg_den || (pack_ptr && !atom_order))
    return X2G_EINVAL;
  if (edge_mode == X2G_EDGE_PER_DST && (!edge || !src_row)) return X2G_EINVAL;
  const auto al = [](const void* p, int m) { return p == nullptr || reinterpret_cast<uintptr_t>(p) % m == 0; };
  if (!al(q, 16) || !al(k, 16) || !al(v, 16) || !al(skip, 16) || !al(edge, 16) || !al(out, 16) || !al(b_sbf, 16) ||
      !al(sbfproj_out, 16) || !al(sbf_p_out, 16) || !al(row_stats, 8) || !al(atom_info, 16))
    return X2G_EUNSUPPORTED;
  FwdSfArgs a{};
  a.info = reinterpret_cast<const int4*>(atom_info);
  a.pp = sbf_p_out;
  a.q = q; a.k = k; a.v = v; a.skip = skip; a.edge = edge; a.src_row = src_row; a.radial = radial; a.y = sph_y;
  a.w = w_sbf; a.bias = b_sbf; a.atom_rowptr = atom_rowptr; a.edge_rev = edge_rev; a.rev_trip = rev_trip;
  a.order = atom_order; a.packs = pack_ptr; a.atom0 = unit0; a.n_atoms = n_units;
  a.max_rows = max_degree > 0 ? max_degree : 1; a.H = heads; a.skip_rows = skip_rows;
  a.sqrt_c = static_cast<float>(sqrt(static_cast<double>(channels)));
  a.out = out; a.alpha = alpha_raw; a.smax = seg_max; a.sden = seg_den; a.sp = sbfproj_out;
  a.row_stats = reinterpret_cast<float2*>(row_stats);
  const bool edge_on = edge_mode == X2G_EDGE_PER_DST;
  const int md = max_degree > 0 ? max_degree : 1;
  hipStream_t st = as_stream(stream);
  switch (channels / 4) {
    case 1: return fwd_sf_tiled_launch<1>(a, edge_on, md, st);
    case 2: return fwd_sf_tiled_launch<2>(a, edge_on, md, st);
    case 4: return fwd_sf_tiled_launch<4>(a, edge_on, md, st);
    case 8: return fwd_sf_tiled_launch<8>(a, edge_on, md, st);
    default: return X2G_EUNSUPPORTED;
  }
}
