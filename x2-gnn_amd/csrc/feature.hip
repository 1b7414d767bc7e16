// Line-node featurisation MLP (xgnn.py:64-67 of this package; reference xgnn.py:49-56):
//     neo_x = SiLU(emb_trans(SiLU(mat_trans(edge_attr * env))))
// edge_attr [E, 338] (per-line-node input features), env [E] (the polynomial envelope), mat_trans
// 338 -> 256, emb_trans 256 -> 128.  As two generic dense launches plus a torch multiply this was
// 108 us forward and ~180 us backward per config-2 step (scalar-load row kernels, a 338-wide
// weight gradient split 132 ways into 45 MB of slabs).  Here:
//
//   forward  — ONE kernel: a workgroup (one per CU) takes 32-row tiles, stages the tile of
//              edge_attr * env in LDS (the span is contiguous: 16-byte loads, scaled and scattered
//              into 388-float rows), runs both products on v_mfma_f32_16x16x4_f32 with the
//              256-wide hidden tile kept in LDS, and writes neo_x plus the backward's operands in
//              the tiled-transposed layout (x2g.h: 16-row tiles, feature-major inside a tile,
//              128-feature planes): x*env, z1, SiLU(z1), z2.
//   backward — ONE data kernel (dz2 = dy SiLU'(z2), dy1 = dz2 W2, dz1 = dy1 SiLU'(z1), both dz in
//              T layout) and the weight gradients as eight 128 x 128 T-layout jobs of
//              x2g_tiled_wgrad (mat_trans: 2 x 3 blocks, emb_trans: 1 x 2), written into the
//              weights through strided slab sums.
//
// MFMA operand convention as the row chains: lane l = (i = l & 15, g = l >> 4); the contraction
// index of k-step s in 16-group q is 16q + 4g + s, so one 16-byte read per lane and group feeds
// four MFMAs; D lane l holds rows 4g + e, column i of a 16 x 16 block — the T layout's f4.
#include "common.hpp"

namespace x2g {
namespace {

typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int kFN1 = 256;             // mat_trans outputs
constexpr int kFN2 = 128;             // emb_trans outputs
constexpr int kFKMax = 384;           // input features, padded: 3 T planes
constexpr int kFRows = 32;            // rows per tile (two 16-row MFMA blocks)
// LDS row strides of the input tile and the hidden tile: == 8 mod 64 floats (2 mod 16 chunks), which
// makes the MFMA operand read of lane (i, g) — 16 bytes at row i, chunk 4q + g — hit 16 distinct bank
// quads in each of ds_read_b128's four lane groups ({0-3, 12-15, 20-27}, {4-11, 16-19, 28-31}, ...).
// The former stride (== 4 mod 64) left 2-way conflicts in those groups: SQ_LDS_BANK_CONFLICT /
// SQ_LDS_IDX_ACTIVE = 0.49 on the r4d PMC pass.  (scripts: the layout search is in DESIGN.md §3.)
constexpr int kFAS = kFKMax + 8;
constexpr int kFYS = kFN1 + 8;
constexpr int kFThreads = 512;

__device__ __forceinline__ f4 mfma4(float a, float b, f4 acc) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
}
// SiLU and its derivative from the hardware exp2 / reciprocal (v_exp_f32, v_rcp_f32: ~1 ulp each), as
// the row chains: libm expf and IEEE division are ~25 VALU instructions per element, 24 elements per
// lane and tile in the forward's epilogues, which run between barriers with no MFMA to hide behind.
// sigmoid(z) = rcp(1 + 2^(-z log2 e)); z -> -inf gives 0, z -> +inf gives 1, NaN stays NaN.
__device__ __forceinline__ float sigmoid_(float z) {
  return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-1.4426950408889634f * z));
}
__device__ __forceinline__ float silu_(float z) { return z * sigmoid_(z); }
__device__ __forceinline__ float silu_grad_(float z) {
  const float s = sigmoid_(z);
  return s * (1.0f + z * (1.0f - s));
}
__device__ __forceinline__ f4 zero4() { return f4{0.f, 0.f, 0.f, 0.f}; }

// 4 x 4 transpose inside each lane quad (DPP quad permutes, no LDS): lane 4m + j holding v[e] =
// element (e, j) of its quad's 4 x 4 block ends with v[k] = element (j, k)
__device__ __forceinline__ f4 quad_t(f4 v, int j) {
  f4 b, c;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float t = dpp_mov<0xB1>(v[k ^ 1]);
    b[k] = ((k ^ j) & 1) ? t : v[k];
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float t = dpp_mov<0x4E>(b[k ^ 2]);
    c[k] = ((k ^ j) & 2) ? t : b[k];
  }
  return c;
}

// T layout: element (r, f) of a [R, 128 P] tensor at plane (f >> 7) * tf + (r >> 4) * 2048 +
// (f & 127) * 16 + (r & 15); a lane's D block rows 4g..4g+3 at column f are one float4.
__device__ __forceinline__ int64_t tpos(int64_t tf, int64_t tile16, int f, int g) {
  return (f >> 7) * tf + tile16 * 2048 + (f & 127) * 16 + 4 * g;
}

struct FeatFwdArgs {
  const float* x;    // [R, K]
  const float* env;  // [R] or NULL
  const float* w1;   // [256, K]
  const float* b1;   // [256] or NULL
  const float* w2;   // [128, 256]
  const float* b2;   // [128] or NULL
  float* y2;         // [R, 128]
  float* xs_t;       // 3 planes: x * env
  float* z1_t;       // 2 planes
  float* y1_t;       // 2 planes
  float* z2_t;       // 1 plane
  int64_t R;
  int64_t tf;        // floats per T plane
  int K;
  int want_t;        // write the backward's T-layout operands (0: inference, the four pointers NULL)
};

// W1 operand of 16-group q for column c: W1[c][16q + 4g .. +3] as two 8-byte loads (K is even,
// so rows start 8-byte aligned), zero (from a clamped in-bounds address) past K.
__device__ __forceinline__ f4 w1_frag(const float* __restrict__ w1, int K, int c, int q, int g) {
  const int k = 16 * q + 4 * g;
  const int k0 = k < K ? k : K - 2, k1 = k + 2 < K ? k + 2 : K - 2;
  const float2 lo = *reinterpret_cast<const float2*>(w1 + c * K + k0);
  const float2 hi = *reinterpret_cast<const float2*>(w1 + c * K + k1);
  const float m0 = k < K ? 1.0f : 0.0f, m1 = k + 2 < K ? 1.0f : 0.0f;
  return f4{lo.x * m0, lo.y * m0, hi.x * m1, hi.y * m1};
}

constexpr int kFX4 = (kFRows * kFKMax / 4 + kFThreads - 1) / kFThreads;  // staged float4 per thread

// The tile's span x[r0 .. r0 + nr) is contiguous and 16-byte aligned (r0 * K * 4 is a multiple of
// 16): thread t holds float4 t + 512 u in registers (the next tile's are loaded during the current
// tile's products); env of the tile's rows rides along in threads 0..31.
struct XTile {
  f4 v[kFX4];
  float env;
};

__device__ __forceinline__ void xtile_load(const FeatFwdArgs& a, int64_t tile, XTile& t) {
  const int64_t r0 = tile * kFRows;
  const int64_t R = a.R;
  const int nr = R - r0 < kFRows ? static_cast<int>(R - r0) : kFRows;
  const float* src = a.x + r0 * a.K;
  const int n = nr * a.K;
#pragma unroll
  for (int u = 0; u < kFX4; ++u) {
    const int q = threadIdx.x + kFThreads * u;
    if (4 * q + 3 < n) {
      t.v[u] = *reinterpret_cast<const f4*>(src + 4 * q);
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) t.v[u][e] = 4 * q + e < n ? src[4 * q + e] : 0.0f;
    }
  }
  const int r = threadIdx.x;
  t.env = (r < nr && a.env) ? a.env[r0 + r] : 1.0f;
}

__global__ void __launch_bounds__(kFThreads, 1) feat_fwd_kernel(const FeatFwdArgs a) {
  __shared__ __attribute__((aligned(16))) float A[kFRows * kFAS];   // x tile (unscaled), zero-padded
  __shared__ __attribute__((aligned(16))) float Y1[kFRows * kFYS];  // SiLU(z1) tile
  __shared__ float envs[kFRows];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int i = lane & 15, g = lane >> 4;
  const int K = a.K, KQ = (K + 15) / 16;
  const float invK = 1.0f / static_cast<float>(K);
  const int64_t R = a.R;
  // emb_trans slice of this wave (output columns 16w + i), kept in registers for every tile
  // emb_trans slice of this wave (output columns 16w + i): read from L2 in the second product, two
  // groups ahead, like mat_trans's in the first (held in registers for every tile it took 64 VGPRs,
  // which left none for the interleaved T-layout stores)
  const float* w2s = a.w2 + (16 * w + i) * kFN1 + 4 * g;
  const float b2v = a.b2 ? a.b2[16 * w + i] : 0.0f;
  const int c1a = 32 * w + i, c1b = c1a + 16;  // this wave's two mat_trans column blocks
  const float b1a = a.b1 ? a.b1[c1a] : 0.0f, b1b = a.b1 ? a.b1[c1b] : 0.0f;
  // the pad columns K..kFKMax stay zero for every tile
  for (int idx = tid; idx < kFRows * (kFKMax - K); idx += kFThreads) {
    const int r = idx / (kFKMax - K), c = K + idx % (kFKMax - K);
    A[r * kFAS + c] = 0.0f;
  }
  const int64_t ntiles = (R + kFRows - 1) / kFRows;
  XTile xt;
  if (static_cast<int64_t>(blockIdx.x) < ntiles) xtile_load(a, blockIdx.x, xt);
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int64_t r0 = tile * kFRows;
    const int nr = R - r0 < kFRows ? static_cast<int>(R - r0) : kFRows;
    __syncthreads();  // the previous tile's products no longer read A / Y1 / envs
    {  // scatter the staged span into 388-float rows (rows past nr: zero)
      const int n = nr * K;
#pragma unroll
      for (int u = 0; u < kFX4; ++u) {
        const int q = tid + kFThreads * u;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int j = 4 * q + e;
          if (j < kFRows * K) {
            int r = static_cast<int>(static_cast<float>(j) * invK);  // j / K, corrected below
            r -= r * K > j ? 1 : 0;
            r += (r + 1) * K <= j ? 1 : 0;
            A[r * kFAS + (j - r * K)] = j < n ? xt.v[u][e] : 0.0f;
          }
        }
      }
      if (tid < kFRows) envs[tid] = xt.env;
    }
    __syncthreads();
    // the first two W1 groups before the next tile's span: loads retire in order, so issued after the
    // span's (HBM) loads they would wait for them at the first MFMA (one HBM round trip per tile)
    f4 wa0 = w1_frag(a.w1, K, c1a, 0, g), wb0 = w1_frag(a.w1, K, c1b, 0, g);
    f4 wa1 = w1_frag(a.w1, K, c1a, 1, g), wb1 = w1_frag(a.w1, K, c1b, 1, g);
    if (tile + gridDim.x < ntiles) xtile_load(a, tile + gridDim.x, xt);  // in flight during the products
    // x * env in T layout: per 16-row tile and plane, float4 u of the 2048-float block holds
    // feature u >> 2, rows 4 (u & 3) .. +3.  (Issuing these 48 KB one piece per iteration of the first
    // product's loop instead measured slower: profiles/r4f_ab_feat.txt, variant fnew vs fw2only.)
    auto xs_store = [&](int it) {  // block it = (16-row tile rt, plane p) of six; float4 u = tid (it uniform)
      const int rt = it / 3, p = it % 3;
      const int64_t t16 = r0 / 16 + rt;
      if (!a.want_t || t16 * 16 >= R || 128 * p >= K) return;
      const int f = tid >> 2, rr = 16 * rt + 4 * (tid & 3);
      f4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = A[(rr + e) * kFAS + 128 * p + f] * envs[rr + e];
      *reinterpret_cast<f4*>(a.xs_t + p * a.tf + t16 * 2048 + 4 * tid) = v;
    };
    // z1 = env (x W1^T) + b1: wave w -> columns c1a, c1b, both 16-row blocks
    f4 acc[2][2] = {{zero4(), zero4()}, {zero4(), zero4()}};
    // W1 operands two groups ahead (set 0: even groups, set 1: odd; a set is reloaded right after
    // its MFMAs issue), the A rows of the next group read before this group's MFMAs
    const int KQn = KQ;
    f4 a0 = *reinterpret_cast<const f4*>(A + i * kFAS + 4 * g);
    f4 a1 = *reinterpret_cast<const f4*>(A + (16 + i) * kFAS + 4 * g);
    auto group = [&](int q, f4& ba, f4& bb) {
      const int qa = q + 1 < KQn ? q + 1 : q;
      const f4 n0 = *reinterpret_cast<const f4*>(A + i * kFAS + 16 * qa + 4 * g);
      const f4 n1 = *reinterpret_cast<const f4*>(A + (16 + i) * kFAS + 16 * qa + 4 * g);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        acc[0][0] = mfma4(a0[e], ba[e], acc[0][0]);
        acc[0][1] = mfma4(a0[e], bb[e], acc[0][1]);
        acc[1][0] = mfma4(a1[e], ba[e], acc[1][0]);
        acc[1][1] = mfma4(a1[e], bb[e], acc[1][1]);
      }
      const int qb = q + 2 < KQn ? q + 2 : q;
      ba = w1_frag(a.w1, K, c1a, qb, g);
      bb = w1_frag(a.w1, K, c1b, qb, g);
      a0 = n0;
      a1 = n1;
    };
    for (int q = 0; q < KQn; q += 2) {
      group(q, wa0, wb0);
      if (q + 1 < KQn) group(q + 1, wa1, wb1);
    }
    f4 wq[3];  // the second product's first two W2 groups, in flight under the epilogue and barrier
    wq[0] = *reinterpret_cast<const f4*>(w2s);
    wq[1] = *reinterpret_cast<const f4*>(w2s + 16);
    // epilogue 1: z1 / SiLU(z1) to T layout (rows past R zero) and SiLU(z1) to LDS.  (Holding z1 / SiLU(z1)
    // in registers and storing them under the second product's MFMAs measured slower:
    // profiles/r4f_ab_feat.txt, variant fnew vs fnot1.)
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
      const int64_t t16 = r0 / 16 + rb;
      const bool tile_ok = t16 * 16 < R;
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {
        const int c = cb ? c1b : c1a;
        const float bias = cb ? b1b : b1a;
        f4 z, y;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int r = 16 * rb + 4 * g + e;
          const bool ok = r < nr;
          z[e] = ok ? fmaf(acc[rb][cb][e], envs[r], bias) : 0.0f;  // (x * env) W^T = env (x W^T)
          y[e] = ok ? silu_(z[e]) : 0.0f;
          Y1[r * kFYS + c] = y[e];
        }
        if (tile_ok && a.want_t) {
          *reinterpret_cast<f4*>(a.z1_t + tpos(a.tf, t16, c, g)) = z;
          *reinterpret_cast<f4*>(a.y1_t + tpos(a.tf, t16, c, g)) = y;
        }
      }
    }
    __syncthreads();
    // z2 = SiLU(z1) W2^T + b2: wave w -> columns 16w + i
    f4 acc2[2] = {zero4(), zero4()};
    {
      f4 y0 = *reinterpret_cast<const f4*>(Y1 + i * kFYS + 4 * g);
      f4 y1 = *reinterpret_cast<const f4*>(Y1 + (16 + i) * kFYS + 4 * g);
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int qa = q + 1 < 16 ? q + 1 : q;
        const f4 n0 = *reinterpret_cast<const f4*>(Y1 + i * kFYS + 16 * qa + 4 * g);
        const f4 n1 = *reinterpret_cast<const f4*>(Y1 + (16 + i) * kFYS + 16 * qa + 4 * g);
        if (q + 2 < 16) wq[(q + 2) % 3] = *reinterpret_cast<const f4*>(w2s + 16 * (q + 2));
        // pins the group-(q + 2) load ahead of group q's MFMAs: left alone, the scheduler hoisted the
        // MFMAs over it, so each load issued one group ahead and was waited for (vmcnt(0)) after only
        // 8 MFMAs — an L2 round trip not covered
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          acc2[0] = mfma4(y0[e], wq[q % 3][e], acc2[0]);
          acc2[1] = mfma4(y1[e], wq[q % 3][e], acc2[1]);
        }
        y0 = n0;
        y1 = n1;
      }
    }
    const int c2 = 16 * w + i;
    // neo_x leaves as 16-byte row pieces: lane (i = 4m + j, g) holds rows 4g + e of column c2, and
    // after the quad transpose row 4g + j, columns 16w + 4m .. +3 (one store per block, not four)
    const int qj = i & 3, qm = i >> 2;
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
      const int64_t t16 = r0 / 16 + rb;
      if (t16 * 16 >= R) continue;
      f4 z, y;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int r = 16 * rb + 4 * g + e;
        z[e] = r < nr ? acc2[rb][e] + b2v : 0.0f;
        y[e] = silu_(z[e]);
      }
      const f4 yt = quad_t(y, qj);
      const int ry = 16 * rb + 4 * g + qj;
      if (ry < nr) *reinterpret_cast<f4*>(a.y2 + (r0 + ry) * kFN2 + 16 * w + 4 * qm) = yt;
      if (a.want_t) *reinterpret_cast<f4*>(a.z2_t + tpos(a.tf, t16, c2, g)) = z;
    }
    // x * env to T layout last (A and envs hold this tile until the next one's barrier): issued before the
    // products, these stores retired in order ahead of every W1 load behind them (a write round trip per tile)
    for (int it = 0; it < 6; ++it) xs_store(it);
  }
}

struct FeatBwdArgs {
  const float* dy;    // [R, 128] dL/d neo_x
  const float* z2_t;  // 1 plane
  const float* z1_t;  // 2 planes
  const float* w2;    // [128, 256]
  float* dz2_t;       // 1 plane
  float* dz1_t;       // 2 planes
  int64_t R;
  int64_t tf;
};

constexpr int kFDS = kFN2 + 8;  // LDS row stride of the dz2 tile (== 8 mod 64: conflict-free operand reads, as kFAS)

__global__ void __launch_bounds__(kFThreads, 1) feat_bwd_kernel(const FeatBwdArgs a) {
  __shared__ __attribute__((aligned(16))) float DZ[kFRows * kFDS];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int i = lane & 15, g = lane >> 4;
  const int64_t R = a.R;
  // dy1 = dz2 W2: B operand (n = 16q + 4g + e, column c) = W2[n][c] for this wave's two column
  // blocks c = 32w + i (+16), kept in registers for every tile
  const int ca = 32 * w + i, cb = ca + 16;
  f4 wa[8], wb[8];
#pragma unroll
  for (int q = 0; q < 8; ++q)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      wa[q][e] = a.w2[(16 * q + 4 * g + e) * kFN1 + ca];
      wb[q][e] = a.w2[(16 * q + 4 * g + e) * kFN1 + cb];
    }
  const int c2 = 16 * w + i;
  const int64_t ntiles = (R + kFRows - 1) / kFRows;
  // a tile's inputs: z2 (T layout) and dy of column c2 for both row blocks, and z1 of the wave's two
  // column blocks.  z2 / dy of the NEXT tile and z1 of this one are issued before this tile's barrier and
  // products, so they arrive under the MFMAs (one memory round trip per tile instead of three)
  struct In {
    f4 z2[2];
    float dy[2][4];
  };
  auto load_in = [&](int64_t tile, In& in) {
    const int64_t r0 = tile * kFRows;
    const int nr = R - r0 < kFRows ? static_cast<int>(R - r0) : kFRows;
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
      const int64_t t16 = r0 / 16 + rb;
      in.z2[rb] = t16 * 16 < R ? *reinterpret_cast<const f4*>(a.z2_t + tpos(a.tf, t16, c2, g)) : zero4();
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int r = 16 * rb + 4 * g + e;
        in.dy[rb][e] = r < nr ? a.dy[(r0 + r) * kFN2 + c2] : 0.0f;
      }
    }
  };
  In cur;
  if (static_cast<int64_t>(blockIdx.x) < ntiles) load_in(blockIdx.x, cur);
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int64_t r0 = tile * kFRows;
    const int nr = R - r0 < kFRows ? static_cast<int>(R - r0) : kFRows;
    __syncthreads();  // the previous tile's product no longer reads DZ
    // dz2 = dy SiLU'(z2): wave w -> column c2, both row blocks
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
      const int64_t t16 = r0 / 16 + rb;
      const bool tile_ok = t16 * 16 < R;
      f4 d;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int r = 16 * rb + 4 * g + e;
        d[e] = r < nr ? cur.dy[rb][e] * silu_grad_(cur.z2[rb][e]) : 0.0f;
        DZ[r * kFDS + c2] = d[e];
      }
      if (tile_ok) *reinterpret_cast<f4*>(a.dz2_t + tpos(a.tf, t16, c2, g)) = d;
    }
    f4 z1v[2][2];
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
      const int64_t t16 = r0 / 16 + rb;
      const int64_t tt = t16 * 16 < R ? t16 : r0 / 16;  // (a past-the-end block reads a valid one, unused)
#pragma unroll
      for (int k = 0; k < 2; ++k) z1v[rb][k] = *reinterpret_cast<const f4*>(a.z1_t + tpos(a.tf, tt, k ? cb : ca, g));
    }
    if (tile + gridDim.x < ntiles) load_in(tile + gridDim.x, cur);
    __syncthreads();
    f4 acc[2][2] = {{zero4(), zero4()}, {zero4(), zero4()}};
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const f4 a0 = *reinterpret_cast<const f4*>(DZ + i * kFDS + 16 * q + 4 * g);
      const f4 a1 = *reinterpret_cast<const f4*>(DZ + (16 + i) * kFDS + 16 * q + 4 * g);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        acc[0][0] = mfma4(a0[e], wa[q][e], acc[0][0]);
        acc[0][1] = mfma4(a0[e], wb[q][e], acc[0][1]);
        acc[1][0] = mfma4(a1[e], wa[q][e], acc[1][0]);
        acc[1][1] = mfma4(a1[e], wb[q][e], acc[1][1]);
      }
    }
    // dz1 = dy1 SiLU'(z1), T layout (rows past R are zero: their dz2 rows are)
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
      const int64_t t16 = r0 / 16 + rb;
      if (t16 * 16 >= R) continue;
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int c = k ? cb : ca;
        f4 d;
#pragma unroll
        for (int e = 0; e < 4; ++e) d[e] = acc[rb][k][e] * silu_grad_(z1v[rb][k][e]);
        *reinterpret_cast<f4*>(a.dz1_t + tpos(a.tf, t16, c, g)) = d;
      }
    }
  }
}

inline bool al16(const void* p) { return reinterpret_cast<uintptr_t>(p) % 16 == 0; }

inline unsigned feat_grid(int64_t R) {
  const int64_t tiles = (R + kFRows - 1) / kFRows;
  return static_cast<unsigned>(tiles < 256 ? tiles : 256);
}

}  // namespace
}  // namespace x2g

using namespace x2g;

X2G_API int x2g_feat_fwd(const float* x, const float* env, int64_t rows, int32_t in_dim, const float* w1,
                         const float* b1, const float* w2, const float* b2, float* y, float* xs_t, float* z1_t,
                         float* y1_t, float* z2_t, void* stream) {
  if (rows < 0 || in_dim <= 0) return X2G_EINVAL;
  if (in_dim > kFKMax || in_dim % 2 || in_dim <= 2 * 128 || rows * kFKMax * 4 >= (int64_t(1) << 31))
    return X2G_EUNSUPPORTED;
  if (rows == 0) return X2G_OK;
  if (!x || !w1 || !w2 || !y) return X2G_EINVAL;
  // the four T-layout outputs feed the backward: all given (training) or all NULL (inference)
  const int nt = (xs_t != nullptr) + (z1_t != nullptr) + (y1_t != nullptr) + (z2_t != nullptr);
  if (nt != 0 && nt != 4) return X2G_EINVAL;
  if (!al16(x) || !al16(w2) || !al16(xs_t) || !al16(z1_t) || !al16(y1_t) || !al16(z2_t) ||
      reinterpret_cast<uintptr_t>(w1) % 8)
    return X2G_EUNSUPPORTED;
  FeatFwdArgs a{x, env, w1, b1, w2, b2, y, xs_t, z1_t, y1_t, z2_t, rows, x2g_chain_t_floats(rows, 128), in_dim,
                nt == 4 ? 1 : 0};
  feat_fwd_kernel<<<feat_grid(rows), kFThreads, 0, as_stream(stream)>>>(a);
  return last_launch_status();
}

X2G_API int x2g_feat_bwd(const float* dy, const float* z2_t, const float* z1_t, const float* w2, int64_t rows,
                         float* dz2_t, float* dz1_t, void* stream) {
  if (rows < 0) return X2G_EINVAL;
  if (rows * kFKMax * 4 >= (int64_t(1) << 31)) return X2G_EUNSUPPORTED;
  if (rows == 0) return X2G_OK;
  if (!dy || !z2_t || !z1_t || !w2 || !dz2_t || !dz1_t) return X2G_EINVAL;
  if (!al16(z2_t) || !al16(z1_t) || !al16(dz2_t) || !al16(dz1_t)) return X2G_EUNSUPPORTED;
  FeatBwdArgs a{dy, z2_t, z1_t, w2, dz2_t, dz1_t, rows, x2g_chain_t_floats(rows, 128)};
  feat_bwd_kernel<<<feat_grid(rows), kFThreads, 0, as_stream(stream)>>>(a);
  return last_launch_status();
}

