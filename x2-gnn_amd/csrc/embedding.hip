// The element embedding table of EmbeddingBlock (atom_embedding.py:13-25) in one launch.
//
// xgnn_poly embeds every atom (and, through edge_attr = emb(Z_j), every triplet) with
// nn.Embedding(10, D, padding_idx=0, max_norm=3, scale_grad_by_freq=True); the model only needs
// the <= 10 distinct rows (model.py / xgnn.py hoist).  The torch form of
// that is a dozen tiny launches per step (counts, norms, the conditional rescale, a copy); here
// it is one workgroup: an integer histogram of Z in LDS, one wave per row for the norm and the
// in-place renorm, and the table copy.  The backward divides by the counts and zeroes the
// padding row, accumulating straight into the gradient buffer.
#include "common.hpp"

namespace x2g {

constexpr int kEmbMaxRows = 64;

__global__ void __launch_bounds__(256) embedding_table_kernel(float* __restrict__ w, const int64_t* __restrict__ z,
                                                              int64_t N, int V, int D, float max_norm,
                                                              float* __restrict__ counts, float* __restrict__ table) {
  __shared__ int hist[kEmbMaxRows];
  for (int v = threadIdx.x; v < V; v += blockDim.x) hist[v] = 0;
  __syncthreads();
  // the atoms' numbers a batch of kEmbUnroll per thread at a time: every load of the batch in flight
  // together (a load-then-add loop runs one memory round trip per 256 atoms)
  constexpr int kEmbUnroll = 16;
  for (int64_t n0 = threadIdx.x; n0 < N; n0 += static_cast<int64_t>(blockDim.x) * kEmbUnroll) {
    int64_t zv[kEmbUnroll];
#pragma unroll
    for (int u = 0; u < kEmbUnroll; ++u) {
      const int64_t n = n0 + static_cast<int64_t>(u) * blockDim.x;
      zv[u] = z[n < N ? n : 0];
    }
#pragma unroll
    for (int u = 0; u < kEmbUnroll; ++u) {
      const int64_t v = zv[u];
      if (n0 + static_cast<int64_t>(u) * blockDim.x < N && v >= 0 && v < V) atomicAdd(&hist[v], 1);
    }
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nwaves = blockDim.x >> 6;
  for (int v = wave; v < V; v += nwaves) {
    float* row = w + static_cast<int64_t>(v) * D;
    float ss = 0.f;
    for (int c = lane; c < D; c += 64) ss = fmaf(row[c], row[c], ss);
    ss = group_sum<64>(ss);
    const float norm = sqrtf(ss);
    const bool rescale = max_norm > 0.f && hist[v] > 0 && norm > max_norm;
    const float scale = max_norm / (norm + 1e-7f);
    for (int c = lane; c < D; c += 64) {
      const float x = rescale ? row[c] * scale : row[c];
      if (rescale) row[c] = x;
      table[static_cast<int64_t>(v) * D + c] = x;
    }
    if (lane == 0 && counts) counts[v] = static_cast<float>(hist[v]);
  }
}

__global__ void embedding_table_bwd_kernel(const float* __restrict__ g, const float* __restrict__ counts, int V, int D,
                                           int pad, int accum, float* __restrict__ dw) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= V * D) return;
  const int v = i / D;
  float d = 0.f;
  if (v != pad) d = counts ? g[i] / fmaxf(counts[v], 1.0f) : g[i];
  dw[i] = accum ? dw[i] + d : d;
}

}  // namespace x2g

using namespace x2g;

X2G_API int x2g_embedding_table(float* weight, const int64_t* z, int64_t N, int32_t V, int32_t D, float max_norm,
                                float* counts, float* table, void* stream) {
  if (N < 0 || V <= 0 || V > kEmbMaxRows || D <= 0 || !weight || !table || (N > 0 && !z)) return X2G_EINVAL;
  embedding_table_kernel<<<1, 256, 0, as_stream(stream)>>>(weight, z, N, V, D, max_norm, counts, table);
  return last_launch_status();
}

X2G_API int x2g_embedding_table_bwd(const float* g, const float* counts, int32_t V, int32_t D, int32_t pad,
                                    float* dw, int flags, void* stream) {
  if (V <= 0 || D <= 0 || !g || !dw) return X2G_EINVAL;
  embedding_table_bwd_kernel<<<blocks_for(static_cast<int64_t>(V) * D, 256), 256, 0, as_stream(stream)>>>(
      g, counts, V, D, pad, (flags & X2G_ACCUM_WGRAD) ? 1 : 0, dw);
  return last_launch_status();
}
