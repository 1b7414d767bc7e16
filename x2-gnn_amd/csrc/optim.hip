// The reference trainer's parameter update (trainer.py:39-48, train_ema.py:45-48) over ONE flat
// fp32 parameter buffer: clip_grad_norm_(max_norm) -> Adam(amsgrad=False) -> EMA
// (AveragedModel with avg_fn = d*avg + (1-d)*p).  torch's capturable Adam issues a few kernels
// per parameter tensor (~300 launches for X2-GNN's 155 tensors); here it is two launches:
//   1. per-block partial sums of g^2 over contiguous chunks (fixed order); block 0 also advances
//      the step count, the learning-rate schedule and Adam's bias corrections (no block of this
//      launch reads them),
//   2. elementwise Adam + EMA (a copy of the parameters at step 1, as AveragedModel does); every
//      block sums the kNormBlocks partials itself in the same fixed order (1 KB of L2 reads a
//      block: one per thread, shuffle sums), so all blocks see one bit-identical norm without a
//      finaliser launch or a fence, and block 0 publishes the norm and clip coefficient.
// Every value the update depends on that changes between steps (step count, norm, clip scale)
// lives in device memory, so a captured HIP graph replays correctly; the hyper-parameters
// (lr, betas, eps, max_norm, ema decay) are read from the same device scalar block so a
// scheduler may rewrite them between replays.
#include <math.h>

#include "common.hpp"

namespace x2g {

constexpr int kNormBlocks = 256;
constexpr int kNormThreads = 256;

// scalars layout (float[16]); see x2g.h X2G_OPT_*
__global__ void __launch_bounds__(kNormThreads) grad_sq_partial(const float4* __restrict__ g4,
                                                                const float* __restrict__ g, int64_t n,
                                                                float* __restrict__ partial,
                                                                float* __restrict__ sc) {
  __shared__ float red[kNormThreads];
  const int64_t n4 = n >> 2;
  const int64_t per = (n4 + gridDim.x - 1) / gridDim.x;
  const int64_t lo = per * blockIdx.x, hi = lo + per < n4 ? lo + per : n4;
  float s = 0.f;
  for (int64_t i = lo + threadIdx.x; i < hi; i += kNormThreads) {
    const float4 v = g4[i];
    s = fmaf(v.x, v.x, s);
    s = fmaf(v.y, v.y, s);
    s = fmaf(v.z, v.z, s);
    s = fmaf(v.w, v.w, s);
  }
  if (blockIdx.x == 0)  // the n % 4 tail
    for (int64_t i = 4 * n4 + threadIdx.x; i < n; i += kNormThreads) s = fmaf(g[i], g[i], s);
  red[threadIdx.x] = s;
  __syncthreads();
  for (int off = kNormThreads / 2; off > 0; off >>= 1) {
    if (static_cast<int>(threadIdx.x) < off) red[threadIdx.x] += red[threadIdx.x + off];
    __syncthreads();
  }
  if (threadIdx.x == 0) partial[blockIdx.x] = red[0];
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    const float step = sc[X2G_OPT_STEP] + 1.0f;
    sc[X2G_OPT_STEP] = step;
    if (sc[X2G_OPT_WARMUP] > 0.f) {  // LinearWarmupExponentialDecay.lr_lambda(t), t = steps taken before this one
      const double w = sc[X2G_OPT_WARMUP], t = static_cast<double>(step) - 1.0;
      const double warm = fmin(1.0 / w + 1.0 / w * t, 1.0);
      double ex = t / static_cast<double>(sc[X2G_OPT_DECAY_STEPS]);
      if (sc[X2G_OPT_STAIRCASE] != 0.f) ex = floor(ex);
      sc[X2G_OPT_LR] = static_cast<float>(static_cast<double>(sc[X2G_OPT_BASE_LR]) * warm *
                                          pow(static_cast<double>(sc[X2G_OPT_DECAY_RATE]), ex));
    }
    // bias corrections as torch.optim.Adam computes them (in double, rounded to float)
    const double b1 = sc[X2G_OPT_BETA1], b2 = sc[X2G_OPT_BETA2];
    sc[X2G_OPT_STEP_SIZE] = static_cast<float>(sc[X2G_OPT_LR] / (1.0 - pow(b1, static_cast<double>(step))));
    sc[X2G_OPT_BC2_SQRT] = static_cast<float>(sqrt(1.0 - pow(b2, static_cast<double>(step))));
  }
}

__global__ void __launch_bounds__(kNormThreads) adam_ema(float* __restrict__ p, float* __restrict__ g,
                                                         float* __restrict__ m, float* __restrict__ v,
                                                         float* __restrict__ ema, int64_t n,
                                                         const float* __restrict__ partial, float* __restrict__ sc,
                                                         int zero_grads) {
  static_assert(kNormBlocks == kNormThreads, "one partial per thread");
  __shared__ float red[kNormThreads / 64];
  __shared__ float clip_s;
  // the squared norm: one partial per thread, xor-shuffle sums per wave, the 4 wave sums in order — the
  // same order in every block, so every block holds the same bits
  float s = partial[threadIdx.x];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float norm = sqrtf((red[0] + red[1]) + (red[2] + red[3]));
    const float max_norm = sc[X2G_OPT_MAX_NORM];
    // torch.nn.utils.clip_grad_norm_: coef = max_norm / (norm + 1e-6), clamped to <= 1
    const float coef = max_norm > 0.f ? fminf(max_norm / (norm + 1e-6f), 1.0f) : 1.0f;
    clip_s = coef;
    if (blockIdx.x == 0) {  // published for the caller; no block of this launch reads them back
      sc[X2G_OPT_NORM] = norm;
      sc[X2G_OPT_CLIP] = coef;
    }
  }
  __syncthreads();
  // step size and bias correction were formed by grad_sq_partial's block 0 (one double pow per step)
  const float clip = clip_s, step_size = sc[X2G_OPT_STEP_SIZE], bc2s = sc[X2G_OPT_BC2_SQRT];
  const float b1 = sc[X2G_OPT_BETA1], b2 = sc[X2G_OPT_BETA2], eps = sc[X2G_OPT_EPS];
  const float d = sc[X2G_OPT_EMA_DECAY];
  // AveragedModel.update_parameters copies the parameters on its first call (n_averaged == 0) and
  // applies avg_fn from the second on; the step count is already on the device (graph-safe)
  const bool first = sc[X2G_OPT_STEP] == 1.0f;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
    const float gi = g[i] * clip;
    if (zero_grads) g[i] = 0.0f;  // zero_grad() folded into the step
    // exp_avg.lerp_(grad, 1 - beta1); exp_avg_sq.mul_(beta2).addcmul_(grad, grad, 1 - beta2)
    const float mi = m[i] + (1.0f - b1) * (gi - m[i]);
    const float vi = v[i] * b2 + (1.0f - b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    // param.addcdiv_(exp_avg, sqrt(exp_avg_sq) / sqrt(bc2) + eps, value=-lr/bc1)
    const float denom = sqrtf(vi) / bc2s + eps;
    const float pi = p[i] - step_size * (mi / denom);
    p[i] = pi;
    // ema.lerp_(p, 1 - d)
    if (ema) ema[i] = first ? pi : ema[i] + (1.0f - d) * (pi - ema[i]);
  }
}

}  // namespace x2g

using namespace x2g;

X2G_API size_t x2g_optimizer_workspace(int64_t n) { return n > 0 ? kNormBlocks * sizeof(float) : 0; }

static int clip_adam_ema(float* params, float* grads, float* exp_avg, float* exp_avg_sq, float* ema, int64_t n,
                         float* scalars, int zero_grads, void* workspace, size_t workspace_bytes, void* stream) {
  if (n < 0 || !scalars) return X2G_EINVAL;
  if (n == 0) return X2G_OK;
  if (!params || !grads || !exp_avg || !exp_avg_sq) return X2G_EINVAL;
  if (!workspace || workspace_bytes < x2g_optimizer_workspace(n)) return X2G_EWORKSPACE;
  if (reinterpret_cast<uintptr_t>(grads) % 16) return X2G_EINVAL;
  hipStream_t st = as_stream(stream);
  float* partial = static_cast<float*>(workspace);
  grad_sq_partial<<<kNormBlocks, kNormThreads, 0, st>>>(reinterpret_cast<const float4*>(grads), grads, n, partial,
                                                         scalars);
  const int64_t want = (n + kNormThreads - 1) / kNormThreads;
  adam_ema<<<static_cast<unsigned>(want < 2048 ? want : 2048), kNormThreads, 0, st>>>(
      params, grads, exp_avg, exp_avg_sq, ema, n, partial, scalars, zero_grads);
  return last_launch_status();
}

X2G_API int x2g_clip_adam_ema(float* params, const float* grads, float* exp_avg, float* exp_avg_sq, float* ema,
                              int64_t n, float* scalars, void* workspace, size_t workspace_bytes, void* stream) {
  return clip_adam_ema(params, const_cast<float*>(grads), exp_avg, exp_avg_sq, ema, n, scalars, 0, workspace,
                       workspace_bytes, stream);
}

X2G_API int x2g_clip_adam_ema_ex(float* params, float* grads, float* exp_avg, float* exp_avg_sq, float* ema, int64_t n,
                                 float* scalars, int flags, void* workspace, size_t workspace_bytes, void* stream) {
  if (flags & ~X2G_OPT_ZERO_GRADS) return X2G_EINVAL;
  return clip_adam_ema(params, grads, exp_avg, exp_avg_sq, ema, n, scalars, (flags & X2G_OPT_ZERO_GRADS) ? 1 : 0,
                       workspace, workspace_bytes, stream);
}
