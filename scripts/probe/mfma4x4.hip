// Probe: operand / result lane maps and issue cost of v_mfma_f32_4x4x1_16b_f32 (16 blocks of 4x4, K = 1)
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f4 __attribute__((ext_vector_type(4)));

__global__ void layout(const float* a, const float* b, float* d) {
  const int l = threadIdx.x;
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  acc = __builtin_amdgcn_mfma_f32_4x4x1f32(a[l], b[l], acc, 0, 0, 0);
  for (int e = 0; e < 4; ++e) d[l * 4 + e] = acc[e];
}

template <int NACC>
__global__ void rate(float* out, long long* cyc, int iters) {
  const int l = threadIdx.x;
  f4 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = f4{0.f, 0.f, 0.f, 0.f};
  float a = 1e-3f * l, b = 2e-3f * l;
  long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, acc[i], 0, 0, 0);
  }
  long long t1 = clock64();
  float s = 0.f;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[l] = s;
  if (l == 0) *cyc = t1 - t0;
}
__global__ void rate16(float* out, long long* cyc, int iters) {
  const int l = threadIdx.x;
  f4 acc[4];
  for (int i = 0; i < 4; ++i) acc[i] = f4{0.f, 0.f, 0.f, 0.f};
  float a = 1e-3f * l, b = 2e-3f * l;
  long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i], 0, 0, 0);
  }
  long long t1 = clock64();
  float s = 0.f;
  for (int i = 0; i < 4; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[l] = s;
  if (l == 0) *cyc = t1 - t0;
}

int main() {
  float ha[64], hb[64], hd[256];
  for (int l = 0; l < 64; ++l) { ha[l] = 1.0f + l; hb[l] = 1000.0f * (1 + l); }
  float *a, *b, *d; long long* c; float* o;
  hipMalloc(&a, 256); hipMalloc(&b, 256); hipMalloc(&d, 1024); hipMalloc(&c, 8); hipMalloc(&o, 256);
  hipMemcpy(a, ha, 256, hipMemcpyHostToDevice); hipMemcpy(b, hb, 256, hipMemcpyHostToDevice);
  layout<<<1, 64>>>(a, b, d);
  hipMemcpy(hd, d, 1024, hipMemcpyDeviceToHost);
  // hypothesis: lane l supplies A_{l>>2}[l&3], B_{l>>2}[l&3]; lane l holds D_{l>>2}[e][l&3]
  int bad = 0;
  for (int l = 0; l < 64; ++l)
    for (int e = 0; e < 4; ++e) {
      const int blk = l >> 2, j = l & 3;
      const float want = ha[4 * blk + e] * hb[4 * blk + j];
      if (hd[l * 4 + e] != want) { if (bad < 8) printf("lane %d e %d got %g want %g\n", l, e, hd[l * 4 + e], want); ++bad; }
    }
  printf("layout hypothesis: %s (%d mismatches)\n", bad ? "WRONG" : "ok", bad);
  long long cy;
  const int iters = 4096;
  rate<4><<<1, 64>>>(o, c, iters); hipDeviceSynchronize();
  rate<4><<<1, 64>>>(o, c, iters); hipMemcpy(&cy, c, 8, hipMemcpyDeviceToHost);
  printf("4x4x1_16b, 4 accumulators: %.2f cycles per MFMA\n", double(cy) / (iters * 4));
  rate<1><<<1, 64>>>(o, c, iters); hipMemcpy(&cy, c, 8, hipMemcpyDeviceToHost);
  printf("4x4x1_16b, 1 accumulator (dependent): %.2f cycles per MFMA\n", double(cy) / (iters * 1));
  rate<8><<<1, 64>>>(o, c, iters); hipMemcpy(&cy, c, 8, hipMemcpyDeviceToHost);
  printf("4x4x1_16b, 8 accumulators: %.2f cycles per MFMA\n", double(cy) / (iters * 8));
  rate<16><<<1, 64>>>(o, c, iters); hipMemcpy(&cy, c, 8, hipMemcpyDeviceToHost);
  printf("4x4x1_16b, 16 accumulators: %.2f cycles per MFMA\n", double(cy) / (iters * 16));
  rate16<<<1, 64>>>(o, c, iters); hipMemcpy(&cy, c, 8, hipMemcpyDeviceToHost);
  printf("16x16x4 f32, 4 accumulators: %.2f cycles per MFMA\n", double(cy) / (iters * 4));
  return 0;
}
