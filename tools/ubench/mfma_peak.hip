// Microbenchmarks for the fp32 MFMA ceiling of k_pn_chain on this MI355X:
//   v1 constant operands in registers (8 independent accumulators per wave)
//   v2 random operands in registers
//   v3 v2 + B fragments streamed from an L2-resident buffer (1 KB per wave per
//      4 MFMA steps, 4 k-groups in flight) -- the chain kernel's weight path
//   v4 v3 + A fragments from LDS (ds_read_b128), the chain kernel's inner loop
//   hipcc --offload-arch=gfx950 -O3 -o mfma_peak mfma_peak.hip && ./mfma_peak
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
typedef float f32x4 __attribute__((ext_vector_type(4)));
#define CHK(x) do { if ((x) != hipSuccess) { printf("hip error line %d\n", __LINE__); exit(1); } } while (0)

template <int V>
__global__ void __launch_bounds__(1024) k_mfma(float* out, const f32x4* __restrict__ w, const float* __restrict__ rnd,
                                               int iters, int wmask) {
  __shared__ f32x4 lds[64 * 16];
  const int lane = threadIdx.x & 63;
  f32x4 acc[4][2];
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 2; j++) acc[i][j] = f32x4{0, 0, 0, 0};
  f32x4 a[4], b[2];
  for (int i = 0; i < 4; i++) a[i] = f32x4{rnd[(lane * 7 + i * 13) & 1023], rnd[(lane * 5 + i) & 1023], rnd[(lane + i * 3) & 1023], rnd[(lane * 3 + 9 * i) & 1023]};
  for (int j = 0; j < 2; j++) b[j] = f32x4{rnd[(lane * 11 + j) & 1023], rnd[(lane * 2 + j * 5) & 1023], rnd[(lane * 13 + j) & 1023], rnd[(lane + 17 * j) & 1023]};
  if (V == 1) {
    for (int i = 0; i < 4; i++) a[i] = f32x4{1, 1, 1, 1};
    for (int j = 0; j < 2; j++) b[j] = f32x4{1, 1, 1, 1};
  }
  for (int e = threadIdx.x; e < 64 * 16; e += blockDim.x) lds[e] = f32x4{rnd[e & 1023], rnd[(e * 3) & 1023], rnd[(e * 7) & 1023], rnd[(e * 5) & 1023]};
  __syncthreads();
  const int wave = threadIdx.x >> 6;
  const int wbase = (blockIdx.x * 16 + wave) * 64 + lane;  // every index below is masked into w
  f32x4 bq[4][2];
  if (V >= 3)
    for (int d = 0; d < 4; d++)
      for (int j = 0; j < 2; j++) bq[d][j] = w[(wbase + (d * 2 + j) * 1024) & wmask];
  int off = 8;
  for (int it = 0; it < iters; it += 4) {
#pragma unroll
    for (int d = 0; d < 4; d++) {
      f32x4 bb[2] = {b[0], b[1]};
      if (V >= 3) { bb[0] = bq[d][0]; bb[1] = bq[d][1]; }
      f32x4 aa[4] = {a[0], a[1], a[2], a[3]};
      if (V >= 4)
        for (int i = 0; i < 4; i++) aa[i] = lds[(i * 16 + (lane & 15)) * 4 + (lane >> 4) + d * 0];
#pragma unroll
      for (int s = 0; s < 4; s++)
#pragma unroll
        for (int i = 0; i < 4; i++)
#pragma unroll
          for (int j = 0; j < 2; j++) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(aa[i][s], bb[j][s], acc[i][j], 0, 0, 0);
      if (V >= 3) {
        for (int j = 0; j < 2; j++) bq[d][j] = w[(wbase + (off + j) * 1024) & wmask];
        off += 2;
      }
    }
  }
  float s = 0;
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 2; j++) s += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  float *out, *rnd;
  f32x4* w;
  const size_t wfloats = 1 << 20;  // 4 MB weight buffer (L2 / MALL resident)
  CHK(hipMalloc(&out, 1024 * 1024 * sizeof(float)));
  CHK(hipMalloc(&rnd, 1024 * sizeof(float)));
  CHK(hipMalloc(&w, wfloats * sizeof(float)));
  float* h = (float*)malloc(wfloats * sizeof(float));
  for (size_t i = 0; i < wfloats; i++) h[i] = (float)rand() / RAND_MAX - 0.5f;
  CHK(hipMemcpy(w, h, wfloats * sizeof(float), hipMemcpyHostToDevice));
  CHK(hipMemcpy(rnd, h, 1024 * sizeof(float), hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  const int iters = 2048, grid = 256, threads = 1024;
  const int wmask = (int)(wfloats / 4 - 1);
  auto run = [&](auto kern, const char* name) {
    kern<<<grid, threads>>>(out, w, rnd, 16, wmask);
    CHK(hipEventRecord(e0));
    kern<<<grid, threads>>>(out, w, rnd, iters, wmask);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    float ms;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    const double flops = (double)grid * (threads / 64) * iters * 4 * 8 * 2048.0;
    printf("%-44s grid %d x %d: %.3f ms, %.1f TFLOP/s\n", name, grid, threads, ms, flops / (ms * 1e-3) / 1e12);
  };
  run(k_mfma<1>, "v1 constant operands");
  run(k_mfma<2>, "v2 random operands (registers)");
  run(k_mfma<3>, "v3 + B streamed from L2 (4 in flight)");
  run(k_mfma<4>, "v4 + A from LDS (ds_read_b128)");
  return 0;
}
