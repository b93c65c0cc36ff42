// fp64_latency.hip -- dependent-chain latency and throughput of the FP64
// operations the per-ND Welford step uses (k_welford_q), one wave alone on
// its SIMD and several waves per SIMD.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o tools/ubench/fp64_latency tools/ubench/fp64_latency.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#pragma clang fp contract(off)

constexpr int kIters = 4096;

// 8 dependent ops per iteration
template <int KIND>
__global__ void chain(double* out, double a, double b, unsigned long long* cyc) {
  double x = a + threadIdx.x * 1e-9, y = b;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
  for (int i = 0; i < kIters; i++) {
#pragma unroll
    for (int k = 0; k < 8; k++) {
      if constexpr (KIND == 0) x = x + y;              // v_add_f64
      else if constexpr (KIND == 1) x = x * y;         // v_mul_f64
      else if constexpr (KIND == 2) x = fma(x, y, b);  // v_fma_f64
      else x = x + (double)(float)k;                   // add with a constant
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

// N independent chains per wave (throughput)
template <int N>
__global__ void indep(double* out, double a, double b, unsigned long long* cyc) {
  double x[N];
  for (int k = 0; k < N; k++) x[k] = a + threadIdx.x * 1e-9 + k;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
  for (int i = 0; i < kIters; i++) {
#pragma unroll
    for (int r = 0; r < 8; r++)
#pragma unroll
      for (int k = 0; k < N; k++) x[k] = fma(x[k], b, a);
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
  double s = 0;
  for (int k = 0; k < N; k++) s += x[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <typename K>
static void run(const char* name, K kern, int blocks, int threads, int ops_per_iter) {
  double* out;
  unsigned long long* cyc;
  hipMalloc(&out, blocks * threads * sizeof(double));
  hipMalloc(&cyc, blocks * sizeof(unsigned long long));
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, out, 1.0000001, 0.9999999, cyc);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, out, 1.0000001, 0.9999999, cyc);
  hipDeviceSynchronize();
  unsigned long long c;
  hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost);
  printf("%-44s blocks %4d threads %4d: %.2f cycles per op per wave\n", name, blocks, threads,
         (double)c / ((double)kIters * ops_per_iter));
  hipFree(out);
  hipFree(cyc);
}

int main() {
  run("dependent v_add_f64", chain<0>, 1, 64, 8);
  run("dependent v_mul_f64", chain<1>, 1, 64, 8);
  run("dependent v_fma_f64", chain<2>, 1, 64, 8);
  run("dependent v_add_f64 (const)", chain<3>, 1, 64, 8);
  run("dependent v_fma_f64, 4 waves/SIMD (1 WG x 1024)", chain<2>, 1, 1024, 8);
  run("independent v_fma_f64 x2", indep<2>, 1, 64, 16);
  run("independent v_fma_f64 x4", indep<4>, 1, 64, 32);
  run("independent v_fma_f64 x8", indep<8>, 1, 64, 64);
  run("independent v_fma_f64 x8, 4 waves (1 per SIMD)", indep<8>, 1, 256, 64);
  run("independent v_fma_f64 x8, 8 waves (2 per SIMD)", indep<8>, 1, 512, 64);
  return 0;
}
