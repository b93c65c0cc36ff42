// Launch cost of a k_front-shaped kernel: grid 14 x 16 of 1024 threads with
// 0 / 64 / 129 KB of dynamic LDS and an empty body, back to back on one stream.
//   hipcc --offload-arch=gfx950 -O3 -o launch_cost launch_cost.hip && ./launch_cost
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#define CHK(x) do { if ((x) != hipSuccess) { printf("hip error line %d\n", __LINE__); exit(1); } } while (0)
__global__ void __launch_bounds__(1024) k_empty(int* out) {
  extern __shared__ int s[];
  if (threadIdx.x == 0) s[0] = blockIdx.x;
  __syncthreads();
  if (threadIdx.x == 0 && s[0] < 0) out[blockIdx.x] = s[0];
}
int main() {
  int* out;
  CHK(hipMalloc(&out, 4096 * sizeof(int)));
  CHK(hipFuncSetAttribute((const void*)k_empty, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  for (int kb : {0, 64, 129, 150}) {
    for (int rep = 0; rep < 2; rep++) {
      CHK(hipEventRecord(e0));
      for (int i = 0; i < 200; i++) k_empty<<<dim3(14, 16), 1024, kb * 1024>>>(out);
      CHK(hipEventRecord(e1));
      CHK(hipEventSynchronize(e1));
      float ms;
      CHK(hipEventElapsedTime(&ms, e0, e1));
      if (rep) printf("dynamic LDS %3d KB: %.2f us per launch\n", kb, ms * 1000 / 200);
    }
  }
  return 0;
}
