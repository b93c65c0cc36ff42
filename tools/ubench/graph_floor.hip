// graph_floor.hip -- cost of one kernel node in a replayed HIP graph, by grid
// shape: a graph of 40 back-to-back kernels that do (almost) nothing, replayed
// 50 times; ms per node = replay time / 40.
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench/graph_floor tools/ubench/graph_floor.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__global__ void k_empty(int* p, int flag) {
  if (flag && threadIdx.x == 0 && blockIdx.x == 0) p[0] = 1;
}

template <int SPIN>
__global__ void k_spin(int* p, int flag) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < SPIN) {
  }
  if (flag && threadIdx.x == 0 && blockIdx.x == 0) p[0] = 1;
}

template <typename K>
static void measure(const char* name, K kern, int grid, int threads, int nodes) {
  int* d;
  hipMalloc(&d, 64);
  hipStream_t s;
  hipStreamCreate(&s);
  hipGraph_t g;
  hipGraphExec_t ge;
  hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
  for (int i = 0; i < nodes; i++) hipLaunchKernelGGL(kern, dim3(grid), dim3(threads), 0, s, d, 0);
  hipStreamEndCapture(s, &g);
  hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  for (int w = 0; w < 5; w++) hipGraphLaunch(ge, s);
  hipStreamSynchronize(s);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int reps = 50;
  hipEventRecord(e0, s);
  for (int r = 0; r < reps; r++) hipGraphLaunch(ge, s);
  hipEventRecord(e1, s);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  // the same kernels launched on the stream directly
  hipEventRecord(e0, s);
  for (int r = 0; r < reps; r++)
    for (int i = 0; i < nodes; i++) hipLaunchKernelGGL(kern, dim3(grid), dim3(threads), 0, s, d, 0);
  hipEventRecord(e1, s);
  hipEventSynchronize(e1);
  float ms2 = 0;
  hipEventElapsedTime(&ms2, e0, e1);
  printf("%-28s grid %5d x %4d: graph %6.2f us/node, stream %6.2f us/kernel\n", name, grid, threads,
         1e3 * ms / (reps * nodes), 1e3 * ms2 / (reps * nodes));
  hipGraphExecDestroy(ge);
  hipGraphDestroy(g);
  hipStreamDestroy(s);
  hipFree(d);
}

int main() {
  measure("empty", k_empty, 1, 64, 40);
  measure("empty", k_empty, 16, 256, 40);
  measure("empty", k_empty, 256, 256, 40);
  measure("empty", k_empty, 256, 1024, 40);
  measure("empty", k_empty, 464, 256, 40);
  measure("empty", k_empty, 2048, 256, 40);
  measure("spin 2us", k_spin<200>, 256, 256, 40);
  measure("spin 2us", k_spin<200>, 16, 256, 40);
  return 0;
}
