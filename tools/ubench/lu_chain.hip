// lu_chain.hip -- cycles per step of the in-place LU chain (lu3 + the event
// flags, csrc/ndt_device.h) on one wave, one ND per lane, as k_welford_q's
// group hand-off runs it (wq_lu_group).
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o tools/ubench/lu_chain tools/ubench/lu_chain.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "../../ndt-net_amd/csrc/ndt_device.h"

#pragma clang fp contract(off)
using namespace ndnet;

template <int FLAGS>
__global__ void chain(const double* __restrict__ cov, double* out, unsigned long long* cyc, int steps) {
  const int u = threadIdx.x;
  double S[9];
  for (int q = 0; q < 9; q++) S[q] = cov[9 * u + q];
  uint32_t okb = 0, acc = 0;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int t = 0; t < steps; t++) {
    uint32_t perm;
    int sg;
    lu3(S, perm, sg);
    if (FLAGS) okb |= (lu3_det(S, sg) != 0 && lu3_sgndet(S, sg) != 0 ? 1u : 0u) << (t & 31);
    acc += perm + (uint32_t)sg;
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (u == 0) cyc[0] = t1 - t0;
  double s = 0;
  for (int q = 0; q < 9; q++) s += S[q];
  out[u] = s + okb + acc;
}

int main() {
  double h[64 * 9];
  unsigned seed = 1;
  for (int i = 0; i < 64 * 9; i++) {
    seed = seed * 1103515245u + 12345u;
    h[i] = ((seed >> 8) & 0xffff) / 65536.0 - 0.5;
  }
  double *cov, *out;
  unsigned long long* cyc;
  hipMalloc(&cov, sizeof h);
  hipMalloc(&out, 64 * sizeof(double));
  hipMalloc(&cyc, sizeof(unsigned long long));
  hipMemcpy(cov, h, sizeof h, hipMemcpyHostToDevice);
  for (int f = 0; f < 2; f++) {
    for (int r = 0; r < 2; r++) {
      if (f) hipLaunchKernelGGL(chain<1>, dim3(1), dim3(64), 0, 0, cov, out, cyc, 12);
      else hipLaunchKernelGGL(chain<0>, dim3(1), dim3(64), 0, 0, cov, out, cyc, 12);
    }
    hipDeviceSynchronize();
    unsigned long long c;
    hipMemcpy(&c, cyc, sizeof c, hipMemcpyDeviceToHost);
    printf("lu3 chain%s: %.1f cycles per step (one wave, 12 steps)\n", f ? " + det/sgndet flags" : "", c / 12.0);
  }
  return 0;
}
