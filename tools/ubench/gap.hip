// gap.hip -- idle time between two back-to-back kernels on one stream, by
// kernel shape: the first workgroup start of B minus the last workgroup end of
// A, both from s_memrealtime (100 MHz) stamped inside the kernels.
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench/gap tools/ubench/gap.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <algorithm>
#include <vector>

struct Stamp {
  unsigned long long t0, t1;
};

// A workgroup spins `spin` ticks, touches `lds` bytes of dynamic LDS and
// writes `wr` floats (strided by `stride` floats) of dst, then stamps.
__global__ void k_shape(Stamp* st, float* dst, uint32_t spin, uint32_t wr, uint32_t stride, int use_lds) {
  extern __shared__ float sm[];
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  if (use_lds) sm[threadIdx.x] = (float)threadIdx.x;
  while (__builtin_amdgcn_s_memrealtime() - t0 < spin) {
  }
  const uint64_t base = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (uint32_t i = 0; i < wr; i++) dst[(base + (uint64_t)i * gridDim.x * blockDim.x) * stride % (64ull << 20)] = 1.0f;
  if (use_lds) {
    __syncthreads();
    if (sm[(threadIdx.x + 1) % blockDim.x] < 0) dst[0] = 2.0f;
  }
  __syncthreads();
  if (threadIdx.x == 0) st[blockIdx.x] = Stamp{t0, __builtin_amdgcn_s_memrealtime()};
}

struct Shape {
  const char* name;
  int grid, threads;
  size_t lds;
  uint32_t spin, wr, stride;
};

static void run_pair(const Shape& a, const Shape& b, Stamp* sa, Stamp* sb, float* dst) {
  std::vector<double> gaps, durs;
  for (int rep = 0; rep < 12; rep++) {
    hipLaunchKernelGGL(k_shape, dim3(a.grid), dim3(a.threads), a.lds, 0, sa, dst, a.spin, a.wr, a.stride,
                       a.lds ? 1 : 0);
    hipLaunchKernelGGL(k_shape, dim3(b.grid), dim3(b.threads), b.lds, 0, sb, dst, b.spin, b.wr, b.stride,
                       b.lds ? 1 : 0);
    hipDeviceSynchronize();
    std::vector<Stamp> ha(a.grid), hb(b.grid);
    hipMemcpy(ha.data(), sa, a.grid * sizeof(Stamp), hipMemcpyDeviceToHost);
    hipMemcpy(hb.data(), sb, b.grid * sizeof(Stamp), hipMemcpyDeviceToHost);
    unsigned long long aend = 0, astart = ~0ull, bstart = ~0ull;
    for (auto& s : ha) aend = std::max(aend, s.t1), astart = std::min(astart, s.t0);
    for (auto& s : hb) bstart = std::min(bstart, s.t0);
    if (rep >= 2) {
      gaps.push_back((double)((long long)(bstart - aend)) * 0.01);
      durs.push_back((double)(aend - astart) * 0.01);
    }
  }
  std::sort(gaps.begin(), gaps.end());
  std::sort(durs.begin(), durs.end());
  printf("%-34s -> %-34s  A busy %6.1f us   gap %6.2f us (min %5.2f max %5.2f)\n", a.name, b.name,
         durs[durs.size() / 2], gaps[gaps.size() / 2], gaps.front(), gaps.back());
}

int main() {
  Stamp *sa, *sb;
  float* dst;
  hipMalloc(&sa, 4096 * sizeof(Stamp));
  hipMalloc(&sb, 4096 * sizeof(Stamp));
  hipMalloc(&dst, (64ull << 20) * sizeof(float));
  hipFuncSetAttribute((const void*)k_shape, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  const Shape small{"small 16x256", 16, 256, 0, 500, 0, 1};
  const Shape full{"full 256x1024", 256, 1024, 0, 1000, 0, 1};
  const Shape full_lds{"full 256x1024 lds160K", 256, 1024, 160 * 1024, 1000, 0, 1};
  const Shape full_lds_nospin{"full 256x1024 lds160K short", 256, 1024, 160 * 1024, 100, 0, 1};
  const Shape wide{"wide 2048x256", 2048, 256, 0, 200, 0, 1};
  const Shape writer{"full 256x1024 write 16MB seq", 256, 1024, 0, 100, 16, 1};
  const Shape scatter{"full 256x1024 write 16MB scattered", 256, 1024, 0, 100, 16, 4099};
  const Shape mid{"128x256", 128, 256, 0, 500, 0, 1};
  run_pair(small, small, sa, sb, dst);
  run_pair(small, mid, sa, sb, dst);
  run_pair(small, full, sa, sb, dst);
  run_pair(small, full_lds, sa, sb, dst);
  run_pair(full, small, sa, sb, dst);
  run_pair(full_lds, small, sa, sb, dst);
  run_pair(full_lds_nospin, small, sa, sb, dst);
  run_pair(full_lds, full_lds, sa, sb, dst);
  run_pair(wide, small, sa, sb, dst);
  run_pair(writer, small, sa, sb, dst);
  run_pair(scatter, small, sa, sb, dst);
  run_pair(mid, full_lds, sa, sb, dst);
  run_pair(mid, mid, sa, sb, dst);
  return 0;
}
