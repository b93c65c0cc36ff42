// write_width.hip -- what WRITE_SIZE (and the time) reports for the store
// patterns of k_front's scatter, against a known byte count.
//
// 16 "clouds" x 100000 f32 xyz points (19.2 MB written per launch), each
// point sent to its ND's run exactly as k_front does it (1000 NDs per cloud,
// a stable counting sort by ND in index order; 16 workgroups of 1024 threads
// per cloud, each owning a contiguous 1/16 of the points):
//   stream16   every lane stores a float4, consecutive lanes consecutive (the
//              guide's calibrated pattern: WRITE_SIZE = bytes)
//   stream4    every lane stores one dword, consecutive
//   scatter12  k_front's store: a lane's point, 3 dword stores to dst * 3
//   staged     the same destinations, but each workgroup stores its points in
//              destination order (lane q: dword q of the workgroup's sorted
//              output), so a wave's store covers whole runs of its segments
// scatter12 / staged also run with XCD-local placement (_x): the 16
// workgroups of a cloud share blockIdx % 8, so they share one L2, as k_front
// places them.
// Run under rocprofv3 --pmc WRITE_SIZE --kernel-trace (one pass per counter).
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench/write_width tools/ubench/write_width.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

constexpr int kClouds = 16, kN = 100000, kNds = 1000, kG = 16, kT = 1024;

#define CK(x)                                                         \
  do {                                                                \
    hipError_t e_ = (x);                                              \
    if (e_ != hipSuccess) {                                           \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                        \
    }                                                                 \
  } while (0)

// workgroup w of a launch handles cloud w / kG, slice w % kG (grid = kClouds * kG);
// XCD-local: w % 8 is the XCD, the 32 slots of an XCD hold two clouds
template <bool XCD>
__device__ inline void slice(int& c, uint32_t& i0, uint32_t& i1) {
  int g;
  if (XCD) {
    const int x = blockIdx.x % 8, s = blockIdx.x / 8;
    c = x + 8 * (s / kG);
    g = s % kG;
  } else {
    c = blockIdx.x / kG;
    g = blockIdx.x % kG;
  }
  i0 = (uint32_t)((uint64_t)kN * g / kG);
  i1 = (uint32_t)((uint64_t)kN * (g + 1) / kG);
}

__global__ void k_stream16(const float4* __restrict__ in, float4* __restrict__ out, uint64_t n4) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (uint64_t)gridDim.x * blockDim.x)
    out[i] = in[i];
}

__global__ void k_stream4(const float* __restrict__ in, float* __restrict__ out, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    out[i] = in[i];
}

template <bool XCD>
__global__ void __launch_bounds__(kT) k_scatter12(const float* __restrict__ in, const uint32_t* __restrict__ dst,
                                                  float* __restrict__ out) {
  int c;
  uint32_t i0, i1;
  slice<XCD>(c, i0, i1);
  const float* p = in + (uint64_t)c * kN * 3;
  float* o = out + (uint64_t)c * kN * 3;
  for (uint32_t i = i0 + threadIdx.x; i < i1; i += kT) {
    const float x = p[3 * i], y = p[3 * i + 1], z = p[3 * i + 2];
    const uint32_t d = dst[(uint64_t)c * kN + i];
    o[3 * d] = x;
    o[3 * d + 1] = y;
    o[3 * d + 2] = z;
  }
}

// order[c][i0..i1): the slice's points sorted by destination (host-built)
template <bool XCD>
__global__ void __launch_bounds__(kT) k_staged(const float* __restrict__ in, const uint32_t* __restrict__ dst,
                                               const uint32_t* __restrict__ order, float* __restrict__ out) {
  int c;
  uint32_t i0, i1;
  slice<XCD>(c, i0, i1);
  const float* p = in + (uint64_t)c * kN * 3;
  float* o = out + (uint64_t)c * kN * 3;
  const uint32_t* ord = order + (uint64_t)c * kN;
  const uint32_t nq = (i1 - i0) * 3;
  for (uint32_t q = threadIdx.x; q < nq; q += kT) {
    const uint32_t src = ord[i0 + q / 3], e = q % 3;
    const uint32_t d = dst[(uint64_t)c * kN + src];
    o[3 * d + e] = p[3 * src + e];
  }
}

int main() {
  const uint64_t npts = (uint64_t)kClouds * kN, nflt = npts * 3;
  std::vector<float> h(nflt);
  for (uint64_t i = 0; i < nflt; i++) h[i] = (float)(i % 977) * 0.5f;
  // k_front's destinations: stable counting sort by a random ND per point
  std::vector<uint32_t> dst(npts), order(npts);
  srand(7);
  for (int c = 0; c < kClouds; c++) {
    std::vector<uint32_t> nd(kN), cnt(kNds + 1, 0);
    for (int i = 0; i < kN; i++) {
      nd[i] = (uint32_t)(rand() % kNds);
      cnt[nd[i] + 1]++;
    }
    for (int d = 0; d < kNds; d++) cnt[d + 1] += cnt[d];
    for (int i = 0; i < kN; i++) dst[(uint64_t)c * kN + i] = cnt[nd[i]]++;
    for (int g = 0; g < kG; g++) {
      const int i0 = (int)((uint64_t)kN * g / kG), i1 = (int)((uint64_t)kN * (g + 1) / kG);
      uint32_t* o = order.data() + (uint64_t)c * kN;
      for (int i = i0; i < i1; i++) o[i] = i;
      std::sort(o + i0, o + i1, [&](uint32_t a, uint32_t b) { return dst[(uint64_t)c * kN + a] < dst[(uint64_t)c * kN + b]; });
    }
  }
  float *din, *dout;
  uint32_t *ddst, *dord;
  CK(hipMalloc(&din, nflt * 4));
  CK(hipMalloc(&dout, nflt * 4));
  CK(hipMalloc(&ddst, npts * 4));
  CK(hipMalloc(&dord, npts * 4));
  CK(hipMemcpy(din, h.data(), nflt * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(ddst, dst.data(), npts * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dord, order.data(), npts * 4, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int reps = 20;
  auto timeit = [&](const char* name, auto launch) {
    launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; r++) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("%-10s %8.2f us/launch  %.1f MB written -> %.0f GB/s\n", name, 1e3 * ms / reps, nflt * 4 / 1e6,
           nflt * 4 / (ms / reps * 1e-3) / 1e9);
  };
  timeit("stream16", [&] { k_stream16<<<2048, 256>>>((const float4*)din, (float4*)dout, nflt / 4); });
  timeit("stream4", [&] { k_stream4<<<2048, 256>>>(din, dout, nflt); });
  timeit("scatter12", [&] { k_scatter12<false><<<kClouds * kG, kT>>>(din, ddst, dout); });
  timeit("staged", [&] { k_staged<false><<<kClouds * kG, kT>>>(din, ddst, dord, dout); });
  timeit("scatter12_x", [&] { k_scatter12<true><<<kClouds * kG, kT>>>(din, ddst, dout); });
  timeit("staged_x", [&] { k_staged<true><<<kClouds * kG, kT>>>(din, ddst, dord, dout); });
  // check: staged and scatter12 produce the same output
  std::vector<float> a(nflt), b(nflt);
  k_scatter12<true><<<kClouds * kG, kT>>>(din, ddst, dout);
  CK(hipMemcpy(a.data(), dout, nflt * 4, hipMemcpyDeviceToHost));
  CK(hipMemset(dout, 0, nflt * 4));
  k_staged<false><<<kClouds * kG, kT>>>(din, ddst, dord, dout);
  CK(hipMemcpy(b.data(), dout, nflt * 4, hipMemcpyDeviceToHost));
  printf("staged == scatter12: %s\n", a == b ? "yes" : "NO");
  return 0;
}
