// Microbenchmarks for the bf16 MFMA ceiling of the split-bf16 ("x6") layers of
// k_pn_chain on this MI355X (16 waves per CU, 256 workgroups):
//   b1 v_mfma_f32_16x16x32_bf16, operands in registers (8 accumulators)
//   b2 v_mfma_f32_32x32x16_bf16, operands in registers (2 accumulators)
//   b3 the x6 inner loop as k_pn_chain runs it: 4 row blocks x 1 column block
//      of 16x16x32, A planes from LDS (12 ds_read_b128 per 24 MFMAs), B planes
//      streamed from an L2-resident buffer (3 KB per wave per k-group, 1 ahead)
//   b4 the same loop on 32x32x16: 2 row blocks x 1 column block of 32, A
//      planes from LDS (6 ds_read_b128 per 12 MFMAs), B 3 KB per k-group
//   hipcc --offload-arch=gfx950 -O3 -o mfma_bf16_peak mfma_bf16_peak.hip && ./mfma_bf16_peak
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
#define CHK(x) do { if ((x) != hipSuccess) { printf("hip error line %d\n", __LINE__); exit(1); } } while (0)

__device__ inline bf16x8 mk(const float* r, int s) {
  bf16x8 v;
  for (int i = 0; i < 8; i++) v[i] = (__bf16)r[(s * 8 + i * 37) & 1023];
  return v;
}

// b1 / b2: register operands
template <int V>
__global__ void __launch_bounds__(1024) k_reg(float* out, const float* __restrict__ rnd, int iters) {
  const int lane = threadIdx.x & 63;
  bf16x8 a[4], b[2];
  for (int i = 0; i < 4; i++) a[i] = mk(rnd, lane * 4 + i);
  for (int j = 0; j < 2; j++) b[j] = mk(rnd, lane * 2 + j + 500);
  float s = 0;
  if (V == 1) {
    f32x4 acc[4][2] = {};
    for (int it = 0; it < iters; it++)
#pragma unroll
      for (int i = 0; i < 4; i++)
#pragma unroll
        for (int j = 0; j < 2; j++) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    for (int i = 0; i < 4; i++)
      for (int j = 0; j < 2; j++) s += acc[i][j][0] + acc[i][j][3];
  } else {
    f32x16 acc[2] = {};
    for (int it = 0; it < iters; it++)
#pragma unroll
      for (int i = 0; i < 4; i++)
#pragma unroll
        for (int j = 0; j < 2; j++) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[j], acc[j], 0, 0, 0);
    for (int j = 0; j < 2; j++) s += acc[j][0] + acc[j][15];
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// b3 / b4: the x6 k-group loop (planes read m, l, h; products mm mh | lh | hl hm hh)
template <int V>
__global__ void __launch_bounds__(1024) k_x6(float* out, const bf16x8* __restrict__ w, const float* __restrict__ rnd,
                                            int iters, int wmask) {
  extern __shared__ bf16x8 lds[];  // 3 planes x 64 rows x 136 bf16 (pitch 128 + 8)
  constexpr int pitch = 136, plane = 64 * pitch;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __bf16* l16 = reinterpret_cast<__bf16*>(lds);
  for (int e = threadIdx.x; e < 3 * plane; e += blockDim.x) l16[e] = (__bf16)rnd[e & 1023];
  __syncthreads();
  const int wbase = (wave * 64 + lane);
  constexpr bool S16 = V != 4;
  constexpr int RB = S16 ? 4 : 2;
  // lane's A offset: 16x16x32 -> row l & 15, k 8 (l >> 4); 32x32x16 -> row l & 31, k 8 (l >> 5)
  const int arow = S16 ? (lane & 15) : (lane & 31), ak = S16 ? 8 * (lane >> 4) : 8 * (lane >> 5);
  const int rstride = (S16 ? 16 : 32) * pitch;
  const int kstep = S16 ? 32 : 16;
  bf16x8 areg[3][RB];
  for (int p = 0; p < 3; p++)
    for (int rb = 0; rb < RB; rb++) areg[p][rb] = mk(rnd, lane + 64 * (p * RB + rb));
  f32x4 acc4[RB] = {};
  f32x16 acc16[RB] = {};
  bf16x8 bq[3];
  int off = 0;
  for (int p = 0; p < 3; p++) bq[p] = w[(wbase + (off * 3 + p) * 1024) & wmask];
  off++;
  for (int it = 0; it < iters; it++) {
    const int kk = (it & 3) * kstep;
    const __bf16* a0 = l16 + arow * pitch + ak + kk;
    bf16x8 bw[3] = {bq[0], bq[1], bq[2]};
    if (V != 6)
      for (int p = 0; p < 3; p++) bq[p] = w[(wbase + (off * 3 + p) * 1024) & wmask];
    off++;
    bf16x8 a[RB];
    bf16x8 a3[3][RB];
    auto ld = [&](int p) {
#pragma unroll
      for (int rb = 0; rb < RB; rb++)
        a[rb] = V == 7 ? areg[p][rb] : V == 5 ? a3[p][rb] : *reinterpret_cast<const bf16x8*>(a0 + p * plane + rb * rstride);
    };
    if (V == 5)
      for (int p = 0; p < 3; p++)
        for (int rb = 0; rb < RB; rb++) a3[p][rb] = *reinterpret_cast<const bf16x8*>(a0 + p * plane + rb * rstride);
    auto mm = [&](int pb) {
#pragma unroll
      for (int rb = 0; rb < RB; rb++) {
        if (S16) acc4[rb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[rb], bw[pb], acc4[rb], 0, 0, 0);
        else acc16[rb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[rb], bw[pb], acc16[rb], 0, 0, 0);
      }
    };
    ld(1); mm(1); mm(0);
    ld(2); mm(0);
    ld(0); mm(2); mm(1); mm(0);
  }
  float s = 0;
  for (int rb = 0; rb < RB; rb++) s += S16 ? acc4[rb][0] + acc4[rb][3] : acc16[rb][0] + acc16[rb][15];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// b8..: fewer waves, more column blocks per wave: WAVES waves per CU (one
// workgroup), RB = 4 row blocks x NB column blocks of 16x16x32 per wave; the
// three A planes of a k-group read up front (APRE) into their own registers,
// the next k-group's B fragments prefetched one step ahead.
template <int WAVES, int NB, bool APRE>
__global__ void __launch_bounds__(WAVES * 64) k_x6w(float* out, const bf16x8* __restrict__ w, const float* __restrict__ rnd,
                                                   int iters, int wmask) {
  extern __shared__ bf16x8 lds[];
  constexpr int pitch = 136, plane = 64 * pitch, RB = 4;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __bf16* l16 = reinterpret_cast<__bf16*>(lds);
  for (int e = threadIdx.x; e < 3 * plane; e += blockDim.x) l16[e] = (__bf16)rnd[e & 1023];
  __syncthreads();
  const int wbase = (wave * 64 + lane);
  const int arow = lane & 15, ak = 8 * (lane >> 4);
  const int rstride = 16 * pitch;
  f32x4 acc[RB][NB] = {};
  bf16x8 bq[NB][3];
  int off = 0;
  auto loadb = [&]() {
#pragma unroll
    for (int j = 0; j < NB; j++)
#pragma unroll
      for (int p = 0; p < 3; p++) bq[j][p] = w[(wbase + ((off * NB + j) * 3 + p) * 1024) & wmask];
    off++;
  };
  loadb();
  for (int it = 0; it < iters; it++) {
    const int kk = (it & 3) * 32;
    const __bf16* a0 = l16 + arow * pitch + ak + kk;
    bf16x8 bw[NB][3];
#pragma unroll
    for (int j = 0; j < NB; j++)
#pragma unroll
      for (int p = 0; p < 3; p++) bw[j][p] = bq[j][p];
    loadb();
    bf16x8 a3[3][RB];
    bf16x8 a[RB];
    if (APRE) {
#pragma unroll
      for (int p = 0; p < 3; p++)
#pragma unroll
        for (int rb = 0; rb < RB; rb++) a3[p][rb] = *reinterpret_cast<const bf16x8*>(a0 + p * plane + rb * rstride);
    }
    auto ld = [&](int p) {
#pragma unroll
      for (int rb = 0; rb < RB; rb++) a[rb] = APRE ? a3[p][rb] : *reinterpret_cast<const bf16x8*>(a0 + p * plane + rb * rstride);
    };
    auto mm = [&](int pb) {
#pragma unroll
      for (int rb = 0; rb < RB; rb++)
#pragma unroll
        for (int j = 0; j < NB; j++) acc[rb][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[j][pb], a[rb], acc[rb][j], 0, 0, 0);
    };
    ld(1); mm(1); mm(0);
    ld(2); mm(0);
    ld(0); mm(2); mm(1); mm(0);
  }
  float s = 0;
  for (int rb = 0; rb < RB; rb++)
    for (int j = 0; j < NB; j++) s += acc[rb][j][0] + acc[rb][j][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  float *out, *rnd;
  bf16x8* w;
  const size_t wbytes = 1 << 20;  // 1 MB of weight fragments (the x6 128 -> 1024 layer holds 768 KB)
  CHK(hipMalloc(&out, 1024 * 1024 * sizeof(float)));
  CHK(hipMalloc(&rnd, 1024 * sizeof(float)));
  CHK(hipMalloc(&w, wbytes));
  float* h = (float*)malloc(wbytes);
  for (size_t i = 0; i < wbytes / 4; i++) h[i] = (float)rand() / RAND_MAX - 0.5f;
  CHK(hipMemcpy(w, h, wbytes, hipMemcpyHostToDevice));
  CHK(hipMemcpy(rnd, h, 1024 * sizeof(float), hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  const int grid = 256, threads = 1024;
  const int wmask = (int)(wbytes / 16 - 1);
  const size_t lds = 3 * 64 * 136 * 2;
  CHK(hipFuncSetAttribute((const void*)k_x6<3>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  CHK(hipFuncSetAttribute((const void*)k_x6<4>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  CHK(hipFuncSetAttribute((const void*)k_x6<5>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  CHK(hipFuncSetAttribute((const void*)k_x6<6>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  CHK(hipFuncSetAttribute((const void*)k_x6<7>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  auto report = [&](const char* name, double flops) {
    CHK(hipEventSynchronize(e1));
    float ms;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    printf("%-58s %.3f ms, %7.1f TFLOP/s bf16\n", name, ms, flops / (ms * 1e-3) / 1e12);
  };
  const int it_reg = 4096, it_x6 = 1024;
  for (int v = 1; v <= 2; v++) {
    auto k = v == 1 ? k_reg<1> : k_reg<2>;
    k<<<grid, threads>>>(out, rnd, 16);
    CHK(hipEventRecord(e0));
    k<<<grid, threads>>>(out, rnd, it_reg);
    CHK(hipEventRecord(e1));
    // b1: 8 MFMAs of 16*16*32*2 per iteration; b2: 8 of 32*32*16*2
    const double per = v == 1 ? 8.0 * 16384 : 8.0 * 32768;
    report(v == 1 ? "b1 16x16x32 bf16, registers" : "b2 32x32x16 bf16, registers",
           (double)grid * 16 * it_reg * per);
  }
  const char* names[] = {"b3 x6 loop 16x16x32, 4x1 tile, A LDS, B L2", "b4 x6 loop 32x32x16, 2x1 tile, A LDS, B L2",
                         "b5 = b3 with the three A planes read up front", "b6 = b3 without the B loads",
                         "b7 = b3 without the A LDS reads"};
  for (int v = 3; v <= 7; v++) {
    auto k = v == 3 ? k_x6<3> : v == 4 ? k_x6<4> : v == 5 ? k_x6<5> : v == 6 ? k_x6<6> : k_x6<7>;
    k<<<grid, threads, lds>>>(out, w, rnd, 16, wmask);
    CHK(hipEventRecord(e0));
    k<<<grid, threads, lds>>>(out, w, rnd, it_x6, wmask);
    CHK(hipEventRecord(e1));
    // per k-group: 6 x RB MFMAs (b3: RB 4 of 16x16x32; b4: RB 2 of 32x32x16)
    const double per = v != 4 ? 24.0 * 16384 : 12.0 * 32768;
    report(names[v - 3], (double)grid * 16 * it_x6 * per);
  }
  // b8..b13: waves per CU x column blocks per wave (the same FLOPs per CU per k-group round
  // when WAVES * NB = 16)
  auto wv = [&](const char* name, auto k, int waves, int nb) {
    CHK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    k<<<grid, waves * 64, lds>>>(out, w, rnd, 16, wmask);
    CHK(hipEventRecord(e0));
    k<<<grid, waves * 64, lds>>>(out, w, rnd, it_x6, wmask);
    CHK(hipEventRecord(e1));
    report(name, (double)grid * waves * it_x6 * 24.0 * nb * 16384);
  };
  wv("b8  16 waves x NB 1, A planes up front", k_x6w<16, 1, true>, 16, 1);
  wv("b9  8 waves x NB 2, A per plane", k_x6w<8, 2, false>, 8, 2);
  wv("b10 8 waves x NB 2, A planes up front", k_x6w<8, 2, true>, 8, 2);
  wv("b11 4 waves x NB 4, A per plane", k_x6w<4, 4, false>, 4, 4);
  wv("b12 4 waves x NB 4, A planes up front", k_x6w<4, 4, true>, 4, 4);
  wv("b13 8 waves x NB 4, A planes up front", k_x6w<8, 4, true>, 8, 4);
  return 0;
}
