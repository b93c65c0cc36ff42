// pointnet_kernels.hip -- NDTNetSegmentation forward (eval) on gfx950.
//
// The reference runs NDTNet as a chain of torch Conv1d(k=1)/BatchNorm1d/ReLU
// ops (ndnet/models/ndtnet.py:45-60, 148-161, 233-241), each a GEMM over
// (points x channels) whose activations round-trip through HBM -- e.g. the
// TNet conv3 output is [B*N x 1024] fp32, 65 MB per batch, written and read
// back only to be max-pooled.  Here one workgroup carries a tile of 32 points
// through a whole per-point MLP chain: activations stay in LDS, each layer is
// an FP32 MFMA GEMM (v_mfma_f32_16x16x4_f32: exact fp32 products and sums, as
// torch's fp32 GEMM), BatchNorm is folded into the weights, and the chain
// ends either in a max-pool over points (fused into the last GEMM's
// epilogue, one float atomic max per channel per tile) or in log-softmax.
//
// Tile geometry: 32 points (two 16-row MFMA blocks) x all output channels;
// 4 waves split the 16-column blocks of each layer, 8 blocks at a time
// (2 x 8 accumulators of 4 floats); the weight fragments for k-step s+1 are
// loaded while the MFMAs of k-step s issue.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>

#include "pointnet.h"

namespace {

constexpr int kP = 32;        // points per workgroup
constexpr int kThreads = 256; // 4 waves
constexpr int kCBG = 8;       // 16-column blocks per wave per pass

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ inline void atomic_max_f32(float* addr, float v) {
  v = v + 0.0f;  // -0 -> +0 so the integer orderings below agree
  if (v >= 0.0f) atomicMax(reinterpret_cast<int*>(addr), __float_as_int(v));
  else atomicMin(reinterpret_cast<unsigned int*>(addr), __float_as_uint(v));
}

__global__ void __launch_bounds__(kThreads) k_pn_chain(ndnet_pn_chain A) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int b = blockIdx.y;
  const int p0 = blockIdx.x * kP;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int pitch = A.max_width + 1;  // odd: a column read by 16 lanes hits 16 banks
  float* bufs[2] = {smem, smem + kP * pitch};
  const int K0 = A.L[0].K;
  for (int e = threadIdx.x; e < kP * K0; e += kThreads) {
    const int r = e / K0, c = e % K0;
    const int p = p0 + r;
    float v = 0.0f;
    if (p < A.num_points && c < A.in_cols) v = A.x[((int64_t)b * A.num_points + p) * A.x_ld + c];
    bufs[0][r * pitch + c] = v;
  }
  __syncthreads();
  const int kr = lane >> 4;   // k row of the A/B fragments
  const int cl = lane & 15;   // row (A) / column (B, C) of the fragments
  int cur = 0;
  for (int l = 0; l < A.num_layers; l++) {
    const ndnet_pn_layer L = A.L[l];
    const float* __restrict__ wT = L.wT + (int64_t)b * L.w_cloud_stride;
    const float* __restrict__ bias = L.bias + (int64_t)b * L.bias_cloud_stride;
    const int K = L.K, N = L.N, ncb = N / 16;
    const bool last = (l == A.num_layers - 1);
    const float* in = bufs[cur];
    float* outb = bufs[cur ^ 1];
    for (int g0 = wave; g0 < ncb; g0 += 4 * kCBG) {
      f32x4 acc[2][kCBG];
#pragma unroll
      for (int j = 0; j < kCBG; j++) {
        acc[0][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        acc[1][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
      float bw[kCBG], bn[kCBG];
#pragma unroll
      for (int j = 0; j < kCBG; j++) {
        const int cb = g0 + 4 * j;
        bw[j] = cb < ncb ? wT[(int64_t)kr * N + cb * 16 + cl] : 0.0f;
      }
      for (int k = 0; k < K; k += 4) {
        const float a0 = in[cl * pitch + k + kr];
        const float a1 = in[(16 + cl) * pitch + k + kr];
        const bool more = k + 4 < K;
#pragma unroll
        for (int j = 0; j < kCBG; j++) {
          const int cb = g0 + 4 * j;
          bn[j] = (more && cb < ncb) ? wT[(int64_t)(k + 4 + kr) * N + cb * 16 + cl] : 0.0f;
        }
#pragma unroll
        for (int j = 0; j < kCBG; j++) {
          if (g0 + 4 * j < ncb) {
            acc[0][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, bw[j], acc[0][j], 0, 0, 0);
            acc[1][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, bw[j], acc[1][j], 0, 0, 0);
          }
        }
#pragma unroll
        for (int j = 0; j < kCBG; j++) bw[j] = bn[j];
      }
      // epilogue: C[row = 16 rb + 4 (lane >> 4) + r][col = lane & 15]
#pragma unroll
      for (int j = 0; j < kCBG; j++) {
        const int cb = g0 + 4 * j;
        if (cb >= ncb) continue;
        const int ch = cb * 16 + cl;
        const float bv = bias[ch];
        if (last && A.mode == 0) {
          float m = -INFINITY;
#pragma unroll
          for (int rb = 0; rb < 2; rb++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
              float v = acc[rb][j][r] + bv;
              if (L.relu) v = fmaxf(v, 0.0f);
              const int row = 16 * rb + 4 * kr + r;
              if (p0 + row < A.num_points) m = fmaxf(m, v);
            }
          m = fmaxf(m, __shfl_xor(m, 16, 64));
          m = fmaxf(m, __shfl_xor(m, 32, 64));
          if (lane < 16) atomic_max_f32(A.gmax + (int64_t)b * A.gmax_ld + ch, m);
        } else {
#pragma unroll
          for (int rb = 0; rb < 2; rb++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
              float v = acc[rb][j][r] + bv;
              if (L.relu) v = fmaxf(v, 0.0f);
              outb[(16 * rb + 4 * kr + r) * pitch + ch] = v;
            }
        }
      }
    }
    __syncthreads();
    cur ^= 1;
  }
  if (A.mode == 1) {  // log_softmax over channels (ndtnet.py:239), [B][N][C+1] layout
    const float* lg = bufs[cur];
    for (int r = threadIdx.x; r < kP; r += kThreads) {
      const int p = p0 + r;
      if (p >= A.num_points) continue;
      float m = -INFINITY;
      for (int c = 0; c < A.out_cols; c++) m = fmaxf(m, lg[r * pitch + c]);
      float s = 0.0f;
      for (int c = 0; c < A.out_cols; c++) s += expf(lg[r * pitch + c] - m);
      const float ls = logf(s);
      float* o = A.out + ((int64_t)b * A.num_points + p) * A.out_cols;
      for (int c = 0; c < A.out_cols; c++) o[c] = (lg[r * pitch + c] - m) - ls;
    }
  }
}

}  // namespace

extern "C" {

// One fused point-MLP chain over `batch` clouds on `stream` (see pointnet.h).
int ndnet_pn_chain_run(const ndnet_pn_chain* args, int batch, void* stream) {
  if (!args || batch <= 0 || args->num_layers < 1 || args->num_layers > NDNET_PN_MAX_LAYERS) return -20;
  if (args->L[0].K > args->max_width) return -20;
  for (int l = 0; l < args->num_layers; l++) {
    const bool stored = l + 1 < args->num_layers || args->mode == 1;
    if (args->L[l].K % 4 || args->L[l].N % 16) return -20;
    if (stored && args->L[l].N > args->max_width) return -20;
  }
  const size_t lds = (size_t)2 * kP * (args->max_width + 1) * sizeof(float);
  static bool attr_set = false;
  if (!attr_set) {
    if (hipFuncSetAttribute((const void*)k_pn_chain, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) !=
        hipSuccess)
      return -21;
    attr_set = true;
  }
  if (lds > 160 * 1024) return -20;
  dim3 grid((args->num_points + kP - 1) / kP, batch);
  k_pn_chain<<<grid, kThreads, lds, (hipStream_t)stream>>>(*args);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    fprintf(stderr, "ndnet_amd: k_pn_chain launch failed: %s\n", hipGetErrorString(e));
    return -21;
  }
  return 0;
}

}  // extern "C"
