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
// Tile geometry: 32 points = two 16-row MFMA blocks; the 4 waves are 2 row
// blocks x 2 column halves of a 256-column chunk (8 accumulator blocks of
// 16x16 each).  Weights stream through LDS in 16-row K-slabs of the chunk,
// loaded with 16-byte global loads by all 256 threads, double-buffered: the
// next slab's loads are issued into registers before the current slab's MFMAs
// and written to LDS after them.  Activations live in two LDS regions sized
// for the widest (input, output) pair of the chain, so the 512-wide seg-head
// layer fits beside its 256-wide successor.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>

#include "../../include/ndnet_pointnet.h"

namespace {

constexpr int kP = 32;          // points per workgroup
constexpr int kThreads = 256;   // 4 waves
constexpr int kNC = 256;        // columns per chunk
constexpr int kKS = 16;         // K rows per weight slab
constexpr int kSlabPitch = kNC + 16;  // floats per slab row (breaks the 2-way bank conflict)
constexpr int kSlabFloats = kKS * kSlabPitch;
constexpr int kSlabVecs = kKS * kNC / 4 / kThreads;  // float4 loads per thread per slab (4)

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ inline void atomic_max_f32(float* addr, float v) {
  v = v + 0.0f;  // -0 -> +0 so the integer orderings below agree
  if (v >= 0.0f) atomicMax(reinterpret_cast<int*>(addr), __float_as_int(v));
  else atomicMin(reinterpret_cast<unsigned int*>(addr), __float_as_uint(v));
}

// Loads this thread's share of slab rows [ks, ks + kr) x columns [c0, c0 + nc)
// of W^T (row stride ldw) into registers.  Branch-free: out-of-range elements
// load a valid address and are zeroed by a select, so no vmcnt wait is forced
// into the middle of the MFMA loop.
__device__ inline unsigned slab_load(f32x4 (&r)[kSlabVecs], const float* __restrict__ wT, int ldw, int ks, int kr,
                                     int c0, int nc) {
  const int vpr = nc / 4;  // float4 per slab row
  unsigned ok_mask = 0;
#pragma unroll
  for (int v = 0; v < kSlabVecs; v++) {
    const int e = threadIdx.x + kThreads * v;
    const int row = e / (kNC / 4), col4 = e % (kNC / 4);
    const bool ok = row < kr && col4 < vpr;
    ok_mask |= (unsigned)ok << v;
    r[v] = *reinterpret_cast<const f32x4*>(wT + (int64_t)(ks + (ok ? row : 0)) * ldw + c0 + (ok ? 4 * col4 : 0));
  }
  return ok_mask;
}

// Writes the staged slab to LDS; the zeroing of out-of-range elements happens
// here, not at load time, so the loads stay in flight across the MFMAs.
__device__ inline void slab_store(const f32x4 (&r)[kSlabVecs], unsigned ok_mask, float* slab) {
#pragma unroll
  for (int v = 0; v < kSlabVecs; v++) {
    const int e = threadIdx.x + kThreads * v;
    const int row = e / (kNC / 4), col4 = e % (kNC / 4);
    *reinterpret_cast<f32x4*>(slab + row * kSlabPitch + 4 * col4) =
        ((ok_mask >> v) & 1) ? r[v] : f32x4{0.f, 0.f, 0.f, 0.f};
  }
}

// dynamic LDS of k_pn_chain; regions are addressed by float offsets into it so
// every activation/slab access compiles to ds_* (a generic pointer would give
// flat_* ops, which count against vmcnt and stall on the weight prefetch)
extern __shared__ __attribute__((aligned(16))) float g_smem[];

struct ChunkCtx {
  const float* __restrict__ wT;
  const float* __restrict__ bias;
  int in, outb, slabs;  // float offsets into g_smem
  float* gmax;  // this cloud's max-pool row (mode 0, last layer) or null
  int ldw, K, pin, pout, relu, c0, nc, rows_valid;
};

// One 256-column chunk of one layer: this wave's NB accumulator blocks
// (16 rows x 16 NB columns) over all K, then the epilogue.  NB is a template
// parameter so the MFMA sequence is straight-line code.
template <int NB>
__device__ __attribute__((always_inline)) void run_chunk(const ChunkCtx& C) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int kq = lane >> 4, cl = lane & 15;
  const int cw = wc * (C.nc / 2);
  const int nslab = (C.K + kKS - 1) / kKS;
  f32x4 acc[NB];
#pragma unroll
  for (int j = 0; j < NB; j++) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 stage[kSlabVecs];
  float* const slabs = g_smem + C.slabs;
  unsigned ok = slab_load(stage, C.wT, C.ldw, 0, C.K < kKS ? C.K : kKS, C.c0, C.nc);
  slab_store(stage, ok, slabs);
  __syncthreads();
  const float* arow = g_smem + C.in + (16 * wr + cl) * C.pin + kq;
  for (int s = 0; s < nslab; s++) {
    const float* slab = slabs + (s & 1) * kSlabFloats;
    const int ks = s * kKS;
    const bool more = s + 1 < nslab;
    if (more) ok = slab_load(stage, C.wT, C.ldw, ks + kKS, C.K - ks - kKS < kKS ? C.K - ks - kKS : kKS, C.c0, C.nc);
    // rows of the slab past K are zero and the activations past K are finite
    // (zero-filled input columns), so all four k-steps run unconditionally.
    // Fragments are software-pipelined one k-step ahead of the MFMAs.
    const float* bbase = slab + kq * kSlabPitch + cw + cl;
    float a = arow[ks];
    float bv[NB];
#pragma unroll
    for (int j = 0; j < NB; j++) bv[j] = bbase[16 * j];
#pragma unroll
    for (int kk = 0; kk < kKS; kk += 4) {
      float an = 0.f, bn[NB];
      if (kk + 4 < kKS) {
        an = arow[ks + kk + 4];
#pragma unroll
        for (int j = 0; j < NB; j++) bn[j] = bbase[(kk + 4) * kSlabPitch + 16 * j];
      }
#pragma unroll
      for (int j = 0; j < NB; j++) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bv[j], acc[j], 0, 0, 0);
      if (kk + 4 < kKS) {
        a = an;
#pragma unroll
        for (int j = 0; j < NB; j++) bv[j] = bn[j];
      }
      // keep the next step's fragment reads interleaved with this step's MFMAs
#pragma unroll
      for (int j = 0; j < NB; j++) {
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
      }
    }
    if (more) slab_store(stage, ok, slabs + ((s + 1) & 1) * kSlabFloats);
    __syncthreads();
  }
  // epilogue: C[row = 16 wr + 4 kq + r][col = c0 + cw + 16 j + cl]
#pragma unroll
  for (int j = 0; j < NB; j++) {
    const int ch = C.c0 + cw + 16 * j + cl;
    const float bv = C.bias[ch];
    if (C.gmax) {
      float m = -INFINITY;
#pragma unroll
      for (int r = 0; r < 4; r++) {
        float v = acc[j][r] + bv;
        if (C.relu) v = fmaxf(v, 0.0f);
        if (16 * wr + 4 * kq + r < C.rows_valid) m = fmaxf(m, v);
      }
      m = fmaxf(m, __shfl_xor(m, 16, 64));
      m = fmaxf(m, __shfl_xor(m, 32, 64));
      if (lane < 16) atomic_max_f32(C.gmax + ch, m);
    } else {
#pragma unroll
      for (int r = 0; r < 4; r++) {
        float v = acc[j][r] + bv;
        if (C.relu) v = fmaxf(v, 0.0f);
        g_smem[C.outb + (16 * wr + 4 * kq + r) * C.pout + ch] = v;
      }
    }
  }
}

__global__ void __launch_bounds__(kThreads) k_pn_chain(ndnet_pn_chain A) {
  float* const smem = g_smem;
  const int b = blockIdx.y;
  const int p0 = blockIdx.x * kP;
  // LDS: activation region 0 | region 1 | two weight slabs
  const int pitch0 = A.max_width + 1, pitch1 = A.max_width2 + 1;
  const int act[2] = {0, kP * pitch0};
  float* const act0 = smem;
  // input tile, zero-filled to a whole slab of columns
  const int K0 = (A.L[0].K + kKS - 1) / kKS * kKS;
  for (int e = threadIdx.x; e < kP * K0; e += kThreads) {
    const int r = e / K0, c = e % K0;
    const int p = p0 + r;
    float v = 0.0f;
    if (p < A.num_points && c < A.in_cols) v = A.x[((int64_t)b * A.num_points + p) * A.x_ld + c];
    act0[r * pitch0 + c] = v;
  }
  __syncthreads();
  const int rows_valid = A.num_points - p0;
  for (int l = 0; l < A.num_layers; l++) {
    const ndnet_pn_layer L = A.L[l];
    const bool last = (l == A.num_layers - 1);
    ChunkCtx C;
    C.wT = L.wT + (int64_t)b * L.w_cloud_stride;
    C.bias = L.bias + (int64_t)b * L.bias_cloud_stride;
    C.in = act[l & 1];
    C.pin = (l & 1) ? pitch1 : pitch0;
    C.outb = act[(l + 1) & 1];
    C.pout = ((l + 1) & 1) ? pitch1 : pitch0;
    C.slabs = kP * (pitch0 + pitch1);
    C.gmax = (last && A.mode == 0) ? A.gmax + (int64_t)b * A.gmax_ld : nullptr;
    C.ldw = L.ldw;
    C.K = L.K;
    C.relu = L.relu;
    C.rows_valid = rows_valid;
    for (int c0 = 0; c0 < L.N; c0 += kNC) {
      C.c0 = c0;
      C.nc = L.N - c0 < kNC ? L.N - c0 : kNC;
      switch (C.nc / 32) {  // accumulator blocks per wave
        case 8: run_chunk<8>(C); break;
        case 7: run_chunk<7>(C); break;
        case 6: run_chunk<6>(C); break;
        case 5: run_chunk<5>(C); break;
        case 4: run_chunk<4>(C); break;
        case 3: run_chunk<3>(C); break;
        case 2: run_chunk<2>(C); break;
        default: run_chunk<1>(C); break;
      }
    }
    __syncthreads();
  }
  if (A.mode == 1) {  // log_softmax over channels (ndtnet.py:239), [B][N][C+1] layout
    const float* lg = smem + act[A.num_layers & 1];
    const int pl = (A.num_layers & 1) ? pitch1 : pitch0;
    for (int r = threadIdx.x; r < kP; r += kThreads) {
      const int p = p0 + r;
      if (p >= A.num_points) continue;
      float m = -INFINITY;
      for (int c = 0; c < A.out_cols; c++) m = fmaxf(m, lg[r * pl + c]);
      float s = 0.0f;
      for (int c = 0; c < A.out_cols; c++) s += expf(lg[r * pl + c] - m);
      const float ls = logf(s);
      float* o = A.out + ((int64_t)b * A.num_points + p) * A.out_cols;
      for (int c = 0; c < A.out_cols; c++) o[c] = (lg[r * pl + c] - m) - ls;
    }
  }
}

}  // namespace

extern "C" {

// One fused point-MLP chain over `batch` clouds on `stream` (see pointnet.h).
int ndnet_pn_chain_run(const ndnet_pn_chain* args, int batch, void* stream) {
  if (!args || batch <= 0 || args->num_layers < 1 || args->num_layers > NDNET_PN_MAX_LAYERS) return -20;
  // activation regions: layer l reads region l & 1 and writes region (l + 1) & 1
  int w[2] = {args->L[0].K, 0};
  for (int l = 0; l < args->num_layers; l++) {
    const ndnet_pn_layer& L = args->L[l];
    if (L.K % 4 || L.N % 32 || L.ldw % 4 || L.ldw < L.N) return -20;
    if (l > 0 && L.K > w[l & 1]) return -20;
    const bool stored = l + 1 < args->num_layers || args->mode == 1;
    if (stored && L.N > w[(l + 1) & 1]) w[(l + 1) & 1] = L.N;
  }
  // the input tile is zero-filled to a whole K-slab of columns
  const int k0 = (args->L[0].K + kKS - 1) / kKS * kKS;
  if (k0 > w[0]) w[0] = k0;
  if (args->max_width < w[0] || args->max_width2 < w[1]) return -20;
  const size_t lds = sizeof(float) * ((size_t)kP * (args->max_width + 1 + args->max_width2 + 1) + 2 * kSlabFloats);
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
