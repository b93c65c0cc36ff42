// pointnet_kernels.hip -- NDTNetSegmentation forward (eval) on gfx950.
//
// The reference runs NDTNet as a chain of torch Conv1d(k=1)/BatchNorm1d/ReLU
// ops (ndnet/models/ndtnet.py:45-60, 148-161, 233-241), each a GEMM over
// (points x channels) whose activations round-trip through HBM -- e.g. the
// TNet conv3 output is [B*N x 1024] fp32, 65 MB per batch, written and read
// back only to be max-pooled.  Here one workgroup carries a tile of 64 points
// through a whole per-point MLP chain: activations stay in LDS, each layer is
// an FP32 MFMA GEMM (v_mfma_f32_16x16x4_f32: exact fp32 products and sums, as
// torch's fp32 GEMM), BatchNorm is folded into the weights, and the chain
// ends either in a max-pool over points (fused into the last GEMM's
// epilogue: a column max over the tile, then one float atomic max per
// channel) or in log-softmax.
//
// Tile geometry: 64 points = four 16-row MFMA blocks; 8 waves = 4 row blocks
// x 2 column halves of a 256-column chunk (up to 8 accumulator blocks of
// 16x16 per wave).  Weights stream through LDS in 16-row K-slabs of the chunk
// (16 KB, shared by the four row blocks), loaded with 16-byte global loads by
// all 512 threads and double-buffered: the next slab's loads are issued into
// registers before the current slab's MFMAs and written to LDS after them.
// B=16 clouds x 1000 points is 256 tiles: one workgroup per CU, one round.
//
// A layer flagged fuse_next (the seg head's 64 -> 512) is produced 64 columns
// at a time into a small LDS buffer and consumed at once by the next layer
// (512 -> 256), whose accumulators persist across the chunks, so the 512-wide
// activation never needs LDS of its own.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>

#include "../../include/ndnet_pointnet.h"

namespace {

constexpr int kP = 64;          // points per workgroup
constexpr int kWaves = 8;
constexpr int kThreads = 64 * kWaves;
constexpr int kRowBlocks = kP / 16;  // 4 (kWaves / 2)
constexpr int kNC = 256;        // columns per chunk
constexpr int kFuseNC = 64;     // columns per chunk of a fused layer
constexpr int kSlabPitch = kNC + 16;  // floats per slab row (breaks the 2-way bank conflict)
// KS: K rows per weight slab (template parameter: 32 where LDS allows, 16 for the seg head)
template <int KS>
struct Slab {
  static constexpr int kFloats = KS * kSlabPitch;
  static constexpr int kVecs = KS * kNC / 4 / kThreads;  // float4 loads per thread per slab
};
static_assert(kWaves == 2 * kRowBlocks, "waves = row blocks x 2 column halves");

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ inline void atomic_max_f32(float* addr, float v) {
  v = v + 0.0f;  // -0 -> +0 so the integer orderings below agree
  if (v >= 0.0f) atomicMax(reinterpret_cast<int*>(addr), __float_as_int(v));
  else atomicMin(reinterpret_cast<unsigned int*>(addr), __float_as_uint(v));
}

// dynamic LDS of k_pn_chain; regions are addressed by float offsets into it so
// every activation/slab access compiles to ds_* (a generic pointer would give
// flat_* ops, which count against vmcnt and stall on the weight prefetch)
extern __shared__ __attribute__((aligned(16))) float g_smem[];

// Loads this thread's share of slab rows [ks, ks + kr) x columns [c0, c0 + nc)
// of W^T (row stride ldw) into registers.  Out-of-range elements load a valid
// address and are zeroed at store time, so no vmcnt wait is forced into the
// middle of the MFMA loop.
template <int KS>
__device__ inline unsigned slab_load(f32x4 (&r)[Slab<KS>::kVecs], const float* __restrict__ wT, int ldw, int ks,
                                     int kr, int c0, int nc) {
  constexpr int kSlabVecs = Slab<KS>::kVecs;
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

template <int KS>
__device__ inline void slab_store(const f32x4 (&r)[Slab<KS>::kVecs], unsigned ok_mask, float* slab) {
  constexpr int kSlabVecs = Slab<KS>::kVecs;
#pragma unroll
  for (int v = 0; v < kSlabVecs; v++) {
    const int e = threadIdx.x + kThreads * v;
    const int row = e / (kNC / 4), col4 = e % (kNC / 4);
    *reinterpret_cast<f32x4*>(slab + row * kSlabPitch + 4 * col4) =
        ((ok_mask >> v) & 1) ? r[v] : f32x4{0.f, 0.f, 0.f, 0.f};
  }
}

// acc[j] += A[this wave's 16 rows][ks, ks + KS) . slab[0, KS)[cw + 16 j + ...]
// One staged slab's MFMAs; rows of the slab past K are zero and activation
// columns past K are finite (zero-filled input columns), so every k-step runs
// unconditionally.  Fragments are software-pipelined one k-step ahead.
template <int NB, int KS>
__device__ __attribute__((always_inline)) void mma_slab(f32x4 (&acc)[NB], const float* arow, int ks,
                                                        const float* slab, int cw) {
  const int lane = threadIdx.x & 63;
  const int kq = lane >> 4, cl = lane & 15;
  const float* bbase = slab + kq * kSlabPitch + cw + cl;
  float a = arow[ks];
  float bv[NB];
#pragma unroll
  for (int j = 0; j < NB; j++) bv[j] = bbase[16 * j];
#pragma unroll
  for (int kk = 0; kk < KS; kk += 4) {
    float an = 0.f, bn[NB];
    if (kk + 4 < KS) {
      an = arow[ks + kk + 4];
#pragma unroll
      for (int j = 0; j < NB; j++) bn[j] = bbase[(kk + 4) * kSlabPitch + 16 * j];
    }
#pragma unroll
    for (int j = 0; j < NB; j++) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bv[j], acc[j], 0, 0, 0);
    if (kk + 4 < KS) {
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
}

// acc[j] += A[rows of this wave][0, K) . W^T[k0 + (0..K)][c0 + cw + 16 j ...]
// A: activations at float offset `in` (pitch pin) of g_smem; W^T rows k0.. of
// the layer, columns [c0, c0 + nc).  Weight slabs double-buffered in LDS.
template <int NB, int KS>
__device__ __attribute__((always_inline)) void accumulate(f32x4 (&acc)[NB], int in, int pin,
                                                          const float* __restrict__ wT, int ldw, int K, int k0,
                                                          int c0, int nc, int slabs_off) {
  constexpr int kSlabFloats = Slab<KS>::kFloats;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int kq = lane >> 4, cl = lane & 15;
  const int cw = wc * (nc / 2);
  const int nslab = (K + KS - 1) / KS;
  float* const slabs = g_smem + slabs_off;
  f32x4 stage[Slab<KS>::kVecs];
  unsigned ok = slab_load<KS>(stage, wT, ldw, k0, K < KS ? K : KS, c0, nc);
  slab_store<KS>(stage, ok, slabs);
  __syncthreads();
  const float* arow = g_smem + in + (16 * wr + cl) * pin + kq;
  for (int s = 0; s < nslab; s++) {
    const int ks = s * KS;
    const bool more = s + 1 < nslab;
    if (more) ok = slab_load<KS>(stage, wT, ldw, k0 + ks + KS, K - ks - KS < KS ? K - ks - KS : KS, c0, nc);
    mma_slab<NB, KS>(acc, arow, ks, slabs + (s & 1) * kSlabFloats, cw);
    if (more) slab_store<KS>(stage, ok, slabs + ((s + 1) & 1) * kSlabFloats);
    __syncthreads();
  }
}

// Bias + ReLU of this wave's accumulators, stored to an activation region
// (column c of the chunk goes to column out_c0 + c).
template <int NB>
__device__ __attribute__((always_inline)) void store_act(const f32x4 (&acc)[NB], const float* __restrict__ bias,
                                                         int c0, int nc, int relu, int out, int pout, int out_c0) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int kq = lane >> 4, cl = lane & 15;
  const int cw = wc * (nc / 2);
#pragma unroll
  for (int j = 0; j < NB; j++) {
    const int c = cw + 16 * j + cl;
    const float bv = bias[c0 + c];
#pragma unroll
    for (int r = 0; r < 4; r++) {
      float v = acc[j][r] + bv;
      if (relu) v = fmaxf(v, 0.0f);
      g_smem[out + (16 * wr + 4 * kq + r) * pout + out_c0 + c] = v;
    }
  }
}

// Bias + ReLU + max over the tile's valid rows, one atomic max per channel:
// each wave reduces its 16 rows with shuffles, the four row blocks meet in LDS.
template <int NB>
__device__ __attribute__((always_inline)) void max_pool(const f32x4 (&acc)[NB], const float* __restrict__ bias, int c0,
                                                        int nc, int relu, int rows_valid, float* gmax, int cmax_off) {
  float* const s_cmax = g_smem + cmax_off;  // [kRowBlocks][kNC]
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int kq = lane >> 4, cl = lane & 15;
  const int cw = wc * (nc / 2);
#pragma unroll
  for (int j = 0; j < NB; j++) {
    const int c = cw + 16 * j + cl;
    const float bv = bias[c0 + c];
    float m = -INFINITY;
#pragma unroll
    for (int r = 0; r < 4; r++) {
      float v = acc[j][r] + bv;
      if (relu) v = fmaxf(v, 0.0f);
      if (16 * wr + 4 * kq + r < rows_valid) m = fmaxf(m, v);
    }
    m = fmaxf(m, __shfl_xor(m, 16, 64));
    m = fmaxf(m, __shfl_xor(m, 32, 64));
    if (lane < 16) s_cmax[wr * kNC + c] = m;
  }
  __syncthreads();
  for (int c = threadIdx.x; c < nc; c += kThreads) {
    float m = s_cmax[c];
#pragma unroll
    for (int q = 1; q < kRowBlocks; q++) m = fmaxf(m, s_cmax[q * kNC + c]);
    if (m > -INFINITY) atomic_max_f32(gmax + c0 + c, m);
  }
  __syncthreads();
}

struct LayerCtx {
  const float* __restrict__ wT;
  const float* __restrict__ bias;
  int ldw, K, relu;
};

__device__ inline LayerCtx layer_ctx(const ndnet_pn_chain& A, int l, int b) {
  const ndnet_pn_layer& L = A.L[l];
  LayerCtx C;
  C.wT = L.wT + (int64_t)b * L.w_cloud_stride;
  C.bias = L.bias + (int64_t)b * L.bias_cloud_stride;
  C.ldw = L.ldw;
  C.K = L.K;
  C.relu = L.relu;
  return C;
}

// An ordinary layer: one continuous mainloop over every (256-column chunk,
// K-slab) pair, so the next chunk's first slab is in flight during the last
// slab (and epilogue) of the current one.  All chunks of a layer share NB
// (N <= 256, or N a multiple of 256: checked by the launcher).
template <int NB, int KS>
__device__ void plain_layer(const LayerCtx& C, int N, int in, int pin, int out, int pout, float* gmax,
                            int rows_valid, int slabs_off, int cmax_off) {
  constexpr int kSlabFloats = Slab<KS>::kFloats;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int kq = lane >> 4, cl = lane & 15;
  const int nc = N < kNC ? N : kNC;
  const int cw = wc * (nc / 2);
  const int nslab = (C.K + KS - 1) / KS;
  const int total = (N / nc) * nslab;
  float* const slabs = g_smem + slabs_off;
  const float* arow = g_smem + in + (16 * wr + cl) * pin + kq;
  f32x4 acc[NB];
#pragma unroll
  for (int j = 0; j < NB; j++) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 stage[Slab<KS>::kVecs];
  unsigned ok = slab_load<KS>(stage, C.wT, C.ldw, 0, C.K < KS ? C.K : KS, 0, nc);
  slab_store<KS>(stage, ok, slabs);
  __syncthreads();
  int c0 = 0, s = 0;
  for (int t = 0; t < total; t++) {
    const bool more = t + 1 < total;
    const bool chunk_end = s + 1 == nslab;
    if (more) {
      const int s1 = chunk_end ? 0 : s + 1, c1 = chunk_end ? c0 + nc : c0;
      const int ks1 = s1 * KS;
      ok = slab_load<KS>(stage, C.wT, C.ldw, ks1, C.K - ks1 < KS ? C.K - ks1 : KS, c1, nc);
    }
    mma_slab<NB, KS>(acc, arow, s * KS, slabs + (t & 1) * kSlabFloats, cw);
    if (chunk_end) {
      if (gmax) max_pool<NB>(acc, C.bias, c0, nc, C.relu, rows_valid, gmax, cmax_off);
      else store_act<NB>(acc, C.bias, c0, nc, C.relu, out, pout, c0);
#pragma unroll
      for (int j = 0; j < NB; j++) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    if (more) slab_store<KS>(stage, ok, slabs + ((t + 1) & 1) * kSlabFloats);
    __syncthreads();
    if (chunk_end) {
      s = 0;
      c0 += nc;
    } else {
      s++;
    }
  }
  (void)lane;
  (void)kq;
  (void)cl;
}

// A fused pair: layer P (K -> N1, produced kFuseNC columns at a time into the
// F buffer) feeding layer Q (N1 -> N2 <= 256, accumulated across the chunks).
template <int NB2, int KS>
__device__ void fused_pair(const LayerCtx& P, int N1, const LayerCtx& Q, int N2, int in, int pin, int fbuf, int out,
                           int pout, float* gmax, int rows_valid, int slabs, int cmax_off) {
  constexpr int kFP = kFuseNC + 1;
  f32x4 acc2[NB2];
#pragma unroll
  for (int j = 0; j < NB2; j++) acc2[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int f0 = 0; f0 < N1; f0 += kFuseNC) {
    f32x4 acc1[kFuseNC / 32];
#pragma unroll
    for (int j = 0; j < kFuseNC / 32; j++) acc1[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    accumulate<kFuseNC / 32, KS>(acc1, in, pin, P.wT, P.ldw, P.K, 0, f0, kFuseNC, slabs);
    store_act<kFuseNC / 32>(acc1, P.bias, f0, kFuseNC, P.relu, fbuf, kFP, 0);  // chunk-local columns
    __syncthreads();
    accumulate<NB2, KS>(acc2, fbuf, kFP, Q.wT, Q.ldw, kFuseNC, f0, 0, N2, slabs);  // ends in a barrier
  }
  if (gmax) max_pool<NB2>(acc2, Q.bias, 0, N2, Q.relu, rows_valid, gmax, cmax_off);
  else store_act<NB2>(acc2, Q.bias, 0, N2, Q.relu, out, pout, 0);
}

#define NDNET_PN_NB_SWITCH(nb, CALL) \
  switch (nb) {                      \
    case 8: CALL(8); break;          \
    case 7: CALL(7); break;          \
    case 6: CALL(6); break;          \
    case 5: CALL(5); break;          \
    case 4: CALL(4); break;          \
    case 3: CALL(3); break;          \
    case 2: CALL(2); break;          \
    default: CALL(1); break;         \
  }

template <int KS>
__global__ void __launch_bounds__(kThreads) k_pn_chain(ndnet_pn_chain A, int has_fuse) {
  constexpr int kSlabFloats = Slab<KS>::kFloats;
  const int b = blockIdx.y;
  const int p0 = blockIdx.x * kP;
  // LDS: activation region 0 | region 1 | [fused-chunk buffer] | two weight slabs | [column maxima]
  const int pitch0 = A.max_width + 1, pitch1 = A.max_width2 + 1;
  const int reg[2] = {0, kP * pitch0};
  const int fbuf = kP * (pitch0 + pitch1);
  const int slabs = fbuf + (has_fuse ? kP * (kFuseNC + 1) : 0);
  const int cmax = slabs + 2 * kSlabFloats;
  // input tile, zero-filled to a whole slab of columns
  const int K0 = (A.L[0].K + KS - 1) / KS * KS;
  for (int e = threadIdx.x; e < kP * K0; e += kThreads) {
    const int r = e / K0, c = e % K0;
    const int p = p0 + r;
    float v = 0.0f;
    if (p < A.num_points && c < A.in_cols) v = A.x[((int64_t)b * A.num_points + p) * A.x_ld + c];
    g_smem[r * pitch0 + c] = v;
  }
  __syncthreads();
  const int rows_valid = A.num_points - p0;
  float* const gmax_b = A.mode == 0 ? A.gmax + (int64_t)b * A.gmax_ld : nullptr;
  for (int l = 0; l < A.num_layers; l++) {
    const int in = reg[l & 1], pin = (l & 1) ? pitch1 : pitch0;
    if (A.L[l].fuse_next) {  // layers l and l + 1 together; l + 1 writes region (l + 2) & 1
      const LayerCtx P = layer_ctx(A, l, b), Q = layer_ctx(A, l + 1, b);
      const bool last = l + 2 == A.num_layers;
      const int out = reg[(l + 2) & 1], pout = ((l + 2) & 1) ? pitch1 : pitch0;
      float* gm = (last && gmax_b) ? gmax_b : nullptr;
#define NDNET_PN_FUSED(NB) \
  fused_pair<NB, KS>(P, A.L[l].N, Q, A.L[l + 1].N, in, pin, fbuf, out, pout, gm, rows_valid, slabs, cmax)
      NDNET_PN_NB_SWITCH(A.L[l + 1].N / 32, NDNET_PN_FUSED)
#undef NDNET_PN_FUSED
      l++;
    } else {
      const LayerCtx C = layer_ctx(A, l, b);
      const bool last = l + 1 == A.num_layers;
      const int out = reg[(l + 1) & 1], pout = ((l + 1) & 1) ? pitch1 : pitch0;
      float* gm = (last && gmax_b) ? gmax_b : nullptr;
      const int N = A.L[l].N;
      const int nc = N < kNC ? N : kNC;
#define NDNET_PN_PLAIN(NB) plain_layer<NB, KS>(C, N, in, pin, out, pout, gm, rows_valid, slabs, cmax)
      NDNET_PN_NB_SWITCH(nc / 32, NDNET_PN_PLAIN)
#undef NDNET_PN_PLAIN
    }
    __syncthreads();
  }
  if (A.clear && blockIdx.x == 0 && blockIdx.y == 0)
    for (int64_t i = threadIdx.x; i < A.clear_count; i += kThreads) A.clear[i] = -INFINITY;
  if (A.mode == 1) {  // log_softmax over channels (ndtnet.py:239), [B][N][C+1] layout
    const int lg = reg[A.num_layers & 1];
    const int pl = (A.num_layers & 1) ? pitch1 : pitch0;
    for (int r = threadIdx.x; r < kP; r += kThreads) {
      const int p = p0 + r;
      if (p >= A.num_points) continue;
      const float* row = g_smem + lg + r * pl;
      float m = -INFINITY;
      for (int c = 0; c < A.out_cols; c++) m = fmaxf(m, row[c]);
      float s = 0.0f;
      for (int c = 0; c < A.out_cols; c++) s += expf(row[c] - m);
      const float ls = logf(s);
      float* o = A.out + ((int64_t)b * A.num_points + p) * A.out_cols;
      for (int c = 0; c < A.out_cols; c++) o[c] = (row[c] - m) - ls;
    }
  }
  (void)kSlabFloats;
}

// ---------------------------------------------------------------------------
// Per-cloud steps between the chains (the TNet FC heads, ndtnet.py:53-60, and
// the weight folds), on the same stream.  The batch is small (B clouds, a
// 16-row GEMM at B = 16), so these are weight-streaming GEMVs, not MFMA tiles.

// out[b][n] = act(bias[n] + sum_k in[b][k] * W[n][k]), b < B <= 16.
// One wave per output channel (4 per workgroup): its 64 lanes split K in
// 16-byte pieces and keep one partial sum per cloud, so the weight row is read
// once for all clouds; the partials meet in a wave reduction.
__global__ void __launch_bounds__(256) k_pn_fc(const float* __restrict__ in, int ld_in, const float* __restrict__ W,
                                               const float* __restrict__ bias, float* __restrict__ out, int ld_out,
                                               int B, int K, int N, int relu) {
  const int lane = threadIdx.x & 63;
  const int n = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (n >= N) return;
  const int kv = K / 4;
  const f32x4* w = reinterpret_cast<const f32x4*>(W + (int64_t)n * K);
  float acc[16];
#pragma unroll
  for (int b = 0; b < 16; b++) acc[b] = 0.0f;
  for (int f = lane; f < kv; f += 64) {
    const f32x4 wv = w[f];
    f32x4 xv[16];
#pragma unroll
    for (int b = 0; b < 16; b++) xv[b] = reinterpret_cast<const f32x4*>(in + (int64_t)(b < B ? b : 0) * ld_in)[f];
#pragma unroll
    for (int b = 0; b < 16; b++) {
      const f32x4 pr = xv[b] * wv;
      acc[b] += (pr[0] + pr[1]) + (pr[2] + pr[3]);
    }
  }
#pragma unroll
  for (int b = 0; b < 16; b++)
    for (int o = 32; o > 0; o >>= 1) acc[b] += __shfl_xor(acc[b], o, 64);
  if (lane < B) {
    float v = 0.0f;
#pragma unroll
    for (int b = 0; b < 16; b++) v = lane == b ? acc[b] : v;
    v += bias[n];
    if (relu) v = fmaxf(v, 0.0f);
    out[(int64_t)lane * ld_out + n] = v;
  }
}

// TNet(3) tail: t1[b] = fc3(h2[b]) (+ I, folded into the bias) and the t1
// fold of conv1, w1T[b] = t1[b] (1 x 9) @ basis (9 x 768).  One workgroup per cloud.
__global__ void __launch_bounds__(256) k_pn_head3(const float* __restrict__ h2, int ld_h, const float* __restrict__ W3,
                                                  const float* __restrict__ b3, const float* __restrict__ basis,
                                                  float* __restrict__ t1_out, float* __restrict__ w1T, int K, int M) {
  __shared__ float s_t[9];
  const int b = blockIdx.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const float* h = h2 + (int64_t)b * ld_h;
  for (int o = wave; o < 9; o += 4) {  // one wave per output, lanes split K
    float acc = 0.0f;
    for (int k = lane; k < K; k += 64) acc += h[k] * W3[(int64_t)o * K + k];
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
    if (lane == 0) {
      s_t[o] = acc + b3[o];
      t1_out[b * 9 + o] = acc + b3[o];
    }
  }
  __syncthreads();
  for (int m = threadIdx.x; m < M; m += blockDim.x) {
    float acc = 0.0f;
#pragma unroll
    for (int a = 0; a < 9; a++) acc += s_t[a] * basis[a * M + m];
    w1T[(int64_t)b * M + m] = acc;
  }
}

// TNet(64) fold: out[b] (64 x N) = t2[b] (64 x 64) @ rhs (64 x N), N % 64 == 0.
// Workgroup (column tile of 64, cloud): both operand tiles in LDS, 4 x 4
// outputs per thread.
__global__ void __launch_bounds__(256) k_pn_fold64(const float* __restrict__ t2, const float* __restrict__ rhs,
                                                   float* __restrict__ out, int N) {
  __shared__ float s_a[64][65];
  __shared__ float s_b[64][68];
  const int b = blockIdx.y, j0 = blockIdx.x * 64;
  const float* A = t2 + (int64_t)b * 4096;
  for (int e = threadIdx.x; e < 4096; e += 256) {
    s_a[e >> 6][e & 63] = A[e];
    s_b[e >> 6][e & 63] = rhs[(int64_t)(e >> 6) * N + j0 + (e & 63)];
  }
  __syncthreads();
  const int ti = (threadIdx.x >> 4) * 4, tj = (threadIdx.x & 15) * 4;
  float acc[4][4] = {};
  for (int k = 0; k < 64; k++) {
    float av[4], bv[4];
#pragma unroll
    for (int r = 0; r < 4; r++) av[r] = s_a[ti + r][k];
#pragma unroll
    for (int c = 0; c < 4; c++) bv[c] = s_b[k][tj + c];
#pragma unroll
    for (int r = 0; r < 4; r++)
#pragma unroll
      for (int c = 0; c < 4; c++) acc[r][c] += av[r] * bv[c];
  }
  float* o = out + (int64_t)b * 64 * N;
#pragma unroll
  for (int r = 0; r < 4; r++)
    *reinterpret_cast<f32x4*>(o + (int64_t)(ti + r) * N + j0 + tj) = f32x4{acc[r][0], acc[r][1], acc[r][2], acc[r][3]};
}

}  // namespace

extern "C" {

int ndnet_pn_fc_run(const float* in, int ld_in, const float* W, const float* bias, float* out, int ld_out, int batch,
                    int K, int N, int relu, void* stream) {
  if (!in || !W || !bias || !out || batch <= 0 || batch > 16 || K <= 0 || K % 4 || N <= 0 || ld_in % 4 ||
      ((uintptr_t)in | (uintptr_t)W) % 16)
    return -20;
  k_pn_fc<<<(N + 3) / 4, 256, 0, (hipStream_t)stream>>>(in, ld_in, W, bias, out, ld_out, batch, K, N, relu);
  return hipGetLastError() == hipSuccess ? 0 : -21;
}

int ndnet_pn_head3_run(const float* h2, int ld_h, const float* W3, const float* b3, const float* basis, float* t1,
                       float* w1T, int batch, int K, int M, void* stream) {
  if (!h2 || !W3 || !b3 || !basis || !t1 || !w1T || batch <= 0 || K <= 0 || M <= 0) return -20;
  k_pn_head3<<<batch, 256, 0, (hipStream_t)stream>>>(h2, ld_h, W3, b3, basis, t1, w1T, K, M);
  return hipGetLastError() == hipSuccess ? 0 : -21;
}

int ndnet_pn_fold64_run(const float* t2, const float* rhs, float* out, int batch, int N, void* stream) {
  if (!t2 || !rhs || !out || batch <= 0 || N <= 0 || N % 64 || ((uintptr_t)out % 16)) return -20;
  k_pn_fold64<<<dim3(N / 64, batch), 256, 0, (hipStream_t)stream>>>(t2, rhs, out, N);
  return hipGetLastError() == hipSuccess ? 0 : -21;
}


// One fused point-MLP chain over `batch` clouds on `stream` (see pointnet.h).
int ndnet_pn_chain_run(const ndnet_pn_chain* args, int batch, void* stream) {
  if (!args || batch <= 0 || args->num_layers < 1 || args->num_layers > NDNET_PN_MAX_LAYERS) return -20;
  // activation regions: layer l reads region l & 1 (or the fused-chunk buffer
  // after a fused layer) and writes region (l + 1) & 1
  int w[2] = {(args->L[0].K + 15) / 16 * 16, 0};  // the input tile is zero-filled to a whole K-slab (>= 16)
  for (int l = 0; l < args->num_layers; l++) {
    const ndnet_pn_layer& L = args->L[l];
    if (L.K % 4 || L.N % 32 || L.ldw % 4 || L.ldw < L.N) return -20;
    const bool fed = l > 0 && args->L[l - 1].fuse_next;
    if (fed) {
      if (L.K != args->L[l - 1].N || L.N > kNC || L.fuse_next) return -20;
    } else if (l > 0 && L.K > w[l & 1]) {
      return -20;
    }
    if (L.fuse_next) {
      if (l + 1 >= args->num_layers || L.N % kFuseNC) return -20;
      continue;  // not stored in a region
    }
    const bool stored = l + 1 < args->num_layers || args->mode == 1;
    if (stored && L.N > w[(l + 1) & 1]) w[(l + 1) & 1] = L.N;
  }
  if (args->max_width < w[0] || args->max_width2 < w[1]) return -20;
  bool has_fuse = false;
  for (int l = 0; l < args->num_layers; l++) {
    const ndnet_pn_layer& L = args->L[l];
    has_fuse |= L.fuse_next != 0;
    const bool fed = l > 0 && args->L[l - 1].fuse_next;
    if (!L.fuse_next && !fed && L.N > kNC && L.N % kNC) return -20;  // chunks of one layer share a width
  }
  // 32-row weight slabs when they fit in LDS, else 16
  auto lds_for = [&](int ks) {
    return sizeof(float) * ((size_t)kP * (args->max_width + 1 + args->max_width2 + 1 + (has_fuse ? kFuseNC + 1 : 0)) +
                            2 * (size_t)ks * kSlabPitch + (args->mode == 0 ? kRowBlocks * kNC : 0));
  };
  // (the input tile is zero-filled to a whole slab of columns, so region 0 must hold that many)
  const int ks = (lds_for(32) <= 160 * 1024 && args->max_width >= (args->L[0].K + 31) / 32 * 32) ? 32 : 16;
  const size_t lds = lds_for(ks);
  static bool attr_set = false;
  if (!attr_set) {
    if (hipFuncSetAttribute((const void*)k_pn_chain<32>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) !=
            hipSuccess ||
        hipFuncSetAttribute((const void*)k_pn_chain<16>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) !=
            hipSuccess)
      return -21;
    attr_set = true;
  }
  if (lds > 160 * 1024) return -20;
  dim3 grid((args->num_points + kP - 1) / kP, batch);
  if (ks == 32)
    k_pn_chain<32><<<grid, kThreads, lds, (hipStream_t)stream>>>(*args, has_fuse ? 1 : 0);
  else
    k_pn_chain<16><<<grid, kThreads, lds, (hipStream_t)stream>>>(*args, has_fuse ? 1 : 0);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    fprintf(stderr, "ndnet_amd: k_pn_chain launch failed: %s\n", hipGetErrorString(e));
    return -21;
  }
  return 0;
}

}  // extern "C"
