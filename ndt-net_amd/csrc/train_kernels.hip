// Train-mode point-MLP kernels for gfx950 (include/ndnet_train.h).
//
// The reference trains NDTNetSegmentation with torch autograd
// (tools/train.py:67-81): every per-point block is Conv1d(k=1) -> BatchNorm1d
// with batch statistics -> ReLU (ndnet/models/ndtnet.py:48-50, 148-152,
// 233-239), and the backward runs the same ops in reverse.  Here each block is
// two kernels each way, on torch's NCL layout ([B][C][N], points contiguous):
//   forward:  k_tr_gemm (y = W x + b, fp32 MFMA)  ->  k_tr_bn_fwd (statistics,
//             normalise, affine, ReLU; running-stat update)
//   backward: k_tr_bn_bwd (ReLU mask, BN backward, bias gradient)  ->
//             k_tr_gemm twice (dx = W^T dy; dW = sum dy x^T as split-K
//             partials) -> k_tr_sum_parts
// The GEMM reads either operand in whichever orientation torch stores it, so
// no transpose kernels run (the MIOpen path of the same step spends a large
// share of its time in NCHW <-> NHWC transposes around the 1x1 convolutions,
// profiles/r03_train_graph_kernel_stats.csv).
//
// GEMM tiling: 64 x 64 output tile per workgroup of 4 waves, each wave 32 x 32
// (2 x 2 blocks of v_mfma_f32_16x16x4_f32, four accumulator sets, exact fp32 products and sums as
// torch's fp32 GEMM), k-steps of 16 through a double-buffered LDS tile with
// the next step's global loads in flight during the current step's MFMAs.
// Loads are bounds-checked (zero fill), so ragged sizes (K = 3 or 12 input
// channels, 29 output classes, 1000 points) need no padding.
//
// BatchNorm statistics: one workgroup per channel holds the channel's B * N
// values in registers (up to 16384), sums in double, two passes (mean, then
// the squared deviations), so the variance has no E[x^2] - E[x]^2
// cancellation.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>

#include <algorithm>

#include "../../include/ndnet_train.h"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kTM = 64, kTN = 64, kTK = 16;
// LDS row pitch of a [k][row] tile, by how the operand is stored (ds_write_b32
// / ds_read_b32 bank = dword address mod 32, two 32-lane groups per wave):
//  * k-major operands (a thread holds 4 consecutive k of one row, stored as 4
//    dwords): pitch = TM + 18 -- the 8 rows x 4 k-quads of a lane group land
//    on distinct banks (4 * 18 = 8 mod 32); the MFMA operand reads (2 k rows x
//    16 columns per group) overlap on 2 banks;
//  * row-major operands (4 consecutive rows of one k, one ds_write_b128):
//    pitch = TM + 16 (16-byte aligned rows; operand reads conflict-free).
// Round 3's single pitch TM + 17 with one scalar load per element:
// profiles/r03t6_train_pad17.txt.
template <int TM, bool KMAJOR>
constexpr int tile_pitch() { return TM + (KMAJOR ? 18 : 16); }

constexpr int kBnThreads = 512;
constexpr int kBnValues = 16384;  // values per channel held in registers across the workgroup (B * N <= this
                                  // reads the channel once)
constexpr int kPoolMaxB = 64;  // pool mode: clouds per launch  // values per thread held in registers: B * N <= 16384 reads the channel once

// global -> registers: this thread's 4 elements of the (k0 .. k0 + 16) x TM
// tile (TM * 4 threads), P contiguous along k (KMAJOR) or along the row
// index.  Each thread loads 4 consecutive elements along the contiguous axis:
// one 16-byte load when they are in range and aligned (the common case:
// k-steps of 16, rows of 1000 points), else element by element with zero fill.
// KMAJOR: row t / 4, k (t % 4) * 4 .. + 3; else k t / (TM / 4), rows
// (t % (TM / 4)) * 4 .. + 3.
template <int TM, bool KMAJOR>
__device__ __forceinline__ void tile_load(const float* __restrict__ P, int64_t ld, int r0, int k0, int R, int kend,
                                          float (&v)[4]) {
  const int t = threadIdx.x;
  const int kk = KMAJOR ? (t & 3) * 4 : t / (TM / 4);
  const int rr = KMAJOR ? t >> 2 : (t % (TM / 4)) * 4;
  const int gr = r0 + rr, gk = k0 + kk;
  const float* p = KMAJOR ? P + (int64_t)gr * ld + gk : P + (int64_t)gk * ld + gr;
  const bool full = KMAJOR ? (gr < R && gk + 3 < kend) : (gk < kend && gr + 3 < R);
  if (full && ((uintptr_t)p & 15) == 0) {
    const f32x4 x = *reinterpret_cast<const f32x4*>(p);
    v[0] = x[0];
    v[1] = x[1];
    v[2] = x[2];
    v[3] = x[3];
  } else {
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const bool in = KMAJOR ? (gr < R && gk + i < kend) : (gk < kend && gr + i < R);
      v[i] = in ? p[i] : 0.0f;
    }
  }
}

// registers -> LDS tile [k][row] (row contiguous: one MFMA operand read per lane)
template <int TM, bool KMAJOR>
__device__ __forceinline__ void tile_store(float* __restrict__ s, const float (&v)[4]) {
  constexpr int P = tile_pitch<TM, KMAJOR>();
  const int t = threadIdx.x;
  if (KMAJOR) {
    const int kk = (t & 3) * 4, rr = t >> 2;
#pragma unroll
    for (int i = 0; i < 4; i++) s[(kk + i) * P + rr] = v[i];
  } else {
    const int kk = t / (TM / 4), rr = (t % (TM / 4)) * 4;
    *reinterpret_cast<f32x4*>(s + kk * P + rr) = f32x4{v[0], v[1], v[2], v[3]};
  }
}

// TM x TM output tile per workgroup of TM / 8 waves: TM = 64 -> 2 x 2 waves of
// 32 x 32 (four accumulator sets), TM = 128 -> 2 x 4 waves of 64 x 32 (two sets,
// twice the MFMAs per LDS operand read; for the wide layers)
template <int TM, bool AK, bool BK, int KT = kTK>  // KT: k per LDS step, 16 or 32 (two 16-deep sub-tiles)
__global__ __launch_bounds__(TM * 4) void k_tr_gemm(const float* __restrict__ A, const float* __restrict__ B,
                                                    float* __restrict__ C, const float* __restrict__ bias,
                                                    int64_t sbias, int M, int N, int K, int64_t lda, int64_t ldb,
                                                    int64_t ldc, int64_t sAz, int64_t sBz, int64_t sCz, int batch,
                                                    int cpz, int nchunks, int kchunk) {
  constexpr int PA = tile_pitch<TM, AK>(), PB = tile_pitch<TM, BK>();  // LDS row pitches
  constexpr int WN = 2 * (TM / 64);       // waves along N
  constexpr int IM = TM / 32;             // 16-row blocks per wave (wave tile TM / 2 rows x 32 columns)
  constexpr int KS = TM == 64 ? 4 : 2;    // accumulator sets (k-quad ks uses set ks % KS)
  constexpr int NS = KT / kTK;             // 16-deep sub-tiles per step
  __shared__ __attribute__((aligned(16))) float sA[2][KT * PA];
  __shared__ __attribute__((aligned(16))) float sB[2][KT * PB];
  const int z = blockIdx.z, zg = z / nchunks, zc = z - zg * nchunks;
  const int cl0 = zg * cpz, ncl = min(cpz, batch - cl0);  // this part's clouds
  C += z * sCz;
  if (bias) bias += cl0 * sbias;
  const int kbeg = zc * kchunk;
  const int kend = min(K, kbeg + kchunk);
  const int m0 = blockIdx.y * TM, n0 = blockIdx.x * TM;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = (wave / WN) * (TM / 2), wn = (wave % WN) * 32;
  const int r16 = lane & 15, q = lane >> 4;

  // several accumulator sets: shorter fp32 sums (added pairwise at the end)
  // than one chain over all of K, and independent MFMA chains
  f32x4 acc[KS][IM][2];
#pragma unroll
  for (int ks = 0; ks < KS; ks++)
#pragma unroll
    for (int i = 0; i < IM; i++)
#pragma unroll
      for (int j = 0; j < 2; j++) acc[ks][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // steps t = cloud * nst + s: the part's clouds one after another (split-K over clouds)
  const int nst = kend > kbeg ? (kend - kbeg + KT - 1) / KT : 0;
  const int total = ncl > 0 ? ncl * nst : 0;
  float ra[NS][4], rb[NS][4];
  auto load = [&](int t) {
    const int cl = t / nst, st = t - cl * nst;
    const int64_t c = cl0 + cl;
#pragma unroll
    for (int u = 0; u < NS; u++) {
      tile_load<TM, AK>(A + c * sAz, lda, m0, kbeg + st * KT + kTK * u, M, kend, ra[u]);
      tile_load<TM, BK>(B + c * sBz, ldb, n0, kbeg + st * KT + kTK * u, N, kend, rb[u]);
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int u = 0; u < NS; u++) {
      tile_store<TM, AK>(sA[buf] + kTK * PA * u, ra[u]);
      tile_store<TM, BK>(sB[buf] + kTK * PB * u, rb[u]);
    }
  };
  if (total > 0) {
    load(0);
    store(0);
  }
  __syncthreads();
  for (int t = 0; t < total; t++) {
    const int cur = t & 1;
    const bool more = t + 1 < total;
    if (more) load(t + 1);  // the next k-step's loads fly under this step's MFMAs
    const float* a = sA[cur];
    const float* b = sB[cur];
#pragma unroll
    for (int ks = 0; ks < KT / 4; ks++) {  // k-quad ks of the step adds into set ks % KS (the global k-quad's)
      const int oa = (ks * 4 + q) * PA, ob = (ks * 4 + q) * PB;
      float av[IM];
#pragma unroll
      for (int i = 0; i < IM; i++) av[i] = a[oa + wm + 16 * i + r16];
      const float b0 = b[ob + wn + r16], b1 = b[ob + wn + 16 + r16];
#pragma unroll
      for (int i = 0; i < IM; i++) {
        acc[ks % KS][i][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i], b0, acc[ks % KS][i][0], 0, 0, 0);
        acc[ks % KS][i][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i], b1, acc[ks % KS][i][1], 0, 0, 0);
      }
    }
    if (more) store(cur ^ 1);  // the other buffer was last read before the previous barrier
    __syncthreads();
  }
  // lane (q, r16) of block (i, j): rows 4 q + r, column r16
#pragma unroll
  for (int i = 0; i < IM; i++)
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const int gm = m0 + wm + 16 * i + 4 * q + r;
      if (gm >= M) continue;
      const float bv = bias ? bias[gm] : 0.0f;
#pragma unroll
      for (int j = 0; j < 2; j++) {
        const int gn = n0 + wn + 16 * j + r16;
        if (gn >= N) continue;
        float v;
        if (KS == 4)
          v = (acc[0][i][j][r] + acc[1 % KS][i][j][r]) + (acc[2 % KS][i][j][r] + acc[3 % KS][i][j][r]);
        else
          v = acc[0][i][j][r] + acc[1 % KS][i][j][r];
        C[(int64_t)gm * ldc + gn] = v + bv;
      }
    }
}

// ---- the same GEMM on the bf16 matrix cores, fp32-accurate ("x6") ----
// Every operand x is split x = h + m + l into three bf16 in the tile store
// (h = bf16(x), m = bf16(x - h), l = bf16(x - h - m): 24 significant bits, each
// residual exact in fp32), and a product keeps the six partial products of
// weight >= 2^-16 (mm, mh, lh, hl, hm, hh, smallest first), each exact and
// accumulated in fp32 by v_mfma_f32_16x16x32_bf16 -- the eval chains' form
// (pointnet_kernels.hip, test_split_bf16_layers_are_fp32_accurate).  Six
// 16-cycle MFMAs per 16x16x32 block against eight 32-cycle fp32 ones.
// 64 x 64 tile, 4 waves of 32 x 32, k-steps of 32; LDS tiles [row][k] per
// plane (pitch 48 bf16), double-buffered; a thread loads and splits 8
// consecutive k of one row per operand and stores each plane with one
// ds_write_b128.
typedef __bf16 tr_bf16x8 __attribute__((ext_vector_type(8)));
constexpr int kX6K = 32, kX6P = 48, kX6Plane = 64 * kX6P;

template <bool KMAJOR>
__device__ __forceinline__ void x6_load(const float* __restrict__ P, int64_t ld, int r0, int k0, int R, int kend,
                                        float (&v)[8]) {
  const int t = threadIdx.x;
  const int rr = KMAJOR ? t >> 2 : t & 63, kk = KMAJOR ? (t & 3) * 8 : (t >> 6) * 8;
  const int gr = r0 + rr, gk = k0 + kk;
  if (KMAJOR) {
    const float* p = P + (int64_t)gr * ld + gk;
    if (gr < R && gk + 7 < kend && ((uintptr_t)p & 15) == 0) {
      const f32x4 x0 = reinterpret_cast<const f32x4*>(p)[0], x1 = reinterpret_cast<const f32x4*>(p)[1];
#pragma unroll
      for (int i = 0; i < 4; i++) {
        v[i] = x0[i];
        v[4 + i] = x1[i];
      }
    } else {
#pragma unroll
      for (int i = 0; i < 8; i++) v[i] = (gr < R && gk + i < kend) ? p[i] : 0.0f;
    }
  } else {  // lanes walk the rows: each of the 8 loads is 64 consecutive floats of a wave
#pragma unroll
    for (int i = 0; i < 8; i++) v[i] = (gr < R && gk + i < kend) ? P[(int64_t)(gk + i) * ld + gr] : 0.0f;
  }
}

template <bool KMAJOR>
__device__ __forceinline__ void x6_store(__bf16* __restrict__ s, const float (&v)[8]) {
  const int t = threadIdx.x;
  const int rr = KMAJOR ? t >> 2 : t & 63, kk = KMAJOR ? (t & 3) * 8 : (t >> 6) * 8;
  tr_bf16x8 h, m, l;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const __bf16 hh = (__bf16)v[i];
    const float r = v[i] - (float)hh;
    const __bf16 mm = (__bf16)r;
    h[i] = hh;
    m[i] = mm;
    l[i] = (__bf16)(r - (float)mm);
  }
  const int e = rr * kX6P + kk;
  *reinterpret_cast<tr_bf16x8*>(s + e) = h;
  *reinterpret_cast<tr_bf16x8*>(s + kX6Plane + e) = m;
  *reinterpret_cast<tr_bf16x8*>(s + 2 * kX6Plane + e) = l;
}

template <bool AK, bool BK>
__global__ __launch_bounds__(256) void k_tr_gemm_x6(const float* __restrict__ A, const float* __restrict__ B,
                                                    float* __restrict__ C, const float* __restrict__ bias,
                                                    int64_t sbias, int M, int N, int K, int64_t lda, int64_t ldb,
                                                    int64_t ldc, int64_t sAz, int64_t sBz, int64_t sCz, int batch,
                                                    int cpz, int nchunks, int kchunk) {
#pragma clang fp contract(off)
  __shared__ __attribute__((aligned(16))) __bf16 sA[2][3 * kX6Plane];
  __shared__ __attribute__((aligned(16))) __bf16 sB[2][3 * kX6Plane];
  const int z = blockIdx.z, zg = z / nchunks, zc = z - zg * nchunks;
  const int cl0 = zg * cpz, ncl = min(cpz, batch - cl0);
  C += z * sCz;
  if (bias) bias += cl0 * sbias;
  const int kbeg = zc * kchunk;
  const int kend = min(K, kbeg + kchunk);
  const int m0 = blockIdx.y * 64, n0 = blockIdx.x * 64;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = (wave >> 1) * 32, wn = (wave & 1) * 32;
  const int r16 = lane & 15, q = lane >> 4;
  f32x4 acc[2][2][2];  // [set][row block][column block]: k-steps alternate between two sets
#pragma unroll
  for (int s = 0; s < 2; s++)
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
      for (int j = 0; j < 2; j++) acc[s][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nst = kend > kbeg ? (kend - kbeg + kX6K - 1) / kX6K : 0;
  const int total = ncl > 0 ? ncl * nst : 0;
  float ra[8], rb[8];
  auto load = [&](int t) {
    const int cl = t / nst, st = t - cl * nst;
    const int64_t c = cl0 + cl;
    x6_load<AK>(A + c * sAz, lda, m0, kbeg + st * kX6K, M, kend, ra);
    x6_load<BK>(B + c * sBz, ldb, n0, kbeg + st * kX6K, N, kend, rb);
  };
  if (total > 0) {
    load(0);
    x6_store<AK>(sA[0], ra);
    x6_store<BK>(sB[0], rb);
  }
  __syncthreads();
  for (int t = 0; t < total; t++) {
    const int cur = t & 1;
    const bool more = t + 1 < total;
    if (more) load(t + 1);
    const __bf16* a = sA[cur] + 8 * q;
    const __bf16* b = sB[cur] + 8 * q;
    tr_bf16x8 af[2][3], bw[2][3];
#pragma unroll
    for (int p = 0; p < 3; p++)
#pragma unroll
      for (int i = 0; i < 2; i++) {
        af[i][p] = *reinterpret_cast<const tr_bf16x8*>(a + p * kX6Plane + (wm + 16 * i + r16) * kX6P);
        bw[i][p] = *reinterpret_cast<const tr_bf16x8*>(b + p * kX6Plane + (wn + 16 * i + r16) * kX6P);
      }
    f32x4(&ac)[2][2] = acc[t & 1];
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
      for (int j = 0; j < 2; j++) {
        f32x4 x = ac[i][j];
        x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][1], bw[j][1], x, 0, 0, 0);  // m m
        x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][1], bw[j][0], x, 0, 0, 0);  // m h
        x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][2], bw[j][0], x, 0, 0, 0);  // l h
        x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][0], bw[j][2], x, 0, 0, 0);  // h l
        x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][0], bw[j][1], x, 0, 0, 0);  // h m
        x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][0], bw[j][0], x, 0, 0, 0);  // h h
        ac[i][j] = x;
      }
    if (more) {
      x6_store<AK>(sA[cur ^ 1], ra);
      x6_store<BK>(sB[cur ^ 1], rb);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 2; i++)
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const int gm = m0 + wm + 16 * i + 4 * q + r;
      if (gm >= M) continue;
      const float bv = bias ? bias[gm] : 0.0f;
#pragma unroll
      for (int j = 0; j < 2; j++) {
        const int gn = n0 + wn + 16 * j + r16;
        if (gn >= N) continue;
        C[(int64_t)gm * ldc + gn] = (acc[0][i][j][r] + acc[1][i][j][r]) + bv;
      }
    }
}

// out[i] = part[0][i] + part[1][i] + ... in part order; one element per
// thread, up to 32 parts' loads issued before their sums (one memory latency
// per launch at the weight gradients' <= 32 parts: round 4's 4 elements and 8
// parts per round left the small layers' launches at 4 workgroups and 4
// dependent rounds, 178 us a step over 19 launches, r05k)
constexpr int kSumParts = 32;
// out[r * ldo + c] = the sum of part[p][r * cols + c] over p in part order
// (ldo == cols: a contiguous output; the seg head's conv1 writes the first
// columns of its [Cout][c + F] weight gradient in place)
__global__ __launch_bounds__(256) void k_tr_sum_parts(const float* __restrict__ part, float* __restrict__ out,
                                                      int64_t count, int nparts, int64_t cols, int64_t ldo) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= count) return;
  float s = 0.0f;
  for (int p0 = 0; p0 < nparts; p0 += kSumParts) {
    float v[kSumParts];
#pragma unroll
    for (int u = 0; u < kSumParts; u++) v[u] = p0 + u < nparts ? part[(int64_t)(p0 + u) * count + i] : 0.0f;
#pragma unroll
    for (int u = 0; u < kSumParts; u++)
      if (p0 + u < nparts) s = (p0 + u == 0) ? v[u] : s + v[u];
  }
  out[cols == ldo ? i : i / cols * ldo + i % cols] = s;
}

// sum over the workgroup in a fixed order (wave shuffles, then the waves in order)
template <int T>
__device__ double block_sum(double v, double* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const int wave = threadIdx.x >> 6;
  __syncthreads();  // red may still be read by the previous call
  if ((threadIdx.x & 63) == 0) red[wave] = v;
  __syncthreads();
  double t = red[0];
  for (int w = 1; w < T / 64; w++) t += red[w];
  return t;
}

// this thread's elements j = tid, tid + T, ... of one channel as (cloud, point),
// advanced without divisions
template <int T>
struct ChanWalk {
  int b, n;
  __device__ explicit ChanWalk(int N) : b(0), n(threadIdx.x) { fold(N); }
  __device__ void fold(int N) {
    while (n >= N) {
      n -= N;
      b++;
    }
  }
  __device__ void next(int N) {
    n += T;
    fold(N);
  }
  __device__ int64_t off(int C, int N, int c) const { return ((int64_t)b * C + c) * N + n; }
};

// Round 6: the channel walked four points at a time (N % 4 == 0, 16-byte aligned
// rows: every [B][C][N] activation of the model at N = 1000), one 16-byte load
// or store per thread and step instead of four 4-byte ones.  Element (b, n4 * 4 + k)
// of the float4 index q = tid + T i.  NDNET_TR_BN_VEC=0 keeps the scalar walk (A/B).
template <int T>
struct ChanWalk4 {
  int b, n4;  // cloud, float4 index in the cloud's row of N / 4
  __device__ explicit ChanWalk4(int N4) : b(0), n4(threadIdx.x) { fold(N4); }
  __device__ void fold(int N4) {
    while (n4 >= N4) {
      n4 -= N4;
      b++;
    }
  }
  __device__ void next(int N4) {
    n4 += T;
    fold(N4);
  }
  __device__ int64_t off(int C, int N, int c) const { return ((int64_t)b * C + c) * N + 4 * (int64_t)n4; }
};
#ifndef NDNET_TR_BN_VEC
#define NDNET_TR_BN_VEC 1
#endif
__device__ inline bool bn_vec_ok(int N, const void* a, const void* b2) {
  return NDNET_TR_BN_VEC && N % 4 == 0 && ((((uintptr_t)a) | ((uintptr_t)b2)) & 15u) == 0;
}

// the normalised, affine value: one rounding per operation (no contraction), so
// the backward's ReLU mask recomputed from y equals the forward's output sign
__device__ __forceinline__ float bn_apply(float v, float fm, float inv, float g, float bt) {
  return __fadd_rn(__fmul_rn(__fmul_rn(__fsub_rn(v, fm), inv), g), bt);
}

template <int T>
__global__ __launch_bounds__(T) void k_tr_bn_fwd(const float* __restrict__ y, float* __restrict__ z,
                                                          float* __restrict__ mean, float* __restrict__ invstd,
                                                          float* __restrict__ rmean, float* __restrict__ rvar,
                                                          const float* __restrict__ gamma,
                                                          const float* __restrict__ beta, int Bn, int C, int N,
                                                          float eps, float momentum, int relu,
                                                          float* __restrict__ pool, int* __restrict__ pool_idx,
                                                          long long* __restrict__ batches_tracked) {
  __shared__ double red[T / 64];
  constexpr int kCache = kBnValues / T;
  __shared__ unsigned long long pk[kPoolMaxB];  // per cloud: (ordered value bits, ~point) -- max = first max
  const int c = blockIdx.x;
  // BatchNorm1d's num_batches_tracked += 1 (torch does it as a launch of its own)
  if (batches_tracked && c == 0 && threadIdx.x == 0) batches_tracked[0] += 1;
  const int64_t M = (int64_t)Bn * N;
  const bool cached = M <= (int64_t)kBnValues;
  if (pool && threadIdx.x < Bn) pk[threadIdx.x] = 0ull;  // ordered before use by block_sum's barriers
  if (cached && bn_vec_ok(N, y, pool ? (const void*)y : (const void*)z)) {
    constexpr int kC4 = kCache / 4;
    const int N4 = N / 4;
    f32x4 v4[kC4];
    double s = 0.0;
    {
      ChanWalk4<T> w(N4);
#pragma unroll
      for (int i = 0; i < kC4; i++, w.next(N4)) v4[i] = w.b < Bn ? *reinterpret_cast<const f32x4*>(y + w.off(C, N, c))
                                                              : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int i = 0; i < kC4; i++) s += ((double)v4[i][0] + (double)v4[i][1]) + ((double)v4[i][2] + (double)v4[i][3]);
    const double mu = block_sum<T>(s, red) / (double)M;
    double s2 = 0.0;
    {
      ChanWalk4<T> w(N4);
#pragma unroll
      for (int i = 0; i < kC4; i++, w.next(N4)) {
        if (w.b < Bn) {
          const double d0 = (double)v4[i][0] - mu, d1 = (double)v4[i][1] - mu;
          const double d2 = (double)v4[i][2] - mu, d3 = (double)v4[i][3] - mu;
          s2 += (d0 * d0 + d1 * d1) + (d2 * d2 + d3 * d3);
        }
      }
    }
    const double var = block_sum<T>(s2, red) / (double)M;
    const float inv = (float)(1.0 / sqrt(var + (double)eps));
    if (threadIdx.x == 0) {
      mean[c] = (float)mu;
      invstd[c] = inv;
      if (rmean) rmean[c] = (1.0f - momentum) * rmean[c] + momentum * (float)mu;
      if (rvar) {
        const double unb = M > 1 ? var * (double)M / (double)(M - 1) : var;
        rvar[c] = (1.0f - momentum) * rvar[c] + momentum * (float)unb;
      }
    }
    const float fm = (float)mu, g = gamma[c], bt = beta[c];
    ChanWalk4<T> w(N4);
#pragma unroll
    for (int i = 0; i < kC4; i++, w.next(N4)) {
      if (w.b >= Bn) continue;
      f32x4 o;
#pragma unroll
      for (int k = 0; k < 4; k++) {
        o[k] = bn_apply(v4[i][k], fm, inv, g, bt);
        if (relu) o[k] = fmaxf(o[k], 0.0f);
      }
      if (!pool) {
        *reinterpret_cast<f32x4*>(z + w.off(C, N, c)) = o;
        continue;
      }
      // the float4's first maximum (the smallest point among equal values), one
      // LDS atomic per float4: (ordered value bits, ~point) keys
      unsigned long long best = 0ull;
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const unsigned u = __float_as_uint(o[k]);
        const unsigned key = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
        const unsigned long long kk = ((unsigned long long)key << 32) | (0xFFFFFFFFu - (unsigned)(4 * w.n4 + k));
        best = kk > best ? kk : best;
      }
      atomicMax(&pk[w.b], best);
    }
    if (!pool) return;
    __syncthreads();
    if (threadIdx.x < Bn) {
      const unsigned long long k = pk[threadIdx.x];
      const unsigned key = (unsigned)(k >> 32);
      const unsigned u = (key & 0x80000000u) ? (key & 0x7FFFFFFFu) : ~key;
      pool[(int64_t)threadIdx.x * C + c] = __uint_as_float(u);
      pool_idx[(int64_t)threadIdx.x * C + c] = (int)(0xFFFFFFFFu - (unsigned)(k & 0xFFFFFFFFu));
    }
    return;
  }
  float v[kCache];
  double s = 0.0;
  if (cached) {
    ChanWalk<T> w(N);
#pragma unroll
    for (int i = 0; i < kCache; i++, w.next(N)) {
      v[i] = w.b < Bn ? y[w.off(C, N, c)] : 0.0f;
      s += v[i];
    }
  } else {
    for (ChanWalk<T> w(N); w.b < Bn; w.next(N)) s += y[w.off(C, N, c)];
  }
  const double mu = block_sum<T>(s, red) / (double)M;
  double s2 = 0.0;
  if (cached) {
    ChanWalk<T> w(N);
#pragma unroll
    for (int i = 0; i < kCache; i++, w.next(N)) {
      const double d = (double)v[i] - mu;
      if (w.b < Bn) s2 += d * d;
    }
  } else {
    for (ChanWalk<T> w(N); w.b < Bn; w.next(N)) {
      const double d = (double)y[w.off(C, N, c)] - mu;
      s2 += d * d;
    }
  }
  const double var = block_sum<T>(s2, red) / (double)M;
  const float inv = (float)(1.0 / sqrt(var + (double)eps));
  if (threadIdx.x == 0) {
    mean[c] = (float)mu;
    invstd[c] = inv;
    if (rmean) rmean[c] = (1.0f - momentum) * rmean[c] + momentum * (float)mu;
    if (rvar) {
      const double unb = M > 1 ? var * (double)M / (double)(M - 1) : var;
      rvar[c] = (1.0f - momentum) * rvar[c] + momentum * (float)unb;
    }
  }
  const float fm = (float)mu, g = gamma[c], bt = beta[c];
  // pool mode: no z; this thread's running max per cloud (its elements visit the
  // clouds in order), merged into pk when the cloud changes.  (A wave-level
  // merge -- the leaving lanes' maxima reduced over the wave, one atomic --
  // measured slower: 39 -> 46 us per 1024-channel launch, r05o; the per-lane
  // atomics cost ~10 of the 39, NDNET_TR_EXP_NOPOOLATOMIC, r05n.)
  unsigned long long best = 0ull;
  int cur = -1;
  auto emit = [&](const ChanWalk<T>& w, float o) {
    if (!pool) {
      z[w.off(C, N, c)] = o;
      return;
    }
    if (w.b != cur) {
#ifndef NDNET_TR_EXP_NOPOOLATOMIC  // timing experiment only (wrong pooled values): no LDS atomics
      if (cur >= 0) atomicMax(&pk[cur], best);
#endif
      cur = w.b;
      best = 0ull;
    }
    const unsigned u = __float_as_uint(o);
    const unsigned key = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
    const unsigned long long k = ((unsigned long long)key << 32) | (0xFFFFFFFFu - (unsigned)w.n);
    best = k > best ? k : best;
  };
  if (cached) {
    ChanWalk<T> w(N);
#pragma unroll
    for (int i = 0; i < kCache; i++, w.next(N)) {
      if (w.b < Bn) {
        float o = bn_apply(v[i], fm, inv, g, bt);
        if (relu) o = fmaxf(o, 0.0f);
        emit(w, o);
      }
    }
  } else {
    for (ChanWalk<T> w(N); w.b < Bn; w.next(N)) {
      float o = bn_apply(y[w.off(C, N, c)], fm, inv, g, bt);
      if (relu) o = fmaxf(o, 0.0f);
      emit(w, o);
    }
  }
  if (!pool) return;
  if (cur >= 0) atomicMax(&pk[cur], best);
  __syncthreads();
  if (threadIdx.x < Bn) {
    const unsigned long long k = pk[threadIdx.x];
    const unsigned key = (unsigned)(k >> 32);
    const unsigned u = (key & 0x80000000u) ? (key & 0x7FFFFFFFu) : ~key;
    pool[(int64_t)threadIdx.x * C + c] = __uint_as_float(u);
    pool_idx[(int64_t)threadIdx.x * C + c] = (int)(0xFFFFFFFFu - (unsigned)(k & 0xFFFFFFFFu));
  }
}

template <int T>
__global__ __launch_bounds__(T) void k_tr_bn_bwd(const float* __restrict__ dz, const float* __restrict__ y,
                                                          const float* __restrict__ mean,
                                                          const float* __restrict__ invstd,
                                                          const float* __restrict__ gamma,
                                                          const float* __restrict__ beta, float* __restrict__ dy,
                                                          float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                          float* __restrict__ dbias, int Bn, int C, int N, int relu,
                                                          const int* __restrict__ pool_idx) {
  __shared__ double red[T / 64];
  constexpr int kCache = kBnValues / T;
  const int c = blockIdx.x;
  const int64_t M = (int64_t)Bn * N;
  const bool cached = M <= (int64_t)kBnValues;
  const float mu = mean[c], inv = invstd[c], gm = gamma[c], bt = beta[c];
  float gv[kCache], xv[kCache];
  double sg = 0.0, sgx = 0.0;
  // pool mode: the channel's per-cloud argmax and pooled gradient, staged once
  // (the element loop read both from global memory per element: three vector
  // loads per element instead of one)
  __shared__ int s_pidx[kPoolMaxB];
  __shared__ float s_pdz[kPoolMaxB];
  if (pool_idx) {
    if (threadIdx.x < Bn) {
      const int64_t bc = (int64_t)threadIdx.x * C + c;
      s_pidx[threadIdx.x] = pool_idx[bc];
      s_pdz[threadIdx.x] = dz[bc];
    }
    __syncthreads();
  }
  // g = dz where the forward's output was > 0 (ReLU), xhat = (y - mean) invstd;
  // pool mode: dz is [B][C], the gradient of the max over points, all of it at
  // the forward's first maximum
  if (cached && bn_vec_ok(N, y, dy) && (pool_idx || (((uintptr_t)dz) & 15u) == 0)) {
    constexpr int kC4 = kCache / 4;
    const int N4 = N / 4;
    f32x4 g4[kC4], x4[kC4];
    {
      ChanWalk4<T> w(N4);
#pragma unroll
      for (int i = 0; i < kC4; i++, w.next(N4)) {
        f32x4 yv = {0.f, 0.f, 0.f, 0.f}, gz = {0.f, 0.f, 0.f, 0.f};
        if (w.b < Bn) {
          const int64_t off = w.off(C, N, c);
          yv = *reinterpret_cast<const f32x4*>(y + off);
          if (!pool_idx) gz = *reinterpret_cast<const f32x4*>(dz + off);
        }
        x4[i] = yv;  // y for now: the loads of every step issued together
        g4[i] = gz;
      }
    }
    {
      ChanWalk4<T> w(N4);
#pragma unroll
      for (int i = 0; i < kC4; i++, w.next(N4)) {
        f32x4 g = g4[i], xh;
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const float yv = x4[i][k];
          if (pool_idx) g[k] = (w.b < Bn && 4 * w.n4 + k == s_pidx[w.b]) ? s_pdz[w.b] : 0.0f;
          if (relu && !(bn_apply(yv, mu, inv, gm, bt) > 0.0f)) g[k] = 0.0f;
          xh[k] = (yv - mu) * inv;
          if (w.b >= Bn) g[k] = xh[k] = 0.0f;
        }
        g4[i] = g;
        x4[i] = xh;
        sg += ((double)g[0] + (double)g[1]) + ((double)g[2] + (double)g[3]);
        sgx += ((double)g[0] * xh[0] + (double)g[1] * xh[1]) + ((double)g[2] * xh[2] + (double)g[3] * xh[3]);
      }
    }
    sg = block_sum<T>(sg, red);
    sgx = block_sum<T>(sgx, red);
    const float k1 = (float)(sg / (double)M), k2 = (float)(sgx / (double)M);
    const float scale = gm * inv;
    double sdy = 0.0;
    {
      ChanWalk4<T> w(N4);
#pragma unroll
      for (int i = 0; i < kC4; i++, w.next(N4)) {
        if (w.b >= Bn) continue;
        f32x4 d;
#pragma unroll
        for (int k = 0; k < 4; k++) d[k] = scale * (g4[i][k] - k1 - x4[i][k] * k2);
        *reinterpret_cast<f32x4*>(dy + w.off(C, N, c)) = d;
        sdy += ((double)d[0] + (double)d[1]) + ((double)d[2] + (double)d[3]);
      }
    }
    sdy = block_sum<T>(sdy, red);
    if (threadIdx.x == 0) {
      if (dgamma) dgamma[c] = (float)sgx;
      if (dbeta) dbeta[c] = (float)sg;
      if (dbias) dbias[c] = (float)sdy;
    }
    return;
  }
  auto grad_at = [&](const ChanWalk<T>& w, float& xh) {
    const int64_t off = w.off(C, N, c);
    const float yv = y[off];
    float g;
    if (pool_idx) {
      g = w.n == s_pidx[w.b] ? s_pdz[w.b] : 0.0f;
    } else {
      g = dz[off];
    }
    if (relu && !(bn_apply(yv, mu, inv, gm, bt) > 0.0f)) g = 0.0f;
    xh = (yv - mu) * inv;
    return g;
  };
  if (cached) {
    ChanWalk<T> w(N);
#pragma unroll
    for (int i = 0; i < kCache; i++, w.next(N)) {
      float g = 0.0f, xh = 0.0f;
      if (w.b < Bn) g = grad_at(w, xh);
      gv[i] = g;
      xv[i] = xh;
      sg += g;
      sgx += (double)g * xh;
    }
  } else {
    for (ChanWalk<T> w(N); w.b < Bn; w.next(N)) {
      float xh;
      const float g = grad_at(w, xh);
      sg += g;
      sgx += (double)g * xh;
    }
  }
  sg = block_sum<T>(sg, red);
  sgx = block_sum<T>(sgx, red);
  const float k1 = (float)(sg / (double)M), k2 = (float)(sgx / (double)M);
  const float scale = gm * inv;
  double sdy = 0.0;
  if (cached) {
    ChanWalk<T> w(N);
#pragma unroll
    for (int i = 0; i < kCache; i++, w.next(N)) {
      if (w.b < Bn) {
        const float d = scale * (gv[i] - k1 - xv[i] * k2);
        dy[w.off(C, N, c)] = d;
        sdy += d;
      }
    }
  } else {
    for (ChanWalk<T> w(N); w.b < Bn; w.next(N)) {
      const int64_t off = w.off(C, N, c);
      float xh;
      const float g = grad_at(w, xh);
      const float d = scale * (g - k1 - xh * k2);
      dy[off] = d;
      sdy += d;
    }
  }
  sdy = block_sum<T>(sdy, red);
  if (threadIdx.x == 0) {
    if (dgamma) dgamma[c] = (float)sgx;
    if (dbeta) dbeta[c] = (float)sg;
    if (dbias) dbias[c] = (float)sdy;
  }
}

__global__ __launch_bounds__(kBnThreads) void k_tr_chan_sum(const float* __restrict__ x, float* __restrict__ out,
                                                            int Bn, int C, int N) {
  __shared__ double red[kBnThreads / 64];
  const int c = blockIdx.x;
  double s = 0.0;
  for (ChanWalk<kBnThreads> w(N); w.b < Bn; w.next(N)) s += x[w.off(C, N, c)];
  s = block_sum<kBnThreads>(s, red);
  if (threadIdx.x == 0) out[c] = (float)s;
}

// out[r] = sum of the N contiguous values of row r: one wave per row, fixed order
__global__ __launch_bounds__(256) void k_tr_row_sum(const float* __restrict__ x, float* __restrict__ out, int64_t R,
                                                   int N) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= R) return;
  const float* row = x + r * N;
  double s = 0.0;
  for (int n = threadIdx.x & 63; n < N; n += 64) s += row[n];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if ((threadIdx.x & 63) == 0) out[r] = (float)s;
}

// first index of the row's maximum, NaN counting as the maximum (torch.argmax)
__device__ __forceinline__ int row_argmax(const float* __restrict__ r, int cols, int64_t stride = 1) {
  int bi = 0;
  float bv = r[0];
  for (int j = 1; j < cols; j++) {
    const float v = r[j * stride];
    if (!(bv != bv) && (v > bv || v != v)) {
      bv = v;
      bi = j;
    }
  }
  return bi;
}

// count[0] += rows whose argmax agrees (tools/train.py:84-87): a thread per row,
// a wave sum per wave, one integer atomic per wave (exact, so order-free)
__global__ __launch_bounds__(256) void k_tr_argmax_match(const float* __restrict__ pred, const float* __restrict__ gt,
                                                         int64_t rows, int cols, unsigned* __restrict__ count) {
  const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
  unsigned n = r < rows ? (row_argmax(pred + r * cols, cols) == row_argmax(gt + r * cols, cols)) : 0u;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) n += __shfl_xor(n, o);
  if ((threadIdx.x & 63) == 0 && n) atomicAdd(count, n);
}

// out[r] = first argmax of row r (NaN as the maximum): a thread per row
__global__ __launch_bounds__(256) void k_row_argmax(const float* __restrict__ x, int64_t rows, int cols,
                                                    int* __restrict__ out) {
  const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (r < rows) out[r] = row_argmax(x + r * cols, cols);
}

// The same for narrow rows (cols <= kArgmaxStagedCols), HBM-bound: a thread per
// row reading its own row strides 4 * cols bytes between lanes, so every load
// instruction touches 64 lines (the labelled path's [B * n][C + 1] one-hot
// classes: 185 MB per 16 x 100k batch took 0.58 ms).  Here the workgroup's 256
// rows -- one contiguous block -- are loaded as 16-byte vectors by consecutive
// lanes into LDS, then each thread scans its row there (an odd row pitch is
// bank-conflict free).
// The LDS is sized to the rows (dynamic: 256 * cols floats, 29.7 KB for the
// train step's 29 classes, five workgroups per CU) and each thread issues its
// share of the 16-byte loads together, so a CU keeps ~150 KB of the stream in
// flight (the static 48-column buffer held three workgroups: 52 us for the
// step's 186 MB, r05u).
constexpr int kArgmaxStagedCols = 48;
constexpr int kArgmaxLoads = 256 * kArgmaxStagedCols / 4 / 256;  // 16-byte loads per thread at most
__global__ __launch_bounds__(256) void k_row_argmax_staged(const float* __restrict__ x, int64_t rows, int cols,
                                                           int* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) float s[];
  const int64_t r0 = (int64_t)blockIdx.x * 256;
  const int nr = (int)min<int64_t>(256, rows - r0);
  const int count = nr * cols;
  const float* src = x + r0 * cols;
  if (((uintptr_t)src & 15) == 0) {
    const int n4 = count >> 2;
    const f32x4* s4 = reinterpret_cast<const f32x4*>(src);
    f32x4 v[kArgmaxLoads];
#pragma unroll
    for (int u = 0; u < kArgmaxLoads; u++) {
      const int i = u * 256 + threadIdx.x;
      if (i < n4) v[u] = __builtin_nontemporal_load(s4 + i);
    }
#pragma unroll
    for (int u = 0; u < kArgmaxLoads; u++) {
      const int i = u * 256 + threadIdx.x;
      if (i < n4) reinterpret_cast<f32x4*>(s)[i] = v[u];
    }
    for (int i = (n4 << 2) + threadIdx.x; i < count; i += 256) s[i] = src[i];
  } else {
    for (int i = threadIdx.x; i < count; i += 256) s[i] = src[i];
  }
  __syncthreads();
  if ((int)threadIdx.x < nr) out[r0 + threadIdx.x] = row_argmax(s + threadIdx.x * cols, cols);
}

// ---- TNet FC heads in train mode (ndtnet.py:53-60): Linear [+ BatchNorm1d
// over the batch + ReLU] on B <= 16 rows (one row per cloud) ----
//
// torch runs each head layer as a 16-row GEMM (hipBLASLt), then BatchNorm's
// batch statistics and ReLU as separate launches, and the same again
// backward.  Here a wave owns one output channel n: its lanes split K in
// float4 pieces with one partial sum per row (the weight row is read once for
// every row), a reduce-scatter over the lanes leaves row b's sum in lanes
// 4 b .. 4 b + 3, and BatchNorm's statistics over the B rows, the affine step
// and ReLU follow in the same wave -- one launch per layer forward.  Backward:
// one wave per channel for BatchNorm's backward, the bias / gamma / beta
// gradients and the weight-gradient row (dW[n] = sum_b dpre[b][n] x[b]); the
// input gradient by k-column blocks and N-splits summed in split order.
constexpr int kFcB = 16;  // rows (clouds) per launch at most

// sums of 16 per-row values over the wave's 64 lanes; lane L ends with row
// ((L >> 2) & 15)'s total (a reduce-scatter: 8 + 4 + 2 + 1 exchanges, then 2)
__device__ inline float fc_reduce16(float (&a)[kFcB], int lane) {
  float v8[8], v4[4], v2[2], v1;
#pragma unroll
  for (int i = 0; i < 8; i++) {  // xor 32: the low half keeps rows 0..7, the high half 8..15
    const bool hi = lane & 32;
    const float send = hi ? a[i] : a[8 + i], keep = hi ? a[8 + i] : a[i];
    v8[i] = keep + __shfl_xor(send, 32);
  }
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const bool hi = lane & 16;
    const float send = hi ? v8[i] : v8[4 + i], keep = hi ? v8[4 + i] : v8[i];
    v4[i] = keep + __shfl_xor(send, 16);
  }
#pragma unroll
  for (int i = 0; i < 2; i++) {
    const bool hi = lane & 8;
    const float send = hi ? v4[i] : v4[2 + i], keep = hi ? v4[2 + i] : v4[i];
    v2[i] = keep + __shfl_xor(send, 8);
  }
  {
    const bool hi = lane & 4;
    const float send = hi ? v2[0] : v2[1], keep = hi ? v2[1] : v2[0];
    v1 = keep + __shfl_xor(send, 4);
  }
  v1 += __shfl_xor(v1, 2);
  v1 += __shfl_xor(v1, 1);
  return v1;
}

__device__ inline double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// y[b][n] = x[b] . W[n] + bias[n] (+1 on the diagonal of an eye x eye transform:
// TNet's fc3 + identity, ndtnet.py:59, added after the bias as torch does);
// gamma != null: z = relu?(BatchNorm1d(y)) with batch statistics over the B
// rows (double sums, biased variance; running stats with the unbiased one).
constexpr int kFcWaves = 8;           // channels in flight per workgroup (a wave each)
constexpr int kFcMaxLds = 64 * 1024;  // the staged input rows: B x K floats

// The workgroup's input rows x [B][K] staged in LDS with float4 loads (one
// memory latency), then each wave's weight row loaded whole (<= 4 float4 per
// lane, issued together) -- round 5: a wave reading its own copy of x from L2
// K / 256 times in sequence took 12.7 us per launch (r05k trace).
__device__ inline void fc_stage_x(f32x4* s_x, const float* __restrict__ x, int Bn, int K4) {
  const f32x4* xv = reinterpret_cast<const f32x4*>(x);
  for (int e = threadIdx.x; e < Bn * K4; e += kFcWaves * 64) s_x[e] = xv[e];
  __syncthreads();
}

__global__ __launch_bounds__(kFcWaves * 64) void k_tr_fc_fwd(const float* __restrict__ x, const float* __restrict__ W,
                                                   const float* __restrict__ bias, float* __restrict__ y,
                                                   float* __restrict__ z, float* __restrict__ mean,
                                                   float* __restrict__ invstd, float* __restrict__ rmean,
                                                   float* __restrict__ rvar, const float* __restrict__ gamma,
                                                   const float* __restrict__ beta, int Bn, int K, int N, float eps,
                                                   float momentum, int relu, int eye,
                                                   long long* __restrict__ batches_tracked, int64_t ldw) {
  extern __shared__ f32x4 s_x[];  // [Bn][K / 4]
  const int lane = threadIdx.x & 63;
  const int K4 = K / 4;
  if (batches_tracked && blockIdx.x == 0 && threadIdx.x == 0) batches_tracked[0] += 1;
  fc_stage_x(s_x, x, Bn, K4);
  for (int n = blockIdx.x * kFcWaves + (threadIdx.x >> 6); n < N; n += gridDim.x * kFcWaves) {
    const f32x4* w = reinterpret_cast<const f32x4*>(W + (int64_t)n * ldw);
    float acc[kFcB];
#pragma unroll
    for (int b = 0; b < kFcB; b++) acc[b] = 0.0f;
    for (int f0 = 0; f0 < K4; f0 += 256) {  // (one round for K <= 1024)
      f32x4 wv[4];
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const int f = f0 + lane + 64 * i;
        if (f < K4) wv[i] = w[f];
      }
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const int f = f0 + lane + 64 * i;
        if (f >= K4) break;
#pragma unroll
        for (int b = 0; b < kFcB; b++) {
          const f32x4 xv = s_x[(b < Bn ? b : 0) * K4 + f];
          const f32x4 pr = xv * wv[i];
          acc[b] += (pr[0] + pr[1]) + (pr[2] + pr[3]);
        }
      }
    }
    const int row = (lane >> 2) & 15;  // the row this lane holds after the reduction
    float v = fc_reduce16(acc, lane) + bias[n];
    if (eye > 0 && n < eye * eye && n % (eye + 1) == 0) v += 1.0f;
    const bool mine = (lane & 3) == 0 && row < Bn;
    if (!gamma) {
      if (mine) z[(int64_t)row * N + n] = v;
      continue;
    }
    const double mu = wave_sum_d(mine ? (double)v : 0.0) / (double)Bn;
    const double dv = (double)v - mu;
    const double var = wave_sum_d(mine ? dv * dv : 0.0) / (double)Bn;
    const float inv = (float)(1.0 / sqrt(var + (double)eps));
    const float fm = (float)mu;
    if (lane == 0) {
      mean[n] = fm;
      invstd[n] = inv;
      if (rmean) rmean[n] = (1.0f - momentum) * rmean[n] + momentum * fm;
      if (rvar) {
        const double unb = Bn > 1 ? var * (double)Bn / (double)(Bn - 1) : var;
        rvar[n] = (1.0f - momentum) * rvar[n] + momentum * (float)unb;
      }
    }
    float o = bn_apply(v, fm, inv, gamma[n], beta[n]);
    if (relu) o = fmaxf(o, 0.0f);
    if (mine) {
      y[(int64_t)row * N + n] = v;
      z[(int64_t)row * N + n] = o;
    }
  }
}

// Backward through BatchNorm (+ ReLU mask) of channel n and its weight row:
// dpre[b][n] (the gradient of y), db[n] = sum_b dpre, dgamma / dbeta, and
// dW[n][k] = sum_b dpre[b][n] x[b][k] in row order.  gamma == null: dpre = dz.
__global__ __launch_bounds__(kFcWaves * 64) void k_tr_fc_bwd_w(const float* __restrict__ dz, const float* __restrict__ x,
                                                     const float* __restrict__ y, const float* __restrict__ mean,
                                                     const float* __restrict__ invstd,
                                                     const float* __restrict__ gamma, const float* __restrict__ beta,
                                                     float* __restrict__ dpre, float* __restrict__ dW,
                                                     float* __restrict__ db, float* __restrict__ dgamma,
                                                     float* __restrict__ dbeta, int Bn, int K, int N, int relu,
                                                     int64_t ldw) {
  extern __shared__ f32x4 s_x[];  // [Bn][K / 4] (dW only)
  const int lane = threadIdx.x & 63;
  const int K4 = K / 4;
  if (dW) fc_stage_x(s_x, x, Bn, K4);
  for (int n = blockIdx.x * kFcWaves + (threadIdx.x >> 6); n < N; n += gridDim.x * kFcWaves) {
    const bool mine = lane < Bn;  // lane b: row b
    float d = 0.0f;
    if (!gamma) {
      d = mine ? dz[(int64_t)lane * N + n] : 0.0f;
    } else {
      const float mu = mean[n], inv = invstd[n], gm = gamma[n], bt = beta[n];
      float g = 0.0f, xh = 0.0f;
      if (mine) {
        const float yv = y[(int64_t)lane * N + n];
        g = dz[(int64_t)lane * N + n];
        if (relu && !(bn_apply(yv, mu, inv, gm, bt) > 0.0f)) g = 0.0f;
        xh = (yv - mu) * inv;
      }
      const double sg = wave_sum_d(g), sgx = wave_sum_d((double)g * xh);
      const float k1 = (float)(sg / (double)Bn), k2 = (float)(sgx / (double)Bn);
      if (mine) d = gm * inv * (g - k1 - xh * k2);
      if (lane == 0) {
        if (dgamma) dgamma[n] = (float)sgx;
        if (dbeta) dbeta[n] = (float)sg;
      }
    }
    const double sd = wave_sum_d(d);
    if (lane == 0 && db) db[n] = (float)sd;
    if (mine && dpre) dpre[(int64_t)lane * N + n] = d;
    if (!dW) continue;
    float dv[kFcB];
#pragma unroll
    for (int b = 0; b < kFcB; b++) dv[b] = __shfl(d, b);  // 0 past the rows
    f32x4* wrow = reinterpret_cast<f32x4*>(dW + (int64_t)n * ldw);
    for (int f = lane; f < K4; f += 64) {
      f32x4 sacc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int b = 0; b < kFcB; b++)
        if (b < Bn) sacc = sacc + s_x[b * K4 + f] * dv[b];
      wrow[f] = sacc;
    }
  }
}

// dx[b][k] = sum_n dpre[b][n] W[n][k]: workgroup (k block of 256 columns, N
// split s); part[s][b][k] (or dx itself with one split), summed in split order.
constexpr int kFcXMaxN = 256;  // channels of a split staged in LDS
__global__ __launch_bounds__(256) void k_tr_fc_bwd_x(const float* __restrict__ dpre, const float* __restrict__ W,
                                                     float* __restrict__ out, int Bn, int K, int N, int nsplit,
                                                     int64_t ldw) {
  __shared__ float s_d[kFcXMaxN][kFcB];
  const int s = blockIdx.y;
  const int n0 = (int)((int64_t)N * s / nsplit), n1 = (int)((int64_t)N * (s + 1) / nsplit);
  for (int e = threadIdx.x; e < (n1 - n0) * kFcB; e += 256) {
    const int nn = e / kFcB, b = e % kFcB;
    s_d[nn][b] = b < Bn ? dpre[(int64_t)b * N + n0 + nn] : 0.0f;
  }
  __syncthreads();
  const int k = blockIdx.x * 256 + threadIdx.x;
  if (k >= K) return;
  float acc[kFcB];
#pragma unroll
  for (int b = 0; b < kFcB; b++) acc[b] = 0.0f;
  int nn = n0;
  for (; nn + 8 <= n1; nn += 8) {  // 8 weight loads in flight, summed in channel order
    float wv[8];
#pragma unroll
    for (int j = 0; j < 8; j++) wv[j] = W[(int64_t)(nn + j) * ldw + k];
#pragma unroll
    for (int j = 0; j < 8; j++)
#pragma unroll
      for (int b = 0; b < kFcB; b++) acc[b] = fmaf(s_d[nn + j - n0][b], wv[j], acc[b]);
  }
  for (; nn < n1; nn++) {
    const float wv = W[(int64_t)nn * ldw + k];
#pragma unroll
    for (int b = 0; b < kFcB; b++) acc[b] = fmaf(s_d[nn - n0][b], wv, acc[b]);
  }
  float* o = out + (int64_t)s * Bn * K;
#pragma unroll
  for (int b = 0; b < kFcB; b++)
    if (b < Bn) o[(int64_t)b * K + k] = acc[b];
}

// ---- the seg head's log_softmax over the class dim (ndtnet.py:241) and the
// training loss (NLL of the one-hot target, ndnet.training.segmentation_loss)
// ----
//
// torch runs log_softmax(dim=1) on [B][C][N] as cunn_SpatialSoftMax (~20 us
// each way at 16 x 29 x 1000) and the loss as ~8 small elementwise / reduce
// launches (r05l trace).  Here one thread per point (b, n) holds its C <=
// kLsmC classes in registers (stride-N loads: consecutive threads read
// consecutive addresses; all of them issued at once -- a loop over C with a
// load per step waited once per class: 18 us, r05o).
constexpr int kLsmC = 32;
// 64-thread workgroups: the B N = 16000 points then spread over ~250 CUs
// (256-thread groups left them on 63 CUs, each waiting on its loads)
constexpr int kLsmT = 64;

__global__ __launch_bounds__(kLsmT) void k_tr_log_softmax_c(const float* __restrict__ x, float* __restrict__ out,
                                                            int Bn, int C, int N) {
  const int64_t t = (int64_t)blockIdx.x * kLsmT + threadIdx.x;
  if (t >= (int64_t)Bn * N) return;
  const int64_t base = t / N * C * N + t % N;
  float v[kLsmC];
#pragma unroll
  for (int c = 0; c < kLsmC; c++) v[c] = c < C ? x[base + (int64_t)c * N] : -__builtin_huge_valf();
  float mx = v[0];
#pragma unroll
  for (int c = 1; c < kLsmC; c++) mx = fmaxf(mx, v[c]);
  float sum = 0.0f;
#pragma unroll
  for (int c = 0; c < kLsmC; c++)
    if (c < C) sum += expf(v[c] - mx);
  const float lse = logf(sum);
#pragma unroll
  for (int c = 0; c < kLsmC; c++)
    if (c < C) out[base + (int64_t)c * N] = (v[c] - mx) - lse;
}

// dx[c] = dy[c] - exp(y[c]) * sum_c' dy[c'] (y the forward's log-probs)
__global__ __launch_bounds__(kLsmT) void k_tr_log_softmax_c_bwd(const float* __restrict__ y,
                                                                const float* __restrict__ dy, float* __restrict__ dx,
                                                                int Bn, int C, int N) {
  const int64_t t = (int64_t)blockIdx.x * kLsmT + threadIdx.x;
  if (t >= (int64_t)Bn * N) return;
  const int64_t base = t / N * C * N + t % N;
  float d[kLsmC], yv[kLsmC];
#pragma unroll
  for (int c = 0; c < kLsmC; c++) {
    d[c] = c < C ? dy[base + (int64_t)c * N] : 0.0f;
    yv[c] = c < C ? y[base + (int64_t)c * N] : 0.0f;
  }
  float s = 0.0f;
#pragma unroll
  for (int c = 0; c < kLsmC; c++) s += d[c];
#pragma unroll
  for (int c = 0; c < kLsmC; c++)
    if (c < C) dx[base + (int64_t)c * N] = d[c] - expf(yv[c]) * s;
}

// the workgroup's gt rows [t0, t0 + kLsmT) x C, staged in LDS with coalesced
// loads (a thread reading its own 116-byte row sent every load instruction to
// 64 lines); row pitch C (odd at C = 29: conflict-free reads)
__device__ inline const float* nll_stage_gt(float* s_gt, const float* __restrict__ gt, int64_t pts, int C) {
  const int64_t t0 = (int64_t)blockIdx.x * kLsmT;
  const int64_t n = (pts - t0 < kLsmT ? pts - t0 : kLsmT) * C;
  const float* src = gt + t0 * C;
  for (int64_t i = threadIdx.x; i < n; i += kLsmT) s_gt[i] = src[i];
  __syncthreads();
  return s_gt + threadIdx.x * C;
}

// Per-workgroup partial of sum_{b,n,c} gt[b][n][c] * logp[b][c][n] (gt
// [B][N][C] one-hot rows, logp the log-softmax output [B][C][N]); a point
// per thread, then the workgroup's sum in a fixed order.
__global__ __launch_bounds__(kLsmT) void k_tr_nll_part(const float* __restrict__ logp, const float* __restrict__ gt,
                                                       double* __restrict__ part, int Bn, int C, int N) {
  __shared__ float s_gt[kLsmT * kLsmC];
  const int64_t pts = (int64_t)Bn * N;
  const int64_t t = (int64_t)blockIdx.x * kLsmT + threadIdx.x;
  // this point's log-probs first, in flight with the gt stage's loads
  const int64_t tc = t < pts ? t : pts - 1;
  const int64_t base = tc / N * C * N + tc % N;
  float lp[kLsmC];
#pragma unroll
  for (int c = 0; c < kLsmC; c++) lp[c] = c < C ? logp[base + (int64_t)c * N] : 0.0f;
  const float* g = nll_stage_gt(s_gt, gt, pts, C);
  double v = 0.0;
  if (t < pts) {
    float a = 0.0f;
#pragma unroll
    for (int c = 0; c < kLsmC; c++)
      if (c < C) a += g[c] * lp[c];
    v = a;
  }
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  if (threadIdx.x == 0) part[blockIdx.x] = v;
}

// loss = -(sum of the parts in order) / (B N)
__global__ __launch_bounds__(64) void k_tr_nll_sum(const double* __restrict__ part, int nparts, float* __restrict__ loss,
                                                   int64_t count) {
  double s = 0.0;
  for (int i = threadIdx.x; i < nparts; i += 64) s += part[i];
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if (threadIdx.x == 0) loss[0] = (float)(-s / (double)count);
}

// dlogp[b][c][n] = -gt[b][n][c] * dloss / (B N)
__global__ __launch_bounds__(kLsmT) void k_tr_nll_bwd(const float* __restrict__ gt, const float* __restrict__ dloss,
                                                      float* __restrict__ dlogp, int Bn, int C, int N) {
  __shared__ float s_gt[kLsmT * kLsmC];
  const int64_t pts = (int64_t)Bn * N;
  const float* g = nll_stage_gt(s_gt, gt, pts, C);
  const int64_t t = (int64_t)blockIdx.x * kLsmT + threadIdx.x;
  if (t >= pts) return;
  const int64_t base = t / N * C * N + t % N;
  const float s = -dloss[0] / (float)pts;
#pragma unroll
  for (int c = 0; c < kLsmC; c++)
    if (c < C) dlogp[base + (int64_t)c * N] = g[c] * s;
}

// The training step's accuracy (tools/train.py:84-87) on pred channel-major
// [B][C][N] (the seg head's log-probs before their transposed view) and the
// one-hot gt [B][N][C]: a point per thread with its <= kLsmC classes loaded
// together (N apart, coalesced across the wave), gt staged in LDS as the loss
// kernels do; first argmax with NaN as the maximum (torch.argmax).  The
// matches go to ctr[0]; the last workgroup (ticket ctr[1]) writes acc =
// ctr[0] / rows -- the caller zeroes ctr[0..1], no count-to-float launches.
__global__ __launch_bounds__(kLsmT) void k_tr_argmax_match_cm(const float* __restrict__ pred,
                                                              const float* __restrict__ gt, int Bn, int C, int N,
                                                              unsigned* __restrict__ ctr, float* __restrict__ acc) {
  __shared__ float s_gt[kLsmT * kLsmC];
  const int64_t pts = (int64_t)Bn * N;
  const int64_t t = (int64_t)blockIdx.x * kLsmT + threadIdx.x;
  const int64_t tc = t < pts ? t : pts - 1;
  const int64_t base = tc / N * C * N + tc % N;
  float v[kLsmC];
#pragma unroll
  for (int c = 0; c < kLsmC; c++) v[c] = c < C ? pred[base + (int64_t)c * N] : 0.0f;
  const float* g = nll_stage_gt(s_gt, gt, pts, C);
  int bi = 0, gi = 0;
  float bv = v[0], gv = g[0];
#pragma unroll
  for (int c = 1; c < kLsmC; c++) {
    if (c < C) {
      if (!(bv != bv) && (v[c] > bv || v[c] != v[c])) {
        bv = v[c];
        bi = c;
      }
      const float x = g[c];
      if (!(gv != gv) && (x > gv || x != x)) {
        gv = x;
        gi = c;
      }
    }
  }
  unsigned n = t < pts && bi == gi ? 1u : 0u;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) n += __shfl_xor(n, o);
  if (threadIdx.x == 0) {
    if (n) __hip_atomic_fetch_add(&ctr[0], n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the count has been added before the ticket
    if (__hip_atomic_fetch_add(&ctr[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1 && acc)
      acc[0] = (float)__hip_atomic_load(&ctr[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) / (float)pts;
  }
}

// ---- the point transform t1 (reference ndtnet.py:141-147: t . p and
// t . C, left product only) of the train forward ----
//
// x[b, i, n] = sum_j t[b,i,j] p[b,n,j] and x[b, 3 + 3 i + k, n] = sum_j
// t[b,i,j] C[b,n,j,k], x [B,12,N] channel-major as the first conv reads it:
// one thread per point (the torch composition: two cats, a permute and a
// batched GEMM).  Backward to t only (the points and covariances are data):
// dt[b,i,j] = sum_n dx[b,i,n] p[n,j] + sum_{n,k} dx[b,3+3i+k,n] C[n,j,k], one
// workgroup per cloud.
constexpr int kPtT = 256;
constexpr int kPtBwdT = 1024;
__global__ __launch_bounds__(kPtT) void k_tr_point_transform(const float* __restrict__ t,
                                                             const float* __restrict__ pts, int pld,
                                                             const float* __restrict__ extra, int eld,
                                                             float* __restrict__ x, int N) {
  const int b = blockIdx.y;
  const int n = blockIdx.x * kPtT + threadIdx.x;
  if (n >= N) return;
  float tm[9], p[3], c[9];
#pragma unroll
  for (int q = 0; q < 9; q++) tm[q] = t[9 * b + q];
  const float* pp = pts + pld * ((int64_t)b * N + n);
  const float* cc = extra + eld * ((int64_t)b * N + n);
#pragma unroll
  for (int q = 0; q < 3; q++) p[q] = pp[q];
#pragma unroll
  for (int q = 0; q < 9; q++) c[q] = cc[q];
  float* xo = x + (int64_t)b * 12 * N + n;
#pragma unroll
  for (int i = 0; i < 3; i++) {
    xo[(int64_t)i * N] = fmaf(tm[3 * i + 2], p[2], fmaf(tm[3 * i + 1], p[1], tm[3 * i] * p[0]));
#pragma unroll
    for (int kk = 0; kk < 3; kk++)
      xo[(int64_t)(3 + 3 * i + kk) * N] =
          fmaf(tm[3 * i + 2], c[6 + kk], fmaf(tm[3 * i + 1], c[3 + kk], tm[3 * i] * c[kk]));
  }
}

__global__ __launch_bounds__(kPtBwdT) void k_tr_point_transform_bwd(const float* __restrict__ dx,
                                                                    const float* __restrict__ pts, int pld,
                                                                    const float* __restrict__ extra, int eld,
                                                                    float* __restrict__ dt, int N) {
  const int b = blockIdx.x;
  float acc[9];
#pragma unroll
  for (int q = 0; q < 9; q++) acc[q] = 0.f;
  const float* d = dx + (int64_t)b * 12 * N;
  for (int n = threadIdx.x; n < N; n += kPtBwdT) {
    float p[3], c[9], g[12];
    const float* pp = pts + pld * ((int64_t)b * N + n);
    const float* cc = extra + eld * ((int64_t)b * N + n);
#pragma unroll
    for (int q = 0; q < 3; q++) p[q] = pp[q];
#pragma unroll
    for (int q = 0; q < 9; q++) c[q] = cc[q];
#pragma unroll
    for (int r = 0; r < 12; r++) g[r] = d[(int64_t)r * N + n];
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
      for (int j = 0; j < 3; j++) {
        float a = g[i] * p[j];
#pragma unroll
        for (int kk = 0; kk < 3; kk++) a = fmaf(g[3 + 3 * i + kk], c[3 * j + kk], a);
        acc[3 * i + j] += a;
      }
  }
  __shared__ float s_red[kPtBwdT / 64][9];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int q = 0; q < 9; q++) {
    float v = acc[q];
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if (lane == 0) s_red[w][q] = v;
  }
  __syncthreads();
  if (threadIdx.x < 9) {
    float v = 0.f;
    for (int i = 0; i < kPtBwdT / 64; i++) v += s_red[i][threadIdx.x];
    dt[9 * b + threadIdx.x] = v;
  }
}

// ---- Adam (torch.optim.Adam's fused, capturable form; tools/train.py's
// optimizer) over up to kAdamMax tensors per launch, the tensors' pointers in
// the kernel arguments (captured by value into a graph: no pointer table to
// upload) ----
//
// torch's fused Adam ran as two multi_tensor_apply launches of ~46 us each on
// the 3.37 M parameters (94 MB of state traffic: ~15 us at HBM speed, r05p).
// Per element, torch's order of operations (ATen fused_adam_utils,
// ADAM_MODE::ORIGINAL): m = b1 m + (1 - b1) g; v = b2 v + (1 - b2) g^2;
// p -= (lr / (1 - b1^t)) m / (sqrt(v) / sqrt(1 - b2^t) + eps), t the step
// after its increment (k_tr_adam_steps runs first).
constexpr int kAdamMax = 32;
constexpr int kAdamChunk = 4096;  // elements per workgroup (256 threads x 16)
struct AdamArgs {
  float* p[kAdamMax];
  const float* g[kAdamMax];
  float* m[kAdamMax];
  float* v[kAdamMax];
  const float* step[kAdamMax];
  int64_t numel[kAdamMax];
  int chunk0[kAdamMax + 1];  // first chunk of each tensor; chunk0[n] = total
  int n;
  float beta1, beta2, omb1, omb2, eps, wd;  // omb = 1 - beta, rounded from double (as torch passes it)
  double beta1d, beta2d;                    // the bias corrections' powers, in double as torch's kernel
  const float* lr;
};

constexpr int kAdamStepsMax = 128;
struct AdamSteps {
  float* s[kAdamStepsMax];
  int n;
};
__global__ __launch_bounds__(64) void k_tr_adam_steps(AdamSteps S) {
  for (int i = threadIdx.x; i < S.n; i += 64) S.s[i][0] += 1.0f;
}

__global__ __launch_bounds__(256) void k_tr_adam(AdamArgs A) {
  const int chunk = blockIdx.x;
  int ti = 0;
  while (ti + 1 < A.n && A.chunk0[ti + 1] <= chunk) ti++;
  const int64_t e0 = (int64_t)(chunk - A.chunk0[ti]) * kAdamChunk;
  const int64_t ne = A.numel[ti];
  const float t = A.step[ti][0];
  const float lr = A.lr[0];
  const float bc1 = (float)(1.0 - pow(A.beta1d, (double)t)), bc2 = (float)(1.0 - pow(A.beta2d, (double)t));
  const float step_size = lr / bc1, bc2s = sqrtf(bc2);
  float* __restrict__ p = A.p[ti];
  const float* __restrict__ g = A.g[ti];
  float* __restrict__ m = A.m[ti];
  float* __restrict__ v = A.v[ti];
  // four elements per thread at a time, their 16 loads issued together
  // (clamped indices; the stores past the tensor are skipped)
#pragma unroll
  for (int k0 = 0; k0 < kAdamChunk / 256; k0 += 4) {
    float gv[4], pv[4], mv[4], vv[4];
    int64_t ix[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      ix[u] = e0 + (int64_t)(k0 + u) * 256 + threadIdx.x;
      const int64_t ic = ix[u] < ne ? ix[u] : ne - 1;
      gv[u] = g[ic];
      pv[u] = p[ic];
      mv[u] = m[ic];
      vv[u] = v[ic];
    }
#pragma unroll
    for (int u = 0; u < 4; u++) {
      float gi = gv[u];
      if (A.wd != 0.0f) gi = gi + pv[u] * A.wd;
      const float mi = A.beta1 * mv[u] + A.omb1 * gi;
      const float vi = A.beta2 * vv[u] + A.omb2 * gi * gi;
      const float denom = sqrtf(vi) / bc2s + A.eps;
      if (ix[u] < ne) {
        m[ix[u]] = mi;
        v[ix[u]] = vi;
        p[ix[u]] = pv[u] - step_size * mi / denom;
      }
    }
  }
}

int launched() { return hipGetLastError() == hipSuccess ? 0 : -21; }

bool getenv_flag(const char* name) {
  const char* v = getenv(name);
  return v && v[0] == '1';
}
// A/B switch NDNET_TR_GEMM64=1 (64 x 64 tiles only), read once: the
// process's tile choice is fixed at the first launch: a graph captured
// before the variable changed and an eager step after it use the same
// summation order
bool gemm64_only() {
  static const bool v = getenv_flag("NDNET_TR_GEMM64");
  return v;
}
// 128 x 128 tiles when they still give this many workgroups (NDNET_TR_WIDE_MIN, A/B)
int64_t wide_min_wgs() {
  static const int64_t v = [] {
    const char* e = getenv("NDNET_TR_WIDE_MIN");
    return e ? (int64_t)atoll(e) : (int64_t)512;
  }();
  return v;
}
// k per LDS step of the fp32 train GEMM: 32 (default; the same sums in the
// same order as 16, half the barriers, twice the LDS: graphed step 2.893 ->
// 2.849 ms, the 128 x 1024 layers' input gradients 61.8 -> 54.5 us,
// profiles/r04_train_x6.txt) or NDNET_TR_KT=16
bool gemm_k32() {
  static const bool v = [] {
    const char* e = getenv("NDNET_TR_KT");
    return !(e && e[0] == '1');
  }();
  return v;
}
// Which train GEMMs run split-bf16 (k_tr_gemm_x6), NDNET_TR_X6, read once
// (it sets the process's summation orders): "dw" (default) the weight
// gradients (both operands k-major: 54 vs 64 us on the 1024 x 128 layers,
// -70 us a step), "all" every GEMM (the forward and input-gradient shapes
// measured slower than the fp32 kernel's 128 x 128 tiles), "0" none
// (profiles/r04_train_x6.txt).
bool gemm_x6(bool a_kmajor, bool b_kmajor) {
  static const int mode = [] {
    const char* e = getenv("NDNET_TR_X6");
    if (!e) return 1;
    if (e[0] == '0') return 0;
    return (e[0] == 'a' || e[0] == '1') ? 2 : 1;
  }();
  return mode == 2 || (mode == 1 && a_kmajor && b_kmajor);
}
// BatchNorm kernels on 1024-thread workgroups for layers of < 512 channels
// (one workgroup per channel: the narrow layers leave most CUs idle at 512
// threads): graphed step 3.021 -> 2.968 ms (profiles/r04_train_hip.txt).
// NDNET_TR_BN1024=0 keeps 512 threads (read once like NDNET_TR_GEMM64: the
// workgroup size sets the statistics' summation order).
bool bn_wide_groups(int C) {
  static const int v = [] {  // 0: never, 1: C < 512 (default), 2: every layer (A/B)
    const char* e = getenv("NDNET_TR_BN1024");
    return e ? (e[0] == '0' ? 0 : e[0] == '2' ? 2 : 1) : 1;
  }();
  return v == 2 || (v == 1 && C < 512);
}

}  // namespace

extern "C" int ndnet_tr_gemm(const float* A, const float* B, float* C, const float* bias, int64_t sbias, int M,
                             int N, int K, int64_t lda, int64_t ldb, int64_t ldc, int64_t sAz, int64_t sBz,
                             int64_t sCz, int batch, int clouds_per_part, int a_kmajor, int b_kmajor, int nchunks,
                             int kchunk, void* stream) {
  if (!A || !B || !C || M <= 0 || N <= 0 || K <= 0 || batch <= 0 || nchunks <= 0 || kchunk <= 0) return -20;
  if (clouds_per_part <= 0 || clouds_per_part > batch) return -20;
  if (lda <= 0 || ldb <= 0 || ldc < N || sAz < 0 || sBz < 0 || sCz < 0 || sbias < 0) return -20;
  if ((int64_t)(nchunks - 1) * kchunk >= K) return -20;  // every chunk starts inside K
  if ((int64_t)nchunks * kchunk < K) return -20;         // and together they cover it
  if ((nchunks > 1 || clouds_per_part > 1) && bias) return -20;  // a bias belongs to one partial only
  const int64_t parts = (batch + clouds_per_part - 1) / clouds_per_part;
  const int64_t gz = parts * nchunks, gy = (M + kTM - 1) / kTM, gx = (N + kTN - 1) / kTN;
  if (gz > 65535 || gy > 65535 || gx > (int64_t)INT32_MAX) return -20;
  // 128 x 128 tiles where they still give the chip >= 512 workgroups
  const int64_t big = ((M + 127) / 128) * ((N + 127) / 128) * gz;
  const bool wide = M >= 128 && N >= 128 && big >= wide_min_wgs() && !gemm64_only();
  const dim3 grid(wide ? (unsigned)((N + 127) / 128) : (unsigned)gx, wide ? (unsigned)((M + 127) / 128) : (unsigned)gy,
                  (unsigned)gz);
  hipStream_t st = (hipStream_t)stream;
#define NDNET_TR_GEMM(AKV, BKV)                                                                                    \
  do {                                                                                                             \
    if (wide && k32)                                                                                               \
      k_tr_gemm<128, AKV, BKV, 32><<<grid, 512, 0, st>>>(A, B, C, bias, sbias, M, N, K, lda, ldb, ldc, sAz, sBz,     \
                                                         sCz, batch, clouds_per_part, nchunks, kchunk);            \
    else if (wide)                                                                                                 \
      k_tr_gemm<128, AKV, BKV><<<grid, 512, 0, st>>>(A, B, C, bias, sbias, M, N, K, lda, ldb, ldc, sAz, sBz, sCz,    \
                                                     batch, clouds_per_part, nchunks, kchunk);                     \
    else if (k32)                                                                                                  \
      k_tr_gemm<64, AKV, BKV, 32><<<grid, 256, 0, st>>>(A, B, C, bias, sbias, M, N, K, lda, ldb, ldc, sAz, sBz, sCz, \
                                                        batch, clouds_per_part, nchunks, kchunk);                  \
    else                                                                                                           \
      k_tr_gemm<64, AKV, BKV><<<grid, 256, 0, st>>>(A, B, C, bias, sbias, M, N, K, lda, ldb, ldc, sAz, sBz, sCz,     \
                                                    batch, clouds_per_part, nchunks, kchunk);                      \
  } while (0)
  const bool k32 = gemm_k32();
  if (gemm_x6(a_kmajor != 0, b_kmajor != 0)) {  // 64 x 64 tiles only
    const dim3 g6((unsigned)gx, (unsigned)gy, (unsigned)gz);
#define NDNET_TR_GEMM6(AKV, BKV)                                                                                   \
  k_tr_gemm_x6<AKV, BKV><<<g6, 256, 0, st>>>(A, B, C, bias, sbias, M, N, K, lda, ldb, ldc, sAz, sBz, sCz, batch,     \
                                           clouds_per_part, nchunks, kchunk)
    if (a_kmajor) {
      if (b_kmajor) NDNET_TR_GEMM6(true, true); else NDNET_TR_GEMM6(true, false);
    } else {
      if (b_kmajor) NDNET_TR_GEMM6(false, true); else NDNET_TR_GEMM6(false, false);
    }
#undef NDNET_TR_GEMM6
    return launched();
  }
  if (a_kmajor) {
    if (b_kmajor) NDNET_TR_GEMM(true, true); else NDNET_TR_GEMM(true, false);
  } else {
    if (b_kmajor) NDNET_TR_GEMM(false, true); else NDNET_TR_GEMM(false, false);
  }
#undef NDNET_TR_GEMM
  return launched();
}

extern "C" int ndnet_tr_sum_parts(const float* part, float* out, int64_t count, int nparts, void* stream) {
  if (!part || !out || count <= 0 || nparts <= 0) return -20;
  const int64_t blocks = (count + 255) / 256;
  if (blocks > (int64_t)INT32_MAX) return -20;
  k_tr_sum_parts<<<(unsigned)blocks, 256, 0, (hipStream_t)stream>>>(part, out, count, nparts, count, count);
  return launched();
}

extern "C" int ndnet_tr_sum_parts_2d(const float* part, float* out, int64_t rows, int64_t cols, int64_t ldo,
                                     int nparts, void* stream) {
  if (!part || !out || rows <= 0 || cols <= 0 || ldo < cols || nparts <= 0) return -20;
  const int64_t count = rows * cols, blocks = (count + 255) / 256;
  if (blocks > (int64_t)INT32_MAX) return -20;
  k_tr_sum_parts<<<(unsigned)blocks, 256, 0, (hipStream_t)stream>>>(part, out, count, nparts, cols, ldo);
  return launched();
}

extern "C" int ndnet_tr_bn_fwd(const float* y, float* z, float* mean, float* invstd, float* running_mean,
                               float* running_var, const float* gamma, const float* beta, int B, int C, int N,
                               float eps, float momentum, int relu, float* pool, int32_t* pool_idx,
                               int64_t* batches_tracked, void* stream) {
  if (!y || !mean || !invstd || !gamma || !beta || B <= 0 || C <= 0 || N <= 0) return -20;
  if (pool ? (!pool_idx || B > kPoolMaxB) : !z) return -20;
  long long* nbt = reinterpret_cast<long long*>(batches_tracked);
  if (bn_wide_groups(C))
    k_tr_bn_fwd<1024><<<C, 1024, 0, (hipStream_t)stream>>>(y, z, mean, invstd, running_mean, running_var, gamma, beta,
                                                           B, C, N, eps, momentum, relu, pool, pool_idx, nbt);
  else
    k_tr_bn_fwd<kBnThreads><<<C, kBnThreads, 0, (hipStream_t)stream>>>(
        y, z, mean, invstd, running_mean, running_var, gamma, beta, B, C, N, eps, momentum, relu, pool, pool_idx, nbt);
  return launched();
}

extern "C" int ndnet_tr_bn_bwd(const float* dz, const float* y, const float* mean, const float* invstd,
                               const float* gamma, const float* beta, float* dy, float* dgamma, float* dbeta,
                               float* dbias, int B, int C, int N, int relu, const int32_t* pool_idx, void* stream) {
  if (!dz || !y || !mean || !invstd || !gamma || !beta || !dy || B <= 0 || C <= 0 || N <= 0) return -20;
  if (pool_idx && B > kPoolMaxB) return -20;  // the pooled gradients are staged per cloud
  if (bn_wide_groups(C))
    k_tr_bn_bwd<1024><<<C, 1024, 0, (hipStream_t)stream>>>(dz, y, mean, invstd, gamma, beta, dy, dgamma, dbeta,
                                                           dbias, B, C, N, relu, pool_idx);
  else
    k_tr_bn_bwd<kBnThreads><<<C, kBnThreads, 0, (hipStream_t)stream>>>(dz, y, mean, invstd, gamma, beta, dy, dgamma,
                                                                       dbeta, dbias, B, C, N, relu, pool_idx);
  return launched();
}

extern "C" int ndnet_tr_chan_sum(const float* x, float* out, int B, int C, int N, void* stream) {
  if (!x || !out || B <= 0 || C <= 0 || N <= 0) return -20;
  k_tr_chan_sum<<<C, kBnThreads, 0, (hipStream_t)stream>>>(x, out, B, C, N);
  return launched();
}

extern "C" int ndnet_tr_row_sum(const float* x, float* out, int64_t rows, int N, void* stream) {
  if (!x || !out || rows <= 0 || N <= 0 || (rows + 3) / 4 > (int64_t)INT32_MAX) return -20;
  k_tr_row_sum<<<(unsigned)((rows + 3) / 4), 256, 0, (hipStream_t)stream>>>(x, out, rows, N);
  return launched();
}

extern "C" int ndnet_tr_argmax_match(const float* pred, const float* gt, int64_t rows, int cols, uint32_t* count,
                                     void* stream) {
  if (!pred || !gt || !count || rows <= 0 || cols <= 0 || (rows + 255) / 256 > (int64_t)INT32_MAX) return -20;
  k_tr_argmax_match<<<(unsigned)((rows + 255) / 256), 256, 0, (hipStream_t)stream>>>(pred, gt, rows, cols, count);
  return launched();
}

extern "C" int ndnet_tr_argmax_match_cm(const float* pred, const float* gt, int B, int C, int N, uint32_t* ctr,
                                        float* acc, void* stream) {
  const int64_t rows = (int64_t)B * N;
  if (!pred || !gt || !ctr || B <= 0 || C <= 0 || N <= 0 || C > kLsmC) return -20;
  if ((rows + kLsmT - 1) / kLsmT > (int64_t)INT32_MAX) return -20;
  k_tr_argmax_match_cm<<<(unsigned)((rows + kLsmT - 1) / kLsmT), kLsmT, 0, (hipStream_t)stream>>>(pred, gt, B, C, N,
                                                                                                 ctr, acc);
  return launched();
}

extern "C" int ndnet_row_argmax(const float* x, int64_t rows, int cols, int32_t* out, void* stream) {
  if (!x || !out || rows <= 0 || cols <= 0 || (rows + 255) / 256 > (int64_t)INT32_MAX) return -20;
  if (cols <= kArgmaxStagedCols)
    k_row_argmax_staged<<<(unsigned)((rows + 255) / 256), 256, 256 * cols * sizeof(float), (hipStream_t)stream>>>(
        x, rows, cols, out);
  else
    k_row_argmax<<<(unsigned)((rows + 255) / 256), 256, 0, (hipStream_t)stream>>>(x, rows, cols, out);
  return launched();
}

// workgroups of the FC kernels: a wave per channel, at most 256 workgroups
// (each stages x once; the waves loop over the channels past the grid)
static unsigned fc_grid(int N) {
  const int g = (N + kFcWaves - 1) / kFcWaves;
  return (unsigned)(g < 256 ? g : 256);
}

extern "C" int ndnet_tr_fc_fwd(const float* x, const float* W, const float* bias, float* y, float* z, float* mean,
                               float* invstd, float* running_mean, float* running_var, const float* gamma,
                               const float* beta, int B, int K, int N, int64_t ldw, float eps, float momentum, int relu,
                               int eye, int64_t* batches_tracked, void* stream) {
  if (ldw == 0) ldw = K;
  if (!x || !W || !bias || !z || B <= 0 || B > kFcB || K <= 0 || K % 4 || N <= 0 || ldw < K || ldw % 4) return -20;
  if (gamma && (!y || !mean || !invstd || !beta)) return -20;
  if (!gamma && (relu || batches_tracked)) return -20;
  if ((((uintptr_t)x | (uintptr_t)W) & 15) != 0) return -20;  // float4 rows
  const size_t lds = (size_t)B * K * sizeof(float);
  if (lds > (size_t)kFcMaxLds) return -20;  // x staged whole (K <= 1024 at 16 rows)
  k_tr_fc_fwd<<<fc_grid(N), kFcWaves * 64, lds, (hipStream_t)stream>>>(x, W, bias, y, z, mean, invstd, running_mean,
                                                              running_var, gamma, beta, B, K, N, eps, momentum, relu,
                                                              eye, reinterpret_cast<long long*>(batches_tracked), ldw);
  return launched();
}

extern "C" int ndnet_tr_fc_bwd_w(const float* dz, const float* x, const float* y, const float* mean,
                                 const float* invstd, const float* gamma, const float* beta, float* dpre, float* dW,
                                 float* db, float* dgamma, float* dbeta, int B, int K, int N, int64_t ldw, int relu,
                                 void* stream) {
  if (ldw == 0) ldw = K;
  if (!dz || !x || B <= 0 || B > kFcB || K <= 0 || K % 4 || N <= 0 || ldw < K || ldw % 4) return -20;
  if (gamma && (!y || !mean || !invstd || !beta)) return -20;
  if (!gamma && relu) return -20;
  if ((((uintptr_t)x | (uintptr_t)dW) & 15) != 0) return -20;
  const size_t lds = dW ? (size_t)B * K * sizeof(float) : 0;
  if (lds > (size_t)kFcMaxLds) return -20;
  k_tr_fc_bwd_w<<<fc_grid(N), kFcWaves * 64, lds, (hipStream_t)stream>>>(dz, x, y, mean, invstd, gamma, beta, dpre, dW, db,
                                                                dgamma, dbeta, B, K, N, relu, ldw);
  return launched();
}

extern "C" int ndnet_tr_fc_bwd_x(const float* dpre, const float* W, float* dx, float* part, int B, int K, int N,
                                 int64_t ldw, int nsplit, void* stream) {
  if (ldw == 0) ldw = K;
  if (!dpre || !W || !dx || B <= 0 || B > kFcB || K <= 0 || N <= 0 || nsplit <= 0 || nsplit > N || ldw < K)
    return -20;
  if ((N + nsplit - 1) / nsplit > kFcXMaxN || (nsplit > 1 && !part)) return -20;
  float* out = nsplit > 1 ? part : dx;
  k_tr_fc_bwd_x<<<dim3((K + 255) / 256, nsplit), 256, 0, (hipStream_t)stream>>>(dpre, W, out, B, K, N, nsplit, ldw);
  if (nsplit > 1) {
    const int64_t count = (int64_t)B * K;
    k_tr_sum_parts<<<(unsigned)((count + 255) / 256), 256, 0, (hipStream_t)stream>>>(part, dx, count, nsplit, count,
                                                                                     count);
  }
  return launched();
}

extern "C" int ndnet_tr_log_softmax_c(const float* x, float* out, int B, int C, int N, void* stream) {
  if (!x || !out || B <= 0 || C <= 0 || N <= 0) return -20;
  if (C > kLsmC) return -20;  // the classes of a point are held in registers
  const int64_t pts = (int64_t)B * N;
  k_tr_log_softmax_c<<<(unsigned)((pts + kLsmT - 1) / kLsmT), kLsmT, 0, (hipStream_t)stream>>>(x, out, B, C, N);
  return launched();
}

extern "C" int ndnet_tr_log_softmax_c_bwd(const float* y, const float* dy, float* dx, int B, int C, int N,
                                          void* stream) {
  if (!y || !dy || !dx || B <= 0 || C <= 0 || N <= 0) return -20;
  if (C > kLsmC) return -20;  // the classes of a point are held in registers
  const int64_t pts = (int64_t)B * N;
  k_tr_log_softmax_c_bwd<<<(unsigned)((pts + kLsmT - 1) / kLsmT), kLsmT, 0, (hipStream_t)stream>>>(y, dy, dx, B, C, N);
  return launched();
}

extern "C" int ndnet_tr_point_transform(const float* t, const float* pts, int pld, const float* extra, int eld,
                                        float* x, int B, int N, void* stream) {
  if (!t || !pts || !extra || !x || B <= 0 || N <= 0 || pld < 3 || eld < 9) return -20;
  k_tr_point_transform<<<dim3((unsigned)((N + kPtT - 1) / kPtT), (unsigned)B), kPtT, 0, (hipStream_t)stream>>>(
      t, pts, pld, extra, eld, x, N);
  return launched();
}

extern "C" int ndnet_tr_point_transform_bwd(const float* dx, const float* pts, int pld, const float* extra, int eld,
                                            float* dt, int B, int N, void* stream) {
  if (!dx || !pts || !extra || !dt || B <= 0 || N <= 0 || pld < 3 || eld < 9) return -20;
  k_tr_point_transform_bwd<<<(unsigned)B, kPtBwdT, 0, (hipStream_t)stream>>>(dx, pts, pld, extra, eld, dt, N);
  return launched();
}

extern "C" int ndnet_tr_nll_onehot(const float* logp, const float* gt, double* part, float* loss, int B, int C, int N,
                                   void* stream) {
  if (!logp || !gt || !part || !loss || B <= 0 || C <= 0 || N <= 0) return -20;
  if (C > kLsmC) return -20;  // the classes of a point are held in registers
  const int64_t pts = (int64_t)B * N;
  const unsigned blocks = (unsigned)((pts + kLsmT - 1) / kLsmT);
  k_tr_nll_part<<<blocks, kLsmT, 0, (hipStream_t)stream>>>(logp, gt, part, B, C, N);
  k_tr_nll_sum<<<1, 64, 0, (hipStream_t)stream>>>(part, (int)blocks, loss, pts);
  return launched();
}

extern "C" int ndnet_tr_nll_onehot_bwd(const float* gt, const float* dloss, float* dlogp, int B, int C, int N,
                                       void* stream) {
  if (!gt || !dloss || !dlogp || B <= 0 || C <= 0 || N <= 0) return -20;
  if (C > kLsmC) return -20;  // the classes of a point are held in registers
  const int64_t pts = (int64_t)B * N;
  k_tr_nll_bwd<<<(unsigned)((pts + kLsmT - 1) / kLsmT), kLsmT, 0, (hipStream_t)stream>>>(gt, dloss, dlogp, B, C, N);
  return launched();
}

extern "C" int ndnet_tr_adam(int n, float* const* params, const float* const* grads, float* const* exp_avg,
                             float* const* exp_avg_sq, float* const* steps, const int64_t* numel, const float* lr,
                             double beta1, double beta2, float eps, float weight_decay, void* stream) {
  if (n <= 0 || !params || !grads || !exp_avg || !exp_avg_sq || !steps || !numel || !lr) return -20;
  hipStream_t st = (hipStream_t)stream;
  for (int b0 = 0; b0 < n; b0 += kAdamStepsMax) {  // one launch for every step count (<= 128 tensors)
    AdamSteps S;
    S.n = n - b0 < kAdamStepsMax ? n - b0 : kAdamStepsMax;
    for (int i = 0; i < S.n; i++) {
      if (!steps[b0 + i]) return -20;
      S.s[i] = steps[b0 + i];
    }
    k_tr_adam_steps<<<1, 64, 0, st>>>(S);
  }
  for (int b0 = 0; b0 < n; b0 += kAdamMax) {
    AdamArgs A;
    A.n = n - b0 < kAdamMax ? n - b0 : kAdamMax;
    int64_t chunks = 0;
    for (int i = 0; i < A.n; i++) {
      const int j = b0 + i;
      if (!params[j] || !grads[j] || !exp_avg[j] || !exp_avg_sq[j] || !steps[j] || numel[j] <= 0) return -20;
      A.p[i] = params[j];
      A.g[i] = grads[j];
      A.m[i] = exp_avg[j];
      A.v[i] = exp_avg_sq[j];
      A.step[i] = steps[j];
      A.numel[i] = numel[j];
      A.chunk0[i] = (int)chunks;
      chunks += (numel[j] + kAdamChunk - 1) / kAdamChunk;
      if (chunks > INT32_MAX) return -20;
    }
    A.chunk0[A.n] = (int)chunks;
    A.beta1 = (float)beta1;
    A.beta2 = (float)beta2;
    A.omb1 = (float)(1.0 - beta1);
    A.omb2 = (float)(1.0 - beta2);
    A.beta1d = beta1;
    A.beta2d = beta2;
    A.eps = eps;
    A.wd = weight_decay;
    A.lr = lr;
    k_tr_adam<<<(unsigned)chunks, 256, 0, st>>>(A);
  }
  return launched();
}

