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
// Tile geometry: 64 points = four 16-row MFMA blocks per workgroup, 16 waves
// (4 per SIMD, so a wave waiting on its weight loads leaves three to keep the
// MFMA pipe busy).  A layer's waves split the tile as (row groups x column
// groups): for N a multiple of 256 each wave takes all four row blocks of one
// 16-column block (16 x 1), so every weight fragment is loaded once per
// workgroup; 2 x 8 for N = 128, 4 x 4 for N = 64 / 32.  Weights are stored
// fragment-major (include/ndnet_pointnet.h) and stream from L2 straight into
// registers, two k-groups ahead; the activations stay in LDS.  Barriers only
// separate layers (and the chunks of a fused pair).
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
#include <stdlib.h>

#include "../../include/ndnet_pointnet.h"

namespace {

// Tile size: 64 points (16 waves), or 32 points (8 waves) in the second build
// of this file (-DNDNET_PN_TILE=32: pointnet_chain_t32.o, entry point
// ndnet_pn_chain_run_t32) for batches whose 64-point tiles would leave CUs
// idle (C5's 500-point level: 128 workgroups on 256 CUs).  Same wave-per-row-
// block ratios, so every layer split below has the same shape per wave.
#ifndef NDNET_PN_TILE
#define NDNET_PN_TILE 64
#endif
constexpr int kP = NDNET_PN_TILE;  // points per workgroup
#ifndef NDNET_PN_WAVES
#define NDNET_PN_WAVES (NDNET_PN_TILE / 4)
#endif
constexpr int kWaves = NDNET_PN_WAVES;
constexpr int kThreads = 64 * kWaves;
constexpr int kRowBlocks = kP / 16;  // 4 (2 for 32-point tiles)
static_assert(kP == 64 || kP == 32, "64- or 32-point tiles");
constexpr int kFuseNC = 64;     // columns per chunk of a fused layer
// LDS row pitch padding.  An A-fragment read (ds_read_b128, 16 B per lane at
// row l & 15, column offset 16 B * (l >> 4)) is conflict-free when the row
// pitch is 32 B mod 256 B (two 4-bank slots per row: the 16 lanes of each
// ds_read_b128 lane group land on 16 distinct slots); a pitch of 16 B mod
// 256 B (one slot per row) puts two lanes of every group on one slot and
// doubles the read.  Activation widths are multiples of 64 (or 16 / 32 / 64
// for the input tile), so width + kPadF floats / width + kPadB bf16 give it.
constexpr int kPadF = 8;        // fp32 regions: pitch = width + 8 floats
constexpr int kPadB = 16;       // bf16 planes: pitch = width + 16 bf16
// bf16 planes, round 6: the epilogues store a lane's 4 channels of one point
// as one ds_write_b64 per plane, and a write's 16-lane group (one kq, points
// cl = 0..15) lands on 16 rows of the same columns.  Writes bank on (a/4) mod
// 32 (MI355X_MICROARCH.md §LDS): with these pitches (32 B + a multiple of
// 128 B: 8 dwords mod 32) rows r and r + 4 share banks -- 4-way, the chain
// D conflicts (25.7% of its LDS cycles, profiles/r05_pmc_summary.txt).  So the
// 16-byte slots of row r are XOR-swizzled by bit 2 of r (slot s at s ^
// ((r >> 2) & 1)): the writes become 2-way, the least 16 rows x 8 bytes at
// 16-byte granularity allow (8 distinct slots mod 128 B), and the
// ds_read_b128 A-fragment reads stay conflict-free (every lane group on 16
// distinct 16-byte slots; checked exhaustively for the pitches used).  A read
// keeps its 16 bytes whole: only which slot of its row it reads moves.
#ifndef NDNET_PN_PLANE_SWZ
#define NDNET_PN_PLANE_SWZ 1
#endif
// the bf16 column where element (row, col) of a plane is stored (bit 3 of the
// column, slot bit 0, flipped on rows 4..7 mod 8)
__device__ inline int plane_col(int row, int col) {
  return NDNET_PN_PLANE_SWZ ? col ^ (((row >> 2) & 1) << 3) : col;
}
#ifndef NDNET_PN_DEPTH
#define NDNET_PN_DEPTH 2
#endif
constexpr int kDepth = NDNET_PN_DEPTH;  // weight k-groups in flight per wave
#ifndef NDNET_PN_DEPTH6
#define NDNET_PN_DEPTH6 1
#endif
constexpr int kDepth6 = NDNET_PN_DEPTH6;  // the same for split-bf16 layers (3 fragment planes each)
// chain D's fused pair computes chunk f + 1's P before chunk f's Q (same
// products, same order): 43.4 -> 42.9 us per chain D (gpurun_out/r05w_v)
#ifndef NDNET_PN_PAIR_PFIRST
#define NDNET_PN_PAIR_PFIRST 1
#endif
#ifndef NDNET_PN_CHUNK_ROT
#define NDNET_PN_CHUNK_ROT 1
#endif
constexpr bool kChunkRot = NDNET_PN_CHUNK_ROT;  // per-workgroup chunk order (run_tiles_x6 rot)
static_assert(kWaves % kRowBlocks == 0, "every row group has whole column groups");

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__device__ inline void atomic_max_f32(float* addr, float v) {
  v = v + 0.0f;  // -0 -> +0 so the integer orderings below agree
  if (v >= 0.0f) atomicMax(reinterpret_cast<int*>(addr), __float_as_int(v));
  else atomicMin(reinterpret_cast<unsigned int*>(addr), __float_as_uint(v));
}

// Output orientation of the MFMA tiles.  With the weights as the A operand
// and the activations as B (NDNET_PN_SWAP = 1, default) a 16 x 16 tile comes
// out transposed: lane (kq, cl) holds point cl, channels 4 kq .. 4 kq + 3 --
// four consecutive channels of one point, which the epilogue stores as one
// ds_write_b128 (fp32) or one ds_write_b64 per bf16 plane instead of 4 / 12
// scalar stores, and max-pools over the 16 points of a lane row with DPP.
// The operands' lane data are the same either way (the fragment layouts are
// symmetric), so only the MFMA argument order and the epilogues change.
// NDNET_PN_SWAP = 0: activations as A, lane (kq, cl) holds points 4 kq + r of
// channel cl.
#ifndef NDNET_PN_SWAP
#define NDNET_PN_SWAP 1
#endif

// v of lane (lane ^ S) within a 16-lane row, through DPP (no LDS)
template <int S>
__device__ inline float xor_row(float v) {
  const int x = __float_as_int(v);
  if constexpr (S == 1) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(x, 0xB1, 0xF, 0xF, false));  // quad_perm [1,0,3,2]
  } else if constexpr (S == 2) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(x, 0x4E, 0xF, 0xF, false));  // quad_perm [2,3,0,1]
  } else if constexpr (S == 4) {
    const int h = __builtin_amdgcn_mov_dpp(x, 0x141, 0xF, 0xF, false);          // row_half_mirror: i ^ 7
    return __int_as_float(__builtin_amdgcn_mov_dpp(h, 0x1B, 0xF, 0xF, false));  // quad_perm [3,2,1,0]: ^ 3
  } else {
    const int h = __builtin_amdgcn_mov_dpp(x, 0x140, 0xF, 0xF, false);           // row_mirror: i ^ 15
    return __int_as_float(__builtin_amdgcn_mov_dpp(h, 0x141, 0xF, 0xF, false));  // row_half_mirror: ^ 7
  }
}

// dynamic LDS of k_pn_chain: the two activation regions and the fused pair's
// double buffer, addressed by float offsets so every access is a ds_* op
extern __shared__ __attribute__((aligned(16))) float g_smem[];
#ifndef NDNET_PN_TID_FRESH
#define NDNET_PN_TID_FRESH 1
#endif
// threadIdx.x as a value the compiler cannot see through: a layer's lane /
// wave / row / column offsets are derived from it where the layer runs
// instead of being hoisted to the kernel's start and kept live through every
// layer (they took ~48 of the 128 VGPRs the 16-wave build has, so the x6
// loops could neither keep a plane's four A fragments nor the next weight
// step in registers)
__device__ inline int pn_tid() {
  int t = (int)threadIdx.x;
#if NDNET_PN_TID_FRESH
  asm volatile("" : "+v"(t));
#endif
  return t;
}


// Timing build only (-DNDNET_PN_STAMPS, tools/pn_stamps.py): s_memrealtime
// (100 MHz) of every workgroup at its start (0), after chain B's head
// prologue or chain C's t2 fold (1), after the input tile (2), after each layer's closing barrier
// (3 + layer) and at its end (15), read back by ndnet_pn_debug_stamps.  The
// product build compiles none of it.
#ifdef NDNET_PN_STAMPS
constexpr int kStampWgs = 1024;
__device__ unsigned long long g_pn_stamps[kStampWgs][16];
#define PN_STAMP(i)                                                                           \
  do {                                                                                        \
    const int w_ = blockIdx.y * gridDim.x + blockIdx.x;                                       \
    if (threadIdx.x == 0 && w_ < kStampWgs) g_pn_stamps[w_][(i)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define PN_STAMP(i) \
  do {              \
  } while (0)
#endif

// Weights are fragment-major (include/ndnet_pointnet.h): the 16 x 16 block
// (k-group kg, column block cb) of W^T is 64 lanes x float4, lane kq * 16 + cl
// holding W^T[16 kg + 4 kq + s][16 cb + cl] for s = 0..3 -- the B operands of
// four consecutive 16x16x4 MFMAs, one coalesced 1 KB global_load_dwordx4 per
// wave.  The A operand uses the same K permutation: lane (kq, cl) reads
// activation row cl, columns 16 kg + 4 kq .. + 3 with one ds_read_b128.  So
// the weights stream from L2 straight into registers (no LDS staging, no
// barrier inside a layer) and only the activations live in LDS.
struct LayerCtx {
  const f32x4* __restrict__ w;     // this cloud's fragments, offset by the lane (prec 0)
  const bf16x8* __restrict__ w6;   // split-bf16 fragments, offset by the lane (prec 1)
  const float* __restrict__ bias;
  int KG, N, relu, prec;           // KG: 16-row k-groups (prec 0) or 32-row (prec 1)
};

// bias: the layer's (this cloud's) bias, staged in LDS by the kernel's prologue
// The first weight step of a layer, loaded by each wave before the barrier
// that closes the previous layer (its latency hides behind the barrier wait;
// 16-wave 64-point build, where every layer's wave tile is one column block):
// r0..r2 = the three bf16x8 planes for prec 1, r0 for prec 0.
struct Pre {
  bool on;
  f32x4 r0, r1, r2;  // prec 1: bf16x8 planes h, m, l (bit_cast); prec 0: r0
};

__device__ inline LayerCtx layer_ctx(const ndnet_pn_chain& A, int l, int b, const float* bias) {
  const ndnet_pn_layer& L = A.L[l];
  LayerCtx C;
  C.w = reinterpret_cast<const f32x4*>(L.w + (int64_t)b * L.w_cloud_stride) + (pn_tid() & 63);
  C.w6 = reinterpret_cast<const bf16x8*>(L.w + (int64_t)b * L.w_cloud_stride) + (pn_tid() & 63);
  C.bias = bias;
  C.prec = L.prec;
  C.KG = L.prec ? L.K / 32 : L.K / 16;  // prec 1 and 2: 32-row k-groups
  C.N = L.N;
  C.relu = L.relu;
  return C;
}

template <int RB, int NB>
__device__ __attribute__((always_inline)) inline void zero_acc(f32x4 (&acc)[RB][NB]) {
#pragma unroll
  for (int rb = 0; rb < RB; rb++)
#pragma unroll
    for (int j = 0; j < NB; j++) acc[rb][j] = f32x4{0.f, 0.f, 0.f, 0.f};
}

// acc[rb][j] += A(row block rb, one k-group) . W(k-group, column block j)
template <int RB, int NB>
__device__ __attribute__((always_inline)) inline void mma_kgroup(f32x4 (&acc)[RB][NB], const f32x4 (&a)[RB],
                                                                 const f32x4 (&bw)[NB]) {
#pragma unroll
  for (int s = 0; s < 4; s++)
#pragma unroll
    for (int rb = 0; rb < RB; rb++)
#pragma unroll
      for (int j = 0; j < NB; j++)
#if NDNET_PN_SWAP
        acc[rb][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(bw[j][s], a[rb][s], acc[rb][j], 0, 0, 0);
#else
        acc[rb][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[rb][s], bw[j][s], acc[rb][j], 0, 0, 0);
#endif
}

// T = nchunk * nkg k-group steps.  Step t is k-group kg0 + t % nkg of column
// chunk c = t / nkg, whose column blocks for this wave are cb0 + c * cbs + j;
// its A fragment sits at abase + 16 (t % nkg) (+ 16 rb rows).  epi(acc, c)
// runs at each chunk end.  The weight fragments are prefetched kDepth steps
// ahead in a ring of register sets; past the last step the loads repeat it.
template <int RB, int NB, class Epi>
__device__ __attribute__((always_inline)) inline void run_tiles(f32x4 (&acc)[RB][NB], const f32x4* __restrict__ w,
                                                                int KG, int kg0, int nkg, int cb0, int cbs,
                                                                int nchunk, const float* abase, int pin, Epi epi,
                                                                Pre pre = {}) {
  const int T = nchunk * nkg;
  const int64_t jstride = (int64_t)KG * 64;
  const int64_t chunk_jump = ((int64_t)cbs * KG - (nkg - 1)) * 64;
  const f32x4* lp = w + ((int64_t)cb0 * KG + kg0) * 64;  // the next load's step
  int lkk = 0, lleft = T;
  auto advance = [&]() {
    if (lleft > 1) {
      lleft--;
      if (++lkk == nkg) {
        lkk = 0;
        lp += chunk_jump;
      } else {
        lp += 64;
      }
    }
  };
  auto load = [&](f32x4 (&bw)[NB]) {
#pragma unroll
    for (int j = 0; j < NB; j++) bw[j] = lp[j * jstride];
    advance();
  };
  // A fragments are software-pipelined one step ahead too (the A region is
  // read-only during the layer, so the prefetch may run into the next chunk)
  int kk = 0, c = 0, akk = 0;
  f32x4 a[RB];
  auto load_a = [&]() {
#pragma unroll
    for (int rb = 0; rb < RB; rb++) a[rb] = *reinterpret_cast<const f32x4*>(abase + rb * 16 * pin + 16 * akk);
    akk = akk + 1 == nkg ? 0 : akk + 1;
  };
  auto step = [&](const f32x4 (&bw)[NB]) {
    f32x4 cur[RB];
#pragma unroll
    for (int rb = 0; rb < RB; rb++) cur[rb] = a[rb];
    load_a();
    mma_kgroup<RB, NB>(acc, cur, bw);
    if (++kk == nkg) {
      epi(acc, c);
      kk = 0;
      c++;
    }
  };
  load_a();
  f32x4 bq[kDepth][NB];
#pragma unroll
  for (int i = 0; i < kDepth; i++) {
    if (NB == 1 && i == 0 && pre.on) {  // the first step, prefetched by the caller
      bq[0][0] = pre.r0;
      advance();
    } else {
      load(bq[i]);
    }
  }
  for (int t = 0; t < T; t += kDepth) {
#pragma unroll
    for (int i = 0; i < kDepth; i++) {
      if (t + i < T) {
        step(bq[i]);
        load(bq[i]);
      }
    }
  }
}

// Bias + ReLU of this wave's tile (rows row0.., bias columns col0 + 16 j + cl)
// into an LDS activation region at columns oc0 + 16 j + cl.
template <int RB, int NB>
__device__ __attribute__((always_inline)) inline void store_cols(const f32x4 (&acc)[RB][NB],
                                                                 const float* __restrict__ bias, int col0, int relu,
                                                                 int row0, int out, int pout, int oc0) {
  const int lane = pn_tid() & 63;
  const int kq = lane >> 4, cl = lane & 15;
#if NDNET_PN_SWAP
#pragma unroll
  for (int j = 0; j < NB; j++) {
    float bv[4];
#pragma unroll
    for (int r = 0; r < 4; r++) bv[r] = bias[col0 + 16 * j + 4 * kq + r];
#pragma unroll
    for (int rb = 0; rb < RB; rb++) {
      f32x4 v;
#pragma unroll
      for (int r = 0; r < 4; r++) {
        v[r] = acc[rb][j][r] + bv[r];
        if (relu) v[r] = fmaxf(v[r], 0.0f);
      }
      *reinterpret_cast<f32x4*>(g_smem + out + (row0 + 16 * rb + cl) * pout + oc0 + 16 * j + 4 * kq) = v;
    }
  }
#else
#pragma unroll
  for (int j = 0; j < NB; j++) {
    const float bv = bias[col0 + 16 * j + cl];
#pragma unroll
    for (int rb = 0; rb < RB; rb++)
#pragma unroll
      for (int r = 0; r < 4; r++) {
        float v = acc[rb][j][r] + bv;
        if (relu) v = fmaxf(v, 0.0f);
        g_smem[out + (row0 + 16 * rb + 4 * kq + r) * pout + oc0 + 16 * j + cl] = v;
      }
  }
#endif
}

// Bias + ReLU + max over this wave's valid rows, one float atomic max per
// column and wave into gmax (the workgroup's row groups meet in the atomics).
template <int RB, int NB>
__device__ __attribute__((always_inline)) inline void pool_cols(const f32x4 (&acc)[RB][NB],
                                                                const float* __restrict__ bias, int col0, int relu,
                                                                int row0, int rows_valid, float* gmax) {
  const int lane = pn_tid() & 63;
  const int kq = lane >> 4, cl = lane & 15;
#if NDNET_PN_SWAP
  // lane (kq, cl): point cl of each row block, channels 4 kq + r; the max over
  // the tile's valid points first (RB values in the lane, then the 16 lanes of
  // a lane row by DPP), then bias + ReLU once on the maximum -- exact, as
  // fl(a + b) and ReLU are monotonic in a -- and lane cl < 4 of the row takes
  // channel 4 kq + cl's atomic
  const bool full = row0 + 16 * RB <= rows_valid;  // wave-uniform: every row of the wave's tile is a point
#pragma unroll
  for (int j = 0; j < NB; j++) {
    float m[4];
#pragma unroll
    for (int r = 0; r < 4; r++) {
      if (full) {
        m[r] = acc[0][j][r];
#pragma unroll
        for (int rb = 1; rb < RB; rb++) m[r] = fmaxf(m[r], acc[rb][j][r]);
      } else {
        m[r] = -INFINITY;
#pragma unroll
        for (int rb = 0; rb < RB; rb++)
          if (row0 + 16 * rb + cl < rows_valid) m[r] = fmaxf(m[r], acc[rb][j][r]);
      }
      m[r] = fmaxf(m[r], xor_row<1>(m[r]));
      m[r] = fmaxf(m[r], xor_row<2>(m[r]));
      m[r] = fmaxf(m[r], xor_row<4>(m[r]));
      m[r] = fmaxf(m[r], xor_row<8>(m[r]));
    }
    const float mm = cl == 0 ? m[0] : cl == 1 ? m[1] : cl == 2 ? m[2] : m[3];
    if (cl < 4 && mm > -INFINITY) {
      float v = mm + bias[col0 + 16 * j + 4 * kq + cl];
      if (relu) v = fmaxf(v, 0.0f);
      atomic_max_f32(gmax + col0 + 16 * j + 4 * kq + cl, v);
    }
  }
#else
#pragma unroll
  for (int j = 0; j < NB; j++) {
    const float bv = bias[col0 + 16 * j + cl];
    float m = -INFINITY;
#pragma unroll
    for (int rb = 0; rb < RB; rb++)
#pragma unroll
      for (int r = 0; r < 4; r++) {
        float v = acc[rb][j][r] + bv;
        if (relu) v = fmaxf(v, 0.0f);
        if (row0 + 16 * rb + 4 * kq + r < rows_valid) m = fmaxf(m, v);
      }
    m = fmaxf(m, __shfl_xor(m, 16, 64));
    m = fmaxf(m, __shfl_xor(m, 32, 64));
    if (lane < 16 && m > -INFINITY) atomic_max_f32(gmax + col0 + 16 * j + cl, m);
  }
#endif
}

// ---------------------------------------------------------------------------
// Split-bf16 layers (ndnet_pn_layer.prec = 1): fp32-accurate GEMMs on the
// bf16 matrix cores.  Every operand x is split x = h + m + l into three bf16
// (8 + 8 + 8 significant bits = fp32's 24; h = bf16(x), m = bf16(x - h),
// l = bf16(x - h - m), each residual exact in fp32).  A product keeps the six
// terms of weight >= 2^-16 (mm, mh, lh, hl, hm, hh in that order) -- each
// an exact bf16 x bf16 product accumulated in fp32 by v_mfma_f32_16x16x32_bf16;
// the dropped ml, lm, ll are below 3 * 2^-24 |x y|, the size of fp32's own
// rounding.  Six 16-cycle MFMAs per 16x16x32 block against eight 32-cycle
// v_mfma_f32_16x16x4_f32 for the same FLOPs: 2.7x less matrix-core time.
//
// The layer's input activations are stored by the producing layer's epilogue
// as three bf16 planes of the LDS region (plane p at p * kP * pitch, element
// (row, k) at row * pitch + k, pitch = width + kPadB bf16); lane l of a 16x16x32
// A fragment reads row l & 15, k = 32 kg + 8 (l >> 4) .. + 7 with one
// ds_read_b128 per plane.  The weights are fragment-major per 32-row k-group:
// [column block][k-group][plane][lane][8 bf16], lane l holding
// W^T[32 kg + 8 (l >> 4) + j][16 cb + (l & 15)] (include/ndnet_pointnet.h).

__device__ inline void split3(float v, __bf16& h, __bf16& m, __bf16& l) {
  h = (__bf16)v;
  const float r = v - (float)h;
  m = (__bf16)r;
  l = (__bf16)(r - (float)m);
}

// Bias + ReLU of this wave's tile into the three bf16 planes of a region
// (`out` in floats; pitch in bf16).
template <int RB, int NB>
__device__ __attribute__((always_inline)) inline void store_cols_planes(const f32x4 (&acc)[RB][NB],
                                                                        const float* __restrict__ bias, int col0,
                                                                        int relu, int row0, int out, int pitchb,
                                                                        int oc0) {
  const int lane = pn_tid() & 63;
  const int kq = lane >> 4, cl = lane & 15;
  __bf16* const base = reinterpret_cast<__bf16*>(g_smem + out);
  const int plane = kP * pitchb;
#if NDNET_PN_SWAP
  typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
#pragma unroll
  for (int j = 0; j < NB; j++) {
    float bv[4];
#pragma unroll
    for (int r = 0; r < 4; r++) bv[r] = bias[col0 + 16 * j + 4 * kq + r];
#pragma unroll
    for (int rb = 0; rb < RB; rb++) {
      bf16x4 h4, m4, l4;
#pragma unroll
      for (int r = 0; r < 4; r++) {
        float v = acc[rb][j][r] + bv[r];
        if (relu) v = fmaxf(v, 0.0f);
        __bf16 h, m, l;
        split3(v, h, m, l);
        h4[r] = h;
        m4[r] = m;
        l4[r] = l;
      }
      const int row = row0 + 16 * rb + cl;
      const int e = row * pitchb + plane_col(row, oc0 + 16 * j + 4 * kq);  // 4 channels: 8 bytes
      *reinterpret_cast<bf16x4*>(base + e) = h4;
      *reinterpret_cast<bf16x4*>(base + plane + e) = m4;
      *reinterpret_cast<bf16x4*>(base + 2 * plane + e) = l4;
    }
  }
#else
#pragma unroll
  for (int j = 0; j < NB; j++) {
    const float bv = bias[col0 + 16 * j + cl];
#pragma unroll
    for (int rb = 0; rb < RB; rb++)
#pragma unroll
      for (int r = 0; r < 4; r++) {
        float v = acc[rb][j][r] + bv;
        if (relu) v = fmaxf(v, 0.0f);
        __bf16 h, m, l;
        split3(v, h, m, l);
        const int row = row0 + 16 * rb + 4 * kq + r;
        const int e = row * pitchb + plane_col(row, oc0 + 16 * j + cl);
        base[e] = h;
        base[plane + e] = m;
        base[2 * plane + e] = l;
      }
  }
#endif
}

// One 32-row k-group: the A planes are read one at a time (m, l, h) so only
// one plane's fragments are live; per plane the B planes its terms need.
template <int RB, int NB>
__device__ __attribute__((always_inline)) inline void mma_kgroup_x6(f32x4 (&acc)[RB][NB], const __bf16* a0, int plane,
                                                                    int rstride, const bf16x8 (&bw)[NB][3]) {
  bf16x8 a[RB];
  auto ld = [&](int p) {
#ifdef NDNET_PN_EXP_NOA  // timing experiment only (wrong results): A fragments from registers
    if (p != 1) return;
#endif
#pragma unroll
    for (int rb = 0; rb < RB; rb++) a[rb] = *reinterpret_cast<const bf16x8*>(a0 + p * plane + rb * rstride);
  };
  auto mm = [&](int pb) {
#pragma unroll
    for (int rb = 0; rb < RB; rb++)
#pragma unroll
      for (int j = 0; j < NB; j++)
#if NDNET_PN_SWAP
        acc[rb][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[j][pb], a[rb], acc[rb][j], 0, 0, 0);
#else
        acc[rb][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[rb], bw[j][pb], acc[rb][j], 0, 0, 0);
#endif
  };
  ld(1);  // m: m*m, m*h
  mm(1);
  mm(0);
  ld(2);  // l: l*h
  mm(0);
  ld(0);  // h: h*l, h*m, h*h
  mm(2);
  mm(1);
  mm(0);
}

// run_tiles for split-bf16 layers: 32-row k-groups; A from the three planes
// (abase: this lane's row / k offset in plane 0, in bf16), B three 1 KB
// fragment pieces per column block, prefetched kDepth6 steps ahead.
template <int RB, int NB, class Epi, int kD = kDepth6>
__device__ __attribute__((always_inline)) inline void run_tiles_x6(f32x4 (&acc)[RB][NB],
                                                                   const bf16x8* __restrict__ w, int KG, int kg0,
                                                                   int nkg, int cb0, int cbs, int nchunk,
                                                                   const __bf16* abase, int pitchb, Epi epi,
                                                                   Pre pre = {}, int rot = 0) {
  // rot: the chunks run in the order rot, rot + 1, .. (mod nchunk), so that
  // workgroups in lockstep do not all stream the same weight fragments at
  // once (different chunks hit different L2 lines); each chunk's columns and
  // sums are unchanged
  const int T = nchunk * nkg;
  const int plane = kP * pitchb;
  const int64_t jstride = (int64_t)KG * 3 * 64;
  const int64_t chunk_jump = ((int64_t)cbs * KG - (nkg - 1)) * 3 * 64;
  const int64_t wrap = (int64_t)nchunk * cbs * KG * 3 * 64;
  const bf16x8* lp = w + ((int64_t)(cb0 + rot * cbs) * KG + kg0) * 3 * 64;
  int lkk = 0, lleft = T, lc = rot;
  auto advance = [&]() {
    if (lleft > 1) {
      lleft--;
      if (++lkk == nkg) {
        lkk = 0;
        lp += chunk_jump;
        if (++lc == nchunk) {
          lc = 0;
          lp -= wrap;
        }
      } else {
        lp += 3 * 64;
      }
    }
  };
  auto load = [&](bf16x8 (&bw)[NB][3]) {
#ifdef NDNET_PN_EXP_NOB  // timing experiment only (wrong results): weights loaded once per layer
    if (lleft == T)
#endif
#pragma unroll
    for (int j = 0; j < NB; j++)
#pragma unroll
      for (int p = 0; p < 3; p++) bw[j][p] = lp[j * jstride + p * 64];
    advance();
  };
  int kk = 0, c = rot;
  auto step = [&](const bf16x8 (&bw)[NB][3]) {
    mma_kgroup_x6<RB, NB>(acc, abase + 32 * kk, plane, 16 * pitchb, bw);
    if (++kk == nkg) {
      epi(acc, c);
      kk = 0;
      if (++c == nchunk) c = 0;
    }
  };
  bf16x8 bq[kD][NB][3];
#pragma unroll
  for (int i = 0; i < kD; i++) {
    if (NB == 1 && i == 0 && pre.on) {  // the first step, prefetched by the caller
      bq[0][0][0] = __builtin_bit_cast(bf16x8, pre.r0);
      bq[0][0][1] = __builtin_bit_cast(bf16x8, pre.r1);
      bq[0][0][2] = __builtin_bit_cast(bf16x8, pre.r2);
      advance();
    } else {
      load(bq[i]);
    }
  }
  for (int t = 0; t < T; t += kD) {
#pragma unroll
    for (int i = 0; i < kD; i++) {
      if (t + i < T) {
        step(bq[i]);
        if (t + i + kD < T) load(bq[i]);  // no reload past the last step
      }
    }
  }
}

// One layer: RB row blocks x NB column blocks per wave; 4 / RB row groups x
// 4 RB column groups of waves; N in chunks of (column groups x NB x 16).
template <int RB, int NB>
__device__ __attribute__((always_inline)) inline void plain_layer(const LayerCtx& C, int in, int pin, int out, int pout, float* gmax, int rows_valid,
                            bool out_planes, Pre pre = {}) {
  constexpr int WR = kRowBlocks / RB, WC = kWaves / WR, CB = WC * NB;
  const int lane = pn_tid() & 63, wave = pn_tid() >> 6;
  const int wr = wave / WC, wc = wave % WC;
  const int kq = lane >> 4, cl = lane & 15;
  const int row0 = wr * RB * 16;
  // N is a multiple of the chunk width, or narrower than one chunk (then the
  // waves past column N / 16 idle; there is no barrier inside a layer)
  if (C.N < CB * 16 && wc * NB * 16 >= C.N) return;
  f32x4 acc[RB][NB];
  zero_acc(acc);
  auto epi = [&](f32x4 (&a)[RB][NB], int c) {
    const int col0 = (c * CB + wc * NB) * 16;
    if (gmax) pool_cols<RB, NB>(a, C.bias, col0, C.relu, row0, rows_valid, gmax);
    else if (out_planes) store_cols_planes<RB, NB>(a, C.bias, col0, C.relu, row0, out, C.N + kPadB, col0);
    else store_cols<RB, NB>(a, C.bias, col0, C.relu, row0, out, pout, col0);
    zero_acc(a);
  };
  const int nchunk = C.N < CB * 16 ? 1 : C.N / (CB * 16);
  if (C.prec) {  // input: three bf16 planes of pitch K + kPadB (the producer's N + kPadB)
    const int pb = 32 * C.KG + kPadB;
    const __bf16* abase6 = reinterpret_cast<const __bf16*>(g_smem + in) + (row0 + cl) * pb + plane_col(cl, 8 * kq);
#ifndef NDNET_PN_SHORT_D2
#define NDNET_PN_SHORT_D2 1
#endif
    // a layer of two k-group steps (K = 64, one chunk: the narrow 64 -> 64 /
    // 64 -> 128 layers) loads both up front, so only one L2 latency is exposed
    if (NDNET_PN_SHORT_D2 && nchunk * C.KG == 2)
      run_tiles_x6<RB, NB, decltype(epi), 2>(acc, C.w6, C.KG, 0, C.KG, wc * NB, CB, nchunk, abase6, pb, epi, pre, 0);
    else
      run_tiles_x6<RB, NB>(acc, C.w6, C.KG, 0, C.KG, wc * NB, CB, nchunk, abase6, pb, epi, pre,
                           kChunkRot ? (int)((blockIdx.x + blockIdx.y) % nchunk) : 0);
  } else {
    const float* abase = g_smem + in + (row0 + cl) * pin + 4 * kq;
    run_tiles<RB, NB>(acc, C.w, C.KG, 0, C.KG, wc * NB, CB, nchunk, abase, pin, epi, pre);
  }
}

// Floats of the fused pair's double buffer: two 64-column chunks, fp32 or
// (split-bf16 consumer) three bf16 planes of pitch 72.
__host__ __device__ inline int fbuf_floats(int qprec) {
  return qprec ? 2 * 3 * kP * (kFuseNC + kPadB) / 2 : 2 * kP * (kFuseNC + kPadF);
}

// A fused pair: layer P (K -> N1) produced 64 columns at a time into a
// double-buffered LDS chunk (waves 4 x 4, one 16 x 16 tile each), each chunk
// consumed at once as 4 k-groups of layer Q (N1 -> N2 = one chunk of Q's
// (RB, NB) split), whose accumulators persist across the chunks: the N1-wide
// activation never needs LDS of its own.  One barrier per chunk.
template <int RB, int NB>
__device__ __attribute__((always_inline)) inline void fused_pair(const LayerCtx& P, const LayerCtx& Q, int in, int pin, int fbuf, int out, int pout,
                           float* gmax, int rows_valid, bool out_planes, Pre pre = {}) {
  constexpr int kFP = kFuseNC + kPadF;
  constexpr int WR = kRowBlocks / RB, WC = kWaves / WR;
  const int lane = pn_tid() & 63, wave = pn_tid() >> 6;
  const int kq = lane >> 4, cl = lane & 15;
  // P: row block wave / PWC, PNB column blocks from 4 f + PNB (wave % PWC)
  constexpr int PWC = kWaves / kRowBlocks, PNB = 4 / PWC;
  const int prow0 = (wave / PWC) * 16, pwc = (wave % PWC) * PNB;
  const float* ain = g_smem + in + (prow0 + cl) * pin + 4 * kq;
  const __bf16* ain6 = reinterpret_cast<const __bf16*>(g_smem + in) + (prow0 + cl) * (32 * P.KG + kPadB) +
                       plane_col(cl, 8 * kq);
  // Q: row group wave / WC, column group wave % WC
  const int qrow0 = (wave / WC) * RB * 16, qwc = wave % WC;
  const bool qidle = qwc * NB * 16 >= Q.N;
  const int nf = P.N / kFuseNC;
  // a split-bf16 Q reads its chunks as three bf16 planes (pitch 72)
  const int fbsz = Q.prec ? fbuf_floats(1) / 2 : kP * kFP;
  auto p_chunk = [&](int f) {
    f32x4 acc1[1][PNB];
    zero_acc(acc1);
    const int fb = fbuf + (f & 1) * fbsz;
    auto epi = [&](f32x4 (&a)[1][PNB], int) {
      if (Q.prec) store_cols_planes<1, PNB>(a, P.bias, 64 * f + 16 * pwc, P.relu, prow0, fb, kFuseNC + kPadB, 16 * pwc);
      else store_cols<1, PNB>(a, P.bias, 64 * f + 16 * pwc, P.relu, prow0, fb, kFP, 16 * pwc);
    };
    Pre pf = pre;
    if (f != 0) pf.on = false;
    if (P.prec) run_tiles_x6<1, PNB>(acc1, P.w6, P.KG, 0, P.KG, 4 * f + pwc, 0, 1, ain6, 32 * P.KG + kPadB, epi, pf);
    else run_tiles<1, PNB>(acc1, P.w, P.KG, 0, P.KG, 4 * f + pwc, 0, 1, ain, pin, epi, pf);
  };
  f32x4 acc2[RB][NB];
  zero_acc(acc2);
  p_chunk(0);
  __syncthreads();
  for (int f = 0; f < nf; f++) {
    if (!qidle) {
      if (Q.prec) {
        const __bf16* af6 = reinterpret_cast<const __bf16*>(g_smem + fbuf + (f & 1) * fbsz) +
                            (qrow0 + cl) * (kFuseNC + kPadB) + plane_col(cl, 8 * kq);
        run_tiles_x6<RB, NB>(acc2, Q.w6, Q.KG, 2 * f, 2, qwc * NB, 0, 1, af6, kFuseNC + kPadB,
                             [](f32x4 (&)[RB][NB], int) {});
      } else {
        const float* af = g_smem + fbuf + (f & 1) * fbsz + (qrow0 + cl) * kFP + 4 * kq;
        run_tiles<RB, NB>(acc2, Q.w, Q.KG, 4 * f, 4, qwc * NB, 0, 1, af, kFP, [](f32x4 (&)[RB][NB], int) {});
      }
    }
    if (f + 1 < nf) p_chunk(f + 1);
    __syncthreads();
  }
  if (qidle) return;
  if (gmax) pool_cols<RB, NB>(acc2, Q.bias, 16 * qwc * NB, Q.relu, qrow0, rows_valid, gmax);
  else if (out_planes) store_cols_planes<RB, NB>(acc2, Q.bias, 16 * qwc * NB, Q.relu, qrow0, out, Q.N + kPadB, 16 * qwc * NB);
  else store_cols<RB, NB>(acc2, Q.bias, 16 * qwc * NB, Q.relu, qrow0, out, pout, 16 * qwc * NB);
}

// The fused pair with both layers split-bf16 and P's K = 64 (the seg head's
// 64 -> 512 -> 256, ndtnet.py:233-234), software-pipelined across chunks.
// fused_pair loads each chunk's weights at the start of the chunk's GEMM, so
// every chunk exposes the L2 latency of P's and Q's first steps -- with all 16
// waves in lockstep between the chunk barriers, nothing covers it (chain D's
// pair ran at ~0.42 of the issued peak against ~0.55 for the plain x6 layers,
// profiles/r04_chain_vgpr_ab.txt).  Here a chunk's weights (P: 2 k-groups, Q:
// 2 k-groups, 3 planes each: 48 VGPRs) are loaded one chunk ahead, right after
// the previous chunk's MFMAs consumed the registers, so each load has a whole
// phase and a barrier to arrive.  Same products, same accumulation order.
template <int RB>
__device__ __attribute__((always_inline)) inline void fused_pair_x6p(const LayerCtx& P, const LayerCtx& Q, int in,
                                                                     int fbuf, int out, int pout, float* gmax,
                                                                     int rows_valid, bool out_planes) {
  constexpr int WR = kRowBlocks / RB, WC = kWaves / WR;  // Q: NB = 1
  constexpr int PWC = kWaves / kRowBlocks;                // P: 4 column groups of one block
  static_assert(PWC == 4 && kFuseNC == 64, "16 waves, 64-column chunks");
  const int lane = pn_tid() & 63, wave = pn_tid() >> 6;
  const int kq = lane >> 4, cl = lane & 15;
  const int prow0 = (wave / PWC) * 16, pwc = wave % PWC;
  const int pinb = 32 * P.KG + kPadB;  // P.KG == 2
  const __bf16* ain6 = reinterpret_cast<const __bf16*>(g_smem + in) + (prow0 + cl) * pinb + plane_col(cl, 8 * kq);
  const int qrow0 = (wave / WC) * RB * 16, qwc = wave % WC;
  const int nf = P.N / kFuseNC;
  const int fbsz = fbuf_floats(1) / 2;
  constexpr int fpb = kFuseNC + kPadB;
  // chunk f's weights: P column block 4 f + pwc, k-groups 0, 1; Q column block qwc, k-groups 2 f, 2 f + 1
  bf16x8 wp[2][1][3], wq[2][1][3];
  auto load_p = [&](int f) {
    const bf16x8* s = P.w6 + ((int64_t)(4 * f + pwc) * P.KG) * 3 * 64;
#pragma unroll
    for (int k = 0; k < 2; k++)
#pragma unroll
      for (int p = 0; p < 3; p++) wp[k][0][p] = s[(k * 3 + p) * 64];
  };
  auto load_q = [&](int f) {
    const bf16x8* s = Q.w6 + ((int64_t)qwc * Q.KG + 2 * f) * 3 * 64;
#pragma unroll
    for (int k = 0; k < 2; k++)
#pragma unroll
      for (int p = 0; p < 3; p++) wq[k][0][p] = s[(k * 3 + p) * 64];
  };
  auto p_chunk = [&](int f) {
    f32x4 acc1[1][1];
    zero_acc(acc1);
#pragma unroll
    for (int k = 0; k < 2; k++) mma_kgroup_x6<1, 1>(acc1, ain6 + 32 * k, kP * pinb, 16 * pinb, wp[k]);
    store_cols_planes<1, 1>(acc1, P.bias, 64 * f + 16 * pwc, P.relu, prow0, fbuf + (f & 1) * fbsz, fpb, 16 * pwc);
  };
  f32x4 acc2[RB][1];
  zero_acc(acc2);
  load_p(0);
  load_q(0);
  p_chunk(0);
  if (nf > 1) load_p(1);
  __syncthreads();
  for (int f = 0; f < nf; f++) {
    const __bf16* af6 =
        reinterpret_cast<const __bf16*>(g_smem + fbuf + (f & 1) * fbsz) + (qrow0 + cl) * fpb + plane_col(cl, 8 * kq);
#if NDNET_PN_PAIR_PFIRST
    // A/B: chunk f + 1's P (into the other buffer, free since the last
    // barrier) before chunk f's Q, so its epilogue overlaps other waves' Q
    // MFMAs and the barrier follows the uniform Q phase
    if (f + 1 < nf) {
      p_chunk(f + 1);
      if (f + 2 < nf) load_p(f + 2);
    }
#pragma unroll
    for (int k = 0; k < 2; k++) mma_kgroup_x6<RB, 1>(acc2, af6 + 32 * k, kP * fpb, 16 * fpb, wq[k]);
    if (f + 1 < nf) load_q(f + 1);
#else
#pragma unroll
    for (int k = 0; k < 2; k++) mma_kgroup_x6<RB, 1>(acc2, af6 + 32 * k, kP * fpb, 16 * fpb, wq[k]);
    if (f + 1 < nf) {
      load_q(f + 1);
      p_chunk(f + 1);
      if (f + 2 < nf) load_p(f + 2);
    }
#endif
    __syncthreads();
  }
  if (gmax) pool_cols<RB, 1>(acc2, Q.bias, 16 * qwc, Q.relu, qrow0, rows_valid, gmax);
  else if (out_planes) store_cols_planes<RB, 1>(acc2, Q.bias, 16 * qwc, Q.relu, qrow0, out, Q.N + kPadB, 16 * qwc);
  else store_cols<RB, 1>(acc2, Q.bias, 16 * qwc, Q.relu, qrow0, out, pout, 16 * qwc);
}

// Loads the first weight step this wave runs in layer l (the 16-wave 64-point
// build; others leave pre off): the column block plain_layer<RB, 1> /
// fused_pair's first chunk gives the wave, at k-group 0 -- the address
// run_tiles* would load first.
__device__ inline void prefetch_first(const ndnet_pn_chain& A, int l, int b, Pre& pre) {
  pre.on = false;
#ifndef NDNET_PN_PREFETCH  // off by default: measured 1-2 us slower per chain (profiles/r03e_stamps_ab.txt)
  return;
#endif
  if constexpr (kP == 64 && kWaves == 16) {
    const ndnet_pn_layer& L = A.L[l];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    int cb0;
    if (L.fuse_next) {
      cb0 = wave % 4;  // fused_pair: PWC = 4 column groups of PNB = 1, chunk 0
    } else {
      const int WC = L.N % 256 == 0 ? 16 : L.N % 128 == 0 ? 8 : 4;  // plain_layer<4 | 2 | 1, 1>
      cb0 = wave % WC;
      if (L.N < WC * 16 && cb0 * 16 >= L.N) return;  // an idle wave of a narrow layer
    }
    const int KG = L.prec ? L.K / 32 : L.K / 16;
    const float* wb = L.w + (int64_t)b * L.w_cloud_stride;
    if (L.prec == 1) {
      const bf16x8* q = reinterpret_cast<const bf16x8*>(wb) + lane + (int64_t)cb0 * KG * 3 * 64;
      pre.r0 = __builtin_bit_cast(f32x4, q[0]);
      pre.r1 = __builtin_bit_cast(f32x4, q[64]);
      pre.r2 = __builtin_bit_cast(f32x4, q[128]);
    } else {
      pre.r0 = (reinterpret_cast<const f32x4*>(wb) + lane + (int64_t)cb0 * KG * 64)[0];
    }
    pre.on = true;
  }
}

// The barrier between layers: LDS traffic retired, then s_barrier, with no
// vmcnt drain (__syncthreads' fence waits for every vector-memory op, the
// next layer's prefetched weights included; nothing between layers is a
// global store -- the max-pool atomics come only in the last layer, which
// closes with __syncthreads).
__device__ inline void layer_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Floats of LDS region r: fp32 activations (pitch width + kPadF) or, when it ever
// holds a split-bf16 layer's input (planes bit r), three bf16 planes.
__host__ __device__ inline int region_floats(int width, int planes) {
  const int f32 = kP * (width + kPadF), b16 = 3 * kP * (width + kPadB) / 2;
  return planes && b16 > f32 ? b16 : f32;
}

// Layer 0 of the chains (conv1 of ndtnet.py:47 / :148, K = 3 or 12 inputs
// padded to 16, N = 64) runs on the VALU straight from the input rows: each
// thread computes 4 channels of one point from the point's 12 input floats
// (three dwordx4 loads) and W0^T staged in LDS row-major ([16][64]) -- no
// input tile, no MFMA fragment loads, one memory round trip for x, W0, every
// layer's bias and (chain B) the TNet(3) tail.  The products are fp32 FMAs
// (k ascending); the MFMA path computed the same sums in another order.
__host__ __device__ inline bool valu_layer0(const ndnet_pn_chain& A) {
#ifdef NDNET_PN_NO_VALU0  // A/B: layer 0 on the MFMA path from an LDS input tile
  return false;
#endif
  return A.num_layers > 1 && A.L[0].K == 16 && A.L[0].N == 64 && A.L[0].prec == 0 && !A.L[0].fuse_next &&
         A.in_cols <= 12 && A.x_ld % 4 == 0;
}

// LDS floats of the VALU layer-0 prologue scratch (W0^T [16][64] + bias [64]),
// overlaid on activation region 0, which layer 0 neither reads nor writes.
constexpr int kValu0Floats = 16 * 64 + 64;

// Floats of activation region 0 (kernel and launcher): room for the layer-0
// prologue's scratch (+ chain B's t1) when layer 0 runs on the VALU.
__host__ __device__ inline int region0_floats(const ndnet_pn_chain& A, int planes) {
  const int r = region_floats(A.max_width, planes & 1);
  return valu_layer0(A) && r < kValu0Floats + 16 ? kValu0Floats + 16 : r;
}

__global__ void __launch_bounds__(kThreads) k_pn_chain(ndnet_pn_chain A, int planes, int fbuf, int bias_base) {
  const int b = blockIdx.y;
  const int p0 = blockIdx.x * kP;
  PN_STAMP(0);
  // LDS: activation region 0 | region 1 | [fused-chunk double buffer] | biases of layers 1..
  const int pitch0 = A.max_width + kPadF, pitch1 = A.max_width2 + kPadF;
  const int reg[2] = {0, region0_floats(A, planes)};
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // every layer's bias (this cloud's) -> LDS at boff[l] (layer 0's into the
  // prologue scratch when it runs on the VALU); the loads are issued together
  // with the prologue's, so the epilogues never wait on a global bias read
  int boff[NDNET_PN_MAX_LAYERS];
  {
    int o = bias_base;
#pragma unroll
    for (int l = 0; l < NDNET_PN_MAX_LAYERS; l++) {
      boff[l] = o;
      if (l < A.num_layers) o += A.L[l].N;
    }
    float bv[NDNET_PN_MAX_LAYERS][2];
#pragma unroll
    for (int l = 0; l < NDNET_PN_MAX_LAYERS; l++)
#pragma unroll
      for (int i = 0; i < 2; i++) {
        const int e = threadIdx.x + i * kThreads;
        bv[l][i] = (l < A.num_layers && e < A.L[l].N) ? A.L[l].bias[(int64_t)b * A.L[l].bias_cloud_stride + e] : 0.0f;
      }
#pragma unroll
    for (int l = 0; l < NDNET_PN_MAX_LAYERS; l++)
#pragma unroll
      for (int i = 0; i < 2; i++) {
        const int e = threadIdx.x + i * kThreads;
        if (l < A.num_layers && e < A.L[l].N) g_smem[boff[l] + e] = bv[l][i];
      }
  }
  const bool v0 = valu_layer0(A);
  Pre pre;  // the next layer's first weight step (prefetched before each layer barrier)
  prefetch_first(A, v0 ? 1 : 0, b, pre);
  float* const s_w0 = g_smem;  // v0: W0^T [16][64] row-major, in region 0
  // v0: this thread's point rows (t / 16 + pass * kThreads / 16) and 4 output
  // channels (4 (t % 16) ..)
  constexpr int kV0Pass = kP * 16 / kThreads;
  static_assert(kV0Pass >= 1 && kV0Pass * kThreads == kP * 16, "whole layer-0 passes");
  const int vq = threadIdx.x & 15;
  f32x4 xin[kV0Pass][3] = {};
  if (v0) {
#pragma unroll
    for (int ps = 0; ps < kV0Pass; ps++) {
      const int vr = (threadIdx.x >> 4) + ps * (kThreads / 16);
      const int p = p0 + vr;
      if (p < A.num_points) {
        const f32x4* xr = reinterpret_cast<const f32x4*>(A.x + ((int64_t)b * A.num_points + p) * A.x_ld);
#pragma unroll
        for (int i = 0; i < 3; i++)
          if (4 * i < A.in_cols) xin[ps][i] = xr[i];
      }
    }
    if (!A.head_h2 && threadIdx.x < 256) {  // W0^T fragment-major [cb][kq][cl][s] -> row-major [k][n]
      const f32x4 wv = reinterpret_cast<const f32x4*>(A.L[0].w + (int64_t)b * A.L[0].w_cloud_stride)[threadIdx.x];
      const int cb = threadIdx.x >> 6, kq = (threadIdx.x >> 4) & 3, cl = threadIdx.x & 15;
#pragma unroll
      for (int s = 0; s < 4; s++) s_w0[(4 * kq + s) * 64 + 16 * cb + cl] = wv[s];
    }
  }
  if (A.head_h2) {
    // TNet(3)'s tail for this cloud (ndnet_pn_head3_run's work, ndtnet.py:57-60):
    // t1 = h2 @ W3^T + b3, then conv1 with t1 folded into layer 0's weights
    float* const s_t1 = g_smem + (v0 ? kValu0Floats : 0);  // [9] (v0: past the scratch; region 0 is free until layer 1)
    const int M = A.head_kin * A.head_nout, total = 16 * A.head_nout;  // one k-group, K padded to 16
    // this thread's fold element(s): basis values loaded ahead of the fc3 reduction
    const int e0 = threadIdx.x;
    const int cb0 = e0 >> 8, ln0 = (e0 >> 2) & 63, k0 = 4 * (ln0 >> 4) + (e0 & 3), n0 = 16 * cb0 + (ln0 & 15);
    float bas[9];
#pragma unroll
    for (int a = 0; a < 9; a++) bas[a] = (e0 < total && k0 < A.head_kin) ? A.head_basis[a * M + k0 * A.head_nout + n0] : 0.0f;
    const float* h = A.head_h2 + (int64_t)b * A.head_ld;
    for (int o = wave; o < 9; o += kWaves) {  // one wave per output, lanes split K
      float acc = 0.0f;
      const float* wr = A.head_w3 + (int64_t)o * A.head_K;
      if (A.head_K == 256) {  // one float4 of h and of the row per lane: one load round trip
        const f32x4 hv = reinterpret_cast<const f32x4*>(h)[lane];
        const f32x4 wv = reinterpret_cast<const f32x4*>(wr)[lane];
        acc = (hv[0] * wv[0] + hv[1] * wv[1]) + (hv[2] * wv[2] + hv[3] * wv[3]);
      } else {
        for (int k = lane; k < A.head_K; k += 64) acc += h[k] * wr[k];
      }
      for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
      if (lane == 0) {
        s_t1[o] = acc + A.head_b3[o];
        if (blockIdx.x == 0) A.head_t1[b * 9 + o] = acc + A.head_b3[o];
      }
    }
    __syncthreads();
    float* w1 = const_cast<float*>(A.L[0].w) + (int64_t)b * A.L[0].w_cloud_stride;
    // v0: only the cloud's first workgroup publishes the fragment-major W0^T
    // (chains C and D read it in later launches); every workgroup keeps its own
    // copy in LDS.  Otherwise every workgroup stores it and its layer 0 reads it.
    const bool publish = !v0 || blockIdx.x == 0;
    for (int e = e0; e < total; e += kThreads) {
      const int cb = e >> 8, ln = (e >> 2) & 63, k = 4 * (ln >> 4) + (e & 3), n = 16 * cb + (ln & 15);
      float acc = 0.0f;
      if (e == e0) {
#pragma unroll
        for (int a = 0; a < 9; a++) acc += s_t1[a] * bas[a];
      } else if (k < A.head_kin) {
#pragma unroll
        for (int a = 0; a < 9; a++) acc += s_t1[a] * A.head_basis[a * M + k * A.head_nout + n];
      }
      if (publish) w1[e] = acc;
      if (v0) s_w0[k * 64 + n] = acc;
    }
    // !v0: layer 0 reads these weights back: __syncthreads' workgroup-scope release
    // / acquire orders this workgroup's stores before its loads (same CU; no
    // lines of them are cached here yet).  Every workgroup of the cloud stores
    // the same bits.  (A device-scope __threadfence here writes back the L2:
    // measured +60 us per launch.)
    PN_STAMP(1);
  }
  if (A.fold_t2) {
    // TNet(64)'s transform through layer 0 (chains C, D; v0 only, checked on
    // the host): x_t2 = t2^T (W0 x + b0) = (W0^T t2)^T x + t2^T b0, so layer 0
    // runs on W0' = W0^T t2 (its 12 used rows) and b0' = b0^T t2: a 16 x 64 x 64
    // GEMM (rows 0..11 W0^T, row 12 the bias, 13..15 zero) on the fp32 MFMA,
    // waves 0..3 one 16-column block each, t2 staged in region 1 (layer 0 has
    // not written it yet; the launcher keeps the biases past it)
    float* const s_t2 = g_smem + reg[1];
    const f32x4* t2b = reinterpret_cast<const f32x4*>(A.fold_t2 + (int64_t)b * A.fold_ld);
    for (int e = threadIdx.x; e < 1024; e += kThreads) reinterpret_cast<f32x4*>(s_t2)[e] = t2b[e];
    __syncthreads();  // + s_w0 (W0^T row-major) and layer 0's bias at boff[0]
    f32x4 fo = {0.f, 0.f, 0.f, 0.f};
    const int fr = lane & 15, fk = lane >> 4;  // operand row / k within a 4-step
    if (wave < 4) {
#pragma unroll
      for (int st = 0; st < 16; st++) {
        const int i = 4 * st + fk;
        const float av = fr < 12 ? s_w0[fr * 64 + i] : fr == 12 ? g_smem[boff[0] + i] : 0.0f;
        const float bv = s_t2[i * 64 + 16 * wave + fr];
        fo = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, fo, 0, 0, 0);
      }
    }
    __syncthreads();
    if (wave < 4) {  // lane (fk, fr): rows 4 fk + r, column 16 wave + fr
      const int n = 16 * wave + fr;
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int row = 4 * fk + r;
        if (row < 12) s_w0[row * 64 + n] = fo[r];
        else if (row == 12) g_smem[boff[0] + n] = fo[r];
      }
      // the cloud's first workgroup publishes W0' (fragment-major, K = 16, rows
      // 12..15 left zero) and b0' for a later chain's plain layer 0 (chain D)
      if (A.fold_out_w && blockIdx.x == 0) {
        float* ow = A.fold_out_w + (int64_t)b * 1024;
#pragma unroll
        for (int r = 0; r < 4; r++) {
          const int row = 4 * fk + r;
          if (row < 12) ow[(((n >> 4) * 64 + ((row >> 2) & 3) * 16 + (n & 15)) << 2) + (row & 3)] = fo[r];
          else if (row == 12) A.fold_out_b[(int64_t)b * 64 + n] = fo[r];
        }
      }
    }
    PN_STAMP(1);  // (timing builds) chains C / D: t2 staged and folded into layer 0
  }
  __syncthreads();
  if (v0) {
    // layer 0: out = act(x W0^T + b0) for 4 channels of one point, into region 1
    // as the next layer reads it (three bf16 planes, or fp32)
#pragma unroll
    for (int ps = 0; ps < kV0Pass; ps++) {
      const int vr = (threadIdx.x >> 4) + ps * (kThreads / 16);
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      const float xs[12] = {xin[ps][0][0], xin[ps][0][1], xin[ps][0][2], xin[ps][0][3], xin[ps][1][0], xin[ps][1][1],
                            xin[ps][1][2], xin[ps][1][3], xin[ps][2][0], xin[ps][2][1], xin[ps][2][2], xin[ps][2][3]};
#pragma unroll
      for (int k = 0; k < 12; k++) {
        if (k < A.in_cols) {
          const f32x4 w = *reinterpret_cast<const f32x4*>(s_w0 + k * 64 + 4 * vq);
#pragma unroll
          for (int j = 0; j < 4; j++) acc[j] = fmaf(xs[k], w[j], acc[j]);
        }
      }
      const f32x4 bb = *reinterpret_cast<const f32x4*>(g_smem + boff[0] + 4 * vq);
#pragma unroll
      for (int j = 0; j < 4; j++) {
        acc[j] += bb[j];
        if (A.L[0].relu) acc[j] = fmaxf(acc[j], 0.0f);
      }
      const int out = reg[1];
      if (A.L[1].prec) {  // three bf16 planes, pitch 64 + kPadB
        typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
        const int pb = 64 + kPadB;
        __bf16* const base = reinterpret_cast<__bf16*>(g_smem + out) + vr * pb + plane_col(vr, 4 * vq);
        bf16x4 h4, m4, l4;
#pragma unroll
        for (int j = 0; j < 4; j++) {
          __bf16 hh, mm, ll;
          split3(acc[j], hh, mm, ll);
          h4[j] = hh;
          m4[j] = mm;
          l4[j] = ll;
        }
        *reinterpret_cast<bf16x4*>(base) = h4;
        *reinterpret_cast<bf16x4*>(base + kP * pb) = m4;
        *reinterpret_cast<bf16x4*>(base + 2 * kP * pb) = l4;
      } else {
        *reinterpret_cast<f32x4*>(g_smem + out + vr * pitch1 + 4 * vq) = acc;
      }
    }
  } else {
    const int K0 = A.L[0].K;
    for (int e = threadIdx.x; e < kP * K0; e += kThreads) {
      const int r = e / K0, c = e % K0;
      const int p = p0 + r;
      float v = 0.0f;
      if (p < A.num_points && c < A.in_cols) v = A.x[((int64_t)b * A.num_points + p) * A.x_ld + c];
      g_smem[r * pitch0 + c] = v;
    }
  }
  __syncthreads();
  PN_STAMP(2);
  const int rows_valid = A.num_points - p0;
  float* const gmax_b = A.mode == 0 ? A.gmax + (int64_t)b * A.gmax_ld : nullptr;
  for (int l = v0 ? 1 : 0; l < A.num_layers; l++) {
    const int in = reg[l & 1], pin = (l & 1) ? pitch1 : pitch0;
    if (A.L[l].fuse_next) {  // layers l and l + 1 together; l + 1 writes region (l + 2) & 1
      const LayerCtx P = layer_ctx(A, l, b, g_smem + boff[l]), Q = layer_ctx(A, l + 1, b, g_smem + boff[l + 1]);
      const bool last = l + 2 == A.num_layers;
      const int out = reg[(l + 2) & 1], pout = ((l + 2) & 1) ? pitch1 : pitch0;
      float* gm = (last && gmax_b) ? gmax_b : nullptr;
      // Q is one chunk of its (RB, NB) split: NB = N2 / (16 * column groups)
      constexpr int kQ = 16 / kWaves > 0 ? 16 / kWaves : 1;
      const bool op = !last && A.L[l + 2].prec;  // the layer after Q reads bf16 planes
      if constexpr (kP == 32) {  // two row blocks: each Q split with half the row groups
        if (Q.N == 256) fused_pair<2, kQ>(P, Q, in, pin, fbuf, out, pout, gm, rows_valid, op);
        else fused_pair<1, kQ>(P, Q, in, pin, fbuf, out, pout, gm, rows_valid, op);
      } else {
#ifndef NDNET_PN_FUSED_PIPE
#define NDNET_PN_FUSED_PIPE 1
#endif
        bool piped = false;
        if constexpr (kWaves == 16) {
          if (NDNET_PN_FUSED_PIPE && Q.N == 256 && P.prec && Q.prec && P.KG == 2) {
            fused_pair_x6p<4>(P, Q, in, fbuf, out, pout, gm, rows_valid, op);
            piped = true;
          }
        }
        if (piped) {
        } else if (Q.N == 256) fused_pair<4, kQ>(P, Q, in, pin, fbuf, out, pout, gm, rows_valid, op, pre);
        else if (Q.N > 64) fused_pair<2, kQ>(P, Q, in, pin, fbuf, out, pout, gm, rows_valid, op, pre);
        else fused_pair<1, kQ>(P, Q, in, pin, fbuf, out, pout, gm, rows_valid, op, pre);
      }
      l++;
    } else {
      const LayerCtx C = layer_ctx(A, l, b, g_smem + boff[l]);
      const bool last = l + 1 == A.num_layers;
      const int out = reg[(l + 1) & 1], pout = ((l + 1) & 1) ? pitch1 : pitch0;
      float* gm = (last && gmax_b) ? gmax_b : nullptr;
      const bool op = !last && A.L[l + 1].prec;  // the next layer reads bf16 planes
      if constexpr (kP == 32) {
        // 32-point tiles, 8 waves: two row blocks, columns per wave as the
        // 64-point form's (one row group, all waves across the columns)
        if (C.N % 256 == 0) plain_layer<2, 2>(C, in, pin, out, pout, gm, rows_valid, op);
        else if (C.N % 128 == 0) plain_layer<2, 1>(C, in, pin, out, pout, gm, rows_valid, op);
        else plain_layer<1, 1>(C, in, pin, out, pout, gm, rows_valid, op);  // N % 64 == 0, or N = 32 (half idle)
      } else if constexpr (kWaves == 8) {
        // 8 waves (2 per SIMD, up to 256 registers each): a wave takes up to
        // four column blocks, so each A fragment feeds NB MFMAs per plane
        // (tools/ubench/mfma_bf16_peak.hip b9 / b13 vs b3)
#ifndef NDNET_PN_W8_NB4
#define NDNET_PN_W8_NB4 1
#endif
        if (NDNET_PN_W8_NB4 && C.N % 512 == 0) plain_layer<4, 4>(C, in, pin, out, pout, gm, rows_valid, op);
        else if (C.N % 256 == 0) plain_layer<4, 2>(C, in, pin, out, pout, gm, rows_valid, op);
        else if (C.N % 128 == 0) plain_layer<4, 1>(C, in, pin, out, pout, gm, rows_valid, op);
        else if (C.N % 64 == 0) plain_layer<2, 1>(C, in, pin, out, pout, gm, rows_valid, op);
        else plain_layer<1, 1>(C, in, pin, out, pout, gm, rows_valid, op);  // N = 32
      } else {
#ifndef NDNET_PN_NB2  // two column blocks per wave on the 1024-wide x6 layers (-5% per layer, r03q)
#define NDNET_PN_NB2 1
#endif
        if (NDNET_PN_NB2 && C.N % 512 == 0 && C.prec) plain_layer<4, 2>(C, in, pin, out, pout, gm, rows_valid, op, pre);
        else if (C.N % 256 == 0) plain_layer<4, 1>(C, in, pin, out, pout, gm, rows_valid, op, pre);
        else if (C.N % 128 == 0) plain_layer<2, 1>(C, in, pin, out, pout, gm, rows_valid, op, pre);
        else plain_layer<1, 1>(C, in, pin, out, pout, gm, rows_valid, op, pre);  // N % 64 == 0, or N = 32 (half idle)
      }
    }
#ifdef NDNET_PN_PREFETCH
    if (l + 1 < A.num_layers) {
      prefetch_first(A, l + 1, b, pre);
      layer_barrier();
    } else {
      __syncthreads();
    }
#elif defined(NDNET_PN_LBAR)  // A/B: the layer barrier without the vmcnt drain, no prefetch
    if (l + 1 < A.num_layers) layer_barrier();
    else __syncthreads();
#else
    __syncthreads();
#endif
    PN_STAMP(3 + l);
  }
  if (A.clear && blockIdx.x == 0 && blockIdx.y == 0)
    for (int64_t i = threadIdx.x; i < A.clear_count; i += kThreads) A.clear[i] = -INFINITY;
  if (A.mode == 1) {  // log_softmax over channels (ndtnet.py:239), [B][N][C+1] layout
    const int lg = reg[A.num_layers & 1];
    const int pl = (A.num_layers & 1) ? pitch1 : pitch0;
    // 16 lanes per point (a quarter wave): columns q, q + 16, ...; the max
    // and the sum of exponentials meet in xor shuffles within the group
    constexpr int kLpr = 16, kRpp = kThreads / kLpr;  // lanes per row, rows per pass
    const int q = threadIdx.x % kLpr;
    for (int r0 = 0; r0 < kP; r0 += kRpp) {
      const int r = r0 + threadIdx.x / kLpr;
      const int p = p0 + r;
      const bool live = r < kP && p < A.num_points;  // uniform per 16-lane group
      const float* row = g_smem + lg + (r < kP ? r : 0) * pl;
      float m = -INFINITY;
      for (int c = q; c < A.out_cols; c += kLpr) m = fmaxf(m, row[c]);
#pragma unroll
      for (int o = kLpr / 2; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
      float sum = 0.0f;
      for (int c = q; c < A.out_cols; c += kLpr) sum += expf(row[c] - m);
#pragma unroll
      for (int o = kLpr / 2; o > 0; o >>= 1) sum += __shfl_xor(sum, o, 64);
      const float ls = logf(sum);
      if (live) {
        float* out = A.out + ((int64_t)b * A.num_points + p) * A.out_cols;
        for (int c = q; c < A.out_cols; c += kLpr) out[c] = (row[c] - m) - ls;
      }
    }
  }
  PN_STAMP(15);
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

// The same FC layer on the fp32 matrix cores: a 16-row GEMM (row = cloud,
// b < B <= 16) with W^T fragment-major (the chain layout, [cb][kg][lane][4]).
// One workgroup per 16-column block; its kFcWaves waves (8: measured best in the
// pipelined step, 16 slowed it) split the K-groups,
// each wave's weight fragments (1 KB each) and input pieces (a float4 of 4
// consecutive k per lane) loaded up front -- one memory round trip per
// launch -- then 4 MFMAs per k-group; the waves' 16 x 16 partial tiles are
// summed in LDS in wave order (deterministic) and wave 0 adds the bias.
// Products are exact and sums fp32, as torch's fp32 GEMM (another order).
#ifndef NDNET_PN_FC_WAVES
#define NDNET_PN_FC_WAVES 8
#endif
constexpr int kFcWaves = NDNET_PN_FC_WAVES, kFcMaxG = 64 / kFcWaves;  // K <= 16 * kFcWaves * kFcMaxG = 1024
// CBW column blocks per workgroup (round 6): a wide, shallow layer (TNet(64)'s
// fc3, 256 -> 4096: 256 one-block workgroups, ~5 us each, the whole chip for
// its duration in the pipelined step) runs as 64 four-block workgroups, each
// wave holding CBW x ng weight fragments (ng * CBW <= kFcMaxG registers'
// worth, the host checks) -- the same per-column sums in the same order, so
// the output is bit-identical for every CBW; only the CU-time shrinks.
template <int CBW>
__global__ void __launch_bounds__(kFcWaves * 64) k_pn_fc_mfma(const float* __restrict__ in, int ld_in,
                                                              const f32x4* __restrict__ wf,
                                                              const float* __restrict__ bias, float* __restrict__ out,
                                                              int ld_out, int B, int KG, int relu) {
  constexpr int kG = kFcMaxG / CBW;
  static_assert(CBW <= kFcWaves && kG >= 1, "one reducing wave per column block");
  __shared__ f32x4 part[kFcWaves][CBW][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int kq = lane >> 4, cl = lane & 15;
  const int cb0 = blockIdx.x * CBW;
  const int kg0 = KG * wave / kFcWaves, ng = KG * (wave + 1) / kFcWaves - kg0;
  const float* xr = in + (int64_t)(cl < B ? cl : 0) * ld_in + 16 * kg0 + 4 * kq;  // rows past B: discarded
  f32x4 wv[CBW][kG], xv[kG];
#pragma unroll
  for (int i = 0; i < kG; i++) {
    if (i < ng) {
      xv[i] = *reinterpret_cast<const f32x4*>(xr + 16 * i);
#pragma unroll
      for (int j = 0; j < CBW; j++) wv[j][i] = wf[((int64_t)(cb0 + j) * KG + kg0 + i) * 64 + lane];
    }
  }
#pragma unroll
  for (int j = 0; j < CBW; j++) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < kG; i++)
      if (i < ng)
#pragma unroll
        for (int s = 0; s < 4; s++) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(xv[i][s], wv[j][i][s], acc, 0, 0, 0);
    part[wave][j][lane] = acc;
  }
  __syncthreads();
  if (wave >= CBW) return;
  const int j = wave;  // wave j reduces column block cb0 + j over the waves in order
  f32x4 t = part[0][j][lane];
#pragma unroll
  for (int w = 1; w < kFcWaves; w++) t += part[w][j][lane];
  // lane (kq, cl): clouds 4 kq + r of column 16 (cb0 + j) + cl
  const int n = 16 * (cb0 + j) + cl;
  const float bv = bias[n];
#pragma unroll
  for (int r = 0; r < 4; r++) {
    const int b = 4 * kq + r;
    if (b < B) {
      float v = t[r] + bv;
      if (relu) v = fmaxf(v, 0.0f);
      out[(int64_t)b * ld_out + n] = v;
    }
  }
}

// Index of W^T element (k, n) in the fragment-major layout (KG k-groups).
__device__ inline int64_t frag_index(int k, int n, int KG) {
  return ((int64_t)((n >> 4) * KG + (k >> 4)) * 64 + ((k >> 2) & 3) * 16 + (n & 15)) * 4 + (k & 3);
}

// The same GEMV with K split across the lanes of WPO waves (K = 256 WPO,
// WPO = 2 or 4; at K = 256 the one-wave kernel above measured faster): every thread loads ONE float4 of the weight row and the
// matching float4 of all B inputs up front -- a single memory round trip
// per launch instead of one per K-chunk of 64 lanes -- then the partial sums
// of the 16 clouds are reduced across the wave (shuffles) and the WPO waves
// (LDS).  4 / WPO output channels per 256-thread workgroup.
template <int WPO>
__global__ void __launch_bounds__(256) k_pn_fc_split(const float* __restrict__ in, int ld_in,
                                                     const float* __restrict__ W, const float* __restrict__ bias,
                                                     float* __restrict__ out, int ld_out, int B, int N, int relu) {
  constexpr int K = 256 * WPO, OPW = 4 / WPO;
  __shared__ float s_part[4][16];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int o = wave / WPO, wq = wave % WPO;  // output within the workgroup, K quarter of that output
  const int n = blockIdx.x * OPW + o;
  const int nn = n < N ? n : N - 1;
  const int c4 = wq * 64 + lane;  // this thread's float4 of the row
  const f32x4 wv = reinterpret_cast<const f32x4*>(W + (int64_t)nn * K)[c4];
  f32x4 xv[16];
#pragma unroll
  for (int b = 0; b < 16; b++) xv[b] = reinterpret_cast<const f32x4*>(in + (int64_t)(b < B ? b : 0) * ld_in)[c4];
  float acc[16];
#pragma unroll
  for (int b = 0; b < 16; b++) {
    const f32x4 pr = xv[b] * wv;
    acc[b] = (pr[0] + pr[1]) + (pr[2] + pr[3]);
  }
#pragma unroll
  for (int b = 0; b < 16; b++)
    for (int off = 32; off > 0; off >>= 1) acc[b] += __shfl_xor(acc[b], off, 64);
  if (WPO > 1) {
    if (lane < 16) {
      float v = 0.0f;
#pragma unroll
      for (int b = 0; b < 16; b++) v = lane == b ? acc[b] : v;
      s_part[wave][lane] = v;
    }
    __syncthreads();
    if (wq != 0) return;
    if (lane < 16) {
      float v = 0.0f;
#pragma unroll
      for (int q = 0; q < WPO; q++) v += s_part[wave + q][lane];
      acc[0] = v;
    }
  } else if (lane < 16) {
    float v = 0.0f;
#pragma unroll
    for (int b = 0; b < 16; b++) v = lane == b ? acc[b] : v;
    acc[0] = v;
  }
  if (lane < B && n < N) {
    float v = acc[0] + bias[n];
    if (relu) v = fmaxf(v, 0.0f);
    out[(int64_t)lane * ld_out + n] = v;
  }
}

// TNet(64)'s transform through conv1 for chains C and D (ndtnet.py:152-155,
// x_t2 = t2^T (W1' x + b1)): W1''[b] = W1'[b]^T t2[b] (12 x 64) and b1''[b] =
// b1^T t2[b], once per cloud, written as chains C / D read their layer 0
// (fragment-major, K padded to 16, rows 12..15 left as they are: zero) and
// the per-cloud bias.  fp32 FMAs in i order.  (Before round 5 every chain-C
// workgroup computed it in its prologue on the fp32 MFMA: 16 workgroups per
// cloud doing the same 16 x 64 x 64 product, ~2 us of each one's time.)
__global__ void __launch_bounds__(1024) k_pn_fold_t2(const float* __restrict__ w1f, int w1_stride,
                                                     const float* __restrict__ b1, const float* __restrict__ t2,
                                                     int t2_ld, float* __restrict__ outf, float* __restrict__ outb) {
  const int b = blockIdx.x, e = threadIdx.x;
  __shared__ float s_w[13 * 64];  // rows 0..11 W1'^T (row-major [k][n]), row 12 the bias
  __shared__ float s_t[64 * 64];
  {
    const float* wb = w1f + (int64_t)b * w1_stride;
    if (e < 16 * 64) {  // fragment-major element e -> (k, n)
      const int cb = e >> 8, ln = (e >> 2) & 63, k = 4 * (ln >> 4) + (e & 3), n = 16 * cb + (ln & 15);
      const float v = wb[e];
      if (k < 12) s_w[k * 64 + n] = v;
    }
    if (e < 64) s_w[12 * 64 + e] = b1[e];
    const f32x4* tb = reinterpret_cast<const f32x4*>(t2 + (int64_t)b * t2_ld);
    reinterpret_cast<f32x4*>(s_t)[e] = tb[e];  // 1024 threads x 4 = the 64 x 64 matrix
  }
  __syncthreads();
  if (e < 13 * 64) {
    const int r = e >> 6, n = e & 63;
    float acc = 0.0f;
#pragma unroll 16
    for (int i = 0; i < 64; i++) acc = fmaf(s_w[r * 64 + i], s_t[i * 64 + n], acc);
    if (r < 12) outf[(int64_t)b * 1024 + ((((n >> 4) * 64 + ((r >> 2) & 3) * 16 + (n & 15)) << 2) + (r & 3))] = acc;
    else outb[(int64_t)b * 64 + n] = acc;
  }
}

// TNet(3) tail: t1[b] = fc3(h2[b]) (+ I, folded into the bias) and the t1
// fold of conv1, W1'^T[b] = t1[b] (1 x 9) @ basis (9 x kin*nout), written
// fragment-major with K padded to 16 (rows kin..15 zero).  One workgroup per cloud.
__global__ void __launch_bounds__(256) k_pn_head3(const float* __restrict__ h2, int ld_h, const float* __restrict__ W3,
                                                  const float* __restrict__ b3, const float* __restrict__ basis,
                                                  float* __restrict__ t1_out, float* __restrict__ w1f, int K, int kin,
                                                  int nout) {
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
  const int M = kin * nout, total = 16 * nout;  // one k-group
  // fragment-major position e -> (k, n); the first kE positions of every
  // thread have their basis values loaded before the barrier, behind fc3
  auto kn = [&](int e, int& k, int& n) {
    const int cb = e >> 8, ln = (e >> 2) & 63;
    k = 4 * (ln >> 4) + (e & 3);
    n = 16 * cb + (ln & 15);
  };
  constexpr int kE = 4;
  float bas[kE][9];
#pragma unroll
  for (int i = 0; i < kE; i++) {
    const int e = threadIdx.x + i * blockDim.x;
    int k, n;
    kn(e, k, n);
#pragma unroll
    for (int a = 0; a < 9; a++) bas[i][a] = (e < total && k < kin) ? basis[a * M + k * nout + n] : 0.0f;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < kE; i++) {
    const int e = threadIdx.x + i * blockDim.x;
    if (e < total) {
      float acc = 0.0f;
#pragma unroll
      for (int a = 0; a < 9; a++) acc += s_t[a] * bas[i][a];
      w1f[(int64_t)b * total + e] = acc;
    }
  }
  for (int e = threadIdx.x + kE * blockDim.x; e < total; e += blockDim.x) {
    int k, n;
    kn(e, k, n);
    float acc = 0.0f;
    if (k < kin) {
#pragma unroll
      for (int a = 0; a < 9; a++) acc += s_t[a] * basis[a * M + k * nout + n];
    }
    w1f[(int64_t)b * total + e] = acc;
  }
}

#if NDNET_PN_TILE == 64
// ---- the BatchNorm fold, in place (ndnet_pn_fold_run, include/ndnet_pointnet.h) ----
// HBM-bound copy work (~14 MB read, ~40 MB written for the F = 1024 model):
// each thread writes one unit (4 fp32 of a fragment, 8 bf16 of each split
// plane, else one float), so every output row is written with full-width,
// contiguous stores; the strided weight reads hit L2.
constexpr int kFoldThreads = 256;

__device__ inline uint16_t fold_bf16(float x) {  // torch's float -> bfloat16: round to nearest even
  uint32_t u = __float_as_uint(x);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40u);
  return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}

__device__ inline float fold_w(const ndnet_pn_fold_job& J, int n, int k) {
#pragma clang fp contract(off)
  if (n >= J.N || k >= J.K) return 0.0f;
  const float w = J.w[(int64_t)n * J.ld + J.k0 + k];
  if (!J.gamma) return w;
  return w * (J.gamma[n] / sqrtf(J.var[n] + J.eps));  // pointnet_hip._bn_fold, operation by operation
}

__host__ __device__ inline int64_t fold_units(const ndnet_pn_fold_job& J) {
  switch (J.kind) {
    case NDNET_FOLD_WT: return (int64_t)J.Kp * J.Np;
    case NDNET_FOLD_FRAG: return (int64_t)J.Kp * J.Np / 4;
    case NDNET_FOLD_FRAG6: return (int64_t)J.Kp * J.Np / 8;
    case NDNET_FOLD_ROWS: return (int64_t)J.N * J.K;
    case NDNET_FOLD_BASIS: return (int64_t)9 * J.K * J.N;
    default: return J.Np;
  }
}

__global__ void __launch_bounds__(kFoldThreads) k_pn_fold(const ndnet_pn_fold_job* __restrict__ jobs, int num_jobs) {
#pragma clang fp contract(off)
  int j = 0;  // this workgroup's job: the last one starting at or before it (block0 ascends)
  for (int i = 1; i < num_jobs; i++)
    if (jobs[i].block0 <= (int64_t)blockIdx.x) j = i;
  const ndnet_pn_fold_job J = jobs[j];
  const int64_t u = ((int64_t)blockIdx.x - J.block0) * kFoldThreads + threadIdx.x;
  if (u >= fold_units(J)) return;
  switch (J.kind) {
    case NDNET_FOLD_WT: {
      const int n = (int)(u % J.Np), k = (int)(u / J.Np);
      static_cast<float*>(J.out)[u] = fold_w(J, n, k);
      break;
    }
    case NDNET_FOLD_FRAG: {  // [cb][kg][kq][cl][s]: k = 16 kg + 4 kq + s, n = 16 cb + cl
      const int kgs = J.Kp / 16;
      const int cl = (int)(u % 16), kq = (int)(u / 16 % 4), kg = (int)(u / 64 % kgs), cb = (int)(u / (64 * kgs));
      const int k = 16 * kg + 4 * kq, n = 16 * cb + cl;
      f32x4 v = {fold_w(J, n, k), fold_w(J, n, k + 1), fold_w(J, n, k + 2), fold_w(J, n, k + 3)};
      reinterpret_cast<f32x4*>(J.out)[u] = v;
      break;
    }
    case NDNET_FOLD_FRAG6: {  // [cb][kg][plane][kq][cl][j]: k = 32 kg + 8 kq + j, n = 16 cb + cl
      const int kgs = J.Kp / 32;
      const int cl = (int)(u % 16), kq = (int)(u / 16 % 4), kg = (int)(u / 64 % kgs), cb = (int)(u / (64 * kgs));
      const int k = 32 * kg + 8 * kq, n = 16 * cb + cl;
      uint32_t p[3][4];
#pragma unroll
      for (int t = 0; t < 8; t += 2) {
        uint16_t hv[2], mv[2], lv[2];
#pragma unroll
        for (int e = 0; e < 2; e++) {
          const float w = fold_w(J, n, k + t + e);
          hv[e] = fold_bf16(w);
          const float r = w - __uint_as_float((uint32_t)hv[e] << 16);
          mv[e] = fold_bf16(r);
          lv[e] = fold_bf16(r - __uint_as_float((uint32_t)mv[e] << 16));
        }
        p[0][t / 2] = hv[0] | ((uint32_t)hv[1] << 16);
        p[1][t / 2] = mv[0] | ((uint32_t)mv[1] << 16);
        p[2][t / 2] = lv[0] | ((uint32_t)lv[1] << 16);
      }
      const int64_t unit = u % 64 + (u / 64) * 192;  // 64 units per (cb, kg), three planes of them
      uint4* o = reinterpret_cast<uint4*>(J.out);
#pragma unroll
      for (int pl = 0; pl < 3; pl++) o[unit + 64 * pl] = make_uint4(p[pl][0], p[pl][1], p[pl][2], p[pl][3]);
      break;
    }
    case NDNET_FOLD_ROWS: {
      const int n = (int)(u / J.K), k = (int)(u % J.K);
      static_cast<float*>(J.out)[u] = fold_w(J, n, k);
      break;
    }
    case NDNET_FOLD_BASIS: {  // out[3a + c][r][n]: r < 3 the point (t1 p), else the covariance rows (t1 C)
      const int n = (int)(u % J.N), r = (int)(u / J.N % J.K), ac = (int)(u / ((int64_t)J.N * J.K));
      const int a = ac / 3, c = ac % 3;
      float v = 0.0f;
      if (r < 3) {
        if (r == c) v = fold_w(J, n, a);
      } else if ((r - 3) / 3 == c) {
        v = fold_w(J, n, 3 + 3 * a + (r - 3) % 3);
      }
      static_cast<float*>(J.out)[u] = v;
      break;
    }
    default: {  // NDNET_FOLD_BIAS
      const int n = (int)u;
      float v = 0.0f;
      if (n < J.N) {
        v = J.bias[n];
        if (J.gamma) v = (v - J.mean[n]) * (J.gamma[n] / sqrtf(J.var[n] + J.eps)) + J.beta[n];
        if (J.eye > 0) v = v + (n / J.eye == n % J.eye ? 1.0f : 0.0f);
      }
      static_cast<float*>(J.out)[u] = v;
    }
  }
}
#endif

#if NDNET_PN_TILE == 64
int fc_mfma_cbw(int nb, int ngmax) {
  static const int cap = [] {
    const char* e = getenv("NDNET_PN_FC_CBW");
    return e ? atoi(e) : 4;
  }();
  for (int c = cap >= 4 ? 4 : cap >= 2 ? 2 : 1; c > 1; c >>= 1)
    if (nb % c == 0 && nb / c >= 32 && ngmax * c <= kFcMaxG) return c;
  return 1;
}
#endif

}  // namespace

extern "C" {

#if NDNET_PN_TILE == 64  // the 32-point build exports only its chain entry point (below)
int ndnet_pn_fc_mfma_run(const float* in, int ld_in, const float* Wf, const float* bias, float* out, int ld_out,
                         int batch, int K, int N, int relu, void* stream) {
  if (!in || !Wf || !bias || !out || batch <= 0 || batch > 16 || K <= 0 || K % 16 || K > 16 * kFcWaves * kFcMaxG ||
      N <= 0 || N % 16 || ld_in % 4 || ld_in < K || ld_out < N || ((uintptr_t)in | (uintptr_t)Wf) % 16)
    return -20;
  const int KG = K / 16, nb = N / 16, ngmax = (KG + kFcWaves - 1) / kFcWaves;
  // column blocks per workgroup: 4 while that keeps >= 32 workgroups and the
  // fragments fit (fc_mfma_cbw; NDNET_PN_FC_CBW=1 restores one block each)
  const int cbw = fc_mfma_cbw(nb, ngmax);
  const f32x4* wf = reinterpret_cast<const f32x4*>(Wf);
  hipStream_t st = (hipStream_t)stream;
  if (cbw == 4)
    k_pn_fc_mfma<4><<<nb / 4, kFcWaves * 64, 0, st>>>(in, ld_in, wf, bias, out, ld_out, batch, KG, relu);
  else if (cbw == 2)
    k_pn_fc_mfma<2><<<nb / 2, kFcWaves * 64, 0, st>>>(in, ld_in, wf, bias, out, ld_out, batch, KG, relu);
  else
    k_pn_fc_mfma<1><<<nb, kFcWaves * 64, 0, st>>>(in, ld_in, wf, bias, out, ld_out, batch, KG, relu);
  return hipGetLastError() == hipSuccess ? 0 : -21;
}

int ndnet_pn_fc_run(const float* in, int ld_in, const float* W, const float* bias, float* out, int ld_out, int batch,
                    int K, int N, int relu, void* stream) {
  if (!in || !W || !bias || !out || batch <= 0 || batch > 16 || K <= 0 || K % 4 || N <= 0 || ld_in % 4 ||
      ((uintptr_t)in | (uintptr_t)W) % 16)
    return -20;
  hipStream_t st = (hipStream_t)stream;
  switch (K % 256 == 0 && K <= 1024 ? K / 256 : 0) {
    case 2: k_pn_fc_split<2><<<(N + 1) / 2, 256, 0, st>>>(in, ld_in, W, bias, out, ld_out, batch, N, relu); break;
    case 4: k_pn_fc_split<4><<<N, 256, 0, st>>>(in, ld_in, W, bias, out, ld_out, batch, N, relu); break;
    default: k_pn_fc<<<(N + 3) / 4, 256, 0, st>>>(in, ld_in, W, bias, out, ld_out, batch, K, N, relu);
  }
  return hipGetLastError() == hipSuccess ? 0 : -21;
}

int ndnet_pn_head3_run(const float* h2, int ld_h, const float* W3, const float* b3, const float* basis, float* t1,
                       float* w1f, int batch, int K, int kin, int nout, void* stream) {
  if (!h2 || !W3 || !b3 || !basis || !t1 || !w1f || batch <= 0 || K <= 0 || kin <= 0 || kin > 16 || nout <= 0 ||
      nout % 16)
    return -20;
  k_pn_head3<<<batch, 256, 0, (hipStream_t)stream>>>(h2, ld_h, W3, b3, basis, t1, w1f, K, kin, nout);
  return hipGetLastError() == hipSuccess ? 0 : -21;
}

int ndnet_pn_fold_t2_run(const float* w1f, int w1_stride, const float* b1, const float* t2, int t2_ld, float* outf,
                         float* outb, int batch, void* stream) {
  if (!w1f || !b1 || !t2 || !outf || !outb || batch <= 0 || w1_stride < 1024 || t2_ld < 4096 || t2_ld % 4 ||
      (uintptr_t)t2 % 16)
    return -20;
  k_pn_fold_t2<<<batch, 1024, 0, (hipStream_t)stream>>>(w1f, w1_stride, b1, t2, t2_ld, outf, outb);
  return hipGetLastError() == hipSuccess ? 0 : -21;
}

int ndnet_pn_fold_prepare(ndnet_pn_fold_job* jobs, int num_jobs, int64_t* num_blocks) {
  if (!jobs || num_jobs <= 0 || !num_blocks) return -20;
  int64_t blocks = 0;
  for (int i = 0; i < num_jobs; i++) {
    ndnet_pn_fold_job& J = jobs[i];
    const bool bn = J.gamma != nullptr;
    if (!J.out || (uintptr_t)J.out % 16 || J.kind < NDNET_FOLD_WT || J.kind > NDNET_FOLD_BIAS || J.N <= 0 ||
        (bn && (!J.beta || !J.mean || !J.var || !(J.eps >= 0.0f))) || (!bn && (J.beta || J.mean || J.var)))
      return -20;
    if (J.kind == NDNET_FOLD_BIAS) {
      if (!J.bias || J.Np < J.N || J.eye < 0 || (J.eye > 0 && J.eye * J.eye != J.N)) return -20;
    } else {
      if (!J.w || J.K <= 0 || J.k0 < 0 || J.ld < J.k0 + J.K) return -20;
      if (J.kind == NDNET_FOLD_WT && (J.Kp < J.K || J.Np < J.N)) return -20;
      if (J.kind == NDNET_FOLD_FRAG && (J.Kp < J.K || J.Np < J.N || J.Kp % 16 || J.Np % 16)) return -20;
      if (J.kind == NDNET_FOLD_FRAG6 && (J.Kp < J.K || J.Np < J.N || J.Kp % 32 || J.Np % 16)) return -20;
      if (J.kind == NDNET_FOLD_BASIS && J.K != 12) return -20;
    }
    J.block0 = blocks;
    blocks += (fold_units(J) + kFoldThreads - 1) / kFoldThreads;
  }
  if (blocks <= 0 || blocks > 0x7fffffff) return -20;
  *num_blocks = blocks;
  return 0;
}

int ndnet_pn_fold_run(const ndnet_pn_fold_job* jobs, int num_jobs, int64_t num_blocks, void* stream) {
  if (!jobs || num_jobs <= 0 || num_blocks <= 0 || num_blocks > 0x7fffffff) return -20;
  k_pn_fold<<<(unsigned)num_blocks, kFoldThreads, 0, (hipStream_t)stream>>>(jobs, num_jobs);
  return hipGetLastError() == hipSuccess ? 0 : -21;
}

// One fused point-MLP chain over `batch` clouds on `stream` (see pointnet.h).

// Timing builds: zeroes the stamp array (before a launch whose stamps are read)
int ndnet_pn_debug_stamps_clear(void) {
#ifdef NDNET_PN_STAMPS
  static unsigned long long zeros[kStampWgs][16];
  return hipMemcpyToSymbol(HIP_SYMBOL(g_pn_stamps), zeros, sizeof(zeros)) == hipSuccess ? 0 : -21;
#else
  return -20;
#endif
}

// Timing builds (-DNDNET_PN_STAMPS): copies the stamps of the last chain
// launch, [wgs][16] u64, to host memory; the product build returns -20.
int ndnet_pn_debug_stamps(unsigned long long* host, int wgs) {
#ifdef NDNET_PN_STAMPS
  if (!host || wgs <= 0 || wgs > kStampWgs) return -20;
  if (hipDeviceSynchronize() != hipSuccess) return -21;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_pn_stamps), (size_t)wgs * 16 * sizeof(unsigned long long)) ==
                 hipSuccess ? 0 : -21;
#else
  (void)host; (void)wgs;
  return -20;
#endif
}
#endif

// an inconsistent argument block: NDNET_ERR_ARG, with the failing check's line on stderr
#define PN_ARG_FAIL()                                                                          \
  do {                                                                                         \
    fprintf(stderr, "ndnet_amd: chain launch: invalid argument (pointnet_kernels.hip:%d)\n", __LINE__); \
    return -20;                                                                                \
  } while (0)

#if NDNET_PN_TILE == 64
int ndnet_pn_chain_run(const ndnet_pn_chain* args, int batch, void* stream) {
#else
int ndnet_pn_chain_run_t32(const ndnet_pn_chain* args, int batch, void* stream) {
#endif
  if (!args || batch <= 0 || args->num_layers < 1 || args->num_layers > NDNET_PN_MAX_LAYERS || args->num_points <= 0 ||
      args->in_cols < 1 || args->in_cols > args->L[0].K || args->in_cols > args->x_ld)
    PN_ARG_FAIL();
  // activation regions: layer l reads region l & 1 (or the fused-chunk buffer
  // after a fused layer) and writes region (l + 1) & 1
  int w[2] = {args->L[0].K, 0};
  bool has_fuse = false;
  int planes = 0, qprec = 0;
  for (int l = 0; l < args->num_layers; l++) {
    const ndnet_pn_layer& L = args->L[l];
    if (!L.w || !L.bias || L.K <= 0 || L.K % 16 || L.N <= 0 || L.N % 32 || (L.N > 32 && L.N % 64) ||
        ((uintptr_t)L.w % 16) ||
        L.w_cloud_stride % 4)
      PN_ARG_FAIL();
    const bool fed = l > 0 && args->L[l - 1].fuse_next;
    if (L.prec < 0 || L.prec > 1) PN_ARG_FAIL();
    if (L.prec) {  // split-bf16: reads planes its producer writes (into a region, or the fused chunks)
      if (l == 0 || L.K % 32 || args->L[l - 1].N != L.K) PN_ARG_FAIL();
      if (fed) qprec = 1;
      else planes |= 1 << (l & 1);
    }
    if (fed) {
      if (L.K != args->L[l - 1].N || (L.N != 64 && L.N != 128 && L.N != 256) || L.fuse_next) PN_ARG_FAIL();
    } else if (l > 0 && L.K > w[l & 1]) {
      PN_ARG_FAIL();
    }
    if (L.fuse_next) {
      if (l + 1 >= args->num_layers || L.N % kFuseNC) PN_ARG_FAIL();
      has_fuse = true;
      continue;  // not stored in a region
    }
    const bool stored = l + 1 < args->num_layers || args->mode == 1;
    if (stored && L.N > w[(l + 1) & 1]) w[(l + 1) & 1] = L.N;
  }
  if (args->max_width < w[0] || args->max_width2 < w[1] || args->max_width % 8 || args->max_width2 % 8) PN_ARG_FAIL();
  if (args->mode == 1 && (!args->out || args->out_cols <= 0 || args->out_cols > args->L[args->num_layers - 1].N))
    PN_ARG_FAIL();
  if (args->mode == 0 && !args->gmax) PN_ARG_FAIL();
  // LDS: region 0 | region 1, then the fused pair's chunks.  Q writes the
  // region P reads, after its last chunk, so the chunks may start right after
  // P's input inside that region (and run past its end when it is region 1)
  const int r0f = region0_floats(*args, planes);
  const int r1f = region_floats(args->max_width2, planes & 2);
  int fbuf_off = r0f + r1f;
  size_t total = (size_t)r0f + r1f;
  if (has_fuse) {
    int lf = 0;
    while (!args->L[lf].fuse_next) lf++;
    const int r = lf & 1, fb = fbuf_floats(qprec);
    const int p_in = args->L[lf].prec ? 3 * kP * (args->L[lf].K + kPadB) / 2    // P's input: bf16 planes, pitch K + kPadB
                                      : kP * ((r ? args->max_width2 : args->max_width) + kPadF);  // or fp32, region pitch
    const int inside = (r ? r0f : 0) + p_in;
    if (r == 1 || inside + fb <= r0f) fbuf_off = inside;
    total = fbuf_off + (size_t)fb > total ? fbuf_off + (size_t)fb : total;
  }
  if ((args->fold_out_w || args->fold_out_b) && (!args->fold_t2 || !args->fold_out_w || !args->fold_out_b))
    PN_ARG_FAIL();
  if (args->fold_t2) {  // the t2 fold runs in layer 0's VALU prologue, t2 staged at region 1
    if (!valu_layer0(*args) || args->head_h2 || args->fold_ld < 4096 || args->fold_ld % 4 || (uintptr_t)args->fold_t2 % 16)
      PN_ARG_FAIL();
    if (total < (size_t)r0f + 4096) total = (size_t)r0f + 4096;
  }
  // every layer's bias after the other regions (layer 0's too: the prologue
  // reads it there when layer 0 runs on the MFMA path)
  const int bias_base = (int)((total + 3) & ~(size_t)3);
  int nbias = 0;
  for (int l = 0; l < args->num_layers; l++) {
    if (args->L[l].N > 2 * kThreads) PN_ARG_FAIL();  // the prologue stages <= 2 bias values per thread and layer
    nbias += args->L[l].N;
  }
  total = (size_t)bias_base + nbias;
  const size_t lds = sizeof(float) * total;
  static bool attr_set = false;
  if (!attr_set) {
    if (hipFuncSetAttribute((const void*)k_pn_chain, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) !=
        hipSuccess)
      return -21;
    attr_set = true;
  }
  if (lds > 160 * 1024) PN_ARG_FAIL();
  dim3 grid((args->num_points + kP - 1) / kP, batch);
  k_pn_chain<<<grid, kThreads, lds, (hipStream_t)stream>>>(*args, planes, fbuf_off, bias_base);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    fprintf(stderr, "ndnet_amd: k_pn_chain launch failed: %s\n", hipGetErrorString(e));
    return -21;
  }
  return 0;
}

}  // extern "C"
