// ndt_kernels.hip -- the NDT downsample path on gfx950.
//
// Replaces core_legacy/src/{pointclouds,voxel,normal_distributions,
// kullback_leibler,ndt}.c (the reference's `ndt_downsample`, ndt.c:119-222)
// with batched HIP kernels.  One batch = B clouds of n points; every kernel
// covers the whole batch, so the per-cloud latency chain (up to 15 voxel-size
// bisection passes) is paid once per batch, not once per cloud.
//
// Kernels, in launch order (see DESIGN.md for the data layout and rooflines):
//   k_reset        per-cloud control block for this call
//   k_limits       bounding box (pointclouds.c:40-66), first grid
//   k_search_pass  one bisection pass: voxel keys of all points, distinct
//                  occupied voxels counted through per-voxel stamps; the last
//                  workgroup of a cloud applies ndt.c:169-187.  Launched 15x.
//   k_dense        occupied voxels of the accepted grid -> dense ids in
//                  ascending linear order (the output order, ndt.c:88-90)
//   k_chunk_sort   stable per-chunk sort of points by dense id
//   k_welford      one lane per ND, sequential Welford in point order
//                  (normal_distributions.c:75-121), bit-exact
//   k_kl           one workgroup per cloud: LU chains, KL events, the
//                  reference's insertion order, prune, compaction
//   k_prune        a further prune level on the retained list (ndt.c:28-73)
//
// The translation unit is compiled with -ffp-contract=off: every double
// operation rounds exactly like the reference's x86-64 build.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "ndt_device.h"
#include "../../include/ndnet_amd.h"

#pragma clang fp contract(off)

using namespace ndnet;

namespace {

constexpr int kChunk = 4096;         // points per k_chunk_sort workgroup
constexpr int kChunkThreads = 1024;
constexpr int kPassThreads = 256;    // threads per search workgroup
constexpr int kPassPPT = 16;         // points per thread per search workgroup
constexpr int kPassPts = kPassThreads * kPassPPT;
constexpr int kHashSlots = 8192;     // LDS dedup table of a search workgroup
constexpr int kKLThreads = 1024;
constexpr int kSortLds = 8192;       // largest event sort kept in LDS

enum State : uint32_t { kSearching = 0, kAccepted = 1, kFailed = 2 };

struct CloudCtl {
  unsigned long long limkey[6];  // order keys: max x,y,z then min x,y,z
  double lim[6];
  double guess, lo, hi;
  double vs;
  double off[3];
  uint32_t len[3];
  uint32_t state;
  int32_t rc;
  uint32_t iter;
  uint32_t epoch;
  uint32_t stamp;
  uint32_t accepted_stamp;
  uint32_t count;
  uint32_t arrive;
  uint32_t nbad;
  uint32_t first_bad[kWorkers];
  uint64_t V;
  uint32_t num_nds;
  double guesses[16];
  uint32_t counts[16];
  // list state kept for further prune levels (ndt_legacy.py:173-240)
  uint32_t num_valid;
  uint32_t num_kl;       // live list length
  uint32_t num_phys;     // entries ever written (the rest is poison)
  uint32_t num_events;
  int32_t prune_rc;
  uint32_t num_out;
  uint32_t last_k;
};

struct Plan {
  int B;
  uint64_t n;
  uint64_t k;
  int ncls;            // num_classes (histograms have ncls+1 bins)
  uint64_t vcap;       // voxels per cloud the stamp / dense tables hold
  uint32_t ndcap;      // max accepted NDs per cloud = floor(1.2 k) + 1
  uint32_t ecap;       // 6 * ndcap
  uint32_t nchunks;    // k_chunk_sort chunks per cloud
  uint32_t G;          // search workgroups per cloud
  int in_f64;          // input element type of the last run
  uint64_t calls;      // runs issued (mirrors the device epoch)
  int timing;          // record stage events
  hipEvent_t ev[8];
  // device buffers
  CloudCtl* ctl;
  uint32_t* stamps;    // [B][vcap]
  uint32_t* dense_of;  // [B][vcap]
  uint32_t* vox;       // [B][ndcap] linear index of dense id
  void* chunk_pts;     // [B][nchunks][kChunk] double[3]
  uint16_t* chunk_lbl; // [B][nchunks][kChunk]
  uint2* chunk_tab;    // [B][nchunks][ndcap] (start, count)
  uint32_t* nd_n;      // [B][ndcap]
  double* nd_mean;     // [B][ndcap][3]
  double* nd_cov;      // [B][ndcap][9] pre-KL
  double* nd_cov_post; // [B][ndcap][9]
  uint16_t* nd_cls;    // [B][ndcap]
  uint32_t* hist;      // [B][ndcap][ncls+1]
  int32_t* nb;         // [B][ndcap][6]
  uint32_t* keys;      // [B][ndcap][12]
  uint32_t* nkeys;     // [B][ndcap]
  double* chain;       // [B][ndcap][12][9]
  uint32_t* chain_ps;  // [B][ndcap][12] perm | (signum < 0) << 8
  double* slot_val;    // [B][ecap]
  uint32_t* slot_flag; // [B][ecap]
  double* ev_val;      // [B][ecap]
  uint32_t* ev_p;      // [B][ecap]
  uint32_t* ev_q;      // [B][ecap]
  double* ev_min;      // [B][ecap] exclusive prefix min (NaN-skipping)
  unsigned long long* sort_key;  // [B][sortcap]
  uint32_t* sort_idx;  // [B][sortcap]
  uint32_t* nan_list;  // [B][ecap]
  uint32_t* nan_pos;   // [B][ecap]
  double* ord_val;     // [B][ecap] the retained list (physical array)
  uint32_t* ord_p;     // [B][ecap]
  uint32_t* ord_q;     // [B][ecap]
  uint32_t* first_occ; // [B][ndcap]
  uint32_t* tmp_u32;   // [B][ecap] scratch
  uint8_t* alive;      // [B][ndcap]
  uint32_t sortcap;
  ndnet_ndt_stats* d_stats;  // [B] device copy of the stats
};

// ------------------------------------------------------------------ helpers

__device__ inline uint32_t hash32(uint32_t k) { return (k * 2654435761u) >> (32 - 13); }

template <typename T>
__device__ inline void load_point(const T* pts, uint64_t i, double* x) {
  x[0] = (double)pts[3 * i + 0];
  x[1] = (double)pts[3 * i + 1];
  x[2] = (double)pts[3 * i + 2];
}

// Inclusive wave scan (64 lanes) with op; returns inclusive value.
template <typename T, typename Op>
__device__ inline T wave_incl_scan(T x, Op op) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    T y = __shfl_up(x, o, 64);
    if (lane >= o) x = op(y, x);
  }
  return x;
}

// Exclusive block scan of one value per thread.  `scratch` holds >= 16 T.
template <typename T, typename Op>
__device__ inline T block_excl_scan(T v, T identity, Op op, T* scratch, T& total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  T incl = wave_incl_scan(v, op);
  T excl_w = __shfl_up(incl, 1, 64);
  if (lane == 0) excl_w = identity;
  if (lane == 63) scratch[wid] = incl;
  __syncthreads();
  if (wid == 0) {
    T s = lane < nw ? scratch[lane] : identity;
    s = wave_incl_scan(s, op);
    if (lane < nw) scratch[lane] = s;
  }
  __syncthreads();
  T pre = wid > 0 ? scratch[wid - 1] : identity;
  total = scratch[nw - 1];
  __syncthreads();
  return op(pre, excl_w);
}

struct AddU32 {
  __device__ uint32_t operator()(uint32_t a, uint32_t b) const { return a + b; }
};
struct MinF64 {
  __device__ double operator()(double a, double b) const { return b < a ? b : a; }
};

__device__ inline void grid_from(const CloudCtl& c, double vs, uint32_t* len, double* off, uint64_t* V) {
  // voxel.c:61-81: len = (int)ceil(dim / vs), offset = min
  uint64_t v = 1;
  for (int a = 0; a < 3; a++) {
    const double d = c.lim[a] - c.lim[3 + a];
    const double q = ceil(d / vs);
    int li;
    if (q >= -2147483648.0 && q < 2147483648.0) li = (int)q;
    else li = (int)0x80000000;  // x86 cvttsd2si overflow value
    len[a] = (uint32_t)li;
    off[a] = c.lim[3 + a];
    v *= (uint64_t)len[a];
  }
  *V = v;
}

// ------------------------------------------------------------------ kernels

__global__ void k_reset(CloudCtl* ctl, int B) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  CloudCtl& c = ctl[b];
  c.epoch = c.epoch + 1;
  if (c.epoch >= (1u << 26)) c.epoch = 1;  // stamps are epoch*32 + pass
  for (int a = 0; a < 3; a++) {
    c.limkey[a] = ord_key(kDblMin);      // max starts at DBL_MIN (pointclouds.c:44-46)
    c.limkey[3 + a] = ord_key(kDblMax);  // min starts at DBL_MAX
  }
  c.state = kSearching;
  c.rc = 0;
  c.iter = 0;
  c.count = 0;
  c.arrive = 0;
  c.nbad = 0;
  for (int w = 0; w < kWorkers; w++) c.first_bad[w] = kInvalid;
  c.num_nds = 0;
  c.num_valid = 0;
  c.num_kl = 0;
  c.num_phys = 0;
  c.num_events = 0;
  c.prune_rc = 0;
  c.num_out = 0;
  c.last_k = 0;
  c.V = 0;
  c.len[0] = c.len[1] = c.len[2] = 0;
  c.off[0] = c.off[1] = c.off[2] = 0.0;
  c.vs = 0.0;
}

// Checks a new guess's grid against the table capacity; updates c.
__device__ inline void set_guess(CloudCtl& c, double guess, uint64_t vcap) {
  c.guess = guess;
  uint64_t V;
  grid_from(c, guess, c.len, c.off, &V);
  c.V = V;
  c.stamp = c.epoch * 32u + c.iter;
  if (V > vcap) {  // the reference's malloc of V NDs would be the failure point
    c.state = kFailed;
    c.rc = -1;
    c.vs = guess;
  }
}

template <typename T>
__global__ void k_limits(const T* __restrict__ pts, CloudCtl* ctl, uint64_t n, uint32_t G, uint64_t vcap) {
  const int b = blockIdx.y;
  const T* p = pts + (uint64_t)b * n * 3;
  double mx[3] = {kDblMin, kDblMin, kDblMin}, mn[3] = {kDblMax, kDblMax, kDblMax};
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)G * blockDim.x) {
    double x[3];
    load_point(p, i, x);
    for (int a = 0; a < 3; a++) {
      mx[a] = x[a] > mx[a] ? x[a] : mx[a];  // maxf(point, cur), pointclouds.c:28-30
      mn[a] = x[a] < mn[a] ? x[a] : mn[a];
    }
  }
  // wave reduce on order keys
  unsigned long long kmx[3], kmn[3];
  for (int a = 0; a < 3; a++) {
    kmx[a] = ord_key(mx[a]);
    kmn[a] = ord_key(mn[a]);
    for (int o = 32; o > 0; o >>= 1) {
      unsigned long long y = __shfl_xor(kmx[a], o, 64);
      kmx[a] = y > kmx[a] ? y : kmx[a];
      y = __shfl_xor(kmn[a], o, 64);
      kmn[a] = y < kmn[a] ? y : kmn[a];
    }
  }
  CloudCtl& c = ctl[b];
  if ((threadIdx.x & 63) == 0) {
    for (int a = 0; a < 3; a++) {
      atomicMax(&c.limkey[a], kmx[a]);
      atomicMin(&c.limkey[3 + a], kmn[a]);
    }
  }
  __syncthreads();
  __shared__ uint32_t last;
  if (threadIdx.x == 0) {
    __atomic_thread_fence(__ATOMIC_RELEASE);
    uint32_t t = __hip_atomic_fetch_add(&c.arrive, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    last = (t == G - 1);
  }
  __syncthreads();
  if (!last || threadIdx.x != 0) return;
  __atomic_thread_fence(__ATOMIC_ACQUIRE);
  for (int a = 0; a < 6; a++)
    c.lim[a] = ord_unkey(__hip_atomic_load(&c.limkey[a], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  c.arrive = 0;
  c.lo = kMinGuess;
  c.hi = kMaxGuess;
  set_guess(c, (kMaxGuess - kMinGuess) / 2.0, vcap);  // ndt.c:136
}

// Distinct-voxel counting of one bisection pass for the points [start, end)
// of one cloud.  Returns this thread's number of newly stamped voxels.
template <typename T>
__device__ inline uint32_t mark_points(const T* p, uint64_t start, uint64_t end, uint64_t chunk, const CloudCtl& c,
                                       uint32_t* stamps, uint32_t stamp, uint32_t* table, bool track_bad,
                                       uint32_t* bad_out, const uint32_t* cutoff) {
  const double vs = c.guess;
  const double inv_vs = 1.0 / vs;
  uint32_t fresh = 0;
  for (uint64_t i = start + threadIdx.x; i < end; i += blockDim.x) {
    if (cutoff && i >= cutoff[i / chunk]) continue;
    double x[3];
    load_point(p, i, x);
    const uint32_t key = voxel_key(x[0], x[1], x[2], c.off, c.len, vs, inv_vs);
    if (key == kInvalid) {
      if (track_bad) atomicMin(&bad_out[i / chunk], (uint32_t)i);
      continue;
    }
    if (table) {
      // LDS dedup: only the thread that inserts a key touches the global stamp
      uint32_t h = hash32(key);
      bool mine = false;
      for (int probe = 0; probe < kHashSlots; probe++) {
        uint32_t cur = table[h];
        if (cur == key) break;
        if (cur == kInvalid) {
          uint32_t old = atomicCAS(&table[h], kInvalid, key);
          if (old == kInvalid) { mine = true; break; }
          if (old == key) break;
        }
        h = (h + 1) & (kHashSlots - 1);
      }
      if (!mine) continue;
    }
    uint32_t* s = stamps + key;
    if (__hip_atomic_load(s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != stamp) {
      uint32_t old = atomicExch(s, stamp);
      fresh += (old != stamp);
    }
  }
  return fresh;
}

__device__ inline uint32_t block_sum_u32(uint32_t v, uint32_t* scratch) {
  uint32_t tot;
  (void)block_excl_scan(v, 0u, AddU32(), scratch, tot);
  return tot;
}

// Bisection decision of ndt.c:168-187 after a pass counted `count` NDs.
__device__ inline void finish_pass(CloudCtl& c, uint32_t count, uint64_t k, uint64_t vcap) {
  c.guesses[c.iter] = c.guess;
  c.counts[c.iter] = count;
  if ((double)count > (double)k * (1 + kUpper)) {
    c.lo = c.guess;
  } else if (count < k) {
    c.hi = c.guess;
  } else {
    c.state = kAccepted;
    c.vs = c.guess;
    c.num_nds = count;
    c.accepted_stamp = c.stamp;
    c.iter++;
    return;
  }
  c.iter++;
  const double g = c.lo + (c.hi - c.lo) / 2.0;
  if (c.iter == (uint32_t)kMaxIters) {
    c.state = kFailed;
    c.rc = -3;  // "Reached maximum number of iterations!" (ndt.c:191-194)
    c.vs = g;
    return;
  }
  for (int w = 0; w < kWorkers; w++) c.first_bad[w] = kInvalid;
  c.nbad = 0;
  set_guess(c, g, vcap);
}

template <typename T>
__global__ void __launch_bounds__(kPassThreads) k_search_pass(const T* __restrict__ pts, CloudCtl* ctl,
                                                              uint32_t* stamps_all, uint64_t n, uint64_t k,
                                                              uint32_t G, uint64_t vcap) {
  const int b = blockIdx.y;
  CloudCtl& c = ctl[b];
  if (__hip_atomic_load(&c.state, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != kSearching) return;
  __shared__ uint32_t table[kHashSlots];
  __shared__ uint32_t scratch[16];
  __shared__ uint32_t last;
  for (int i = threadIdx.x; i < kHashSlots; i += blockDim.x) table[i] = kInvalid;
  __syncthreads();
  const uint64_t chunk = n / kWorkers;       // pcl_worker range, normal_distributions.c:34-35
  const uint64_t n8 = chunk * kWorkers;      // the n % 8 tail is never estimated
  const T* p = pts + (uint64_t)b * n * 3;
  uint32_t* stamps = stamps_all + (uint64_t)b * vcap;
  const uint32_t stamp = c.stamp;
  const uint64_t start = (uint64_t)blockIdx.x * kPassPts;
  const uint64_t end = start + kPassPts < n8 ? start + kPassPts : n8;
  uint32_t fresh = 0;
  if (start < end)
    fresh = mark_points(p, start, end, chunk, c, stamps, stamp, table, true, c.first_bad, nullptr);
  fresh = block_sum_u32(fresh, scratch);
  if (threadIdx.x == 0) {
    if (fresh) atomicAdd(&c.count, fresh);
    __atomic_thread_fence(__ATOMIC_RELEASE);
    uint32_t t = __hip_atomic_fetch_add(&c.arrive, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    last = (t == G - 1);
  }
  __syncthreads();
  if (!last) return;
  __atomic_thread_fence(__ATOMIC_ACQUIRE);
  // Last workgroup of this cloud.  If some point fell outside the grid, its
  // reference worker abandoned the rest of its chunk (normal_distributions.c
  // :47-52): recount with those cut-offs (rare: needs dim/vs integral).
  __shared__ uint32_t any_bad;
  __shared__ uint32_t cut[kWorkers];
  if (threadIdx.x < kWorkers)
    cut[threadIdx.x] = __hip_atomic_load(&c.first_bad[threadIdx.x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  if (threadIdx.x == 0) {
    any_bad = 0;
    for (int w = 0; w < kWorkers; w++) any_bad |= cut[w] != kInvalid;
  }
  __syncthreads();
  uint32_t count;
  if (any_bad) {
    const uint32_t stamp2 = c.epoch * 32u + 16u + c.iter;
    uint32_t f = mark_points(p, 0, n8, chunk, c, stamps, stamp2, nullptr, false, nullptr, cut);
    count = block_sum_u32(f, scratch);
    if (threadIdx.x == 0) c.stamp = stamp2;
  } else {
    count = __hip_atomic_load(&c.count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    c.count = 0;
    c.arrive = 0;
    finish_pass(c, count, k, vcap);
  }
}

// Occupied voxels of the accepted grid -> dense ids in ascending linear order.
__global__ void __launch_bounds__(1024) k_dense(CloudCtl* ctl, const uint32_t* stamps_all, uint32_t* dense_all,
                                                uint32_t* vox_all, uint64_t vcap, uint32_t ndcap) {
  const int b = blockIdx.x;
  const CloudCtl& c = ctl[b];
  if (c.state != kAccepted) return;
  __shared__ uint32_t scratch[16];
  const uint32_t* st = stamps_all + (uint64_t)b * vcap;
  uint32_t* dense = dense_all + (uint64_t)b * vcap;
  uint32_t* vox = vox_all + (uint64_t)b * ndcap;
  const uint32_t stamp = c.accepted_stamp;
  const uint64_t V = c.V;
  uint32_t carry = 0;
  for (uint64_t base = 0; base < V; base += blockDim.x) {
    const uint64_t v = base + threadIdx.x;
    const uint32_t occ = (v < V) && st[v] == stamp;
    uint32_t tot;
    const uint32_t ex = block_excl_scan(occ, 0u, AddU32(), scratch, tot);
    if (v < V) {
      const uint32_t d = carry + ex;
      dense[v] = occ ? d : kInvalid;
      if (occ && d < ndcap) vox[d] = (uint32_t)v;
    }
    carry += tot;
  }
}

// Per chunk of kChunk points: dense id of each point (kInvalid when the
// reference would not estimate it), stable sort by (dense id, index) in LDS,
// then the sorted coordinates and a (start, count) table per dense id.
template <typename T>
__global__ void __launch_bounds__(kChunkThreads) k_chunk_sort(const T* __restrict__ pts, const int32_t* __restrict__ lbl,
                                                              const CloudCtl* ctl, const uint32_t* dense_all,
                                                              double* cpts_all, uint16_t* clbl_all, uint2* ctab_all,
                                                              uint64_t n, uint64_t vcap, uint32_t ndcap,
                                                              uint32_t nchunks) {
  const int b = blockIdx.y, ch = blockIdx.x;
  const CloudCtl& c = ctl[b];
  if (c.state != kAccepted) return;
  __shared__ uint32_t skey[kChunk];
  const uint64_t chunk = n / kWorkers;
  const uint64_t n8 = chunk * kWorkers;
  const T* p = pts + (uint64_t)b * n * 3;
  const uint32_t* dense = dense_all + (uint64_t)b * vcap;
  const double vs = c.vs, inv_vs = 1.0 / vs;
  const uint64_t base = (uint64_t)ch * kChunk;
  for (int t = threadIdx.x; t < kChunk; t += blockDim.x) {
    const uint64_t i = base + t;
    uint32_t key = kInvalid;
    if (i < n8 && i < c.first_bad[i / chunk]) {
      double x[3];
      load_point(p, i, x);
      const uint32_t lin = voxel_key(x[0], x[1], x[2], c.off, c.len, vs, inv_vs);
      if (lin != kInvalid) {
        const uint32_t d = dense[lin];
        if (d != kInvalid) key = (d << 12) | (uint32_t)t;
      }
    }
    skey[t] = key;
  }
  __syncthreads();
  // bitonic sort, ascending (keys are unique except kInvalid padding)
  for (int size = 2; size <= kChunk; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = threadIdx.x; t < kChunk / 2; t += blockDim.x) {
        const int lo = 2 * t - (t & (stride - 1));
        const int hi = lo + stride;
        const bool up = (lo & size) == 0;
        const uint32_t a = skey[lo], bb = skey[hi];
        if ((a > bb) == up) { skey[lo] = bb; skey[hi] = a; }
      }
      __syncthreads();
    }
  }
  uint2* tab = ctab_all + ((uint64_t)b * nchunks + ch) * ndcap;
  const uint32_t nd = c.num_nds;
  for (uint32_t d = threadIdx.x; d < nd; d += blockDim.x) tab[d] = make_uint2(0, 0);
  __syncthreads();
  double* cp = cpts_all + ((uint64_t)b * nchunks + ch) * kChunk * 3;
  uint16_t* cl = clbl_all ? clbl_all + ((uint64_t)b * nchunks + ch) * kChunk : nullptr;
  for (int s = threadIdx.x; s < kChunk; s += blockDim.x) {
    const uint32_t key = skey[s];
    if (key == kInvalid) continue;
    const uint32_t d = key >> 12, t = key & 0xfff;
    double x[3];
    load_point(p, base + t, x);
    cp[3 * s + 0] = x[0];
    cp[3 * s + 1] = x[1];
    cp[3 * s + 2] = x[2];
    if (cl) cl[s] = (uint16_t)lbl[(uint64_t)b * n + base + t];
    if (s == 0 || (skey[s - 1] >> 12) != d) tab[d].x = (uint32_t)s;  // run start
  }
  __syncthreads();
  for (int s = threadIdx.x; s < kChunk; s += blockDim.x) {
    const uint32_t key = skey[s];
    if (key == kInvalid) continue;
    const uint32_t d = key >> 12;
    const bool run_end = (s + 1 == kChunk) || skey[s + 1] == kInvalid || (skey[s + 1] >> 12) != d;
    if (run_end) tab[d].y = (uint32_t)s + 1 - tab[d].x;
  }
}

// One lane per ND: sequential Welford over its points in index order.
__global__ void __launch_bounds__(256) k_welford(const CloudCtl* ctl, const double* __restrict__ cpts_all,
                                                 const uint16_t* __restrict__ clbl_all, const uint2* __restrict__ ctab_all,
                                                 uint32_t* nd_n, double* nd_mean, double* nd_cov, uint16_t* nd_cls,
                                                 uint32_t* hist_all, int ncls, uint32_t ndcap, uint32_t nchunks) {
  const int b = blockIdx.y;
  const CloudCtl& c = ctl[b];
  if (c.state != kAccepted) return;
  const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= c.num_nds) return;
  Welford w;
  welford_init(w);
  const uint64_t cb = (uint64_t)b * nchunks;
  uint32_t* hist = clbl_all ? hist_all + ((uint64_t)b * ndcap + d) * (uint32_t)(ncls + 1) : nullptr;
  if (hist)
    for (int j = 0; j <= ncls; j++) hist[j] = 0;
  for (uint32_t ch = 0; ch < nchunks; ch++) {
    const uint2 se = ctab_all[(cb + ch) * ndcap + d];
    const double* cp = cpts_all + (cb + ch) * kChunk * 3;
    for (uint32_t j = 0; j < se.y; j++) {
      double x[3];
      x[0] = cp[3 * (se.x + j) + 0];
      x[1] = cp[3 * (se.x + j) + 1];
      x[2] = cp[3 * (se.x + j) + 2];
      welford_update(w, x);
      if (hist) {
        const uint32_t l = clbl_all[(cb + ch) * kChunk + se.x + j];
        if (l <= (uint32_t)ncls) hist[l]++;
      }
    }
  }
  const uint64_t o = (uint64_t)b * ndcap + d;
  nd_n[o] = (uint32_t)w.n;
  for (int j = 0; j < 3; j++) nd_mean[3 * o + j] = w.mean[j];
  for (int j = 0; j < 9; j++) nd_cov[9 * o + j] = w.cov[j];
  uint16_t cls = 0;
  if (hist) {  // first index of the max count (normal_distributions.c:107-121)
    uint32_t best = 0;
    for (int j = 0; j <= ncls; j++)
      if (hist[j] > best) { best = hist[j]; cls = (uint16_t)j; }
  }
  nd_cls[o] = cls;
}

// Bitonic sort of (key, idx) pairs ascending, n a power of two, within one workgroup.
__device__ void bitonic_pairs(unsigned long long* key, uint32_t* idx, uint32_t n) {
  for (uint32_t size = 2; size <= n; size <<= 1) {
    for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
      for (uint32_t t = threadIdx.x; t < n / 2; t += blockDim.x) {
        const uint32_t lo = 2 * t - (t & (stride - 1));
        const uint32_t hi = lo + stride;
        const bool up = (lo & size) == 0;
        const unsigned long long ka = key[lo], kb = key[hi];
        const uint32_t ia = idx[lo], ib = idx[hi];
        const bool gt = ka > kb || (ka == kb && ia > ib);
        if (gt == up) {
          key[lo] = kb; key[hi] = ka;
          idx[lo] = ib; idx[hi] = ia;
        }
      }
      __syncthreads();
    }
  }
}

struct KLArgs {
  CloudCtl* ctl;
  const uint32_t* dense_all;
  const uint32_t* vox_all;
  const uint32_t* nd_n;
  const double* nd_mean;
  const double* nd_cov;
  double* nd_cov_post;
  const uint16_t* nd_cls;
  int32_t* nb_all;
  uint32_t* keys_all;
  uint32_t* nkeys_all;
  double* chain_all;
  uint32_t* chain_ps_all;
  double* slot_val_all;
  uint32_t* slot_flag_all;
  double* ev_val_all;
  uint32_t* ev_p_all;
  uint32_t* ev_q_all;
  double* ev_min_all;
  unsigned long long* sort_key_all;
  uint32_t* sort_idx_all;
  uint32_t* nan_list_all;
  uint32_t* nan_pos_all;
  double* ord_val_all;
  uint32_t* ord_p_all;
  uint32_t* ord_q_all;
  uint32_t* first_occ_all;
  uint32_t* tmp_all;
  uint8_t* alive_all;
  float* out;            // [B][k][12] or null
  float* out_cls;        // [B][k][ncls+1] or null
  double* out_pc64;      // [B][k][3] or null (legacy ABI)
  double* out_cov64;     // [B][k][9] or null
  uint16_t* out_cls16;   // [B][k] or null
  ndnet_ndt_stats* stats;
  uint64_t vcap;
  uint32_t ndcap, ecap, sortcap;
  uint64_t k;
  int ncls;
};

// Prune (ndt.c:28-73) of cloud b's retained list to k NDs, then the output
// rows (ndt.c:75-117).  Shared by k_kl (level 1) and k_prune (later levels).
__device__ void prune_and_emit(const KLArgs& A, int b, uint64_t k, uint32_t* s_u32, uint32_t* scratch) {
  CloudCtl& c = A.ctl[b];
  const uint32_t nd = c.num_nds;
  const uint64_t ob = (uint64_t)b * A.ndcap, eb = (uint64_t)b * A.ecap;
  uint8_t* alive = A.alive_all + ob;
  uint32_t* first = A.first_occ_all + ob;
  const uint32_t* op = A.ord_p_all + eb;
  uint32_t* tmp = A.tmp_all + eb;
  __shared__ uint32_t s_failc, s_kpos, s_poison, s_kills;
  int32_t rc = 0;
  uint32_t kills = 0;
  const uint32_t nv0 = c.num_valid, nkl0 = c.num_kl;
  if (k > nv0) {
    rc = -1;  // "Number of desired normal distributions is greater ..." (ndt.c:36-39)
  } else {
    const uint32_t to_remove = (uint32_t)(nv0 - k);
    for (uint32_t u = threadIdx.x; u < nd; u += blockDim.x) first[u] = kInvalid;
    if (threadIdx.x == 0) { s_failc = kInvalid; s_kpos = kInvalid; s_poison = kInvalid; }
    __syncthreads();
    // first occurrence of each live p (entries of dead p are skipped by the walk)
    for (uint32_t i = threadIdx.x; i < nkl0; i += blockDim.x) {
      const uint32_t pp = op[i];
      if (pp == kInvalid) { atomicMin(&s_poison, i); continue; }
      if (alive[pp]) atomicMin(&first[pp], i);
    }
    __syncthreads();
    // walk order: the c-th first (1-based) at position f_c is killed iff
    // f_c < nkl0 - (c-1) for it and for every earlier first.
    uint32_t carry = 0;
    for (uint32_t base = 0; base < nkl0; base += blockDim.x) {
      const uint32_t i = base + threadIdx.x;
      uint32_t isf = 0;
      if (i < nkl0) {
        const uint32_t pp = op[i];
        isf = (pp != kInvalid && alive[pp] && first[pp] == i);
      }
      uint32_t tot;
      const uint32_t ex = block_excl_scan(isf, 0u, AddU32(), scratch, tot);
      if (isf) {
        const uint32_t cth = carry + ex + 1;
        tmp[i] = cth;
        if (cth <= to_remove && i >= nkl0 - (cth - 1)) atomicMin(&s_failc, cth);
        if (cth == to_remove) s_kpos = i;
      } else if (i < nkl0) {
        tmp[i] = 0;
      }
      carry += tot;
    }
    __syncthreads();
    const uint32_t F = carry;
    uint32_t failc = s_failc;
    if (failc == kInvalid && F < to_remove) failc = F + 1;  // the walk runs off the end
    // the walk visits positions [0, stop): up to the last kill, or up to the
    // bound check that fails (idx >= nkl - kills, ndt.c:53)
    uint32_t stop;
    if (to_remove == 0) stop = 0;
    else if (failc == kInvalid) stop = s_kpos + 1;
    else stop = nkl0 - (failc - 1);
    const bool poisoned = s_poison != kInvalid && s_poison < stop;
    if (poisoned) stop = s_poison;  // the reference would dereference an uninitialised entry here
    if (threadIdx.x == 0) s_kills = 0;
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < stop; i += blockDim.x) {
      const uint32_t cth = tmp[i];
      if (cth) {
        alive[op[i]] = 0;
        atomicMax(&s_kills, cth);
      }
    }
    __syncthreads();
    kills = s_kills;
    if (poisoned) rc = -8;
    else if (kills < to_remove) rc = -2;  // "Reached the end of the divergences array!"
    __syncthreads();
    if (rc == 0 && to_remove > 0) {
      // shift left by idx_to_remove = f_{to_remove} + 1 (ndt.c:69-72)
      const uint32_t shift = s_kpos + 1;
      const uint32_t nkl1 = nkl0 - to_remove;
      double* ov = A.ord_val_all + eb;
      uint32_t* oq = A.ord_q_all + eb;
      uint32_t* opw = A.ord_p_all + eb;
      // gather into registers in passes, then write (in-place left shift)
      for (uint32_t base = 0; base < nkl1; base += blockDim.x) {
        const uint32_t i = base + threadIdx.x;
        double v = 0;
        uint32_t pq = kInvalid, qq = kInvalid;
        if (i < nkl1) {
          const uint32_t src = i + shift;
          if (src < c.num_phys) { v = ov[src]; pq = opw[src]; qq = oq[src]; }
        }
        __syncthreads();
        if (i < nkl1) { ov[i] = v; opw[i] = pq; oq[i] = qq; }
        __syncthreads();
      }
      if (threadIdx.x == 0) c.num_kl = nkl1;
    } else if (threadIdx.x == 0) {
      c.num_kl = nkl0 - kills;
    }
    if (threadIdx.x == 0) c.num_valid = nv0 - kills;
  }
  __syncthreads();
  // output rows: survivors in ascending voxel order
  const uint64_t kout = k;
  const uint32_t* vn = A.nd_n + ob;
  uint32_t carry = 0;
  for (uint32_t base = 0; base < nd; base += blockDim.x) {
    const uint32_t u = base + threadIdx.x;
    const uint32_t live = (u < nd) && alive[u];
    uint32_t tot;
    const uint32_t row = carry + block_excl_scan(live, 0u, AddU32(), scratch, tot);
    if (live && row < kout) {
      const uint64_t o = (uint64_t)b * kout + row;
      const double* m = A.nd_mean + 3 * (ob + u);
      const double* cv = A.nd_cov_post + 9 * (ob + u);
      if (A.out) {
        float* r = A.out + 12 * o;
        for (int j = 0; j < 3; j++) {
          const float f = (float)m[j];
          r[j] = isfinite(f) ? f : 0.0f;  // nan_to_num(nan=0, posinf=0, neginf=0)
        }
        for (int j = 0; j < 9; j++) {
          const float f = (float)cv[j];
          r[3 + j] = isfinite(f) ? f : 0.0f;
        }
      }
      if (A.out_cls) {
        float* r = A.out_cls + (uint64_t)(A.ncls + 1) * o;
        r[A.nd_cls[ob + u]] = 1.0f;
      }
      if (A.out_pc64) {
        for (int j = 0; j < 3; j++) A.out_pc64[3 * o + j] = m[j];
        for (int j = 0; j < 9; j++) A.out_cov64[9 * o + j] = cv[j];
      }
      if (A.out_cls16) A.out_cls16[o] = A.nd_cls[ob + u];
    }
    carry += tot;
  }
  (void)vn;
  __syncthreads();
  if (threadIdx.x == 0) {
    c.prune_rc = rc;
    c.num_out = carry;
    c.last_k = (uint32_t)k;
  }
  (void)s_u32;
}

__device__ void write_stats(const KLArgs& A, int b) {
  const CloudCtl& c = A.ctl[b];
  ndnet_ndt_stats& s = A.stats[b];
  s.rc = c.rc;
  s.prune_rc = c.prune_rc;
  s.iters = c.iter;
  for (int a = 0; a < 3; a++) {
    s.len[a] = c.len[a];
    s.offset[a] = c.off[a];
  }
  s.voxel_size = c.vs;
  s.num_nds = c.num_nds;
  s.num_valid = c.num_valid;
  s.num_kl = c.num_kl;
  s.num_events = c.num_events;
  s.num_out = c.num_out;
}

// Zero the output rows of cloud b (np.zeros in ndt_legacy.py:126-143).
__device__ void zero_outputs(const KLArgs& A, int b, uint64_t k) {
  const uint64_t r0 = (uint64_t)b * k;
  if (A.out)
    for (uint64_t i = threadIdx.x; i < 12 * k; i += blockDim.x) A.out[12 * r0 + i] = 0.0f;
  if (A.out_cls) {
    const uint64_t w = (uint64_t)(A.ncls + 1);
    for (uint64_t i = threadIdx.x; i < w * k; i += blockDim.x) A.out_cls[w * r0 + i] = 0.0f;
  }
  if (A.out_pc64) {
    for (uint64_t i = threadIdx.x; i < 3 * k; i += blockDim.x) A.out_pc64[3 * r0 + i] = 0.0;
    for (uint64_t i = threadIdx.x; i < 9 * k; i += blockDim.x) A.out_cov64[9 * r0 + i] = 0.0;
  }
  if (A.out_cls16)
    for (uint64_t i = threadIdx.x; i < k; i += blockDim.x) A.out_cls16[r0 + i] = 0;
  __syncthreads();
}

// The class one-hot of rows past the survivors is class 0 (ndtnet_preprocessing.py:55-57).
__device__ void pad_class_rows(const KLArgs& A, int b, uint64_t k) {
  if (!A.out_cls) return;
  const CloudCtl& c = A.ctl[b];
  const uint64_t w = (uint64_t)(A.ncls + 1);
  for (uint64_t r = c.num_out + threadIdx.x; r < k; r += blockDim.x) A.out_cls[w * ((uint64_t)b * k + r)] = 1.0f;
}

__global__ void __launch_bounds__(kKLThreads) k_kl(KLArgs A) {
  const int b = blockIdx.x;
  CloudCtl& c = A.ctl[b];
  __shared__ double s_f64[16];
  __shared__ uint32_t s_u32[16];
  extern __shared__ __attribute__((aligned(16))) unsigned char dyn[];
  zero_outputs(A, b, A.k);
  if (c.state != kAccepted) {
    if (threadIdx.x == 0) {
      c.num_out = 0;
      write_stats(A, b);
    }
    pad_class_rows(A, b, A.k);
    return;
  }
  const uint32_t nd = c.num_nds;
  const uint64_t ob = (uint64_t)b * A.ndcap, eb = (uint64_t)b * A.ecap;
  const uint32_t* vox = A.vox_all + ob;
  const uint32_t* dense = A.dense_all + (uint64_t)b * A.vcap;
  const uint32_t* vn = A.nd_n + ob;
  int32_t* nb = A.nb_all + 6 * ob;
  uint32_t* keys = A.keys_all + 12 * ob;
  uint32_t* nkeys = A.nkeys_all + ob;
  double* chain = A.chain_all + 108 * ob;
  uint32_t* chain_ps = A.chain_ps_all + 12 * ob;
  const uint32_t lx = c.len[0], ly = c.len[1], lz = c.len[2];
  // -- neighbours (voxel.c:116-175, directions X+,X-,Y+,Y-,Z+,Z-)
  for (uint32_t u = threadIdx.x; u < nd; u += blockDim.x) {
    const uint32_t lin = vox[u];
    const uint32_t z = lin / (lx * ly), y = (lin % (lx * ly)) / lx, x = lin % lx;
    const int dx[6] = {1, -1, 0, 0, 0, 0}, dy[6] = {0, 0, 1, -1, 0, 0}, dz[6] = {0, 0, 0, 0, 1, -1};
    for (int d = 0; d < 6; d++) {
      const uint32_t xx = x + (uint32_t)dx[d], yy = y + (uint32_t)dy[d], zz = z + (uint32_t)dz[d];
      int32_t w = -1;
      if (xx < lx && yy < ly && zz < lz) {
        const uint32_t dn = dense[zz * lx * ly + yy * lx + xx];
        if (dn != kInvalid) w = (int32_t)dn;
      }
      nb[6 * u + d] = w;
    }
  }
  __syncthreads();
  // -- per ND: the sorted keys (6 v + d) of the mutating events it takes part in,
  //    and its chain of in-place LU factorisations
  for (uint32_t u = threadIdx.x; u < nd; u += blockDim.x) {
    uint32_t kk[12];
    int T = 0;
    const uint32_t nu = vn[u];
    if (nu > 1) {
      for (int d = 0; d < 6; d++) {
        const int32_t w = nb[6 * u + d];
        if (w < 0 || vn[w] <= 1) continue;
        kk[T++] = 6 * u + d;                 // u as p
        kk[T++] = 6 * (uint32_t)w + (d ^ 1); // u as q of w's opposite direction
      }
    }
    for (int i = 1; i < T; i++) {  // insertion sort
      const uint32_t v = kk[i];
      int j = i - 1;
      while (j >= 0 && kk[j] > v) { kk[j + 1] = kk[j]; j--; }
      kk[j + 1] = v;
    }
    double S[9];
    for (int j = 0; j < 9; j++) S[j] = A.nd_cov[9 * (ob + u) + j];
    for (int t = 0; t < T; t++) {
      uint32_t perm;
      int sg;
      lu3(S, perm, sg);
      for (int j = 0; j < 9; j++) chain[108 * u + 9 * t + j] = S[j];
      chain_ps[12 * u + t] = perm | (sg < 0 ? 0x100u : 0u);
      keys[12 * u + t] = kk[t];
    }
    nkeys[u] = (uint32_t)T;
    for (int j = 0; j < 9; j++) A.nd_cov_post[9 * (ob + u) + j] = S[j];
  }
  __syncthreads();
  // -- events, one per (voxel, direction) slot (kullback_leibler.c:141-180)
  double* slot_val = A.slot_val_all + eb;
  uint32_t* slot_flag = A.slot_flag_all + eb;
  const uint32_t nslots = 6 * nd;
  for (uint32_t s = threadIdx.x; s < nslots; s += blockDim.x) {
    const uint32_t u = s / 6, d = s % 6;
    const int32_t w = nb[6 * u + d];
    uint32_t flag = 0;
    double val = 0.0;
    if (w >= 0) {
      if (vn[u] <= 1 || vn[w] <= 1) {
        flag = 1;  // kl_divergence returns -1 with div 0 and the entry is kept
      } else {
        const uint32_t key = 6 * u + d;
        int rp = 0, rq = 0;
        while (keys[12 * u + rp] != key) rp++;
        while (keys[12 * (uint32_t)w + rq] != key) rq++;
        const double* LUp = chain + 108 * u + 9 * rp;
        const double* LUq = chain + 108 * (uint32_t)w + 9 * rq;
        const uint32_t psp = chain_ps[12 * u + rp], psq = chain_ps[12 * (uint32_t)w + rq];
        const int sp = (psp & 0x100) ? -1 : 1, sq = (psq & 0x100) ? -1 : 1;
        double Lp[9], Lq[9];
        for (int j = 0; j < 9; j++) { Lp[j] = LUp[j]; Lq[j] = LUq[j]; }
        const double pd = lu3_det(Lp, sp), qd = lu3_det(Lq, sq);
        if (!(pd == 0 || qd == 0) && lu3_sgndet(Lp, sp) != 0 && lu3_sgndet(Lq, sq) != 0) {
          flag = 1;
          val = kl_score(Lp, Lq, psq & 0x3f, pd, qd);
        }
      }
    }
    slot_val[s] = val;
    slot_flag[s] = flag;
  }
  __syncthreads();
  // -- compaction into enumeration order; NaN-skipping exclusive prefix min
  double* ev_val = A.ev_val_all + eb;
  uint32_t* ev_p = A.ev_p_all + eb;
  uint32_t* ev_q = A.ev_q_all + eb;
  uint32_t E = 0;
  {
    uint32_t carry = 0;
    for (uint32_t base = 0; base < nslots; base += blockDim.x) {
      const uint32_t s = base + threadIdx.x;
      const uint32_t f = s < nslots ? slot_flag[s] : 0u;
      uint32_t tot;
      const uint32_t e = carry + block_excl_scan(f, 0u, AddU32(), s_u32, tot);
      if (f) {
        ev_val[e] = slot_val[s];
        ev_p[e] = s / 6;
        ev_q[e] = (uint32_t)nb[s];
      }
      carry += tot;
    }
    E = carry;
  }
  __syncthreads();
  double* ev_min = A.ev_min_all + eb;
  uint32_t* nan_list = A.nan_list_all + eb;
  uint32_t* nan_pos = A.nan_pos_all + eb;
  unsigned long long* skey;
  uint32_t* sidx;
  uint32_t NN = 0, NNaN = 0;
  {
    // count non-NaN first to size the sort
    uint32_t carry = 0, carry_nan = 0;
    double mcarry = __builtin_inf();
    const bool fits = true;
    (void)fits;
    for (uint32_t base = 0; base < E; base += blockDim.x) {
      const uint32_t e = base + threadIdx.x;
      const double v = e < E ? ev_val[e] : 0.0;
      const bool isn = e < E && v != v;
      const uint32_t nn = (e < E && !isn) ? 1u : 0u;
      uint32_t tot;
      (void)block_excl_scan(nn, 0u, AddU32(), s_u32, tot);
      double mt;
      const double mv = (e < E && !isn) ? v : __builtin_inf();
      const double mex = block_excl_scan(mv, __builtin_inf(), MinF64(), s_f64, mt);
      if (e < E) ev_min[e] = MinF64()(mcarry, mex);
      mcarry = MinF64()(mcarry, mt);
      carry += tot;
      uint32_t totn;
      const uint32_t jn = carry_nan + block_excl_scan(isn ? 1u : 0u, 0u, AddU32(), s_u32, totn);
      if (isn) nan_list[jn] = e;
      carry_nan += totn;
    }
    NN = carry;
    NNaN = carry_nan;
  }
  uint32_t sortn = 1;
  while (sortn < NN) sortn <<= 1;
  if (sortn <= (uint32_t)kSortLds) {
    skey = reinterpret_cast<unsigned long long*>(dyn);
    sidx = reinterpret_cast<uint32_t*>(dyn + 8 * kSortLds);
  } else {
    skey = A.sort_key_all + (uint64_t)b * A.sortcap;
    sidx = A.sort_idx_all + (uint64_t)b * A.sortcap;
  }
  {
    uint32_t carry = 0;
    for (uint32_t base = 0; base < E; base += blockDim.x) {
      const uint32_t e = base + threadIdx.x;
      const double v = e < E ? ev_val[e] : 0.0;
      const uint32_t nn = (e < E && v == v) ? 1u : 0u;
      uint32_t tot;
      const uint32_t r = carry + block_excl_scan(nn, 0u, AddU32(), s_u32, tot);
      if (nn) {
        skey[r] = ~ord_key(v);  // ascending key == descending value
        sidx[r] = e;
      }
      carry += tot;
    }
    for (uint32_t r = NN + threadIdx.x; r < sortn; r += blockDim.x) {
      skey[r] = ~0ull;
      sidx[r] = kInvalid;
    }
  }
  __syncthreads();
  bitonic_pairs(skey, sidx, sortn);
  // NaN event t sits after the non-NaN x with x > m_t, or x == m_t occurring
  // before t: its insertion point in the sorted list.
  for (uint32_t j = threadIdx.x; j < NNaN; j += blockDim.x) {
    const uint32_t t = nan_list[j];
    const unsigned long long km = ~ord_key(ev_min[t]);
    uint32_t lo = 0, hi = NN;
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      const bool before = skey[mid] < km || (skey[mid] == km && sidx[mid] < t);
      if (before) lo = mid + 1;
      else hi = mid;
    }
    nan_pos[j] = lo;
  }
  __syncthreads();
  double* ov = A.ord_val_all + eb;
  uint32_t* opp = A.ord_p_all + eb;
  uint32_t* oq = A.ord_q_all + eb;
  for (uint32_t r = threadIdx.x; r < NN; r += blockDim.x) {
    // NaNs with insertion point <= r precede it (nan_pos is non-decreasing)
    uint32_t lo = 0, hi = NNaN;
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (nan_pos[mid] <= r) lo = mid + 1;
      else hi = mid;
    }
    const uint32_t pos = r + lo;
    const uint32_t e = sidx[r];
    ov[pos] = ev_val[e];
    opp[pos] = ev_p[e];
    oq[pos] = ev_q[e];
  }
  for (uint32_t j = threadIdx.x; j < NNaN; j += blockDim.x) {
    const uint32_t pos = nan_pos[j] + j;
    const uint32_t e = nan_list[j];
    ov[pos] = ev_val[e];
    opp[pos] = ev_p[e];
    oq[pos] = ev_q[e];
  }
  // poison beyond the written list (the reference's uninitialised tail)
  for (uint32_t i = E + threadIdx.x; i < A.ecap; i += blockDim.x) {
    opp[i] = kInvalid;
    oq[i] = kInvalid;
    ov[i] = 0.0;
  }
  for (uint32_t u = threadIdx.x; u < nd; u += blockDim.x) A.alive_all[ob + u] = 1;
  if (threadIdx.x == 0) {
    c.num_events = E;
    c.num_kl = E;
    c.num_phys = E;
    c.num_valid = nd;
  }
  __syncthreads();
  prune_and_emit(A, b, A.k, s_u32, s_u32);
  pad_class_rows(A, b, A.k);
  if (threadIdx.x == 0) write_stats(A, b);
}

__global__ void __launch_bounds__(kKLThreads) k_prune(KLArgs A) {
  const int b = blockIdx.x;
  CloudCtl& c = A.ctl[b];
  __shared__ uint32_t s_u32[16];
  zero_outputs(A, b, A.k);
  if (c.state != kAccepted) {
    pad_class_rows(A, b, A.k);
    if (threadIdx.x == 0) write_stats(A, b);
    return;
  }
  prune_and_emit(A, b, A.k, s_u32, s_u32);
  pad_class_rows(A, b, A.k);
  if (threadIdx.x == 0) write_stats(A, b);
}

// ------------------------------------------------------------------ host side

#define HIPCHK(x)                                                             \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "ndnet_amd: %s failed: %s\n", #x, hipGetErrorString(e_)); \
      return NDNET_ERR_HIP;                                                   \
    }                                                                         \
  } while (0)

template <typename T>
static hipError_t alloc(T** p, size_t count) {
  return hipMalloc((void**)p, (count ? count : 1) * sizeof(T));
}

static void plan_free(Plan* P) {
  if (!P) return;
  if (P->timing)
    for (int i = 0; i < 7; i++) (void)hipEventDestroy(P->ev[i]);
  void* bufs[] = {P->ctl, P->stamps, P->dense_of, P->vox, P->chunk_pts, P->chunk_lbl, P->chunk_tab, P->nd_n,
                  P->nd_mean, P->nd_cov, P->nd_cov_post, P->nd_cls, P->hist, P->nb, P->keys, P->nkeys,
                  P->chain, P->chain_ps, P->slot_val, P->slot_flag, P->ev_val, P->ev_p, P->ev_q, P->ev_min,
                  P->sort_key, P->sort_idx, P->nan_list, P->nan_pos, P->ord_val, P->ord_p, P->ord_q,
                  P->first_occ, P->tmp_u32, P->alive, P->d_stats};
  for (void* b : bufs)
    if (b) (void)hipFree(b);
  delete P;
}

static KLArgs kl_args(Plan* P, uint64_t k, float* out, float* out_cls, double* pc64, double* cov64, uint16_t* cls16) {
  KLArgs A;
  A.ctl = P->ctl;
  A.dense_all = P->dense_of;
  A.vox_all = P->vox;
  A.nd_n = P->nd_n;
  A.nd_mean = P->nd_mean;
  A.nd_cov = P->nd_cov;
  A.nd_cov_post = P->nd_cov_post;
  A.nd_cls = P->nd_cls;
  A.nb_all = P->nb;
  A.keys_all = P->keys;
  A.nkeys_all = P->nkeys;
  A.chain_all = P->chain;
  A.chain_ps_all = P->chain_ps;
  A.slot_val_all = P->slot_val;
  A.slot_flag_all = P->slot_flag;
  A.ev_val_all = P->ev_val;
  A.ev_p_all = P->ev_p;
  A.ev_q_all = P->ev_q;
  A.ev_min_all = P->ev_min;
  A.sort_key_all = P->sort_key;
  A.sort_idx_all = P->sort_idx;
  A.nan_list_all = P->nan_list;
  A.nan_pos_all = P->nan_pos;
  A.ord_val_all = P->ord_val;
  A.ord_p_all = P->ord_p;
  A.ord_q_all = P->ord_q;
  A.first_occ_all = P->first_occ;
  A.tmp_all = P->tmp_u32;
  A.alive_all = P->alive;
  A.out = out;
  A.out_cls = out_cls;
  A.out_pc64 = pc64;
  A.out_cov64 = cov64;
  A.out_cls16 = cls16;
  A.stats = P->d_stats;
  A.vcap = P->vcap;
  A.ndcap = P->ndcap;
  A.ecap = P->ecap;
  A.sortcap = P->sortcap;
  A.k = k;
  A.ncls = P->ncls;
  return A;
}

static size_t kl_lds_bytes() { return (size_t)kSortLds * (8 + 4); }

template <typename T>
static int run_impl(Plan* P, hipStream_t st, const T* pts, const int32_t* lbl, float* out, float* out_cls,
                    double* pc64, double* cov64, uint16_t* cls16, ndnet_ndt_stats* stats_dst) {
  const int B = P->B;
  const uint64_t n = P->n;
  if (lbl && P->ncls < 0) return NDNET_ERR_ARG;
  if (P->timing) HIPCHK(hipEventRecord(P->ev[0], st));
  k_reset<<<(B + 63) / 64, 64, 0, st>>>(P->ctl, B);
  const uint32_t Gl = (uint32_t)((n + 4095) / 4096);
  // stamps are epoch * 32 + pass; the device epoch wraps to 1 after 2^26 - 1 calls
  if (++P->calls % ((1u << 26) - 1) == 0)
    HIPCHK(hipMemsetAsync(P->stamps, 0, (size_t)B * P->vcap * sizeof(uint32_t), st));
  k_limits<T><<<dim3(Gl, B), 256, 0, st>>>(pts, P->ctl, n, Gl, P->vcap);
  if (P->timing) HIPCHK(hipEventRecord(P->ev[1], st));
  for (int it = 0; it < kMaxIters; it++)
    k_search_pass<T><<<dim3(P->G, B), kPassThreads, 0, st>>>(pts, P->ctl, P->stamps, n, P->k, P->G, P->vcap);
  if (P->timing) HIPCHK(hipEventRecord(P->ev[2], st));
  k_dense<<<B, 1024, 0, st>>>(P->ctl, P->stamps, P->dense_of, P->vox, P->vcap, P->ndcap);
  if (P->timing) HIPCHK(hipEventRecord(P->ev[3], st));
  k_chunk_sort<T><<<dim3(P->nchunks, B), kChunkThreads, 0, st>>>(
      pts, lbl, P->ctl, P->dense_of, (double*)P->chunk_pts, lbl ? P->chunk_lbl : nullptr, P->chunk_tab, n, P->vcap,
      P->ndcap, P->nchunks);
  if (P->timing) HIPCHK(hipEventRecord(P->ev[4], st));
  k_welford<<<dim3((P->ndcap + 255) / 256, B), 256, 0, st>>>(P->ctl, (const double*)P->chunk_pts,
                                                              lbl ? P->chunk_lbl : nullptr, P->chunk_tab, P->nd_n,
                                                              P->nd_mean, P->nd_cov, P->nd_cls, P->hist, P->ncls,
                                                              P->ndcap, P->nchunks);
  if (P->timing) HIPCHK(hipEventRecord(P->ev[5], st));
  KLArgs A = kl_args(P, P->k, out, out_cls, pc64, cov64, cls16);
  k_kl<<<B, kKLThreads, kl_lds_bytes(), st>>>(A);
  if (P->timing) HIPCHK(hipEventRecord(P->ev[6], st));
  if (stats_dst)
    HIPCHK(hipMemcpyAsync(stats_dst, P->d_stats, sizeof(ndnet_ndt_stats) * B, hipMemcpyDeviceToDevice, st));
  HIPCHK(hipGetLastError());
  return NDNET_OK;
}

}  // namespace

// ------------------------------------------------------------------ C ABI

extern "C" {

int ndnet_ndt_plan_create(int batch, uint64_t num_points, uint64_t num_desired, int num_classes,
                          uint64_t voxel_capacity, void** plan_out) {
  if (!plan_out || batch <= 0 || num_points == 0 || num_desired == 0 || num_points >= (1ull << 31))
    return NDNET_ERR_ARG;
  *plan_out = nullptr;
  Plan* P = new Plan();
  memset(P, 0, sizeof(Plan));
  P->B = batch;
  P->n = num_points;
  P->k = num_desired;
  P->ncls = num_classes;
  P->vcap = voxel_capacity ? voxel_capacity : (1ull << 22);
  const double upper = (double)num_desired * (1 + 0.2);
  P->ndcap = (uint32_t)upper + 1;
  P->ecap = 6 * P->ndcap;
  uint32_t sc = 1;
  while (sc < P->ecap) sc <<= 1;
  P->sortcap = sc;
  P->nchunks = (uint32_t)((num_points + kChunk - 1) / kChunk);
  const uint64_t n8 = (num_points / kWorkers) * kWorkers;
  P->G = (uint32_t)((n8 + kPassPts - 1) / kPassPts);
  if (P->G == 0) P->G = 1;
  if (P->ndcap >= (1u << 20)) {  // dense ids share a 32-bit sort key with a 12-bit chunk index
    delete P;
    return NDNET_ERR_ARG;
  }
  const size_t B = (size_t)batch, nd = P->ndcap, ec = P->ecap, nc = P->nchunks;
  const int nb = num_classes >= 0 ? num_classes + 1 : 1;
  hipError_t e = hipSuccess;
#define A_(ptr, cnt) \
  if (e == hipSuccess) e = alloc(&P->ptr, (cnt));
  A_(ctl, B);
  A_(stamps, B * P->vcap);
  A_(dense_of, B * P->vcap);
  A_(vox, B * nd);
  if (e == hipSuccess) e = hipMalloc(&P->chunk_pts, B * nc * kChunk * 3 * sizeof(double));
  A_(chunk_lbl, num_classes >= 0 ? B * nc * kChunk : 1);
  A_(chunk_tab, B * nc * nd);
  A_(nd_n, B * nd);
  A_(nd_mean, B * nd * 3);
  A_(nd_cov, B * nd * 9);
  A_(nd_cov_post, B * nd * 9);
  A_(nd_cls, B * nd);
  A_(hist, num_classes >= 0 ? B * nd * nb : 1);
  A_(nb, B * nd * 6);
  A_(keys, B * nd * 12);
  A_(nkeys, B * nd);
  A_(chain, B * nd * 108);
  A_(chain_ps, B * nd * 12);
  A_(slot_val, B * ec);
  A_(slot_flag, B * ec);
  A_(ev_val, B * ec);
  A_(ev_p, B * ec);
  A_(ev_q, B * ec);
  A_(ev_min, B * ec);
  A_(sort_key, B * P->sortcap);
  A_(sort_idx, B * P->sortcap);
  A_(nan_list, B * ec);
  A_(nan_pos, B * ec);
  A_(ord_val, B * ec);
  A_(ord_p, B * ec);
  A_(ord_q, B * ec);
  A_(first_occ, B * nd);
  A_(tmp_u32, B * ec);
  A_(alive, B * nd);
  A_(d_stats, B);
#undef A_
  if (e == hipSuccess) e = hipMemset(P->ctl, 0, B * sizeof(CloudCtl));
  if (e == hipSuccess) e = hipMemset(P->stamps, 0, B * P->vcap * sizeof(uint32_t));
  if (e == hipSuccess) e = hipMemset(P->d_stats, 0, B * sizeof(ndnet_ndt_stats));
  if (e == hipSuccess) e = hipFuncSetAttribute((const void*)k_kl, hipFuncAttributeMaxDynamicSharedMemorySize,
                                               (int)kl_lds_bytes());
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e != hipSuccess) {
    fprintf(stderr, "ndnet_amd: plan allocation failed: %s\n", hipGetErrorString(e));
    plan_free(P);
    return NDNET_ERR_HIP;
  }
  *plan_out = P;
  return NDNET_OK;
}

void ndnet_ndt_plan_destroy(void* plan) { plan_free((Plan*)plan); }

int ndnet_ndt_set_timing(void* plan, int enable) {
  Plan* P = (Plan*)plan;
  if (!P) return NDNET_ERR_ARG;
  if (enable && !P->timing)
    for (int i = 0; i < 7; i++) HIPCHK(hipEventCreate(&P->ev[i]));
  P->timing = P->timing || enable;
  return NDNET_OK;
}

int ndnet_ndt_stage_ms(void* plan, float* ms) {
  Plan* P = (Plan*)plan;
  if (!P || !P->timing || !ms) return NDNET_ERR_ARG;
  HIPCHK(hipEventSynchronize(P->ev[6]));
  for (int i = 0; i < 6; i++) HIPCHK(hipEventElapsedTime(&ms[i], P->ev[i], P->ev[i + 1]));
  return NDNET_OK;
}

int ndnet_ndt_run(void* plan, void* stream, const float* d_points, const int32_t* d_labels, float* d_out,
                  float* d_out_classes, ndnet_ndt_stats* d_stats) {
  Plan* P = (Plan*)plan;
  if (!P || !d_points) return NDNET_ERR_ARG;
  if (d_labels && P->ncls < 0) return NDNET_ERR_ARG;
  P->in_f64 = 0;
  return run_impl<float>(P, (hipStream_t)stream, d_points, d_labels, d_out, d_out_classes, nullptr, nullptr,
                         nullptr, d_stats);
}

int ndnet_ndt_run_f64(void* plan, void* stream, const double* d_points, const int32_t* d_labels, double* d_out_points,
                      double* d_out_covariances, uint16_t* d_out_classes, float* d_out, ndnet_ndt_stats* d_stats) {
  Plan* P = (Plan*)plan;
  if (!P || !d_points) return NDNET_ERR_ARG;
  if (d_labels && P->ncls < 0) return NDNET_ERR_ARG;
  P->in_f64 = 1;
  return run_impl<double>(P, (hipStream_t)stream, d_points, d_labels, d_out, nullptr, d_out_points,
                          d_out_covariances, d_out_classes, d_stats);
}

int ndnet_ndt_prune(void* plan, void* stream, uint64_t num_desired, float* d_out, float* d_out_classes,
                    double* d_out_points, double* d_out_covariances, uint16_t* d_out_classes16,
                    ndnet_ndt_stats* d_stats) {
  Plan* P = (Plan*)plan;
  if (!P || num_desired == 0) return NDNET_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  KLArgs A = kl_args(P, num_desired, d_out, d_out_classes, d_out_points, d_out_covariances, d_out_classes16);
  k_prune<<<P->B, kKLThreads, 0, st>>>(A);
  if (d_stats)
    HIPCHK(hipMemcpyAsync(d_stats, P->d_stats, sizeof(ndnet_ndt_stats) * P->B, hipMemcpyDeviceToDevice, st));
  HIPCHK(hipGetLastError());
  return NDNET_OK;
}

// Stage dumps for the parity tests (host copies of one cloud's intermediates).
int ndnet_ndt_debug_dump(void* plan, int cloud, uint32_t* nd_n, double* nd_mean, double* nd_cov_pre,
                         double* nd_cov_post, uint32_t* vox, double* ord_val, uint32_t* ord_p, uint32_t* ord_q,
                         double* guesses, uint32_t* counts, uint32_t* iters, uint8_t* alive) {
  Plan* P = (Plan*)plan;
  if (!P || cloud < 0 || cloud >= P->B) return NDNET_ERR_ARG;
  CloudCtl c;
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpy(&c, P->ctl + cloud, sizeof(CloudCtl), hipMemcpyDeviceToHost));
  const size_t ob = (size_t)cloud * P->ndcap, eb = (size_t)cloud * P->ecap;
  const size_t nd = c.num_nds;
  if (iters) *iters = c.iter;
  if (guesses) memcpy(guesses, c.guesses, sizeof(double) * (c.iter < 16 ? c.iter : 16));
  if (counts) memcpy(counts, c.counts, sizeof(uint32_t) * (c.iter < 16 ? c.iter : 16));
  if (c.state != kAccepted) return NDNET_OK;
  if (nd_n) HIPCHK(hipMemcpy(nd_n, P->nd_n + ob, nd * 4, hipMemcpyDeviceToHost));
  if (nd_mean) HIPCHK(hipMemcpy(nd_mean, P->nd_mean + 3 * ob, nd * 24, hipMemcpyDeviceToHost));
  if (nd_cov_pre) HIPCHK(hipMemcpy(nd_cov_pre, P->nd_cov + 9 * ob, nd * 72, hipMemcpyDeviceToHost));
  if (nd_cov_post) HIPCHK(hipMemcpy(nd_cov_post, P->nd_cov_post + 9 * ob, nd * 72, hipMemcpyDeviceToHost));
  if (vox) HIPCHK(hipMemcpy(vox, P->vox + ob, nd * 4, hipMemcpyDeviceToHost));
  if (ord_val) HIPCHK(hipMemcpy(ord_val, P->ord_val + eb, (size_t)c.num_events * 8, hipMemcpyDeviceToHost));
  if (ord_p) HIPCHK(hipMemcpy(ord_p, P->ord_p + eb, (size_t)c.num_events * 4, hipMemcpyDeviceToHost));
  if (ord_q) HIPCHK(hipMemcpy(ord_q, P->ord_q + eb, (size_t)c.num_events * 4, hipMemcpyDeviceToHost));
  if (alive) HIPCHK(hipMemcpy(alive, P->alive + ob, nd, hipMemcpyDeviceToHost));
  return NDNET_OK;
}

}  // extern "C"
