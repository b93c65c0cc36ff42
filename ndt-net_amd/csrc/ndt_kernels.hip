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
//   k_welford      a lane quad per ND, sequential Welford in point order
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
#include <stdlib.h>
#include <string.h>
#include <mutex>
#include <type_traits>
#include <vector>

#include "ndt_device.h"
#include "../../include/ndnet_amd.h"

#pragma clang fp contract(off)

using namespace ndnet;

namespace {

constexpr int kPassThreads = 256;    // threads per search workgroup
constexpr int kPassPPT = 4;          // points per thread per search workgroup
constexpr int kPassPts = kPassThreads * kPassPPT;
constexpr int kHashSlots = 2048;     // LDS dedup table of a search workgroup (>= kBitsWords)
constexpr int kBitsCap = 32768;      // grids up to this many voxels count through bitmaps
constexpr int kBitsWords = kBitsCap / 32;
constexpr int kKLThreads = 1024;
constexpr int kChunk = 256;          // slots per chunk of the chip-wide event sort
constexpr int kKLMarks = 32;  // phase stamps per cloud of the KL kernels (timing level 2)
constexpr int kMergeLdsChunks = 34;  // k_kl_merge stages score + NaN keys in LDS up to this many chunks (136 KB)
constexpr int kMergeScoreChunks = 72; // ... and the score runs alone up to this many (144 KB; k <= 2440)
constexpr int kMaxChunks = 6 * 16384 / kChunk;  // ndcap <= 16384
// NDs with at least this many samples get a whole wave each in k_welford_q
// (wq_heavy): k_front / k_bin_offsets list them per cloud.  The plan's
// default (ndnet_ndt_set_heavy_threshold).
#ifndef NDNET_WQ_HEAVY
#define NDNET_WQ_HEAVY 256
#endif
constexpr uint32_t kWqHeavy = NDNET_WQ_HEAVY;

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
  uint32_t acc_mode;     // occupancy of the accepted pass: 0/1 bitmap buffer, 2 stamps
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
  uint32_t clear_stamps; // the epoch wrapped this run: k_limits zeroes the cloud's stamps
  uint32_t kl_deferred;  // the retained list was not built by the run (lazy list, num_nds <= k)
  uint32_t flag_count;   // events of a deferred cloud, counted by k_kl_rank_chunks (zeroed per run)
  uint32_t list_off;     // physical index of the retained list's first entry (the prunes' pending
                         // left shifts, ndt.c:69-72; always 0 on the global-memory prune path)
  uint32_t heavy_n;      // NDs of the accepted grid with >= kWqHeavy samples, listed in Plan::heavy
                         // (written by the binning of every run that accepts a grid)
  uint32_t heavy_t;      // the threshold that list was built with: k_welford_q's light items skip
                         // exactly the NDs it holds, whatever the plan's threshold is by then
  uint32_t kl_arrive;    // k_kl_merge<.., kTail> workgroups of the cloud done (re-armed by the last)
};

struct Plan {
  int B;
  uint64_t n;
  uint64_t k;
  int ncls;            // num_classes (histograms have ncls+1 bins)
  uint64_t vcap;       // voxels per cloud the stamp / dense tables hold
  uint32_t ndcap;      // max accepted NDs per cloud = floor(1.2 k) + 1
  uint32_t ecap;       // 6 * ndcap
  uint32_t nbins;      // 1024-point binning chunks per cloud
  uint32_t G;          // search workgroups per cloud
  int in_f64;          // input element type of the last run
  uint64_t calls;      // runs issued from the host (graph replays not counted)
  int timing;          // 0 off, 1 stage events, 2 + k_kl phase marks
  int ev_created;
  hipEvent_t ev[8];
  unsigned long long* kl_marks;  // [B][kKLMarks] s_memrealtime stamps (timing level 2)
  unsigned long long* wq_marks;  // [wq_items][kWqMarkW] k_welford_q per-item stamps (timing level 2)
  // device buffers
  CloudCtl* ctl;
  uint32_t* stamps;    // [B][vcap]
  uint32_t* dense_of;  // [B][vcap]
  uint32_t* vox;       // [B][ndcap] linear index of dense id
  uint32_t* gbits;     // [B][2][kBitsWords] occupancy bitmaps of small-grid passes
  uint32_t* pkeys;     // [B][n] voxel key of every point in the latest pass
  uint32_t* did;       // [B][n] dense id of every point in the accepted pass
  uint32_t* bin_cnt;   // [B][nbins][ndcap] per-chunk histograms -> offsets
  uint32_t* nd_base;   // [B][ndcap]
  void* nd_pts;        // [B][n][3] points grouped by ND (input element type)
  uint16_t* nd_lbl;    // [B][n]
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
  uint32_t* chain_ok;  // [B][ndcap] bit t: LU state t has det != 0 and sgndet != 0 (lazy clouds only)
  double* slot_val;    // [B][ecap]
  uint32_t* slot_flag; // [B][ecap]
  double* ev_val;      // [B][ecap]
  uint32_t* ev_p;      // [B][ecap]
  uint32_t* ev_q;      // [B][ecap]
  double* ev_min;      // [B][ecap] exclusive prefix min (NaN-skipping)
  unsigned long long* sort_key;  // [B][sortcap]
  uint32_t* sort_idx;  // [B][sortcap]
  uint32_t* nan_list;  // [B][ecap] NaN slots per chunk (chunk * kChunk + j)
  unsigned long long* nan_key;  // [B][ecap] NaN keys, contiguous in slot order
  uint32_t* nan_slot;  // [B][ecap] their slots
  uint32_t* chunk_nanbase;  // [B][nchunk] NaN events in earlier chunks
  double* ord_val;     // [B][ecap] the retained list (physical array)
  uint32_t* ord_p;     // [B][ecap]
  uint32_t* ord_q;     // [B][ecap]
  uint32_t* first_occ; // [B][ndcap]
  uint32_t* tmp_u32;   // [B][ecap] scratch
  uint8_t* alive;      // [B][ndcap]
  uint32_t sortcap;    // chunked sort arrays per cloud: roundup(ecap, kChunk)
  uint32_t nchunk;     // kChunk-slot chunks per cloud (max)
  uint32_t* chunk_cnt; // [B][nchunk] (non-NaN count << 16) | NaN count
  double* chunk_min;   // [B][nchunk] min non-NaN value of the chunk (+inf if none)
  ndnet_ndt_stats* d_stats;  // [B] device copy of the stats
  // k_front (ndt_front.h): the fused front of the pipeline
  int front;                 // 1: k_front path, 0: the multi-kernel path
  int front_ok;              // the plan's shape admits k_front
  uint32_t fG, fbpw, frbs;   // workgroups per cloud, 1024-point bins per workgroup, points per rank bin
  size_t flds;               // dynamic LDS bytes of k_front
  unsigned long long* flims; // [B][fG][6]
  uint32_t* frec;            // [B][kFrontPhases][fG][kRecWords]
  uint32_t* fwgcnt;          // [B][fG][ndcap]
  uint32_t* fbar;            // [B][kBarStride]
  unsigned long long* fmarks; // [B][kFrontMarkStride]: k_front phase stamps of WG 0 + start/end of every WG (timing level 2)
  int exact_counts;           // k_front counts every bisection grid (ndnet_ndt_set_exact_counts)
  int wq_l64;                 // k_welford_q light form: 1 light64 (one ND per lane), 0 lane quads
  int wq_form;                // 0 auto (quads at CU share 1, light64 above), 1 light64, 2 quads
  uint32_t wq_grid;           // k_welford_q workgroups: one per CU (of the plan's CU share)
  int cus;                    // the device's CUs
  int cu_share;               // k_front / k_welford_q use CUs / cu_share (ndnet_ndt_set_cu_share)
  uint32_t* wq_ctr;           // [8][16] k_welford_q dynamic item counters, one per XCD (re-armed by k_kl_rank_chunks)
  int eager_list;             // build every cloud's retained list in the run (ndnet_ndt_set_lazy_list(plan, 0))
  int kl_fuse;                // the run's prune rides on the merge launch (kl_fusable; NDNET_KL_FUSE=0: k_kl)
  int list_sort;              // 2 (auto): k_kl_sort at a CU share > 1 where the list fits (sort_fits); 1: wherever it fits;
                              // 3: as 1 in k_kl_rank_sort's one launch; 0: k_kl_merge (NDNET_KL_SORT)
  uint64_t front_sync_ticks;  // k_front's cloud-barrier timeout (ndnet_ndt_debug_set_sync_timeout)
  int lists_built;            // the deferred lists of the last run are built (no further build launches)
  int front_staged;           // k_front's scatter through LDS records (ndnet_ndt_set_front_staged; default 1)
  int run_part;               // ndnet_ndt_set_run_part: 0 whole run, 1 front only, 2 from k_welford_q on
  int lane_rec;               // this run's k_front still to be recorded on its lanes (front_lanes_finish)
  int lane_g;                 // this plan's share of FrontLaneSet::gsum (G - 1)
  uint32_t* heavy;            // [B][ndcap] the heavy NDs of each cloud (CloudCtl::heavy_n of them)
  double* rtab;               // [n + 1][2] (rc, rl) per count for wq_heavy's divisions
  uint32_t* lu_done;          // [B][ceil(ndcap / 64)] k_welford_q's per-group completion counters (re-armed to 0)
  uint32_t heavy_t;           // NDs with >= heavy_t samples take wq_heavy (ndnet_ndt_set_heavy_threshold)
  // k_front admission (front_gate): the device's front lanes this plan's
  // k_front occupies, and the barrier-timeout flag k_front raises in host memory
  int dev;                    // the device the plan lives on
  int lane0, nlanes;          // lanes [lane0, lane0 + nlanes) mod kFrontLanes
  hipEvent_t front_ev;        // records this plan's k_front launches (the lanes' admission)
  uint32_t* sync_fail_h;      // pinned host word (mapped): nonzero after a k_front barrier timeout
  uint32_t* sync_fail_d;      // its device address
};

// ------------------------------------------------------------------ helpers

__device__ inline uint32_t hash32(uint32_t k) { return (k * 2654435761u) >> (32 - 11); }

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

// Exclusive block scan over ITEMS consecutive elements per thread (one
// barrier round for blockDim * ITEMS elements).  v[j] becomes the exclusive
// prefix of element j within the round; total is the round's reduction.
template <int ITEMS, typename T, typename Op>
__device__ inline void block_scan_items(T (&v)[ITEMS], T identity, Op op, T* scratch, T& total) {
  T local = identity;
#pragma unroll
  for (int j = 0; j < ITEMS; j++) {
    const T x = v[j];
    v[j] = local;
    local = op(local, x);
  }
  const T ex = block_excl_scan(local, identity, op, scratch, total);
#pragma unroll
  for (int j = 0; j < ITEMS; j++) v[j] = op(ex, v[j]);
}

struct AddU64 {
  __device__ unsigned long long operator()(unsigned long long a, unsigned long long b) const { return a + b; }
};

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

__global__ void k_reset(CloudCtl* ctl, int B, uint32_t* bar, uint32_t* lu_done, uint32_t gcap) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  // k_welford_q's 64-ND group counters: re-armed by the wave that completes a
  // group, and here at the start of every run (a run that failed half way
  // cannot leave one non-zero)
  if (lu_done)
    for (uint32_t i = 0; i < gcap; i++) lu_done[(uint64_t)b * gcap + i] = 0;
  if (bar)  // k_front's cloud barrier counter and its two pass-sum slots (kBarStride)
    for (int i = 0; i < 6; i++) bar[(uint64_t)b * 16 + i] = 0;
  CloudCtl& c = ctl[b];
  c.epoch = c.epoch + 1;
  // stamps are epoch*32 + pass; on a wrap the stale stamps are cleared on the
  // device (k_limits), so a captured graph replayed any number of times stays
  // correct without host bookkeeping
  c.clear_stamps = 0;
  if (c.epoch >= (1u << 26)) {
    c.epoch = 1;
    c.clear_stamps = 1;
  }
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
  c.flag_count = 0;
  c.kl_arrive = 0;
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

// Workgroup arrival ticket of a cloud: true for the last of G arrivals.
// Everything the workgroups hand to the last one (counts, cut-offs, bitmap
// and stamp words) is written with device-scope atomics, which the caller has
// drained (s_waitcnt vmcnt(0) in every wave before the barrier), so the
// ticket needs no release fence (an L2 write-back per workgroup), and the last
// workgroup reads those words with atomic loads, so it needs no acquire.
__device__ inline bool arrive_ticket(uint32_t* arrive, uint32_t G) {
  return __hip_atomic_fetch_add(arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == G - 1;
}

constexpr int kLimPPT = 16;        // flat coordinates per thread in k_limits

// Bounding box (pointclouds.c:40-66) over every point, the n % 8 tail
// included.  Coordinates are read as a flat, coalesced stream; element f is
// axis f % 3.
template <typename T>
__global__ void __launch_bounds__(256) k_limits(const T* __restrict__ pts, CloudCtl* ctl, uint32_t* gbits_all,
                                                uint32_t* stamps, uint64_t n, uint32_t G, uint64_t vcap) {
  const int b = blockIdx.y;
  if (ctl[b].clear_stamps) {  // epoch wrap (k_reset): rare, cost irrelevant
    uint32_t* sb = stamps + (uint64_t)b * vcap;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < vcap; i += (uint64_t)G * 256) sb[i] = 0;
  }
  const T* p = pts + (uint64_t)b * n * 3;
  const uint64_t nf = 3 * n;
  double mx[3] = {kDblMin, kDblMin, kDblMin}, mn[3] = {kDblMax, kDblMax, kDblMax};
  const uint64_t f0 = (uint64_t)blockIdx.x * 256 * kLimPPT + threadIdx.x;
  T v[kLimPPT];
#pragma unroll
  for (int j = 0; j < kLimPPT; j++) {
    const uint64_t f = f0 + 256 * j;
    v[j] = f < nf ? p[f] : T(0);
  }
  const uint32_t a0 = (uint32_t)(f0 % 3);  // 256 = 1 (mod 3): element j is axis (a0 + j) % 3
#pragma unroll
  for (int j = 0; j < kLimPPT; j++) {
    const uint64_t f = f0 + 256 * j;
    if (f >= nf) continue;
    const uint32_t a = (a0 + j) % 3;
    const double x = (double)v[j];
#pragma unroll
    for (int ax = 0; ax < 3; ax++) {
      // maxf(point, cur) / minf(point, cur): a NaN coordinate never wins
      mx[ax] = (a == (uint32_t)ax && x > mx[ax]) ? x : mx[ax];
      mn[ax] = (a == (uint32_t)ax && x < mn[ax]) ? x : mn[ax];
    }
  }
  unsigned long long kmx[3], kmn[3];
#pragma unroll
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
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  __shared__ uint32_t last;
  if (threadIdx.x == 0) last = arrive_ticket(&c.arrive, G);
  __syncthreads();
  if (!last) return;
  if (threadIdx.x == 0) {
    for (int a = 0; a < 6; a++)
      c.lim[a] = ord_unkey(__hip_atomic_load(&c.limkey[a], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    c.arrive = 0;
    c.lo = kMinGuess;
    c.hi = kMaxGuess;
    set_guess(c, (kMaxGuess - kMinGuess) / 2.0, vcap);  // ndt.c:136
  }
  __syncthreads();
  if (c.state == kSearching && c.V <= (uint64_t)kBitsCap) {  // clear pass 0's occupancy bitmap
    uint32_t* gb = gbits_all + (uint64_t)b * 2 * kBitsWords;
    for (uint32_t w = threadIdx.x; w < (uint32_t)((c.V + 31) / 32); w += blockDim.x) gb[w] = 0;
  }
}

// Large-grid path of a pass: dedup keys in an LDS hash table; the thread that
// inserts a key flips the voxel's global stamp.  Returns the new voxels.
__device__ inline uint32_t stamp_key(uint32_t key, uint32_t* table, uint32_t* stamps, uint32_t stamp) {
  if (table) {
    uint32_t h = hash32(key);
    bool mine = false;
    for (int probe = 0; probe < kHashSlots; probe++) {
      const uint32_t cur = table[h];
      if (cur == key) break;
      if (cur == kInvalid) {
        const uint32_t old = atomicCAS(&table[h], kInvalid, key);
        if (old == kInvalid) { mine = true; break; }
        if (old == key) break;
      }
      h = (h + 1) & (kHashSlots - 1);
    }
    if (!mine) return 0;
  }
  uint32_t* s = stamps + key;
  if (__hip_atomic_load(s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == stamp) return 0;
  return atomicExch(s, stamp) != stamp;
}

__device__ inline uint32_t block_sum_u32(uint32_t v, uint32_t* scratch) {
  uint32_t tot;
  (void)block_excl_scan(v, 0u, AddU32(), scratch, tot);
  return tot;
}

// Bisection decision of ndt.c:168-187 after a pass counted `count` NDs.
__device__ inline void finish_pass(CloudCtl& c, uint32_t count, uint64_t k, uint64_t vcap, uint32_t mode) {
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
    c.acc_mode = mode;
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

// One bisection pass (estimate_ndt's occupancy, normal_distributions.c:38-60
// + ndt.c:158-176) over kPassPts points of one cloud per workgroup.  The
// points are staged through LDS with coalesced loads; each point's voxel key
// is kept (keys_all) for the binning of the accepted pass.  Small grids
// (V <= kBitsCap) count distinct voxels with an LDS bitmap per workgroup
// merged by one global atomicOr per word; larger grids use per-voxel stamps.
template <typename T>
__global__ void __launch_bounds__(kPassThreads) k_search_pass(const T* __restrict__ pts, CloudCtl* ctl,
                                                              uint32_t* stamps_all, uint32_t* gbits_all,
                                                              uint32_t* keys_all, uint64_t n, uint64_t k, uint32_t G,
                                                              uint64_t vcap) {
  const int b = blockIdx.y;
  CloudCtl& c = ctl[b];
  if (__hip_atomic_load(&c.state, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != kSearching) return;
  __shared__ T sp[3 * kPassPts];
  __shared__ uint32_t table[kHashSlots];  // LDS bitmap (small grids) or hash table
  __shared__ uint32_t scratch[16];
  __shared__ uint32_t last;
  const uint64_t chunk = n / kWorkers;       // pcl_worker range, normal_distributions.c:34-35
  const uint64_t n8 = chunk * kWorkers;      // the n % 8 tail is never estimated
  const T* p = pts + (uint64_t)b * n * 3;
  uint32_t* stamps = stamps_all + (uint64_t)b * vcap;
  const uint32_t stamp = c.stamp;
  const uint32_t parity = c.iter & 1u;
  uint32_t* gbits = gbits_all + ((uint64_t)b * 2 + parity) * kBitsWords;
  const bool small = c.V <= (uint64_t)kBitsCap;
  const uint32_t words = small ? (uint32_t)((c.V + 31) / 32) : 0u;
  const uint64_t start = (uint64_t)blockIdx.x * kPassPts;
  const uint32_t cnt = start < n8 ? (uint32_t)(n8 - start < (uint64_t)kPassPts ? n8 - start : kPassPts) : 0u;
#pragma unroll
  for (int j = 0; j < 3 * kPassPPT; j++) {
    const uint32_t f = threadIdx.x + kPassThreads * j;
    if (f < 3 * cnt) sp[f] = p[3 * start + f];
  }
  if (small) {
    for (uint32_t w = threadIdx.x; w < words; w += blockDim.x) table[w] = 0;
  } else {
    for (int i = threadIdx.x; i < kHashSlots; i += blockDim.x) table[i] = kInvalid;
  }
  __syncthreads();
  const double vs = c.guess, inv_vs = 1.0 / vs;
  uint32_t fresh = 0;
#pragma unroll
  for (int q = 0; q < kPassPPT; q++) {
    const uint32_t il = threadIdx.x + kPassThreads * q;
    if (il >= cnt) continue;
    const uint64_t i = start + il;
    const uint32_t key = voxel_key((double)sp[3 * il], (double)sp[3 * il + 1], (double)sp[3 * il + 2], c.off, c.len,
                                   vs, inv_vs);
    keys_all[(uint64_t)b * n + i] = key;
    if (key == kInvalid) {
      atomicMin(&c.first_bad[i / chunk], (uint32_t)i);
    } else if (small) {
      atomicOr(&table[key >> 5], 1u << (key & 31));
    } else {
      fresh += stamp_key(key, table, stamps, stamp);
    }
  }
  if (small) {
    __syncthreads();
    for (uint32_t w = threadIdx.x; w < words; w += blockDim.x) {
      const uint32_t bits = table[w];
      if (bits) fresh += __popc(bits & ~atomicOr(&gbits[w], bits));
    }
  }
  fresh = block_sum_u32(fresh, scratch);
  if (threadIdx.x == 0 && fresh) atomicAdd(&c.count, fresh);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) last = arrive_ticket(&c.arrive, G);
  __syncthreads();
  if (!last) return;
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
  uint32_t mode = small ? parity : 2u;
  if (any_bad) {
    const uint32_t stamp2 = c.epoch * 32u + 16u + c.iter;
    uint32_t f = 0;
    for (uint64_t i = threadIdx.x; i < n8; i += blockDim.x) {
      if (i >= cut[i / chunk]) continue;
      double x[3];
      load_point(p, i, x);
      const uint32_t key = voxel_key(x[0], x[1], x[2], c.off, c.len, vs, inv_vs);
      if (key != kInvalid) f += stamp_key(key, nullptr, stamps, stamp2);
    }
    count = block_sum_u32(f, scratch);
    if (threadIdx.x == 0) c.stamp = stamp2;
    mode = 2u;
  } else {
    count = __hip_atomic_load(&c.count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    c.count = 0;
    c.arrive = 0;
    finish_pass(c, count, k, vcap, mode);
  }
  __syncthreads();
  if (c.state == kSearching && c.V <= (uint64_t)kBitsCap) {  // clear the next pass's bitmap
    uint32_t* gb = gbits_all + ((uint64_t)b * 2 + (c.iter & 1u)) * kBitsWords;
    for (uint32_t w = threadIdx.x; w < (uint32_t)((c.V + 31) / 32); w += blockDim.x) gb[w] = 0;
  }
}

// Occupied voxels of the accepted grid -> dense ids in ascending linear order.
__global__ void __launch_bounds__(1024) k_dense(CloudCtl* ctl, const uint32_t* stamps_all,
                                                const uint32_t* gbits_all, uint32_t* dense_all, uint32_t* vox_all,
                                                uint64_t vcap, uint32_t ndcap) {
  const int b = blockIdx.x;
  const CloudCtl& c = ctl[b];
  if (c.state != kAccepted) return;
  __shared__ uint32_t scratch[16];
  uint32_t* dense = dense_all + (uint64_t)b * vcap;
  uint32_t* vox = vox_all + (uint64_t)b * ndcap;
  const uint64_t V = c.V;
  if (c.acc_mode < 2) {  // the pass's occupancy bitmap: one word per thread
    const uint32_t* gb = gbits_all + ((uint64_t)b * 2 + c.acc_mode) * kBitsWords;
    const uint32_t words = (uint32_t)((V + 31) / 32);
    uint32_t carry = 0;
    for (uint32_t base = 0; base < words; base += blockDim.x) {
      const uint32_t w = base + threadIdx.x;
      const uint32_t bits = w < words ? gb[w] : 0u;
      uint32_t tot;
      uint32_t d = carry + block_excl_scan((uint32_t)__popc(bits), 0u, AddU32(), scratch, tot);
      if (w < words) {
        for (int j = 0; j < 32; j++) {
          const uint64_t v = 32ull * w + j;
          if (v >= V) break;
          if ((bits >> j) & 1u) {
            dense[v] = d;
            if (d < ndcap) vox[d] = (uint32_t)v;
            d++;
          } else {
            dense[v] = kInvalid;
          }
        }
      }
      carry += tot;
    }
    return;
  }
  const uint32_t* st = stamps_all + (uint64_t)b * vcap;
  const uint32_t stamp = c.accepted_stamp;
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

// --- binning of the accepted pass: points grouped by ND, in index order ---
//
// k_bin_count   per 1024-point chunk: dense id of every point the reference
//               estimates (kInvalid past a worker's cut-off or the n % 8 tail)
//               and the chunk's histogram over NDs
// k_bin_offsets per ND: its base (prefix over NDs) and its start within every
//               chunk (prefix over chunks): a stable counting sort
// k_bin_scatter per chunk: stable rank within the chunk (LDS bitonic sort of
//               (id, index)), points written to their ND's contiguous run
constexpr int kBinPts = 1024;
constexpr int kNdSlack = 64;  // points of padding after the last cloud's ND runs
constexpr int kBinThreads = 256;

__global__ void __launch_bounds__(kBinThreads) k_bin_count(const CloudCtl* ctl, const uint32_t* __restrict__ keys_all,
                                                           const uint32_t* __restrict__ dense_all, uint32_t* did_all,
                                                           uint32_t* counts_all, uint64_t n, uint64_t vcap,
                                                           uint32_t ndcap, uint32_t nbins) {
  const int b = blockIdx.y, ch = blockIdx.x;
  const CloudCtl& c = ctl[b];
  if (c.state != kAccepted) return;
  extern __shared__ __attribute__((aligned(16))) uint32_t hist[];
  const uint32_t nd = c.num_nds;
  for (uint32_t d = threadIdx.x; d < nd; d += blockDim.x) hist[d] = 0;
  __syncthreads();
  const uint64_t chunk = n / kWorkers, n8 = chunk * kWorkers;
  const uint32_t* dense = dense_all + (uint64_t)b * vcap;
  const uint64_t base = (uint64_t)ch * kBinPts;
#pragma unroll
  for (int q = 0; q < kBinPts / kBinThreads; q++) {
    const uint64_t i = base + threadIdx.x + kBinThreads * q;
    if (i >= n) continue;
    uint32_t d = kInvalid;
    if (i < n8 && i < c.first_bad[i / chunk]) {
      const uint32_t key = keys_all[(uint64_t)b * n + i];
      if (key != kInvalid) d = dense[key];
    }
    did_all[(uint64_t)b * n + i] = d;
    if (d != kInvalid) atomicAdd(&hist[d], 1u);
  }
  __syncthreads();
  uint32_t* row = counts_all + ((uint64_t)b * nbins + ch) * ndcap;
  for (uint32_t d = threadIdx.x; d < nd; d += blockDim.x) row[d] = hist[d];
}

__global__ void __launch_bounds__(1024) k_bin_offsets(CloudCtl* ctl, uint32_t* counts_all, uint32_t* nd_n,
                                                      uint32_t* nd_base, uint32_t* heavy, uint32_t heavy_t,
                                                      uint32_t ndcap, uint32_t nbins) {
  const int b = blockIdx.x;
  CloudCtl& c = ctl[b];
  if (c.state != kAccepted) return;
  __shared__ uint32_t scratch[16];
  __shared__ uint32_t s_heavy;
  if (threadIdx.x == 0) s_heavy = 0;
  __syncthreads();
  const uint32_t nd = c.num_nds;
  uint32_t* cnt = counts_all + (uint64_t)b * nbins * ndcap;
  uint32_t carry = 0;
  for (uint32_t base = 0; base < nd; base += blockDim.x) {
    const uint32_t d = base + threadIdx.x;
    uint32_t tot_d = 0;
    if (d < nd) {
      uint32_t part[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      uint32_t ch = 0;
      for (; ch + 8 <= nbins; ch += 8) {
#pragma unroll
        for (int j = 0; j < 8; j++) part[j] += cnt[(uint64_t)(ch + j) * ndcap + d];
      }
      for (; ch < nbins; ch++) part[0] += cnt[(uint64_t)ch * ndcap + d];
#pragma unroll
      for (int j = 0; j < 8; j++) tot_d += part[j];
    }
    uint32_t tot;
    const uint32_t start = carry + block_excl_scan(tot_d, 0u, AddU32(), scratch, tot);
    if (d < nd) {
      nd_n[(uint64_t)b * ndcap + d] = tot_d;
      nd_base[(uint64_t)b * ndcap + d] = start;
      if (tot_d >= heavy_t) heavy[(uint64_t)b * ndcap + atomicAdd(&s_heavy, 1u)] = d;  // a wave each in k_welford_q
      uint32_t run = start;
      uint32_t ch = 0;
      for (; ch + 8 <= nbins; ch += 8) {
        uint32_t x[8];
#pragma unroll
        for (int j = 0; j < 8; j++) x[j] = cnt[(uint64_t)(ch + j) * ndcap + d];
#pragma unroll
        for (int j = 0; j < 8; j++) {
          cnt[(uint64_t)(ch + j) * ndcap + d] = run;
          run += x[j];
        }
      }
      for (; ch < nbins; ch++) {
        const uint32_t x = cnt[(uint64_t)ch * ndcap + d];
        cnt[(uint64_t)ch * ndcap + d] = run;
        run += x;
      }
    }
    carry += tot;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    c.heavy_n = s_heavy;
    c.heavy_t = heavy_t;
  }
}

template <typename T>
__global__ void __launch_bounds__(kBinThreads) k_bin_scatter(const T* __restrict__ pts, const int32_t* __restrict__ lbl,
                                                             const CloudCtl* ctl, const uint32_t* __restrict__ did_all,
                                                             const uint32_t* __restrict__ offs_all, T* nd_pts,
                                                             uint16_t* nd_lbl, uint64_t n, uint32_t ndcap,
                                                             uint32_t nbins) {
  const int b = blockIdx.y, ch = blockIdx.x;
  const CloudCtl& c = ctl[b];
  if (c.state != kAccepted) return;
  __shared__ uint32_t skey[kBinPts];
  __shared__ uint32_t scratch[16];
  const uint64_t base = (uint64_t)ch * kBinPts;
#pragma unroll
  for (int q = 0; q < kBinPts / kBinThreads; q++) {
    const uint32_t t = threadIdx.x + kBinThreads * q;
    const uint64_t i = base + t;
    const uint32_t d = i < n ? did_all[(uint64_t)b * n + i] : kInvalid;
    skey[t] = d == kInvalid ? kInvalid : (d << 10) | t;
  }
  __syncthreads();
  for (int size = 2; size <= kBinPts; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = threadIdx.x; t < kBinPts / 2; t += blockDim.x) {
        const int lo = 2 * t - (t & (stride - 1));
        const int hi = lo + stride;
        const bool up = (lo & size) == 0;
        const uint32_t a = skey[lo], bb = skey[hi];
        if ((a > bb) == up) { skey[lo] = bb; skey[hi] = a; }
      }
      __syncthreads();
    }
  }
  // rank within the run of equal ids: position - first position of the run
  const uint32_t* offs = offs_all + ((uint64_t)b * nbins + ch) * ndcap;
  const T* p = pts + (uint64_t)b * n * 3;
  uint32_t run_carry = 0;
#pragma unroll
  for (int q = 0; q < kBinPts / kBinThreads; q++) {
    const uint32_t s = threadIdx.x + kBinThreads * q;  // consecutive per pass: a block scan of run starts
    const uint32_t key = skey[s];
    const bool head = key != kInvalid && (s == 0 || (skey[s - 1] >> 10) != (key >> 10));
    uint32_t tot;
    // max-scan of run heads via an exclusive scan of (head ? s : 0) with max
    uint32_t hs = head ? s + 1 : 0u;
    uint32_t x = wave_incl_scan(hs, [](uint32_t a, uint32_t bb) { return a > bb ? a : bb; });
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 63) scratch[wid] = x;
    __syncthreads();
    uint32_t pre = run_carry;
    for (int w2 = 0; w2 < wid; w2++) pre = pre > scratch[w2] ? pre : scratch[w2];
    tot = run_carry;
    for (int w2 = 0; w2 < (int)(blockDim.x >> 6); w2++) tot = tot > scratch[w2] ? tot : scratch[w2];
    __syncthreads();
    const uint32_t head_pos = (x > pre ? x : pre) - 1;  // last run head at or before s
    run_carry = tot;
    if (key == kInvalid) continue;
    const uint32_t d = key >> 10, t = key & 1023;
    const uint32_t dst = offs[d] + (s - head_pos);
    const uint64_t i = base + t;
    T* o = nd_pts + ((uint64_t)b * n + dst) * 3;
    o[0] = p[3 * i + 0];
    o[1] = p[3 * i + 1];
    o[2] = p[3 * i + 2];
    if (nd_lbl) nd_lbl[(uint64_t)b * n + dst] = (uint16_t)lbl[(uint64_t)b * n + i];
  }
}

#include "ndt_front.h"

// k_welford_q: the same per-ND Welford (same lane quad, same double
// operations on the same operands, so the same bits), without LDS windows:
// every quad streams its own ND's points from nd_pts, so a wave runs as long as
// its longest ND and no ND waits for another's window.  Per sample, lane j
// (< 3) loads its own coordinate x_j, updates
//   t = x - mean; mean += t / n; u = x - mean; m2 += t * u
// and for its off-diagonal pair (a, b) = (0,1), (1,2), (0,2) takes u_a (axis
// a already updated) and t_b (axis b not yet: x_b - old mean_b) from the quad
// by DPP: cov_ab += u_a * t_b / n (normal_distributions.c:82-103, axes in
// order).  The two divisions by n use the refined reciprocal of n
// (div_fast: bit-identical to the division over the operand range that
// finite float coordinates guarantee); n = step + 1 is the same for every
// quad of a wave at a given step, so the reciprocal comes from a
// plan-lifetime table by a scalar load.  Coordinates are prefetched into two
// register blocks of kWqU samples (one block in flight while the other is
// folded).  A quad that meets a coordinate outside that range (non-finite
// float, or a double outside [2^-300, 2^300]) refolds its ND with IEEE
// divisions and the reference's NaN -> 0 step.  Labelled runs: the whole
// quad builds the class histogram in LDS (first index of the max,
// normal_distributions.c:107-121).
constexpr int kWqMarkW = 8;  // per item at timing level 2: realtime start, memtime start / moments done / end, meta,
                             // heavy items: cycles in phases 0 + 2, 1, 3
constexpr int kWqThreads = 256;              // 4 waves x 16 quads
constexpr int kWqNDs = kWqThreads / 4;
constexpr int kWqU = 16;                     // samples per prefetch block
constexpr int kWqNB = 4;                     // register blocks in the prefetch ring
#ifndef NDNET_WQ_RT
#define NDNET_WQ_RT 4096
#endif
#ifdef NDNET_WQ_WPE  // A/B: cap the registers (waves per SIMD) so other kernels' waves fit beside it
#define NDNET_WQ_ATTR __attribute__((amdgpu_waves_per_eu(NDNET_WQ_WPE)))
#else
#define NDNET_WQ_ATTR
#endif
constexpr int kWqRt = NDNET_WQ_RT;           // reciprocals tabled in LDS at most (32 KB; larger counts compute theirs)
// Entries of the table a run needs: the light quads' counts stay below the
// heavy threshold, so 256 entries (2 KB) by default instead of 32 KB -- LDS
// another stream's kernels can use beside k_welford_q (pipelined U +2 %,
// profiles/r04_wq_lds.txt); counts past the table compute their reciprocal.
__host__ __device__ inline uint32_t wq_rt_entries(uint32_t heavy_t) {
#ifdef NDNET_WQ_RTFULL  // A/B: the whole table whatever the threshold (round 1-4 form)
  return (uint32_t)kWqRt;
#endif
  // + 32: a light64 group's last round reads the pairs of up to 3 x 8 counts past its longest ND
  return heavy_t + 32u < (uint32_t)kWqRt ? (heavy_t + 32u + 31u) & ~31u : (uint32_t)kWqRt;
}
constexpr int kWqHistMax = 64 * 1024;        // LDS class histograms up to this size, else global
// Float input: a lane loads whole (x, y, z) records -- a quarter of its quad's
// block, one dwordx3 each -- and the quad transposes them through LDS (lane j
// then holds coordinate j of every sample): a quarter of the load
// instructions per sample.  L's heaviest ND spent 16 of its 122 us on point
// loads (23 with their issue); records took 6 us off it, and 2-3 us off C5's
// welford (profiles/r02h_welford_loads.txt).  NDNET_WQ_VU = 2 (32-sample
// blocks, 128 samples in flight -- the per-coordinate loads were capped by the
// 63 outstanding loads a wave can count) gained 1 us more on L but lost 2 on
// C2 and 3 on C5 (longer masked tails).
#ifndef NDNET_WQ_VLOAD
#define NDNET_WQ_VLOAD 1
#endif
constexpr int kWqStageQ = 100;               // LDS words per quad stage (96 + pad: conflict-free reads)
template <typename T, bool kVec, int kU>
struct WqBlk { T v[kU]; };                       // coordinate j of samples q0 .. q0 + kU - 1 (lane j)
template <int kU>
struct WqBlk<float, true, kU> { float3 v[kU / 4]; };  // records q0 + (kU / 4) j + i, i < kU / 4 (lane j)

template <int CTRL>
__device__ inline double dpp_d(double v) {
  const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)u, CTRL, 0xF, 0xF, false);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(u >> 32), CTRL, 0xF, 0xF, false);
  return __builtin_bit_cast(double, (unsigned long long)lo | ((unsigned long long)hi << 32));
}

template <typename T>
__device__ inline bool wq_in_range(T v) {
  if constexpr (sizeof(T) == 4) {
    return (__builtin_bit_cast(uint32_t, v) & 0x7f800000u) != 0x7f800000u;  // finite
  } else {
    const double a = fabs((double)v);
    return a == 0.0 || (a >= 0x1p-300 && a <= 0x1p300);
  }
}

// v_cndmask on both halves of a double, as inline asm: a plain `c ? a : b`
// lets the compiler turn the update it selects into an exec-masked branch,
// which ends the basic block and with it the overlap of consecutive samples.
__device__ inline double sel_d(unsigned long long lanes, double a, double b) {  // lanes set: a
  const unsigned long long ua = __builtin_bit_cast(unsigned long long, a);
  const unsigned long long ub = __builtin_bit_cast(unsigned long long, b);
  uint32_t lo, hi;
  asm("v_cndmask_b32 %0, %1, %2, %3" : "=v"(lo) : "v"((uint32_t)ub), "v"((uint32_t)ua), "s"(lanes));
  asm("v_cndmask_b32 %0, %1, %2, %3" : "=v"(hi) : "v"((uint32_t)(ub >> 32)), "v"((uint32_t)(ua >> 32)), "s"(lanes));
  return __builtin_bit_cast(double, (unsigned long long)lo | ((unsigned long long)hi << 32));
}

__device__ inline uint32_t wave_min_u32(uint32_t v) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t w = (uint32_t)__shfl_xor((int)v, o, 64);
    v = w < v ? w : v;
  }
  return __builtin_amdgcn_readfirstlane(v);
}

__device__ inline uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t w = (uint32_t)__shfl_xor((int)v, o, 64);
    v = w > v ? w : v;
  }
  return __builtin_amdgcn_readfirstlane(v);
}

// Event order of one ND's in-place LU chain: the mutating events
// it takes part in, by ascending key 6 * dense(v) + d.  Neighbours below it
// (Z-, Y-, X-: smaller linear index) come first, as q; then its own six
// directions, as p; then the neighbours above (X+, Y+, Z+), as q.  So the
// chain position of an event is a popcount over a 12-slot mask:
//   slot 0 Z-(q), 1 Y-(q), 2 X-(q), 3..8 own d = 0..5 (p), 9 X+(q), 10 Y+(q), 11 Z+(q)
__device__ inline uint32_t chain_mask(uint32_t e) {  // e: 6 eligible-direction bits
  return ((e >> 5) & 1u) | (((e >> 3) & 1u) << 1) | (((e >> 1) & 1u) << 2) | ((e & 0x3fu) << 3) |
         ((e & 1u) << 9) | (((e >> 2) & 1u) << 10) | (((e >> 4) & 1u) << 11);
}
__device__ inline uint32_t qslot_of_dir(uint32_t d) {  // q-slot of the neighbour in direction d
  return (0x0b1a29u >> (4 * d)) & 0xfu;  // {d0: 9, d1: 2, d2: 10, d3: 1, d4: 11, d5: 0}
}

// ---- one long ND's moments on a whole wave (wq_heavy) ----
//
// The lane-quad fold issues ~18 wave instructions per sample for the 16 NDs
// of a wave, so a wave lasts as long as its longest ND: on L clouds (heaviest
// ND 1675 samples) that one quad set the whole kernel's time.  Only the mean
// is a true recurrence:
//   t_i = x_i - mean_{i-1};  mean_i = mean_{i-1} + t_i / n_i
// Everything else of a sample -- u_i = x_i - mean_i, t_i u_i, the
// off-diagonal u_a t_b and its division by n_i -- depends only on that
// sequence and the sample, and only the sums m2 += t u and cov_ab += u_a t_b / n
// must run in sample order.  So per 64-sample block:
//   0. every lane loads one sample (its record and (rc, rl)), the block's
//      coordinates go to LDS;
//   1. lanes 0..2 (one axis each) run the mean recurrence, 4 dependent FP64
//      operations per sample, (rc, rl) from scalar loads, the means to LDS;
//      in the same loop lanes 3..8 add the PREVIOUS block's addends in sample
//      order (one accumulator each: m2 of the three axes, cov_01, cov_12,
//      cov_02): one add per sample beside the recurrence, its latency hidden;
//   2. every lane computes its own sample's six addends from the means.
// The same IEEE operations on the same operands in the same order as the
// reference (normal_distributions.c:75-103), so the same bits.  LDS traffic
// of the loop is one 16-byte read and one 16-byte write per lane per two
// samples (the loop's operands are loaded a group ahead; a lone wave pays
// ~15-30 cycles per LDS instruction: tools/ubench/fp64_latency.hip).
//
// The division t / n is RN(t rc + RN(t rl)) with rc ~ 1/n (within an ulp) and
// rl = RN((1 - n rc) / n) (1 - n rc is exact): t rc + RN(t rl) is within
// 2^-104 |t/n| of t/n, while t/n (t a double, n < 2^32 an integer) is never a
// rounding midpoint and never within 2^-86 |t/n| of one, so the fused add
// rounds to RN(t / n) -- two dependent operations instead of three
// (div_fast).  Range: every operand here is normal (|t| >= 2^-353 or 0 for
// the coordinates the fast path admits); a zero t may give a zero of the
// other sign, which no sum can see (they start at +0 and never become -0).
// tests/test_oracle.py::test_rtab_division_is_ieee checks the rule against
// the division on 10^7 operands.  rtab[0] = (0, 0): a step with it is an
// exact no-op (t + 0), which pads the last block's recurrence to 64 steps.
constexpr int kHvS = 66;  // LDS row stride (doubles): 16-byte rows on distinct banks for lanes 0..8
constexpr int kHvLds = 12 * kHvS;  // X[3], M[3], V[6] rows: 792 doubles = 6336 B per wave

template <typename T>
struct HvRec {
  T x, y, z;
  double2 r;  // (rc, rl) of n = this sample's count
};

template <typename T>
__device__ inline void hv_load(HvRec<T>& h, const T* __restrict__ rec, const double2* __restrict__ rtab,
                               uint32_t q0, uint32_t lane, uint32_t cnt) {
  const uint32_t q0l = q0 + lane, q = q0l < cnt ? q0l : cnt - 1;
  const T* p = rec + 3u * q;
  h.x = p[0];
  h.y = p[1];
  h.z = p[2];
  h.r = rtab[q + 1];
}

// 8 steps of the fused loop: lanes 0..2 the recurrence (m), lanes 3..8 the
// ordered sums (acc); xv = the lane's coordinate or addend, r = (rc, rl) in
// scalar registers; the means (garbage in lanes 3..8) kept for the write.
__device__ inline void hv_steps8(double& m, double& acc, const double (&xv)[8], const double2 (&r)[8],
                                 double (&mo)[8]) {
#pragma unroll
  for (int u = 0; u < 8; u++) {
    const double t = xv[u] - m;
    m = m + fma(t, r[u].x, t * r[u].y);
    acc = acc + xv[u];
    mo[u] = m;
  }
}

template <bool kTail>  // kTail: the last block, steps past nb use rtab[0] (no-ops)
__device__ inline void hv_ops8(double (&xv)[8], double2 (&r)[8], const double* __restrict__ rd,
                               const double2* __restrict__ rtab, uint32_t q0, uint32_t i0, uint32_t nb) {
#pragma unroll
  for (int u = 0; u < 8; u += 2) {
    const double2 v = *reinterpret_cast<const double2*>(rd + i0 + u);
    xv[u] = v.x;
    xv[u + 1] = v.y;
  }
#pragma unroll
  for (int u = 0; u < 8; u++) r[u] = rtab[kTail ? (i0 + u < nb ? q0 + i0 + u + 1 : 0u) : q0 + i0 + u + 1];
}

__device__ inline void hv_write8(double* __restrict__ wr, const double (&mo)[8], uint32_t i0) {
#pragma unroll
  for (int u = 0; u < 8; u += 2) *reinterpret_cast<double2*>(wr + i0 + u) = make_double2(mo[u], mo[u + 1]);
}

// the fused loop over one block: 64 steps, operands a group of 8 ahead, each
// group's means written while the next group runs
template <bool kTail>
__device__ inline void hv_block(double& m, double& acc, const double* __restrict__ rd, double* __restrict__ wr,
                                const double2* __restrict__ rtab, uint32_t q0, uint32_t nb) {
  double xA[8], xB[8], mA[8], mB[8];
  double2 rA[8], rB[8];
  hv_ops8<kTail>(xA, rA, rd, rtab, q0, 0, nb);
  hv_ops8<kTail>(xB, rB, rd, rtab, q0, 8, nb);
  asm volatile("" ::: "memory");
  hv_steps8(m, acc, xA, rA, mA);
#pragma unroll
  for (uint32_t i0 = 8; i0 < 64; i0 += 16) {
    hv_write8(wr, mA, i0 - 8);
    if (i0 + 8 < 64) hv_ops8<kTail>(xA, rA, rd, rtab, q0, i0 + 8, nb);
    asm volatile("" ::: "memory");
    hv_steps8(m, acc, xB, rB, mB);
    hv_write8(wr, mB, i0);
    if (i0 + 16 < 64) hv_ops8<kTail>(xB, rB, rd, rtab, q0, i0 + 16, nb);
    asm volatile("" ::: "memory");
    if (i0 + 8 < 64) hv_steps8(m, acc, xA, rA, mA);
  }
}

// The full-block loop with its memory operations as inline asm, so that
// their order and waits are exactly this: per group G of 8 steps, one
// s_waitcnt lgkmcnt(0) covers its operands (issued a group earlier: four
// ds_read_b128 of the lane's row, two s_load_dwordx16 of the (rc, rl) table)
// and the mean writes of group G - 2; then the means of group G - 1 are
// written and group G + 1's operands issued before group G's steps.  (With
// compiler-placed loads the scalar loads, which return out of order, made
// every wait an lgkmcnt(0) right at the use.)  The wait's in-out operands
// keep every use of the loaded registers behind it.
typedef unsigned int hv_u16 __attribute__((ext_vector_type(16)));
typedef double hv_d2 __attribute__((ext_vector_type(2)));  // native vector (HIP's double2 is a struct)

#ifndef NDNET_WQ_HV_RLDS
#define NDNET_WQ_HV_RLDS 1
#endif
#if NDNET_WQ_HV_RLDS
// (rc, rl) of the 8 steps from the block's LDS row (every lane the same
// address: a broadcast), written in phase 0 from the (rc, rl) each lane
// loaded for its own sample three blocks ahead (HvRec::r) -- no scalar loads,
// whose scalar-cache misses cost ~14 cycles per sample (profiles/r04_wq_rtab.txt)
struct HvOps {
  hv_d2 x[4];  // 8 steps' coordinates (lanes 0..2) or addends (lanes 3..8)
  hv_d2 r[8];  // (rc, rl) of the 8 steps
};

template <int G>
__device__ inline void hv_issue(HvOps& o, uint32_t rda, uint32_t rra) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(o.x[0]) : "v"(rda), "n"(64 * G));
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(o.x[1]) : "v"(rda), "n"(64 * G + 16));
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(o.x[2]) : "v"(rda), "n"(64 * G + 32));
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(o.x[3]) : "v"(rda), "n"(64 * G + 48));
#pragma unroll
  for (int u = 0; u < 8; u++)
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(o.r[u]) : "v"(rra), "n"(128 * G + 16 * u));
}
__device__ inline void hv_wait(HvOps& o) {
  asm volatile("s_waitcnt lgkmcnt(0)"
               : "+v"(o.x[0]), "+v"(o.x[1]), "+v"(o.x[2]), "+v"(o.x[3]), "+v"(o.r[0]), "+v"(o.r[1]), "+v"(o.r[2]),
                 "+v"(o.r[3]), "+v"(o.r[4]), "+v"(o.r[5]), "+v"(o.r[6]), "+v"(o.r[7]));
}
#else
struct HvOps {
  hv_d2 x[4];  // 8 steps' coordinates (lanes 0..2) or addends (lanes 3..8)
  hv_u16 r0, r1;  // (rc, rl) of the 8 steps, in scalar registers
};

template <int G>
__device__ inline void hv_issue(HvOps& o, uint32_t rda, const double2* rtq) {
  hv_d2 x0, x1, x2, x3;
  hv_u16 r0, r1;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(x0) : "v"(rda), "n"(64 * G));
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(x1) : "v"(rda), "n"(64 * G + 16));
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(x2) : "v"(rda), "n"(64 * G + 32));
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(x3) : "v"(rda), "n"(64 * G + 48));
  asm volatile("s_load_dwordx16 %0, %1, %2" : "=s"(r0) : "s"(rtq), "n"(128 * G));
  asm volatile("s_load_dwordx16 %0, %1, %2" : "=s"(r1) : "s"(rtq), "n"(128 * G + 64));
  o.x[0] = x0;
  o.x[1] = x1;
  o.x[2] = x2;
  o.x[3] = x3;
  o.r0 = r0;
  o.r1 = r1;
}
__device__ inline void hv_wait(HvOps& o) {
  hv_d2 x0 = o.x[0], x1 = o.x[1], x2 = o.x[2], x3 = o.x[3];
  hv_u16 r0 = o.r0, r1 = o.r1;
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+s"(r0), "+s"(r1));
  o.x[0] = x0;
  o.x[1] = x1;
  o.x[2] = x2;
  o.x[3] = x3;
  o.r0 = r0;
  o.r1 = r1;
}
#endif
template <int G>
__device__ inline void hv_put(uint32_t wra, const double (&mo)[8]) {
  const hv_d2 a = {mo[0], mo[1]}, b = {mo[2], mo[3]}, c = {mo[4], mo[5]}, d = {mo[6], mo[7]};
  asm volatile("ds_write_b128 %0, %1 offset:%2" ::"v"(wra), "v"(a), "n"(64 * G));
  asm volatile("ds_write_b128 %0, %1 offset:%2" ::"v"(wra), "v"(b), "n"(64 * G + 16));
  asm volatile("ds_write_b128 %0, %1 offset:%2" ::"v"(wra), "v"(c), "n"(64 * G + 32));
  asm volatile("ds_write_b128 %0, %1 offset:%2" ::"v"(wra), "v"(d), "n"(64 * G + 48));
}
__device__ inline double hv_sd(const hv_u16& v, int k) {
  return __builtin_bit_cast(double, (unsigned long long)v[2 * k] | ((unsigned long long)v[2 * k + 1] << 32));
}
__device__ inline void hv_steps(double& m, double& acc, const HvOps& o, double (&mo)[8]) {
#pragma unroll
  for (int u = 0; u < 8; u++) {
    const double xv = o.x[u >> 1][u & 1];
#if NDNET_WQ_HV_RLDS
    const double rc = o.r[u][0], rl = o.r[u][1];
#else
    const hv_u16& r = u < 4 ? o.r0 : o.r1;
    const double rc = hv_sd(r, 2 * (u & 3)), rl = hv_sd(r, 2 * (u & 3) + 1);
#endif
    const double t = xv - m;
    m = m + fma(t, rc, t * rl);
    acc = acc + xv;
    mo[u] = m;
  }
}
#if NDNET_WQ_HV_RLDS
typedef uint32_t HvRt;  // LDS byte address of the block's (rc, rl) row
#else
typedef const double2* HvRt;  // the block's first (rc, rl) in the global table
#endif
template <int G>  // group G of a full block: wait for its operands, write G - 1's means, issue G + 1's operands, step
__device__ inline void hv_group(double& m, double& acc, HvOps& cur, HvOps& nxt, double (&mcur)[8],
                                double (&mprev)[8], uint32_t rda, uint32_t wra, HvRt rtq) {
  hv_wait(cur);
  if constexpr (G > 0) hv_put<G - 1>(wra, mprev);
  if constexpr (G < 7) hv_issue<G + 1>(nxt, rda, rtq);
  // the steps are plain VALU code, which the compiler may move above the
  // asm statements before it: without this the next group's reads went out
  // after this group's steps, right before their wait (the LDS latency
  // exposed once per group).  m and acc pass through an asm statement placed
  // after the reads, so the steps start only once they are issued.
#ifndef NDNET_WQ_HV_ORDER
#define NDNET_WQ_HV_ORDER 1
#endif
#if NDNET_WQ_HV_ORDER
  asm volatile("" : "+v"(m), "+v"(acc));
#endif
  hv_steps(m, acc, cur, mcur);
}
__device__ inline void hv_block_asm(double& m, double& acc, uint32_t rda, uint32_t wra, HvRt rtq) {
  HvOps A, B;
  double mA[8], mB[8];
  hv_issue<0>(A, rda, rtq);
  hv_group<0>(m, acc, A, B, mA, mB, rda, wra, rtq);
  hv_group<1>(m, acc, B, A, mB, mA, rda, wra, rtq);
  hv_group<2>(m, acc, A, B, mA, mB, rda, wra, rtq);
  hv_group<3>(m, acc, B, A, mB, mA, rda, wra, rtq);
  hv_group<4>(m, acc, A, B, mA, mB, rda, wra, rtq);
  hv_group<5>(m, acc, B, A, mB, mA, rda, wra, rtq);
  hv_group<6>(m, acc, A, B, mA, mB, rda, wra, rtq);
  hv_group<7>(m, acc, B, A, mB, mA, rda, wra, rtq);
  hv_put<7>(wra, mB);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the block's means are in LDS for phase 2
}

template <typename T, bool kStamp = false>  // kStamp: phase cycle totals to ph[0..2] (timing level 2)
__device__ inline void wq_heavy(const T* __restrict__ rec, uint32_t cnt, const double2* __restrict__ rtab,
                                double* __restrict__ lds, double2* __restrict__ hr, uint32_t lane, double& mean,
                                double& m2, double& off, bool& bad, unsigned long long* ph = nullptr) {
  unsigned long long ts = 0, c0 = 0, c1 = 0, c2 = 0;
  auto stamp = [&](unsigned long long& acc) __attribute__((always_inline)) {
    if constexpr (kStamp) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      acc += t - ts;
      ts = t;
    }
  };
  if constexpr (kStamp) ts = __builtin_amdgcn_s_memtime();
  double* X = lds;              // [3][kHvS] the block's coordinates
  double* M = lds + 3 * kHvS;   // [3][kHvS] [1] the mean before the block, [2 + i] after sample i
  double* V = lds + 6 * kHvS;   // [6][kHvS] the previous block's addends: t u (3 axes), u_a t_b / n (3 pairs)
  const uint32_t a = lane < 3 ? lane : 0;
  // the fused loop's rows: lanes 0..2 read X[a] and write M[a][2..]; lanes
  // 3..8 read V[lane - 3] and write their (unused) means back over what they
  // have read
  const double* rd = lane < 3 ? X + a * kHvS : V + (lane < 9 ? lane - 3 : 0) * kHvS;
  double* wr = lane < 3 ? M + a * kHvS + 2 : V + (lane < 9 ? lane - 3 : 0) * kHvS;
  double m = 0.0, acc = 0.0;
  bool out = false;
#pragma unroll
  for (int p = 0; p < 6; p++) V[p * kHvS + lane] = 0.0;  // block 0 has no previous addends
  HvRec<T> h0, h1, h2;  // blocks q0, q0 + 64, q0 + 128 in flight
  hv_load(h0, rec, rtab, 0, lane, cnt);
  hv_load(h1, rec, rtab, 64, lane, cnt);
  hv_load(h2, rec, rtab, 128, lane, cnt);
  uint32_t nb = 64;
  for (uint32_t q0 = 0; q0 < cnt; q0 += 64) {
    const HvRec<T> h = h0;
    h0 = h1;
    h1 = h2;
    hv_load(h2, rec, rtab, q0 + 192, lane, cnt);
    nb = cnt - q0 < 64u ? cnt - q0 : 64u;  // samples of this block (wave-uniform)
    const double x0 = (double)h.x, x1 = (double)h.y, x2 = (double)h.z;
    if constexpr (!std::is_same<T, float>::value)
      out |= lane < nb && !(wq_in_range(h.x) && wq_in_range(h.y) && wq_in_range(h.z));
    // 0. the block to LDS; the running mean as M[.][1]
    X[lane] = x0;
    X[kHvS + lane] = x1;
    X[2 * kHvS + lane] = x2;
    if (lane < 3) M[a * kHvS + 1] = m;
#if NDNET_WQ_HV_RLDS
    hr[lane] = h.r;  // the block's (rc, rl) row for the loop's broadcast reads
#endif
    asm volatile("" ::: "memory");  // one wave's LDS operations complete in order
    stamp(c0);
    // 1. the recurrence (lanes 0..2) + the previous block's ordered sums (lanes 3..8)
    if (lane < 9) {
      if (nb == 64)
        hv_block_asm(m, acc, (uint32_t)(uintptr_t)(__attribute__((address_space(3))) const double*)rd,
                     (uint32_t)(uintptr_t)(__attribute__((address_space(3))) double*)wr,
#if NDNET_WQ_HV_RLDS
                     (uint32_t)(uintptr_t)(__attribute__((address_space(3))) double2*)hr);
#elif defined(NDNET_WQ_HV_FIXRT)  // timing experiment only (wrong results): every block reads block 0's (rc, rl)
                     rtab + 1);
#else
                     rtab + q0 + 1);
#endif
      else
        hv_block<true>(m, acc, rd, wr, rtab, q0, nb);
    }
    asm volatile("" ::: "memory");
    stamp(c1);
    // 2. every lane: its sample's addends (lanes past nb: unused)
    {
      const double t0 = x0 - M[lane + 1], u0 = x0 - M[lane + 2];
      const double t1 = x1 - M[kHvS + lane + 1], u1 = x1 - M[kHvS + lane + 2];
      const double t2 = x2 - M[2 * kHvS + lane + 1], u2 = x2 - M[2 * kHvS + lane + 2];
      const double p01 = u0 * t1, p12 = u1 * t2, p02 = u0 * t2;
      V[lane] = t0 * u0;
      V[kHvS + lane] = t1 * u1;
      V[2 * kHvS + lane] = t2 * u2;
      V[3 * kHvS + lane] = fma(p01, h.r.x, p01 * h.r.y);
      V[4 * kHvS + lane] = fma(p12, h.r.x, p12 * h.r.y);
      V[5 * kHvS + lane] = fma(p02, h.r.x, p02 * h.r.y);
    }
    asm volatile("" ::: "memory");
    stamp(c2);
  }
  // the last block's ordered sums
  if (lane >= 3 && lane < 9) {
    const double* v = V + (lane - 3) * kHvS;
    for (uint32_t i = 0; i < nb; i++) acc = acc + v[i];
  }
  stamp(c1);
  if constexpr (kStamp) {
    ph[0] = c0 + c2;
    ph[1] = c1;
    ph[2] = 0;
  }
  // lane j < 3: mean_j, m2_j (lane 3 + j) and the pair the quad layout gives
  // lane j ((0,1), (1,2), (0,2): lane 6 + j)
  const double s3 = __shfl_down(acc, 3, 64), s6 = __shfl_down(acc, 6, 64);
  const bool anyout = __any(out);
  if (lane < 3) {
    mean = m;
    m2 = s3;
    off = s6;
    bad = anyout;
  }
}

// What k_welford_q writes for the KL stage after an ND's moments (the LU
// chains, formerly their own kernel): neighbours, chain masks, the chain's
// in-place LU states and the final (post-KL) covariance.
struct WqChainArgs {
  const uint32_t* vox;     // [B][ndcap] linear voxel of each ND
  const uint32_t* dense;   // [B][vcap] dense id of each voxel (kInvalid: empty)
  int32_t* nb;             // [B][ndcap][6]
  uint32_t* nkeys;         // [B][ndcap] chain masks
  const double* cov_pre;   // [B][ndcap][9] the moments' covariances (k_welford_q's nd_cov)
  double* chain;           // [B][108][ndcap] step-major LU states
  uint32_t* chain_ps;      // [B][12][ndcap]
  double* cov_post;        // [B][ndcap][9]
  uint64_t vcap;
  // lazy run (KLArgs.mode kKLLazy): a cloud with num_nds <= lazy_k defers its
  // list (kl_list_deferrable), so its events are only flagged: it stores, per
  // ND, which LU states have a non-zero determinant (chain_ok) instead of the
  // states themselves (k_kl_chains recomputes them if the list is ever built).
  // 0: every cloud stores its states.
  uint64_t lazy_k;
  uint32_t* chain_ok;      // [B][ndcap]
  uint32_t* lu_done;       // [B][ceil(ndcap / 64)] NDs of each 64-ND group whose moments are stored (re-armed to 0)
};

__device__ inline void st_sc1_f64(double* p, double v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), __builtin_bit_cast(unsigned long long, v),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline double ld_sc1_f64(const double* p) {
  return __builtin_bit_cast(double, __hip_atomic_load(reinterpret_cast<const unsigned long long*>(p), __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_AGENT));
}

// The in-place LU chain of ND u (the GSL calls of
// kullback_leibler.c:57-63 per event, in chain_mask's order), one ND per
// lane, by the wave that completed u's 64-ND group: the covariances and masks
// other waves stored (sc1) are read with sc1 loads.  Each state is stored
// step-major ([t][q][ND], coalesced), the last as the post-KL covariance.  A
// cloud whose list is deferred (lazy run, num_nds <= lazy_k) keeps only
// which states have det != 0 and sgndet != 0 (chain_ok: all its event flags
// read); k_kl_chains stores its states if the list is ever built.
__device__ inline void wq_lu_chain(const WqChainArgs& CA, int b, uint32_t u, uint32_t nd, uint32_t ndcap, double (&S)[9],
                                   int nT) {
  const uint64_t ob = (uint64_t)b * ndcap;
  const bool flags_only = CA.lazy_k && nd <= CA.lazy_k;  // a deferred cloud
  double* ch = CA.chain + ob * 108 + u;
  uint32_t* ps = CA.chain_ps + ob * 12 + u;
  uint32_t okb = 0;
  for (int t = 0; t < nT; t++) {
    uint32_t perm;
    int sg;
    lu3(S, perm, sg);
    if (flags_only) {  // what kl_event's flag reads of the state (kullback_leibler.c:57-70)
      okb |= (lu3_det(S, sg) != 0 && lu3_sgndet(S, sg) != 0 ? 1u : 0u) << t;
      continue;
    }
#pragma unroll
    for (int q = 0; q < 9; q++) ch[(uint64_t)(9 * t + q) * ndcap] = S[q];
    ps[(uint64_t)t * ndcap] = perm | (sg < 0 ? 0x100u : 0u);
  }
  if (flags_only) CA.chain_ok[ob + u] = okb;
#pragma unroll
  for (int q = 0; q < 9; q++) CA.cov_post[9 * (ob + u) + q] = S[q];
}

__device__ inline void wq_lu_group(const WqChainArgs& CA, int b, uint32_t u, uint32_t nd, uint32_t ndcap) {
  if (u >= nd) return;
  const uint64_t ob = (uint64_t)b * ndcap;
  double S[9];
#pragma unroll
  for (int q = 0; q < 9; q++) S[q] = ld_sc1_f64(&CA.cov_pre[9 * (ob + u) + q]);
  const int nT = __popc(__hip_atomic_load(&CA.nkeys[ob + u], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  wq_lu_chain(CA, b, u, nd, ndcap, S, nT);
}

// ndnet_debug_lu_chain: the device LU chain (lu3 + the event flags, as
// wq_lu_group runs them) on n given matrices, every state recorded.
__global__ void __launch_bounds__(64) k_debug_lu_chain(const double* A, uint32_t n, int steps, double* states,
                                                        uint32_t* ps, uint32_t* flags) {
  const uint32_t m = blockIdx.x * 64 + threadIdx.x;
  if (m >= n) return;
  double S[9];
#pragma unroll
  for (int q = 0; q < 9; q++) S[q] = A[9 * (uint64_t)m + q];
  for (int t = 0; t < steps; t++) {
    uint32_t perm;
    int sg;
    lu3(S, perm, sg);
    const uint64_t r = (uint64_t)m * steps + t;
#pragma unroll
    for (int q = 0; q < 9; q++) states[9 * r + q] = S[q];
    ps[r] = perm | (sg < 0 ? 0x100u : 0u);
    flags[r] = lu3_det(S, sg) != 0 && lu3_sgndet(S, sg) != 0 ? 1u : 0u;
  }
}

// ---- light NDs, one per lane (wq_light64, round 5) ----
//
// The lane-quad fold (one ND per quad, lane j = axis j) runs ~18 wave
// instructions per sample for 16 NDs with only two independent dependency
// chains per lane, ~9 cycles each: 227 cycles per sample (profiles/
// r04_welford_ab.txt), and U's 16 x 1000 NDs filled every wave of the chip
// for ~25 us (r04_wq_items_U.txt) -- while the FP64 work itself is ~5 us of
// the chip.  Here a lane holds a whole ND (3 axes: three independent mean
// recurrences, and the m2 / off-diagonal chains beside them), so a wave folds
// 64 NDs, one 64-ND LU group, with ~33 FP64 instructions per sample and ILP
// enough to issue them back to back: U needs 256 waves instead of 1008, the
// persistent grid packs them four to a CU (items by workgroup), and the
// other 192 CUs are free for another stream's kernels from the start.  The
// group's LU chains (wq_lu_chain) run right after, from registers, in the
// same wave -- no covariance hand-off through L2 and no group counter --
// unless a heavy ND of the group is being folded by another wave; then the
// round-4 protocol (sc1 stores, lu_done counter, the completing wave runs
// wq_lu_group) applies.
//
// Per sample, in the reference's order (normal_distributions.c:75-103):
//   t_j = x_j - mean_j;  mean_j += t_j / n;  u_j = x_j - mean_j;
//   m2_j += t_j u_j;  off_jk += (u_j t_k) / n  (j < k: (0,1), (1,2), (0,2))
// with t / n = fma(t, rc, t rl), (rc, rl) the per-count pair of Plan::rtab
// (always the IEEE quotient: test_rtab_division_is_ieee), staged in LDS.  A
// lane past its count folds x = mean (t = u = +0: an exact no-op, the sums
// never being -0).  A lane whose coordinates leave the fast range (non-finite
// floats; doubles outside [2^-300, 2^300]) refolds its ND with IEEE divisions
// and the reference's per-step NaN -> 0 of the off-diagonal sums.
// Both light forms are built; a plan picks one by its CU share (Plan::wq_l64,
// ndnet_ndt_set_welford_form): the lane quads for a plan that has the whole
// chip (isolated U 30.5 us against light64's 37: profiles/r05final_*), light64
// where the pipeline runs the forward beside it (a quarter of the CUs).
constexpr uint32_t wq_light_nds(bool l64) { return l64 ? 64u : 16u; }  // NDs per light item (one wave)
constexpr int kL64B = 8;                                      // samples per register block
static_assert(4 * kL64B <= 32, "wq_rt_entries' margin covers a light64 group's last round (ring <= 4)");
#ifndef NDNET_WQ_L64_COALESCE
#define NDNET_WQ_L64_COALESCE 1
#endif
constexpr size_t wq_rt_bytes(bool l64) { return l64 ? sizeof(double2) : sizeof(double); }  // LDS table entry
constexpr uint32_t wq_hist_nds(bool l64) { return l64 ? kWqThreads : kWqNDs; }          // NDs of a workgroup at once

template <typename T>
struct L64Blk {
  T v[kL64B][3];
};

template <typename T>
__device__ __attribute__((always_inline)) inline void l64_load(L64Blk<T>& r, const T* __restrict__ src, uint32_t q0,
                                                               uint32_t last) {
#pragma unroll
  for (int u = 0; u < kL64B; u++) {
    const uint32_t q = q0 + (uint32_t)u < last ? q0 + (uint32_t)u : last;
    const T* p = src + 3u * q;
    r.v[u][0] = p[0];
    r.v[u][1] = p[1];
    r.v[u][2] = p[2];
  }
}

// Float records, coalesced: a lane owning a whole ND reading its own records
// sends the wave's 64 loads to 64 cache lines ~1.2 KB apart, and with four
// waves per CU each holding a ring of 3 blocks the lines are evicted from the
// 32 KB L1 before their next sample is read -- r05f: 490 cycles per sample
// against ~132 of FP64 work (profiles/r05_wq_items_U.txt).  Here load k of a
// block reads sample q0 + (lane & 7) of ND 8k + (lane >> 3): eight NDs' 96-byte
// runs per instruction.  kL64Pitch dwords per ND row: conflict-free reads.
constexpr int kL64Pitch = 3 * kL64B + 1;
static_assert(64 * kL64Pitch * sizeof(float) <= 16 * kWqStageQ * sizeof(float), "a block fits a wave's stage rows");

// the 8 NDs a lane loads for, as record offsets from the cloud's first record and last samples
struct L64Src {
  uint32_t off[8], last[8];
};

__device__ __attribute__((always_inline)) inline void l64_sload(L64Blk<float>& r, const float* __restrict__ cloud,
                                                                const L64Src& s, uint32_t q0, uint32_t lane) {
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const uint32_t q0u = q0 + (lane & 7u);
    const uint32_t q = q0u < s.last[k] ? q0u : s.last[k];
    const float* p = cloud + 3u * (s.off[k] + q);
    r.v[k][0] = p[0];
    r.v[k][1] = p[1];
    r.v[k][2] = p[2];
  }
}

// the coalesced block (load k: ND 8k + lane / 8, sample lane % 8) -> the lane's own ND's 8 samples
__device__ __attribute__((always_inline)) inline void l64_transpose(const L64Blk<float>& r, L64Blk<float>& x,
                                                                    float* __restrict__ stg, uint32_t lane) {
#pragma unroll
  for (int k = 0; k < 8; k++) {
    float* w = stg + (8u * (uint32_t)k + (lane >> 3)) * kL64Pitch + 3u * (lane & 7u);
    w[0] = r.v[k][0];
    w[1] = r.v[k][1];
    w[2] = r.v[k][2];
  }
  asm volatile("" ::: "memory");  // one wave's LDS operations complete in order
  const float* rd = stg + lane * kL64Pitch;
#pragma unroll
  for (int u = 0; u < kL64B; u++) {
    x.v[u][0] = rd[3 * u];
    x.v[u][1] = rd[3 * u + 1];
    x.v[u][2] = rd[3 * u + 2];
  }
  asm volatile("" ::: "memory");
}

// one block of kL64B samples of the lane's ND (kMask: some lane ends inside it)
template <typename T, bool kMask>
__device__ __attribute__((always_inline)) inline void l64_fold(const L64Blk<T>& r, const double2 (&rr)[kL64B],
                                                               uint32_t q0, uint32_t cnt, double (&m)[3],
                                                               double (&m2)[3], double (&of)[3], bool& bad) {
#pragma unroll
  for (int u = 0; u < kL64B; u++) {
    const double rc = rr[u].x, rl = rr[u].y;
    double x[3];
#pragma unroll
    for (int a = 0; a < 3; a++) {
      if constexpr (!std::is_same<T, float>::value) bad |= (q0 + (uint32_t)u < cnt) && !wq_in_range(r.v[u][a]);
      x[a] = (double)r.v[u][a];
    }
    if constexpr (kMask) {
      const unsigned long long lanes = __ballot(q0 + (uint32_t)u < cnt);
#pragma unroll
      for (int a = 0; a < 3; a++) x[a] = sel_d(lanes, x[a], m[a]);
    }
    double t[3], uu[3];
#pragma unroll
    for (int a = 0; a < 3; a++) {
      t[a] = x[a] - m[a];
      m[a] = m[a] + fma(t[a], rc, t[a] * rl);
      uu[a] = x[a] - m[a];
      m2[a] = m2[a] + t[a] * uu[a];
    }
    const double p01 = uu[0] * t[1], p12 = uu[1] * t[2], p02 = uu[0] * t[2];
    of[0] = of[0] + fma(p01, rc, p01 * rl);
    of[1] = of[1] + fma(p12, rc, p12 * rl);
    of[2] = of[2] + fma(p02, rc, p02 * rl);
  }
}

template <typename T>
__device__ __attribute__((always_inline)) inline void wq_light64(const CloudCtl* __restrict__ ctl, int b, uint32_t wd0,
                                                     const T* __restrict__ nd_pts, const uint16_t* __restrict__ nd_lbl,
                                                     const uint32_t* __restrict__ nd_n,
                                                     const uint32_t* __restrict__ nd_base, double* nd_mean,
                                                     double* nd_cov, uint16_t* nd_cls, uint32_t* hist_all, int ncls,
                                                     uint64_t n, uint32_t ndcap, const double2* __restrict__ lrt2,
                                                     uint32_t rtn, const double2* __restrict__ rtab,
                                                     uint32_t* __restrict__ wq_hist, bool hist_lds,
                                                     const WqChainArgs& CA, uint32_t lane, float* __restrict__ stg,
                                                     unsigned long long& t_loop, unsigned long long& t_mom,
                                                     unsigned long long& t_lbl, uint32_t& mx_out) {
  const uint32_t nd = ctl[b].num_nds, heavy_t = ctl[b].heavy_t;
  const uint32_t d = wd0 + lane;
  const bool inr = d < nd;
  const uint64_t o = (uint64_t)b * ndcap + (inr ? d : wd0);
  const uint32_t beg = nd_base[o], c0 = nd_n[o];
  const bool live = inr && c0 < heavy_t;  // heavy NDs of the group are folded by their own items
  const uint32_t cnt = live ? c0 : 0u;
  const uint32_t last = cnt ? cnt - 1u : 0u;
  const uint32_t mx = wave_max_u32(cnt);
  const uint32_t full = wave_min_u32(live ? cnt : 0xffffffffu);  // blocks every live lane fills: no selects
  const T* src = nd_pts + ((uint64_t)b * n + beg) * 3;
  // the ND's neighbours (voxel.c:116-175: X+, X-, Y+, Y-, Z+, Z-), loaded behind the first point loads
  int32_t nw[6];
  uint32_t ncn[6];
  {
    const uint32_t lx = ctl[b].len[0], ly = ctl[b].len[1], lz = ctl[b].len[2];
    const uint32_t lin = CA.vox[o];
    const uint32_t zc = lin / (lx * ly), yc = (lin % (lx * ly)) / lx, xc = lin % lx;
    const uint32_t* dense = CA.dense + (uint64_t)b * CA.vcap;
    uint32_t dn[6];
    bool in[6];
#pragma unroll
    for (int dd = 0; dd < 6; dd++) {
      const uint32_t xx = xc + (dd == 0 ? 1u : dd == 1 ? ~0u : 0u);
      const uint32_t yy = yc + (dd == 2 ? 1u : dd == 3 ? ~0u : 0u);
      const uint32_t zz = zc + (dd == 4 ? 1u : dd == 5 ? ~0u : 0u);
      in[dd] = xx < lx && yy < ly && zz < lz;
      dn[dd] = dense[in[dd] ? zz * lx * ly + yy * lx + xx : lin];
    }
#pragma unroll
    for (int dd = 0; dd < 6; dd++) {
      nw[dd] = (in[dd] && dn[dd] != kInvalid) ? (int32_t)dn[dd] : -1;
      ncn[dd] = nd_n[(uint64_t)b * ndcap + (nw[dd] >= 0 ? (uint32_t)nw[dd] : (uint32_t)(o - (uint64_t)b * ndcap))];
    }
  }
  double m[3] = {0.0, 0.0, 0.0}, m2[3] = {0.0, 0.0, 0.0}, of[3] = {0.0, 0.0, 0.0};
  bool bad = false;
  // (rc, rl) of counts q0 + 1 .. q0 + kL64B: LDS broadcast reads, the global
  // table past the LDS one (a threshold raised after the heavy list was built)
  auto ldr = [&](double2 (&rr)[kL64B], uint32_t q0) __attribute__((always_inline)) {
    if (q0 + kL64B < rtn) {  // wave-uniform
#pragma unroll
      for (int u = 0; u < kL64B; u++) rr[u] = lrt2[q0 + (uint32_t)u + 1u];
    } else {  // counts past the table (clamped to the plan's n: a masked step only needs a finite pair)
#pragma unroll
      for (int u = 0; u < kL64B; u++) {
        const uint64_t c = (uint64_t)q0 + (uint32_t)u + 1u;
        rr[u] = rtab[c <= n ? c : n];
      }
    }
  };
  // a ring of register blocks: kR - 1 blocks in flight while one is folded
  constexpr bool kCo = std::is_same<T, float>::value && NDNET_WQ_L64_COALESCE;  // coalesced loads + LDS transpose
#ifndef NDNET_WQ_L64_RING
#define NDNET_WQ_L64_RING 3
#endif
  constexpr int kR = std::is_same<T, float>::value ? NDNET_WQ_L64_RING : 2;
  L64Blk<T> rb[kR];
  L64Src ss;
  const T* const cloud = nd_pts + (uint64_t)b * n * 3;
  if constexpr (kCo) {
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const int sl = 8 * k + (int)(lane >> 3);
      ss.off[k] = (uint32_t)__shfl((int)beg, sl);
      ss.last[k] = (uint32_t)__shfl((int)last, sl);
    }
  }
  auto blk_load = [&](L64Blk<T>& r, uint32_t q0) __attribute__((always_inline)) {
    if constexpr (kCo) l64_sload(r, cloud, ss, q0, lane);
    else l64_load(r, src, q0, last);
  };
#pragma unroll
  for (int i = 0; i < kR; i++) blk_load(rb[i], (uint32_t)(i * kL64B));
  bool slow = false;  // the exact refold below for every live lane
  t_loop = __builtin_amdgcn_s_memtime();  // timing level 2: the prologue is done
  if constexpr (kCo) {
    // The loop has no load under a branch and takes (rc, rl) from the LDS
    // table only, so the compiler's waits stay counted: block i waits for its
    // own loads, issued kR blocks earlier, with the later ones in flight.  (A
    // conditional refill, or the global-table fallback's loads, left it one
    // vmcnt(0) per block: every block paid a memory latency, r05g ~440 cycles
    // per sample.)  A group past the table (a threshold raised between a
    // front call and this one) takes the exact path.
    // whole rounds of kR blocks: a block past every lane's count folds x = mean
    // (exact no-ops), so the round has no branch around its loads and waits
    constexpr uint32_t kRound = (uint32_t)(kR * kL64B);
    const uint32_t qend = (mx + kRound - 1u) / kRound * kRound;
    if (qend < rtn) {
      for (uint32_t q0 = 0; q0 < qend; q0 += kRound) {
#pragma unroll
        for (int i = 0; i < kR; i++) {
          const uint32_t qb = q0 + (uint32_t)(i * kL64B);
          double2 cr[kL64B];
#pragma unroll
          for (int u = 0; u < kL64B; u++) cr[u] = lrt2[qb + (uint32_t)u + 1u];
          L64Blk<T> xb;
          l64_transpose(rb[i], xb, stg, lane);
          blk_load(rb[i], qb + kRound);
          if (qb + kL64B <= full) l64_fold<T, false>(xb, cr, qb, cnt, m, m2, of, bad);
          else l64_fold<T, true>(xb, cr, qb, cnt, m, m2, of, bad);
        }
      }
    } else {
      slow = true;
    }
  }
  double2 rr[kL64B];
  if constexpr (!kCo) ldr(rr, 0);
  for (uint32_t q0 = 0; !kCo && q0 < mx; q0 += kR * kL64B) {  // every branch below is wave-uniform
#pragma unroll
    for (int i = 0; i < kR; i++) {
      const uint32_t qb = q0 + (uint32_t)(i * kL64B);
      if (qb >= mx) break;
      double2 cr[kL64B];
#pragma unroll
      for (int u = 0; u < kL64B; u++) cr[u] = rr[u];
      if (qb + kL64B < mx) ldr(rr, qb + kL64B);
      if (qb + kL64B <= full) l64_fold<T, false>(rb[i], cr, qb, cnt, m, m2, of, bad);
      else l64_fold<T, true>(rb[i], cr, qb, cnt, m, m2, of, bad);
      if (qb + kR * kL64B < mx) blk_load(rb[i], qb + kR * kL64B);
    }
  }
  t_mom = __builtin_amdgcn_s_memtime();  // timing level 2: the moments are done
  mx_out = mx;
  // float input: a non-finite coordinate leaves a non-finite mean
  if constexpr (std::is_same<T, float>::value)
    bad = live && !(fabs(m[0]) <= 0x1.fffffffffffffp+1023 && fabs(m[1]) <= 0x1.fffffffffffffp+1023 &&
                    fabs(m[2]) <= 0x1.fffffffffffffp+1023);
  bad = (bad || slow) && live;
  if (__any(bad) && bad) {  // the reference's exact steps (IEEE division, NaN -> 0 per off-diagonal step)
#pragma unroll
    for (int a = 0; a < 3; a++) m[a] = m2[a] = of[a] = 0.0;
    for (uint32_t q = 0; q < cnt; q++) {
      const double cn = (double)(q + 1u);
      double t[3], uu[3];
#pragma unroll
      for (int a = 0; a < 3; a++) {
        const double x = (double)src[3u * q + a];
        t[a] = x - m[a];
        m[a] = m[a] + t[a] / cn;
        uu[a] = x - m[a];
        m2[a] = m2[a] + t[a] * uu[a];
      }
      const double c01 = of[0] + (uu[0] * t[1]) / cn, c12 = of[1] + (uu[1] * t[2]) / cn,
                   c02 = of[2] + (uu[0] * t[2]) / cn;
      of[0] = c01 != c01 ? 0.0 : c01;
      of[1] = c12 != c12 ? 0.0 : c12;
      of[2] = c02 != c02 ? 0.0 : c02;
    }
  }
  double S[9];
  {
    const double cn = (double)cnt;
    double vd[3];
#pragma unroll
    for (int a = 0; a < 3; a++) {
      const double v = m2[a] / cn;
      vd[a] = v != v ? 0.0 : v;
    }
    S[0] = vd[0];
    S[4] = vd[1];
    S[8] = vd[2];
    S[1] = S[3] = of[0];
    S[5] = S[7] = of[1];
    S[2] = S[6] = of[2];
  }
  // the group's LU chains need every ND of the group: a heavy ND among them is
  // folded by another wave, which then meets this one at the group counter
  const bool grp_heavy = __any(inr && c0 >= heavy_t);
  uint32_t el = 0;
#pragma unroll
  for (int dd = 0; dd < 6; dd++)
    if (nw[dd] >= 0 && cnt > 1 && ncn[dd] > 1) el |= 1u << dd;
  const uint32_t mask = chain_mask(el);
  if (live) {
#pragma unroll
    for (int a = 0; a < 3; a++) nd_mean[3 * o + a] = m[a];
#pragma unroll
    for (int q = 0; q < 9; q++) st_sc1_f64(&nd_cov[9 * o + q], S[q]);
#pragma unroll
    for (int dd = 0; dd < 6; dd++) CA.nb[6 * o + dd] = nw[dd];
    __hip_atomic_store(&CA.nkeys[o], mask, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // labelled runs: the ND's class histogram (first index of the max, normal_distributions.c:107-121)
  const unsigned long long t_l0 = __builtin_amdgcn_s_memtime();
  if (nd_lbl) {
    const uint32_t nbins = (uint32_t)ncls + 1u;
    const uint16_t* l = nd_lbl + (uint64_t)b * n + beg;
    uint32_t* hist = hist_lds ? wq_hist + (threadIdx.x & (kWqThreads - 1)) * nbins : hist_all + o * nbins;
    if (live)
      for (uint32_t k = 0; k < nbins; k++) hist[k] = 0;
    if (hist_lds) {
      // Coalesced, as the records: load k of a 32-sample block reads samples
      // q0 .. q0 + 31 of NDs 2k and 2k + 1 (lanes 0..31, 32..63: one or two
      // 64-byte runs per instruction), staged in the wave's rows (pitch
      // kLblPitch dwords: conflict-free reads), then each lane counts its own
      // ND's 32 with return-less LDS adds.  (Per-lane loads sent each
      // instruction to 64 lines: ~225 cycles per sample, r05m.)
      constexpr uint32_t kLblPitch = 17;  // dwords per ND row (32 labels + 1)
      static_assert(64 * kLblPitch * 4 <= 16 * kWqStageQ * sizeof(float), "label block fits the stage rows");
      const uint16_t* lc = nd_lbl + (uint64_t)b * n;
      uint16_t* st16 = reinterpret_cast<uint16_t*>(stg);
      const uint32_t* st32 = reinterpret_cast<const uint32_t*>(stg) + lane * kLblPitch;
      const uint32_t lastl = cnt ? cnt - 1u : 0u;
      const uint32_t half = lane >> 5, ql = lane & 31u;
      // two 32-sample blocks in registers: block j + 1's loads are in flight
      // while block j is staged and counted (one exposed latency per item,
      // not per block: 34k cycles per light item before, r05o)
      auto ld = [&](uint16_t (&v)[32], uint32_t q0) __attribute__((always_inline)) {
#pragma unroll
        for (int k = 0; k < 32; k++) {
          const uint32_t b0 = __builtin_amdgcn_readlane(beg, 2 * k), b1 = __builtin_amdgcn_readlane(beg, 2 * k + 1);
          const uint32_t e0 = __builtin_amdgcn_readlane(lastl, 2 * k), e1 = __builtin_amdgcn_readlane(lastl, 2 * k + 1);
          const uint32_t bb = half ? b1 : b0, ee = half ? e1 : e0;
          const uint32_t q = q0 + ql < ee ? q0 + ql : ee;
          v[k] = lc[bb + q];
        }
      };
      auto count = [&](const uint16_t (&v)[32], uint32_t q0) __attribute__((always_inline)) {
        asm volatile("" ::: "memory");  // the previous block's reads are issued (one wave's LDS ops run in order)
#pragma unroll
        for (int k = 0; k < 32; k++) st16[2u * ((2u * (uint32_t)k + half) * kLblPitch) + ql] = v[k];
        asm volatile("" ::: "memory");
        uint32_t w[16];
#pragma unroll
        for (int i = 0; i < 16; i++) w[i] = st32[i];
        asm volatile("" ::: "memory");
        if (live) {
#pragma unroll
          for (int j = 0; j < 32; j++) {
            const uint32_t lb = (w[j >> 1] >> (16 * (j & 1))) & 0xffffu;
            if (q0 + (uint32_t)j < cnt && lb < nbins) atomicAdd(&hist[lb], 1u);  // return-less LDS adds
          }
        }
      };
      uint16_t va[32], vb[32];
      ld(va, 0);
      for (uint32_t q0 = 0; q0 < mx; q0 += 64) {  // wave-uniform; loads past mx are clamped (unused)
        ld(vb, q0 + 32);
        count(va, q0);
        ld(va, q0 + 64);
        if (q0 + 32 < mx) count(vb, q0 + 32);
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
    } else if (live) {
      for (uint32_t s = 0; s < cnt; s++)
        if (l[s] < nbins) hist[l[s]]++;
    }
    if (live) {
      uint32_t best = 0;
      uint16_t cls = 0;
      for (uint32_t k = 0; k < nbins; k++) {
        const uint32_t h = hist[k];
        if (h > best) {
          best = h;
          cls = (uint16_t)k;
        }
      }
      nd_cls[o] = cls;
    }
  } else if (live) {
    nd_cls[o] = 0;
  }
  t_lbl = __builtin_amdgcn_s_memtime() - t_l0;  // timing level 2: the class histogram's cycles
  if (!grp_heavy) {
    if (live) wq_lu_chain(CA, b, d, nd, ndcap, S, __popc(mask));
    return;
  }
  const uint32_t nlive = (uint32_t)__popcll(__ballot(live));
  if (nlive) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's sc1 stores are done
    const uint32_t g = wd0 / 64u, gcap = (ndcap + 63u) / 64u;
    const uint32_t total = nd - 64u * g < 64u ? nd - 64u * g : 64u;
    uint32_t* gc = CA.lu_done + (uint64_t)b * gcap + g;
    uint32_t old = 0;
    if (lane == 0) old = __hip_atomic_fetch_add(gc, nlive, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    old = __builtin_amdgcn_readfirstlane(old);
    if (old + nlive == total) {
      if (lane == 0) __hip_atomic_store(gc, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-armed
      wq_lu_group(CA, b, 64u * g + lane, nd, ndcap);
    }
  }
}

template <typename T, bool L64>
__global__ void __launch_bounds__(kWqThreads) NDNET_WQ_ATTR k_welford_q(const CloudCtl* ctl, int B, const T* __restrict__ nd_pts,
                                                          const uint16_t* __restrict__ nd_lbl,
                                                          const uint32_t* __restrict__ nd_n,
                                                          const uint32_t* __restrict__ nd_base, double* nd_mean,
                                                          double* nd_cov, uint16_t* nd_cls, uint32_t* hist_all,
                                                          int ncls, uint64_t n, uint32_t ndcap, uint32_t* wq_ctr,
                                                          const uint32_t* __restrict__ heavy, uint32_t heavy_t,
                                                          const double2* __restrict__ rtab,
                                                          unsigned long long* __restrict__ wq_marks, WqChainArgs CA) {
  extern __shared__ __attribute__((aligned(16))) unsigned char wq_smem[];
  // the quads' record transposes; a heavy item's wave uses its 16 rows (6400 B) as its wq_heavy stage
  __shared__ __attribute__((aligned(16))) float wq_stage[kWqNDs][kWqStageQ];
  __shared__ double2 wq_hr[kWqThreads / 64][64];  // a heavy wave's block row of (rc, rl)
  static_assert(kHvLds * sizeof(double) <= 16 * kWqStageQ * sizeof(float), "heavy stage fits a wave's rows");
  static_assert((16 * kWqStageQ * sizeof(float)) % 16 == 0, "16-byte aligned heavy stage");
  const uint32_t rtn = wq_rt_entries(heavy_t);
  double* lrt = (double*)wq_smem;                                // quads: [rtn] refined reciprocals of 1..rtn
  double2* lrt2 = (double2*)wq_smem;                             // light64: [rtn] (rc, rl) of counts 0..rtn - 1
  const uint32_t bw = (uint32_t)((B + 1 + 3) & ~3);
  constexpr uint32_t kWqLightNDs = wq_light_nds(L64);
  constexpr uint32_t kWqHistNDs = wq_hist_nds(L64);
  uint32_t* pre = (uint32_t*)(wq_smem + rtn * wq_rt_bytes(L64)); // [B + 1] first light item of each cloud
  uint32_t* hpre = pre + bw;                                      // [B + 1] first heavy item of each cloud
  uint32_t* wq_hist = hpre + bw;                                  // labelled runs: [kWqHistNDs][ncls + 1]
  if constexpr (L64) {
    // every entry finite: a masked step past a lane's count reads one (x = mean
    // makes t = +0, and 0 * rl must not be 0 * inf); rtab holds counts 0..n
    for (uint32_t i = threadIdx.x; i < rtn; i += kWqThreads) lrt2[i] = rtab[i <= n ? i : n];
  } else {
    for (uint32_t i = threadIdx.x; i < rtn; i += kWqThreads) lrt[i] = recip_refined((double)(i + 1));
  }
  // items: first the heavy NDs (>= kWqHeavy samples, listed by k_front /
  // k_bin_offsets), one per wave, so the longest work starts at once; then
  // (cloud, group of 16 NDs), in cloud order, whose heavy NDs are skipped.
  // One item per wave of a persistent grid (one workgroup per CU, one wave
  // per SIMD), so no SIMD holds two ND groups while another idles.
  for (int i = threadIdx.x; i < B; i += kWqThreads) {
    const bool acc = ctl[i].state == kAccepted;
    pre[i + 1] = acc ? (ctl[i].num_nds + kWqLightNDs - 1u) / kWqLightNDs : 0u;
    hpre[i + 1] = acc ? ctl[i].heavy_n : 0u;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    pre[0] = hpre[0] = 0;
    for (int i = 0; i < B; i++) {
      pre[i + 1] += pre[i];
      hpre[i + 1] += hpre[i];
    }
  }
  __syncthreads();
  const uint32_t H = hpre[B];
  const uint32_t total = H + pre[B];
  const uint32_t lane = threadIdx.x & 63, j = lane & 3;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // first round static (one item per wave), then a shared counter: a wave
  // that finishes a light ND group takes the next one, so a heavy group is
  // never queued behind another.  A wave first reads the counter and only
  // increments it while items remain (one contended word takes ~11 ns per
  // atomic: a thousand waves each adding would cost ~10 us).  k_kl_rank_chunks,
  // the next kernel on the stream, re-arms it.
  // The dynamic items are sharded over one counter per XCD (workgroups are
  // dealt round-robin to the 8 XCDs, so blockIdx % 8 is the XCD): XCD x takes
  // items nwaves + 8 c + x.  One shared word saturates at ~88 dequeues / us
  // (MI355X_MICROARCH.md, dequeue), and when every wave finishes a uniform
  // first round together (C5's 2000-ND level: 2400 items on 1024 waves) the
  // ~1400 dequeues on it took ~15 us.
  const uint32_t nwaves = gridDim.x * (kWqThreads / 64);
  const uint32_t nx = gridDim.x < 8u ? gridDim.x : 8u, xs = blockIdx.x % nx;
  uint32_t* const ctr = wq_ctr + 16u * xs;  // one 64-byte line per shard
  auto next_item = [&]() -> uint32_t {
    uint32_t v = total;
    if (lane == 0) {
      const uint32_t seen = __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (nwaves + nx * seen + xs < total) {
        const uint32_t it = nwaves + nx * __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + xs;
        v = it < total ? it : total;
      }
    }
    return __builtin_amdgcn_readfirstlane(v);
  };
  for (uint32_t item = blockIdx.x * (kWqThreads / 64) + wave; item < total; item = next_item()) {
#ifdef NDNET_WQ_EXP_LIGHTONLY  // register probe only (wrong results): the light path alone
  const bool hv = false;
#else
  const bool hv = item < H;  // a heavy ND (wave-uniform)
#endif
#ifdef NDNET_WQ_EXP_HEAVYONLY  // timing experiment only (wrong results): light items skipped
  if (!hv) continue;
#endif
  unsigned long long mk_rt = 0, mk_t0 = 0, mk_t1 = 0;
  if (wq_marks) {
    mk_rt = __builtin_amdgcn_s_memrealtime();
    mk_t0 = __builtin_amdgcn_s_memtime();
  }
  const uint32_t li = hv ? item : item - H;
  const uint32_t* const ip = hv ? hpre : pre;
  int lo = 0, hi = B - 1;  // the cloud whose items hold `item`
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (ip[mid] <= li) lo = mid;
    else hi = mid - 1;
  }
  const int b = lo;
  if (L64 && !hv) {  // 64 NDs, one per lane
    unsigned long long t_mom = 0, t_loop = 0, t_lbl = 0;
    uint32_t lmx = 0;
    wq_light64<T>(ctl, b, (li - pre[b]) * kWqLightNDs, nd_pts, nd_lbl, nd_n, nd_base, nd_mean, nd_cov, nd_cls,
                  hist_all, ncls, n, ndcap, lrt2, rtn, rtab, wq_hist,
                  (size_t)kWqHistNDs * ((uint32_t)ncls + 1u) * sizeof(uint32_t) <= (size_t)kWqHistMax, CA, lane,
                  &wq_stage[(threadIdx.x >> 6) * 16][0], t_loop, t_mom, t_lbl, lmx);
    if (wq_marks && lane == 0) {
      unsigned long long* w = wq_marks + (uint64_t)item * kWqMarkW;
      w[0] = mk_rt;
      w[1] = mk_t0;
      w[2] = t_mom;
      w[3] = __builtin_amdgcn_s_memtime();
      const uint32_t hwid = __builtin_amdgcn_s_getreg((31 << 11) | 4);
      const uint32_t xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20) & 15u;
      w[4] = ((unsigned long long)xcc << 56) | ((unsigned long long)(lmx & 0xFFFFFFu) << 32) | hwid;
      w[5] = t_loop - mk_t0;  // light items: the prologue's cycles
      w[6] = t_lbl;           // and the class histogram's
      w[7] = 0;
    }
    continue;
  }
  const uint32_t nd = ctl[b].num_nds;
  // heavy: quad 0 holds the ND, the other quads idle; light: 16 NDs
  const uint32_t wd0 = hv ? heavy[(uint64_t)b * ndcap + (li - hpre[b])] : (li - pre[b]) * 16u;
  const uint32_t d = hv ? wd0 : wd0 + (lane >> 2);
  const uint64_t o = (uint64_t)b * ndcap + (d < nd ? d : wd0);
  const uint32_t beg = nd_base[o];
  const uint32_t c0 = nd_n[o];
  // a light group's heavy NDs are done by their own items
  const bool live = hv ? lane < 4 : (d < nd && c0 < ctl[b].heavy_t);  // the heavy list's own threshold
  const uint32_t cnt = live ? c0 : 0u;
  const uint32_t last = cnt ? cnt - 1u : 0u;
  const uint32_t jj = j < 3 ? j : 0u;
  const T* src = nd_pts + ((uint64_t)b * n + beg) * 3 + jj;
  constexpr bool kVec = NDNET_WQ_VLOAD && std::is_same<T, float>::value;
#ifndef NDNET_WQ_VU
#define NDNET_WQ_VU 1
#endif
  constexpr int kU = kVec ? NDNET_WQ_VU * kWqU : kWqU;  // samples per ring block
  float* const stg = kVec ? &wq_stage[threadIdx.x >> 2][0] : nullptr;
  const uint32_t mx = wave_max_u32(cnt);
  // the ND's neighbours (voxel.c:116-175, directions X+, X-, Y+, Y-, Z+, Z-):
  // lane j of the quad takes directions j and j + 4; their dense ids and
  // counts are loaded before the fold, behind the first point loads
  int32_t nw[2];
  uint32_t ncn[2];
  {
    const uint32_t lx = ctl[b].len[0], ly = ctl[b].len[1], lz = ctl[b].len[2];
    const uint32_t lin = CA.vox[o];
    const uint32_t zc = lin / (lx * ly), yc = (lin % (lx * ly)) / lx, xc = lin % lx;
    const uint32_t* dense = CA.dense + (uint64_t)b * CA.vcap;
    uint32_t dn[2];
    bool in[2];
#pragma unroll
    for (int k = 0; k < 2; k++) {
      const uint32_t dd = j + 4u * (uint32_t)k;
      const uint32_t xx = xc + (dd == 0 ? 1u : dd == 1 ? ~0u : 0u);
      const uint32_t yy = yc + (dd == 2 ? 1u : dd == 3 ? ~0u : 0u);
      const uint32_t zz = zc + (dd == 4 ? 1u : dd == 5 ? ~0u : 0u);
      in[k] = dd < 6u && xx < lx && yy < ly && zz < lz;
      dn[k] = dense[in[k] ? zz * lx * ly + yy * lx + xx : lin];
    }
#pragma unroll
    for (int k = 0; k < 2; k++) {
      nw[k] = (in[k] && dn[k] != kInvalid) ? (int32_t)dn[k] : -1;
      ncn[k] = nd_n[(uint64_t)b * ndcap + (nw[k] >= 0 ? (uint32_t)nw[k] : (uint32_t)(o - (uint64_t)b * ndcap))];
    }
  }

  double mean = 0.0, m2 = 0.0, off = 0.0;
  bool bad = false;
  // points: a ring of kWqNB register blocks of kU samples, kWqNB - 1 blocks
  // in flight ahead of the one being folded (memory latency ~2 us under load
  // against ~0.5 us per block of compute)
  using Blk = WqBlk<T, kVec, kU>;
  Blk r0, r1, r2, r3;
  auto load = [&](Blk& r, uint32_t q0) __attribute__((always_inline)) {
    if constexpr (kVec) {
      const float* rec = nd_pts + ((uint64_t)b * n + beg) * 3;
#pragma unroll
      for (int i = 0; i < kU / 4; i++) {
        const uint32_t q = q0 + (uint32_t)(kU / 4) * j + (uint32_t)i;
#ifdef NDNET_WQ_NOLOAD  // timing experiment only: no point loads (wrong results)
        r.v[i] = make_float3(1.0f + 0.001f * (float)(q & 7), 2.0f, 3.0f);
#else
        const float* pq = rec + 3u * (q < last ? q : last);
        r.v[i] = make_float3(pq[0], pq[1], pq[2]);
#endif
      }
    } else {
#pragma unroll
      for (int u = 0; u < kU; u++) {
        const uint32_t q = q0 + (uint32_t)u;
#ifdef NDNET_WQ_NOLOAD  // timing experiment only: no point loads (wrong results)
        r.v[u] = (T)(1.0f + 0.001f * (float)(q & 7));
#elif defined(NDNET_WQ_HOTLOAD)  // timing experiment only: loads of a few cached lines (wrong results)
        r.v[u] = nd_pts[jj + 3u * (q & 7u)];
#else
        r.v[u] = src[3u * (q < last ? q : last)];
#endif
      }
    }
  };
  // the block's reciprocals: broadcast LDS reads, computed past the table
  auto recips = [&](double (&cr)[kU], uint32_t q0) __attribute__((always_inline)) {
    if (q0 + kU <= rtn) {  // wave-uniform
#pragma unroll
      for (int u = 0; u < kU; u++) cr[u] = lrt[q0 + u];
    } else {
#pragma unroll
      for (int u = 0; u < kU; u++) cr[u] = recip_refined((double)(q0 + u + 1));
    }
  };
  // One block of samples; kExact: IEEE divisions and the NaN -> 0 step.
  // Branch-free over the block (a lane past its count keeps its state by
  // selects).  Two dependent chains per sample: the head of sample q (the
  // mean: t = x - mean, mean += t / n, u = x - mean; 6 FP64 ops of ~10 cycles
  // latency each) and the tail of sample q - 1 (m2 += t u, the off-diagonal
  // product u_a t_b through two DPP moves and its division, 6 deep).  The
  // fast fold issues them interleaved in pairs, with a scheduling barrier
  // after each pair, so every head op finds its operand ready: the in-order
  // wave issues ~18 instructions per sample back to back instead of waiting
  // out each chain link.
  auto fold = [&](const Blk& rb, uint32_t q0, bool act, auto exact_tag,
                  auto masked_tag) __attribute__((always_inline)) {
    constexpr bool kExact = decltype(exact_tag)::value;
    constexpr bool kMasked = decltype(masked_tag)::value;  // false: every live quad has >= q0 + kU samples
    T r[kU];
    if constexpr (kVec) {
      // the quad's records to its LDS stage (word 3 s + c = coordinate c of
      // sample s), then lane j reads coordinate jj of each sample; one wave's
      // LDS operations complete in order, so the compiler barriers suffice
#pragma unroll
      for (int i = 0; i < kU / 4; i += 4) {
        float4* d = reinterpret_cast<float4*>(stg + 3 * (kU / 4) * j + 3 * i);
        const float3 a0 = rb.v[i], a1 = rb.v[i + 1], a2 = rb.v[i + 2], a3 = rb.v[i + 3];
        d[0] = make_float4(a0.x, a0.y, a0.z, a1.x);
        d[1] = make_float4(a1.y, a1.z, a2.x, a2.y);
        d[2] = make_float4(a2.z, a3.x, a3.y, a3.z);
      }
      asm volatile("" ::: "memory");
#pragma unroll
      for (int u = 0; u < kU; u++) r[u] = stg[3 * u + jj];
      asm volatile("" ::: "memory");
    } else {
#pragma unroll
      for (int u = 0; u < kU; u++) r[u] = rb.v[u];
    }
    double cr[kU];
#ifdef NDNET_WQ_NORECIP  // timing experiment only (wrong results): reciprocals without their LDS reads
    if constexpr (!kExact)
#pragma unroll
      for (int u = 0; u < kU; u++) cr[u] = 1.0 / 3.0 + u;
#else
    if constexpr (!kExact) recips(cr, q0);
#endif
    double pt = 0.0, pu = 0.0, pcn = 1.0, prc = 1.0;       // the previous sample's head results
    unsigned long long plane = 0;
    if constexpr (kExact) {
      // the refold (never on ordinary data): plain order
#pragma unroll
      for (int u = 0; u < kU; u++) {
        const uint32_t q = q0 + (uint32_t)u;
        const unsigned long long lanes = __ballot(act && q < cnt);
        const double cn = (double)(q + 1u);
        const double x = (double)r[u];
        const double t = x - mean;
        const double nm = mean + t / cn;
        const double uu = x - nm;
        const double nm2 = m2 + t * uu;
        const double pr = dpp_d<0xC4>(uu) * dpp_d<0xE9>(t);
        const double cv = off + pr / cn;
        mean = sel_d(lanes, nm, mean);
        m2 = sel_d(lanes, nm2, m2);
        off = sel_d(lanes, (cv != cv) ? 0.0 : cv, off);
      }
    } else {
// pins a pair's results at this point of the instruction stream (an empty
// volatile asm that "modifies" them: nothing computing them sinks below it,
// nothing using them hoists above it, and volatile asms keep their order)
#define WQ_PIN2(a, b) asm volatile("" : "+v"(a), "+v"(b))
      // A lane past its count folds x = mean: t = 0, the mean gains +0, u = 0,
      // m2 and the off-diagonal gain +0 -- an exact no-op (the sums start at +0
      // and never become -0), so one select on x replaces three on the state.
#pragma unroll
      for (int u = 0; u <= kU; u++) {  // u == kU: the last sample's tail alone
        const bool head = u < kU, tail = u > 0;
        const uint32_t q = q0 + (uint32_t)u;
        const double cn = (double)(q + 1u);
        const double rc = head ? cr[u < kU ? u : 0] : 0.0;
        double x = 0.0, t = 0.0, q0v = 0.0, rem = 0.0, qq = 0.0, nm = 0.0, uu = 0.0;
        double pm = 0.0, ua = 0.0, tb = 0.0, pr = 0.0, q1 = 0.0, rm1 = 0.0, qq1 = 0.0;
        if constexpr (!std::is_same<T, float>::value) {
          if (head) bad |= (!kMasked || (act && q < cnt)) && !wq_in_range(r[u < kU ? u : 0]);
        }
        // pair 1: t | u_a
        if (head) {
          x = (double)r[u < kU ? u : 0];
          if constexpr (kMasked) x = sel_d(__ballot(act && q < cnt), x, mean);
          t = x - mean;
        }
        if (tail) { ua = dpp_d<0xC4>(pu); }
        WQ_PIN2(t, ua);
        // pair 2: t / n (1) | t_b, t u
        if (head) q0v = t * rc;
        if (tail) { tb = dpp_d<0xE9>(pt); pm = pt * pu; }
        WQ_PIN2(q0v, tb);
        // pair 3: t / n (2) | u_a t_b
        if (head) rem = fma(-cn, q0v, t);
        if (tail) pr = ua * tb;
        WQ_PIN2(rem, pr);
        // pair 4: t / n (3) | its division (1)
        if (head) qq = fma(rem, rc, q0v);
        if (tail) q1 = pr * prc;
        WQ_PIN2(qq, q1);
        // pair 5: the new mean | the division (2), m2
        if (head) nm = mean + qq;
        if (tail) {
          rm1 = fma(-pcn, q1, pr);
          m2 = m2 + pm;
        }
        WQ_PIN2(nm, rm1);
        // pair 6: u | the division (3)
        if (head) {
          uu = x - nm;
          mean = nm;
        }
        if (tail) qq1 = fma(rm1, prc, q1);
        WQ_PIN2(uu, qq1);
        if (tail) off = off + qq1;
        pt = t;
        pu = uu;
        pcn = cn;
        prc = rc;
      }
#undef WQ_PIN2
    }
  };
  auto run = [&](uint32_t lim, bool act, auto exact_tag) __attribute__((always_inline)) {
    load(r0, 0);
    load(r1, kU);
    load(r2, 2 * kU);
    load(r3, 3 * kU);
    // blocks every live quad fills run without the per-sample selects
    // (the exact refold keeps the state of the quads it does not redo: always masked)
    const uint32_t full = decltype(exact_tag)::value ? 0u : wave_min_u32(live ? cnt : 0xffffffffu);
    auto step = [&](const Blk& r, uint32_t q0) __attribute__((always_inline)) {
      if (q0 + kU <= full) fold(r, q0, act, exact_tag, std::false_type{});
      else fold(r, q0, act, exact_tag, std::true_type{});
    };
    for (uint32_t q0 = 0; q0 < lim; q0 += kWqNB * kU) {  // every branch below is wave-uniform
      step(r0, q0);
      load(r0, q0 + 4 * kU);
      if (q0 + kU >= lim) break;
      step(r1, q0 + kU);
      load(r1, q0 + 5 * kU);
      if (q0 + 2 * kU >= lim) break;
      step(r2, q0 + 2 * kU);
      load(r2, q0 + 6 * kU);
      if (q0 + 3 * kU >= lim) break;
      step(r3, q0 + 3 * kU);
      load(r3, q0 + 7 * kU);
    }
  };
  unsigned long long ph[3] = {0, 0, 0};
  if (hv) {
    const T* rec = nd_pts + ((uint64_t)b * n + __builtin_amdgcn_readfirstlane(beg)) * 3;
    const uint32_t hc = __builtin_amdgcn_readfirstlane(c0);  // c0, beg: the same in every lane here
    double* hl = reinterpret_cast<double*>(&wq_stage[wave * 16][0]);
    if (wq_marks) wq_heavy<T, true>(rec, hc, rtab, hl, wq_hr[wave], lane, mean, m2, off, bad, ph);
    else wq_heavy<T>(rec, hc, rtab, hl, wq_hr[wave], lane, mean, m2, off, bad);
  } else if constexpr (!L64) {  // (light64: light items never reach this point)
    run(mx, true, std::false_type{});
  }
  if (wq_marks) mk_t1 = __builtin_amdgcn_s_memtime();
  // float input: every finite coordinate is in div_fast's exact range, and a
  // non-finite one makes the running mean non-finite from then on (x - mean
  // and mean + ... stay inf / NaN), so the final state flags it
  if constexpr (std::is_same<T, float>::value) bad = !(fabs(mean) <= 0x1.fffffffffffffp+1023);
  // a quad whose coordinates left the fast range refolds exactly
  const bool qbad = __builtin_amdgcn_mov_dpp((int)bad, 0x00, 0xF, 0xF, false) |
                    __builtin_amdgcn_mov_dpp((int)bad, 0x55, 0xF, 0xF, false) |
                    __builtin_amdgcn_mov_dpp((int)bad, 0xAA, 0xF, 0xF, false);  // lanes 0..2 of the quad
  if (__any(qbad)) {
    const uint32_t mx2 = wave_max_u32(qbad ? cnt : 0u);
    if (qbad) {
      mean = 0.0;
      m2 = 0.0;
      off = 0.0;
    }
    run(mx2, qbad, std::true_type{});
  }
  const double vraw = m2 / (double)cnt;
  const double vd = (vraw != vraw) ? 0.0 : vraw;
  if (live && j < 3) {
    // the covariance and (below) the chain mask are handed to the wave that
    // completes this ND's 64-ND group (wq_lu_group): write-through (sc1)
    // stores, drained before the group counter (MI355X_MICROARCH.md,
    // inter-workgroup visibility)
    nd_mean[3 * o + j] = mean;
    st_sc1_f64(&nd_cov[9 * o + 4 * j], vd);
    const uint32_t ia = j == 2 ? 0u : j, ib = j == 2 ? 2u : j + 1u;
    st_sc1_f64(&nd_cov[9 * o + 3 * ia + ib], off);
    st_sc1_f64(&nd_cov[9 * o + 3 * ib + ia], off);
  }
  // The ND's KL chain: eligible directions (a neighbour, and
  // more than one sample on both sides) and the chain mask.  The in-place LU
  // states of the chain: wq_lu_group, one ND per lane.
  {
    uint32_t el = 0;
#pragma unroll
    for (int k = 0; k < 2; k++) {
      const uint32_t dd = j + 4u * (uint32_t)k;
      if (live && dd < 6u) CA.nb[6 * o + dd] = nw[k];
      if (nw[k] >= 0 && cnt > 1 && ncn[k] > 1) el |= 1u << dd;
    }
    el |= (uint32_t)__builtin_amdgcn_mov_dpp((int)el, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
    el |= (uint32_t)__builtin_amdgcn_mov_dpp((int)el, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
    if (live && j == 0) __hip_atomic_store(&CA.nkeys[o], chain_mask(el), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  const uint32_t nbins = (uint32_t)ncls + 1u;
  const bool hist_lds = (size_t)kWqHistNDs * nbins * sizeof(uint32_t) <= (size_t)kWqHistMax;
  if (live && nd_lbl && hist_lds) {
    // the whole quad counts: lane j takes the 8-label runs j, j + 4, ... of
    // each 128-label round (the quad reads 256 contiguous bytes per round, 32
    // loads in flight per lane) and adds into the ND's LDS histogram with
    // return-less LDS atomics, so no increment waits on the previous one.
    // One lane counting alone waited on a load and an LDS read-modify-write
    // per label: L's 1675-label ND took ~100 us of a labelled run.
    // light64: a lane per slot, [wave * 64, wave * 64 + 64) per wave, so a heavy
    // wave's quad 0 takes its own wave's first slot (a quad index would land
    // in another wave's range while that wave's light64 item counts into it)
    uint32_t* hist = wq_hist + (L64 ? (threadIdx.x & ~3u) : (threadIdx.x >> 2)) * nbins;
    for (uint32_t k = j; k < nbins; k += 4) hist[k] = 0;
    __builtin_amdgcn_wave_barrier();
    const uint16_t* l = nd_lbl + (uint64_t)b * n + beg;
    uint32_t s0 = 0;
    for (; s0 + 128 <= cnt; s0 += 128) {
      uint16_t v[32];
#pragma unroll
      for (int g = 0; g < 4; g++)
#pragma unroll
        for (int t = 0; t < 8; t++) v[8 * g + t] = l[s0 + 32 * g + 8 * j + t];
#pragma unroll
      for (int k = 0; k < 32; k++)
        if (v[k] < nbins) atomicAdd(&hist[v[k]], 1u);
    }
    for (uint32_t s = s0 + j; s < cnt; s += 4)
      if (l[s] < nbins) atomicAdd(&hist[l[s]], 1u);
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS atomics are done
    if (j == 0) {
      uint32_t best = 0;
      uint16_t cls = 0;
      for (uint32_t k = 0; k < nbins; k++) {
        const uint32_t h = hist[k];
        if (h > best) { best = h; cls = (uint16_t)k; }
      }
      nd_cls[o] = cls;
    }
  } else if (live && j == 0) {
    uint16_t cls = 0;
    if (nd_lbl) {  // histograms too large for LDS: one lane, in global memory
      const uint32_t nb = nbins;
      uint32_t* hist = hist_all + o * nb;
      for (uint32_t k = 0; k < nb; k++) hist[k] = 0;
      const uint16_t* l = nd_lbl + (uint64_t)b * n + beg;
      uint32_t s2 = 0;
      for (; s2 + 8 <= cnt; s2 += 8) {
        uint16_t v[8];
#pragma unroll
        for (int k = 0; k < 8; k++) v[k] = l[s2 + k];
#pragma unroll
        for (int k = 0; k < 8; k++)
          if (v[k] < nb) hist[v[k]]++;
      }
      for (; s2 < cnt; s2++)
        if (l[s2] < nb) hist[l[s2]]++;
      uint32_t best = 0;
      for (uint32_t k = 0; k < nb; k++)
        if (hist[k] > best) { best = hist[k]; cls = (uint16_t)k; }
    }
    nd_cls[o] = cls;
  }
  // count this item's NDs into their 64-ND group; the wave that completes a
  // group runs its LU chains, one ND per lane
  {
    const uint32_t nlive = hv ? 1u : (uint32_t)__popcll(__ballot(live && j == 0));
    if (nlive) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's sc1 stores are done
      const uint32_t g = wd0 / 64u, gcap = (ndcap + 63u) / 64u;
      const uint32_t total = nd - 64u * g < 64u ? nd - 64u * g : 64u;
      uint32_t* gc = CA.lu_done + (uint64_t)b * gcap + g;
      uint32_t old = 0;
      if (lane == 0) old = __hip_atomic_fetch_add(gc, nlive, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      old = __builtin_amdgcn_readfirstlane(old);
      if (old + nlive == total) {
        if (lane == 0) __hip_atomic_store(gc, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-armed
        wq_lu_group(CA, b, 64u * g + lane, nd, ndcap);
      }
    }
  }
  if (wq_marks) {
    const unsigned long long t2 = __builtin_amdgcn_s_memtime();
    const uint32_t mxc = hv ? c0 : mx;
    if (lane == 0) {
      unsigned long long* w = wq_marks + (uint64_t)item * kWqMarkW;
      w[0] = mk_rt;
      w[1] = mk_t0;
      w[2] = mk_t1;
      w[3] = t2;
      // placement: HW_ID (wave, SIMD, CU, SH, SE) and the XCC, to see which items shared a SIMD
      const uint32_t hwid = __builtin_amdgcn_s_getreg((31 << 11) | 4);
      const uint32_t xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20) & 15u;
      w[4] = ((unsigned long long)hv << 63) | ((unsigned long long)xcc << 56) | ((unsigned long long)(mxc & 0xFFFFFFu) << 32) | hwid;
      w[5] = ph[0];
      w[6] = ph[1];
      w[7] = ph[2];
    }
  }
  }  // item
}

// Bitonic sort of (key, idx) pairs ascending, n a power of two, within one workgroup.
// phase stamp of k_kl (timing level 2): 100 MHz constant clock
#define KL_MARK(i)                                                                   \
  do {                                                                               \
    if (A.marks && threadIdx.x == 0) A.marks[(uint64_t)b * kKLMarks + (i)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)

struct KLArgs {
  unsigned long long* marks;  // [B][kKLMarks] phase stamps of the KL kernels, or null
  CloudCtl* ctl;
  uint32_t* wq_ctr;           // k_welford_q's item counter, re-armed by k_kl_rank_chunks
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
  uint32_t* chain_ok_all;
  double* slot_val_all;
  uint32_t* slot_flag_all;
  double* ev_val_all;
  uint32_t* ev_p_all;
  uint32_t* ev_q_all;
  double* ev_min_all;
  unsigned long long* sort_key_all;
  uint32_t* sort_idx_all;
  uint32_t* nan_list_all;
  unsigned long long* nan_key_all;
  uint32_t* nan_slot_all;
  uint32_t* chunk_nanbase;
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
  ndnet_ndt_stats* stats_out;  // the caller's copy (written alongside; replaces a D2D copy launch), or null
  uint64_t vcap;
  uint32_t ndcap, ecap, sortcap, nchunk;
  uint32_t* chunk_cnt;
  double* chunk_min;
  uint64_t k;
  int ncls;
  int kl_lds;            // prune_and_emit keeps its per-cloud arrays in LDS (kl_lds_bytes)
  int mode;              // kKLEager, kKLLazy or kKLBuild (see kl_list_skipped)
  uint32_t merge_lds_keys;  // k_kl_merge<1>: 64-bit keys its dynamic LDS holds (score runs, then NaN keys if they fit)
};

// The retained list (the reference's kl_divergences array, in insertion
// order) only matters to the level-1 prune when it removes something: with
// num_nds <= k the prune keeps every ND (to_remove = 0) or fails with rc -1
// before reading it (ndt.c:36-39), and the output rows are the NDs in voxel
// order either way.  A lazy run (kKLLazy) then scores no events and sorts
// nothing for that cloud, it only counts the events (num_events / num_kl
// as the reference reports them); the list is built on demand (kKLBuild)
// before anything reads it: a further prune level (ndnet_ndt_prune, the
// legacy prune_nds) or a debug dump.  The built list is the one the eager
// run builds, entry for entry.
enum KLMode : int { kKLEager = 0, kKLLazy = 1, kKLBuild = 2 };
__device__ inline bool kl_list_deferrable(const KLArgs& A, const CloudCtl& c) {
  return A.mode == kKLLazy && (uint64_t)c.num_nds <= A.k;
}
// the sort kernels skip a cloud whose list this launch does not build
__device__ inline bool kl_list_skipped(const KLArgs& A, const CloudCtl& c) {
  return A.mode == kKLBuild ? !c.kl_deferred : kl_list_deferrable(A, c);
}

// Prune (ndt.c:28-73) of cloud b's retained list to k NDs, then the output
// rows (ndt.c:75-117).  Shared by k_kl (level 1) and k_prune (later levels).
// One workgroup per cloud, so the walk is latency-bound: with kLds the list's
// ND column, the per-ND first occurrences / alive flags and the walk's
// scratch live in LDS (lds: 5 ndcap + 8 ecap bytes, dynamic), else in global
// scratch.
// The cloud's stats as kl_cloud's thread 0 knows them by the end (its ctl
// fields loaded at the start, the prune's results recorded here as they are
// set), so the stats need no read-back of the ctl words just written.
struct KLStatsSnap {
  int32_t rc, prune_rc;
  uint32_t iters, num_nds, num_valid, num_kl, num_events, num_out;
  uint32_t list_off, num_phys;  // (not stats: the prune's starting list state)
  uint32_t len[3];
  double off[3], vs;
};

// kCoh: the list's p column was stored in this launch by workgroups on other
// XCDs (sc1): read it with sc1 loads (k_kl_merge's tail).  sn: where thread 0
// records the prune's stats fields (kl_cloud), or null.
template <bool kLds, bool kCoh = false>
__device__ uint32_t prune_and_emit(const KLArgs& A, int b, uint64_t k, uint32_t* s_u32, uint32_t* scratch,
                                   KLStatsSnap* sn = nullptr) {
  static_assert(kLds || !kCoh, "the coherent prune stages the list in LDS");
  extern __shared__ __attribute__((aligned(16))) uint32_t kl_smem[];
  CloudCtl& c = A.ctl[b];
  const uint32_t nd = sn ? sn->num_nds : c.num_nds;
  const uint64_t ob = (uint64_t)b * A.ndcap, eb = (uint64_t)b * A.ecap;
  uint8_t* const g_alive = A.alive_all + ob;
  const uint32_t* const g_op = A.ord_p_all + eb;
  uint32_t* first;
  uint32_t* tmp;
  const uint32_t* op;
  uint32_t* s_op = nullptr;  // kLds: the list's p column in LDS
  uint8_t* alive;
  const uint32_t nv0 = sn ? sn->num_valid : c.num_valid, nkl0 = sn ? sn->num_kl : c.num_kl;
  const uint32_t off = sn ? sn->list_off : c.list_off, nphys = sn ? sn->num_phys : c.num_phys;
  const bool walk = k < nv0;  // the prune removes something: the walk reads the list
  // no ND dead and none to remove: the survivors are every ND, the rows the
  // NDs in order (the level-1 prune of a cloud with num_nds == k)
  const bool identity = !walk && nv0 == nd;
  if constexpr (kLds) {
    first = kl_smem;                                       // [ndcap]
    tmp = kl_smem + A.ndcap;                               // [ecap]
    s_op = kl_smem + A.ndcap + A.ecap;                     // [ecap]
    alive = (uint8_t*)(kl_smem + A.ndcap + 2 * A.ecap);    // [ndcap]
    // (the list's p column is staged block by block by the walk below)
    if (!identity)
      for (uint32_t u = threadIdx.x; u < nd; u += blockDim.x) alive[u] = g_alive[u];
    op = s_op;
    __syncthreads();
  } else {
    first = A.first_occ_all + ob;
    tmp = A.tmp_all + eb;
    op = g_op;
    alive = g_alive;
  }
  __shared__ uint32_t s_failc, s_kpos, s_poison, s_kills;
  int32_t rc = 0;
  uint32_t kills = 0;
  if (k > nv0) {
    rc = -1;  // "Number of desired normal distributions is greater ..." (ndt.c:36-39)
  } else if (!walk) {
    // to_remove = 0: the loop of ndt.c:44-67 runs no iteration, the shift
    // moves nothing; list, counts and flags stay as they are
    if (threadIdx.x == 0) {
      c.num_kl = nkl0;
      if (sn) sn->num_kl = nkl0;
    }
  } else {
    const uint32_t to_remove = (uint32_t)(nv0 - k);
    for (uint32_t u = threadIdx.x; u < nd; u += blockDim.x) first[u] = kInvalid;
    if (threadIdx.x == 0) { s_failc = kInvalid; s_kpos = kInvalid; s_poison = kInvalid; }
    __syncthreads();
    // The walk, a block of the list at a time from the front: first
    // occurrences of the live p within the prefix so far (entries of dead p
    // are skipped by the walk), then their count (the c-th first, 1-based, at
    // position f_c is killed iff f_c < nkl0 - (c-1) for it and every earlier
    // first).  It stops at the block holding the to_remove-th first
    // occurrence: the rest of the list cannot change the kills (a C5 level
    // removes ~200 NDs, found in the first of two 8192-entry blocks).
    uint32_t carry = 0;
    KL_MARK(6);
    // one block of ITB entries per thread: returns whether the
    // to_remove-th first occurrence has been reached
    auto walk_block = [&](auto itc, uint32_t base) -> bool {
      constexpr int ITB = decltype(itc)::value;
      const uint32_t bend = base + blockDim.x * ITB < nkl0 ? base + blockDim.x * ITB : nkl0;
      if constexpr (kLds) {
        // logical entry i is physical entry off + i; past the entries ever
        // written it is poison (the reference's uninitialised tail)
        for (uint32_t i = base + threadIdx.x; i < bend; i += blockDim.x) {
          uint32_t v = kInvalid;
          if (i + off < nphys)
            v = kCoh ? __hip_atomic_load(&g_op[i + off], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : g_op[i + off];
          s_op[i] = v;
        }
        __syncthreads();
      }
      for (uint32_t i = base + threadIdx.x; i < bend; i += blockDim.x) {
        const uint32_t pp = op[i];
        if (pp == kInvalid) { atomicMin(&s_poison, i); continue; }
        if (alive[pp]) atomicMin(&first[pp], i);
      }
      __syncthreads();
      const uint32_t i0 = base + threadIdx.x * ITB;
      uint32_t isf[ITB];
#pragma unroll
      for (int j = 0; j < ITB; j++) {
        const uint32_t i = i0 + j;
        isf[j] = 0;
        if (i < nkl0) {
          const uint32_t pp = op[i];
          isf[j] = (pp != kInvalid && alive[pp] && first[pp] == i);
        }
      }
      uint32_t pre[ITB];
#pragma unroll
      for (int j = 0; j < ITB; j++) pre[j] = isf[j];
      uint32_t tot;
      block_scan_items(pre, 0u, AddU32(), scratch, tot);
#pragma unroll
      for (int j = 0; j < ITB; j++) {
        const uint32_t i = i0 + j;
        if (i >= nkl0) continue;
        if (isf[j]) {
          const uint32_t cth = carry + pre[j] + 1;
          tmp[i] = cth;
          if (cth <= to_remove && i >= nkl0 - (cth - 1)) atomicMin(&s_failc, cth);
          if (cth == to_remove) s_kpos = i;
        } else {
          tmp[i] = 0;
        }
      }
      carry += tot;
      __syncthreads();
      return carry >= to_remove;  // uniform: carry is the block's total
    };
    // a first block of 1024 entries (one or two per thread; the kills usually
    // end there: ~120 of ~1120 NDs at C2-L, ~200 of ~2200 at C5), then 8 per thread
    const bool wide = blockDim.x >= 1024;
    const bool found = wide ? walk_block(std::integral_constant<int, 1>{}, 0u)
                            : walk_block(std::integral_constant<int, 2>{}, 0u);
    if (!found)
      for (uint32_t base = wide ? blockDim.x : 2 * blockDim.x; base < nkl0; base += blockDim.x * 8)
        if (walk_block(std::integral_constant<int, 8>{}, base)) break;
    KL_MARK(7);
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
    KL_MARK(8);
    kills = s_kills;
    if (poisoned) rc = -8;
    else if (kills < to_remove) rc = -2;  // "Reached the end of the divergences array!"
    __syncthreads();
    if (rc == 0 && to_remove > 0 && kLds) {
      // shift left by idx_to_remove = f_{to_remove} + 1 (ndt.c:69-72): kept
      // pending as the list's offset (a further prune level or a dump applies it)
      if (threadIdx.x == 0) {
        c.list_off = off + s_kpos + 1;
        c.num_kl = nkl0 - to_remove;
        if (sn) sn->num_kl = nkl0 - to_remove;
      }
    } else if (rc == 0 && to_remove > 0) {
      // shift left by idx_to_remove = f_{to_remove} + 1 (ndt.c:69-72)
      const uint32_t shift = s_kpos + 1;
      const uint32_t nkl1 = nkl0 - to_remove;
      double* ov = A.ord_val_all + eb;
      uint32_t* oq = A.ord_q_all + eb;
      uint32_t* opw = A.ord_p_all + eb;
      // in-place left shift through the event arrays (free once the list is built)
      double* tv = A.ev_val_all + eb;
      uint32_t* tp = A.ev_p_all + eb;
      uint32_t* tq = A.ev_q_all + eb;
      for (uint32_t i = threadIdx.x; i < nkl1; i += blockDim.x) {
        const uint32_t src = i + shift;
        const bool ok = src < c.num_phys;  // past it: entries the reference never wrote
        const uint32_t sc = ok ? src : 0u;
        const double v = ov[sc];
        const uint32_t pv = opw[sc], qv = oq[sc];
        tv[i] = ok ? v : 0.0;
        tp[i] = ok ? pv : kInvalid;
        tq[i] = ok ? qv : kInvalid;
      }
      __syncthreads();
      for (uint32_t i = threadIdx.x; i < nkl1; i += blockDim.x) {
        ov[i] = tv[i];
        opw[i] = tp[i];
        oq[i] = tq[i];
      }
      __syncthreads();
      if (threadIdx.x == 0) {
        c.num_kl = nkl1;
        if (sn) sn->num_kl = nkl1;
      }
    } else if (threadIdx.x == 0) {
      c.num_kl = nkl0 - kills;
      if (sn) sn->num_kl = nkl0 - kills;
    }
    if (threadIdx.x == 0) {
      c.num_valid = nv0 - kills;
      if (sn) sn->num_valid = nv0 - kills;
    }
  }
  __syncthreads();
  KL_MARK(9);
  // output rows: survivors in ascending voxel order.  Row numbers by a scan
  // of the alive flags (rowmap[r] = ND of row r), then one row per thread
  // with every load issued unconditionally.
  const uint64_t kout = k;
  uint32_t* rowmap = tmp;  // the walk's scratch is free again
  uint32_t carry = identity ? nd : 0u;
  constexpr int IT = 8;
  for (uint32_t base = 0; !identity && base < nd; base += blockDim.x * IT) {
    const uint32_t u0 = base + threadIdx.x * IT;
    uint32_t row[IT], live[IT];
#pragma unroll
    for (int j = 0; j < IT; j++) live[j] = row[j] = (u0 + j < nd) && alive[u0 + j];
    uint32_t tot;
    block_scan_items(row, 0u, AddU32(), scratch, tot);
#pragma unroll
    for (int j = 0; j < IT; j++) {
      const uint32_t rw = carry + row[j];
      if (live[j] && rw < kout) rowmap[rw] = u0 + j;
    }
    carry += tot;
  }
  __syncthreads();
  if constexpr (kLds) {  // the alive flags back to global (further prune levels, dumps)
    if (walk)
      for (uint32_t u = threadIdx.x; u < nd; u += blockDim.x) g_alive[u] = alive[u];
  }
  const uint32_t nrows = carry < kout ? carry : (uint32_t)kout;
  // two rows per thread per round, their loads issued together
  for (uint32_t rw0 = threadIdx.x; rw0 < nrows; rw0 += 2 * blockDim.x) {
    double v2[2][12];
    uint32_t u2[2];
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const uint32_t rw = rw0 + h * blockDim.x;
      const uint32_t rc2 = rw < nrows ? rw : rw0;
      const uint32_t u = identity ? rc2 : rowmap[rc2];
      u2[h] = u;
      const double* m = A.nd_mean + 3 * (ob + u);
      const double* cv = A.nd_cov_post + 9 * (ob + u);
#pragma unroll
      for (int q = 0; q < 3; q++) v2[h][q] = m[q];
#pragma unroll
      for (int q = 0; q < 9; q++) v2[h][3 + q] = cv[q];
    }
#pragma unroll
    for (int h = 0; h < 2; h++) {
    const uint32_t rw = rw0 + h * blockDim.x;
    if (rw >= nrows) break;
    const uint32_t u = u2[h];
    const uint64_t o = (uint64_t)b * kout + rw;
    const double(&v)[12] = v2[h];
    if (A.out) {
      float* r = A.out + 12 * o;
#pragma unroll
      for (int q = 0; q < 12; q++) {
        const float f = (float)v[q];
        r[q] = isfinite(f) ? f : 0.0f;  // nan_to_num(nan=0, posinf=0, neginf=0)
      }
    }
    if (A.out_cls) {  // the whole one-hot row (rows past the survivors: fill_tail)
      float* r = A.out_cls + (uint64_t)(A.ncls + 1) * o;
      const uint32_t cl = A.nd_cls[ob + u];
      for (int q = 0; q <= A.ncls; q++) r[q] = (uint32_t)q == cl ? 1.0f : 0.0f;
    }
    if (A.out_pc64) {
      for (int q = 0; q < 3; q++) A.out_pc64[3 * o + q] = v[q];
      for (int q = 0; q < 9; q++) A.out_cov64[9 * o + q] = v[3 + q];
    }
    if (A.out_cls16) A.out_cls16[o] = A.nd_cls[ob + u];
    }
  }
  __syncthreads();
  KL_MARK(10);
  if (threadIdx.x == 0) {
    c.prune_rc = rc;
    c.num_out = carry;
    c.last_k = (uint32_t)k;
    if (sn) {
      sn->prune_rc = rc;
      sn->num_out = carry;
    }
  }
  (void)s_u32;
  return carry;  // survivors (block-uniform)
}

__device__ void write_stats_to(const KLArgs& A, int b, ndnet_ndt_stats& s);
__device__ inline void write_snap_to(const KLStatsSnap& v, ndnet_ndt_stats& s) {
  s.rc = v.rc;
  s.prune_rc = v.prune_rc;
  s.iters = v.iters;
  for (int a = 0; a < 3; a++) {
    s.len[a] = v.len[a];
    s.offset[a] = v.off[a];
  }
  s.voxel_size = v.vs;
  s.num_nds = v.num_nds;
  s.num_valid = v.num_valid;
  s.num_kl = v.num_kl;
  s.num_events = v.num_events;
  s.num_out = v.num_out;
}
__device__ void write_stats(const KLArgs& A, int b) {
  write_stats_to(A, b, A.stats[b]);
  if (A.stats_out) write_stats_to(A, b, A.stats_out[b]);
}

__device__ void write_stats_to(const KLArgs& A, int b, ndnet_ndt_stats& s) {
  const CloudCtl& c = A.ctl[b];
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

// Rows [r0, k) of cloud b past the survivors: zero (np.zeros in
// ndt_legacy.py:126-143), the class one-hot class 0 (ndtnet_preprocessing.py:55-57).
// The emission writes every row below r0 whole.
__device__ void fill_tail(const KLArgs& A, int b, uint64_t k, uint32_t r0) {
  const uint64_t rb = (uint64_t)b * k;
  if (A.out)
    for (uint64_t i = 12 * (uint64_t)r0 + threadIdx.x; i < 12 * k; i += blockDim.x) A.out[12 * rb + i] = 0.0f;
  if (A.out_cls) {
    const uint64_t w = (uint64_t)(A.ncls + 1);
    for (uint64_t i = w * r0 + threadIdx.x; i < w * k; i += blockDim.x) A.out_cls[w * rb + i] = (i % w) == 0 ? 1.0f : 0.0f;
  }
  if (A.out_pc64) {
    for (uint64_t i = 3 * (uint64_t)r0 + threadIdx.x; i < 3 * k; i += blockDim.x) A.out_pc64[3 * rb + i] = 0.0;
    for (uint64_t i = 9 * (uint64_t)r0 + threadIdx.x; i < 9 * k; i += blockDim.x) A.out_cov64[9 * rb + i] = 0.0;
  }
  if (A.out_cls16)
    for (uint64_t i = r0 + threadIdx.x; i < k; i += blockDim.x) A.out_cls16[rb + i] = 0;
}

// The class one-hot of rows past the survivors is class 0 (ndtnet_preprocessing.py:55-57).
__device__ void pad_class_rows(const KLArgs& A, int b, uint64_t k, uint32_t num_out) {
  if (!A.out_cls) return;
  const uint64_t w = (uint64_t)(A.ncls + 1);
  for (uint64_t r = num_out + threadIdx.x; r < k; r += blockDim.x) A.out_cls[w * ((uint64_t)b * k + r)] = 1.0f;
}

// KL score of one (ND, direction) slot (kullback_leibler.c:129-202 calling
// kl_divergence, :28-127) from the two chain states at the event's rank;
// score = false only flags it.  Every load is issued unconditionally from
// clamped indices, in three rounds (neighbour -> counts and chain masks -> LU
// states).
// The flag of an event of a deferred cloud from the chains' determinant bits
// (k_welford_q's chain_ok): the same rules as kl_event without the states.
__device__ inline uint32_t kl_event_flag(const KLArgs& A, int b, uint32_t s) {
  const uint64_t ob = (uint64_t)b * A.ndcap;
  const uint32_t u = s / 6, d = s % 6;
  const int32_t w = A.nb_all[6 * ob + s];
  if (w < 0) return 0;
  const uint32_t wu = (uint32_t)w;
  if (A.nd_n[ob + u] <= 1 || A.nd_n[ob + wu] <= 1) return 1;  // kl_divergence returns -1, the entry is kept
  const uint32_t mu = A.nkeys_all[ob + u], mw = A.nkeys_all[ob + wu];
  const int rp = __popc(mu & ((1u << (3 + d)) - 1u));
  const int rq = __popc(mw & ((1u << qslot_of_dir(d ^ 1u)) - 1u));
  return (A.chain_ok_all[ob + u] >> rp) & (A.chain_ok_all[ob + wu] >> rq) & 1u;
}

__device__ inline void kl_event(const KLArgs& A, int b, uint32_t s, bool score, uint32_t& flag, double& val) {
  const uint64_t ob = (uint64_t)b * A.ndcap;
  const uint32_t u = s / 6, d = s % 6;
  const uint32_t* vn = A.nd_n + ob;
  const int32_t w = A.nb_all[6 * ob + s];
  const uint32_t wu = w >= 0 ? (uint32_t)w : u;
  const uint32_t nu = vn[u], nw = vn[wu];
  const uint32_t mu = A.nkeys_all[ob + u], mw = A.nkeys_all[ob + wu];
  const int rp = __popc(mu & ((1u << (3 + d)) - 1u));
  const int rq = __popc(mw & ((1u << qslot_of_dir(d ^ 1u)) - 1u));
  const uint32_t rpc = rp < 12 ? (uint32_t)rp : 0u, rqc = rq < 12 ? (uint32_t)rq : 0u;
  const double* chain = A.chain_all + (uint64_t)b * 108 * A.ndcap;
  const uint32_t* cps = A.chain_ps_all + (uint64_t)b * 12 * A.ndcap;
  double Lp[9], Lq[9];
#pragma unroll
  for (int j = 0; j < 9; j++) {
    Lp[j] = chain[(uint64_t)(9 * rpc + j) * A.ndcap + u];
    Lq[j] = chain[(uint64_t)(9 * rqc + j) * A.ndcap + wu];
  }
  const uint32_t psp = cps[(uint64_t)rpc * A.ndcap + u], psq = cps[(uint64_t)rqc * A.ndcap + wu];
  flag = 0;
  val = 0.0;
  if (w >= 0) {
    if (nu <= 1 || nw <= 1) {
      flag = 1;  // kl_divergence returns -1 with div 0 and the entry is kept
    } else {
      const int sp = (psp & 0x100) ? -1 : 1, sq = (psq & 0x100) ? -1 : 1;
      const double pd = lu3_det(Lp, sp), qd = lu3_det(Lq, sq);
      if (!(pd == 0 || qd == 0) && lu3_sgndet(Lp, sp) != 0 && lu3_sgndet(Lq, sq) != 0) {
        flag = 1;
        if (score) val = kl_score(Lp, Lq, psq & 0x3f, pd, qd);
      }
    }
  }
}

// ---- the reference's insertion order as one chip-wide sort ----
//
// kl_divergences inserts every event into a list kept in descending order,
// a tie going after the entries already there; a NaN score compares false
// with everything and lands after the entries x with x > m or x == m
// inserted earlier, m being the minimum non-NaN score inserted before it.
// Both rules are one total order on composite keys (key, slot):
//   non-NaN event at slot s with score v:   (~ord(v), s)
//   NaN event at slot s:                    (~ord(m_s), s), m_s the NaN-skipping
//                                           exclusive prefix min over slots
// (ascending key = descending score; slot order is the insertion order).  For
// a NaN t and a non-NaN x, t precedes x exactly when x is not among the p_t
// entries ahead of t; two NaNs keep slot order because m_s is non-increasing.
// -0.0 is keyed as +0.0 (the reference compares with >, where they are equal).
//
// k_kl_rank_chunks scores its chunk's slots and sorts them (rank by counting
// in LDS);
// k_kl_merge gives every event its global position: its rank in its chunk
// plus, per other chunk, a binary search.  Chunks cover ordered, disjoint slot
// ranges, so a tie against a chunk below counts and against a chunk above
// does not, and the searches need only the 64-bit keys.

__device__ inline unsigned long long score_key(double v) { return ~ord_key(v + 0.0); }

// A lazy run only flags the events of a deferred cloud (kl_list_deferrable).
__global__ void __launch_bounds__(kChunk) k_kl_rank_chunks(KLArgs A) {
  if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x < 8) A.wq_ctr[16 * threadIdx.x] = 0u;  // k_welford_q has finished
  const int b = blockIdx.y;
  const CloudCtl& c = A.ctl[b];
  if (c.state != kAccepted) return;
  if (A.mode == kKLBuild && !c.kl_deferred) return;
  const uint32_t nslots = 6 * c.num_nds;
  const uint32_t ch = blockIdx.x;
  if (ch * kChunk >= nslots) return;
  const uint64_t eb = (uint64_t)b * A.ecap, kb = (uint64_t)b * A.sortcap + (uint64_t)ch * kChunk;
  const uint32_t t = threadIdx.x;
  const uint32_t sl = ch * kChunk + t;
  const bool deferred = kl_list_deferrable(A, c);
  // phase stamps of chunk 0 (timing level 2): start, scores done, end
#define RANK_MARK(i)                                                                               \
  do {                                                                                             \
    if (A.marks && ch == 0 && t == 0) A.marks[(uint64_t)b * kKLMarks + (i)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
  RANK_MARK(3);
  uint32_t fl = 0;
  double vl = 0.0;
  if (deferred) {
    fl = kl_event_flag(A, b, sl < nslots ? sl : 0u);
  } else {
#ifdef NDNET_RANK_NOSCORE  // timing experiment only (wrong results): flags without the KL scores
    kl_event(A, b, sl < nslots ? sl : 0u, false, fl, vl);
#else
    kl_event(A, b, sl < nslots ? sl : 0u, true, fl, vl);  // the clamped slot's result is dropped
#endif
  }
  if (deferred) {  // count the cloud's events (stats num_events / num_kl), one atomic per wave
    const unsigned long long bal = __ballot(sl < nslots && fl);
    if ((t & 63) == 0 && bal)
      __hip_atomic_fetch_add(&A.ctl[b].flag_count, (uint32_t)__popcll(bal), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  RANK_MARK(4);
  if (sl < nslots) A.slot_flag_all[eb + sl] = fl;
  if (sl < nslots) A.slot_val_all[eb + sl] = vl;
  const bool f = sl < nslots && fl;
  const double v = f ? vl : 0.0;
  const bool isn = f && v != v;
  const bool num = f && !isn;
  const unsigned long long key = num ? score_key(v) : ~0ull;
  __shared__ __attribute__((aligned(16))) unsigned long long s_key[kChunk];
  __shared__ double s_f64[16];
  __shared__ uint32_t s_u32[16];
  __shared__ __attribute__((aligned(16))) unsigned long long s_nkey[kChunk + 2];  // the scores' keys, compacted
  s_key[t] = key;
  double pm[1] = {num ? v : __builtin_inf()};
  uint32_t cnt[1] = {(uint32_t)isn | ((uint32_t)num << 16)};
  double mtot;
  uint32_t ctot;
  block_scan_items(pm, __builtin_inf(), MinF64(), s_f64, mtot);
  block_scan_items(cnt, 0u, AddU32(), s_u32, ctot);
  const uint32_t nnum = ctot >> 16;
  if (num) s_nkey[cnt[0] >> 16] = key;
  if (t < 2) s_nkey[nnum + t] = ~0ull;  // pad to an even count (~0 is never a score key)
  __syncthreads();
  // rank in the chunk: keys below, then equal keys at lower slots.  One pass
  // over the chunk's score keys only (compacted) counts keys below and keys
  // equal (two keys per LDS read: 25 -> 21 us at C5's 2000-ND level; a first
  // pass on the keys' 32-bit high words measured slower); the slot order
  // among equal scores is recounted only where a score tie exists (rare).
  // Non-score slots (key ~0) go after the chunk's scores in slot order: only
  // the scores' positions are read (k_kl_merge), the rest must only be ~0.
  uint32_t lt = 0, eq = 0;
#ifdef NDNET_RANK_NORANK  // timing experiment only (wrong results): no in-chunk rank count
  if (false)
#endif
#pragma unroll 4
  for (uint32_t j = 0; j < nnum; j += 2) {
    const ulonglong2 kk = *reinterpret_cast<const ulonglong2*>(&s_nkey[j]);
    lt += (kk.x < key ? 1u : 0u) + (kk.y < key ? 1u : 0u);
    eq += (kk.x == key ? 1u : 0u) + (kk.y == key ? 1u : 0u);
  }
  uint32_t r;
  if (num) {
    r = lt;
    if (eq > 1) {  // a tie: equal scores at lower slots of the chunk come first
      for (uint32_t j = 0; j < t; j++) r += s_key[j] == key ? 1u : 0u;
    }
  } else {
    r = (ctot >> 16) + (t - (cnt[0] >> 16));
  }
  A.sort_key_all[kb + r] = key;  // positions past the chunk's scores hold ~0
  A.sort_idx_all[kb + r] = sl;
  if (isn) {
    const uint32_t j = cnt[0] & 0xffffu;
    A.nan_list_all[eb + ch * kChunk + j] = sl;
    A.ev_min_all[eb + ch * kChunk + j] = pm[0];
  }
  if (t == 0) {
    A.chunk_cnt[(uint64_t)b * A.nchunk + ch] = ctot;
    A.chunk_min[(uint64_t)b * A.nchunk + ch] = mtot;
  }
  RANK_MARK(15);
  if (A.marks && t == 0)  // the cloud's last chunk to end (the stamps only grow, so no reset is needed)
    __hip_atomic_fetch_max(&A.marks[(uint64_t)b * kKLMarks + 18], (unsigned long long)__builtin_amdgcn_s_memrealtime(),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#undef RANK_MARK
}

// NaN keys need the min over all earlier chunks: one pass writes every NaN
// event's key and slot contiguously in slot order (a sorted sequence: keys
// non-decreasing, slots increasing) and the per-chunk NaN bases.
__global__ void __launch_bounds__(kChunk) k_kl_nan_keys(KLArgs A) {
  const int b = blockIdx.y;
  const CloudCtl& c = A.ctl[b];
  if (c.state != kAccepted || kl_list_skipped(A, c)) return;
  const uint32_t nch = (6 * c.num_nds + kChunk - 1) / kChunk;
  const uint32_t ch = blockIdx.x;
  if (ch >= nch) return;
  const uint32_t t = threadIdx.x;
  const uint64_t eb = (uint64_t)b * A.ecap, cb = (uint64_t)b * A.nchunk;
  constexpr int ITC = (kMaxChunks + kChunk - 1) / kChunk;
  __shared__ double s_f64[16];
  __shared__ uint32_t s_u32[16];
  __shared__ uint32_t s_base;
  __shared__ double s_carry;
  uint32_t nanb[ITC];
  double cmin[ITC];
#pragma unroll
  for (int i = 0; i < ITC; i++) {
    const uint32_t c2 = t * ITC + i;
    nanb[i] = c2 < nch ? (A.chunk_cnt[cb + c2] & 0xffffu) : 0u;
    cmin[i] = c2 < nch ? A.chunk_min[cb + c2] : __builtin_inf();
  }
  uint32_t nan_total;
  double min_total;
  block_scan_items(nanb, 0u, AddU32(), s_u32, nan_total);
  block_scan_items(cmin, __builtin_inf(), MinF64(), s_f64, min_total);
#pragma unroll
  for (int i = 0; i < ITC; i++) {
    const uint32_t c2 = t * ITC + i;
    if (c2 == ch) {
      s_base = nanb[i];
      s_carry = cmin[i];
    }
    if (ch == 0 && c2 < nch) A.chunk_nanbase[cb + c2] = nanb[i];
  }
  __syncthreads();
  const uint32_t nn = A.chunk_cnt[cb + ch] & 0xffffu;
  if (t < nn) {
    const uint32_t o = ch * kChunk + t;
    A.nan_key_all[eb + s_base + t] = score_key(MinF64()(s_carry, A.ev_min_all[eb + o]));
    A.nan_slot_all[eb + s_base + t] = A.nan_list_all[eb + o];
  }
}

// #entries of a sorted, ~0-padded kChunk-key run ahead of x: keys <= x (le)
// or keys < x; Q runs searched together (eight halving probes each), so a
// lane has Q independent LDS reads in flight per probe round.  "k <= x" is
// "k < x + 1" (x + 1 saturating: ~0 is padding, never a score key), so a probe
// is one read at a constant offset from the run cursor, one 64-bit compare
// and a conditional cursor step.
template <int Q, typename KP>
__device__ inline void count_before_q(KP K, const uint32_t (&run)[Q], unsigned long long x, const bool (&le)[Q],
                                      uint32_t (&base)[Q]) {
  KP cur[Q];
  unsigned long long xq[Q];
#pragma unroll
  for (int q = 0; q < Q; q++) {
    cur[q] = K + run[q] * kChunk;
    xq[q] = le[q] && x != ~0ull ? x + 1 : x;
  }
#pragma unroll
  for (uint32_t half = kChunk / 2; half >= 1; half >>= 1) {
#pragma unroll
    for (int q = 0; q < Q; q++) cur[q] += cur[q][half - 1] < xq[q] ? half : 0u;
  }
#pragma unroll
  for (int q = 0; q < Q; q++) base[q] = (uint32_t)(cur[q] - (K + run[q] * kChunk)) + (cur[q][0] < xq[q] ? 1u : 0u);
}

// The three NaN-run counts of a score event x (slot s) interleaved, one probe
// of each per round: NaN keys of the earlier chunks <= x, of its own chunk
// before (x, s), of the later chunks < x.  N: the cloud's NaN keys in slot
// order [0, total); own chunk's at [nb0, nb0 + nn), slots S[0, nn).
// Branch-free halving (the range lengths, hence the rounds, are the same for
// every lane of the wave): b moves to b + h where the probe is still ahead of
// x; the count is b - lo + [N[b] ahead of x].
template <typename KP, typename SP>
__device__ inline uint32_t count_nan3(KP N, SP S, uint32_t nb0, uint32_t nn, uint32_t total, unsigned long long x,
                                      uint32_t s) {
  const unsigned long long x1 = x != ~0ull ? x + 1 : x;  // k <= x as k < x1
  auto ahead1 = [&](uint32_t i) {
    const unsigned long long k = N[i];
    return k < x || (k == x && S[i - nb0] < s);
  };
  uint32_t n0 = nb0, n1 = nn, n2 = total - nb0 - nn;
  uint32_t b0 = 0, b1 = nb0, b2 = nb0 + nn;
  while (n0 > 1 || n1 > 1 || n2 > 1) {
    if (n0 > 1) {
      const uint32_t h = n0 >> 1;
      b0 += N[b0 + h] < x1 ? h : 0u;
      n0 -= h;
    }
    if (n1 > 1) {
      const uint32_t h = n1 >> 1;
      b1 += ahead1(b1 + h) ? h : 0u;
      n1 -= h;
    }
    if (n2 > 1) {
      const uint32_t h = n2 >> 1;
      b2 += N[b2 + h] < x ? h : 0u;
      n2 -= h;
    }
  }
  const uint32_t c0 = n0 ? b0 + (N[b0] < x1 ? 1u : 0u) : 0u;
  const uint32_t c1 = n1 ? b1 - nb0 + (ahead1(b1) ? 1u : 0u) : 0u;
  const uint32_t c2 = n2 ? b2 - nb0 - nn + (N[b2] < x ? 1u : 0u) : 0u;
  return c0 + c1 + c2;
}

// #entries (K[i], S[i]), i < n, preceding (x, s) (keys and slots both sorted).
template <typename KP, typename SP>
__device__ inline uint32_t count_composite(KP K, SP S, uint32_t n, unsigned long long x, uint32_t s) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    const unsigned long long k = K[mid];
    if (k < x || (k == x && S[mid] < s)) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

#ifndef NDNET_MERGE_Q
#define NDNET_MERGE_Q 8
#endif
constexpr int kMergeQ = NDNET_MERGE_Q;  // other runs searched together per probe round
#ifndef NDNET_MERGE_RUNS
#define NDNET_MERGE_RUNS 2
#endif
constexpr int kMergeRuns = NDNET_MERGE_RUNS;  // chunks merged per k_kl_merge workgroup (512 threads; ~one workgroup per CU at B = 16)
// mode 1 (score runs staged whole per workgroup, 144 KB: one workgroup per
// CU) merges 4 chunks per workgroup: C5's 57-chunk clouds then fit one round
// of workgroups on the chip instead of two, and stage the runs half as often
#ifndef NDNET_MERGE_RUNS1
#define NDNET_MERGE_RUNS1 4
#endif
constexpr int kMergeRuns1 = NDNET_MERGE_RUNS1;

// kMode 2: score runs and NaN keys in LDS, the NaN keys computed here (up to
// kMergeLdsChunks chunks); 1: score runs in LDS, NaN keys from k_kl_nan_keys
// (up to kMergeScoreChunks); 0: everything from global memory.
// kCoh: the list entries are stored write-through (sc1) for a last
// workgroup on another XCD to read in the same launch (k_kl_merge's tail).
template <int kMode, int kMergeRuns, bool kCoh>
__device__ inline void merge_runs(const KLArgs& A, const int b) {
  constexpr bool kLds = kMode == 2;
  const CloudCtl& c = A.ctl[b];
  if (c.state != kAccepted || kl_list_skipped(A, c)) return;
  const uint32_t nch = (6 * c.num_nds + kChunk - 1) / kChunk;
  if (blockIdx.x * kMergeRuns >= nch) return;
  const uint64_t eb = (uint64_t)b * A.ecap, kb = (uint64_t)b * A.sortcap, cb = (uint64_t)b * A.nchunk;
  const uint32_t tid = threadIdx.x;
  const uint32_t lc = tid / kChunk, t = tid % kChunk;
  // chunk groups blockIdx.x, blockIdx.x + gridDim.x, ...: a plan with a CU
  // share gives the merge fewer, longer workgroups (round 6, merge_wgs)
  uint32_t ch = blockIdx.x * kMergeRuns + lc;
#define MERGE_MARK(i)                                                                              \
  do {                                                                                             \
    if (A.marks && blockIdx.x == 0 && tid == 0) A.marks[(uint64_t)b * kKLMarks + (i)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
  MERGE_MARK(12);
  extern __shared__ __attribute__((aligned(16))) unsigned long long dynk[];
  const unsigned long long* gK = A.sort_key_all + kb;
  unsigned long long* lK = dynk;
  unsigned long long* lN = dynk + (uint64_t)nch * kChunk;
  // the score runs to stage in LDS: every load issued here, in the same
  // round as the chunk counters below, written to LDS after them
  constexpr int kStageU = (kMergeLdsChunks * kChunk / 2 + kChunk * kMergeRuns - 1) / (kChunk * kMergeRuns);
  const uint32_t nv = kLds ? nch * kChunk / 2 : 0u;
  ulonglong2 sv[kStageU];
  // mode 2 also loads, in the same round, its chunk's NaN slots and the first
  // kNanPre NaN minima of every chunk (indices clamped into the cloud's
  // slots), which the NaN keys below would otherwise fetch after the scans
  constexpr uint32_t kNanPre = kChunk * kMergeRuns / kMergeLdsChunks;
  uint32_t own_nan = 0;
  double pre_min = 0.0;
  if (kLds) {
    const ulonglong2* src = reinterpret_cast<const ulonglong2*>(gK);
#pragma unroll
    for (int u = 0; u < kStageU; u++) {
      const uint32_t i = u * blockDim.x + tid;
      sv[u] = src[i < nv ? i : 0];
    }
    const uint32_t os = ch * kChunk + t, ps = (tid / kNanPre) * kChunk + tid % kNanPre;
    own_nan = A.nan_list_all[eb + (os < A.ecap ? os : A.ecap - 1)];
    pre_min = A.ev_min_all[eb + (ps < A.ecap ? ps : A.ecap - 1)];
  } else if (kMode == 1) {  // score runs only: eight 16-byte loads in flight per thread
    const uint32_t nv1 = nch * kChunk / 2;
    const ulonglong2* src = reinterpret_cast<const ulonglong2*>(gK);
    ulonglong2* dst = reinterpret_cast<ulonglong2*>(lK);
    constexpr int U = 8;
    for (uint32_t i0 = 0; i0 < nv1; i0 += U * blockDim.x) {
      ulonglong2 v[U];
#pragma unroll
      for (int u = 0; u < U; u++) {
        const uint32_t i = i0 + u * blockDim.x + tid;
        v[u] = src[i < nv1 ? i : 0];
      }
#pragma unroll
      for (int u = 0; u < U; u++) {
        const uint32_t i = i0 + u * blockDim.x + tid;
        if (i < nv1) dst[i] = v[u];
      }
    }
  }
  __shared__ uint32_t s_cnt[kMaxChunks];
  __shared__ uint32_t s_nb[kMaxChunks + 1];
  __shared__ double s_pm[kMergeLdsChunks];
  __shared__ uint32_t s_own_num_slot[kMergeRuns][kChunk];
  __shared__ uint32_t s_own_nan_slot[kMergeRuns][kChunk];
  __shared__ double s_pre_min[kLds ? kChunk * kMergeRuns : 1];
  if (kLds && tid < nch * kNanPre) s_pre_min[tid] = pre_min;
  for (uint32_t c2 = tid; c2 < nch; c2 += blockDim.x) {
    s_cnt[c2] = A.chunk_cnt[cb + c2];
    if (kLds) s_pm[c2] = A.chunk_min[cb + c2];
    else s_nb[c2] = A.chunk_nanbase[cb + c2];
  }
  if (!kLds && tid == 0) s_nb[nch] = A.chunk_nanbase[cb + nch - 1] + (A.chunk_cnt[cb + nch - 1] & 0xffffu);  // NaN total
  const unsigned long long* gN = A.nan_key_all + eb;
  if (kLds) {
    ulonglong2* dst = reinterpret_cast<ulonglong2*>(lK);
#pragma unroll
    for (int u = 0; u < kStageU; u++) {
      const uint32_t i = u * blockDim.x + tid;
      if (i < nv) dst[i] = sv[u];
    }
  }
  __syncthreads();
  MERGE_MARK(16);
  if (kLds) {
    // the NaN bases and the min over earlier chunks (k_kl_nan_keys' scans),
    // one lane per chunk (nch <= kMergeLdsChunks < 64)
    if (tid < 64) {
      uint32_t nn = tid < nch ? (s_cnt[tid] & 0xffffu) : 0u;
      double cm = tid < nch ? s_pm[tid] : __builtin_inf();
      for (int off = 1; off < 64; off <<= 1) {
        const uint32_t o = __shfl_up(nn, off, 64);
        const double om = __shfl_up(cm, off, 64);
        if ((int)tid >= off) {
          nn += o;
          cm = MinF64()(cm, om);
        }
      }
      uint32_t ex = __shfl_up(nn, 1, 64);
      double exm = __shfl_up(cm, 1, 64);
      if (tid == 0) {
        ex = 0;
        exm = __builtin_inf();
      }
      if (tid < nch) {
        s_nb[tid] = ex;
        s_pm[tid] = exm;
      }
      if (tid + 1 == nch) s_nb[nch] = nn;
    }
    __syncthreads();
    MERGE_MARK(17);
  }
  const uint32_t nnan_tot = s_nb[nch];
  // mode 1: the NaN keys (from k_kl_nan_keys) join the score runs in LDS when they fit
  const bool nan_lds = kMode == 1 && (uint64_t)nch * kChunk + nnan_tot <= A.merge_lds_keys;
  if (nan_lds) {
    for (uint32_t i = tid; i < nnan_tot; i += blockDim.x) lN[i] = gN[i];
  }
  if (kLds) {  // the NaN keys, computed in place
    for (uint32_t i = tid; i < nnan_tot; i += blockDim.x) {
      // the chunk of NaN i: the last one whose base is <= i
      uint32_t lo = 0, hi = nch;
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (s_nb[mid] <= i) lo = mid;
        else hi = mid;
      }
      const uint32_t j = i - s_nb[lo];
      const double em = j < kNanPre ? s_pre_min[lo * kNanPre + j] : A.ev_min_all[eb + lo * kChunk + j];
      lN[i] = score_key(MinF64()(s_pm[lo], em));
    }
  }
  __syncthreads();
  MERGE_MARK(13);
  for (uint32_t grp = blockIdx.x; grp * kMergeRuns < nch; grp += gridDim.x) {
  ch = grp * kMergeRuns + lc;
  if (grp != blockIdx.x) {
    __syncthreads();  // the previous group's slot tables are read
    if (kLds && ch < nch) own_nan = A.nan_list_all[eb + ch * kChunk + t];
  }
  const uint32_t cc = ch < nch ? s_cnt[ch] : 0u;
  const uint32_t nnum = cc >> 16, nnan = cc & 0xffffu;
  const uint32_t nb0 = ch < nch ? s_nb[ch] : 0u;
  if (ch < nch) s_own_num_slot[lc][t] = A.sort_idx_all[kb + ch * kChunk + t];
  if (ch < nch && t < nnan) s_own_nan_slot[lc][t] = kLds ? own_nan : A.nan_slot_all[eb + nb0 + t];
  __syncthreads();
  const bool is_num = t < nnum;
  if (ch >= nch || (!is_num && t >= nnum + nnan)) continue;
  const uint32_t* own_num_slot = s_own_num_slot[lc];
  const uint32_t* own_nan_slot = s_own_nan_slot[lc];
  auto body = [&](auto K, auto N) {
    uint32_t sl;
    unsigned long long x;
    uint32_t pos;
    if (is_num) {
      x = K[ch * kChunk + t];
      sl = own_num_slot[t];
      pos = t;
      // NaN events ahead: earlier chunks (key <= x), this chunk (composite), later chunks (key < x)
      if (nnan_tot) {
        pos += count_nan3(N, own_nan_slot, nb0, nnan, nnan_tot, x, sl);
      }
    } else {
      const uint32_t j = t - nnum;
      x = N[nb0 + j];
      sl = own_nan_slot[j];
      // scores of its own chunk ahead of it, then every earlier NaN
      pos = count_composite(K + ch * kChunk, own_num_slot, nnum, x, sl) + nb0 + j;
    }
    // scores of the other chunks ahead of it, kMergeQ runs per pass
    for (uint32_t c0 = 0; c0 < nch; c0 += kMergeQ) {
      uint32_t run[kMergeQ], add[kMergeQ];
      bool le[kMergeQ];
#pragma unroll
      for (int q = 0; q < kMergeQ; q++) {
        const uint32_t c2 = c0 + q;
        run[q] = (c2 < nch && c2 != ch) ? c2 : ch;  // own run: masked below
        le[q] = c2 < ch;
      }
      count_before_q<kMergeQ>(K, run, x, le, add);
#pragma unroll
      for (int q = 0; q < kMergeQ; q++)
        if (c0 + q < nch && c0 + q != ch) pos += add[q];
    }
    const double ov = A.slot_val_all[eb + sl];
    const uint32_t oq = (uint32_t)A.nb_all[6 * (uint64_t)b * A.ndcap + sl];
    if constexpr (kCoh) {
      st_sc1_f64(&A.ord_val_all[eb + pos], ov);
      __hip_atomic_store(&A.ord_p_all[eb + pos], sl / 6, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&A.ord_q_all[eb + pos], oq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      A.ord_val_all[eb + pos] = ov;
      A.ord_p_all[eb + pos] = sl / 6;
      A.ord_q_all[eb + pos] = oq;
    }
  };
  if (kLds) body(static_cast<const unsigned long long*>(lK), static_cast<const unsigned long long*>(lN));
  else if (kMode == 1 && nan_lds)
    body(static_cast<const unsigned long long*>(lK), static_cast<const unsigned long long*>(lN));
  else if (kMode == 1) body(static_cast<const unsigned long long*>(lK), gN);
  else body(gK, gN);
  }  // chunk groups
  MERGE_MARK(14);
  if (A.marks && t == 0)  // the cloud's last merge workgroup to end
    __hip_atomic_fetch_max(&A.marks[(uint64_t)b * kKLMarks + 19], (unsigned long long)__builtin_amdgcn_s_memrealtime(),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#undef MERGE_MARK
}

// Poison beyond the written list (the reference's uninitialised tail).
__device__ void kl_poison_tail(const KLArgs& A, uint64_t eb, uint32_t E) {
  double* ov = A.ord_val_all + eb;
  uint32_t* opp = A.ord_p_all + eb;
  uint32_t* oq = A.ord_q_all + eb;
  for (uint32_t i = E + threadIdx.x; i < A.ecap; i += blockDim.x) {
    opp[i] = kInvalid;
    oq[i] = kInvalid;
    ov[i] = 0.0;
  }
}

// The end of an on-demand list build (kKLBuild): the tail poisoned, the
// cloud's list marked built.  Counts and flags were set by the run.
__global__ void __launch_bounds__(256) k_kl_list_done(KLArgs A) {
  const int b = blockIdx.x;
  CloudCtl& c = A.ctl[b];
  if (c.state != kAccepted || !c.kl_deferred) return;
  kl_poison_tail(A, (uint64_t)b * A.ecap, c.num_events);
  __syncthreads();
  if (threadIdx.x == 0) c.kl_deferred = 0;
}

// Prune and output rows of cloud b by one workgroup (k_kl, or the last
// k_kl_merge workgroup of the cloud: kCoh).
template <bool kCoh>
__device__ void kl_cloud(const KLArgs& A, const int b) {
  CloudCtl& c = A.ctl[b];
  __shared__ uint32_t s_u32[16];
  __shared__ KLStatsSnap s_sn;
  KL_MARK(0);
  if (c.state != kAccepted) {
    zero_outputs(A, b, A.k);
    if (threadIdx.x == 0) {
      c.num_out = 0;
      c.kl_deferred = 0;
      write_stats(A, b);
    }
    pad_class_rows(A, b, A.k, 0);
    return;
  }
  KL_MARK(1);
  const uint32_t nd = c.num_nds;
  const uint64_t ob = (uint64_t)b * A.ndcap, eb = (uint64_t)b * A.ecap;
  const uint32_t nch = (6 * nd + kChunk - 1) / kChunk;
  const bool deferred = kl_list_deferrable(A, c);
  if (threadIdx.x == 0) {  // the stats fields the KL stage does not change, loaded with the chunk counters
    s_sn.rc = c.rc;
    s_sn.iters = c.iter;
    for (int a = 0; a < 3; a++) {
      s_sn.len[a] = c.len[a];
      s_sn.off[a] = c.off[a];
    }
    s_sn.vs = c.vs;
    s_sn.num_nds = nd;
  }
  // event count: from the chunk counters, or (deferred list) k_kl_rank_chunks' count
  uint32_t e_part = 0;
  if (!deferred) {
    for (uint32_t c2 = threadIdx.x; c2 < nch; c2 += blockDim.x) {
      const uint32_t* cp = &A.chunk_cnt[(uint64_t)b * A.nchunk + c2];
      const uint32_t cc = kCoh ? ld_sc1(cp) : *cp;  // (kCoh: k_kl_rank_sort stored them in this launch)
      e_part += (cc >> 16) + (cc & 0xffffu);
    }
  }
  uint32_t ev[1] = {e_part};
  uint32_t E;
  block_scan_items(ev, 0u, AddU32(), s_u32, E);
  if (deferred) E = kCoh ? ld_sc1(&c.flag_count) : c.flag_count;
  KL_MARK(2);
  if (!deferred) kl_poison_tail(A, eb, E);
  for (uint32_t u = threadIdx.x; u < nd; u += blockDim.x) A.alive_all[ob + u] = 1;
  if (threadIdx.x == 0) {
    c.kl_deferred = deferred ? 1u : 0u;
    c.list_off = 0;
    c.num_events = E;
    c.num_kl = E;
    c.num_phys = E;
    c.num_valid = nd;
    s_sn.list_off = 0;
    s_sn.num_events = s_sn.num_kl = s_sn.num_phys = E;
    s_sn.num_valid = nd;
  }
  __syncthreads();
  KL_MARK(5);
  uint32_t nout;
  if constexpr (kCoh) nout = prune_and_emit<true, true>(A, b, A.k, s_u32, s_u32, &s_sn);  // the host fuses only kl_lds plans
  else
    nout = A.kl_lds ? prune_and_emit<true>(A, b, A.k, s_u32, s_u32, &s_sn)
                    : prune_and_emit<false>(A, b, A.k, s_u32, s_u32, &s_sn);
  fill_tail(A, b, A.k, nout < A.k ? nout : (uint32_t)A.k);
  __syncthreads();
  if (threadIdx.x == 0) {
    write_snap_to(s_sn, A.stats[b]);
    if (A.stats_out) write_snap_to(s_sn, A.stats_out[b]);
  }
  KL_MARK(11);
}

__global__ void __launch_bounds__(kKLThreads) k_kl(KLArgs A) { kl_cloud<false>(A, blockIdx.x); }

// The event order of every cloud (merge_runs); with kTail the cloud's last
// workgroup to finish then prunes it and writes its rows (kl_cloud), which
// saves k_kl's launch and the kernel boundary.  The list entries are stored
// and read write-through (sc1, as k_welford_q's LU groups hand over their
// covariances); each wave drains its stores before the workgroup's ticket.
template <int kMode, int kMergeRuns = ::kMergeRuns, bool kTail = false>
__global__ void __launch_bounds__(kChunk * kMergeRuns) k_kl_merge(KLArgs A) {
  const int b = blockIdx.y;
  merge_runs<kMode, kMergeRuns, kTail>(A, b);
  if constexpr (kTail) {
    __shared__ uint32_t s_last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's list stores are done
    __syncthreads();
    if (threadIdx.x == 0)
      s_last = __hip_atomic_fetch_add(&A.ctl[b].kl_arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
               gridDim.x - 1;
    __syncthreads();
    if (!s_last) return;
    if (threadIdx.x == 0) __hip_atomic_store(&A.ctl[b].kl_arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    kl_cloud<true>(A, b);
  }
}

// ------------------------------------------------- the one-workgroup list sort
// Round 6: when a cloud's whole event list fits one CU's
// LDS twice -- 20 bytes per slot (64-bit key + 16-bit slot, two buffers):
// ecap <= 7680, i.e. k <= 1065, C2's k = 1000 -- one workgroup per cloud
// sorts it instead of merge_runs' workgroups per chunk group.  The total
// order is the composite (key, slot) of merge_runs (above): k_kl_rank_chunks'
// chunk runs are sorted by it, and so is the NaN run (keys non-decreasing in
// slot order).  The score runs are merged pairwise in LDS, log2(chunks)
// levels; two adjacent runs hold ordered slot ranges, so a tie against the
// run below counts and one against the run above does not -- the key alone
// decides, and an element's chunk (its group at every level) is its slot / 256.
// The last level merges the score list with the NaN run comparing (key, slot).
// Each element does ~9-13 fixed halving probes per level (6 levels at C2:
// ~70 in all) where merge_runs does ~8 per other chunk plus three NaN-run
// searches (~250), and the launch holds 16 CUs instead of the merge's ~110-224:
// the L line's KL stage is CU time the chains share.
constexpr uint32_t kSortMaxChunks = 64;          // the offsets are one wave's scan
static_assert(kKLThreads == 1024, "k_kl_sort's item loops assume 1024 threads");

// One buffer of the sort: the 64-bit keys and the slots.
struct SortBuf {
  unsigned long long* k;
  uint16_t* s;
};

// pos[q]: keys of the sorted run [st[q], st[q] + n[q]) below xq[q], `rounds`
// halving probes (2^rounds > every n).  A probe past the run reads its last
// key instead: if that is below xq the whole run is, and pos lands on n, so
// the bound needs no test of its own -- a probe is an add, a min, the address,
// one 8-byte LDS read, a 64-bit compare and a select (the kernel is VALU-issue
// bound: 4 cycles per wave64 op on a SIMD).  An empty run (n = 0) counts 0.
template <int Q>
__device__ inline void run_count_q(const unsigned long long* K, const uint32_t (&st)[Q], const uint32_t (&n)[Q],
                                   const unsigned long long (&xq)[Q], int rounds, uint32_t (&pos)[Q]) {
  const unsigned long long* base[Q];
  unsigned long long xe[Q];
#pragma unroll
  for (int q = 0; q < Q; q++) {
    pos[q] = 0;
    base[q] = K + (n[q] ? st[q] - 1 : 0u);
    xe[q] = n[q] ? xq[q] : 0ull;
  }
  for (int r = rounds - 1; r >= 0; r--) {
    const uint32_t h = 1u << r;
    uint32_t m[Q];
    unsigned long long k[Q];
#pragma unroll
    for (int q = 0; q < Q; q++) {
      m[q] = min(pos[q] + h, n[q]);
      k[q] = base[q][m[q]];
    }
#pragma unroll
    for (int q = 0; q < Q; q++) pos[q] = k[q] < xe[q] ? m[q] : pos[q];
  }
}

__device__ inline int bit_len(uint32_t v) { return v ? 32 - __clz(v) : 0; }

// One merge level over elements [e0, e0 + Q * 1024) of the score list: runs of
// 2^l chunks merged pairwise from I into O (an element's group: slot / 256 >> l;
// against the run below it counts keys <= x, i.e. < x + 1: score keys are
// never ~0)
template <int Q>
__device__ inline void sort_level_items(const SortBuf& I, const SortBuf& O, const uint32_t* soff, uint32_t nch,
                                        uint32_t l, uint32_t S, int rounds, uint32_t e0) {
  unsigned long long x[Q], xq[Q];
  uint32_t sl[Q], st[Q], n[Q], dst[Q], pos[Q];
#pragma unroll
  for (int q = 0; q < Q; q++) {
    const uint32_t e = e0 + q * kKLThreads + threadIdx.x;
    const uint32_t ec = e < S ? e : 0u;
    x[q] = I.k[ec];
    sl[q] = I.s[ec];
    const uint32_t g = (sl[q] / kChunk) >> l, p = g ^ 1u;
    const uint32_t lp = p << l, lm = (g < p ? g : p) << l;
    dst[q] = soff[lm] + (e - soff[g << l]);
    xq[q] = p < g ? x[q] + 1 : x[q];
    st[q] = 0;
    n[q] = 0;
    if (e < S && lp < nch) {
      st[q] = soff[lp];
      n[q] = soff[lp + (1u << l) < nch ? lp + (1u << l) : nch] - st[q];
    }
  }
  run_count_q<Q>(I.k, st, n, xq, rounds, pos);
#pragma unroll
  for (int q = 0; q < Q; q++) {
    if (e0 + q * kKLThreads + threadIdx.x < S) {
      O.k[dst[q] + pos[q]] = x[q];
      O.s[dst[q] + pos[q]] = (uint16_t)sl[q];
    }
  }
}

// The last level over elements [e0, e0 + Q * 1024) of [0, S + NN): the score
// list with the NaN run (a score counts the NaNs ahead of it, a NaN the
// scores) in the composite order: keys below x, then the partner's entries of
// key x at lower slots (its equal keys are in slot order; a NaN's key, a
// prefix minimum, usually equals one score's), then each element's list entry
// (ndt.c's kl_divergences row: value, p, q) at its final position
template <int Q, bool kCoh>
__device__ inline void sort_final_items(const KLArgs& A, int b, const SortBuf& I, uint32_t S, uint32_t NN, int rounds,
                                        uint32_t e0) {
  const uint64_t eb = (uint64_t)b * A.ecap;
  const uint32_t E = S + NN;
  unsigned long long x[Q];
  uint32_t xs[Q], st[Q], n[Q], pos[Q];
#pragma unroll
  for (int q = 0; q < Q; q++) {
    const uint32_t e = e0 + q * kKLThreads + threadIdx.x;
    const uint32_t ec = e < E ? e : 0u;
    x[q] = I.k[ec];
    xs[q] = I.s[ec];
    st[q] = e < S ? S : 0u;
    n[q] = e >= E ? 0u : e < S ? NN : S;
  }
  // the entry's value and neighbour depend on the slot only: loaded under the search
  double ov[Q];
  uint32_t oq[Q];
#pragma unroll
  for (int q = 0; q < Q; q++) {
    ov[q] = kCoh ? ld_sc1_f64(&A.slot_val_all[eb + xs[q]]) : A.slot_val_all[eb + xs[q]];
    oq[q] = (uint32_t)A.nb_all[6 * (uint64_t)b * A.ndcap + xs[q]];
  }
  run_count_q<Q>(I.k, st, n, x, rounds, pos);
#pragma unroll
  for (int q = 0; q < Q; q++)
    while (pos[q] < n[q] && I.k[st[q] + pos[q]] == x[q] && I.s[st[q] + pos[q]] < xs[q]) pos[q]++;
#pragma unroll
  for (int q = 0; q < Q; q++) {
    const uint32_t e = e0 + q * kKLThreads + threadIdx.x;
    pos[q] += e < S ? e : e - S;
  }
#pragma unroll
  for (int q = 0; q < Q; q++) {
    if (e0 + q * kKLThreads + threadIdx.x < E) {
      A.ord_val_all[eb + pos[q]] = ov[q];
      A.ord_p_all[eb + pos[q]] = xs[q] / 6;
      A.ord_q_all[eb + pos[q]] = oq[q];
    }
  }
}

// count elements in passes of up to 5 per thread, f(integral_constant<Q>, e0)
// covering e0 + q * 1024 + tid, q < Q.  Q is per wave: the items none of a
// wave's lanes holds are not searched (count = 2360: waves 5-15 run two items,
// not three), a wave-uniform branch (no barrier inside f).
template <typename F>
__device__ inline void for_items(uint32_t count, F&& f) {
  const uint32_t wb = threadIdx.x & ~63u;
  uint32_t nq = (count + kKLThreads - 1) / kKLThreads, e0 = 0;
  while (nq) {
    const uint32_t q = nq < 6 ? nq : 4;
    uint32_t qw = count > e0 + wb ? (count - e0 - wb + kKLThreads - 1) / kKLThreads : 0u;
    qw = qw < q ? qw : q;
    switch (qw) {
      case 0: break;
      case 1: f(std::integral_constant<int, 1>{}, e0); break;
      case 2: f(std::integral_constant<int, 2>{}, e0); break;
      case 3: f(std::integral_constant<int, 3>{}, e0); break;
      case 4: f(std::integral_constant<int, 4>{}, e0); break;
      default: f(std::integral_constant<int, 5>{}, e0); break;
    }
    e0 += q * kKLThreads;
    nq -= q;
  }
}

// kCoh: the chunks' runs were stored in this launch by workgroups on other
// XCDs (write-through, k_kl_rank_sort): read them with sc1 loads.
template <bool kCoh>
__device__ void sort_cloud(const KLArgs& A, const int b) {
  const CloudCtl& c = A.ctl[b];
  const uint32_t nch = (6 * c.num_nds + kChunk - 1) / kChunk;
  if (nch == 0) return;  // no slots, no list (uniform: before any barrier)
  const uint64_t eb = (uint64_t)b * A.ecap, kb = (uint64_t)b * A.sortcap, cb = (uint64_t)b * A.nchunk;
  const uint32_t tid = threadIdx.x;
  if (A.marks && tid == 0) A.marks[(uint64_t)b * kKLMarks + 12] = __builtin_amdgcn_s_memrealtime();
  extern __shared__ __attribute__((aligned(16))) unsigned long long dyn_sort[];
  const uint32_t ec = A.ecap;
  SortBuf B0{dyn_sort, reinterpret_cast<uint16_t*>(dyn_sort + 2 * ec)};
  SortBuf B1{dyn_sort + ec, reinterpret_cast<uint16_t*>(dyn_sort + 2 * ec) + ec};
  __shared__ uint32_t s_soff[kSortMaxChunks + 1], s_noff[kSortMaxChunks + 1], s_cnt[kSortMaxChunks];
  __shared__ double s_pm[kSortMaxChunks];
  __shared__ uint32_t s_maxrun[8];
  // every slot of the chunks' runs and NaN lists loaded in one round (the
  // counts arrive with them), placed once the offsets are known
  constexpr int U = (kSortMaxChunks * kChunk / 2 + kKLThreads - 1) / kKLThreads;  // 7680 slots at most: 8 rounds
  const uint32_t nslot = nch * kChunk;
  unsigned long long key[U];
  uint32_t sidx[U], nsl[U];
  double emin[U];
  uint32_t cc = 0;
  double cm = __builtin_inf();
  if (tid < nch) {
    cc = kCoh ? ld_sc1(&A.chunk_cnt[cb + tid]) : A.chunk_cnt[cb + tid];
    cm = kCoh ? ld_sc1_f64(&A.chunk_min[cb + tid]) : A.chunk_min[cb + tid];
  }
#pragma unroll
  for (int u = 0; u < U; u++) {
    const uint32_t i = u * kKLThreads + tid;
    const uint32_t ie = i < ec ? i : ec - 1;
    if (i < nslot) {
      if (kCoh) {
        key[u] = __hip_atomic_load(&A.sort_key_all[kb + i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        sidx[u] = ld_sc1(&A.sort_idx_all[kb + i]);
        nsl[u] = ld_sc1(&A.nan_list_all[eb + ie]);
        emin[u] = ld_sc1_f64(&A.ev_min_all[eb + ie]);
      } else {
        key[u] = A.sort_key_all[kb + i];
        sidx[u] = A.sort_idx_all[kb + i];
        nsl[u] = A.nan_list_all[eb + ie];
        emin[u] = A.ev_min_all[eb + ie];
      }
    }
  }
  if (tid < 64) {  // score and NaN offsets, the min over earlier chunks (nch <= 64)
    uint32_t nn = cc;  // (scores << 16) | NaNs, both < 2^16
    double m = cm;
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t o = __shfl_up(nn, off, 64);
      const double om = __shfl_up(m, off, 64);
      if ((int)tid >= off) {
        nn += o;
        m = MinF64()(m, om);
      }
    }
    uint32_t ex = __shfl_up(nn, 1, 64);
    double exm = __shfl_up(m, 1, 64);
    if (tid == 0) {
      ex = 0;
      exm = __builtin_inf();
    }
    if (tid < nch) {
      s_soff[tid] = ex >> 16;
      s_noff[tid] = ex & 0xffffu;
      s_pm[tid] = exm;
      s_cnt[tid] = cc;
    }
    if (tid + 1 == nch) {
      s_soff[nch] = nn >> 16;
      s_noff[nch] = nn & 0xffffu;
    }
    if (tid < 8) s_maxrun[tid] = 0;
  }
  __syncthreads();
  const uint32_t S = s_soff[nch], NN = s_noff[nch];
  // each level's probe count from its longest run (not the 256 << l a run may
  // hold): thread 64 l + g measures group g of level l (2^l chunks), read
  // after the placement's barrier
  if (tid < 7 * 64) {
    const uint32_t l = tid / 64, g = tid % 64, c0 = g << l;
    if (c0 < nch) {
      const uint32_t c1 = c0 + (1u << l) < nch ? c0 + (1u << l) : nch;
      atomicMax(&s_maxrun[l], s_soff[c1] - s_soff[c0]);
    }
  }
#pragma unroll
  for (int u = 0; u < U; u++) {
    const uint32_t i = u * kKLThreads + tid;
    if (i < nslot) {
      const uint32_t ch = i / kChunk, r = i % kChunk, cn = s_cnt[ch];
      if (r < (cn >> 16)) {
        const uint32_t o = s_soff[ch] + r;
        B0.k[o] = key[u];
        B0.s[o] = (uint16_t)sidx[u];
      }
      if (r < (cn & 0xffffu)) {  // the NaN run sits after the scores in both buffers
        const uint32_t o = S + s_noff[ch] + r;
        const unsigned long long nk = score_key(MinF64()(s_pm[ch], emin[u]));
        B0.k[o] = B1.k[o] = nk;
        B0.s[o] = B1.s[o] = (uint16_t)nsl[u];
      }
    }
  }
  __syncthreads();
  if (A.marks && tid == 0) A.marks[(uint64_t)b * kKLMarks + 16] = __builtin_amdgcn_s_memrealtime();
  SortBuf I = B0, O = B1;
  for (uint32_t l = 0; (1u << l) < nch; l++) {
    const int rounds = bit_len(s_maxrun[l < 7 ? l : 6]);
    for_items(S, [&](auto qc, uint32_t e0) {
      sort_level_items<decltype(qc)::value>(I, O, s_soff, nch, l, S, rounds, e0);
    });
    if (A.marks && tid == 0 && l < 6) A.marks[(uint64_t)b * kKLMarks + 20 + 2 * l] = __builtin_amdgcn_s_memrealtime();
    __syncthreads();
    if (A.marks && tid == 0 && l < 6) A.marks[(uint64_t)b * kKLMarks + 21 + 2 * l] = __builtin_amdgcn_s_memrealtime();
    const SortBuf t = I;
    I = O;
    O = t;
  }
  if (A.marks && tid == 0) A.marks[(uint64_t)b * kKLMarks + 17] = __builtin_amdgcn_s_memrealtime();
  const int rounds = bit_len(S > NN ? S : NN);
  for_items(S + NN, [&](auto qc, uint32_t e0) { sort_final_items<decltype(qc)::value, kCoh>(A, b, I, S, NN, rounds, e0); });
  if (A.marks && tid == 0) {
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    A.marks[(uint64_t)b * kKLMarks + 13] = t1;
    A.marks[(uint64_t)b * kKLMarks + 14] = t1;
    A.marks[(uint64_t)b * kKLMarks + 19] = t1;
  }
}

// One workgroup per cloud: the list sort, then (tail) the prune and the rows
// on the same workgroup (kl_cloud; the list entries are this workgroup's own
// stores, drained before the barrier).
__global__ void __launch_bounds__(kKLThreads) k_kl_sort(KLArgs A, int tail) {
  const int b = blockIdx.x;
  const CloudCtl& c = A.ctl[b];
  if (c.state == kAccepted && !kl_list_skipped(A, c)) sort_cloud<false>(A, b);
  if (!tail) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  kl_cloud<true>(A, b);
}

// Exclusive scan over each 256-thread quarter (four waves) of the workgroup;
// scratch: 16 T; total: the quarter's reduction.  (min / integer add: the
// same values as block_scan_items over a 256-thread block.)
template <typename T, typename Op>
__device__ inline T quarter_excl_scan(T v, T identity, Op op, T* scratch, T& total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, w0 = wid & ~3;
  const T incl = wave_incl_scan(v, op);
  T excl_w = __shfl_up(incl, 1, 64);
  if (lane == 0) excl_w = identity;
  if (lane == 63) scratch[wid] = incl;
  __syncthreads();
  T pre = identity;
  for (int w = w0; w < wid; w++) pre = op(pre, scratch[w]);
  total = op(op(op(scratch[w0], scratch[w0 + 1]), scratch[w0 + 2]), scratch[w0 + 3]);
  __syncthreads();
  return op(pre, excl_w);
}

// Round 6: k_kl_rank_chunks and k_kl_sort in one launch.  Four chunks per
// 1024-thread workgroup, each quarter ranking one chunk exactly as
// k_kl_rank_chunks does (its scans per quarter, its LDS in the dynamic
// region the sort reuses), the outputs the sort reads stored write-through;
// the cloud's last workgroup to finish (a ticket, as k_kl_merge's tail) then
// sorts the list (sort_cloud, sc1 loads) and, with kTail, prunes and writes
// the rows (kl_cloud).  The rank -> sort kernel boundary (~6 us at C2-L)
// becomes an atomic hand-over (3.6 us: the write-through stores' drain), but
// the ranks run 3.7 us longer on 112 one-per-CU workgroups than on 432
// small ones (the events' FP64 scores on fewer CUs): 51 against 50 us for
// the stage on L clouds (profiles/r06z_list_sort_ab.txt), so it is the
// ndnet_ndt_debug_set_list_sort form 3, not a default.
template <bool kTail>
__global__ void __launch_bounds__(kKLThreads) k_kl_rank_sort(KLArgs A) {
  if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x < 8) A.wq_ctr[16 * threadIdx.x] = 0u;  // k_welford_q has finished
  const int b = blockIdx.y;
  CloudCtl& c = A.ctl[b];
  const uint32_t tid = threadIdx.x, qtr = tid / kChunk, t = tid % kChunk;
  const uint32_t nslots = 6 * c.num_nds;
  const uint32_t ch = blockIdx.x * 4 + qtr;
  // this launch scores the cloud (a build: its deferred clouds only), this quarter a chunk of it
  const bool part = c.state == kAccepted && (A.mode != kKLBuild || c.kl_deferred);
  const bool live = part && ch * kChunk < nslots;
  const uint64_t eb = (uint64_t)b * A.ecap, kb = (uint64_t)b * A.sortcap + (uint64_t)ch * kChunk;
  const uint32_t sl = ch * kChunk + t;
  const bool deferred = kl_list_deferrable(A, c);
  extern __shared__ __attribute__((aligned(16))) unsigned long long dyn_rank[];
  unsigned long long* s_key = dyn_rank + qtr * kChunk;
  unsigned long long* s_nkey = dyn_rank + 4 * kChunk + qtr * (kChunk + 4);  // 16-byte aligned rows
  __shared__ double s_f64[16];
  __shared__ uint32_t s_u32[16];
  if (A.marks && ch == 0 && t == 0) A.marks[(uint64_t)b * kKLMarks + 3] = __builtin_amdgcn_s_memrealtime();
  uint32_t fl = 0;
  double vl = 0.0;
  if (live) {
    if (deferred) fl = kl_event_flag(A, b, sl < nslots ? sl : 0u);
    else kl_event(A, b, sl < nslots ? sl : 0u, true, fl, vl);  // the clamped slot's result is dropped
  }
  if (deferred) {  // count the cloud's events (stats num_events / num_kl), one atomic per wave
    const unsigned long long bal = __ballot(live && sl < nslots && fl);
    if ((t & 63) == 0 && bal)
      __hip_atomic_fetch_add(&c.flag_count, (uint32_t)__popcll(bal), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else {
    if (A.marks && ch == 0 && t == 0) A.marks[(uint64_t)b * kKLMarks + 4] = __builtin_amdgcn_s_memrealtime();
    if (live && sl < nslots) {
      A.slot_flag_all[eb + sl] = fl;
      st_sc1_f64(&A.slot_val_all[eb + sl], vl);
    }
    const bool f = live && sl < nslots && fl;
    const double v = f ? vl : 0.0;
    const bool isn = f && v != v;
    const bool num = f && !isn;
    const unsigned long long key = num ? score_key(v) : ~0ull;
    s_key[t] = key;
    double mtot;
    uint32_t ctot;
    const double pm = quarter_excl_scan(num ? v : __builtin_inf(), __builtin_inf(), MinF64(), s_f64, mtot);
    const uint32_t cnt = quarter_excl_scan((uint32_t)isn | ((uint32_t)num << 16), 0u, AddU32(), s_u32, ctot);
    const uint32_t nnum = ctot >> 16;
    if (num) s_nkey[cnt >> 16] = key;
    if (t < 2) s_nkey[nnum + t] = ~0ull;  // pad to an even count (~0 is never a score key)
    __syncthreads();
    // rank in the chunk (k_kl_rank_chunks): keys below, then equal keys at lower slots
    uint32_t lt = 0, eq = 0;
#pragma unroll 4
    for (uint32_t j = 0; j < nnum; j += 2) {
      const ulonglong2 kk = *reinterpret_cast<const ulonglong2*>(&s_nkey[j]);
      lt += (kk.x < key ? 1u : 0u) + (kk.y < key ? 1u : 0u);
      eq += (kk.x == key ? 1u : 0u) + (kk.y == key ? 1u : 0u);
    }
    uint32_t r;
    if (num) {
      r = lt;
      if (eq > 1)
        for (uint32_t j = 0; j < t; j++) r += s_key[j] == key ? 1u : 0u;
    } else {
      r = nnum + (t - (cnt >> 16));
    }
    if (live) {
      __hip_atomic_store(&A.sort_key_all[kb + r], key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      st_sc1(&A.sort_idx_all[kb + r], sl);
      if (isn) {
        const uint32_t j = cnt & 0xffffu;
        st_sc1(&A.nan_list_all[eb + ch * kChunk + j], sl);
        st_sc1_f64(&A.ev_min_all[eb + ch * kChunk + j], pm);
      }
      if (t == 0) {
        st_sc1(&A.chunk_cnt[(uint64_t)b * A.nchunk + ch], ctot);
        st_sc1_f64(&A.chunk_min[(uint64_t)b * A.nchunk + ch], mtot);
      }
    }
    if (A.marks && ch == 0 && t == 0) A.marks[(uint64_t)b * kKLMarks + 15] = __builtin_amdgcn_s_memrealtime();
  }
  if (A.marks && t == 0 && live)
    __hip_atomic_fetch_max(&A.marks[(uint64_t)b * kKLMarks + 18], (unsigned long long)__builtin_amdgcn_s_memrealtime(),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // the cloud's last workgroup sorts (and prunes)
  __shared__ uint32_t s_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's write-through stores are done
  __syncthreads();
  if (tid == 0)
    s_last = __hip_atomic_fetch_add(&c.kl_arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  __syncthreads();
  if (!s_last) return;
  if (tid == 0) __hip_atomic_store(&c.kl_arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (part && !kl_list_skipped(A, c)) sort_cloud<true>(A, b);
  if constexpr (kTail) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    kl_cloud<true>(A, b);
  }
}

__global__ void __launch_bounds__(kKLThreads) k_prune(KLArgs A) {
  const int b = blockIdx.x;
  CloudCtl& c = A.ctl[b];
  __shared__ uint32_t s_u32[16];
  if (c.state != kAccepted) {
    zero_outputs(A, b, A.k);
    pad_class_rows(A, b, A.k, 0);
    if (threadIdx.x == 0) write_stats(A, b);
    return;
  }
  const uint32_t nout = A.kl_lds ? prune_and_emit<true>(A, b, A.k, s_u32, s_u32)
                                 : prune_and_emit<false>(A, b, A.k, s_u32, s_u32);
  fill_tail(A, b, A.k, nout < A.k ? nout : (uint32_t)A.k);
  __syncthreads();
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

static std::mutex g_lane_mu;
static void front_lanes_forget(Plan* P);

static void plan_free(Plan* P) {
  if (!P) return;
  if (P->ev_created)
    for (int i = 0; i < 7; i++) (void)hipEventDestroy(P->ev[i]);
  if (P->kl_marks) (void)hipFree(P->kl_marks);
  if (P->wq_marks) (void)hipFree(P->wq_marks);
  if (P->fmarks) (void)hipFree(P->fmarks);
  if (P->sync_fail_h) (void)hipHostFree(P->sync_fail_h);
  if (P->front_ev) {
    (void)hipEventSynchronize(P->front_ev);
    std::lock_guard<std::mutex> lk(g_lane_mu);
    front_lanes_forget(P);  // the event goes back to the device's pool, not destroyed (graphs may wait on it)
  }
  void* bufs[]= {P->flims, P->frec, P->fwgcnt, P->fbar, P->ctl, P->stamps, P->dense_of, P->vox, P->gbits, P->pkeys, P->did, P->bin_cnt, P->nd_base,
                  P->nd_pts, P->nd_lbl, P->nd_n,
                  P->nd_mean, P->nd_cov, P->nd_cov_post, P->nd_cls, P->hist, P->nb, P->keys, P->nkeys,
                  P->chain, P->chain_ps, P->chain_ok, P->slot_val, P->slot_flag, P->ev_val, P->ev_p, P->ev_q, P->ev_min,
                  P->sort_key, P->sort_idx, P->nan_list, P->nan_key, P->nan_slot, P->chunk_nanbase, P->ord_val, P->ord_p, P->ord_q,
                  P->first_occ, P->tmp_u32, P->alive, P->d_stats, P->chunk_cnt, P->chunk_min, P->wq_ctr,
                  P->heavy, P->rtab, P->lu_done};
  for (void* b : bufs)
    if (b) (void)hipFree(b);
  delete P;
}

constexpr int kKLLdsMax = 150 * 1024;
// dynamic LDS of k_kl / k_prune's LDS-resident prune (prune_and_emit<true>)
static size_t kl_lds_bytes(const Plan* P) {
  return 4 * ((size_t)P->ndcap + 2 * (size_t)P->ecap) + ((P->ndcap + 3) & ~3u);
}

static KLArgs kl_args(Plan* P, uint64_t k, float* out, float* out_cls, double* pc64, double* cov64, uint16_t* cls16) {
  KLArgs A;
  A.marks = P->timing >= 2 ? P->kl_marks : nullptr;
  A.ctl = P->ctl;
  A.wq_ctr = P->wq_ctr;
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
  A.chain_ok_all = P->chain_ok;
  A.slot_val_all = P->slot_val;
  A.slot_flag_all = P->slot_flag;
  A.ev_val_all = P->ev_val;
  A.ev_p_all = P->ev_p;
  A.ev_q_all = P->ev_q;
  A.ev_min_all = P->ev_min;
  A.sort_key_all = P->sort_key;
  A.sort_idx_all = P->sort_idx;
  A.nan_list_all = P->nan_list;
  A.nan_key_all = P->nan_key;
  A.nan_slot_all = P->nan_slot;
  A.chunk_nanbase = P->chunk_nanbase;
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
  A.stats_out = nullptr;
  A.vcap = P->vcap;
  A.ndcap = P->ndcap;
  A.ecap = P->ecap;
  A.sortcap = P->sortcap;
  A.nchunk = P->nchunk;
  A.chunk_cnt = P->chunk_cnt;
  A.chunk_min = P->chunk_min;
  A.k = k;
  A.ncls = P->ncls;
  A.kl_lds = kl_lds_bytes(P) <= (size_t)kKLLdsMax ? 1 : 0;
  A.mode = P->eager_list ? kKLEager : kKLLazy;
  A.merge_lds_keys = 0;
  return A;
}

static size_t merge_lds_bytes(const Plan* P);

// The event sort of the clouds in A's scope (every cloud in a run, the
// deferred ones in a build).
// The LU chain states of a deferred cloud (k_welford_q stored only their
// determinant bits): from the pre-KL covariance and the chain mask, the same
// in-place lu3 sequence as k_welford_q's epilogue, one thread per ND.
__global__ void __launch_bounds__(256) k_kl_chains(KLArgs A) {
  const int b = blockIdx.y;
  const CloudCtl& c = A.ctl[b];
  if (c.state != kAccepted || !c.kl_deferred) return;
  const uint32_t u = blockIdx.x * 256 + threadIdx.x;
  if (u >= c.num_nds) return;
  const uint64_t ob = (uint64_t)b * A.ndcap;
  double S[9];
#pragma unroll
  for (int q = 0; q < 9; q++) S[q] = A.nd_cov[9 * (ob + u) + q];
  const int nT = __popc(A.nkeys_all[ob + u]);
  double* chain = A.chain_all + ob * 108 + u;
  uint32_t* ps = A.chain_ps_all + ob * 12 + u;
  for (int t = 0; t < nT; t++) {
    uint32_t perm;
    int sg;
    lu3(S, perm, sg);
#pragma unroll
    for (int q = 0; q < 9; q++) chain[(uint64_t)(9 * t + q) * A.ndcap] = S[q];
    ps[(uint64_t)t * A.ndcap] = perm | (sg < 0 ? 0x100u : 0u);
  }
}

// The dynamic LDS of the fused merge + prune launches (k_kl_merge<.., true>):
// the larger of the merge's and the LDS-resident prune's (kl_lds_bytes).
constexpr size_t kKLFusedLds = kMergeScoreChunks * kChunk * sizeof(unsigned long long);  // 144 KB
static size_t kl_lds_bytes(const Plan* P);

// Merge workgroups per cloud for chunk groups of `runs` chunks: one per group,
// or at a CU share s > 1 (a pipeline's plan) 1 / s of that, each workgroup
// taking several groups after one staging of the runs: the merge's workgroups
// hold a CU each (110 KB of LDS at C2-L) and no chain workgroup fits beside
// them, so a pipeline trades the merge's latency for its CU footprint.
// NDNET_MERGE_SHARE (A/B, read once): 1 = one workgroup per group always.
static uint32_t merge_grid(const Plan* P, uint32_t runs) {
  static const int env = [] {
    const char* e = getenv("NDNET_MERGE_SHARE");
    return e ? atoi(e) : 0;
  }();
  const uint32_t groups = (P->nchunk + runs - 1) / runs;
  const uint32_t share = env > 0 ? (uint32_t)env : (P->cu_share > 1 ? (uint32_t)P->cu_share : 1u);
  return (groups + share - 1) / share;
}

// tail: the merge's last workgroup per cloud also prunes and emits the rows
// (k_kl's work; the caller checked kl_fusable).
// k_kl_sort takes the list when its two key/slot buffers (20 bytes per slot)
// fit its LDS and its offsets one wave's scan (ecap <= 7680: k <= 1065), and
// by default only for a plan with a CU share (a pipeline's): one workgroup per
// cloud sorts in ~19 us what k_kl_merge's ~7-14 workgroups per cloud merge in
// ~17-18 us (the KL stage 49.8 vs 47.7 us on L clouds), so a plan alone on
// the chip keeps the merge, while a pipeline gains the merge's CU time (its
// 110 KB workgroups hold ~110 CUs): the L line 66.2 / 66.6k vs 65.2 / 64.8k
// clouds/s (profiles/r06z_list_sort_ab.txt)
static size_t sort_lds_bytes(const Plan* P) { return 20 * (size_t)P->ecap; }
static bool sort_fits(const Plan* P) {
  const bool want = P->list_sort == 1 || P->list_sort == 3 || (P->list_sort == 2 && P->cu_share > 1);
  return want && sort_lds_bytes(P) <= (size_t)kKLLdsMax && P->nchunk <= kSortMaxChunks && P->ecap <= 65536;
}

static void launch_list_sort(Plan* P, const KLArgs& A, hipStream_t st, bool tail = false) {
  const int B = P->B;
  if (sort_fits(P)) {
    const size_t kl = tail ? kl_lds_bytes(P) : 0, so = sort_lds_bytes(P);
    size_t dyn = so > kl ? so : kl;
    if (P->list_sort == 3) {  // one launch: the ranks, then the cloud's last workgroup sorts (and prunes)
      const size_t rk = (size_t)(8 * kChunk + 16) * sizeof(unsigned long long);
      dyn = dyn > rk ? dyn : rk;
      const dim3 grid((P->nchunk + 3) / 4, B);
      if (tail) k_kl_rank_sort<true><<<grid, kKLThreads, dyn, st>>>(A);
      else k_kl_rank_sort<false><<<grid, kKLThreads, dyn, st>>>(A);
      return;
    }
    k_kl_rank_chunks<<<dim3(P->nchunk, B), kChunk, 0, st>>>(A);
    k_kl_sort<<<B, kKLThreads, dyn, st>>>(A, tail ? 1 : 0);
    return;
  }
  k_kl_rank_chunks<<<dim3(P->nchunk, B), kChunk, 0, st>>>(A);
  const uint32_t mg = merge_grid(P, kMergeRuns);
  const size_t kl = tail ? kl_lds_bytes(P) : 0;
  auto dyn = [&](size_t m) { return m > kl ? m : kl; };
  if (P->nchunk <= (uint32_t)kMergeLdsChunks) {  // the merge computes the NaN keys itself
    if (tail) k_kl_merge<2, kMergeRuns, true><<<dim3(mg, B), kChunk * kMergeRuns, dyn(merge_lds_bytes(P)), st>>>(A);
    else k_kl_merge<2><<<dim3(mg, B), kChunk * kMergeRuns, merge_lds_bytes(P), st>>>(A);
  } else if (P->nchunk <= (uint32_t)kMergeScoreChunks) {
    k_kl_nan_keys<<<dim3(P->nchunk, B), kChunk, 0, st>>>(A);
    KLArgs A1 = A;
    const size_t keys = kMergeScoreChunks * kChunk;  // the launch's dynamic LDS, in 64-bit keys (144 KB)
    A1.merge_lds_keys = (uint32_t)keys;
    const uint32_t mg1 = merge_grid(P, kMergeRuns1);
    if (tail)
      k_kl_merge<1, kMergeRuns1, true><<<dim3(mg1, B), kChunk * kMergeRuns1, dyn(keys * sizeof(unsigned long long)),
                                          st>>>(A1);
    else
      k_kl_merge<1, kMergeRuns1><<<dim3(mg1, B), kChunk * kMergeRuns1, keys * sizeof(unsigned long long), st>>>(A1);
  } else {
    k_kl_nan_keys<<<dim3(P->nchunk, B), kChunk, 0, st>>>(A);
    if (tail) k_kl_merge<0, kMergeRuns, true><<<dim3(mg, B), kChunk * kMergeRuns, dyn(0), st>>>(A);
    else k_kl_merge<0><<<dim3(mg, B), kChunk * kMergeRuns, 0, st>>>(A);
  }
}

// The run's prune can ride on the merge launch: the prune's arrays fit the
// fused launch's LDS (the LDS-resident prune) and NDNET_KL_FUSE is not 0.
static bool kl_fusable(const Plan* P, const KLArgs& A) {
  return P->kl_fuse && A.kl_lds && kl_lds_bytes(P) <= kKLFusedLds;
}

// Builds the retained lists a lazy run deferred (no-op for the others).
static int build_deferred_lists(Plan* P, hipStream_t st) {
  if (P->eager_list || P->lists_built) return NDNET_OK;
  P->lists_built = 1;  // stream order: every later prune / dump of this run follows the build
  KLArgs A = kl_args(P, P->k, nullptr, nullptr, nullptr, nullptr, nullptr);
  A.marks = nullptr;
  A.mode = kKLBuild;
  k_kl_chains<<<dim3((P->ndcap + 255) / 256, P->B), 256, 0, st>>>(A);  // the states k_welford_q did not store
  launch_list_sort(P, A, st);
  k_kl_list_done<<<P->B, 256, 0, st>>>(A);
  HIPCHK(hipGetLastError());
  return NDNET_OK;
}

static size_t merge_lds_bytes(const Plan* P) { return 2 * (size_t)P->nchunk * kChunk * sizeof(unsigned long long); }

// ---- k_front admission: the device's front lanes ----
//
// k_front's workgroups of a cloud meet at cloud barriers, so all of them must
// be resident at once.  Two k_front grids that together want more workgroups
// than the chip holds can each get part of their workgroups resident and then
// wait on each other until the barrier timeout fails their clouds (measured:
// 640 ms per step, profiles/r04_ndt_streams_guard.txt).  The library rules that
// out itself, for any number of plans and streams, eager or captured in HIP
// graphs: the chip is split into kFrontLanes lanes of CUs / kFrontLanes; a
// plan's k_front occupies ceil(kFrontLanes * workgroups / CUs) of them (all four
// at CU share 1, two at share 2); before its launch the stream waits for the
// last k_front launched on each of its lanes, and after it the launch is
// recorded in the plan's own event, which becomes those lanes' last launch
// (explicit event graph nodes when the stream is being captured, so a replayed
// graph waits for the k_front launches before it, whatever stream they ran
// on).  A wait is left out when stream order already gives it (the lane's last
// launch came from the same stream in the same capture, or both eager), and
// lanes whose last launch shares an event are waited on once (round-5 r05e:
// four waits + four records per run cost 19 us of k_front stage).  So the
// k_front launches in flight at any time never want more workgroups than
// there are CUs, and grids on disjoint lanes (two share-2 plans: the
// pipeline's NDT streams) still run concurrently.  The other kernels never
// wait on anything, so they drain.
//
// Round 6: the admission is engaged only where it is needed.  k_front deals a
// launch's clouds cloud-major within each XCD (ndt_front.h), so a launch
// leaves at most G - 1 workgroups of one partially resident cloud waiting on
// an XCD.  While the live path-2 plans of the device together have
// sum (G - 1) < CUs per XCD (32), every XCD always keeps a CU free or a cloud
// completing, whatever the plans' launches overlap: no barrier can wait on a
// workgroup that never starts, and no admission is needed.  That covers one or
// two share-1 plans (15 + 15), and up to four share-2 plans (7 each).  Past
// the bound the lanes order the launches as above.  The bound matters: an
// event node in a replayed graph costs ~6 us (C2 alone: 151k clouds/s with
// the lanes' record and wait nodes, 171k without: profiles/r06d_lanes_ab.txt).
constexpr int kFrontLanes = 4;
constexpr int kMaxDevices = 64;
struct FrontLaneSet {
  int next;                          // the lane the next plan's lanes start at (round robin)
  int plans;                         // live plans holding a lane event on this device
  int gsum;                          // sum over them of (G - 1): their partial workgroups per XCD at most
  hipEvent_t ev[kFrontLanes];        // the event of the lane's last k_front launch (null: none yet)
  hipStream_t st[kFrontLanes];       // the stream it was launched on
  unsigned long long cap[kFrontLanes];  // the capture it was launched in (0: eager)
  std::vector<hipEvent_t> pool;      // events of freed plans, reused by later plans
};
static FrontLaneSet g_lanes[kMaxDevices];

// Drops a freed plan's event from the lanes (caller holds g_lane_mu; the
// event has completed, so nothing left to wait for).  The event itself is
// kept in the device's pool and handed to the next plan: a graph captured
// while this plan held a lane may still hold a wait node on it,
// and waiting on a pooled event only ever waits for a completed or a later
// k_front launch.
static void front_lanes_forget(Plan* P) {
  if (P->dev < 0 || P->dev >= kMaxDevices || !P->front_ev) return;
  FrontLaneSet& L = g_lanes[P->dev];
  for (int i = 0; i < kFrontLanes; i++)
    if (L.ev[i] == P->front_ev) L.ev[i] = nullptr;
  L.pool.push_back(P->front_ev);
  L.plans--;
  L.gsum -= P->lane_g;
  P->lane_g = 0;
  P->front_ev = nullptr;
}

// Assigns the plan's lanes for its current k_front geometry (caller holds g_lane_mu).
static hipError_t front_lanes_assign(Plan* P) {
  if (P->dev < 0 || P->dev >= kMaxDevices) return hipErrorInvalidDevice;
  FrontLaneSet& L = g_lanes[P->dev];
  if (!P->front_ev) {
    if (!L.pool.empty()) {
      P->front_ev = L.pool.back();
      L.pool.pop_back();
    } else {
      const hipError_t e = hipEventCreateWithFlags(&P->front_ev, hipEventDisableTiming);
      if (e != hipSuccess) return e;
    }
    L.plans++;
  }
  L.gsum -= P->lane_g;
  P->lane_g = P->fG > 1 ? (int)P->fG - 1 : 0;
  L.gsum += P->lane_g;
  const uint64_t wgs = (uint64_t)P->fG * (uint64_t)P->B;
  const int cus = P->cus > 0 ? P->cus : 1;
  int nl = (int)((wgs * kFrontLanes + (uint64_t)cus - 1) / (uint64_t)cus);
  nl = nl < 1 ? 1 : nl > kFrontLanes ? kFrontLanes : nl;
  P->nlanes = nl;
  P->lane0 = L.next;
  L.next = (L.next + nl) % kFrontLanes;
  return hipSuccess;
}

// Launches k_front between the lane waits and records (front_lanes_assign).
// A stream being captured is admitted with explicit graph nodes
// (hipGraphAddEventWaitNode / hipGraphAddEventRecordNode on the capture's
// graph, then the capture's dependencies moved past them).  The capture forms
// hipStreamWaitEvent(hipEventWaitExternal) and
// hipEventRecordWithFlags(hipEventRecordExternal) abort inside HIP on ROCm 7.2
// (std::bad_alloc; error -21: profiles/r05_capture_lane_probe.txt) and are not
// used.  NDNET_LANE_CAPTURE=0 (A/B only, read once) puts no lane nodes in a
// captured graph.
static bool lane_capture_nodes() {
  static const bool v = [] {
    const char* e = getenv("NDNET_LANE_CAPTURE");
    return !(e && e[0] == '0');
  }();
  return v;
}

// Whether the device's live plans need the admission (the bound above);
// NDNET_FRONT_ADMIT=1 (A/B, tests) engages it always.  A launch made while
// the bound held records nothing; when more plans make it fail, their
// launches and the earlier ones' last runs may overlap once: the earlier plans
// alone were within the bound, and the lanes order everything after.
static bool admit_always() {
  static const bool v = [] {
    const char* e = getenv("NDNET_FRONT_ADMIT");
    return e && e[0] == '1';
  }();
  return v;
}
static bool admission_needed(const Plan* P, const FrontLaneSet& L) {
  const int per_xcd = P->cus >= 8 ? P->cus / 8 : 1;
  return admit_always() || L.gsum >= per_xcd;
}

// Adds an event node (wait or record) after the capture's current
// dependencies and makes it the capture's only dependency.
static hipError_t capture_event_node(hipStream_t st, hipEvent_t ev, bool wait) {
  hipStreamCaptureStatus cs;
  unsigned long long id = 0;
  hipGraph_t g = nullptr;
  const hipGraphNode_t* deps = nullptr;
  size_t nd = 0;
  hipError_t e = hipStreamGetCaptureInfo_v2(st, &cs, &id, &g, &deps, &nd);
  if (e != hipSuccess) return e;
  std::vector<hipGraphNode_t> dv(deps, deps + nd);
  hipGraphNode_t node;
  e = wait ? hipGraphAddEventWaitNode(&node, g, dv.data(), dv.size(), ev)
           : hipGraphAddEventRecordNode(&node, g, dv.data(), dv.size(), ev);
  if (e != hipSuccess) return e;
  return hipStreamUpdateCaptureDependencies(st, &node, 1, hipStreamSetCaptureDependencies);
}

// NDNET_FRONT_LANES=0 (A/B only, read once): no admission at all -- the round-4
// behaviour, concurrent path-2 plans then need front_share >= N
static bool lanes_enabled() {
  static const bool v = [] {
    const char* e = getenv("NDNET_FRONT_LANES");
    return !(e && e[0] == '0');
  }();
  return v;
}

// Where a plan's k_front is recorded on its lanes: at the end of its run (the
// default: a record node between k_front and k_welford_q held the next launch
// back -- the isolated C2 k_front stage 51 -> 55 us, profiles/r05_lanes_ab.txt;
// at the run's end it follows the last KL launch, where the pipeline records
// its own stage event anyway), or right after k_front (NDNET_FRONT_REC_END=0,
// A/B).  A later k_front on those lanes then waits for the whole run instead
// of its k_front only: stricter, and still one chip's worth at a time.
static bool rec_at_end() {
  static const bool v = [] {
    const char* e = getenv("NDNET_FRONT_REC_END");
    return !(e && e[0] == '0');
  }();
  return v;
}

// Records the plan's last k_front launch on its lanes (caller holds g_lane_mu).
static int front_lanes_record(Plan* P, hipStream_t st) {
  FrontLaneSet& L = g_lanes[P->dev];
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  unsigned long long cap_id = 0;
  HIPCHK(hipStreamGetCaptureInfo(st, &cs, &cap_id));
  const bool cap = cs == hipStreamCaptureStatusActive;
  if (!cap) cap_id = 0;
  if (cap && !lane_capture_nodes()) return NDNET_OK;  // the lanes keep their last launch
  if (!cap) HIPCHK(hipEventRecord(P->front_ev, st));
  else HIPCHK(capture_event_node(st, P->front_ev, false));
  for (int i = 0; i < P->nlanes; i++) {
    const int l = (P->lane0 + i) % kFrontLanes;
    L.ev[l] = P->front_ev;
    L.st[l] = st;
    L.cap[l] = cap_id;
  }
  return NDNET_OK;
}

// The record a run deferred to its end (rec_at_end): after its last launch.
static int front_lanes_finish(Plan* P, hipStream_t st) {
  if (!P->lane_rec) return NDNET_OK;
  P->lane_rec = 0;
  std::lock_guard<std::mutex> lk(g_lane_mu);
  return front_lanes_record(P, st);
}

template <typename T>
static int front_launch(Plan* P, hipStream_t st, const T* pts, const FrontArgs& F) {
  P->lane_rec = 0;
  if (!lanes_enabled()) {
    k_front<T><<<P->fG * P->B, kFrontThreads, P->flds, st>>>(pts, F);
    HIPCHK(hipGetLastError());
    return NDNET_OK;
  }
  std::lock_guard<std::mutex> lk(g_lane_mu);  // waits and launch in one host order
  FrontLaneSet& L = g_lanes[P->dev];
  if (!admission_needed(P, L)) {
    k_front<T><<<P->fG * P->B, kFrontThreads, P->flds, st>>>(pts, F);
    HIPCHK(hipGetLastError());
    return NDNET_OK;
  }
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  unsigned long long cap_id = 0;
  HIPCHK(hipStreamGetCaptureInfo(st, &cs, &cap_id));
  const bool cap = cs == hipStreamCaptureStatusActive;
  if (!cap) cap_id = 0;
  const bool nodes = !cap || lane_capture_nodes();
  hipEvent_t waited[kFrontLanes];
  int nw = 0;
  for (int i = 0; i < P->nlanes; i++) {
    const int l = (P->lane0 + i) % kFrontLanes;
    hipEvent_t ev = L.ev[l];
    if (!ev || (L.st[l] == st && L.cap[l] == cap_id)) continue;  // nothing yet / stream order covers it
    bool dup = false;
    for (int j = 0; j < nw; j++) dup |= waited[j] == ev;
    if (dup) continue;
    waited[nw++] = ev;
    if (!cap) HIPCHK(hipStreamWaitEvent(st, ev, 0));
    else if (nodes) HIPCHK(capture_event_node(st, ev, true));
  }
  k_front<T><<<P->fG * P->B, kFrontThreads, P->flds, st>>>(pts, F);
  HIPCHK(hipGetLastError());
  if (rec_at_end()) {
    P->lane_rec = 1;
    return NDNET_OK;
  }
  return front_lanes_record(P, st);
}

// k_welford_q's class-histogram LDS of a labelled run (0: the global histograms)
static size_t wq_hist_lds(const Plan* P, bool l64) {
  if (P->ncls < 0) return 0;
  const size_t hb = (size_t)wq_hist_nds(l64) * (size_t)(P->ncls + 1) * sizeof(uint32_t);
  return hb <= (size_t)kWqHistMax ? hb : 0;
}

// The light form for the plan's CU share (Plan::wq_form; ndnet_ndt_set_welford_form)
static void wq_pick_form(Plan* P) { P->wq_l64 = P->wq_form == 1 ? 1 : P->wq_form == 2 ? 0 : (P->cu_share > 1); }

template <typename T>
static int run_impl(Plan* P, hipStream_t st, const T* pts, const int32_t* lbl, float* out, float* out_cls,
                    double* pc64, double* cov64, uint16_t* cls16, ndnet_ndt_stats* stats_dst) {
  const int B = P->B;
  const uint64_t n = P->n;
  if (lbl && P->ncls < 0) return NDNET_ERR_ARG;
  if (P->run_part == 2) goto welford;  // the front ran in an earlier call on this stream order
  if (P->timing) HIPCHK(hipEventRecord(P->ev[0], st));
  P->lists_built = 0;
  // k_front re-arms its clouds itself (epoch, barrier words, list counters)
  if (!P->front) k_reset<<<(B + 63) / 64, 64, 0, st>>>(P->ctl, B, nullptr, P->lu_done, (P->ndcap + 63) / 64);
  P->calls++;
  if (P->front) {
    FrontArgs F;
    F.ctl = P->ctl;
    F.lbl = lbl;
    F.stamps = P->stamps;
    F.gbits = P->gbits;
    F.dense_of = P->dense_of;
    F.vox = P->vox;
    F.nd_n = P->nd_n;
    F.nd_base = P->nd_base;
    F.heavy = P->heavy;
    F.heavy_t = P->heavy_t;
    F.nd_pts = P->nd_pts;
    F.nd_lbl = lbl ? P->nd_lbl : nullptr;
    F.lims = P->flims;
    F.rec = P->frec;
    F.wgcnt = P->fwgcnt;
    F.bar = P->fbar;
    F.marks = P->timing >= 2 ? P->fmarks : nullptr;
    F.n = n;
    F.k = P->k;
    F.vcap = P->vcap;
    F.ndcap = P->ndcap;
    F.G = P->fG;
    F.bpw = P->fbpw;
    F.rbs = P->frbs;
#ifndef NDNET_FRONT_STORE
#define NDNET_FRONT_STORE 0
#endif
    F.dbg_store = NDNET_FRONT_STORE;  // binning scatter stores: 0 plain, 1 nontemporal, 2 agent-scope atomic (A/B)
    // staged scatter (float input): every point held in registers, delta[ndcap]
    // in the table region, a 16-byte LDS record per point of the workgroup
    F.staged = P->front_staged && F.dbg_store == 0 && sizeof(T) == 4 && P->fbpw <= (uint32_t)kFrontR &&
               2 * P->ndcap <= (uint32_t)kFrontTable && (size_t)16 * 1024 * P->fbpw <= P->flds;
    F.eval_all = P->exact_counts;
    F.B = (uint32_t)B;
    F.nbins = P->nbins;
    F.xcd_local = (B % 8) == 0 ? 1 : 0;
    F.sync_ticks = P->front_sync_ticks;
    F.lu_done = P->lu_done;
    F.lu_gcap = (P->ndcap + 63) / 64;
    F.sync_fail = P->sync_fail_d;
    const int frc = front_launch<T>(P, st, pts, F);
    if (frc != NDNET_OK) return frc;
    if (P->timing)
      for (int e = 1; e <= 4; e++) HIPCHK(hipEventRecord(P->ev[e], st));
  } else {
  const uint32_t Gl = (uint32_t)((3 * n + 256 * kLimPPT - 1) / (256 * kLimPPT));
  k_limits<T><<<dim3(Gl, B), 256, 0, st>>>(pts, P->ctl, P->gbits, P->stamps, n, Gl, P->vcap);
  if (P->timing) HIPCHK(hipEventRecord(P->ev[1], st));
  for (int it = 0; it < kMaxIters; it++)
    k_search_pass<T><<<dim3(P->G, B), kPassThreads, 0, st>>>(pts, P->ctl, P->stamps, P->gbits, P->pkeys, n, P->k,
                                                              P->G, P->vcap);
  if (P->timing) HIPCHK(hipEventRecord(P->ev[2], st));
  k_dense<<<B, 1024, 0, st>>>(P->ctl, P->stamps, P->gbits, P->dense_of, P->vox, P->vcap, P->ndcap);
  if (P->timing) HIPCHK(hipEventRecord(P->ev[3], st));
  k_bin_count<<<dim3(P->nbins, B), kBinThreads, P->ndcap * sizeof(uint32_t), st>>>(
      P->ctl, P->pkeys, P->dense_of, P->did, P->bin_cnt, n, P->vcap, P->ndcap, P->nbins);
  k_bin_offsets<<<B, 1024, 0, st>>>(P->ctl, P->bin_cnt, P->nd_n, P->nd_base, P->heavy, P->heavy_t, P->ndcap,
                                     P->nbins);
  k_bin_scatter<T><<<dim3(P->nbins, B), kBinThreads, 0, st>>>(pts, lbl, P->ctl, P->did, P->bin_cnt,
                                                               (T*)P->nd_pts, lbl ? P->nd_lbl : nullptr, n,
                                                               P->ndcap, P->nbins);
  if (P->timing) HIPCHK(hipEventRecord(P->ev[4], st));
  }
  if (P->run_part == 1) {
    HIPCHK(hipGetLastError());
    return front_lanes_finish(P, st);
  }
welford:
  P->lists_built = 0;
  auto wq = [&](auto l64_tag) {
    constexpr bool L64 = decltype(l64_tag)::value;
    k_welford_q<T, L64><<<P->wq_grid, kWqThreads,
                      wq_rt_entries(P->heavy_t) * wq_rt_bytes(L64) + 8 * ((B + 1 + 3) & ~3) + (lbl ? wq_hist_lds(P, L64) : 0),
                      st>>>(
        P->ctl, B, (const T*)P->nd_pts, lbl ? P->nd_lbl : nullptr, P->nd_n, P->nd_base, P->nd_mean, P->nd_cov,
        P->nd_cls, P->hist, P->ncls, n, P->ndcap, P->wq_ctr, P->heavy, P->heavy_t, (const double2*)P->rtab,
        P->timing >= 2 ? P->wq_marks : nullptr,
        WqChainArgs{P->vox, P->dense_of, P->nb, P->nkeys, P->nd_cov, P->chain, P->chain_ps, P->nd_cov_post, P->vcap,
                    P->eager_list ? 0ull : (uint64_t)P->k, P->chain_ok, P->lu_done});
  };
  if (P->wq_l64) wq(std::true_type{});
  else wq(std::false_type{});
  if (P->timing) HIPCHK(hipEventRecord(P->ev[5], st));
  KLArgs A = kl_args(P, P->k, out, out_cls, pc64, cov64, cls16);
  A.stats_out = stats_dst;
  if (kl_fusable(P, A)) {
    launch_list_sort(P, A, st, true);
  } else {
    launch_list_sort(P, A, st);
    k_kl<<<B, kKLThreads, A.kl_lds ? kl_lds_bytes(P) : 0, st>>>(A);
  }
  if (P->timing) HIPCHK(hipEventRecord(P->ev[6], st));
  HIPCHK(hipGetLastError());
  return front_lanes_finish(P, st);
}

__global__ void k_set_epoch(CloudCtl* ctl, int B, uint32_t epoch) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b < B) ctl[b].epoch = epoch;
}

}  // namespace

// ------------------------------------------------------------------ C ABI

extern "C" {

}  // extern "C" (reopened below)

namespace {

// k_front's geometry for a CU share: G = CUs / (share * B) workgroups per
// cloud (at most the plan's bins), bpw bins per workgroup, rank-bin size and
// dynamic LDS; front_ok when the shape fits (LDS, residency).  At share 1
// every CU runs a k_front workgroup (B = 16: G = 16); a larger share leaves
// CUs to work on another stream (PipelinedSegmentation) at the cost of more
// bins per workgroup.
hipError_t front_config(Plan* P, int share) {
  const uint32_t B = (uint32_t)P->B;
  const int cus = P->cus;
  const uint32_t gt = (uint32_t)(cus / (share * (int)B) > 0 ? cus / (share * (int)B) : 1);
  const uint32_t G = gt < P->nbins ? gt : P->nbins;
  const uint32_t bpw = (P->nbins + G - 1) / G;
  // rank bins of 512 points when that keeps every wave busy and fits
  auto lds_of = [&](uint32_t rbs) {  // table + binfo (u32) + the rank-bin ND histograms (u16)
    return sizeof(uint32_t) * ((size_t)kFrontTable + (size_t)bpw * 1024) +
           ((sizeof(uint16_t) * (size_t)bpw * (1024 / rbs) * P->ndcap + 3) & ~(size_t)3);
  };
  const uint32_t rbs = (2 * bpw <= (uint32_t)kFrontWaves && lds_of(512) <= 150 * 1024) ? 512u : 1024u;
  size_t lds = lds_of(rbs);
  // the staged scatter's records (16 bytes per point of the workgroup, over
  // the whole dynamic LDS): reserved when they fit, else the direct scatter
  // runs.  (Round 3's u16 histograms shrank lds_of below the records' need at
  // B = 16, k = 1000, silently turning the staged scatter off: k_front's
  // WRITE_SIZE 20.6 -> 39.5 MB, profiles/r04_pmc_summary.txt.)
  const size_t staged_lds = (size_t)16 * 1024 * bpw;
  if (bpw <= (uint32_t)kFrontR && staged_lds > lds && staged_lds <= 150 * 1024) lds = staged_lds;
  hipError_t e = hipSuccess;
  // (addv, the per-ND base words of the binning, live in the table region)
  int ok = lds <= 150 * 1024 && (G == 1 || (uint64_t)G * B <= (uint64_t)cus) && P->ndcap <= (uint32_t)kFrontTable;
  if (ok) e = hipFuncSetAttribute((const void*)k_front<float>, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
  if (ok && e == hipSuccess)
    e = hipFuncSetAttribute((const void*)k_front<double>, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
  if (ok && e == hipSuccess) {
    int nb = 0;
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_front<double>, kFrontThreads, lds);
    if (e == hipSuccess && nb < 1) ok = 0;
  }
  P->fG = G;
  P->fbpw = bpw;
  P->frbs = rbs;
  P->flds = lds;
  P->front_ok = e == hipSuccess && ok;
  P->cu_share = share;
  wq_pick_form(P);
  if (e == hipSuccess && P->front_ok) {
    std::lock_guard<std::mutex> lk(g_lane_mu);
    e = front_lanes_assign(P);
  }
  return e;
}

}  // namespace

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
  P->front_sync_ticks = 200000000ull;  // 2 s at the 100 MHz constant clock
  P->front_staged = 1;
  P->heavy_t = kWqHeavy;
  if (const char* e = getenv("NDNET_HEAVY_T")) {  // A/B of the default threshold (tools/gpu.sh ab)
    const long v = atol(e);
    if (v >= 1) P->heavy_t = (uint32_t)v;
  }
  P->kl_fuse = 1;
  if (const char* e = getenv("NDNET_KL_FUSE")) P->kl_fuse = atoi(e) != 0;  // A/B: 0 launches k_kl
  P->list_sort = 2;
  if (const char* e = getenv("NDNET_KL_SORT")) P->list_sort = atoi(e);  // A/B: 0 k_kl_merge, 1 k_kl_sort wherever it fits
  if (const char* e = getenv("NDNET_WQ_FORM"))  // A/B: "light64" / "quad" for every plan (default: by CU share)
    P->wq_form = !strcmp(e, "light64") ? 1 : !strcmp(e, "quad") ? 2 : 0;
  const double upper = (double)num_desired * (1 + 0.2);
  P->ndcap = (uint32_t)upper + 1;
  P->ecap = 6 * P->ndcap;
  P->nchunk = (P->ecap + kChunk - 1) / kChunk;
  P->sortcap = P->nchunk * kChunk;
  P->nbins = (uint32_t)((num_points + kBinPts - 1) / kBinPts);
  const uint64_t n8 = (num_points / kWorkers) * kWorkers;
  P->G = (uint32_t)((n8 + kPassPts - 1) / kPassPts);
  if (P->G == 0) P->G = 1;
  if (P->ndcap > 16384) {  // per-chunk ND histograms live in LDS (k_bin_count)
    delete P;
    return NDNET_ERR_ARG;
  }
  const size_t B = (size_t)batch, nd = P->ndcap, ec = P->ecap, nbn = P->nbins, n = num_points;
  const int nb = num_classes >= 0 ? num_classes + 1 : 1;
  hipError_t e = hipSuccess;
#define A_(ptr, cnt) \
  if (e == hipSuccess) e = alloc(&P->ptr, (cnt));
  A_(ctl, B);
  A_(stamps, B * P->vcap);
  A_(dense_of, B * P->vcap);
  A_(vox, B * nd);
  A_(gbits, B * 2 * kBitsWords);
  A_(pkeys, B * n);
  A_(did, B * n);
  A_(bin_cnt, B * nbn * nd);
  A_(nd_base, B * nd);
  if (e == hipSuccess) e = hipMalloc(&P->nd_pts, (B * n + kNdSlack) * 3 * sizeof(double));
  A_(nd_lbl, num_classes >= 0 ? B * n : 1);
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
  A_(chain_ok, B * nd);
  A_(slot_val, B * ec);
  A_(slot_flag, B * ec);
  A_(ev_val, B * ec);
  A_(ev_p, B * ec);
  A_(ev_q, B * ec);
  A_(ev_min, B * ec);
  A_(sort_key, B * P->sortcap);
  A_(sort_idx, B * P->sortcap);
  A_(nan_list, B * ec);
  A_(nan_key, B * ec);
  A_(nan_slot, B * ec);
  A_(chunk_nanbase, B * P->nchunk);
  A_(ord_val, B * ec);
  A_(ord_p, B * ec);
  A_(ord_q, B * ec);
  A_(first_occ, B * nd);
  A_(tmp_u32, B * ec);
  A_(alive, B * nd);
  A_(chunk_cnt, B * P->nchunk);
  A_(chunk_min, B * P->nchunk);
  A_(d_stats, B);
  A_(wq_ctr, 128);
  A_(heavy, B * nd);
  A_(rtab, 2 * (n + 1));
  A_(lu_done, B * ((nd + 63) / 64));
  // k_front: G workgroups per cloud, all resident together (G * B <= CUs);
  // each owns bpw bins, whose per-ND counts and ranks live in its LDS.  The
  // per-workgroup buffers are sized for the largest G (CU share 1).
  {
    int dev = 0, cus = 0;
    if (e == hipSuccess) e = hipGetDevice(&dev);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    P->cus = cus;
    P->dev = dev;
    if (e == hipSuccess) e = front_config(P, 1);
    P->front = P->front_ok;
    const uint32_t G = P->fG;
    A_(flims, B * G * 6);
    A_(frec, B * kFrontPhases * G * kRecWords);
    A_(fwgcnt, B * G * nd);
    A_(fbar, B * kBarStride);
  }
#undef A_
  if (e == hipSuccess) e = hipHostMalloc((void**)&P->sync_fail_h, sizeof(uint32_t), hipHostMallocMapped | hipHostMallocCoherent);
  if (e == hipSuccess) {
    *P->sync_fail_h = 0;
    e = hipHostGetDevicePointer((void**)&P->sync_fail_d, P->sync_fail_h, 0);
  }
  if (e == hipSuccess) e = hipMemset(P->ctl, 0, B * sizeof(CloudCtl));
  if (e == hipSuccess) e = hipMemset(P->fbar, 0, B * kBarStride * sizeof(uint32_t));
  if (e == hipSuccess) e = hipMemset(P->stamps, 0, B * P->vcap * sizeof(uint32_t));
  if (e == hipSuccess) e = hipMemset(P->d_stats, 0, B * sizeof(ndnet_ndt_stats));
  if (e == hipSuccess) e = hipMemset(P->wq_ctr, 0, 128 * sizeof(uint32_t));
  if (e == hipSuccess) e = hipMemset(P->lu_done, 0, B * ((nd + 63) / 64) * sizeof(uint32_t));
  if (e == hipSuccess) {
    // wq_heavy's division table: rc = RN(1/c), rl = RN((1 - c rc) / c), 1 - c rc exact (one fma)
    std::vector<double> rt(2 * (n + 1), 0.0);
    for (size_t c = 1; c <= n; c++) {
      const double dc = (double)c, rc = 1.0 / dc;
      rt[2 * c] = rc;
      rt[2 * c + 1] = fma(-dc, rc, 1.0) / dc;
    }
    e = hipMemcpy(P->rtab, rt.data(), rt.size() * sizeof(double), hipMemcpyHostToDevice);
  }
  {
    int dv = 0, ncu = 0;
    if (e == hipSuccess) e = hipGetDevice(&dv);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dv);
#ifndef NDNET_WQ_WPC
#define NDNET_WQ_WPC 1
#endif
    // NDNET_WQ_WPC workgroups per CU (1, 2 and 3 measured equal on C2 and C5:
    // profiles/r02c_welford_parts.txt -- the kernel is issue-bound, not
    // latency-bound, so a second wave per SIMD shares the same issue slots)
    P->wq_grid = ncu > 0 ? (uint32_t)ncu * NDNET_WQ_WPC : 1u;
  }
  {
    const int wq_dyn = (int)(kWqRt * wq_rt_bytes(true) + 8 * ((batch + 1 + 3) & ~3) + kWqHistMax);
    const void* wqk[] = {(const void*)k_welford_q<float, true>, (const void*)k_welford_q<double, true>,
                         (const void*)k_welford_q<float, false>, (const void*)k_welford_q<double, false>};
    for (const void* f : wqk)
      if (e == hipSuccess) e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, wq_dyn);
  }
  if (e == hipSuccess)
    e = hipFuncSetAttribute((const void*)k_kl_merge<2>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)(2 * kMergeLdsChunks * kChunk * sizeof(unsigned long long)));
  if (e == hipSuccess)
    e = hipFuncSetAttribute((const void*)k_kl_merge<1, kMergeRuns1>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)(kMergeScoreChunks * kChunk * sizeof(unsigned long long)));
  if (e == hipSuccess)
    e = hipFuncSetAttribute((const void*)k_kl_merge<2, kMergeRuns, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)kKLFusedLds);
  if (e == hipSuccess)
    e = hipFuncSetAttribute((const void*)k_kl_merge<1, kMergeRuns1, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)kKLFusedLds);
  if (e == hipSuccess)
    e = hipFuncSetAttribute((const void*)k_kl_merge<0, kMergeRuns, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)kKLFusedLds);
  if (e == hipSuccess) e = hipFuncSetAttribute((const void*)k_kl, hipFuncAttributeMaxDynamicSharedMemorySize, kKLLdsMax);
  if (e == hipSuccess) e = hipFuncSetAttribute((const void*)k_kl_sort, hipFuncAttributeMaxDynamicSharedMemorySize, kKLLdsMax);
  if (e == hipSuccess)
    e = hipFuncSetAttribute((const void*)k_kl_rank_sort<true>, hipFuncAttributeMaxDynamicSharedMemorySize, kKLLdsMax);
  if (e == hipSuccess)
    e = hipFuncSetAttribute((const void*)k_kl_rank_sort<false>, hipFuncAttributeMaxDynamicSharedMemorySize, kKLLdsMax);
  if (e == hipSuccess) e = hipFuncSetAttribute((const void*)k_prune, hipFuncAttributeMaxDynamicSharedMemorySize, kKLLdsMax);
  if (e == hipSuccess) e = hipFuncSetAttribute((const void*)k_bin_count, hipFuncAttributeMaxDynamicSharedMemorySize,
                                               (int)(16384 * sizeof(uint32_t)));
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

int ndnet_ndt_set_path(void* plan, int path) {
  Plan* P = (Plan*)plan;
  if (!P || path < 0 || path > 2) return NDNET_ERR_ARG;
  if (path == 2 && !P->front_ok) return NDNET_ERR_ARG;
  P->front = path == 1 ? 0 : P->front_ok;
  return NDNET_OK;
}

int ndnet_ndt_set_cu_share(void* plan, int front_share, int welford_share) {
  Plan* P = (Plan*)plan;
  if (!P || front_share < 1 || front_share > P->cus || welford_share < 1 || welford_share > P->cus)
    return NDNET_ERR_ARG;
  const int prev = P->cu_share;
  const bool on_front = P->front != 0;  // path 2 in use (not forced to path 1)
  if (front_config(P, front_share) != hipSuccess) return NDNET_ERR_HIP;
  if (!P->front_ok) {  // k_front does not fit this share: keep the previous one
    (void)front_config(P, prev);  // the previous share fitted when it was set
    return NDNET_ERR_ARG;
  }
  P->front = on_front ? 1 : 0;
  P->wq_grid = (uint32_t)(P->cus / welford_share > 0 ? P->cus / welford_share : 1) * NDNET_WQ_WPC;
  return NDNET_OK;
}

int ndnet_ndt_set_welford_form(void* plan, int form) {
  Plan* P = (Plan*)plan;
  if (!P || form < 0 || form > 2) return NDNET_ERR_ARG;
  P->wq_form = form;
  wq_pick_form(P);
  return NDNET_OK;
}

int ndnet_ndt_get_welford_form(void* plan) {
  Plan* P = (Plan*)plan;
  if (!P) return NDNET_ERR_ARG;
  return P->wq_l64 ? 1 : 2;
}

int ndnet_ndt_set_exact_counts(void* plan, int on) {
  Plan* P = (Plan*)plan;
  if (!P || on < 0 || on > 1) return NDNET_ERR_ARG;
  P->exact_counts = on;
  return NDNET_OK;
}

int ndnet_ndt_set_front_staged(void* plan, int on) {
  Plan* P = (Plan*)plan;
  if (!P || on < 0 || on > 1) return NDNET_ERR_ARG;
  P->front_staged = on;
  return NDNET_OK;
}

int ndnet_ndt_get_front_staged(void* plan) {
  const Plan* P = (const Plan*)plan;
  if (!P) return NDNET_ERR_ARG;
  return P->front_ok && P->front_staged && P->fbpw <= (uint32_t)kFrontR && 2 * P->ndcap <= (uint32_t)kFrontTable &&
                 (size_t)16 * 1024 * P->fbpw <= P->flds
             ? 1
             : 0;
}

int ndnet_ndt_set_heavy_threshold(void* plan, uint32_t min_samples) {
  Plan* P = (Plan*)plan;
  if (!P || min_samples == 0) return NDNET_ERR_ARG;
  P->heavy_t = min_samples;
  return NDNET_OK;
}

int ndnet_ndt_set_run_part(void* plan, int part) {
  Plan* P = (Plan*)plan;
  if (!P || part < 0 || part > 2) return NDNET_ERR_ARG;
  P->run_part = part;
  return NDNET_OK;
}

int ndnet_ndt_set_lazy_list(void* plan, int on) {
  Plan* P = (Plan*)plan;
  if (!P || on < 0 || on > 1) return NDNET_ERR_ARG;
  P->eager_list = on ? 0 : 1;
  return NDNET_OK;
}

int ndnet_ndt_get_path(void* plan) {
  Plan* P = (Plan*)plan;
  if (!P) return NDNET_ERR_ARG;
  return P->front ? 2 : 1;
}

int ndnet_ndt_set_timing(void* plan, int enable) {
  Plan* P = (Plan*)plan;
  if (!P) return NDNET_ERR_ARG;
  if (enable < 0 || enable > 2) return NDNET_ERR_ARG;
  if (enable && !P->ev_created) {
    for (int i = 0; i < 7; i++) HIPCHK(hipEventCreate(&P->ev[i]));
    P->ev_created = 1;
  }
  if (enable >= 2 && !P->fmarks) {
    HIPCHK(hipMalloc(&P->fmarks, (size_t)P->B * kFrontMarkStride * sizeof(unsigned long long)));
    HIPCHK(hipMemset(P->fmarks, 0, (size_t)P->B * kFrontMarkStride * sizeof(unsigned long long)));
  }
  if (enable >= 2 && !P->wq_marks) {
    const size_t items = (size_t)P->B * (P->ndcap + (P->ndcap + 15) / 16);
    HIPCHK(hipMalloc(&P->wq_marks, items * kWqMarkW * sizeof(unsigned long long)));
    HIPCHK(hipMemset(P->wq_marks, 0, items * kWqMarkW * sizeof(unsigned long long)));
  }
  if (enable >= 2 && !P->kl_marks) {
    HIPCHK(hipMalloc(&P->kl_marks, (size_t)P->B * kKLMarks * sizeof(unsigned long long)));
    HIPCHK(hipMemset(P->kl_marks, 0, (size_t)P->B * kKLMarks * sizeof(unsigned long long)));
  }
  P->timing = enable;
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
  const int rc = build_deferred_lists(P, st);
  if (rc != NDNET_OK) return rc;
  KLArgs A = kl_args(P, num_desired, d_out, d_out_classes, d_out_points, d_out_covariances, d_out_classes16);
  A.stats_out = d_stats;
  k_prune<<<P->B, kKLThreads, A.kl_lds ? kl_lds_bytes(P) : 0, st>>>(A);
  HIPCHK(hipGetLastError());
  return NDNET_OK;
}

// Stage dumps for the parity tests (host copies of one cloud's intermediates).
int ndnet_ndt_debug_kl_marks(void* plan, unsigned long long* marks) {
  Plan* P = (Plan*)plan;
  if (!P || !marks || !P->kl_marks) return NDNET_ERR_ARG;
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpy(marks, P->kl_marks, (size_t)P->B * kKLMarks * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  return NDNET_OK;
}

int ndnet_debug_lu_chain(const double* d_A, uint32_t n, int steps, double* d_states, uint32_t* d_ps,
                         uint32_t* d_flags, void* stream) {
  if (!d_A || !d_states || !d_ps || !d_flags || steps <= 0 || steps > 12) return NDNET_ERR_ARG;
  if (n == 0) return NDNET_OK;
  k_debug_lu_chain<<<(n + 63) / 64, 64, 0, (hipStream_t)stream>>>(d_A, n, steps, d_states, d_ps, d_flags);
  HIPCHK(hipGetLastError());
  return NDNET_OK;
}

int ndnet_ndt_debug_wq_marks(void* plan, unsigned long long* marks, uint32_t* items) {
  Plan* P = (Plan*)plan;
  if (!P || !marks || !items || !P->wq_marks) return NDNET_ERR_ARG;
  HIPCHK(hipDeviceSynchronize());
  const size_t cap = (size_t)P->B * (P->ndcap + (P->ndcap + 15) / 16);
  *items = (uint32_t)cap;
  HIPCHK(hipMemcpy(marks, P->wq_marks, cap * kWqMarkW * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  return NDNET_OK;
}

int ndnet_ndt_debug_front_marks(void* plan, unsigned long long* marks) {
  Plan* P = (Plan*)plan;
  if (!P || !marks || !P->fmarks) return NDNET_ERR_ARG;
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpy2D(marks, 32 * sizeof(unsigned long long), P->fmarks, kFrontMarkStride * sizeof(unsigned long long),
                     32 * sizeof(unsigned long long), P->B, hipMemcpyDeviceToHost));
  return NDNET_OK;
}

int ndnet_ndt_debug_front_wg_marks(void* plan, unsigned long long* marks, int* G) {
  Plan* P = (Plan*)plan;
  if (!P || !marks || !G || !P->fmarks) return NDNET_ERR_ARG;
  HIPCHK(hipDeviceSynchronize());
  *G = (int)P->fG;
  HIPCHK(hipMemcpy2D(marks, 2 * P->fG * sizeof(unsigned long long),
                     P->fmarks + 32, kFrontMarkStride * sizeof(unsigned long long),
                     2 * P->fG * sizeof(unsigned long long), P->B, hipMemcpyDeviceToHost));
  return NDNET_OK;
}

int ndnet_ndt_take_sync_failures(void* plan) {
  Plan* P = (Plan*)plan;
  if (!P || !P->sync_fail_h) return NDNET_ERR_ARG;
  const uint32_t v = __atomic_exchange_n(P->sync_fail_h, 0u, __ATOMIC_ACQ_REL);
  return v ? 1 : 0;
}

int ndnet_ndt_get_front_lanes(void* plan, int* lane0, int* nlanes) {
  Plan* P = (Plan*)plan;
  if (!P || !lane0 || !nlanes) return NDNET_ERR_ARG;
  std::lock_guard<std::mutex> lk(g_lane_mu);
  *lane0 = P->lane0;
  *nlanes = P->front ? P->nlanes : 0;
  return NDNET_OK;
}

int ndnet_ndt_debug_set_sync_timeout(void* plan, uint64_t ticks) {
  Plan* P = (Plan*)plan;
  if (!P) return NDNET_ERR_ARG;
  P->front_sync_ticks = ticks ? ticks : 200000000ull;
  return NDNET_OK;
}

int ndnet_ndt_debug_set_epoch(void* plan, uint32_t epoch) {
  Plan* P = (Plan*)plan;
  if (!P || epoch >= (1u << 26)) return NDNET_ERR_ARG;
  HIPCHK(hipDeviceSynchronize());
  k_set_epoch<<<(P->B + 63) / 64, 64>>>(P->ctl, P->B, epoch);
  HIPCHK(hipGetLastError());
  HIPCHK(hipDeviceSynchronize());
  return NDNET_OK;
}

int ndnet_ndt_debug_set_kl_fuse(void* plan, int on) {
  Plan* P = (Plan*)plan;
  if (!P) return NDNET_ERR_ARG;
  P->kl_fuse = on ? 1 : 0;
  return NDNET_OK;
}

int ndnet_ndt_debug_set_list_sort(void* plan, int on) {
  Plan* P = (Plan*)plan;
  if (!P) return NDNET_ERR_ARG;
  if (on < 0 || on > 3) return NDNET_ERR_ARG;
  P->list_sort = on;
  return NDNET_OK;
}

int ndnet_ndt_debug_get_list_sort(void* plan) {
  const Plan* P = (const Plan*)plan;
  if (!P) return NDNET_ERR_ARG;
  return sort_fits(P) ? 1 : 0;
}

int ndnet_ndt_debug_dump(void* plan, int cloud, uint32_t* nd_n, double* nd_mean, double* nd_cov_pre,
                         double* nd_cov_post, uint32_t* vox, double* ord_val, uint32_t* ord_p, uint32_t* ord_q,
                         double* guesses, uint32_t* counts, uint32_t* iters, uint8_t* alive) {
  Plan* P = (Plan*)plan;
  if (!P || cloud < 0 || cloud >= P->B) return NDNET_ERR_ARG;
  CloudCtl c;
  HIPCHK(hipDeviceSynchronize());
  const int rc = build_deferred_lists(P, nullptr);
  if (rc != NDNET_OK) return rc;
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
  // the retained list as the reference holds it after its left shift
  // (ndt.c:69-72): live entry i < num_kl = physical entry list_off + i, poison
  // past the entries ever written (value 0, ids 0xFFFFFFFF); the entries past
  // the live length are the ones the shift did not write (after one prune
  // level: the run's list, as the reference's; after several: the run's list
  // too, where the reference keeps what its earlier shifts left there)
  if (ord_val || ord_p || ord_q) {
    const size_t E = c.num_events, off = c.list_off, nphys = c.num_phys, nkl = c.num_kl;
    std::vector<double> v(P->ecap);
    std::vector<uint32_t> pp(P->ecap), qq(P->ecap);
    HIPCHK(hipMemcpy(v.data(), P->ord_val + eb, (size_t)P->ecap * 8, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(pp.data(), P->ord_p + eb, (size_t)P->ecap * 4, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(qq.data(), P->ord_q + eb, (size_t)P->ecap * 4, hipMemcpyDeviceToHost));
    for (size_t i = 0; i < E && i < P->ecap; i++) {
      const size_t src = i < nkl ? i + off : i;
      const bool ok = i < nkl ? src < nphys : true;
      if (ord_val) ord_val[i] = ok ? v[src] : 0.0;
      if (ord_p) ord_p[i] = ok ? pp[src] : kInvalid;
      if (ord_q) ord_q[i] = ok ? qq[src] : kInvalid;
    }
  }
  if (alive) HIPCHK(hipMemcpy(alive, P->alive + ob, nd, hipMemcpyDeviceToHost));
  return NDNET_OK;
}

}  // extern "C"
