// ndt_front.h -- k_front: the whole front of ndt_downsample in ONE launch.
//
// Included by ndt_kernels.hip inside its anonymous namespace (it uses
// CloudCtl, voxel_key, the block scans and finish_pass from there).
//
// What it replaces, per cloud (reference: pointclouds.c:40-66 limits,
// ndt.c:136-194 bisection over estimate_ndt's occupancy,
// normal_distributions.c:28-175 voxel assignment in worker order):
//   k_limits + 15 x k_search_pass + k_dense + k_bin_count + k_bin_offsets +
//   k_bin_scatter  (19 launches, ~260 us at 16 x 100k points)
//
// Geometry: G workgroups of 1024 threads per cloud (blockIdx.x = g,
// blockIdx.y = cloud), G * B <= CUs so every workgroup of a cloud is resident
// at once (checked on the host; G = 1 needs no residency at all).  Workgroup
// g owns `bpw` consecutive 1024-point bins; thread t holds point t of each of
// its bins in registers for the whole bisection, so the points are read from
// HBM once per run instead of once per pass.
//
// The G workgroups of a cloud meet at cloud barriers (one per phase): every
// wave drains its write-through (sc1) stores / atomics, the workgroup
// barriers, lane 0 adds to the cloud's counter and polls it with sc1 loads;
// everything handed across the barrier is read back with sc1 loads
// (MI355X_MICROARCH.md, inter-workgroup visibility, table row 1).  Each
// workgroup applies the bisection rule itself to the same summed counts, so
// no decision has to be broadcast.  A barrier that has not completed after
// ~2 s fails the cloud (NDNET_ERR_SYNC) instead of hanging.
//
// Phases:
//   0     limits: per-workgroup min/max keys -> [B][G][6], barrier, reduce
//   pass  voxel key of every estimated point; distinct voxels through an LDS
//         bitmap OR'd into the pass's global bitmap (V <= 32768), or an LDS
//         hash + per-voxel stamps (larger grids); per-workgroup fresh counts
//         -> record slots, barrier, sum, ndt.c:168-187.  A point out of the
//         grid abandons the rest of its worker chunk (normal_distributions.c
//         :47-52): on that rare pass the survivors are recounted.
//   dense accepted occupancy -> dense ids in ascending voxel order
//         (normal_distributions.c NDs are allocated per linear index); each
//         workgroup writes its slice of dense_of / vox.
//   bins  per point its ND; per bin a stable rank of the point among the
//         bin's points of the same ND (one wave per bin: ballot matching of
//         the ND ids bit by bit, an LDS cursor per ND); per-workgroup ND counts
//         -> [B][G][ndcap], barrier, ND bases (scan over NDs) + the counts of
//         earlier workgroups and bins, and every point written to its ND's
//         contiguous run in index order -- the order the reference's
//         1-worker schedule feeds each ND's Welford update.
#pragma once

constexpr int kFrontThreads = 1024;
constexpr int kFrontWaves = kFrontThreads / 64;
#ifndef NDNET_FRONT_R
#define NDNET_FRONT_R 8
#endif
constexpr int kFrontR = NDNET_FRONT_R;  // bins per workgroup whose points stay in registers
#ifndef NDNET_FRONT_BYTEMAP_READ
#define NDNET_FRONT_BYTEMAP_READ 0  // 1: read a voxel's byte before marking it (round 1-4 form)
#endif
#ifndef NDNET_FRONT_LDSMATCH
#define NDNET_FRONT_LDSMATCH 1  // the rank loop's low ND-id bits matched through LDS slots
#endif
#ifndef NDNET_FRONT_HEAVYSORT
#define NDNET_FRONT_HEAVYSORT 1  // 0: heavy NDs in listing order (A/B)
#endif
constexpr int kHeavySort = 256;     // heavy NDs per cloud that k_front lists by descending count
constexpr int kFrontTable = 8192;   // LDS words: byte map of a small grid (32768 voxels) or hash slots
constexpr int kFrontPhases = 40;    // record slots per cloud and run
constexpr int kRecWords = 16;       // per-workgroup record: [0] count, [1] any bad, [2..9] first bad per worker
constexpr int kPhDenseLarge = 36;
constexpr int kFrontMarkStride = 32 + 2 * 256;  // per cloud: 32 phase stamps of WG 0, then start/end of WG g < 256
constexpr int kBarStride = 16;      // u32 between the barrier counters of two clouds (64 B)
constexpr int kNdtErrSync = -22;    // NDNET_ERR_SYNC
static_assert(kFrontTable * 4 >= kBitsCap, "the byte map holds a whole small grid");

struct FrontArgs {
  CloudCtl* ctl;
  const int32_t* lbl;           // [B][n] or null
  uint32_t* stamps;             // [B][vcap]
  uint32_t* gbits;              // [B][2][kBitsWords]
  uint32_t* dense_of;           // [B][vcap]
  uint32_t* vox;                // [B][ndcap]
  uint32_t* nd_n;               // [B][ndcap]
  uint32_t* nd_base;            // [B][ndcap]
  uint32_t* heavy;              // [B][ndcap] NDs with >= heavy_t points (CloudCtl::heavy_n)
  uint32_t heavy_t;
  void* nd_pts;                 // [B * n + slack][3] T
  uint16_t* nd_lbl;             // [B][n] or null
  unsigned long long* lims;     // [B][G][6]
  uint32_t* rec;                // [B][kFrontPhases][G][kRecWords]
  uint32_t* wgcnt;              // [B][G][ndcap]
  uint32_t* bar;                // [B * kBarStride]
  unsigned long long* marks;    // [B][32] phase stamps of workgroup 0 (timing level 2), or null
  uint64_t n, k, vcap;
  uint32_t ndcap, G, bpw;
  uint32_t B;                   // clouds in the launch
  uint32_t nbins;               // 1024-point bins per cloud
  int xcd_local;                // 1: the G workgroups of a cloud share blockIdx % 8 (one XCD)
  uint32_t rbs;                 // points per rank bin (512 or 1024)
  int dbg_store;
  int staged;                   // 1: scatter through LDS records in ND order (float input; host checks the fit)
  int eval_all;                 // 1: count every bisection grid (debug / parity); 0: skip grids too small to matter
  uint64_t sync_ticks;          // cloud-barrier timeout in 100 MHz ticks (2e8 = 2 s; tests shorten it)
  uint32_t* lu_done;            // [B][lu_gcap] k_welford_q's group counters, re-armed with the cloud
  uint32_t lu_gcap;
  uint32_t* sync_fail;          // mapped host word: set on a barrier timeout (ndnet_ndt_take_sync_failures), or null
};

// The shared bisection state of one workgroup (every workgroup of a cloud
// holds an identical copy).
struct FrontState {
  double lim[6];
  double guess, lo, hi, vs;
  double off[3];
  uint32_t len[3];
  uint64_t V;
  uint32_t state, iter, stamp, mode, num_nds;
  uint32_t npass;                   // passes actually counted (their parity alternates the pass slots)
  uint32_t skip;                    // this iteration's grid has fewer voxels than k: no pass
  int32_t rc;
  uint32_t cut[kWorkers];
  uint32_t sync_no;
  uint64_t sync_ticks;              // barrier timeout, 100 MHz ticks (FrontArgs.sync_ticks)
  uint32_t puse[2];                 // uses of the two pass-sum slots
  unsigned long long psum_prev[2];  // their value after the previous use
  uint32_t ok;
  uint32_t count;
  uint32_t anybad;
  unsigned long long limkey[6];
};

__device__ inline uint32_t ld_sc1(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline void st_sc1(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// v of lane (lane ^ S), through DPP where the pattern allows (strides 1..8
// stay inside a row), ds_swizzle for 16, ds_bpermute for 32.
template <int S>
__device__ inline uint32_t xor_lane(uint32_t v) {
  const int x = (int)v;
  if constexpr (S == 1) {
    return (uint32_t)__builtin_amdgcn_mov_dpp(x, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
  } else if constexpr (S == 2) {
    return (uint32_t)__builtin_amdgcn_mov_dpp(x, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
  } else if constexpr (S == 4) {
    const int h = __builtin_amdgcn_mov_dpp(x, 0x141, 0xF, 0xF, false);    // row_half_mirror: i ^ 7
    return (uint32_t)__builtin_amdgcn_mov_dpp(h, 0x1B, 0xF, 0xF, false);  // quad_perm [3,2,1,0]: ^ 3
  } else if constexpr (S == 8) {
    const int h = __builtin_amdgcn_mov_dpp(x, 0x140, 0xF, 0xF, false);    // row_mirror: i ^ 15
    return (uint32_t)__builtin_amdgcn_mov_dpp(h, 0x141, 0xF, 0xF, false); // row_half_mirror: ^ 7
  } else if constexpr (S == 16) {
    return (uint32_t)__builtin_amdgcn_ds_swizzle(x, 0x401F);              // bitmask mode, xor 16
  } else {
    return (uint32_t)__shfl_xor(x, 32, 64);
  }
}

template <int S>
__device__ inline unsigned long long xor_lane64(unsigned long long v) {
  return (unsigned long long)xor_lane<S>((uint32_t)v) | ((unsigned long long)xor_lane<S>((uint32_t)(v >> 32)) << 32);
}

template <bool MAX>
__device__ inline unsigned long long wave_minmax64(unsigned long long v) {
  auto f = [](unsigned long long a, unsigned long long b) { return MAX ? (a > b ? a : b) : (a < b ? a : b); };
  v = f(v, xor_lane64<1>(v));
  v = f(v, xor_lane64<2>(v));
  v = f(v, xor_lane64<4>(v));
  v = f(v, xor_lane64<8>(v));
  v = f(v, xor_lane64<16>(v));
  v = f(v, xor_lane64<32>(v));
  return v;
}

// Cloud barrier of the G workgroups of one cloud.  Returns false (and fails
// the cloud) if the other workgroups did not arrive within ~2 s.
__device__ inline bool cloud_sync(FrontState& s, uint32_t* bar, uint32_t G) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    s.sync_no++;
    if (G > 1) {
      const uint32_t target = G * s.sync_no;
      __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      while (ld_sc1(bar) < target) {
        __builtin_amdgcn_s_sleep(1);
        if (__builtin_amdgcn_s_memrealtime() - t0 > s.sync_ticks) {  // 100 MHz clock (2 s by default)
          s.ok = 0;
          break;
        }
      }
    }
  }
  __syncthreads();
  return s.ok != 0;
}

// The barrier that ends a bisection pass, carrying the pass's count: each
// workgroup adds (1 << 48) + (bad << 32) + fresh to the pass-parity slot
// (u64 at bar + 2 + 2 parity, zeroed at plan creation and by the last workgroup out) and waits until G arrivals
// of this use are in; the count and the number of workgroups that saw an
// out-of-grid point are the slot's growth since its previous use.  One atomic
// and the poll replace a record per workgroup read back after the barrier.  A
// workgroup can only be one pass ahead (the next pass's barrier needs
// everyone), so no use of a slot overlaps the next one.
__device__ inline bool pass_sync(FrontState& s, uint32_t* bar, uint32_t G, uint32_t fresh, uint32_t anyb,
                                 uint32_t parity) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long* slot = reinterpret_cast<unsigned long long*>(bar + 2) + parity;
    const unsigned long long add = (1ull << 48) + ((unsigned long long)anyb << 32) + fresh;
    s.puse[parity]++;
    const unsigned long long target = (unsigned long long)G * s.puse[parity];
    unsigned long long v = __hip_atomic_fetch_add(slot, add, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + add;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while ((v >> 48) < target) {
      __builtin_amdgcn_s_sleep(1);
      v = __hip_atomic_load(slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (__builtin_amdgcn_s_memrealtime() - t0 > s.sync_ticks) {  // 100 MHz clock (2 s by default)
        s.ok = 0;
        break;
      }
    }
    const unsigned long long low = v & ((1ull << 48) - 1);
    const unsigned long long d = low - s.psum_prev[parity];
    s.psum_prev[parity] = low;
    s.count = (uint32_t)d;
    s.anybad = (uint32_t)(d >> 32);
  }
  __syncthreads();
  return s.ok != 0;
}

// Large-grid dedup: an LDS hash in front of the per-voxel stamps (bounded
// probing; a full table falls through to the global stamp, which dedups too).
__device__ inline uint32_t stamp_key_front(uint32_t key, uint32_t* table, uint32_t* stamps, uint32_t stamp) {
  uint32_t h = (key * 2654435761u) >> (32 - 13);
#pragma unroll 1
  for (int probe = 0; probe < 32; probe++) {
    const uint32_t cur = table[h];
    if (cur == key) return 0;
    if (cur == kInvalid) {
      const uint32_t old = atomicCAS(&table[h], kInvalid, key);
      if (old == kInvalid) break;
      if (old == key) return 0;
    }
    h = (h + 1) & (kFrontTable - 1);
  }
  uint32_t* sp = stamps + key;
  if (ld_sc1(sp) == stamp) return 0;
  return atomicExch(sp, stamp) != stamp;
}

template <typename T>
__device__ inline void front_point(const T* p, uint64_t i, T& x, T& y, T& z) {
  x = p[3 * i + 0];
  y = p[3 * i + 1];
  z = p[3 * i + 2];
}

#ifndef NDNET_FRONT_XB
#define NDNET_FRONT_XB 4
#endif
constexpr int kFrontXB = NDNET_FRONT_XB;  // bins past kFrontR loaded together

// the points of bins j0 .. j0 + kFrontXB - 1 of this thread (index clamped to
// the cloud's last point: every load valid, all of them in flight together)
template <typename T>
__device__ inline void front_points_xb(const T* p, uint64_t bin0, uint32_t j0, uint32_t t, uint64_t n,
                                       T (&xs)[kFrontXB], T (&ys)[kFrontXB], T (&zs)[kFrontXB]) {
#pragma unroll
  for (int u = 0; u < kFrontXB; u++) {
    const uint64_t i = (bin0 + j0 + u) * 1024 + t;
    front_point(p, i < n ? i : n - 1, xs[u], ys[u], zs[u]);
  }
}

// phase stamp (s_memrealtime, 100 MHz) of workgroup 0 of the cloud
#define FRONT_MARK(i)                                                                                  \
  do {                                                                                                 \
    if (A.marks && g == 0 && t == 0)                                                                   \
      A.marks[(uint64_t)b * kFrontMarkStride + (i)] = __builtin_amdgcn_s_memrealtime();               \
  } while (0)
#define FRONT_WG_MARK(e)                                                                               \
  do {                                                                                                 \
    if (A.marks && t == 0 && g < 256)                                                                  \
      A.marks[(uint64_t)b * kFrontMarkStride + 32 + 2 * g + (e)] = __builtin_amdgcn_s_memrealtime();  \
  } while (0)

template <typename T>
__global__ void __launch_bounds__(kFrontThreads) k_front(const T* __restrict__ pts, FrontArgs A) {
  extern __shared__ __attribute__((aligned(16))) uint32_t f_smem[];
  __shared__ FrontState s;
  __shared__ uint32_t scratch[32];
  __shared__ unsigned long long scratch64[16];
  __shared__ uint32_t s_heavy;  // workgroup 0: heavy NDs listed so far
  __shared__ unsigned long long s_hkey[kHeavySort];  // workgroup 0: (~count, ND) of the first kHeavySort heavy NDs
  __shared__ uint32_t s_bad[kWorkers];
  // Workgroup -> (cloud, g).  Blocks are dealt round-robin over the 8 XCDs
  // (MI355X_MICROARCH.md, speed only: the barriers below hold whatever the
  // placement), so with B % 8 == 0 the G workgroups of a cloud are given
  // linear ids with one residue mod 8: the cloud's points, bitmaps and grouped
  // output stay in one XCD's L2, whose partial 12-byte writes then merge
  // into whole lines before write-back instead of leaving partial lines dirty
  // in several XCDs.
  // Within an XCD the clouds are dealt cloud-major (slot s: cloud s / G,
  // workgroup s % G): workgroups start in linear-id order, so at any moment
  // a launch has at most ONE cloud per XCD with only part of its workgroups
  // resident -- the last one dispatched -- and every earlier cloud complete.
  // Two k_front launches that share the chip (two processes, or graphs whose
  // admission the front lanes could not order) then leave at most 2 (G - 1)
  // of an XCD's 32 CUs waiting on workgroups not yet dispatched, so one of
  // them always completes a cloud and frees its CUs: no cross-launch deadlock
  // at the cloud barriers.  (Rounds 2-5 dealt them slot-minor, s % (B / 8):
  // with two launches interleaved every cloud of both could be partial, and
  // the one-card two-process rehearsal timed out, gpurun_out/r05g.)
  const uint32_t L = blockIdx.x, G = A.G, bpw = A.bpw, rbs = A.rbs, nrb = bpw * (1024 / A.rbs);
  uint32_t g;
  int b;
  if (A.xcd_local) {
    const uint32_t slot = L / 8u;  // slot within the XCD
#ifdef NDNET_FRONT_DEAL_MINOR  // A/B only: the round 2-5 deal (deadlocks two concurrent launches)
    const uint32_t cpx = A.B / 8u;
    b = (int)((slot % cpx) * 8u + L % 8u);
    g = slot / cpx;
#else
    b = (int)((slot / G) * 8u + L % 8u);
    g = slot % G;
#endif
  } else {
    b = (int)(L / G);
    g = L % G;
  }
  const uint32_t t = threadIdx.x, lane = t & 63, wave = t >> 6;
  CloudCtl& c = A.ctl[b];
  const uint64_t n = A.n;
  const uint64_t chunk = n / kWorkers, n8 = chunk * kWorkers;
  const T* p = pts + (uint64_t)b * n * 3;
  uint32_t* bar = A.bar + (uint64_t)b * kBarStride;
  uint32_t* table = f_smem;                                   // kFrontTable words
  uint8_t* bytemap = (uint8_t*)f_smem;                        // small grids: one byte per voxel
  uint32_t* binfo = f_smem + kFrontTable;                     // [bpw][1024]: key, then did << 10 | rank
  // [nrb][ndcap] u16: per rank bin and ND a count (<= 1024), then the
  // workgroup-local prefix over rank bins (< 65536: a workgroup that fits
  // its LDS holds fewer points); the ND's global base goes to a per-ND word
  // in the table region (addv), so the u16 array halves the LDS that bounds
  // bins per workgroup (k = 2000 fits 8 workgroups per cloud)
  uint16_t* hist = reinterpret_cast<uint16_t*>(binfo + (uint64_t)bpw * 1024);
  uint32_t* stamps = A.stamps + (uint64_t)b * A.vcap;
  // my bins: [bin0, bin0 + nbw), nbw <= bpw (the bins of a cloud split as evenly as G allows)
  const uint64_t bin0 = (uint64_t)g * A.nbins / G;
  const uint64_t bin1 = (uint64_t)(g + 1) * A.nbins / G;
  const uint64_t iend = bin1 * 1024u < n ? bin1 * 1024u : n;    // my points: [bin0 * 1024, iend)
  const uint64_t iend8 = iend < n8 ? iend : n8;                   // ... that the workers estimate
  // this run's stamp epoch: every workgroup derives it from the previous
  // run's (stamps are epoch * 32 + pass; on the 2^26 wrap the stale stamps are
  // cleared here), and the last workgroup out stores it (no k_reset launch)
  uint32_t epoch = c.epoch + 1;
  const bool clear_stamps = epoch >= (1u << 26);
  if (clear_stamps) epoch = 1;
  FRONT_MARK(0);
  FRONT_WG_MARK(0);

  if (t == 0) {
    s.sync_no = 0;
    s.sync_ticks = A.sync_ticks;
    s.npass = 0;
    s.puse[0] = s.puse[1] = 0;
    s.psum_prev[0] = s.psum_prev[1] = 0;
    s.ok = 1;
    s.rc = 0;
    for (int a = 0; a < 3; a++) {
      s.limkey[a] = ord_key(kDblMin);      // max starts at DBL_MIN (pointclouds.c:44-46)
      s.limkey[3 + a] = ord_key(kDblMax);  // min starts at DBL_MAX
    }
  }
  if (clear_stamps) {  // epoch wrap: rare, cost irrelevant
    for (uint64_t v = (uint64_t)g * kFrontThreads + t; v < A.vcap; v += (uint64_t)G * kFrontThreads)
      st_sc1(stamps + v, 0u);
  }
  // ---- phase 0: points into registers, bounding box over all n points ----
  T px[kFrontR], py[kFrontR], pz[kFrontR];
  // per-thread extremes in T (the double of a float is exact and ordered
  // alike; NaN never wins, pointclouds.c maxf / minf)
  T mx[3] = {-INFINITY, -INFINITY, -INFINITY}, mn[3] = {INFINITY, INFINITY, INFINITY};
  auto lim_acc = [&](T x, T y, T z) {
    const T v[3] = {x, y, z};
#pragma unroll
    for (int a = 0; a < 3; a++) {
      mx[a] = v[a] > mx[a] ? v[a] : mx[a];
      mn[a] = v[a] < mn[a] ? v[a] : mn[a];
    }
  };
  // all loads issued unconditionally (clamped index) so they are in flight
  // together; a predicated load would compile to a branch + vmcnt(0) each
#pragma unroll
  for (int j = 0; j < kFrontR; j++) {
    const uint64_t i = (bin0 + j) * 1024 + t;
    const uint64_t ic = i < n ? i : n - 1;
    front_point(p, ic, px[j], py[j], pz[j]);
  }
#pragma unroll
  for (int j = 0; j < kFrontR; j++) {
    const uint64_t i = (bin0 + j) * 1024 + t;
    if ((uint32_t)j < bpw && i < iend) {
      lim_acc(px[j], py[j], pz[j]);
    } else {
      px[j] = py[j] = pz[j] = T(0);
    }
  }
  // bins past kFrontR (a CU share > 1: 13 bins per workgroup at share 2) are
  // re-read in every phase; their loads go out kFrontXB at a time (clamped
  // addresses), not one dependent round trip per bin
  for (uint32_t j0 = kFrontR; j0 < bpw; j0 += kFrontXB) {
    T xs[kFrontXB], ys[kFrontXB], zs[kFrontXB];
    front_points_xb(p, bin0, j0, t, n, xs, ys, zs);
#pragma unroll
    for (int u = 0; u < kFrontXB; u++) {
      const uint64_t i = (bin0 + j0 + u) * 1024 + t;
      if (j0 + u < bpw && i < iend) lim_acc(xs[u], ys[u], zs[u]);
    }
  }
  {
    unsigned long long kk[6];
#pragma unroll
    for (int a = 0; a < 3; a++) {
      const double dx = (double)mx[a], dn = (double)mn[a];
      kk[a] = wave_minmax64<true>(ord_key(dx > kDblMin ? dx : kDblMin));
      kk[3 + a] = wave_minmax64<false>(ord_key(dn < kDblMax ? dn : kDblMax));
    }
    __syncthreads();  // s.limkey initialised
    if (lane == 0) {
      for (int a = 0; a < 3; a++) {
        atomicMax(&s.limkey[a], kk[a]);
        atomicMin(&s.limkey[3 + a], kk[3 + a]);
      }
    }
  }
  // zero pass 0's bitmap (my slice), write-through
  {
    uint32_t* gb = A.gbits + (uint64_t)b * 2 * kBitsWords;
    for (uint32_t w = g * kFrontThreads + t; w < (uint32_t)kBitsWords; w += G * kFrontThreads) st_sc1(gb + w, 0u);
  }
  __syncthreads();
  unsigned long long* lims = A.lims + (uint64_t)b * G * 6;
  if (t < 6) __hip_atomic_store(lims + (uint64_t)g * 6 + t, s.limkey[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  FRONT_MARK(1);
  if (!cloud_sync(s, bar, G)) goto fail;
  FRONT_MARK(2);
  if (t < 6) s.limkey[t] = t < 3 ? 0ull : ~0ull;
  __syncthreads();
  for (uint32_t e = t; e < 6 * G; e += kFrontThreads) {
    const unsigned long long v = __hip_atomic_load(lims + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t a = e % 6;
    if (a < 3) atomicMax(&s.limkey[a], v);
    else atomicMin(&s.limkey[a], v);
  }
  __syncthreads();
  if (t == 0) {
    for (int a = 0; a < 6; a++) s.lim[a] = ord_unkey(s.limkey[a]);
    s.lo = kMinGuess;
    s.hi = kMaxGuess;
    s.iter = 0;
    s.state = kSearching;
    s.guess = (kMaxGuess - kMinGuess) / 2.0;  // ndt.c:136
  }
  __syncthreads();

  // ---- bisection passes ----
  for (;;) {
#ifndef NDNET_FRONT_BINMARKS
    if (s.npass == 0) FRONT_MARK(27);
#endif
    // grid of this guess (voxel.c:61-81), identical in every workgroup.
    // Thread 0 runs the passes a grid too small to count decides (hi = guess)
    // back to back, without a workgroup barrier per pass; after each such
    // pass the next guess's grid is computed, also when the pass ended the
    // search (as the reference's loop would before it exits).
    if (t == 0) {
      for (;;) {
        uint64_t V = 1;
        for (int a = 0; a < 3; a++) {
          const double d = s.lim[a] - s.lim[3 + a];
          const double q = ceil(d / s.guess);
          int li;
          if (q >= -2147483648.0 && q < 2147483648.0) li = (int)q;
          else li = (int)0x80000000;  // x86 cvttsd2si overflow value
          s.len[a] = (uint32_t)li;
          s.off[a] = s.lim[3 + a];
          V *= (uint64_t)s.len[a];
        }
        s.V = V;
        s.stamp = epoch * 32u + s.iter;
        // A grid of fewer voxels than k (or than the n8 estimated points)
        // cannot hold k occupied voxels: ndt.c:176-179 takes hi = guess
        // whatever the count, so the pass is not run (eval_all: it is, for the
        // parity tests that compare every count with the reference's).
        const uint64_t bound = V < n8 ? V : n8;
        s.skip = !A.eval_all && bound < A.k;
        if (V > A.vcap) {  // the reference's malloc of V NDs would be the failure point
          s.state = kFailed;
          s.rc = -1;
          s.vs = s.guess;
          s.skip = 0;
        }
        if (s.state != kSearching || !s.skip) break;
        if (g == 0 && s.iter < 16) {
          c.guesses[s.iter] = s.guess;
          c.counts[s.iter] = kInvalid;  // not counted (< k)
        }
        s.hi = s.guess;
        s.iter++;
        const double gn = s.lo + (s.hi - s.lo) / 2.0;
        s.guess = gn;
        if (s.iter == (uint32_t)kMaxIters) {
          s.state = kFailed;
          s.rc = -3;  // "Reached maximum number of iterations!" (ndt.c:191-194)
          s.vs = gn;
        }
      }
    }
    __syncthreads();
    if (s.npass == 0) FRONT_MARK(19);
    if (s.state != kSearching) break;
    const uint64_t V = s.V;
    const bool small = V <= (uint64_t)kBitsCap;
    const uint32_t words = small ? (uint32_t)((V + 31) / 32) : 0u;
    const uint32_t parity = s.npass & 1u;
    const uint32_t stamp = s.stamp;
    uint32_t* gb = A.gbits + ((uint64_t)b * 2 + parity) * kBitsWords;
    if (small) {
      for (uint32_t w = t; w < 8 * words; w += kFrontThreads) table[w] = 0;
    } else {
      for (uint32_t w = t; w < (uint32_t)kFrontTable; w += kFrontThreads) table[w] = kInvalid;
    }
    if (t < (uint32_t)kWorkers) s_bad[t] = kInvalid;
    __syncthreads();
    const double vs = s.guess, inv_vs = 1.0 / vs;
    double off[3] = {s.off[0], s.off[1], s.off[2]};
    uint32_t len[3] = {s.len[0], s.len[1], s.len[2]};
    // float points: keys screened in single precision (voxel_key_f32), valid
    // when the grid offset is a float (it is the minimum of float points)
    const float off32[3] = {(float)off[0], (float)off[1], (float)off[2]};
    const float inv32 = (float)inv_vs;
    const float lenf[3] = {(float)len[0], (float)len[1], (float)len[2]};
    const float lmax = fmaxf(lenf[0], fmaxf(lenf[1], lenf[2]));
    const float half_tol = 0.5f - lmax * 0x1p-19f;  // |frac(q) - 1/2| bound of voxel_key_f32
    const bool fast32 = std::is_same<T, float>::value && (double)off32[0] == off[0] &&
                        (double)off32[1] == off[1] && (double)off32[2] == off[2];
    uint32_t fresh = 0;
    // Hot, unrolled over the register-resident points: the key of every
    // estimated point into binfo (the accepted pass's keys feed the binning),
    // single precision for float input; small grids mark the byte map.  The
    // rest -- the double path where the screen cannot decide (the point is
    // re-read), out-of-grid points, the stamp dedup of large grids -- runs in
    // rolled loops below, so the unrolled code stays small.
    bool redo = false, cold = false;
    auto visit = [&](uint32_t j, uint64_t i, T x, T y, T z) {
      uint32_t key = kInvalid;
      if (i < iend8) {
        key = fast32 ? voxel_key_f32((float)x, (float)y, (float)z, off32, inv32, half_tol, lenf, len) : kKeyRedo;
        redo |= key == kKeyRedo;
        cold |= key == kInvalid;
        if (small && key < kKeyRedo) {
#if NDNET_FRONT_BYTEMAP_READ
          if (!bytemap[key]) bytemap[key] = 1;  // read first: most lanes of a small grid hit set bytes
#else
          bytemap[key] = 1;  // a plain store: no LDS round trip per point before the next point's key
#endif
        }
      }
      binfo[j * 1024 + t] = key;
    };
#pragma unroll
    for (int j = 0; j < kFrontR; j++)
      if ((uint32_t)j < bpw) visit(j, (bin0 + j) * 1024 + t, px[j], py[j], pz[j]);
    for (uint32_t j0 = kFrontR; j0 < bpw; j0 += kFrontXB) {
      T xs[kFrontXB], ys[kFrontXB], zs[kFrontXB];
      front_points_xb(p, bin0, j0, t, n, xs, ys, zs);
#pragma unroll
      for (int u = 0; u < kFrontXB; u++)
        if (j0 + u < bpw) visit(j0 + u, (bin0 + j0 + u) * 1024 + t, xs[u], ys[u], zs[u]);  // (visit checks iend8)
    }
    if (__any(redo)) {
#pragma unroll 1
      for (uint32_t j = 0; j < bpw; j++) {
        const uint32_t e = j * 1024 + t;
        if (binfo[e] == kKeyRedo) {
          T x, y, z;
          front_point(p, (bin0 + j) * 1024 + t, x, y, z);
          const uint32_t key = voxel_key((double)x, (double)y, (double)z, off, len, vs, inv_vs);
          binfo[e] = key;
          cold |= key == kInvalid;
          if (small && key != kInvalid && !bytemap[key]) bytemap[key] = 1;
        }
      }
    }
    if (!small || __any(cold)) {
#pragma unroll 1
      for (uint32_t j = 0; j < bpw; j++) {
        const uint64_t i = (bin0 + j) * 1024 + t;
        const uint32_t key = binfo[j * 1024 + t];
        if (i >= iend8) continue;
        if (key == kInvalid) atomicMin(&s_bad[i / chunk], (uint32_t)i);
        else if (!small) fresh += stamp_key_front(key, table, stamps, stamp);
      }
    }
    __syncthreads();
#ifndef NDNET_FRONT_BINMARKS
    if (s.npass == 0) FRONT_MARK(28);
#endif
    if (small) {  // byte map -> 32-voxel words, OR'd into the pass's global bitmap
      for (uint32_t w = t; w < words; w += kFrontThreads) {
        uint32_t bits = 0;
#pragma unroll
        for (int q = 0; q < 8; q++) {
          const uint32_t v = table[8 * w + q];
          bits |= ((v & 1u) | ((v >> 7) & 2u) | ((v >> 14) & 4u) | ((v >> 21) & 8u)) << (4 * q);
        }
        if (bits) fresh += __popc(bits & ~atomicOr(&gb[w], bits));
      }
    }
    {  // the other parity's bitmap is the next pass's: zero my slice
      uint32_t* gn = A.gbits + ((uint64_t)b * 2 + (parity ^ 1u)) * kBitsWords;
      for (uint32_t w = g * kFrontThreads + t; w < (uint32_t)kBitsWords; w += G * kFrontThreads) st_sc1(gn + w, 0u);
    }
#ifndef NDNET_FRONT_BINMARKS
    if (s.npass == 0) FRONT_MARK(29);
#endif
    fresh = block_sum_u32(fresh, scratch);
#ifndef NDNET_FRONT_BINMARKS
    if (s.npass == 0) FRONT_MARK(30);
#endif
    uint32_t* rec = A.rec + (((uint64_t)b * kFrontPhases + 1 + 2 * s.iter) * G) * kRecWords;
    uint32_t anyb = 0;
    for (int w = 0; w < kWorkers; w++) anyb |= s_bad[w] != kInvalid;
    if (t == 0) {  // the record is read back only on a pass with an out-of-grid point
      st_sc1(rec + g * kRecWords + 1, anyb);
      if (anyb)
        for (int w = 0; w < kWorkers; w++) st_sc1(rec + g * kRecWords + 2 + w, s_bad[w]);
    }
    FRONT_MARK(3 + 2 * (s.iter < 7 ? s.iter : 7));
    if (!pass_sync(s, bar, G, fresh, anyb, parity)) goto fail;
    FRONT_MARK(4 + 2 * (s.iter < 7 ? s.iter : 7));
    if (t < (uint32_t)kWorkers) s.cut[t] = kInvalid;
    __syncthreads();
#ifndef NDNET_FRONT_BINMARKS
    if (s.npass == 0) FRONT_MARK(31);
#endif
    uint32_t mode = small ? parity : 2u;
    if (s.anybad) {
      // a point out of the grid abandoned the rest of its worker chunk
      // (normal_distributions.c:47-52): recount the survivors through stamps
      for (uint32_t e = t; e < G * kWorkers; e += kFrontThreads) {
        const uint32_t gg = e / kWorkers, w = e % kWorkers;
        if (ld_sc1(rec + gg * kRecWords + 1)) atomicMin(&s.cut[w], ld_sc1(rec + gg * kRecWords + 2 + w));
      }
      for (uint32_t w = t; w < (uint32_t)kFrontTable; w += kFrontThreads) table[w] = kInvalid;
      __syncthreads();
      const uint32_t stamp2 = epoch * 32u + 16u + s.iter;
      uint32_t f2 = 0;
      for (uint32_t j = 0; j < bpw; j++) {
        const uint64_t i = (bin0 + j) * 1024 + t;
        const uint32_t key = binfo[j * 1024 + t];
        if (key != kInvalid && i < s.cut[i / chunk]) f2 += stamp_key_front(key, table, stamps, stamp2);
      }
      f2 = block_sum_u32(f2, scratch);
      uint32_t* rec2 = A.rec + (((uint64_t)b * kFrontPhases + 2 + 2 * s.iter) * G) * kRecWords;
      if (t == 0) {
        st_sc1(rec2 + g * kRecWords, f2);
        s.count = 0;
        s.stamp = stamp2;
      }
      if (!cloud_sync(s, bar, G)) goto fail;
      if (t < G) atomicAdd(&s.count, ld_sc1(rec2 + t * kRecWords));
      mode = 2u;
      __syncthreads();
    }
    // ndt.c:168-187, every workgroup alike
    if (t == 0) {
      const uint32_t count = s.count;
      if (g == 0 && s.iter < 16) {
        c.guesses[s.iter] = s.guess;
        c.counts[s.iter] = count;
      }
      s.mode = mode;
      s.npass++;
      if ((double)count > (double)A.k * (1 + kUpper)) {
        s.lo = s.guess;
      } else if (count < A.k) {
        s.hi = s.guess;
      } else {
        s.state = kAccepted;
        s.vs = s.guess;
        s.num_nds = count;
      }
      s.iter++;
      if (s.state == kSearching) {
        const double gn = s.lo + (s.hi - s.lo) / 2.0;
        s.guess = gn;
        if (s.iter == (uint32_t)kMaxIters) {
          s.state = kFailed;
          s.rc = -3;  // "Reached maximum number of iterations!" (ndt.c:191-194)
          s.vs = gn;
        } else {
          for (int w = 0; w < kWorkers; w++) s.cut[w] = kInvalid;
        }
      }
    }
    __syncthreads();
    if (s.state != kSearching) break;
  }

  // ---- publish the search outcome for the later kernels ----
  if (g == 0 && t == 0) {
    for (int a = 0; a < 6; a++) c.lim[a] = s.lim[a];
    c.guess = s.guess;
    c.lo = s.lo;
    c.hi = s.hi;
    c.vs = s.vs;
    for (int a = 0; a < 3; a++) {
      c.len[a] = s.len[a];
      c.off[a] = s.off[a];
    }
    c.V = s.V;
    c.state = s.state;
    c.rc = s.rc;
    c.iter = s.iter;
    c.stamp = s.stamp;
    c.accepted_stamp = s.stamp;
    c.acc_mode = s.mode;
    c.num_nds = s.state == kAccepted ? s.num_nds : 0u;
    for (int w = 0; w < kWorkers; w++) c.first_bad[w] = s.cut[w];
  }
  if (s.state != kAccepted) goto out;
  FRONT_MARK(20);

  {
    // ---- dense ids of the accepted grid ----
    const uint64_t V = s.V;
    const uint32_t ndcap = A.ndcap, nd = s.num_nds;
    uint32_t* dense = A.dense_of + (uint64_t)b * A.vcap;
    uint32_t* vox = A.vox + (uint64_t)b * ndcap;
    const bool bitmap = s.mode < 2;
    uint32_t* bits_l = table;              // [1024] accepted bitmap
    uint32_t* pref_l = table + kBitsWords; // [1024] exclusive popcount prefix
    if (bitmap) {
      const uint32_t words = (uint32_t)((V + 31) / 32);
      const uint32_t* gbw = A.gbits + ((uint64_t)b * 2 + s.mode) * kBitsWords;
      const uint32_t bits = t < words ? ld_sc1(gbw + t) : 0u;  // words <= 1024 = blockDim
      uint32_t tot;
      const uint32_t ex = block_excl_scan((uint32_t)__popc(bits), 0u, AddU32(), scratch, tot);
      bits_l[t] = bits;
      pref_l[t] = ex;
      __syncthreads();
      // my slice of dense_of / vox, one voxel per thread
      const uint64_t v0 = V * g / G, v1 = V * (g + 1) / G;
      for (uint64_t v = v0 + t; v < v1; v += kFrontThreads) {
        const uint32_t w = (uint32_t)(v >> 5), bit = (uint32_t)(v & 31);
        const uint32_t bw = bits_l[w];
        if ((bw >> bit) & 1u) {
          const uint32_t d = pref_l[w] + __popc(bw & ((1u << bit) - 1u));
          dense[v] = d;
          if (d < ndcap) vox[d] = (uint32_t)v;
        } else {
          dense[v] = kInvalid;
        }
      }
    } else {
      // stamps: my slice of the voxels, counted, then numbered after the
      // counts of the earlier workgroups' slices
      const uint32_t astamp = s.stamp;
      const uint64_t v0 = V * g / G, v1 = V * (g + 1) / G;
      uint32_t cnt = 0;
      for (uint64_t v = v0 + t; v < v1; v += kFrontThreads) cnt += ld_sc1(stamps + v) == astamp;
      cnt = block_sum_u32(cnt, scratch);
      uint32_t* rec = A.rec + (((uint64_t)b * kFrontPhases + kPhDenseLarge) * G) * kRecWords;
      if (t == 0) {
        st_sc1(rec + g * kRecWords, cnt);
        s.count = 0;
      }
      if (!cloud_sync(s, bar, G)) goto fail;
      if (t < g) atomicAdd(&s.count, ld_sc1(rec + t * kRecWords));
      __syncthreads();
      uint32_t carry = s.count;
      for (uint64_t base = v0; base < v1; base += kFrontThreads) {
        const uint64_t v = base + t;
        const uint32_t occ = v < v1 && ld_sc1(stamps + v) == astamp;
        uint32_t tot;
        const uint32_t ex = block_excl_scan(occ, 0u, AddU32(), scratch, tot);
        if (v < v1) {
          const uint32_t d = carry + ex;
          st_sc1(dense + v, occ ? d : kInvalid);
          if (occ && d < ndcap) vox[d] = (uint32_t)v;
        }
        carry += tot;
      }
      if (!cloud_sync(s, bar, G)) goto fail;
    }
    FRONT_MARK(21);

    // ---- per point: its ND (did), in place of its key ----
    {
      const uint32_t nh = nrb * ndcap;  // u16 counters; hist is 16-byte aligned (after the u32 binfo)
      for (uint32_t e = t; e < nh / 8u; e += kFrontThreads) reinterpret_cast<uint4*>(hist)[e] = make_uint4(0, 0, 0, 0);
      for (uint32_t e = (nh / 8u) * 8u + t; e < nh; e += kFrontThreads) hist[e] = 0;
    }
    {
      // the bins of kFrontR: every lookup issued before any is used
      // (addresses clamped, results selected), the worker-chunk cut (an
      // out-of-grid point, normal_distributions.c:47-52) checked only when
      // the accepted pass had one.  Round 4: "point NDs" 2.75 -> 2.25 us
      // (profiles/r04_front_ab.txt)
      bool cuts = false;
#pragma unroll
      for (int w = 0; w < kWorkers; w++) cuts |= s.cut[w] != kInvalid;
      uint32_t keys[kFrontR], dv[kFrontR];
#pragma unroll
      for (int j = 0; j < kFrontR; j++) keys[j] = (uint32_t)j < bpw ? binfo[j * 1024 + t] : kInvalid;
#pragma unroll
      for (int j = 0; j < kFrontR; j++) {
        const uint32_t kc = keys[j] != kInvalid ? keys[j] : 0u;
        if (bitmap) {
          const uint32_t bw = bits_l[kc >> 5];
          dv[j] = pref_l[kc >> 5] + __popc(bw & ((1u << (kc & 31)) - 1u));
        } else {
          dv[j] = ld_sc1(dense + kc);
        }
      }
#pragma unroll
      for (int j = 0; j < kFrontR; j++) {
        if ((uint32_t)j < bpw) {
          const uint64_t i = (bin0 + j) * 1024 + t;
          bool ok = keys[j] != kInvalid;
          if (cuts) ok = ok && i < s.cut[i / chunk];
          binfo[j * 1024 + t] = ok ? dv[j] : kInvalid;
        }
      }
    }
    for (uint32_t j = kFrontR; j < bpw; j++) {
      const uint64_t i = (bin0 + j) * 1024 + t;
      const uint32_t key = binfo[j * 1024 + t];
      uint32_t d = kInvalid;
      if (key != kInvalid && i < s.cut[i / chunk]) {
        if (bitmap) {
          const uint32_t bw = bits_l[key >> 5];
          d = pref_l[key >> 5] + __popc(bw & ((1u << (key & 31)) - 1u));
        } else {
          d = ld_sc1(dense + key);
        }
      }
      binfo[j * 1024 + t] = d;
    }
    __syncthreads();
    FRONT_MARK(22);

    // ---- per rank bin (one wave): stable rank of each point among its ND's
    //      points in the bin, in index order; the bin's ND counts ----
    // Lanes holding the same ND are found by matching the ND id bit by bit
    // with ballots (no sort): a lane's rank is the number of lower lanes in
    // its match set, and the set's last lane advances the ND's bin counter.
    // nbits is uniform (readfirstlane) so the unrolled bit loop branches on
    // SGPRs; per bit: a 1-bit signed extract (0 / -1), its ballot, and
    // m &= ~(ballot ^ mask) on both halves -- the lanes that agree on the bit.
    const uint32_t nbits = __builtin_amdgcn_readfirstlane(32u - (uint32_t)__clz((int)(ndcap > 1 ? ndcap - 1 : 1)));
    const unsigned long long below = (1ull << lane) - 1ull;
#if NDNET_FRONT_LDSMATCH
    // Round 4: the low 8 bits of the ND id matched through LDS instead of 8
    // ballot rounds: each lane ORs its bit into its wave's slot d & 255
    // (the table region is free once the point NDs are found: 16 waves x 256
    // slots x 8 B = kFrontTable words) and reads the slot back; only the
    // high bits are matched by ballots.  The loop is VALU-issue bound
    // (~6 instructions per matched bit), not LDS bound.
    unsigned long long* slots = reinterpret_cast<unsigned long long*>(table) + (uint64_t)wave * 256u;
    static_assert(kFrontWaves * 256 * 2 <= kFrontTable, "a wave's 256 match slots fit the table region");
#pragma unroll
    for (int e = 0; e < 4; e++) slots[lane + 64 * e] = 0ull;
    const unsigned long long mybit = 1ull << lane;
#endif
    for (uint32_t r = wave; r < nrb; r += kFrontWaves) {
      uint16_t* hr = hist + (uint64_t)r * ndcap;
      uint32_t* br = binfo + (uint64_t)r * rbs;
      for (uint32_t st = 0; st < rbs / 64; st++) {
        const uint32_t d = br[st * 64 + lane];
        const bool valid = d != kInvalid;
#if NDNET_FRONT_LDSMATCH
        const uint32_t h = d & 255u;
        if (valid) __hip_atomic_fetch_or(&slots[h], mybit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        // the wave's ORs are one LDS instruction, executed before this read
        const unsigned long long mv = valid ? __hip_atomic_load(&slots[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) : 0ull;
        uint32_t mlo = (uint32_t)mv, mhi = (uint32_t)(mv >> 32);
        constexpr uint32_t kBit0 = 8;
#else
        const unsigned long long mv = __ballot(valid);
        uint32_t mlo = (uint32_t)mv, mhi = (uint32_t)(mv >> 32);
        constexpr uint32_t kBit0 = 0;
#endif
#pragma unroll
        for (uint32_t bit = kBit0; bit < 15; bit++) {  // ndcap <= 16384 (k_front host check)
          if (bit < nbits) {
            const uint32_t mask = (uint32_t)__builtin_amdgcn_sbfe((int)d, bit, 1);
            const unsigned long long bb = __ballot(mask != 0u);
            mlo &= ~((uint32_t)bb ^ mask);
            mhi &= ~((uint32_t)(bb >> 32) ^ mask);
          }
        }
        const unsigned long long m = ((unsigned long long)mhi << 32) | mlo;
#if NDNET_FRONT_LDSMATCH
        // every lane of the slot has read it (the read above is one
        // instruction): cleared for the next step
        if (valid) __hip_atomic_store(&slots[h], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#endif
        if (valid) {
          const uint32_t rank = (uint32_t)__popcll(m & below), cnt = (uint32_t)__popcll(m);
          const uint32_t cur = hr[d];  // read by every lane of the set before its last lane writes
          br[st * 64 + lane] = (d << 10) | (cur + rank);
          if (rank + 1 == cnt) hr[d] = (uint16_t)(cur + cnt);
        }
      }
    }
#ifdef NDNET_FRONT_BINMARKS
    FRONT_MARK(27);
#endif
    __syncthreads();
#ifdef NDNET_FRONT_BINMARKS
    FRONT_MARK(28);
#endif
    // per ND: my workgroup's count -> wgcnt; hist[r][d] -> exclusive prefix over my rank bins
    uint32_t* wg = A.wgcnt + (uint64_t)b * G * ndcap;
    for (uint32_t d = t; d < nd; d += kFrontThreads) {
      uint32_t run = 0, r = 0;
      for (; r + 4 <= nrb; r += 4) {  // four rank bins per LDS round trip
        uint32_t x[4];
#pragma unroll
        for (int q = 0; q < 4; q++) x[q] = hist[(uint64_t)(r + q) * ndcap + d];
#pragma unroll
        for (int q = 0; q < 4; q++) {
          hist[(uint64_t)(r + q) * ndcap + d] = (uint16_t)run;
          run += x[q];
        }
      }
      for (; r < nrb; r++) {
        const uint32_t x = hist[(uint64_t)r * ndcap + d];
        hist[(uint64_t)r * ndcap + d] = (uint16_t)run;
        run += x;
      }
      st_sc1(wg + (uint64_t)g * ndcap + d, run);
    }
    FRONT_MARK(23);
    if (t == 0) s_heavy = 0;
    if (!cloud_sync(s, bar, G)) goto fail;
    FRONT_MARK(24);
    // ND bases (scan of the per-ND totals over NDs) + earlier workgroups'
    // counts.  Staged scatter: the same scan also places my points in ND
    // order (local position = my count prefix over NDs + the point's rank
    // among my points of its ND); delta[d] = global - local is kept in the
    // table region (free since the per-point NDs were found).
    const bool staged = A.staged != 0;
    uint32_t* addv = table;           // [ndcap]: the ND's global base + earlier workgroups' counts
    uint32_t* delta = table + ndcap;  // [ndcap] (staged: 2 ndcap <= kFrontTable, host check)
    uint32_t carry = 0, lcarry = 0;
    for (uint32_t base = 0; base < nd; base += kFrontThreads) {
      const uint32_t d = base + t;
      uint32_t tot_d = 0, pre = 0, mine = 0;
      if (d < nd) {
        uint32_t gg = 0;
        for (; gg + 16 <= G; gg += 16) {  // 16 loads in flight: one memory round trip for G <= 16
          uint32_t x[16];
#pragma unroll
          for (int q = 0; q < 16; q++) x[q] = ld_sc1(wg + (uint64_t)(gg + q) * ndcap + d);
#pragma unroll
          for (int q = 0; q < 16; q++) {
            if (gg + q < g) pre += x[q];
            if (gg + q == g) mine = x[q];
            tot_d += x[q];
          }
        }
        if (gg < G) {  // the rest, loads clamped to workgroup G - 1 and masked
          uint32_t x[16];
#pragma unroll
          for (int q = 0; q < 16; q++) x[q] = ld_sc1(wg + (uint64_t)(gg + q < G ? gg + q : G - 1) * ndcap + d);
#pragma unroll
          for (int q = 0; q < 16; q++) {
            if (gg + q < G) {
              if (gg + q < g) pre += x[q];
              if (gg + q == g) mine = x[q];
              tot_d += x[q];
            }
          }
        }
      }
      uint32_t start;
      if (staged) {  // both scans in one: the ND total in the high word, my count in the low
        unsigned long long tot2;
        const unsigned long long ex2 =
            block_excl_scan(((unsigned long long)tot_d << 32) | mine, 0ull, AddU64(), scratch64, tot2);
        start = carry + (uint32_t)(ex2 >> 32);
        if (d < nd) delta[d] = start + pre - (lcarry + (uint32_t)ex2);
        carry += (uint32_t)(tot2 >> 32);
        lcarry += (uint32_t)tot2;
      } else {
        uint32_t tot;
        start = carry + block_excl_scan(tot_d, 0u, AddU32(), scratch, tot);
        carry += tot;
      }
      if (d < nd) {
        if (g == 0) {
          A.nd_n[(uint64_t)b * ndcap + d] = tot_d;
          A.nd_base[(uint64_t)b * ndcap + d] = start;
          // k_welford_q gives these a wave each (their order changes no result)
          if (tot_d >= A.heavy_t) {
            const uint32_t hi = atomicAdd(&s_heavy, 1u);
            A.heavy[(uint64_t)b * ndcap + hi] = d;
            if (hi < (uint32_t)kHeavySort) s_hkey[hi] = ((unsigned long long)~tot_d << 32) | d;
          }
        }
        addv[d] = start + pre;  // a point's destination: addv[d] + hist[r][d] + its rank
      }
    }
    __syncthreads();
    if (g == 0 && t == 0) {
      c.heavy_n = s_heavy;
      c.heavy_t = A.heavy_t;
    }
    if (NDNET_FRONT_HEAVYSORT && g == 0 && s_heavy > 1u && s_heavy <= (uint32_t)kHeavySort && t < s_heavy) {
      // the cloud's heavy NDs by descending count: k_welford_q's first round
      // gives item i to wave i % 4 of workgroup i / 4, so a cloud's longest
      // NDs share a few workgroups (CUs) instead of each holding one CU to
      // the end of the launch (profiles/r04_wq_heavy_order.txt)
      const unsigned long long key = s_hkey[t];
      uint32_t rank = 0;
      for (uint32_t j = 0; j < s_heavy; j++) rank += s_hkey[j] < key ? 1u : 0u;
      A.heavy[(uint64_t)b * ndcap + rank] = (uint32_t)key;
    }
    FRONT_MARK(25);
    // ---- scatter: every point to its ND's run, in index order ----
    T* out = (T*)A.nd_pts + (uint64_t)b * n * 3;
    const uint32_t rsub = t / rbs;  // my rank bin within a 1024-point bin
    if constexpr (sizeof(T) == 4) {
      if (staged) {
        // Each workgroup's points form one contiguous segment of every ND's
        // run (its bins are consecutive, ranks are in index order).  A point
        // stored by its own lane is a 12-byte piece of a random line: 3.2x
        // the bytes in L2 write-backs (tools/ubench/write_width.hip).  So the
        // points are first placed in ND order in LDS (16-byte records: x, y,
        // z, destination), then stored by consecutive lanes as consecutive
        // dwords of those segments (1.3x).  Records for every local position
        // fit the whole dynamic LDS (host check: 4 words per point), which is
        // free once each thread holds its points' positions in registers.
        uint32_t gd[kFrontR], lp[kFrontR];
#pragma unroll
        for (int j = 0; j < kFrontR; j++) {
          gd[j] = kInvalid;
          if ((uint32_t)j < bpw) {
            const uint32_t bi = binfo[j * 1024 + t];
            if (bi != kInvalid) {
              const uint32_t d = bi >> 10;
              gd[j] = addv[d] + hist[(uint64_t)(j * (1024 / rbs) + rsub) * ndcap + d] + (bi & 1023u);
              lp[j] = gd[j] - delta[d];
              if (A.nd_lbl) A.nd_lbl[(uint64_t)b * n + gd[j]] = (uint16_t)A.lbl[(uint64_t)b * n + (bin0 + j) * 1024 + t];
            }
          }
        }
        __syncthreads();  // binfo / hist / delta read: the records may overwrite them
        float4* rec = reinterpret_cast<float4*>(f_smem);
#pragma unroll
        for (int j = 0; j < kFrontR; j++)
          if (gd[j] != kInvalid)
            rec[lp[j]] = make_float4((float)px[j], (float)py[j], (float)pz[j], __uint_as_float(gd[j]));
        __syncthreads();
        // lane l stores record l: 12 bytes (one global_store_dwordx3) right
        // after lane l - 1's within a segment
        float3* o3 = reinterpret_cast<float3*>(out);
        for (uint32_t l = t; l < lcarry; l += kFrontThreads) {
          const float4 r = rec[l];
#ifdef NDNET_FRONT_STAGED_NT  // A/B: streaming (nontemporal) stores
          float* o = reinterpret_cast<float*>(o3 + __float_as_uint(r.w));
          __builtin_nontemporal_store(r.x, o);
          __builtin_nontemporal_store(r.y, o + 1);
          __builtin_nontemporal_store(r.z, o + 2);
#else
          o3[__float_as_uint(r.w)] = make_float3(r.x, r.y, r.z);
#endif
        }
      }
    }
    if (sizeof(T) != 4 || !staged) {
    auto put = [&](uint32_t j, uint64_t i, T x, T y, T z) {
      const uint32_t bi = binfo[j * 1024 + t];
      if (bi == kInvalid) return;
      const uint32_t d = bi >> 10;
      const uint32_t r = j * (1024 / rbs) + rsub;
      const uint32_t dst = addv[d] + hist[(uint64_t)r * ndcap + d] + (bi & 1023u);
      T* o = out + (uint64_t)dst * 3;
      if (A.dbg_store == 1) {
        __builtin_nontemporal_store(x, o);
        __builtin_nontemporal_store(y, o + 1);
        __builtin_nontemporal_store(z, o + 2);
      } else if (A.dbg_store == 2) {
        __hip_atomic_store(o, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(o + 1, y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(o + 2, z, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        o[0] = x;
        o[1] = y;
        o[2] = z;
      }
      if (A.nd_lbl) A.nd_lbl[(uint64_t)b * n + dst] = (uint16_t)A.lbl[(uint64_t)b * n + i];
    };
#pragma unroll
    for (int j = 0; j < kFrontR; j++)
      if ((uint32_t)j < bpw) put(j, (bin0 + j) * 1024 + t, px[j], py[j], pz[j]);
    for (uint32_t j0 = kFrontR; j0 < bpw; j0 += kFrontXB) {
      T xs[kFrontXB], ys[kFrontXB], zs[kFrontXB];
      front_points_xb(p, bin0, j0, t, n, xs, ys, zs);
#pragma unroll
      for (int u = 0; u < kFrontXB; u++) {
        const uint64_t i = (bin0 + j0 + u) * 1024 + t;
        if (j0 + u < bpw && i < iend8) put(j0 + u, i, xs[u], ys[u], zs[u]);
      }
    }
    }
    FRONT_MARK(26);
  }
  FRONT_WG_MARK(1);
  goto out;
fail:
  if (t == 0) {
    c.state = kFailed;
    c.rc = kNdtErrSync;
    // sticky, in host memory: the host raises it without synchronising
    if (A.sync_fail) __hip_atomic_store(A.sync_fail, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
out:
  // The last workgroup of the cloud out (every one has passed its last
  // barrier poll) re-arms the cloud for the next run: barrier counter and
  // pass-sum slots zeroed, the epoch stored, the prune-list counters (set by
  // the KL kernels, read by further prune levels) and k_welford_q's group
  // counters cleared (this run's k_welford_q follows in stream order).
  if (t == 0 && __hip_atomic_fetch_add(bar + 6, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == G - 1) {
    for (int i = 0; i < 7; i++) st_sc1(bar + i, 0u);
    for (uint32_t i = 0; i < A.lu_gcap; i++) A.lu_done[(uint64_t)b * A.lu_gcap + i] = 0u;
    c.epoch = epoch;
    c.clear_stamps = clear_stamps ? 1u : 0u;
    c.num_valid = c.num_kl = c.num_phys = c.num_events = c.flag_count = 0;
    c.prune_rc = 0;
    c.num_out = c.last_k = 0;
  }
}
