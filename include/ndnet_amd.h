/*
 * ndnet_amd.h -- C ABI of libndnet_amd.so, the MI355X (gfx950) NDT path.
 *
 * Two groups of entry points:
 *
 * 1. The reference's own ABI (core_legacy/include/ndnet_core/ndt.h:59-116 and
 *    kullback_leibler.h:74), same names, argument order, meaning and return
 *    codes, host pointers in and out.  The reference's ctypes wrapper
 *    (ndnet/preprocessing/ndt_legacy.py:28-43) binds these unchanged once its
 *    library path points at libndnet_amd.so.  The ND and KL
 *    handles are opaque, as they already are to the reference's Python side
 *    (ndt_legacy.py:5-25 declares `__fields__`, so ctypes never sees a field).
 *
 * 2. A batched device API for B clouds resident in HBM (no PCIe in the hot
 *    path): plan once, run many times on a HIP stream.  The run functions do
 *    no allocation and no synchronisation, so they can be captured in a graph.
 *
 * Return codes: the reference's (0 success; -1 voxel table allocation /
 * capacity; -3 "Reached maximum number of iterations!"; prune: -1 "desired >
 * valid", -2 "Reached the end of the divergences array!") plus
 * NDNET_ERR_* for API misuse and HIP failures.  Nothing aborts.
 */
#ifndef NDNET_AMD_H_
#define NDNET_AMD_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NDNET_OK 0
#define NDNET_ERR_ARG (-20)  /* bad argument (NULL, zero size, unsupported point_dim) */
#define NDNET_ERR_HIP (-21)  /* HIP runtime failure; message on stderr */
#define NDNET_ERR_SYNC (-22) /* a cloud's workgroups did not meet within ~2 s (k_front barrier): the cloud fails */
#define NDNET_PRUNE_POISON (-8) /* a prune walk reached a list entry the reference never wrote */

/* Per-cloud outcome of a batched run; written on the device. */
typedef struct ndnet_ndt_stats {
  int32_t rc;          /* ndt_downsample return code for this cloud */
  int32_t prune_rc;    /* prune_nds return code of the last prune level */
  uint32_t iters;      /* estimate passes of the voxel-size bisection */
  uint32_t len[3];     /* voxel grid of the accepted (or last tried) size */
  double offset[3];
  double voxel_size;
  uint64_t num_nds;    /* occupied voxels at the accepted size */
  uint64_t num_valid;  /* NDs left after the prune */
  uint64_t num_kl;     /* live divergence-list length after the prune */
  uint64_t num_events; /* divergence entries created */
  uint64_t num_out;    /* surviving NDs (rows written = min(num_out, k)) */
} ndnet_ndt_stats;

/* ---------------------------------------------------------------------------
 * 1. Reference ABI (host pointers).
 * ------------------------------------------------------------------------ */

/* Replaces ndt_downsample (ndt.h:100-110, ndt.c:119-222).  point_dim must be 3
 * (the reference's workers hard-code a stride of 3, normal_distributions.c:47).
 * out_pc/out_cov/out_classes hold num_desired_points rows; out_classes may be
 * NULL; classes may be NULL (unlabelled).  *nd_array and *kl_divergences
 * receive opaque handles for prune_nds / to_point_cloud / free_*. */
int ndt_downsample(double *point_cloud, unsigned short point_dim, unsigned long num_points,
                   unsigned int *len_x, unsigned int *len_y, unsigned int *len_z,
                   double *offset_x, double *offset_y, double *offset_z,
                   double *voxel_size,
                   unsigned short *classes, unsigned short num_classes,
                   unsigned long num_desired_points,
                   double *downsampled_point_cloud, unsigned long *num_downsampled_points,
                   double *covariances,
                   unsigned short *downsampled_classes,
                   void **nd_array, unsigned long *num_valid_nds,
                   void **kl_divergences, unsigned long *num_kl_divergences);

/* Replaces prune_nds (ndt.h:59-62, ndt.c:28-73): prunes the retained list of a
 * handle to num_desired_nds, with the reference's walk, bound check and
 * left shift. */
int prune_nds(void *nd_array,
              unsigned int len_x, unsigned int len_y, unsigned int len_z,
              unsigned long num_desired_nds, unsigned long *num_valid_nds,
              void *kl_divergences, unsigned long *num_kl_divergences);

/* Replaces to_point_cloud (ndt.h:76-82, ndt.c:75-117): surviving NDs in
 * ascending voxel order.  Writes at most the row count of the last
 * downsample/prune (the reference has no capacity argument and overruns its
 * buffers when a prune fails); *num_points receives the survivor count. */
int to_point_cloud(void *nd_array,
                   unsigned int len_x, unsigned int len_y, unsigned int len_z,
                   double offset_x, double offset_y, double offset_z,
                   double voxel_size,
                   double *point_cloud, unsigned long *num_points,
                   double *covariances,
                   unsigned short *classes);

/* Replaces free_nds (ndt.h:116) and free_kl_divergences (kullback_leibler.h:74).
 * NULL is accepted (the reference dereferences it after a failed search). */
void free_nds(void *nd_array, unsigned long num_nds);
void free_kl_divergences(void *kl_divergences);

/* Replaces print_matrix (matrix.h:40, matrix.c:28-35): prints a rows x cols
 * row-major double matrix to stdout, one row per line, "%f " per element.
 * The reference's own library test binds it (ndnet/test/suites/libs.py:13-26). */
void print_matrix(double *matrix, int rows, int cols);

/* ---------------------------------------------------------------------------
 * 2. Batched device API (the ndt_preprocessing hot path,
 *    ndnet/preprocessing/ndtnet_preprocessing.py:6-73).
 * ------------------------------------------------------------------------ */

/* Allocates the device workspace for `batch` clouds of `num_points` points
 * downsampled to `num_desired` NDs.  num_classes >= 0 enables labelled runs
 * (class histograms of num_classes + 1 bins); -1 disables them.
 * voxel_capacity bounds the voxels of any grid the bisection visits (0: 2^22);
 * a grid beyond it fails that cloud with rc -1, as the reference's malloc
 * would. */
int ndnet_ndt_plan_create(int batch, uint64_t num_points, uint64_t num_desired, int num_classes,
                          uint64_t voxel_capacity, void **plan);
void ndnet_ndt_plan_destroy(void *plan);

/* Launch path of a plan: 1 = one launch per stage (limits, 15 bisection
 * passes, dense ids, three binning kernels), 2 = the fused front kernel
 * k_front (limits through binning in one launch; needs every workgroup of a
 * cloud resident, so only where the plan's shape allows it), 0 = 2 where
 * allowed, else 1 (the default).  Both paths give identical results.
 * ndnet_ndt_get_path returns the path in use.
 * Concurrency: path 2's cloud barriers need every workgroup of a cloud
 * resident at once.  k_front deals each launch's clouds cloud-major within an
 * XCD (workgroups start in id order), so a launch has at most one partially
 * resident cloud per XCD, and ANY TWO k_front launches at once -- two plans,
 * two streams, two graphs, two processes on one GPU -- always complete.  On
 * top of that the library keeps one process's k_front launches to one chip's
 * worth: the chip is split into 4 front lanes, a plan's k_front occupies
 * ceil(4 * workgroups / CUs) of them (4 at CU share 1, 2 at share 2), waits
 * for the previous k_front of each of its lanes and records itself on them
 * (HIP events; explicit event nodes when the stream is being captured, so the
 * replays of a graph wait for the launches its capture saw on its lanes).  A
 * plan that is its device's only plan skips the admission.  k_fronts whose
 * lanes are disjoint (two share-2 plans) run side by side.  What the lanes
 * cannot order -- launches of other processes, a graph replayed beside a plan
 * created after its capture -- overlaps at most pairwise in practice; three
 * or more share-1 launches at once can still time out (NDNET_ERR_SYNC, never
 * a hang).  ndnet_ndt_get_front_lanes reports a plan's lanes (nlanes 0 on
 * path 1). */
int ndnet_ndt_set_path(void *plan, int path);
int ndnet_ndt_get_path(void *plan);
int ndnet_ndt_get_front_lanes(void *plan, int *lane0, int *nlanes);

/* 1 if a k_front barrier of an earlier run of the plan timed out (a cloud
 * failed with NDNET_ERR_SYNC) since the last call, else 0; clears the flag.
 * k_front sets it in mapped host memory, so this reads it without
 * synchronising: ndt_preprocessing raises on it at its next call (graph
 * replays of ndnet.pipeline at theirs). */
int ndnet_ndt_take_sync_failures(void *plan);

/* CU shares of the plan's two widest kernels: k_front runs
 * CUs / (front_share * batch) workgroups per cloud and k_welford_q
 * CUs / welford_share workgroups, leaving the other CUs to kernels on other
 * streams (ndnet.pipeline.PipelinedSegmentation overlaps the NDT stage with the
 * PointNet forward that way).  Default 1, 1 (every CU).  Results are identical
 * for every share.  NDNET_ERR_ARG when k_front does not fit front_share (the
 * previous shares are kept). */
int ndnet_ndt_set_cu_share(void *plan, int front_share, int welford_share);

/* The bisection (ndt.c:144-187) takes hi = guess whenever a grid has fewer
 * voxels (or the cloud fewer estimated points) than num_desired: such a grid
 * cannot reach k occupied voxels, so path 2 does not count it and the debug
 * dump reports its count as 0xFFFFFFFF.  Guesses, decisions and outputs are
 * unchanged.  on = 1 counts every grid anyway (the parity tests compare every
 * count with the reference's); default 0.  Path 1 always counts. */
int ndnet_ndt_set_exact_counts(void *plan, int on);

/* k_front's last phase writes every point to its ND's run (the grouped
 * points k_welford_q reads).  on = 1 (default) places a workgroup's points in
 * ND order in LDS first and stores them as consecutive dwords of its run
 * segments; on = 0 stores each point from its own lane (12-byte pieces of
 * random lines: ~2x the HBM write bytes).  Identical results either way;
 * float input with the plan's shapes in LDS only (otherwise direct). */
int ndnet_ndt_set_front_staged(void *plan, int on);
/* 1 when k_front's scatter of float input runs staged for this plan's shapes
 * (and CU share), 0 when it runs direct; NDNET_ERR_ARG for a NULL plan. */
int ndnet_ndt_get_front_staged(void *plan);

/* k_welford_q computes the moments of an ND with at least min_samples points
 * on a whole wave (the mean recurrence alone on three lanes, the per-sample
 * products on all 64, the ordered sums on six), every other ND on a lane
 * quad of a 16-ND wave.  Identical results either way (the same IEEE
 * operations in the reference's order, normal_distributions.c:75-103); the
 * threshold only moves work.  Default 256; min_samples >= 1. */
int ndnet_ndt_set_heavy_threshold(void *plan, uint32_t min_samples);

/* k_welford_q's form for the NDs below the heavy threshold: 1 = one ND per
 * lane (64 NDs per wave: a quarter of the CUs on C2, for a plan whose k_front
 * leaves the chip to other streams), 2 = a lane quad per ND (16 NDs per wave:
 * every CU, the faster form alone), 0 = by the CU share: 2 at share 1, 1 above
 * (the default; NDNET_WQ_FORM=light64|quad overrides it for every plan).
 * Identical results either way.  ndnet_ndt_get_welford_form returns the form
 * in use (1 or 2). */
int ndnet_ndt_set_welford_form(void *plan, int form);
int ndnet_ndt_get_welford_form(void *plan);

/* Split ndnet_ndt_run in two stream-ordered calls (a caller that overlaps the
 * run with other work on another stream, e.g. ndnet.pipeline): part 1 runs the
 * front only (k_front: limits, bisection, dense ids, binning), part 2 the rest
 * (k_welford_q onwards) and must follow a part-1 call of the same plan in
 * stream order, with the same arguments.  0 (default) = the whole run. */
int ndnet_ndt_set_run_part(void *plan, int part);

/* The retained divergence list (kl_divergences, ndt.c:189-205) is read by the
 * level-1 prune only when it removes NDs.  A cloud with num_nds <= num_desired
 * keeps every ND (or fails with rc -1 before reading the list), so by default
 * its run only counts the events (stats num_events / num_kl are unchanged)
 * and builds the list on demand, before ndnet_ndt_prune or
 * ndnet_ndt_debug_dump reads it; the built list is the eagerly built one,
 * entry for entry.  on = 0 builds every list in the run.  Default 1. */
int ndnet_ndt_set_lazy_list(void *plan, int on);

/* d_points: [batch][num_points][3] float32 on the device (the tensor
 * ndt_preprocessing receives).  d_labels: [batch][num_points] int32 class ids
 * or NULL.  d_out: [batch][num_desired][12] float32 = mean(3) | covariance(9)
 * row-major, nan_to_num applied (ndtnet_preprocessing.py:66-67), zero rows
 * past the survivors.  d_out_classes: [batch][num_desired][num_classes+1]
 * one-hot or NULL.  d_stats: [batch] device array or NULL.  stream: a
 * hipStream_t (NULL = default stream). */
int ndnet_ndt_run(void *plan, void *stream, const float *d_points, const int32_t *d_labels, float *d_out,
                  float *d_out_classes, ndnet_ndt_stats *d_stats);

/* Same on float64 points, with float64 outputs as the reference's
 * ndt_downsample writes them: d_out_points [batch][k][3], d_out_covariances
 * [batch][k][9], d_out_classes [batch][k] (any may be NULL), and optionally
 * the float32 [batch][k][12] block. */
int ndnet_ndt_run_f64(void *plan, void *stream, const double *d_points, const int32_t *d_labels,
                      double *d_out_points, double *d_out_covariances, uint16_t *d_out_classes, float *d_out,
                      ndnet_ndt_stats *d_stats);

/* A further prune level of every cloud of the last run (NDT_Sampler.prune,
 * ndt_legacy.py:173-240): outputs sized [batch][num_desired][...]. */
int ndnet_ndt_prune(void *plan, void *stream, uint64_t num_desired, float *d_out, float *d_out_classes,
                    double *d_out_points, double *d_out_covariances, uint16_t *d_out_classes16,
                    ndnet_ndt_stats *d_stats);

/* Stage timing with HIP events on the run's stream (bench.py): after
 * ndnet_ndt_set_timing(plan, 1), each run records events around its stages;
 * ndnet_ndt_stage_ms fills ms[6] of the last run (synchronises): path 1 =
 * reset+limits, 15 bisection passes, dense ids, binning, Welford + LU chains,
 * KL+prune+rows; path 2 = k_front, three empty intervals (events recorded
 * back to back), Welford + LU chains, KL+prune+rows. */
int ndnet_ndt_set_timing(void *plan, int enable);  /* 0 off, 1 stage events, 2 + k_kl phase stamps */
int ndnet_ndt_stage_ms(void *plan, float *ms);

/* Host copies of one cloud's intermediates after a run (parity tests). */
int ndnet_ndt_debug_dump(void *plan, int cloud, uint32_t *nd_n, double *nd_mean, double *nd_cov_pre,
                         double *nd_cov_post, uint32_t *vox, double *ord_val, uint32_t *ord_p, uint32_t *ord_q,
                         double *guesses, uint32_t *counts, uint32_t *iters, uint8_t *alive);

/* k_front's cloud-barrier timeout in 100 MHz ticks for the plan's next runs
 * (0 restores the default 2e8 = 2 s).  A workgroup that waits longer fails its
 * cloud with NDNET_ERR_SYNC; tests shorten it to reach that path. */
int ndnet_ndt_debug_set_sync_timeout(void *plan, uint64_t ticks);

/* Sets every cloud's stamp epoch (synchronises).  The epoch advances once per
 * run and wraps after 2^26 - 1 runs, when the device clears the stale voxel
 * stamps itself; tests use this to reach the wrap. */
int ndnet_ndt_debug_set_epoch(void *plan, uint32_t epoch);

/* The run's prune and rows on the merge launch's last workgroup per cloud
 * (on = 1, the default; NDNET_KL_FUSE=0 in the environment at plan creation
 * turns it off) or on a k_kl launch of their own (0).  Same outputs either way. */
int ndnet_ndt_debug_set_kl_fuse(void *plan, int on);

/* The event list's sort (round 6): 1 sorts each cloud's list on one
 * workgroup (k_kl_sort) when the plan's list fits its LDS (ecap <= 7680 slots,
 * k <= 1065), else on k_kl_merge's workgroups per chunk group; 0 always takes
 * k_kl_merge; 2 (the default; NDNET_KL_SORT in the environment at plan
 * creation overrides it) takes k_kl_sort only at a CU share > 1
 * (ndnet_ndt_set_cu_share: a pipeline's plan, where the merge's CU time
 * matters more than its latency); 3 as 1 with the chunks ranked in the
 * sort's own launch (k_kl_rank_sort: the cloud's last ranking workgroup
 * sorts) instead of a launch of their own (k_kl_rank_chunks, then k_kl_sort).
 * Same lists, rows and stats every way.  _get_ returns 1 when the plan's runs sort (k_kl_rank_sort or
 * k_kl_sort), 0 when they merge (k_kl_merge). */
int ndnet_ndt_debug_set_list_sort(void *plan, int on);
int ndnet_ndt_debug_get_list_sort(void *plan);

/* KL-stage phase stamps of the last run at timing level 2: marks[cloud * 32 + i],
 * 100 MHz s_memrealtime ticks.  k_kl: 0 start, 1 cloud state checked, 2 event
 * count, 5 list initialised, 6 first occurrences, 7 walk scan, 8 kills, 9 shift,
 * 10 rows emitted, 11 end; k_kl_rank_chunks (chunk 0): 3 start, 4 scores, 15 end;
 * k_kl_merge (workgroup 0): 12 start, 16 runs staged, 17 NaN bases scanned,
 * 13 NaN keys, 14 end; 18 / 19 the last rank / merge workgroup's end; the rest unused.  marks holds B * 32 values; synchronises. */
int ndnet_ndt_debug_kl_marks(void *plan, unsigned long long *marks);

/* k_front phase stamps of the last run at timing level 2 (workgroup 0 of each
 * cloud): marks[cloud * 32 + i], 100 MHz ticks; 0 start, 1/2 limits barrier
 * in/out, 3+2p/4+2p pass p barrier in/out (p < 7; later passes share 17/18),
 * 20 accepted, 21 dense ids, 22 point NDs, 23/24 offsets barrier in/out,
 * 25 offsets, 26 scattered; synchronises. */
int ndnet_ndt_debug_front_marks(void *plan, unsigned long long *marks);
/* Start / end stamps (s_memrealtime) of every k_front workgroup of the last
 * run at timing level 2: marks[B][G][2]; *G = workgroups per cloud. */
int ndnet_ndt_debug_front_wg_marks(void *plan, unsigned long long *marks, int *G);

/* k_welford_q per-item stamps of the last run at timing level 2: *items =
 * capacity B * (ndcap + ceil(ndcap / 16)) (items past the run's count keep
 * old values); marks[item * 8 + i]: 0 s_memrealtime at the item's start
 * (100 MHz), 1..3 s_memtime (shader clock) at its start, after the moments,
 * at its end; 4 = heavy << 63 | samples of its longest ND << 32 | wave id;
 * 5..7 (heavy items) shader cycles in the whole-wave path's phases 0 + 2
 * (loads, per-sample products), 1 (mean recurrence), 3 (ordered sums).
 * Heavy items come first.  marks must hold 8 * capacity values; synchronises. */
int ndnet_ndt_debug_wq_marks(void *plan, unsigned long long *marks, uint32_t *items);

/* The device's in-place LU chain (the GSL 2.7.1 LU_decomp restatement the
 * KL stage applies once per event, kullback_leibler.c:57-63) on n row-major
 * 3x3 matrices d_A [n][9]: `steps` (1..12) successive decompositions of each,
 * every state to d_states [n][steps][9], its permutation (p0 | p1 << 2 |
 * p2 << 4) | (signum < 0) << 8 to d_ps [n][steps], and d_flags [n][steps] =
 * det != 0 && sgndet != 0 (the event flag, kullback_leibler.c:57-70).  For
 * the parity tests; stream-ordered on `stream`. */
int ndnet_debug_lu_chain(const double *d_A, uint32_t n, int steps, double *d_states, uint32_t *d_ps,
                         uint32_t *d_flags, void *stream);

/* Library identification (no GPU needed). */
const char *ndnet_amd_version(void);

#ifdef __cplusplus
}
#endif

#endif /* NDNET_AMD_H_ */
