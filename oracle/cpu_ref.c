/*
 * cpu_ref.c -- the CPU baseline with the reference core's cost structure.
 *
 * TEST / MEASUREMENT INFRASTRUCTURE ONLY: bench.py's cpu_baseline leg loads
 * it (oracle/libcpu_ref.so); the product never does.
 *
 * The reference's compiled core cannot travel to the GPU box, and
 * its KL stage cannot be built here at all (GSL absent), so the baseline timed
 * beside the GPU is this restatement.  The arithmetic is the oracle's
 * (ndt_oracle.c is included below, so the results are the oracle's, bit for
 * bit, up to the thread interleaving of the off-diagonal Welford terms that
 * the reference has too).  What this file adds is the reference's
 * execution structure, which is what its run time is made of:
 *
 *   estimate   normal_distributions.c:139-285 -- per bisection pass: V ND
 *              records initialised serially, V mutexes and V condition
 *              variables created, 8 pthreads (NUM_PCL_WORKERS) over
 *              contiguous chunks, and per point: voxel index, lock the
 *              voxel's mutex, wait on its condition variable while it is
 *              being updated, Welford update, unlock, signal; join; destroy
 *              the mutexes (the condition variables are not destroyed).
 *   KL call    kullback_leibler.c:28-127 -- per neighbour pair the GSL objects
 *              the reference allocates and frees (seven 3x3 / 3x1 / 1x3
 *              matrices and two permutations: gsl_matrix_alloc is three heap
 *              blocks, gsl_permutation_alloc two), the in-place LU of both
 *              covariances, the determinant and sign checks, the mean
 *              difference and its transpose, the inverse, the full 3x3 dgemm
 *              for the trace and the aliased 1x3 dgemm + ddot.
 *   insertion  kullback_leibler.c:181-195 -- O(E^2) descending insertion with
 *              the element shift (the oracle's orc_kl_all already does this).
 *
 * Built -O0 like the reference (CMakeLists.txt:6 CMAKE_BUILD_TYPE Debug);
 * bench.py runs one cloud at a time, as ndtnet_preprocessing.py:27 does.
 * Calibration against the compiled reference estimate stage (oracle/_ref,
 * build container only) is tests/test_cpu_ref.py / DESIGN.md §5.
 */
#include <pthread.h>
#include <stdbool.h>
#include <stdint.h>

struct orc_nd;
static int cref_estimate(const double* pc, uint64_t n, const uint16_t* cls, int ncls, double vs, const int* len,
                         const double* off, struct orc_nd* nds, uint64_t* num_nds);
static int cref_kl_divergence(struct orc_nd* p, struct orc_nd* q, double* div);
#define ORC_ESTIMATE cref_estimate
#define ORC_KL_DIVERGENCE cref_kl_divergence
#include "ndt_oracle.c"

/* ---------------- estimate: 8 workers, a mutex + condvar per voxel ---------------- */

typedef struct {
  const double* pc;
  uint64_t n;
  const uint16_t* cls;
  int ncls;
  double vs;
  const int* len;
  const double* off;
  orc_nd* nds;
  volatile bool* busy;
  pthread_mutex_t* mtx;
  pthread_cond_t* cnd;
  int id;
} cref_worker_t;

static void* cref_worker(void* arg) {
  cref_worker_t* a = (cref_worker_t*)arg;
  const uint64_t chunk = a->n / ORC_WORKERS;
  for (uint64_t i = (uint64_t)a->id * chunk; i < (uint64_t)(a->id + 1) * chunk; i++) {
    uint64_t v;
    if (orc_voxel_index(a->pc + 3 * i, a->vs, a->len, a->off, &v) < 0) return NULL;  /* abandons the chunk */
    pthread_mutex_lock(&a->mtx[v]);
    while (a->busy[v]) pthread_cond_wait(&a->cnd[v], &a->mtx[v]);
    a->busy[v] = true;
    orc_update(&a->nds[v], a->pc + 3 * i, a->cls ? a->cls + i : NULL, a->ncls);
    a->busy[v] = false;
    pthread_mutex_unlock(&a->mtx[v]);
    pthread_cond_signal(&a->cnd[v]);
  }
  return NULL;
}

static int cref_estimate(const double* pc, uint64_t n, const uint16_t* cls, int ncls, double vs, const int* len,
                         const double* off, orc_nd* nds, uint64_t* num_nds) {
  const uint64_t V = (uint64_t)(unsigned)len[0] * (unsigned)len[1] * (unsigned)len[2];
  bool* busy = (bool*)malloc((V ? V : 1) * sizeof(bool));
  if (!busy) return -1;
  for (uint64_t v = 0; v < V; v++) {  /* serial record initialisation */
    memset(&nds[v], 0, sizeof(orc_nd));
    busy[v] = false;
    if (cls) {
      nds[v].class_counts = (uint32_t*)calloc((size_t)ncls + 1, sizeof(uint32_t));
      if (!nds[v].class_counts) return -1;
    }
  }
  pthread_mutex_t* mtx = (pthread_mutex_t*)malloc((V ? V : 1) * sizeof(pthread_mutex_t));
  if (!mtx) return -2;
  for (uint64_t v = 0; v < V; v++) pthread_mutex_init(&mtx[v], NULL);
  pthread_cond_t* cnd = (pthread_cond_t*)malloc((V ? V : 1) * sizeof(pthread_cond_t));
  if (!cnd) return -5;
  for (uint64_t v = 0; v < V; v++) pthread_cond_init(&cnd[v], NULL);
  pthread_t* th = (pthread_t*)malloc(ORC_WORKERS * sizeof(pthread_t));
  cref_worker_t* args = (cref_worker_t*)calloc(ORC_WORKERS, sizeof(cref_worker_t));
  if (!th || !args) return -7;
  for (int w = 0; w < ORC_WORKERS; w++) {
    cref_worker_t* a = &args[w];
    a->pc = pc; a->n = n; a->cls = cls; a->ncls = ncls; a->vs = vs; a->len = len; a->off = off;
    a->nds = nds; a->busy = busy; a->mtx = mtx; a->cnd = cnd; a->id = w;
    if (pthread_create(&th[w], NULL, cref_worker, a) != 0) return -9;
  }
  for (int w = 0; w < ORC_WORKERS; w++)
    if (pthread_join(th[w], NULL) != 0) return -10;
  for (uint64_t v = 0; v < V; v++) pthread_mutex_destroy(&mtx[v]);
  uint64_t c = 0;
  for (uint64_t v = 0; v < V; v++) c += nds[v].n > 0;
  *num_nds = c;
  free(mtx);
  free(cnd);
  free(th);
  free(args);
  free(busy);
  return 0;
}

/* ---------------- KL call with the reference's GSL object traffic ---------------- */

/* gsl_matrix_alloc: the matrix struct, the block struct, the block's data */
typedef struct { size_t r, c; void* block; double* data; } cref_mat;
static cref_mat* cref_mat_alloc(size_t r, size_t c) {
  cref_mat* m = (cref_mat*)malloc(sizeof(cref_mat));
  m->block = malloc(2 * sizeof(size_t));
  m->data = (double*)malloc(r * c * sizeof(double));
  m->r = r;
  m->c = c;
  return m;
}
static void cref_mat_free(cref_mat* m) {
  free(m->data);
  free(m->block);
  free(m);
}
/* gsl_permutation_alloc: the struct and its data */
typedef struct { size_t n; size_t* data; } cref_perm;
static cref_perm* cref_perm_alloc(size_t n) {
  cref_perm* p = (cref_perm*)malloc(sizeof(cref_perm));
  p->data = (size_t*)malloc(n * sizeof(size_t));
  p->n = n;
  return p;
}
static void cref_perm_free(cref_perm* p) {
  free(p->data);
  free(p);
}
/* gslcblas dgemm, row-major, NoTrans x NoTrans, beta = 0 */
static void cref_dgemm(int M, int N, int K, const double* A, const double* B, double* C) {
  for (int i = 0; i < M; i++)
    for (int j = 0; j < N; j++) C[i * N + j] = 0.0;
  for (int k = 0; k < K; k++)
    for (int i = 0; i < M; i++) {
      const double t = 1.0 * A[i * K + k];
      if (t != 0.0)
        for (int j = 0; j < N; j++) C[i * N + j] += t * B[k * N + j];
    }
}

static int cref_kl_divergence(orc_nd* p, orc_nd* q, double* div) {
  *div = 0;
  if (p->n <= 1 || q->n <= 1) return -1;
  cref_mat* p_lu = cref_mat_alloc(3, 3);   /* allocated and never used, as in the reference */
  cref_mat* q_lu = cref_mat_alloc(3, 3);
  cref_perm* pp = cref_perm_alloc(3);
  cref_perm* qp = cref_perm_alloc(3);
  int pperm[3], qperm[3], ps, qs;
  orc_lu_decomp(p->cov, pperm, &ps);
  orc_lu_decomp(q->cov, qperm, &qs);
  for (int i = 0; i < 3; i++) { pp->data[i] = (size_t)pperm[i]; qp->data[i] = (size_t)qperm[i]; }
  cref_perm_free(pp);
  const double pd = orc_lu_det(p->cov, ps), qd = orc_lu_det(q->cov, qs);
  /* the reference leaks its objects on these early returns (kullback_leibler.c:66-78) */
  if (pd == 0 || qd == 0) return -2;
  if (orc_lu_sgndet(p->cov, ps) == 0 || orc_lu_sgndet(q->cov, qs) == 0) return -2;
  if (orc_lu_sgndet(q->cov, qs) == 0 || orc_lu_sgndet(q->cov, qs) == 0) return -2;
  cref_mat* md = cref_mat_alloc(3, 1);
  for (int i = 0; i < 3; i++) md->data[i] = q->mean[i];
  for (int i = 0; i < 3; i++) md->data[i] -= p->mean[i];
  cref_mat* mdt = cref_mat_alloc(1, 3);
  for (int i = 0; i < 3; i++) mdt->data[i] = md->data[i];
  cref_mat* qinv = cref_mat_alloc(3, 3);
  orc_lu_invert(q->cov, qperm, qinv->data);
  cref_perm_free(qp);
  cref_mat* tm = cref_mat_alloc(3, 3);
  memcpy(tm->data, qinv->data, 9 * sizeof(double));
  cref_dgemm(3, 3, 3, qinv->data, p->cov, tm->data);
  double tr = 0;
  for (int i = 0; i < 3; i++) tr += tm->data[i * 3 + i];
  cref_mat* fp = cref_mat_alloc(1, 3);
  memcpy(fp->data, mdt->data, 3 * sizeof(double));
  cref_dgemm(1, 3, 3, fp->data, qinv->data, fp->data);  /* aliased: C zeroed first, so 0 */
  double first = 0.0;
  for (int i = 0; i < 3; i++) first += fp->data[i] * md->data[i];
  *div = 0.5 * (first + tr - orc_log(qd / pd) - 3);
  cref_mat_free(p_lu);
  cref_mat_free(q_lu);
  cref_mat_free(md);
  cref_mat_free(mdt);
  cref_mat_free(qinv);
  cref_mat_free(tm);
  cref_mat_free(fp);
  return 0;
}

/* ---------------- entry points ---------------- */

/* One ndt_downsample (ndt.c:119-222) of one cloud: bisection over the
 * threaded estimate, KL list, prune, rows.  Returns the reference's code. */
int cref_downsample(const double* pc, uint64_t n, uint64_t k, double* out_pc, double* out_cov, uint64_t* nout) {
  orc_search_t s;
  orc_nd* nds = NULL;
  int rc = orc_search_impl(pc, 3, n, NULL, 0, k, &s, &nds);
  if (rc < 0) return rc;
  const uint64_t V = (uint64_t)(unsigned)s.len[0] * (unsigned)s.len[1] * (unsigned)s.len[2];
  orc_kl* list = (orc_kl*)calloc((V ? V : 1) * 6, sizeof(orc_kl));
  if (!list) return -4;
  uint64_t nv = 0, nk = 0;
  orc_kl_all(nds, s.len, &nv, list, &nk, NULL, NULL, NULL, NULL, NULL);
  orc_prune(nds, k, &nv, list, &nk, 6 * V);
  *nout = orc_to_point_cloud(nds, s.len, out_pc, out_cov, NULL, k);
  free(list);
  free(nds);
  return 0;
}

/* The estimate stage alone at a given grid (calibration against the
 * reference's own estimate_ndt, oracle/_ref ref_estimate_threads). */
int cref_estimate_only(const double* pc, uint64_t n, double vs, const int* len, const double* off, uint64_t* num_nds) {
  const uint64_t V = (uint64_t)(unsigned)len[0] * (unsigned)len[1] * (unsigned)len[2];
  orc_nd* nds = (orc_nd*)malloc((V ? V : 1) * sizeof(orc_nd));
  if (!nds) return -1;
  int rc = cref_estimate(pc, n, NULL, 0, vs, len, off, nds, num_nds);
  free(nds);
  return rc;
}
