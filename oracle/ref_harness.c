/*
 * ref_harness.c -- drives the reference's own estimate stage.  TEST INFRASTRUCTURE ONLY.
 *
 * Linked (by oracle/Makefile) against the UNMODIFIED reference sources
 * core_legacy/src/{normal_distributions,voxel,pointclouds,matrix}.c, compiled
 * in place from /root/reference like the reference's CMake Debug build
 * (-O0 -g, no -fopenmp: SURVEY F6).  Output goes to oracle/_ref/ only.
 * kullback_leibler.c and ndt.c include GSL headers that this image lacks
 * (SURVEY §8c), so they are not built; the ndt.c bisection loop (ndt.c:131-194,
 * twenty lines around the calls below) is restated here verbatim in behaviour.
 *
 * ref_estimate_seq runs the reference's pcl_worker for worker ids 0..7 one
 * after the other on one thread: a legal schedule of estimate_ndt
 * (normal_distributions.c:139-285) whose result is deterministic.
 * ref_estimate_threads calls estimate_ndt itself (8 pthreads; off-diagonal
 * covariances then depend on thread interleaving).
 */
#include <ndnet_core/normal_distributions.h>
#include <stdint.h>
#include <stdlib.h>

void ref_limits(double* pc, short dim, unsigned long n, double* lim) {
  get_pointcloud_limits(pc, dim, n, &lim[0], &lim[1], &lim[2], &lim[3], &lim[4], &lim[5]);
}

void ref_grid(const double* lim, double vs, int* len, double* off) {
  estimate_voxel_grid(lim[0], lim[1], lim[2], lim[3], lim[4], lim[5], vs, &len[0], &len[1], &len[2], &off[0],
                      &off[1], &off[2]);
}

static void copy_out(struct normal_distribution_t* nd, unsigned long V, uint64_t* cnt, double* mean, double* cov,
                     uint16_t* cls) {
  for (unsigned long v = 0; v < V; v++) {
    cnt[v] = nd[v].num_samples;
    for (int j = 0; j < 3; j++) mean[3 * v + j] = nd[v].mean[j];
    for (int j = 0; j < 9; j++) cov[9 * v + j] = nd[v].covariance[j];
    if (cls) cls[v] = nd[v].num_class_samples ? nd[v].class : 0;
  }
}

static void free_classes(struct normal_distribution_t* nd, unsigned long V) {
  for (unsigned long v = 0; v < V; v++) free(nd[v].num_class_samples);
}

/* Sequential schedule of the reference's own worker routine. */
int ref_estimate_seq(double* pc, unsigned long n, unsigned short* classes, unsigned short ncls, double vs,
                     const int* len, const double* off, uint64_t* cnt, double* mean, double* cov, uint16_t* cls,
                     uint64_t* num_nds) {
  const unsigned long V = (unsigned long)len[0] * len[1] * len[2];
  struct normal_distribution_t* nd = malloc((V ? V : 1) * sizeof(*nd));
  pthread_mutex_t* mtx = malloc((V ? V : 1) * sizeof(*mtx));
  pthread_cond_t* cnd = malloc((V ? V : 1) * sizeof(*cnd));
  if (!nd || !mtx || !cnd) return -1;
  /* the initialisation estimate_ndt performs (normal_distributions.c:149-172) */
  for (unsigned long i = 0; i < V; i++) {
    nd[i].num_samples = 0;
    nd[i].index = i;
    nd[i].num_class_samples = classes ? calloc(ncls + 1, sizeof(unsigned int)) : NULL;
    for (int j = 0; j < 3; j++) {
      nd[i].mean[j] = 0;
      nd[i].m2[j] = 0;
      for (int k = 0; k < 3; k++) nd[i].covariance[j * 3 + k] = 0;
    }
    nd[i].class = 0;
    nd[i].being_updated = false;
    pthread_mutex_init(&mtx[i], NULL);
    pthread_cond_init(&cnd[i], NULL);
  }
  for (int w = 0; w < NUM_PCL_WORKERS; w++) {
    struct pcl_worker_args_t a = {0};
    a.point_cloud = pc;
    a.num_points = n;
    a.classes = classes;
    a.num_classes = ncls;
    a.nd_array = nd;
    a.mutex_array = mtx;
    a.cond_array = cnd;
    a.voxel_size = vs;
    a.len_x = len[0];
    a.len_y = len[1];
    a.len_z = len[2];
    a.x_offset = off[0];
    a.y_offset = off[1];
    a.z_offset = off[2];
    a.worker_id = w;
    pcl_worker(&a);
  }
  uint64_t c = 0;
  for (unsigned long i = 0; i < V; i++) c += nd[i].num_samples > 0;
  *num_nds = c;
  copy_out(nd, V, cnt, mean, cov, cls);
  for (unsigned long i = 0; i < V; i++) {
    pthread_mutex_destroy(&mtx[i]);
    pthread_cond_destroy(&cnd[i]);
  }
  free_classes(nd, V);
  free(nd);
  free(mtx);
  free(cnd);
  return 0;
}

/* The shipped 8-thread estimate_ndt. */
int ref_estimate_threads(double* pc, unsigned long n, unsigned short* classes, unsigned short ncls, double vs,
                         const int* len, const double* off, uint64_t* cnt, double* mean, double* cov, uint16_t* cls,
                         uint64_t* num_nds) {
  const unsigned long V = (unsigned long)len[0] * len[1] * len[2];
  struct normal_distribution_t* nd = malloc((V ? V : 1) * sizeof(*nd));
  if (!nd) return -1;
  unsigned long c = 0;
  int rc = estimate_ndt(pc, n, classes, ncls, vs, len[0], len[1], len[2], off[0], off[1], off[2], nd, &c);
  if (rc < 0) return rc;
  *num_nds = c;
  copy_out(nd, V, cnt, mean, cov, cls);
  free_classes(nd, V);
  free(nd);
  return 0;
}

/* ndt.c:131-194 around the reference's estimate_voxel_grid/estimate_ndt (here the
 * sequential schedule).  Records every guess and count. */
int ref_search(double* pc, unsigned long n, unsigned long k, double* guesses, uint64_t* counts, int* iters, int* len,
               double* off, double* voxel_size) {
  double lim[6];
  ref_limits(pc, 3, n, lim);
  double guess = (double)(30.0 - 0.01) / 2.0;
  double lo = 0.01, hi = 30.0;
  unsigned iter = 0;
  *iters = 0;
  do {
    ref_grid(lim, guess, len, off);
    const unsigned long V = (unsigned long)(unsigned)len[0] * (unsigned)len[1] * (unsigned)len[2];
    uint64_t* cnt = malloc((V ? V : 1) * 8);
    double* mean = malloc((V ? V : 1) * 24);
    double* cov = malloc((V ? V : 1) * 72);
    uint64_t c = 0;
    ref_estimate_seq(pc, n, NULL, 0, guess, len, off, cnt, mean, cov, NULL, &c);
    free(cnt);
    free(mean);
    free(cov);
    guesses[*iters] = guess;
    counts[*iters] = c;
    (*iters)++;
    if (c > k * (1 + 0.2)) {
      lo = guess;
    } else if (c < k) {
      hi = guess;
    } else {
      break;
    }
    guess = lo + (hi - lo) / 2.0;
    iter++;
  } while (iter < 15);
  *voxel_size = guess;
  return iter == 15 ? -3 : 0;
}
