/*
 * ndt_oracle.c -- CPU restatement of the reference NDT downsample path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the checker for the HIP path: only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 * The product (ndt-net_amd/) never links or calls it.
 *
 * It restates, sequentially and in point-index order (the single-worker
 * schedule of the reference), each step of
 * core_legacy/src/ndt.c:119-222 `ndt_downsample`:
 *   limits        pointclouds.c:40-66   (max starts at DBL_MIN)
 *   grid          voxel.c:61-81
 *   voxel index   voxel.c:83-103, 177-189
 *   estimate      normal_distributions.c:28-285 (Welford, order-dependent
 *                 off-diagonal, per-chunk abandon on an out-of-grid point,
 *                 n % 8 tail dropped)
 *   search        ndt.c:136-194
 *   KL            kullback_leibler.c:28-202 (in-place LU mutation, Mahalanobis
 *                 term 0, descending insertion)
 *   prune         ndt.c:28-73
 *   output        ndt.c:75-117
 * The GSL 2.7.1 routines the KL step calls (absent from this image: SURVEY
 * §8c) are restated from their published algorithm below (orc_lu_decomp etc.).
 * Parity pins: the estimate/search stages are checked bit-exactly against the
 * reference's own normal_distributions.c/voxel.c/pointclouds.c compiled into
 * oracle/_ref (oracle/Makefile); the KL/prune stages have no reference-side
 * pin (GSL absent; no reference test pins a KL value): "parity unpinned" for
 * them, see DESIGN.md.
 *
 * It also exports the reference's five legacy entry points (ndt.h:59-116,
 * kullback_leibler.h:74) so the reference's own ctypes driver
 * (ndnet/preprocessing/ndt_legacy.py) can be pointed at it when generating
 * fixtures in the build container.
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define NDNET_FN static inline
#include "../ndt-net_amd/csrc/ndt_log.h"

#define ORC_WORKERS 8            /* NUM_PCL_WORKERS, normal_distributions.h:39 */

/* Stage hooks: oracle/cpu_ref.c includes this file and swaps in the
 * reference-structured (threaded, mutex-per-voxel, heap-allocating) estimate
 * and KL call for its CPU baseline; the arithmetic stays this file's. */
#ifndef ORC_ESTIMATE
#define ORC_ESTIMATE orc_estimate
#endif
#ifndef ORC_KL_DIVERGENCE
#define ORC_KL_DIVERGENCE orc_kl_divergence
#endif
#define ORC_MIN_GUESS 0.01       /* ndt.h:41 */
#define ORC_MAX_GUESS 30.0       /* ndt.h:42 */
#define ORC_MAX_ITERS 15         /* ndt.h:43 */
#define ORC_UPPER 0.2            /* ndt.h:38 */

/* 0: glibc log (what the reference calls); 1: the portable log the HIP path uses. */
int orc_use_portable_log = 0;
static double orc_log(double x) { return orc_use_portable_log ? ndnet_log(x) : log(x); }

typedef struct orc_nd {
  uint64_t n;
  double mean[3];
  double m2[3];
  double cov[9];
  uint16_t cls;
  uint32_t* class_counts;
} orc_nd;

typedef struct orc_kl {
  double div;
  orc_nd* p;
  orc_nd* q;
} orc_kl;

/* ---------------- limits / grid / voxel index ---------------- */

/* pointclouds.c:40-66.  lim = {max_x, max_y, max_z, min_x, min_y, min_z}. */
void orc_limits(const double* pc, int dim, uint64_t n, double* lim) {
  double mx = DBL_MIN, my = DBL_MIN, mz = DBL_MIN;
  double nx = DBL_MAX, ny = DBL_MAX, nz = DBL_MAX;
  for (uint64_t i = 0; i < n; i++) {
    const double* p = pc + i * (uint64_t)dim;
    mx = p[0] > mx ? p[0] : mx;
    nx = p[0] < nx ? p[0] : nx;
    my = p[1] > my ? p[1] : my;
    ny = p[1] < ny ? p[1] : ny;
    mz = p[2] > mz ? p[2] : mz;
    nz = p[2] < nz ? p[2] : nz;
  }
  lim[0] = mx; lim[1] = my; lim[2] = mz;
  lim[3] = nx; lim[4] = ny; lim[5] = nz;
}

/* voxel.c:61-81 */
void orc_grid(const double* lim, double vs, int* len, double* off) {
  for (int a = 0; a < 3; a++) {
    double d = lim[a] - lim[3 + a];
    len[a] = (int)ceil(d / vs);
    off[a] = lim[3 + a];
  }
}

/* voxel.c:83-103 + 177-189: returns 0 and the linear index, or -1 when out of grid.
 * The double -> unsigned conversion follows x86-64 gcc (cvttsd2si, low 32 bits). */
static int orc_voxel_index(const double* p, double vs, const int* len, const double* off, uint64_t* idx) {
  unsigned v[3];
  for (int a = 0; a < 3; a++) {
    double f = floor((p[a] - off[a]) / vs);
    v[a] = (f != f) ? 0u : (unsigned)(int64_t)f;
  }
  for (int a = 0; a < 3; a++)
    if (v[a] >= (unsigned)len[a]) return -1;
  *idx = (uint64_t)(unsigned)(v[2] * (unsigned)len[0] * (unsigned)len[1] + v[1] * (unsigned)len[0] + v[0]);
  return 0;
}

/* ---------------- estimate (normal_distributions.c:139-285) ---------------- */

/* Per-voxel Welford update, normal_distributions.c:76-121. */
static void orc_update(orc_nd* nd, const double* x, const uint16_t* cls, int ncls) {
  nd->n++;
  const double n = (double)nd->n;
  double old[3];
  for (int j = 0; j < 3; j++) {
    old[j] = nd->mean[j];
    nd->mean[j] += (x[j] - nd->mean[j]) / n;
    nd->m2[j] += (x[j] - old[j]) * (x[j] - nd->mean[j]);
    nd->cov[j * 3 + j] = nd->m2[j] / n;
    if (isnan(nd->cov[j * 3 + j])) nd->cov[j * 3 + j] = 0.0;
    for (int k = j + 1; k < 3; k++) {
      nd->cov[j * 3 + k] += (x[j] - nd->mean[j]) * (x[k] - nd->mean[k]) / n;
      if (isnan(nd->cov[j * 3 + k])) nd->cov[j * 3 + k] = 0.0;
      nd->cov[k * 3 + j] = nd->cov[j * 3 + k];
    }
  }
  if (cls) {
    nd->class_counts[*cls]++;
    unsigned best = 0;
    for (int j = 0; j <= ncls; j++) {
      if (nd->class_counts[j] > best) {
        best = nd->class_counts[j];
        nd->cls = (uint16_t)j;
      }
    }
  }
}

/* Estimate with the canonical schedule: worker chunks [w*(n/8), (w+1)*(n/8)) in
 * order w = 0..7; a worker abandons the rest of its chunk at its first
 * out-of-grid point (normal_distributions.c:47-52).  nds must hold V entries. */
int orc_estimate(const double* pc, uint64_t n, const uint16_t* cls, int ncls, double vs, const int* len,
                 const double* off, orc_nd* nds, uint64_t* num_nds) {
  const uint64_t V = (uint64_t)(unsigned)len[0] * (unsigned)len[1] * (unsigned)len[2];
  for (uint64_t v = 0; v < V; v++) {
    memset(&nds[v], 0, sizeof(orc_nd));
    if (cls) {
      nds[v].class_counts = (uint32_t*)calloc((size_t)ncls + 1, sizeof(uint32_t));
      if (!nds[v].class_counts) return -1;
    }
  }
  const uint64_t chunk = n / ORC_WORKERS;
  for (int w = 0; w < ORC_WORKERS; w++) {
    for (uint64_t i = (uint64_t)w * chunk; i < (uint64_t)(w + 1) * chunk; i++) {
      uint64_t idx;
      if (orc_voxel_index(pc + 3 * i, vs, len, off, &idx) < 0) break;
      orc_update(&nds[idx], pc + 3 * i, cls ? cls + i : NULL, ncls);
    }
  }
  uint64_t c = 0;
  for (uint64_t v = 0; v < V; v++) c += nds[v].n > 0;
  *num_nds = c;
  return 0;
}

static void orc_free_class_counts(orc_nd* nds, uint64_t V) {
  for (uint64_t v = 0; v < V; v++) {
    free(nds[v].class_counts);
    nds[v].class_counts = NULL;
  }
}

/* ---------------- search (ndt.c:131-194) ---------------- */

typedef struct orc_search_t {
  int rc;                    /* 0 or -3 (iteration cap), -1 (allocation) */
  int iters;                 /* estimate passes run */
  double guesses[ORC_MAX_ITERS];
  uint64_t counts[ORC_MAX_ITERS];
  double lim[6];
  int len[3];
  double off[3];
  double voxel_size;
  uint64_t num_nds;
} orc_search_t;

/* Runs the bisection.  On success *nds_out holds the accepted estimate (V entries). */
static int orc_search_impl(const double* pc, int dim, uint64_t n, const uint16_t* cls, int ncls, uint64_t k,
                           orc_search_t* s, orc_nd** nds_out) {
  memset(s, 0, sizeof(*s));
  orc_limits(pc, dim, n, s->lim);
  double guess = (ORC_MAX_GUESS - ORC_MIN_GUESS) / 2.0;
  double lo = ORC_MIN_GUESS, hi = ORC_MAX_GUESS;
  unsigned iter = 0;
  *nds_out = NULL;
  do {
    orc_grid(s->lim, guess, s->len, s->off);
    const uint64_t V = (uint64_t)(unsigned)s->len[0] * (unsigned)s->len[1] * (unsigned)s->len[2];
    orc_nd* nds = (orc_nd*)malloc((V ? V : 1) * sizeof(orc_nd));
    if (!nds) { s->rc = -1; return -1; }
    uint64_t c = 0;
    if (ORC_ESTIMATE(pc, n, cls, ncls, guess, s->len, s->off, nds, &c) < 0) {
      orc_free_class_counts(nds, V);
      free(nds);
      s->rc = -2;
      return -2;
    }
    s->guesses[s->iters] = guess;
    s->counts[s->iters] = c;
    s->iters++;
    if ((double)c > (double)k * (1 + ORC_UPPER)) {
      lo = guess;
    } else if (c < k) {
      hi = guess;
    } else {
      s->num_nds = c;
      *nds_out = nds;
      break;
    }
    orc_free_class_counts(nds, V);
    free(nds);
    guess = lo + (hi - lo) / 2.0;
    iter++;
  } while (iter < ORC_MAX_ITERS);
  s->voxel_size = guess;
  if (iter == ORC_MAX_ITERS) { s->rc = -3; return -3; }
  s->rc = 0;
  return 0;
}

int orc_search(const double* pc, int dim, uint64_t n, uint64_t k, orc_search_t* s) {
  orc_nd* nds = NULL;
  int rc = orc_search_impl(pc, dim, n, NULL, 0, k, s, &nds);
  if (nds) free(nds);
  return rc;
}

int orc_search_struct_size(void) { return (int)sizeof(orc_search_t); }

/* ---------------- GSL 2.7.1 restatement (3x3) ---------------- */
/* gsl_linalg_LU_decomp -> LU_decomp_L3 -> LU_decomp_L2 (N <= CROSSOVER_LU),
 * with gslcblas idamax (first max |x|), dswap, dscal(1/Ajj) and dger(-1). */
static void orc_lu_decomp(double* A, int* perm, int* signum) {
  const int N = 3;
  int ipiv[3];
  for (int j = 0; j < N; j++) {
    /* idamax over column j, rows j..N-1 */
    double mx = 0.0;
    int r = 0;
    for (int i = 0; i < N - j; i++) {
      double a = fabs(A[(j + i) * 3 + j]);
      if (a > mx) { mx = a; r = i; }
    }
    const int jp = j + r;
    ipiv[j] = jp;
    if (jp != j)
      for (int c = 0; c < N; c++) {
        double t = A[j * 3 + c];
        A[j * 3 + c] = A[jp * 3 + c];
        A[jp * 3 + c] = t;
      }
    if (j < N - 1) {
      const double ajj = A[j * 3 + j];
      if (fabs(ajj) >= DBL_MIN) {
        const double s = 1.0 / ajj;
        for (int i = j + 1; i < N; i++) A[i * 3 + j] = s * A[i * 3 + j];
      } else {
        for (int i = j + 1; i < N; i++) A[i * 3 + j] /= ajj;
      }
    }
    if (j < N - 1) {
      /* dger(-1, A[j+1:, j], A[j, j+1:], A22): row-major, i outer */
      for (int i = j + 1; i < N; i++) {
        const double tmp = -1.0 * A[i * 3 + j];
        for (int c = j + 1; c < N; c++) A[i * 3 + c] += A[j * 3 + c] * tmp;
      }
    }
  }
  for (int i = 0; i < N; i++) perm[i] = i;
  *signum = 1;
  for (int i = 0; i < N; i++) {
    const int pi = ipiv[i];
    if (perm[i] != perm[pi]) {
      int t = perm[i];
      perm[i] = perm[pi];
      perm[pi] = t;
      *signum = -*signum;
    }
  }
}

static double orc_lu_det(const double* LU, int signum) {
  double d = (double)signum;
  for (int i = 0; i < 3; i++) d *= LU[i * 3 + i];
  return d;
}

static int orc_lu_sgndet(const double* LU, int signum) {
  int s = signum;
  for (int i = 0; i < 3; i++) {
    const double u = LU[i * 3 + i];
    if (u < 0) s *= -1;
    else if (u == 0) { s = 0; break; }
  }
  return s;
}

/* Variant: inverse from the LU factors column by column (b = P e_j, then
 * gslcblas dtrsv lower-unit forward and upper-nonunit back substitution).
 * This is what round 1 used; it rounds differently from GSL 2.7.1's
 * LU_invert (below) by <= 3.7e-13 relative on a KL score.
 * Selected by orc_use_gsl_invert = 0, for A/B comparisons only. */
static void orc_lu_invert_columns(const double* LU, const int* perm, double* inv) {
  for (int j = 0; j < 3; j++) {
    double x[3];
    for (int i = 0; i < 3; i++) x[i] = (perm[i] == j) ? 1.0 : 0.0;
    for (int i = 1; i < 3; i++) {
      double t = x[i];
      for (int c = 0; c < i; c++) t -= LU[i * 3 + c] * x[c];
      x[i] = t;
    }
    x[2] = x[2] / LU[2 * 3 + 2];
    for (int i = 1; i >= 0; i--) {
      double t = x[i];
      for (int c = i + 1; c < 3; c++) t -= LU[i * 3 + c] * x[c];
      x[i] = t / LU[i * 3 + i];
    }
    for (int i = 0; i < 3; i++) inv[i * 3 + j] = x[i];
  }
}

/* ---- GSL 2.7.1 gsl_linalg_LU_invert, as published (the reference's call at
 * kullback_leibler.c:92; GSL version inferred).  linalg/lu.c:
 * LU_invert = memcpy(inverse, LU) + gsl_linalg_LU_invx(inverse, p), which is
 *   tri_invert(Upper, NonUnit); tri_invert(Lower, Unit); tri_UL; then
 *   gsl_permute_vector_inverse(p, row i) for every row.
 * linalg/tri.c runs the Level-2 forms for N = 3 (below the Level-3
 * crossover); the BLAS calls are gslcblas's (cblas/source_*_r.h) and are
 * restated with their loop orders below.  Row-major T, leading dim 3. */

/* gslcblas dtrmv, RowMajor, NoTrans, on the n x n block at T (ld 3), x stride sx */
static void orc_trmv(int upper, int nonunit, int n, const double* T, double* x, int sx) {
  if (upper) {
    for (int i = 0; i < n; i++) {
      double temp = 0.0;
      for (int j = i + 1; j < n; j++) temp += x[j * sx] * T[3 * i + j];
      if (nonunit) x[i * sx] = temp + x[i * sx] * T[3 * i + i];
      else x[i * sx] += temp;
    }
  } else {
    for (int i = n - 1; i >= 0; i--) {
      double temp = 0.0;
      for (int j = 0; j < i; j++) temp += x[j * sx] * T[3 * i + j];
      if (nonunit) x[i * sx] = temp + x[i * sx] * T[3 * i + i];
      else x[i * sx] += temp;
    }
  }
}

static void orc_scal(int n, double alpha, double* x, int sx) {
  for (int i = 0; i < n; i++) x[i * sx] *= alpha;
}

/* linalg/tri.c triangular_inverse_L2 */
static void orc_tri_invert_L2(int upper, int nonunit, double* T) {
  const int N = 3;
  if (upper) {
    for (int i = 0; i < N; i++) {
      double aii;
      if (nonunit) {
        T[3 * i + i] = 1.0 / T[3 * i + i];
        aii = -T[3 * i + i];
      } else {
        aii = -1.0;
      }
      if (i > 0) {
        orc_trmv(1, nonunit, i, T, &T[i], 3);          /* m = T[0:i,0:i], v = T[0:i, i] */
        orc_scal(i, aii, &T[i], 3);
      }
    }
  } else {
    for (int i = 0; i < N; i++) {
      const int j = N - i - 1;
      double ajj;
      if (nonunit) {
        T[3 * j + j] = 1.0 / T[3 * j + j];
        ajj = -T[3 * j + j];
      } else {
        ajj = -1.0;
      }
      if (j < N - 1) {
        const int m = N - j - 1;
        orc_trmv(0, nonunit, m, &T[3 * (j + 1) + (j + 1)], &T[3 * (j + 1) + j], 3);
        orc_scal(m, ajj, &T[3 * (j + 1) + j], 3);
      }
    }
  }
}

/* linalg/tri.c triangular_mult_L2, Upper: A <- U L (U upper, L unit lower).
 * (gcc -O2 warns about indices of loop trips that i < N - 1 excludes.) */
#pragma GCC diagnostic push
#pragma GCC diagnostic ignored "-Warray-bounds"
static void orc_tri_UL_L2(double* A) {
  const int N = 3;
  for (int i = 0; i < N; i++) {
    double* Aii = &A[3 * i + i];
    const double aii = *Aii;
    if (i < N - 1) {
      const int m = N - i - 1;
      /* ddot(lb = A[i+1:, i], ur = A[i, i+1:]) */
      double tmp = 0.0;
      for (int k = 0; k < m; k++) tmp += A[3 * (i + 1 + k) + i] * A[3 * i + (i + 1 + k)];
      *Aii += tmp;
      if (i > 0) {
        /* dgemv(Trans, 1.0, L_BL = A[i+1:, 0:i], ur, aii, lr = A[i, 0:i]) */
        for (int c = 0; c < i; c++) {
          double* y = &A[3 * i + c];
          if (aii == 0.0) *y = 0.0;
          else if (aii != 1.0) *y *= aii;
        }
        for (int r = 0; r < m; r++) {
          const double temp = 1.0 * A[3 * i + (i + 1 + r)];
          if (temp != 0.0)
            for (int c = 0; c < i; c++) A[3 * i + c] += temp * A[3 * (i + 1 + r) + c];
        }
        /* dgemv(NoTrans, 1.0, U_TR = A[0:i, i+1:], lb, 1.0, ut = A[0:i, i]) */
        for (int r = 0; r < i; r++) {
          double temp = 0.0;
          for (int c = 0; c < m; c++) temp += A[3 * (i + 1 + c) + i] * A[3 * r + (i + 1 + c)];
          A[3 * r + i] += 1.0 * temp;
        }
      }
    } else {
      /* the last row's L part (A[N-1, 0:N-1]) times a_NN */
      orc_scal(N - 1, aii, &A[3 * (N - 1)], 1);
    }
  }
}

#pragma GCC diagnostic pop

static void orc_lu_invert_gsl(const double* LU, const int* perm, double* inv) {
  double A[9];
  memcpy(A, LU, sizeof(A));
  orc_tri_invert_L2(1, 1, A);  /* U^-1 */
  orc_tri_invert_L2(0, 0, A);  /* L^-1, unit diagonal */
  orc_tri_UL_L2(A);            /* U^-1 L^-1 */
  /* gsl_permute_vector_inverse(p, row): row[p[k]] <- row[k] */
  for (int r = 0; r < 3; r++)
    for (int k = 0; k < 3; k++) inv[3 * r + perm[k]] = A[3 * r + k];
}

int orc_use_gsl_invert = 1;

static void orc_lu_invert(const double* LU, const int* perm, double* inv) {
  if (orc_use_gsl_invert) orc_lu_invert_gsl(LU, perm, inv);
  else orc_lu_invert_columns(LU, perm, inv);
}

/* test hook: one inverse through the selected variant */
void orc_lu_invert_test(const double* A, double* LU_out, int* perm_out, double* inv, int variant) {
  double LU[9];
  int perm[3], sg;
  memcpy(LU, A, sizeof(LU));
  orc_lu_decomp(LU, perm, &sg);
  if (variant) orc_lu_invert_gsl(LU, perm, inv);
  else orc_lu_invert_columns(LU, perm, inv);
  memcpy(LU_out, LU, sizeof(LU));
  for (int i = 0; i < 3; i++) perm_out[i] = perm[i];
}

/* kullback_leibler.c:28-127.  Returns -1 (n<=1, div 0, no mutation), -2 (singular,
 * mutation done, no event) or 0. */
static int orc_kl_divergence(orc_nd* p, orc_nd* q, double* div) {
  *div = 0;
  if (p->n <= 1 || q->n <= 1) return -1;
  int pperm[3], qperm[3], ps, qs;
  orc_lu_decomp(p->cov, pperm, &ps);
  orc_lu_decomp(q->cov, qperm, &qs);
  const double pd = orc_lu_det(p->cov, ps);
  const double qd = orc_lu_det(q->cov, qs);
  if (pd == 0 || qd == 0) return -2;
  if (orc_lu_sgndet(p->cov, ps) == 0 || orc_lu_sgndet(q->cov, qs) == 0) return -2;
  double qinv[9];
  orc_lu_invert(q->cov, qperm, qinv);
  /* gslcblas dgemm, beta = 0: C zeroed, then C[i][j] += (1*A[i][k]) * B[k][j] for
   * A[i][k] != 0.  Only the diagonal is used. */
  double tr = 0;
  for (int i = 0; i < 3; i++) {
    double cii = 0.0;
    for (int kk = 0; kk < 3; kk++) {
      const double t = 1.0 * qinv[i * 3 + kk];
      if (t != 0.0) cii += t * p->cov[kk * 3 + i];
    }
    tr += cii;
  }
  /* first_part aliases A and C in dgemm (kullback_leibler.c:105): zeroed -> 0. */
  const double first = 0.0;
  *div = 0.5 * (first + tr - orc_log(qd / pd) - 3);
  return 0;
}

/* kullback_leibler.c:129-202.  Also records events in enumeration order
 * (ev_* arrays, may be NULL) for stage-wise parity. */
static int orc_neighbor(uint64_t idx, const int* len, int d, uint64_t* nb) {
  const unsigned lx = (unsigned)len[0], ly = (unsigned)len[1], lz = (unsigned)len[2];
  unsigned z = (unsigned)(idx / ((uint64_t)lx * ly));
  unsigned y = (unsigned)((idx % ((uint64_t)lx * ly)) / lx);
  unsigned x = (unsigned)(idx % lx);
  static const int dx[6] = {1, -1, 0, 0, 0, 0}, dy[6] = {0, 0, 1, -1, 0, 0}, dz[6] = {0, 0, 0, 0, 1, -1};
  x += (unsigned)dx[d];
  y += (unsigned)dy[d];
  z += (unsigned)dz[d];
  if (x >= lx || y >= ly || z >= lz) return -4;
  *nb = (uint64_t)(unsigned)(z * lx * ly + y * lx + x);
  return 0;
}

static int orc_kl_all(orc_nd* nds, const int* len, uint64_t* num_valid, orc_kl* kl, uint64_t* nkl, double* ev_div,
                      int64_t* ev_p, int64_t* ev_q, int32_t* ev_rc, uint64_t* nev) {
  const uint64_t V = (uint64_t)(unsigned)len[0] * (unsigned)len[1] * (unsigned)len[2];
  *num_valid = 0;
  *nkl = 0;
  uint64_t e = 0;
  for (uint64_t v = 0; v < V; v++) {
    if (nds[v].n == 0) continue;
    (*num_valid)++;
    for (int d = 0; d < 6; d++) {
      uint64_t w;
      if (orc_neighbor(v, len, d, &w) < 0) continue;
      if (nds[w].n == 0) continue;
      double div = 0;
      const int rc = ORC_KL_DIVERGENCE(&nds[v], &nds[w], &div);
      if (ev_div) {
        ev_div[e] = div;
        ev_p[e] = (int64_t)v;
        ev_q[e] = (int64_t)w;
        ev_rc[e] = rc;
      }
      e++;
      if (rc == -2) continue;
      uint64_t j = 0;
      while (j < *nkl) {
        if (kl[j].div < div) break;
        j++;
      }
      for (uint64_t m = *nkl; m > j; m--) kl[m] = kl[m - 1];
      kl[j].div = div;
      kl[j].p = &nds[v];
      kl[j].q = &nds[w];
      (*nkl)++;
    }
  }
  if (nev) *nev = e;
  return 0;
}

/* ndt.c:28-73, including its quirks: the bound check compares against the
 * decremented count, and the array shift can read past the old count. */
static int orc_prune(orc_nd* nds, uint64_t k, uint64_t* num_valid, orc_kl* kl, uint64_t* nkl, uint64_t kl_cap) {
  (void)nds;
  if (k > *num_valid) return -1;
  const unsigned to_remove = (unsigned)(*num_valid - k);
  uint64_t idx = 0;
  for (uint64_t i = 0; i < to_remove; idx++) {
    if (idx >= *nkl) return -2;
    if (kl[idx].p == NULL) return -8; /* an entry never written (the reference reads garbage) */
    if (kl[idx].p->n == 0) continue;
    kl[idx].p->n = 0;
    (*num_valid)--;
    (*nkl)--;
    i++;
  }
  for (uint64_t i = 0; i < *nkl; i++) {
    if (i + idx < kl_cap) kl[i] = kl[i + idx];
    else { kl[i].div = NAN; kl[i].p = NULL; kl[i].q = NULL; }
  }
  return 0;
}

/* ndt.c:75-117, writing at most cap rows (the reference has no capacity and
 * overruns its k-row buffers when more than k NDs survive). */
static uint64_t orc_to_point_cloud(const orc_nd* nds, const int* len, double* pc, double* cov, uint16_t* cls,
                                   uint64_t cap) {
  const uint64_t V = (uint64_t)(unsigned)len[0] * (unsigned)len[1] * (unsigned)len[2];
  uint64_t m = 0;
  for (uint64_t v = 0; v < V; v++) {
    if (nds[v].n == 0) continue;
    if (m < cap) {
      memcpy(pc + 3 * m, nds[v].mean, 3 * sizeof(double));
      memcpy(cov + 9 * m, nds[v].cov, 9 * sizeof(double));
      if (cls) cls[m] = nds[v].cls;
    }
    m++;
  }
  return m;
}

/* ---------------- stage-wise entry point for the tests ---------------- */

/* Full path with every intermediate exposed.  Arrays sized by the caller:
 *   per voxel (vcap):  vox_n, vox_mean[3], vox_cov_pre[9], vox_cov_post[9], vox_cls, vox_kept
 *   per event (ecap):  ev_div/ev_p/ev_q/ev_rc (enumeration order), ord_div/ord_p/ord_q (final order)
 * Returns the ndt_downsample code; *nvox = V, *nev = enumerated events, *nord = kept
 * list length, *nout = survivors (rows written <= k). */
int orc_run(const double* pc, uint64_t n, const uint16_t* cls, int ncls, uint64_t k, orc_search_t* s, uint64_t vcap,
            uint64_t* vox_n, double* vox_mean, double* vox_cov_pre, double* vox_cov_post, uint16_t* vox_cls,
            uint8_t* vox_kept, uint64_t ecap, double* ev_div, int64_t* ev_p, int64_t* ev_q, int32_t* ev_rc,
            double* ord_div, int64_t* ord_p, int64_t* ord_q, uint64_t* nvox, uint64_t* nev, uint64_t* nord,
            int* prune_rc, uint64_t* num_valid_out, double* out_pc, double* out_cov, uint16_t* out_cls,
            uint64_t* nout, double* post_div, int64_t* post_p, int64_t* post_q, uint64_t* post_nkl) {
  orc_nd* nds = NULL;
  *nvox = *nev = *nord = *nout = 0;
  int rc = orc_search_impl(pc, 3, n, cls, ncls, k, s, &nds);
  if (rc < 0) return rc;
  const uint64_t V = (uint64_t)(unsigned)s->len[0] * (unsigned)s->len[1] * (unsigned)s->len[2];
  *nvox = V;
  if (V > vcap || 6 * V > ecap) {
    orc_free_class_counts(nds, V);
    free(nds);
    return -100;
  }
  for (uint64_t v = 0; v < V; v++) {
    vox_n[v] = nds[v].n;
    memcpy(vox_mean + 3 * v, nds[v].mean, 24);
    memcpy(vox_cov_pre + 9 * v, nds[v].cov, 72);
    vox_cls[v] = nds[v].cls;
  }
  orc_kl* kl = (orc_kl*)calloc((V ? V : 1) * 6, sizeof(orc_kl)); /* p == NULL marks never-written entries */
  uint64_t num_valid = 0, nkl = 0;
  orc_kl_all(nds, s->len, &num_valid, kl, &nkl, ev_div, ev_p, ev_q, ev_rc, nev);
  for (uint64_t i = 0; i < nkl; i++) {
    ord_div[i] = kl[i].div;
    ord_p[i] = kl[i].p - nds;
    ord_q[i] = kl[i].q - nds;
  }
  *nord = nkl;
  *prune_rc = orc_prune(nds, k, &num_valid, kl, &nkl, 6 * V);
  *num_valid_out = num_valid;
  /* the physical list after the prune's left shift, first *nord entries */
  for (uint64_t i = 0; i < *nord; i++) {
    post_div[i] = kl[i].div;
    post_p[i] = kl[i].p ? kl[i].p - nds : -1;
    post_q[i] = kl[i].q ? kl[i].q - nds : -1;
  }
  *post_nkl = nkl;
  for (uint64_t v = 0; v < V; v++) {
    memcpy(vox_cov_post + 9 * v, nds[v].cov, 72);
    vox_kept[v] = nds[v].n > 0;
  }
  *nout = orc_to_point_cloud(nds, s->len, out_pc, out_cov, out_cls, k);
  free(kl);
  orc_free_class_counts(nds, V);
  free(nds);
  return 0;
}

/* ---------------- the reference's legacy ABI (ndt.h, kullback_leibler.h) ---------------- */

int prune_nds(orc_nd* nd_array, unsigned lx, unsigned ly, unsigned lz, unsigned long k, unsigned long* num_valid,
              orc_kl* kl, unsigned long* nkl) {
  (void)lx; (void)ly; (void)lz;
  uint64_t nv = *num_valid, nk = *nkl;
  /* the shift reads past the live count; the handle was allocated with 6V entries */
  const uint64_t cap = (uint64_t)lx * ly * lz * 6;
  int rc = orc_prune(nd_array, k, &nv, kl, &nk, cap);
  *num_valid = nv;
  *nkl = nk;
  return rc;
}

int to_point_cloud(orc_nd* nd_array, unsigned lx, unsigned ly, unsigned lz, double ox, double oy, double oz,
                   double vs, double* pc, unsigned long* num_points, double* cov, unsigned short* classes) {
  (void)ox; (void)oy; (void)oz; (void)vs;
  int len[3] = {(int)lx, (int)ly, (int)lz};
  /* the caller sized its buffers for *num_points rows at most; the reference has
   * no capacity argument, so the legacy entry writes every survivor */
  *num_points = orc_to_point_cloud(nd_array, len, pc, cov, classes, UINT64_MAX);
  return 0;
}

int ndt_downsample(double* pc, unsigned short dim, unsigned long n, unsigned* lx, unsigned* ly, unsigned* lz,
                   double* ox, double* oy, double* oz, double* vs, unsigned short* classes, unsigned short ncls,
                   unsigned long k, double* out_pc, unsigned long* out_n, double* out_cov,
                   unsigned short* out_classes, orc_nd** nd_array, unsigned long* num_valid, orc_kl** kl,
                   unsigned long* nkl) {
  orc_search_t s;
  orc_nd* nds = NULL;
  *nd_array = NULL;
  *kl = NULL;
  int rc = orc_search_impl(pc, dim, n, classes, ncls, k, &s, &nds);
  *lx = (unsigned)s.len[0];
  *ly = (unsigned)s.len[1];
  *lz = (unsigned)s.len[2];
  *ox = s.off[0];
  *oy = s.off[1];
  *oz = s.off[2];
  *vs = s.voxel_size;
  if (rc < 0) return rc;
  const uint64_t V = (uint64_t)(*lx) * (*ly) * (*lz);
  orc_kl* list = (orc_kl*)calloc((V ? V : 1) * 6, sizeof(orc_kl));
  if (!list) return -4;
  uint64_t nv = 0, nk = 0;
  orc_kl_all(nds, s.len, &nv, list, &nk, NULL, NULL, NULL, NULL, NULL);
  orc_prune(nds, k, &nv, list, &nk, 6 * V);
  *num_valid = nv;
  *nkl = nk;
  *out_n = orc_to_point_cloud(nds, s.len, out_pc, out_cov, out_classes, k);
  *nd_array = nds;
  *kl = list;
  return 0;
}

void free_nds(orc_nd* nd_array, unsigned long num_nds) {
  if (!nd_array) return;
  orc_free_class_counts(nd_array, num_nds);
  free(nd_array);
}

void free_kl_divergences(orc_kl* kl) { free(kl); }

/* portable log, exposed for tests/test_log.py */
double orc_portable_log(double x) { return ndnet_log(x); }
void orc_portable_log_many(const double* x, double* y, uint64_t n) {
  for (uint64_t i = 0; i < n; i++) y[i] = ndnet_log(x[i]);
}
void orc_libm_log_many(const double* x, double* y, uint64_t n) {
  for (uint64_t i = 0; i < n; i++) y[i] = log(x[i]);
}

/* The point generator of the reference's smoke test core_legacy/tests/
 * ndt_downsample.c:21-27: srand(seed) once, then (double)rand() / RAND_MAX. */
void orc_glibc_rand_points(double* out, uint64_t count, unsigned seed, int reseed) {
  if (reseed) srand(seed);
  for (uint64_t i = 0; i < count; i++) out[i] = (double)rand() / RAND_MAX;
}

/* The division rule of the device's long-ND Welford path (k_welford_q,
 * wq_heavy): t / n as fma(t, rc, t * rl) with rc = 1.0 / n and
 * rl = fma(-n, rc, 1.0) / n.  Returns how many of `samples` random (t, n)
 * pairs -- t over the operand range the fast path admits (2^-360 .. 2^302,
 * both signs, random and few-bit mantissas), n in 1 .. n_max plus powers of
 * two and their neighbours -- differ from the IEEE division t / n in any bit.
 * Test infrastructure (tests/test_oracle.py). */
static uint64_t rtab_rng(uint64_t* s) {
  *s ^= *s << 13;
  *s ^= *s >> 7;
  *s ^= *s << 17;
  return *s;
}
uint64_t orc_rtab_div_mismatches(uint64_t n_max, uint64_t samples, uint64_t seed) {
  uint64_t s = seed * 0x9E3779B97F4A7C15ull + 1, bad = 0;
  for (uint64_t i = 0; i < samples; i++) {
    uint64_t r = rtab_rng(&s);
    uint64_t n;
    switch (r & 3) {
      case 0: { const int k = (int)((r >> 2) % 32); n = (1ull << k) + ((r >> 8) % 3) - 1; if (!n) n = 1; break; }
      default: n = 1 + (r >> 2) % n_max;
    }
    r = rtab_rng(&s);
    uint64_t mant = (r >> 11) | (1ull << 52);
    if ((r & 7) == 0) mant = ((r >> 3) & 0xffff) | 1;             /* few significant bits */
    else if ((r & 7) == 1) mant = (1ull << 52) | ((r >> 3) & 0xf); /* near a power of two */
    const int e = -360 + (int)(rtab_rng(&s) % 662);
    double t = ldexp((double)mant, e - 52);
    if (r & 8) t = -t;
    const double dn = (double)n, rc = 1.0 / dn, rl = fma(-dn, rc, 1.0) / dn;
    const double q = fma(t, rc, t * rl), ref = t / dn;
    if (memcmp(&q, &ref, sizeof q) != 0 && !(q == 0.0 && ref == 0.0)) bad++;
  }
  return bad;
}

/* The in-place LU chain of one ND: `steps` successive
 * gsl_linalg_LU_decomp calls on the same matrix, recording every state
 * (9 doubles), its permutation | (signum < 0) << 8 packed as the device packs
 * it (p0 | p1 << 2 | p2 << 4), and the event flag kl_divergence reads of it
 * (det != 0 and sgndet != 0, kullback_leibler.c:57-70).  n matrices. */
void orc_lu_chain(const double* A, uint64_t n, int steps, double* states, uint32_t* ps, uint32_t* flags) {
  for (uint64_t m = 0; m < n; m++) {
    double S[9];
    memcpy(S, A + 9 * m, sizeof S);
    for (int t = 0; t < steps; t++) {
      int perm[3], sg;
      orc_lu_decomp(S, perm, &sg);
      memcpy(states + (m * steps + t) * 9, S, sizeof S);
      ps[m * steps + t] = (uint32_t)perm[0] | ((uint32_t)perm[1] << 2) | ((uint32_t)perm[2] << 4) | (sg < 0 ? 0x100u : 0u);
      flags[m * steps + t] = (orc_lu_det(S, sg) != 0 && orc_lu_sgndet(S, sg) != 0) ? 1u : 0u;
    }
  }
}
