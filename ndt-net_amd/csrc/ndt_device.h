// Device-side arithmetic of the NDT path (gfx950).  Every function here performs
// the same IEEE double operations, in the same order, as the reference C core
// on x86-64 without FMA; the translation unit is compiled with
// -ffp-contract=off so no multiply-add is fused.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define NDNET_FN __device__ static inline
#define NDNET_TABQ __constant__
#include "ndt_log.h"

namespace ndnet {

constexpr uint32_t kInvalid = 0xffffffffu;
constexpr int kWorkers = 8;          // NUM_PCL_WORKERS, normal_distributions.h:39
constexpr int kMaxIters = 15;        // MAX_GUESS_ITERATIONS, ndt.h:43
constexpr double kMinGuess = 0.01;   // ndt.h:41
constexpr double kMaxGuess = 30.0;   // ndt.h:42
constexpr double kUpper = 0.2;       // DOWNSAMPLE_UPPER_THRESHOLD, ndt.h:38
constexpr double kDblMin = 2.2250738585072014e-308;
constexpr double kDblMax = 1.7976931348623157e308;

// Order-preserving map of a double onto u64 (NaN excluded by the callers).
NDNET_FN uint64_t ord_key(double x) {
  uint64_t u = ndnet_dbits(x);
  return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}
NDNET_FN double ord_unkey(uint64_t k) {
  return ndnet_bitsd((k >> 63) ? (k & 0x7fffffffffffffffull) : ~k);
}

// (unsigned int) floor(x) as x86-64 gcc lowers it (cvttsd2si to 64 bits, low
// half kept): NaN and |x| >= 2^63 give 0.  voxel.c:89-91.
NDNET_FN uint32_t floor_to_u32(double f) {
  if (!(f > -9.2233720368547758e18 && f < 9.2233720368547758e18)) return 0u;
  return (uint32_t)(uint64_t)(int64_t)f;
}

// One axis of metric_to_voxel_space (voxel.c:89-91): floor((p - off) / vs).
// The quotient is first estimated with a multiply by 1/vs; only when that
// estimate lies within a few ulps of an integer is the correctly rounded
// division performed, so the floor always equals the reference's.
NDNET_FN uint32_t axis_index(double p, double off, double vs, double inv_vs) {
  const double d = p - off;
  const double qa = d * inv_vs;
  const double f = floor(qa);
  const double r = qa - f;
  const double tol = fabs(qa) * 0x1p-46 + 0x1p-60;
  if (r > tol && r < 1.0 - tol) return floor_to_u32(f);
  return floor_to_u32(floor(d / vs));
}

// Fast path of one axis of metric_to_voxel_space: the floor of d * (1/vs)
// where that product lies safely away from an integer and the floor fits an
// int32 (then it equals the reference's floor of the division and its
// unsigned conversion); *ok is false otherwise and the caller takes the
// exact path.
NDNET_FN uint32_t axis_index_fast(double p, double off, double inv_vs, bool& ok) {
  const double d = p - off;
  const double qa = d * inv_vs;
  const double f = floor(qa);
  const double r = qa - f;
  const double tol = fabs(qa) * 0x1p-46 + 0x1p-60;
  ok = r > tol && r < 1.0 - tol && f >= -2147483648.0 && f < 2147483648.0;
  return (uint32_t)(int32_t)(ok ? f : 0.0);
}

// voxel.c:83-103 + 177-189.  Returns kInvalid when the point is out of grid.
// The exact division runs behind a wave-uniform branch, only when some lane
// of the wave needs it, so the common case issues no double division.
NDNET_FN uint32_t voxel_key(double x, double y, double z, const double* off, const uint32_t* len, double vs,
                            double inv_vs) {
  bool o0, o1, o2;
  uint32_t vx = axis_index_fast(x, off[0], inv_vs, o0);
  uint32_t vy = axis_index_fast(y, off[1], inv_vs, o1);
  uint32_t vz = axis_index_fast(z, off[2], inv_vs, o2);
  const bool ok = o0 && o1 && o2;
  if (!__all(ok)) {
    if (!ok) {
      vx = axis_index(x, off[0], vs, inv_vs);
      vy = axis_index(y, off[1], vs, inv_vs);
      vz = axis_index(z, off[2], vs, inv_vs);
    }
  }
  if (vx >= len[0] || vy >= len[1] || vz >= len[2]) return kInvalid;
  return vz * len[0] * len[1] + vy * len[0] + vx;
}

// Single-precision screen of voxel_key for float points (the reference casts
// them to double, ndtnet_preprocessing.py:30).  off32 = the float-exact grid
// offset, inv32 = (float)(1 / vs).  The computed q = fl(fl(p - off) * inv32)
// is within 3 * 2^-24 |Q| (plus 2^-53 terms) of the real quotient
// Q = (p - off) / vs, and the reference's fl64(fl64(p - off) / vs) within
// 2^-52 |Q|; so where frac(q) is more than |q| 2^-19 away from 0 and 1, both
// floor to the same integer.  Otherwise (including q = 0 and NaN) the caller
// takes voxel_key.  (axis_index_f32 is the per-axis form, kept for tests.)
NDNET_FN uint32_t axis_index_f32(float p, float off32, float inv32, bool& ok) {
  const float q = (p - off32) * inv32;
  const float f = floorf(q);
  const float r = q - f;
  const float tol = q * 0x1p-19f;
  ok = r > tol && r < 1.0f - tol && q < 8388608.0f;
  return (uint32_t)(int32_t)(ok ? f : 0.0f);
}

constexpr uint32_t kKeyRedo = 0xfffffffeu;  // voxel_key_f32: take voxel_key for this point

// voxel_key for a float point, or kKeyRedo where the screen cannot decide.
// No fallback inside, so callers can keep the (rare) double path out of
// their unrolled hot loops.  tol32 = max(len) * 2^-19 >= q * 2^-19 for every
// in-grid q (a point whose q is past the grid either floors past len, and is
// out of grid in the reference too, or sits within tol32 of len and is
// redone): the per-axis screen is |frac(q) - 1/2| < 1/2 - tol32, no per-point
// tolerance product, and the in-grid test is on the float floor.
NDNET_FN uint32_t voxel_key_f32(float x, float y, float z, const float* off32, float inv32, float half_tol,
                                const float* lenf, const uint32_t* len) {
  const float qx = (x - off32[0]) * inv32, qy = (y - off32[1]) * inv32, qz = (z - off32[2]) * inv32;
  const float fx = floorf(qx), fy = floorf(qy), fz = floorf(qz);
  // branch-free (selects, no exec-mask regions in the caller's unrolled loop)
  const bool ok = ((int)(fabsf(qx - fx - 0.5f) < half_tol) & (int)(fabsf(qy - fy - 0.5f) < half_tol) &
                   (int)(fabsf(qz - fz - 0.5f) < half_tol)) != 0;
  const bool in = ((int)(fx < lenf[0]) & (int)(fy < lenf[1]) & (int)(fz < lenf[2])) != 0;
  const uint32_t k = ((uint32_t)fz * len[1] + (uint32_t)fy) * len[0] + (uint32_t)fx;
  return ok ? (in ? k : kInvalid) : kKeyRedo;
}

// x / n with the reciprocal of n shared between divisions.  The compiler's
// correctly rounded f64 division is the sequence
//   d = div_scale(n), r = rcp(d), two Newton steps r += r (1 - d r),
//   q0 = x' r, rem = x' - d q0, q1 = div_fmas(rem, r, q0), div_fixup(q1, n, x)
// where div_scale / div_fmas scale only for extreme exponents and div_fixup
// only changes special operands.  For n >= 1 integer-valued and
// 2^-900 < |x| < 2^900 none of that applies, so the result is exactly
// fma(x - n q0, r, q0) with r = recip_refined(n): bit-identical to x / n, and
// r (depending on n only) is computed once per sample instead of once per
// division.  Zero is returned as is (0 / n keeps the sign of the zero).
// Callers take x / n when *ok is false.
NDNET_FN double recip_refined(double n) {
  double r = __builtin_amdgcn_rcp(n);
  double e = fma(-n, r, 1.0);
  r = fma(r, e, r);
  e = fma(-n, r, 1.0);
  r = fma(r, e, r);
  return r;
}
NDNET_FN double div_by_recip(double x, double n, double r, bool& ok) {
  const double ax = fabs(x);
  ok = (ax > 0x1p-900 && ax < 0x1p900) || x == 0.0;
  const double q0 = x * r;
  const double rem = fma(-n, q0, x);
  // x / n has the sign of x (n > 0); for x = -0 the fma sequence gives +0
  return copysign(fma(rem, r, q0), x);
}

// div_by_recip without the operand checks, for callers that have bounded the
// operands (2^-969 < |x| < 2^900 or x == 0) beforehand.  A zero x gives +0:
// only its sign could differ from x / n, and the Welford sums it feeds start
// at +0 and can never become -0, so no sum changes.
NDNET_FN double div_fast(double x, double n, double r) {
  const double q0 = x * r;
  const double rem = fma(-n, q0, x);
  return fma(rem, r, q0);
}

// Welford state of one voxel (normal_distributions.h:41-51, class handled apart).
struct Welford {
  double mean[3];
  double m2[3];
  double cov[9];
  uint64_t n;
};

NDNET_FN void welford_init(Welford& w) {
  for (int j = 0; j < 3; j++) { w.mean[j] = 0.0; w.m2[j] = 0.0; }
  for (int j = 0; j < 9; j++) w.cov[j] = 0.0;
  w.n = 0;
}

// normal_distributions.c:75-104, one sample.
NDNET_FN void welford_update(Welford& w, const double* x) {
  w.n++;
  const double n = (double)w.n;
#pragma unroll
  for (int j = 0; j < 3; j++) {
    const double old = w.mean[j];
    w.mean[j] = w.mean[j] + (x[j] - w.mean[j]) / n;
    w.m2[j] = w.m2[j] + (x[j] - old) * (x[j] - w.mean[j]);
    double v = w.m2[j] / n;
    w.cov[j * 3 + j] = (v != v) ? 0.0 : v;
#pragma unroll
    for (int k = j + 1; k < 3; k++) {
      double c = w.cov[j * 3 + k] + (x[j] - w.mean[j]) * (x[k] - w.mean[k]) / n;
      c = (c != c) ? 0.0 : c;
      w.cov[j * 3 + k] = c;
      w.cov[k * 3 + j] = c;
    }
  }
}

// gsl_linalg_LU_decomp for a 3x3 (GSL 2.7: LU_decomp_L2 via LU_decomp_L3):
// per column, first max |a| as pivot (cblas idamax), full row swap, scale the
// sub-column by 1/a_jj (divide when |a_jj| < DBL_MIN), rank-1 update
// a_ic += a_jc * (-a_ij).  perm/signum from the pivot sequence.
// c ? a : b as two v_cndmask_b32 on a lane mask: a plain select of two
// elements of the caller's matrix can be folded into a select of their
// addresses, which turns the register-resident matrix into scratch memory.
NDNET_FN double lu_sel(bool c, double a, double b) {
  const unsigned long long lanes = __ballot(c);
  const unsigned long long ua = __builtin_bit_cast(unsigned long long, a);
  const unsigned long long ub = __builtin_bit_cast(unsigned long long, b);
  uint32_t lo, hi;
  asm("v_cndmask_b32 %0, %1, %2, %3" : "=v"(lo) : "v"((uint32_t)ub), "v"((uint32_t)ua), "s"(lanes));
  asm("v_cndmask_b32 %0, %1, %2, %3" : "=v"(hi) : "v"((uint32_t)(ub >> 32)), "v"((uint32_t)(ua >> 32)), "s"(lanes));
  return __builtin_bit_cast(double, (unsigned long long)lo | ((unsigned long long)hi << 32));
}

NDNET_FN void lu3(double* A, uint32_t& perm_packed, int& signum) {
  // Written out per column with selects, no loops over rows: every index is
  // a compile-time constant (A stays in registers) and no pivot decision
  // becomes a branch (the generic loop form compiled to ~300 instructions
  // per decomposition with 14 exec-masked branches, tools/ubench/lu_chain.hip).
  // Column 0: first max |a| over rows 0..2 (cblas idamax: a > max, max from 0).
  const double a00 = fabs(A[0]), a10 = fabs(A[3]), a20 = fabs(A[6]);
  const double m0 = a00 > 0.0 ? a00 : 0.0;
  const bool b1 = a10 > m0;
  const double m1 = b1 ? a10 : m0;
  const bool b2 = a20 > m1;
  const bool s1 = b1 && !b2;  // pivot row 1
  double r0[3], r1[3], r2[3];  // the rows after swapping row 0 with the pivot row
#pragma unroll
  for (int c = 0; c < 3; c++) {
    r0[c] = lu_sel(b2, A[6 + c], lu_sel(b1, A[3 + c], A[c]));
    r1[c] = lu_sel(s1, A[c], A[3 + c]);
    r2[c] = lu_sel(b2, A[c], A[6 + c]);
  }
  {
    const double ajj = r0[0];
    if (fabs(ajj) >= kDblMin) {
      const double s = 1.0 / ajj;
      r1[0] = s * r1[0];
      r2[0] = s * r2[0];
    } else {
      r1[0] = r1[0] / ajj;
      r2[0] = r2[0] / ajj;
    }
    const double t1 = -1.0 * r1[0], t2 = -1.0 * r2[0];
    r1[1] = r1[1] + r0[1] * t1;
    r1[2] = r1[2] + r0[2] * t1;
    r2[1] = r2[1] + r0[1] * t2;
    r2[2] = r2[2] + r0[2] * t2;
  }
  // Column 1: pivot between rows 1 and 2 (full-row swap)
  const double a11 = fabs(r1[1]), a21 = fabs(r2[1]);
  const bool bb = a21 > (a11 > 0.0 ? a11 : 0.0);
  double n1[3], n2[3];
#pragma unroll
  for (int c = 0; c < 3; c++) {
    n1[c] = lu_sel(bb, r2[c], r1[c]);
    n2[c] = lu_sel(bb, r1[c], r2[c]);
  }
  {
    const double ajj = n1[1];
    if (fabs(ajj) >= kDblMin) {
      const double s = 1.0 / ajj;
      n2[1] = s * n2[1];
    } else {
      n2[1] = n2[1] / ajj;
    }
    const double t = -1.0 * n2[1];
    n2[2] = n2[2] + n1[2] * t;
  }
#pragma unroll
  for (int c = 0; c < 3; c++) {
    A[c] = r0[c];
    A[3 + c] = n1[c];
    A[6 + c] = n2[c];
  }
  // permutation from the pivots (gsl_permutation_swap per step; a swap of
  // two distinct positions flips the sign; column 2 never swaps):
  // pivot row 1 -> (1, 0, 2), row 2 -> (2, 1, 0); then rows 1, 2 swapped by bb
  const uint32_t q0 = b2 ? 2u : (s1 ? 1u : 0u);
  const uint32_t q1 = s1 ? 0u : 1u;
  const uint32_t q2 = b2 ? 0u : 2u;
  const uint32_t p1 = bb ? q2 : q1, p2 = bb ? q1 : q2;
  perm_packed = q0 | (p1 << 2) | (p2 << 4);
  signum = ((b1 || b2) != bb) ? -1 : 1;
}

NDNET_FN double lu3_det(const double* LU, int signum) {
  double d = (double)signum;
  d = d * LU[0];
  d = d * LU[4];
  d = d * LU[8];
  return d;
}

NDNET_FN int lu3_sgndet(const double* LU, int signum) {
  int s = signum;
  for (int i = 0; i < 3; i++) {
    const double u = LU[i * 4];
    if (u < 0) s = -s;
    else if (u == 0) return 0;
  }
  return s;
}

#ifdef NDNET_LU_INVERT_COLUMNS
// Variant (round 1): inverse from LU column by column (P e_j, unit-lower
// forward, upper back substitution in gslcblas dtrsv order).  Rounds
// differently from GSL 2.7.1's LU_invert below (<= 3.7e-13 relative on a KL
// score); kept for A/B runs only.
NDNET_FN void lu3_invert(const double* LU, uint32_t perm_packed, double* inv) {
  int perm[3] = {(int)(perm_packed & 3), (int)((perm_packed >> 2) & 3), (int)((perm_packed >> 4) & 3)};
#pragma unroll
  for (int j = 0; j < 3; j++) {
    double x0 = (perm[0] == j) ? 1.0 : 0.0;
    double x1 = (perm[1] == j) ? 1.0 : 0.0;
    double x2 = (perm[2] == j) ? 1.0 : 0.0;
    x1 = x1 - LU[3] * x0;
    x2 = x2 - LU[6] * x0;
    x2 = x2 - LU[7] * x1;
    x2 = x2 / LU[8];
    x1 = x1 - LU[5] * x2;
    x1 = x1 / LU[4];
    double t = x0 - LU[1] * x1;
    t = t - LU[2] * x2;
    x0 = t / LU[0];
    inv[0 * 3 + j] = x0;
    inv[1 * 3 + j] = x1;
    inv[2 * 3 + j] = x2;
  }
}
#else
// gsl_linalg_LU_invert as GSL 2.7.1 publishes it (linalg/lu.c): the inverse
// is the LU copy run through gsl_linalg_LU_invx --
//   1. gsl_linalg_tri_invert(CblasUpper, CblasNonUnit): U^-1 in place
//      (linalg/tri.c triangular_inverse_L2, N = 3 below the Level-3
//      crossover): per column i, T_ii = 1 / T_ii, then the column above the
//      diagonal = -T_ii * dtrmv(Upper, NoTrans, NonUnit, T[0:i,0:i]) of itself;
//   2. gsl_linalg_tri_invert(CblasLower, CblasUnit): L^-1 in place, columns
//      j = N-1 .. 0, the column below the diagonal = -dtrmv(Lower, NoTrans,
//      Unit, T[j+1:,j+1:]) of itself;
//   3. gsl_linalg_tri_UL: U^-1 L^-1 in place (triangular_mult_L2, Upper):
//      per row i, A_ii += ddot(L col below, U row right); for 0 < i < N-1 the
//      row's L part = dgemv(Trans, 1, L_BL, U row, beta = a_ii) and the
//      column's U part += dgemv(NoTrans, 1, U_TR, L col); the last row's L
//      part scaled by a_NN;
//   4. every row through gsl_permute_vector_inverse (out[p[k]] = row[k]).
// Each BLAS call in gslcblas's loop order (cblas/source_trmv_r.h,
// source_dot_r.h, source_gemv_r.h, source_scal_r.h), every operation rounded
// separately (no contraction): the same IEEE sequence as oracle/ndt_oracle.c
// orc_lu_invert_gsl.
NDNET_FN void lu3_invert(const double* LU, uint32_t perm_packed, double* inv) {
  double a00 = LU[0], a01 = LU[1], a02 = LU[2];
  double a10 = LU[3], a11 = LU[4], a12 = LU[5];
  double a20 = LU[6], a21 = LU[7], a22 = LU[8];
  // 1. U^-1.  i = 0: the diagonal only
  a00 = 1.0 / a00;
  {  // i = 1: v = (a01), trmv over [a00]: v0 = 0 + v0 * a00; scal(-a11)
    a11 = 1.0 / a11;
    const double s = -a11;
    a01 = 0.0 + a01 * a00;
    a01 = a01 * s;
  }
  {  // i = 2: v = (a02, a12), trmv over [[a00, a01], [., a11]]; scal(-a22)
    a22 = 1.0 / a22;
    const double s = -a22;
    const double t0 = 0.0 + a12 * a01;
    a02 = t0 + a02 * a00;
    a12 = 0.0 + a12 * a11;
    a02 = a02 * s;
    a12 = a12 * s;
  }
  // 2. L^-1 (unit).  j = 2: nothing below the diagonal
  {  // j = 1: v = (a21), trmv over [1]: v0 += 0; scal(-1)
    a21 = a21 + 0.0;
    a21 = a21 * -1.0;
  }
  {  // j = 0: v = (a10, a20), trmv over [[1, .], [a21, 1]] bottom-up; scal(-1)
    const double t1 = 0.0 + a10 * a21;
    a20 = a20 + t1;
    a10 = a10 + 0.0;
    a10 = a10 * -1.0;
    a20 = a20 * -1.0;
  }
  // 3. U^-1 L^-1
  {  // i = 0: a00 += ddot((a10, a20), (a01, a02))
    double t = 0.0 + a10 * a01;
    t = t + a20 * a02;
    a00 = a00 + t;
  }
  {  // i = 1
    const double aii = a11;
    const double t = 0.0 + a21 * a12;
    a11 = a11 + t;
    // lr = (a10): beta = aii first, then += (1 * a12) * a20 when non-zero
    a10 = aii == 0.0 ? 0.0 : (aii != 1.0 ? a10 * aii : a10);
    const double x = 1.0 * a12;
    if (x != 0.0) a10 = a10 + x * a20;
    // ut = (a01): beta = 1; += 1 * (0 + a21 * a02)
    const double u = 0.0 + a21 * a02;
    a01 = a01 + 1.0 * u;
  }
  {  // i = 2: the last row's L part times a22
    const double aii = a22;
    a20 = a20 * aii;
    a21 = a21 * aii;
  }
  // 4. column permutation of every row: out[p[k]] = row[k]
  const int p0 = (int)(perm_packed & 3), p1 = (int)((perm_packed >> 2) & 3), p2 = (int)((perm_packed >> 4) & 3);
  const double r[9] = {a00, a01, a02, a10, a11, a12, a20, a21, a22};
#pragma unroll
  for (int row = 0; row < 3; row++) {
#pragma unroll
    for (int c = 0; c < 3; c++) {
      // column c of the output row is the input element k with p[k] == c
      inv[row * 3 + c] = p0 == c ? r[row * 3 + 0] : (p1 == c ? r[row * 3 + 1] : r[row * 3 + 2]);
    }
  }
}
#endif

// kullback_leibler.c:98-115 given both operands already decomposed:
// 0.5 * (0 + tr(inv_q * LU_p) - log(det_q / det_p) - 3), the trace summed as
// gslcblas dgemm does (C zeroed, skip zero A entries, k ascending).
NDNET_FN double kl_score(const double* LUp, const double* LUq, uint32_t perm_q, double det_p, double det_q) {
  double inv[9];
  lu3_invert(LUq, perm_q, inv);
  double tr = 0.0;
#pragma unroll
  for (int i = 0; i < 3; i++) {
    double c = 0.0;
#pragma unroll
    for (int k = 0; k < 3; k++) {
      const double t = 1.0 * inv[i * 3 + k];
      if (t != 0.0) c = c + t * LUp[k * 3 + i];
    }
    tr = tr + c;
  }
  const double first = 0.0;
  return 0.5 * (((first + tr) - ndnet_log(det_q / det_p)) - 3.0);
}

}  // namespace ndnet
