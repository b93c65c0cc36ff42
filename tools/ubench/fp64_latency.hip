// fp64_latency.hip -- dependent-chain latency and throughput of the FP64
// operations the per-ND Welford step uses (k_welford_q), one wave alone on
// its SIMD and several waves per SIMD.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o tools/ubench/fp64_latency tools/ubench/fp64_latency.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#pragma clang fp contract(off)

constexpr int kIters = 4096;

// 8 dependent ops per iteration
template <int KIND>
__global__ void chain(double* out, double a, double b, unsigned long long* cyc) {
  double x = a + threadIdx.x * 1e-9, y = b;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
  for (int i = 0; i < kIters; i++) {
#pragma unroll
    for (int k = 0; k < 8; k++) {
      if constexpr (KIND == 0) x = x + y;              // v_add_f64
      else if constexpr (KIND == 1) x = x * y;         // v_mul_f64
      else if constexpr (KIND == 2) x = fma(x, y, b);  // v_fma_f64
      else x = x + (double)(float)k;                   // add with a constant
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

// N independent chains per wave (throughput)
template <int N>
__global__ void indep(double* out, double a, double b, unsigned long long* cyc) {
  double x[N];
  for (int k = 0; k < N; k++) x[k] = a + threadIdx.x * 1e-9 + k;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
  for (int i = 0; i < kIters; i++) {
#pragma unroll
    for (int r = 0; r < 8; r++)
#pragma unroll
      for (int k = 0; k < N; k++) x[k] = fma(x[k], b, a);
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
  double s = 0;
  for (int k = 0; k < N; k++) s += x[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// The Welford mean chain per sample: t = x - m, then m += t / n as
// RN(t rc + RN(t rl)) -- 4 dependent ops (sub, mul, fma, add) -- or the
// refined-reciprocal division (sub, mul, fma, fma, add: 5), with FILL
// independent FP64 ops per sample issued beside it (the work that could hide
// in the chain's bubbles).
template <int FIVE, int FILL>
__global__ void meanchain(double* out, double a, double b, unsigned long long* cyc) {
  double m = a + threadIdx.x * 1e-9, x = b, rc = 1.0 / 3.0, rl = 1e-17, cn = 3.0;
  double f[FILL > 0 ? FILL : 1];
  for (int k = 0; k < (FILL > 0 ? FILL : 1); k++) f[k] = a + k;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
  for (int i = 0; i < kIters; i++) {
#pragma unroll
    for (int r = 0; r < 8; r++) {
      const double t = x - m;
      double q;
      if constexpr (FIVE) {
        const double q0 = t * rc;
        const double rem = fma(-cn, q0, t);
        q = fma(rem, rc, q0);
      } else {
        const double p = t * rl;
        q = fma(t, rc, p);
      }
      m = m + q;
#pragma unroll
      for (int k = 0; k < FILL; k++) f[k] = fma(f[k], b, a);
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
  double s = m;
  for (int k = 0; k < FILL; k++) s += f[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// wq_heavy's phase 1 as it runs in k_welford_q: lanes 0..2 (or all lanes,
// EXEC3 = 0) run the mean recurrence over 64-sample blocks whose x and
// (rc, rl) come from LDS (XR: 0 registers, 1 LDS), writing each mean to LDS
// (MW), the next group's operands loaded a group ahead.
template <int XR, int MW, int EXEC3, int PIN = 0>
__global__ void phase1(double* out, double a, double b, unsigned long long* cyc) {
  __shared__ double X[3][65];
  __shared__ double M[3][67];
  __shared__ double2 R[64];
  const int lane = threadIdx.x;
  for (int i = lane; i < 3 * 65; i += 64) (&X[0][0])[i] = a + i * 1e-3;
  R[lane] = make_double2(1.0 / (lane + 1), 1e-17 * (lane + 1));
  __syncthreads();
  double m = b;
  const int ax = lane < 3 ? lane : 0;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  if (!EXEC3 || lane < 3) {
    const double* xa = &X[ax][0];
    double* ma = &M[ax][1];
#pragma unroll 1
    for (int it = 0; it < kIters / 8; it++) {
      double xA[8], xB[8];
      double2 rA[8], rB[8];
      auto ld = [&](double (&x)[8], double2 (&r)[8], int i0) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
          if (XR) { x[u] = xa[i0 + u]; r[u] = R[i0 + u]; }
          else { x[u] = a + u; r[u] = make_double2(0.25 + u, 1e-17); }
        }
      };
      auto ch = [&](const double (&x)[8], const double2 (&r)[8], int i0) {
        double mm[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
          const double t = x[u] - m;
          m = m + fma(t, r[u].x, t * r[u].y);
          mm[u] = m;
          if (MW == 1) ma[i0 + u] = m;
        }
        if (MW == 2) {
#pragma unroll
          for (int u = 0; u < 8; u++) ma[i0 + u] = mm[u];
        }
      };
      ld(xA, rA, 0);
      for (int i0 = 0; i0 < 64; i0 += 16) {
        ld(xB, rB, i0 + 8);
        if (PIN) asm volatile("" ::: "memory");  // the loads stay ahead of the chain they do not feed
        ch(xA, rA, i0);
        if (i0 + 16 < 64) ld(xA, rA, i0 + 16);
        if (PIN) asm volatile("" ::: "memory");
        ch(xB, rB, i0 + 8);
      }
      asm volatile("" ::: "memory");
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
  out[blockIdx.x * blockDim.x + threadIdx.x] = m + M[ax][5];
}

// Phase 1 without LDS reads: lanes 0..2 load their own coordinate from global
// memory (a dword per sample, immediate offsets), (rc, rl) arrive in SGPRs
// (scalar loads of a uniform table), the mean goes out per sample
// (MW: 0 none, 1 ds_write_b64, 2 global_store_dwordx2).
template <int MW>
__global__ void phase1g(double* out, const float* __restrict__ pts, const double2* __restrict__ rt,
                        double* mout, unsigned long long* cyc) {
  __shared__ double M[3][67];
  const int lane = threadIdx.x;
  const int ax = lane < 3 ? lane : 0;
  double m = 0.5;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  if (lane < 3) {
    double* ma = &M[ax][1];
#pragma unroll 1
    for (int it = 0; it < kIters / 8; it++) {
      const float* p = pts + 3 * 64 * (it & 15) + ax;
      const double2* r = rt + 64 * (it & 15);
      double* mg = mout + 3 * 64 * (it & 15) + ax * 64;
      float xA[8], xB[8];
#pragma unroll
      for (int u = 0; u < 8; u++) xA[u] = p[3 * u];
      for (int i0 = 0; i0 < 64; i0 += 16) {
#pragma unroll
        for (int u = 0; u < 8; u++) xB[u] = p[3 * (i0 + 8 + u)];
        asm volatile("" ::: "memory");
#pragma unroll
        for (int u = 0; u < 8; u++) {
          const double2 q = r[i0 + u];
          const double t = (double)xA[u] - m;
          m = m + fma(t, q.x, t * q.y);
          if (MW == 1) ma[i0 + u] = m;
          if (MW == 2) mg[i0 + u] = m;
        }
        if (i0 + 16 < 64) {
#pragma unroll
          for (int u = 0; u < 8; u++) xA[u] = p[3 * (i0 + 16 + u)];
        }
        asm volatile("" ::: "memory");
#pragma unroll
        for (int u = 0; u < 8; u++) {
          const double2 q = r[i0 + 8 + u];
          const double t = (double)xB[u] - m;
          m = m + fma(t, q.x, t * q.y);
          if (MW == 1) ma[i0 + 8 + u] = m;
          if (MW == 2) mg[i0 + 8 + u] = m;
        }
      }
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
  out[blockIdx.x * blockDim.x + threadIdx.x] = m + M[ax][5];
}

template <int MW>
static void rung(const char* name) {
  double *out, *mout;
  float* pts;
  double2* rt;
  unsigned long long* cyc;
  hipMalloc(&out, 64 * sizeof(double));
  hipMalloc(&mout, 3 * 64 * 16 * sizeof(double));
  hipMalloc(&pts, 3 * 64 * 16 * sizeof(float));
  hipMalloc(&rt, 64 * 16 * sizeof(double2));
  hipMemset(pts, 0, 3 * 64 * 16 * sizeof(float));
  hipMemset(rt, 0, 64 * 16 * sizeof(double2));
  hipMalloc(&cyc, sizeof(unsigned long long));
  for (int r = 0; r < 2; r++) hipLaunchKernelGGL(phase1g<MW>, dim3(1), dim3(64), 0, 0, out, pts, rt, mout, cyc);
  hipDeviceSynchronize();
  unsigned long long c;
  hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost);
  printf("%-44s: %.2f cycles per sample\n", name, (double)c / ((double)(kIters / 8) * 64));
}

// ---- k_welford_q's heavy-ND loop (copied from csrc/ndt_kernels.hip) alone on one wave ----
typedef unsigned int hv_u16 __attribute__((ext_vector_type(16)));
typedef double hv_d2 __attribute__((ext_vector_type(2)));  // native vector (HIP's double2 is a struct)

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
    const hv_u16& r = u < 4 ? o.r0 : o.r1;
    const double rc = hv_sd(r, 2 * (u & 3)), rl = hv_sd(r, 2 * (u & 3) + 1);
    const double t = xv - m;
    m = m + fma(t, rc, t * rl);
    acc = acc + xv;
    mo[u] = m;
  }
}
template <int G>  // group G of a full block: wait for its operands, write G - 1's means, issue G + 1's operands, step
__device__ inline void hv_group(double& m, double& acc, HvOps& cur, HvOps& nxt, double (&mcur)[8],
                                double (&mprev)[8], uint32_t rda, uint32_t wra, const double2* rtq) {
  hv_wait(cur);
  if constexpr (G > 0) hv_put<G - 1>(wra, mprev);
  if constexpr (G < 7) hv_issue<G + 1>(nxt, rda, rtq);
  hv_steps(m, acc, cur, mcur);
}
// The same loop with (rc, rl) from an LDS row R[64] (written with the
// block) instead of scalar loads: every memory operation of the loop is then
// LDS, which completes in order, so the waits count (lgkmcnt(N)) and the
// operands are issued two groups ahead.  Per group: 4 ds_read_b128 of the
// lane's row, 8 broadcast ds_read_b128 of R, 4 ds_write_b128 of the means.
struct HvOps2 {
  hv_d2 x[4];
  hv_d2 r[8];  // (rc, rl) of the 8 steps
};
template <int G>
__device__ inline void hv_issue2(HvOps2& o, uint32_t rda, uint32_t ra) {
  hv_d2 x0, x1, x2, x3, r0, r1, r2, r3, r4, r5, r6, r7;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(x0) : "v"(rda), "n"(64 * G));
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(x1) : "v"(rda), "n"(64 * G + 16));
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(x2) : "v"(rda), "n"(64 * G + 32));
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(x3) : "v"(rda), "n"(64 * G + 48));
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r0) : "v"(ra), "n"(128 * G));
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r1) : "v"(ra), "n"(128 * G + 16));
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r2) : "v"(ra), "n"(128 * G + 32));
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r3) : "v"(ra), "n"(128 * G + 48));
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r4) : "v"(ra), "n"(128 * G + 64));
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r5) : "v"(ra), "n"(128 * G + 80));
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r6) : "v"(ra), "n"(128 * G + 96));
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r7) : "v"(ra), "n"(128 * G + 112));
  o.x[0] = x0; o.x[1] = x1; o.x[2] = x2; o.x[3] = x3;
  o.r[0] = r0; o.r[1] = r1; o.r[2] = r2; o.r[3] = r3; o.r[4] = r4; o.r[5] = r5; o.r[6] = r6; o.r[7] = r7;
}
template <int N>  // all but the N youngest LDS operations done; the group's registers held behind it
__device__ inline void hv_wait2(HvOps2& o) {
  hv_d2 x0 = o.x[0], x1 = o.x[1], x2 = o.x[2], x3 = o.x[3];
  hv_d2 r0 = o.r[0], r1 = o.r[1], r2 = o.r[2], r3 = o.r[3], r4 = o.r[4], r5 = o.r[5], r6 = o.r[6], r7 = o.r[7];
  asm volatile("s_waitcnt lgkmcnt(%12)"
               : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5),
                 "+v"(r6), "+v"(r7)
               : "n"(N));
  o.x[0] = x0; o.x[1] = x1; o.x[2] = x2; o.x[3] = x3;
  o.r[0] = r0; o.r[1] = r1; o.r[2] = r2; o.r[3] = r3; o.r[4] = r4; o.r[5] = r5; o.r[6] = r6; o.r[7] = r7;
}
__device__ inline void hv_steps2(double& m, double& acc, const HvOps2& o, double (&mo)[8]) {
#pragma unroll
  for (int u = 0; u < 8; u++) {
    const double xv = o.x[u >> 1][u & 1];
    const double t = xv - m;
    m = m + fma(t, o.r[u][0], t * o.r[u][1]);
    acc = acc + xv;
    mo[u] = m;
  }
}
// group G: wait for its operands R(G), write G - 1's means W(G - 1), issue
// R(G + 2), step.  R(G + 2) and W(G - 1) go out at the top of group G, so
// the operations younger than R(G) at its wait are: G = 0, 1: R(G + 1) (12);
// G = 2..6: W(G - 2) and R(G + 1) (16: lgkmcnt(15), the field's maximum, waits
// for one more); G = 7: W(5) (4).
template <int G>
__device__ inline void hv_group2(double& m, double& acc, HvOps2 (&ops)[3], double (&mcur)[8], double (&mprev)[8],
                                 uint32_t rda, uint32_t wra, uint32_t ra) {
  if constexpr (G < 2) hv_wait2<12>(ops[G % 3]);
  else if constexpr (G < 7) hv_wait2<15>(ops[G % 3]);
  else hv_wait2<4>(ops[G % 3]);
  if constexpr (G > 0) hv_put<G - 1>(wra, mprev);
  if constexpr (G + 2 < 8) hv_issue2<G + 2>(ops[(G + 2) % 3], rda, ra);
  hv_steps2(m, acc, ops[G % 3], mcur);
}
__device__ inline void hv_block_lds(double& m, double& acc, uint32_t rda, uint32_t wra, uint32_t ra) {
  HvOps2 ops[3];
  double mA[8], mB[8];
  hv_issue2<0>(ops[0], rda, ra);
  hv_issue2<1>(ops[1], rda, ra);
  hv_group2<0>(m, acc, ops, mA, mB, rda, wra, ra);
  hv_group2<1>(m, acc, ops, mB, mA, rda, wra, ra);
  hv_group2<2>(m, acc, ops, mA, mB, rda, wra, ra);
  hv_group2<3>(m, acc, ops, mB, mA, rda, wra, ra);
  hv_group2<4>(m, acc, ops, mA, mB, rda, wra, ra);
  hv_group2<5>(m, acc, ops, mB, mA, rda, wra, ra);
  hv_group2<6>(m, acc, ops, mA, mB, rda, wra, ra);
  hv_group2<7>(m, acc, ops, mB, mA, rda, wra, ra);
  hv_put<7>(wra, mB);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the block's means are in LDS for phase 2
}

__device__ inline void hv_block_asm(double& m, double& acc, uint32_t rda, uint32_t wra, const double2* rtq) {
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


__global__ void hv_loop(double* out, const double2* __restrict__ rtab, unsigned long long* cyc, int blocks) {
  __shared__ __attribute__((aligned(16))) double lds[12 * 66 + 128];
  const int lane = threadIdx.x;
  for (int i = lane; i < 12 * 66 + 128; i += 64) lds[i] = 1.0 + i * 1e-3;
  __syncthreads();
  const double* rd = lane < 3 ? lds + lane * 66 : lds + (6 + (lane < 9 ? lane - 3 : 0)) * 66;
  double* wr = lane < 3 ? lds + (3 + lane) * 66 + 2 : lds + (6 + (lane < 9 ? lane - 3 : 0)) * 66;
  double m = 0.5, acc = 0.0;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  if (lane < 9) {
    for (int k = 0; k < blocks; k++) {
      if (blocks > 0)
        hv_block_asm(m, acc, (uint32_t)(uintptr_t)(__attribute__((address_space(3))) const double*)rd,
                     (uint32_t)(uintptr_t)(__attribute__((address_space(3))) double*)wr, rtab + 64 * (k & 7) + 1);
    }
    for (int k = 0; k < -blocks; k++)
      hv_block_lds(m, acc, (uint32_t)(uintptr_t)(__attribute__((address_space(3))) const double*)rd,
                   (uint32_t)(uintptr_t)(__attribute__((address_space(3))) double*)wr,
                   (uint32_t)(uintptr_t)(__attribute__((address_space(3))) const double*)(lds + 12 * 66));
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
  out[blockIdx.x * blockDim.x + threadIdx.x] = m + acc;
}

template <typename K>
static void run(const char* name, K kern, int blocks, int threads, int ops_per_iter) {
  double* out;
  unsigned long long* cyc;
  hipMalloc(&out, blocks * threads * sizeof(double));
  hipMalloc(&cyc, blocks * sizeof(unsigned long long));
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, out, 1.0000001, 0.9999999, cyc);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, out, 1.0000001, 0.9999999, cyc);
  hipDeviceSynchronize();
  unsigned long long c;
  hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost);
  printf("%-44s blocks %4d threads %4d: %.2f cycles per op per wave\n", name, blocks, threads,
         (double)c / ((double)kIters * ops_per_iter));
  hipFree(out);
  hipFree(cyc);
}

int main() {
  run("dependent v_add_f64", chain<0>, 1, 64, 8);
  run("dependent v_mul_f64", chain<1>, 1, 64, 8);
  run("dependent v_fma_f64", chain<2>, 1, 64, 8);
  run("dependent v_add_f64 (const)", chain<3>, 1, 64, 8);
  run("dependent v_fma_f64, 4 waves/SIMD (1 WG x 1024)", chain<2>, 1, 1024, 8);
  run("independent v_fma_f64 x2", indep<2>, 1, 64, 16);
  run("independent v_fma_f64 x4", indep<4>, 1, 64, 32);
  run("independent v_fma_f64 x8", indep<8>, 1, 64, 64);
  run("independent v_fma_f64 x8, 4 waves (1 per SIMD)", indep<8>, 1, 256, 64);
  run("independent v_fma_f64 x8, 8 waves (2 per SIMD)", indep<8>, 1, 512, 64);
  // cycles per sample (ops_per_iter = 8 samples)
  run("mean chain 4-op, per sample", meanchain<0, 0>, 1, 64, 8);
  run("mean chain 5-op, per sample", meanchain<1, 0>, 1, 64, 8);
  run("mean chain 4-op + 2 fill, per sample", meanchain<0, 2>, 1, 64, 8);
  run("mean chain 4-op + 4 fill, per sample", meanchain<0, 4>, 1, 64, 8);
  run("mean chain 4-op + 8 fill, per sample", meanchain<0, 8>, 1, 64, 8);
  run("mean chain 4-op, 2 waves/SIMD, per sample", meanchain<0, 0>, 1, 512, 8);
  run("mean chain 4-op + 4 fill, 2 waves/SIMD", meanchain<0, 4>, 1, 512, 8);
  run("mean chain 5-op + 8 fill, per sample", meanchain<1, 8>, 1, 64, 8);
  // cycles per sample (64 samples per iteration, kIters / 8 iterations)
  run("phase1: chain only, 3 lanes", phase1<0, 0, 1>, 1, 64, 8);
  run("phase1: + LDS x, R reads, 3 lanes", phase1<1, 0, 1>, 1, 64, 8);
  run("phase1: + LDS M writes, 3 lanes", phase1<1, 1, 1>, 1, 64, 8);
  run("phase1: chain + M writes (no reads), 3 lanes", phase1<0, 1, 1>, 1, 64, 8);
  run("phase1: LDS reads + writes, 64 lanes", phase1<1, 1, 0>, 1, 64, 8);
  run("phase1: pinned LDS reads, 3 lanes", phase1<1, 0, 1, 1>, 1, 64, 8);
  run("phase1: pinned LDS reads + writes, 3 lanes", phase1<1, 1, 1, 1>, 1, 64, 8);
  run("phase1: pinned reads + group-end writes", phase1<1, 2, 1, 1>, 1, 64, 8);
  run("phase1: group-end writes only", phase1<0, 2, 1, 1>, 1, 64, 8);
  {
    double* out;
    double2* rt;
    unsigned long long* cyc;
    hipMalloc(&out, 1024 * 64 * sizeof(double));
    hipMalloc(&rt, 600 * sizeof(double2));
    hipMemset(rt, 0, 600 * sizeof(double2));
    hipMalloc(&cyc, sizeof(unsigned long long));
    for (int r = 0; r < 2; r++) hipLaunchKernelGGL(hv_loop, dim3(1), dim3(64), 0, 0, out, rt, cyc, 256);
    hipDeviceSynchronize();
    unsigned long long c;
    hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost);
    printf("%-44s: %.2f cycles per sample\n", "hv_block_asm alone (one wave)", (double)c / (256.0 * 64));
    for (int r = 0; r < 2; r++) hipLaunchKernelGGL(hv_loop, dim3(1), dim3(64), 0, 0, out, rt, cyc, -256);
    hipDeviceSynchronize();
    hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost);
    printf("%-44s: %.2f cycles per sample\n", "hv_block_lds alone (one wave)", (double)c / (256.0 * 64));
    // one wave per SIMD on every CU: the LDS loop beside three others
    for (int r = 0; r < 2; r++) hipLaunchKernelGGL(hv_loop, dim3(1024), dim3(64), 0, 0, out, rt, cyc, -256);
    hipDeviceSynchronize();
    hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost);
    printf("%-44s: %.2f cycles per sample\n", "hv_block_lds, 1024 waves", (double)c / (256.0 * 64));
    for (int r = 0; r < 2; r++) hipLaunchKernelGGL(hv_loop, dim3(1024), dim3(64), 0, 0, out, rt, cyc, 256);
    hipDeviceSynchronize();
    hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost);
    printf("%-44s: %.2f cycles per sample\n", "hv_block_asm, 1024 waves", (double)c / (256.0 * 64));
  }
  rung<0>("phase1g: global x, SGPR rc/rl, no M out");
  rung<1>("phase1g: + ds_write_b64 per sample");
  rung<2>("phase1g: + global_store_dwordx2 per sample");
  return 0;
}
