/*
 * ndnet_pointnet.h -- C ABI of the fused point-MLP kernel of libndnet_amd.so
 * (ndt-net_amd/csrc/pointnet_kernels.hip), the NDTNetSegmentation eval forward
 * on gfx950.
 *
 * It replaces the per-point Conv1d(k=1) + BatchNorm1d + ReLU chains of
 * ndnet/models/ndtnet.py:45-60 (TNet convs), :148-161 (NDTNet convs) and
 * :233-241 (segmentation head), each of which the reference runs as separate
 * torch ops with activations round-tripping through memory.  Host side:
 * ndt-net_amd/ndnet/models/pointnet_hip.py (BatchNorm folding, per-cloud
 * steps, the four chains A-D).
 *
 * Layer weights are W^T (K input channels x N output channels) with BatchNorm
 * folded in, K padded to a multiple of 16 and N to 32 (N <= 32) or 64, stored FRAGMENT-MAJOR
 * for the 16x16x4 fp32 MFMA: element (k, n) at
 *   ((n / 16) * (K / 16) + k / 16) * 256 + (((k / 4) % 4) * 16 + n % 16) * 4 + k % 4
 * i.e. [column block][k-group][lane = 16 ((k/4)%4) + n%16][k%4] -- one 1 KB
 * (k-group, column block) piece is what one wave loads per k-group, lane l
 * holding the B operands of four consecutive MFMAs.  Padding is zero.
 */
#ifndef NDNET_POINTNET_H_
#define NDNET_POINTNET_H_
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NDNET_PN_MAX_LAYERS 5

typedef struct ndnet_pn_layer {
  const float* w;         // fragment-major W^T, K * N floats (+ cloud * w_cloud_stride), 16-byte aligned
  int64_t w_cloud_stride; // 0 for shared weights, else the per-cloud stride (floats) of folded weights
  const float* bias;      // [N] (+ cloud * bias_cloud_stride)
  int64_t bias_cloud_stride;
  int32_t K, N;           // padded sizes: K % 16 == 0; N == 32 or N % 64 == 0
  int32_t relu;
  int32_t prec;           // 0: fp32 MFMA (v_mfma_f32_16x16x4_f32) on fp32 fragment-major weights;
                          // 1: split-bf16 "x6" (fp32-accurate, v_mfma_f32_16x16x32_bf16): K % 32 == 0,
                          //    `w` = bf16 [N/16][K/32][3 planes][64 lanes][8] with W^T = h + m + l and
                          //    lane l's 8 values W^T[32 kg + 8 (l/16) + j][16 cb + l%16]; the layer's
                          //    producer must be the previous, unfused layer (it stores bf16 planes)
  int32_t fuse_next;      // 1: this layer's output (N % 64 == 0) is produced in 64-column chunks, each
                          // consumed at once by the next layer (whose N is 64, 128 or 256) -- the
                          // activation never occupies LDS whole
} ndnet_pn_layer;

// mode: 0 = max-pool the last layer over points into gmax[cloud][N]
//       1 = log-softmax over the first `out_cols` channels of the last layer,
//           written to out[cloud][point][out_cols]
typedef struct ndnet_pn_chain {
  const float* x;         // [B][num_points][x_ld] input rows
  int32_t x_ld;           // floats per input row (12)
  int32_t in_cols;        // columns of x the first layer reads (3 or 12); the rest of K is zero
  int32_t num_points;
  int32_t num_layers;
  ndnet_pn_layer L[NDNET_PN_MAX_LAYERS];
  int32_t mode;
  int32_t out_cols;
  float* gmax;            // mode 0: [B][gmax_ld], pre-set to -inf
  int32_t gmax_ld;
  int32_t max_width;      // widest activation of LDS region 0 (the input, layers 1, 3, ... outputs), % 8 == 0
  int32_t max_width2;     // widest activation of LDS region 1 (layers 0, 2, ... outputs), % 8 == 0; a fused
                          // layer's output is not stored in either region
  float* out;             // mode 1
  float* clear;           // optional: set clear[0 .. clear_count) to -inf once the chain no longer
  int64_t clear_count;    // reads it (re-arms a max-pool buffer for the next forward), or NULL
  // optional prologue (head_h2 != NULL; chain B): the TNet(3) tail of ndnet_pn_head3_run computed by
  // every workgroup of a cloud before layer 0, which reads its result -- t1[b] = h2[b] @ W3^T + b3 (9
  // outputs, the identity folded into b3) and conv1 with t1 folded, written fragment-major (K padded to
  // 16) to L[0].w + b * L[0].w_cloud_stride (every workgroup writes the same bits); t1 to head_t1[b]
  const float* head_h2;   // [B][head_ld]
  int32_t head_ld, head_K;
  const float* head_w3;   // [9][head_K]
  const float* head_b3;   // [9]
  const float* head_basis;  // [9][head_kin * head_nout]
  int32_t head_kin, head_nout;
  float* head_t1;         // [B][9]
  // optional prologue (fold_t2 != NULL; chains C and D, layer 0 on the VALU): TNet(64)'s feature
  // transform applied through layer 0 -- x_t2 = t2[b]^T (W0 x + b0) (ndtnet.py:150-157: bmm of the
  // bn1(conv1) rows with t2, no ReLU between) -- as the per-cloud layer W0' = W0^T t2[b], b0' = b0^T t2[b],
  // computed by every workgroup in LDS before layer 0; t2[b] = fold_t2 + b * fold_ld, 64 x 64 row-major
  // (row = the input channel of conv1's output).  Layer 0 must be 64 wide; its relu flag is applied after.
  const float* fold_t2;
  int32_t fold_ld;
  // optional with fold_t2: the cloud's first workgroup also writes W0' fragment-major (K = 16, rows
  // 12..15 untouched: zero-initialise them) to fold_out_w + b * 1024 and b0' to fold_out_b + b * 64,
  // so a later chain runs the same transformed layer 0 as a plain per-cloud layer (chain D)
  float* fold_out_w;
  float* fold_out_b;
} ndnet_pn_chain;

/* Runs one chain over `batch` clouds on `stream` (a hipStream_t; NULL = default
 * stream).  Returns 0, NDNET_ERR_ARG (-20) for an inconsistent argument block
 * (layer sizes, LDS region widths) or NDNET_ERR_HIP (-21) on a launch failure.
 * No allocation, no synchronisation: graph-capturable. */
int ndnet_pn_chain_run(const ndnet_pn_chain *args, int batch, void *stream);
/* The same chain on 32-point tiles (8 waves per workgroup; same arguments,
 * results within fp32 summation order): for batches whose 64-point tiles
 * would leave CUs idle, e.g. 16 clouds of 500 points. */
int ndnet_pn_chain_run_t32(const ndnet_pn_chain *args, int batch, void *stream);

/* Timing builds only (-DNDNET_PN_STAMPS, tools/pn_stamps.py): the
 * s_memrealtime stamps (100 MHz) of every workgroup of the last chain
 * launch, [wgs][16] (0 start, 1 head prologue, 2 input tile, 3 + l after
 * layer l, 15 end), copied to host memory.  The product build returns -20. */
int ndnet_pn_debug_stamps(unsigned long long *host, int wgs);
int ndnet_pn_debug_stamps_clear(void);  /* zeroes them (timing builds; else -20) */

/* The per-cloud steps between the chains (TNet FC heads ndtnet.py:53-60 and
 * the t1 weight fold of pointnet_hip.py), for batch <= 16 clouds:
 *   ndnet_pn_fc_run:     out[b][n] = act(bias[n] + sum_k in[b][k] W[n][k]),
 *                        W row-major [N][K], K % 4 == 0, act = ReLU if relu
 *                        (Linear + folded BatchNorm1d + ReLU, ndtnet.py:55-56)
 *   ndnet_pn_head3_run:  t1[b] = h2[b] @ W3^T + b3 (9 outputs; the TNet
 *                        identity folded into b3, ndtnet.py:57-60) and
 *                        w1f[b] = t1[b] @ basis ([9][kin * nout] row-major) --
 *                        conv1 with t1 folded, written fragment-major with K
 *                        padded to 16 (16 * nout floats per cloud)
 * Same return codes as ndnet_pn_chain_run; graph-capturable. */
int ndnet_pn_fc_run(const float *in, int ld_in, const float *W, const float *bias, float *out, int ld_out,
                    int batch, int K, int N, int relu, void *stream);
/* The same FC layer on the fp32 MFMA (the default): Wf = W^T in the chain's
 * fragment-major layout ([N/16][K/16][64 lanes][4], as ndnet_pn_layer.w with
 * prec 0), K % 16 == 0, K <= 1024, N % 16 == 0; one launch of N / 16
 * workgroups, each summing its waves' K-slices in a fixed order. */
int ndnet_pn_fc_mfma_run(const float *in, int ld_in, const float *Wf, const float *bias, float *out, int ld_out,
                         int batch, int K, int N, int relu, void *stream);
/* BatchNorm fold of the eval forward's weights, re-run in place after a
 * weight update (the host-side first fold: pointnet_hip._Folded; the folds
 * it restates: ndtnet.py's Conv1d / Linear + BatchNorm1d pairs, :45-60,
 * :148-161, :218-241, with running statistics).  One job writes one output
 * tensor from one layer's parameters; the folded weight of layer row n and
 * input column k is
 *   fw(n, k) = w[n * ld + k0 + k] * (gamma[n] / sqrt(var[n] + eps))
 * (no BatchNorm: gamma == NULL, fw = w), every operation a separately
 * rounded fp32 operation as torch computes the fold.  Kinds:
 *   NDNET_FOLD_WT     out[k][n] (Kp x Np floats) = fw(n, k), zero padded
 *   NDNET_FOLD_FRAG   the same W^T fragment-major (ndnet_pn_layer.w, prec 0)
 *   NDNET_FOLD_FRAG6  the same W^T split-bf16 (ndnet_pn_layer.w, prec 1;
 *                     bf16 rounding to nearest even, residuals exact)
 *   NDNET_FOLD_ROWS   out[n][k] (N x K floats) = fw(n, k)
 *   NDNET_FOLD_BASIS  TNet(3)'s t1 basis of conv1 (K == 12):
 *                     out[3a + c][r][n] = E_ac^T fw^T with E_ac the 0/1
 *                     matrix of p -> t1 p, C -> t1 C (pointnet_hip._Folded)
 *   NDNET_FOLD_BIAS   out[n] (Np floats) = (bias[n] - mean[n]) * s[n] + beta[n]
 *                     (no BatchNorm: bias[n]), + 1 on the diagonal of an
 *                     eye x eye matrix when eye > 0, zero padded
 * ndnet_pn_fold_prepare validates a host copy of the job list and fills each
 * job's block0 (its first workgroup), returning the grid size in
 * *num_blocks; ndnet_pn_fold_run then runs the list from DEVICE memory in
 * one launch (graph-capturable, no allocation).  NDNET_ERR_ARG (-20) on an
 * invalid job. */
#define NDNET_FOLD_WT 0
#define NDNET_FOLD_FRAG 1
#define NDNET_FOLD_FRAG6 2
#define NDNET_FOLD_ROWS 3
#define NDNET_FOLD_BASIS 4
#define NDNET_FOLD_BIAS 5
typedef struct ndnet_pn_fold_job {
  const float *w;                          /* layer weight, rows of ld floats (not read by BIAS) */
  const float *bias;                       /* layer bias [N] (BIAS only) */
  const float *gamma, *beta, *mean, *var;  /* BatchNorm1d weight, bias, running mean / var; NULL: none */
  void *out;                               /* the output tensor (bf16 for FRAG6, else fp32), 16-byte aligned */
  int32_t kind;
  int32_t N, K;                            /* layer rows (outputs) and the input columns used */
  int32_t ld, k0;                          /* row stride of w and the first column used */
  int32_t Kp, Np;                          /* padded sizes (WT / FRAG / FRAG6: Kp x Np; BIAS: Np) */
  int32_t eye;
  float eps;
  int32_t reserved;
  int64_t block0;                          /* filled by ndnet_pn_fold_prepare */
} ndnet_pn_fold_job;
int ndnet_pn_fold_prepare(ndnet_pn_fold_job *host_jobs, int num_jobs, int64_t *num_blocks);
int ndnet_pn_fold_run(const ndnet_pn_fold_job *device_jobs, int num_jobs, int64_t num_blocks, void *stream);

int ndnet_pn_head3_run(const float *h2, int ld_h, const float *W3, const float *b3, const float *basis,
                       float *t1, float *w1f, int batch, int K, int kin, int nout, void *stream);

/* TNet(64)'s transform through conv1 (ndtnet.py:152-155), once per cloud, for
 * chains C and D's layer 0 (round 5; chain C's fold_t2 prologue did it per
 * workgroup): outf[b] = (w1f[b] as W1'^T, 12 of its 16 rows) @ t2[b] in the
 * fragment-major K = 16 layout (rows 12..15 untouched), outb[b] = b1^T t2[b].
 * w1f [batch][w1_stride >= 1024], b1 [64], t2 [batch][t2_ld >= 4096] (16-byte
 * aligned), outf [batch][1024], outb [batch][64]. */
int ndnet_pn_fold_t2_run(const float *w1f, int w1_stride, const float *b1, const float *t2, int t2_ld, float *outf,
                         float *outb, int batch, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* NDNET_POINTNET_H_ */
