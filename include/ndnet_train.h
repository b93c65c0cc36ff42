/*
 * ndnet_train.h -- C ABI of the train-mode point-MLP kernels of
 * libndnet_amd.so (ndt-net_amd/csrc/train_kernels.hip): the forward and
 * backward of the reference's per-point Conv1d(k=1) + BatchNorm1d (batch
 * statistics) [+ ReLU] blocks on gfx950, for the training step of
 * tools/train.py:67-81.
 *
 * Replaces, in train mode:
 *   ndnet/models/ndtnet.py:48-50   TNet conv1..3 + bn1..3 + ReLU
 *   ndnet/models/ndtnet.py:53-60   TNet fc1 + bn4 + ReLU, fc2 + bn5 + ReLU, fc3 + identity
 *   ndnet/models/ndtnet.py:153-155 the x^T t2 product (ndnet_tr_gemm, per cloud)
 *   ndnet/models/ndtnet.py:148-152 NDTNet conv1 + bn1 (no ReLU), conv2/conv3 + bn2/bn3
 *   ndnet/models/ndtnet.py:233-239 seg head conv1..3 + bn1..3 + ReLU, conv4
 * and the autograd backward torch runs through them.  Host side:
 * ndt-net_amd/ndnet/models/train_hip.py (the autograd Functions).
 *
 * Layouts are torch's Conv1d NCL: activations [B][C][N] fp32 (N points
 * contiguous), weights [Cout][Cin] row-major.  Every entry point launches on
 * `stream` (a hipStream_t; NULL = default stream), allocates nothing and does
 * not synchronise (graph-capturable).  Returns 0, NDNET_ERR_ARG (-20) for an
 * inconsistent argument or NDNET_ERR_HIP (-21) on a launch failure.
 */
#ifndef NDNET_TRAIN_H_
#define NDNET_TRAIN_H_
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* C[z] (M x N) = sum over the part's clouds of A[c] (M x K) . B[c] (K x N)
 * (+ bias[c * sbias + m]) on the fp32 MFMA (v_mfma_f32_16x16x4_f32: exact fp32
 * products, fp32 sums in four interleaved accumulator sets; 64 x 64 tiles).
 * Element addressing (floats):
 *   A(m, k) = A[m * lda + k] if a_kmajor else A[k * lda + m]
 *   B(k, n) = B[n * ldb + k] if b_kmajor else B[k * ldb + n]
 *   C(m, n) = C[m * ldc + n]
 * Grid z covers ceil(batch / clouds_per_part) * nchunks: z = zg * nchunks + zc
 * sums clouds c in [zg * clouds_per_part, min(batch, (zg + 1) * clouds_per_part))
 * (A + c * sAz, B + c * sBz) over k in [zc * kchunk, min(K, (zc + 1) * kchunk))
 * and writes C + z * sCz.  More than one part is split-K into partial
 * products, summed by ndnet_tr_sum_parts.  Conv1d forward: A = W (a_kmajor),
 * B = x[b]; input gradient: A = W^T (not a_kmajor), B = dy[b]; weight gradient:
 * A = dy[b] (a_kmajor), B = x[b]^T (b_kmajor), parts over (cloud groups,
 * point chunks).  sbias = 0: one bias vector; sbias = M: a bias per cloud (the
 * segmentation head's global-feature term, ndtnet.py:230-233, folded into a
 * per-cloud bias); a bias needs one cloud per part and one chunk. */
int ndnet_tr_gemm(const float *A, const float *B, float *C, const float *bias, int64_t sbias, int M, int N, int K,
                  int64_t lda, int64_t ldb, int64_t ldc, int64_t sAz, int64_t sBz, int64_t sCz,
                  int batch, int clouds_per_part, int a_kmajor, int b_kmajor, int nchunks, int kchunk,
                  void *stream);

/* out[i] = sum_{p < nparts} part[p * count + i], in p order (deterministic). */
int ndnet_tr_sum_parts(const float *part, float *out, int64_t count, int nparts, void *stream);
/* The same over a [rows][cols] block written into rows of stride ldo >= cols
 * (a column slice of a wider matrix). */
int ndnet_tr_sum_parts_2d(const float *part, float *out, int64_t rows, int64_t cols, int64_t ldo, int nparts,
                          void *stream);

/* BatchNorm1d forward with batch statistics (torch's training mode) over
 * y [B][C][N], one workgroup per channel: mean and biased variance over the
 * B * N values (summed in double, two passes), invstd = 1 / sqrt(var + eps),
 * z = (y - mean) * invstd * gamma + beta, then ReLU if `relu`.  Saves mean /
 * invstd [C] for the backward and updates running_mean / running_var (may be
 * NULL) with `momentum` and the unbiased variance, as torch does.
 * Pool mode (pool != NULL, B <= 64): z is not written; instead pool[b][c] =
 * max over the points of cloud b of z, pool_idx[b][c] = its first point --
 * the block followed by ``amax(dim=2)`` (TNet conv3, ndtnet.py:50-51; NDTNet
 * conv3 into the segmentation head's global feature, :152, :231), without the
 * [B][C][N] activation.  batches_tracked (may be NULL): the module's int64
 * num_batches_tracked, incremented by the launch (no launch of its own). */
int ndnet_tr_bn_fwd(const float *y, float *z, float *mean, float *invstd, float *running_mean,
                    float *running_var, const float *gamma, const float *beta, int B, int C, int N,
                    float eps, float momentum, int relu, float *pool, int32_t *pool_idx,
                    int64_t *batches_tracked, void *stream);

/* Its backward, one workgroup per channel: g = dz, masked by ReLU where the
 * forward's output (recomputed from y, mean, invstd, gamma, beta with the
 * forward's exact roundings) was not > 0; xhat = (y - mean) * invstd,
 * dgamma = sum g xhat, dbeta = sum g,
 * dy = gamma invstd (g - dbeta / M - xhat dgamma / M), dbias = sum dy (the
 * gradient of the convolution's bias).  dgamma / dbeta / dbias may be NULL.
 * Pool mode (pool_idx != NULL): dz is [B][C], the gradient of the pooled
 * output, which reaches only point pool_idx[b][c] of each cloud. */
int ndnet_tr_bn_bwd(const float *dz, const float *y, const float *mean, const float *invstd, const float *gamma,
                    const float *beta, float *dy, float *dgamma, float *dbeta, float *dbias, int B, int C, int N,
                    int relu, const int32_t *pool_idx, void *stream);

/* out[c] = sum over b, n of x[b][c][n] (a bias gradient), one workgroup per channel. */
int ndnet_tr_chan_sum(const float *x, float *out, int B, int C, int N, void *stream);

/* out[r] = sum over n of x[r][n] for `rows` rows of N contiguous values (per-cloud bias gradients). */
int ndnet_tr_row_sum(const float *x, float *out, int64_t rows, int N, void *stream);

/* count[0] += the number of the `rows` rows (of `cols` floats) whose first
 * argmax in pred equals that in gt, NaN counting as a maximum as in
 * torch.argmax: the training step's accuracy (tools/train.py:84-87) without a
 * host sync; the caller zeroes count. */
int ndnet_tr_argmax_match(const float *pred, const float *gt, int64_t rows, int cols, uint32_t *count, void *stream);
/* The same with pred channel-major, [B][C][N] (gt [B][N][C], C <= 32): the seg
 * head's log-probs as the model computes them, before their transposed view.
 * ctr[0] += the matches; ctr[1] counts workgroups, and the last writes
 * acc[0] = ctr[0] / (B N) (acc may be NULL).  The caller zeroes ctr[0..1]. */
int ndnet_tr_argmax_match_cm(const float *pred, const float *gt, int B, int C, int N, uint32_t *ctr, float *acc,
                             void *stream);

/* out[r] = the first argmax of row r of x [rows][cols] (NaN counting as a
 * maximum, as torch.argmax): the labelled NDT path's class of each point from
 * its one-hot label (ndtnet_preprocessing.py:34), batched over the clouds. */
int ndnet_row_argmax(const float *x, int64_t rows, int cols, int32_t *out, void *stream);

/* TNet FC heads in train mode (ndtnet.py:53-60: fc1 + bn4 + ReLU, fc2 + bn5 +
 * ReLU, fc3 + identity), B <= 16 rows (one per cloud), x [B][K] and W [N][K]
 * row-major (torch's Linear layout), K % 4 == 0, 16-byte aligned rows, and
 * B * K <= 16384 (x is staged whole in LDS: K <= 1024 at 16 rows).
 * Forward, one wave per output channel:
 *   y[b][n] = x[b] . W[n] + bias[n], + 1 where eye > 0 and n is a diagonal
 *   entry of the eye x eye transform (added after the bias, as torch adds the
 *   identity); with gamma: z = relu?(BatchNorm1d(y)) over the B rows (batch
 *   statistics summed in double, biased variance; mean / invstd [N] saved;
 *   running stats updated with `momentum` and the unbiased variance;
 *   batches_tracked incremented), y kept for the backward; without gamma
 *   z = y (relu and batches_tracked must be 0 / NULL).
 * Backward: ndnet_tr_fc_bwd_w (one wave per channel) -- the BatchNorm and
 * ReLU backward of channel n (as ndnet_tr_bn_bwd over B rows), dpre [B][N]
 * (the gradient of y), db = sum_b dpre, dgamma, dbeta, and the weight
 * gradient dW[n][k] = sum_b dpre[b][n] x[b][k] (any output may be NULL);
 * ndnet_tr_fc_bwd_x -- dx[b][k] = sum_n dpre[b][n] W[n][k], over `nsplit`
 * channel ranges of at most 256 (partials part [nsplit][B][K], summed in split
 * order into dx; part may be NULL with nsplit == 1).
 * ldw: the row stride of W (forward, input gradient) and of dW (weight
 * gradient) in floats, >= K (a multiple of 4 where rows are read or written
 * as float4); 0 = K.  A column slice W[:, c:] of a wider weight runs in place:
 * the seg head's per-cloud bias b + W[:, 64:] g (ndtnet.py:230-234). */
int ndnet_tr_fc_fwd(const float *x, const float *W, const float *bias, float *y, float *z, float *mean,
                    float *invstd, float *running_mean, float *running_var, const float *gamma, const float *beta,
                    int B, int K, int N, int64_t ldw, float eps, float momentum, int relu, int eye,
                    int64_t *batches_tracked, void *stream);
int ndnet_tr_fc_bwd_w(const float *dz, const float *x, const float *y, const float *mean, const float *invstd,
                      const float *gamma, const float *beta, float *dpre, float *dW, float *db, float *dgamma,
                      float *dbeta, int B, int K, int N, int64_t ldw, int relu, void *stream);
int ndnet_tr_fc_bwd_x(const float *dpre, const float *W, float *dx, float *part, int B, int K, int N, int64_t ldw,
                      int nsplit, void *stream);

/* The seg head's log_softmax over the class dim (ndtnet.py:241; x, out
 * [B][C][N]) and its backward (dx = dy - exp(y) sum_c dy, y the forward's
 * output); the training loss -sum(gt * logp) / (B N) of the one-hot target gt
 * [B][N][C] (ndnet.training.segmentation_loss) -- part: (B N + 63) / 64
 * doubles of scratch, summed in a fixed order -- and its gradient
 * dlogp[b][c][n] = -gt[b][n][c] dloss / (B N) (dloss a 1-element device
 * tensor); C <= 32. */
int ndnet_tr_log_softmax_c(const float *x, float *out, int B, int C, int N, void *stream);
int ndnet_tr_log_softmax_c_bwd(const float *y, const float *dy, float *dx, int B, int C, int N, void *stream);
int ndnet_tr_nll_onehot(const float *logp, const float *gt, double *part, float *loss, int B, int C, int N,
                        void *stream);
int ndnet_tr_nll_onehot_bwd(const float *gt, const float *dloss, float *dlogp, int B, int C, int N, void *stream);

/* The point transform t1 of the train forward (ndtnet.py:141-147, t . p and
 * t . C with the covariance multiplied on the left only): t [B][3][3], pts
 * [B][N][pld] (p in columns 0-2), extra [B][N][eld] (C row-major in columns
 * 0-8) -- e.g. both views of ndt_preprocessing's [B][N][12] rows, pld = eld =
 * 12 -- -> x [B][12][N] (rows 0-2 t . p, row 3 + 3 i + k (t . C)[i][k]); the
 * backward gives dt [B][3][3] from dx (the points and covariances are data,
 * no gradient). */
int ndnet_tr_point_transform(const float *t, const float *pts, int pld, const float *extra, int eld, float *x, int B,
                             int N, void *stream);
int ndnet_tr_point_transform_bwd(const float *dx, const float *pts, int pld, const float *extra, int eld, float *dt,
                                 int B, int N, void *stream);

/* Adam, torch.optim.Adam's fused capturable form (tools/train.py's
 * optimizer): for each of the n tensors i, steps[i][0] += 1 (device float,
 * torch's capturable step state), then m = b1 m + (1 - b1) g, v = b2 v +
 * (1 - b2) g^2, p -= (lr / (1 - b1^t)) m / (sqrt(v) / sqrt(1 - b2^t) + eps)
 * with t the new step and lr a device float (g += wd p first when
 * weight_decay != 0).  The arrays are host arrays of device pointers; the
 * launches take them by value (graph-capturable, no table upload).  The betas
 * come as doubles: 1 - beta is rounded from double, as torch's kernel gets it. */
int ndnet_tr_adam(int n, float *const *params, const float *const *grads, float *const *exp_avg,
                  float *const *exp_avg_sq, float *const *steps, const int64_t *numel, const float *lr, double beta1,
                  double beta2, float eps, float weight_decay, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* NDNET_TRAIN_H_ */
