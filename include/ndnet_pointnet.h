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
 * Layer weights are stored transposed, W^T[K][N] row-major (K input channels x
 * N output channels), with BatchNorm folded in, K padded to a multiple of 4
 * and N to 32.
 */
#ifndef NDNET_POINTNET_H_
#define NDNET_POINTNET_H_
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NDNET_PN_MAX_LAYERS 5

typedef struct ndnet_pn_layer {
  const float* wT;        // [K][ldw] (+ cloud * w_cloud_stride), 16-byte aligned
  int64_t w_cloud_stride; // 0 for shared weights, else the per-cloud stride of folded weights
  const float* bias;      // [N] (+ cloud * bias_cloud_stride)
  int64_t bias_cloud_stride;
  int32_t K, N;           // padded sizes: K % 4 == 0, N % 32 == 0
  int32_t relu;
  int32_t ldw;            // row stride of wT in floats (>= N, % 4 == 0)
  int32_t fuse_next;      // 1: this layer's output is produced in 64-column chunks, each consumed at once
                          // by the next layer (whose N <= 256) -- the activation never occupies LDS whole
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
  int32_t max_width;      // widest activation of LDS region 0 (the input, layers 1, 3, ... outputs)
  int32_t max_width2;     // widest activation of LDS region 1 (layers 0, 2, ... outputs); a fused
                          // layer's output is not stored in either region
  float* out;             // mode 1
} ndnet_pn_chain;

/* Runs one chain over `batch` clouds on `stream` (a hipStream_t; NULL = default
 * stream).  Returns 0, NDNET_ERR_ARG (-20) for an inconsistent argument block
 * (layer sizes, LDS region widths) or NDNET_ERR_HIP (-21) on a launch failure.
 * No allocation, no synchronisation: graph-capturable. */
int ndnet_pn_chain_run(const ndnet_pn_chain *args, int batch, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* NDNET_POINTNET_H_ */
