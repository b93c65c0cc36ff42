// ndt_legacy_abi.cpp -- the reference's libndnet.so entry points over the
// batched device path (B = 1).  Host pointers in and out, as
// core_legacy/include/ndnet_core/ndt.h:59-116 declares them; the handles the
// reference hands back as struct pointers are opaque objects here.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "../../include/ndnet_amd.h"

namespace {

struct Legacy {
  void* plan = nullptr;
  hipStream_t stream = nullptr;
  uint64_t n = 0, k = 0;
  double* d_points = nullptr;
  int32_t* d_labels = nullptr;
  double* d_pc = nullptr;
  double* d_cov = nullptr;
  uint16_t* d_cls = nullptr;
  ndnet_ndt_stats* d_stats = nullptr;
  uint64_t rows = 0;  // row count of the last downsample / prune
  int refs = 0;
};

struct KLToken {
  Legacy* owner;
};

void release(Legacy* h) {
  if (!h || --h->refs > 0) return;
  if (h->plan) ndnet_ndt_plan_destroy(h->plan);
  void* bufs[] = {h->d_points, h->d_labels, h->d_pc, h->d_cov, h->d_cls, h->d_stats};
  for (void* b : bufs)
    if (b) (void)hipFree(b);
  if (h->stream) (void)hipStreamDestroy(h->stream);
  delete h;
}

#define CHK(x)                                                                         \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "ndnet_amd legacy: %s failed: %s\n", #x, hipGetErrorString(e_)); \
      return NDNET_ERR_HIP;                                                            \
    }                                                                                  \
  } while (0)

int fetch(Legacy* h, ndnet_ndt_stats* st) {
  CHK(hipMemcpyAsync(st, h->d_stats, sizeof(*st), hipMemcpyDeviceToHost, h->stream));
  CHK(hipStreamSynchronize(h->stream));
  return NDNET_OK;
}

}  // namespace

extern "C" {

const char* ndnet_amd_version(void) { return "ndnet_amd 0.1 (gfx950)"; }

int ndt_downsample(double* point_cloud, unsigned short point_dim, unsigned long num_points, unsigned int* len_x,
                   unsigned int* len_y, unsigned int* len_z, double* offset_x, double* offset_y, double* offset_z,
                   double* voxel_size, unsigned short* classes, unsigned short num_classes,
                   unsigned long num_desired_points, double* downsampled_point_cloud,
                   unsigned long* num_downsampled_points, double* covariances, unsigned short* downsampled_classes,
                   void** nd_array, unsigned long* num_valid_nds, void** kl_divergences,
                   unsigned long* num_kl_divergences) {
  if (nd_array) *nd_array = nullptr;
  if (kl_divergences) *kl_divergences = nullptr;
  if (!point_cloud || num_points == 0 || num_desired_points == 0) return NDNET_ERR_ARG;
  if (point_dim != 3) {
    fprintf(stderr, "ndnet_amd: point_dim %u unsupported (the reference core assumes 3)\n", point_dim);
    return NDNET_ERR_ARG;
  }
  Legacy* h = new Legacy();
  h->n = num_points;
  h->k = num_desired_points;
  h->refs = 1;
  int rc = ndnet_ndt_plan_create(1, num_points, num_desired_points, (int)num_classes, 0, &h->plan);
  // One launch per stage, not the fused k_front: k_front's grid barrier needs
  // every workgroup of the cloud resident at once (at B = 1 that is one per
  // CU), and this entry point is called concurrently -- the reference's
  // DataLoader workers (tools/train.py:135-137) each run NDT_Sampler in their
  // own process -- so two partly resident k_front grids could each wait for
  // the other until the barrier timeout.  The multi-launch path has no
  // residency requirement and computes the same bits (test_front_kernel_equals_multikernel_path).
  if (rc == NDNET_OK) rc = ndnet_ndt_set_path(h->plan, 1);
  if (rc != NDNET_OK) {
    release(h);
    return rc;
  }
  hipError_t e = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking);
  const size_t k = num_desired_points;
  if (e == hipSuccess) e = hipMalloc(&h->d_points, num_points * 3 * sizeof(double));
  if (e == hipSuccess && classes) e = hipMalloc(&h->d_labels, num_points * sizeof(int32_t));
  if (e == hipSuccess) e = hipMalloc(&h->d_pc, k * 3 * sizeof(double));
  if (e == hipSuccess) e = hipMalloc(&h->d_cov, k * 9 * sizeof(double));
  if (e == hipSuccess) e = hipMalloc(&h->d_cls, k * sizeof(uint16_t));
  if (e == hipSuccess) e = hipMalloc(&h->d_stats, sizeof(ndnet_ndt_stats));
  if (e == hipSuccess)
    e = hipMemcpyAsync(h->d_points, point_cloud, num_points * 3 * sizeof(double), hipMemcpyHostToDevice, h->stream);
  std::vector<int32_t> lbl;
  if (e == hipSuccess && classes) {
    lbl.assign(classes, classes + num_points);
    e = hipMemcpyAsync(h->d_labels, lbl.data(), num_points * sizeof(int32_t), hipMemcpyHostToDevice, h->stream);
  }
  if (e != hipSuccess) {
    fprintf(stderr, "ndnet_amd legacy: setup failed: %s\n", hipGetErrorString(e));
    release(h);
    return NDNET_ERR_HIP;
  }
  rc = ndnet_ndt_run_f64(h->plan, h->stream, h->d_points, h->d_labels, h->d_pc, h->d_cov, h->d_cls, nullptr,
                         h->d_stats);
  ndnet_ndt_stats st;
  if (rc == NDNET_OK) rc = fetch(h, &st);
  if (rc != NDNET_OK) {
    release(h);
    return rc;
  }
  *len_x = st.len[0];
  *len_y = st.len[1];
  *len_z = st.len[2];
  *offset_x = st.offset[0];
  *offset_y = st.offset[1];
  *offset_z = st.offset[2];
  *voxel_size = st.voxel_size;
  if (st.rc != 0) {
    release(h);
    return st.rc;
  }
  h->rows = k;
  const uint64_t rows = st.num_out < k ? st.num_out : k;
  if (downsampled_point_cloud) e = hipMemcpy(downsampled_point_cloud, h->d_pc, rows * 24, hipMemcpyDeviceToHost);
  if (e == hipSuccess && covariances) e = hipMemcpy(covariances, h->d_cov, rows * 72, hipMemcpyDeviceToHost);
  if (e == hipSuccess && downsampled_classes)
    e = hipMemcpy(downsampled_classes, h->d_cls, rows * 2, hipMemcpyDeviceToHost);
  if (e != hipSuccess) {
    release(h);
    return NDNET_ERR_HIP;
  }
  if (num_downsampled_points) *num_downsampled_points = st.num_out;
  if (num_valid_nds) *num_valid_nds = st.num_valid;
  if (num_kl_divergences) *num_kl_divergences = st.num_kl;
  h->refs = 2;  // one for the ND handle, one for the KL handle
  if (nd_array) *nd_array = h;
  else release(h);
  if (kl_divergences) *kl_divergences = new KLToken{h};
  else release(h);
  return 0;
}

int prune_nds(void* nd_array, unsigned int len_x, unsigned int len_y, unsigned int len_z,
              unsigned long num_desired_nds, unsigned long* num_valid_nds, void* kl_divergences,
              unsigned long* num_kl_divergences) {
  (void)len_x; (void)len_y; (void)len_z; (void)kl_divergences;
  Legacy* h = (Legacy*)nd_array;
  if (!h || num_desired_nds == 0) return NDNET_ERR_ARG;
  if (num_desired_nds > h->k) {  // more rows than the handle's buffers; the list can only shrink
    if (num_valid_nds && num_desired_nds > *num_valid_nds) return -1;
    return NDNET_ERR_ARG;
  }
  int rc = ndnet_ndt_prune(h->plan, h->stream, num_desired_nds, nullptr, nullptr, h->d_pc, h->d_cov, h->d_cls,
                           h->d_stats);
  ndnet_ndt_stats st;
  if (rc == NDNET_OK) rc = fetch(h, &st);
  if (rc != NDNET_OK) return rc;
  if (st.prune_rc != -1) h->rows = num_desired_nds;
  if (num_valid_nds) *num_valid_nds = st.num_valid;
  if (num_kl_divergences) *num_kl_divergences = st.num_kl;
  return st.prune_rc;
}

int to_point_cloud(void* nd_array, unsigned int len_x, unsigned int len_y, unsigned int len_z, double offset_x,
                   double offset_y, double offset_z, double voxel_size, double* point_cloud,
                   unsigned long* num_points, double* covariances, unsigned short* classes) {
  (void)len_x; (void)len_y; (void)len_z; (void)offset_x; (void)offset_y; (void)offset_z; (void)voxel_size;
  Legacy* h = (Legacy*)nd_array;
  if (!h) return NDNET_ERR_ARG;
  ndnet_ndt_stats st;
  int rc = fetch(h, &st);
  if (rc != NDNET_OK) return rc;
  const uint64_t rows = st.num_out < h->rows ? st.num_out : h->rows;
  if (point_cloud) CHK(hipMemcpy(point_cloud, h->d_pc, rows * 24, hipMemcpyDeviceToHost));
  if (covariances) CHK(hipMemcpy(covariances, h->d_cov, rows * 72, hipMemcpyDeviceToHost));
  if (classes) CHK(hipMemcpy(classes, h->d_cls, rows * 2, hipMemcpyDeviceToHost));
  if (num_points) *num_points = st.num_out;
  return 0;
}

void free_nds(void* nd_array, unsigned long num_nds) {
  (void)num_nds;
  release((Legacy*)nd_array);
}

void free_kl_divergences(void* kl_divergences) {
  KLToken* t = (KLToken*)kl_divergences;
  if (!t) return;
  release(t->owner);
  delete t;
}

void print_matrix(double* matrix, int rows, int cols) {
  if (!matrix) return;
  for (int r = 0; r < rows; r++) {
    for (int c = 0; c < cols; c++) printf("%f ", matrix[(size_t)r * cols + c]);
    printf("\n");
  }
  fflush(stdout);
}

}  // extern "C"
