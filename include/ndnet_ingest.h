/*
 * ndnet_ingest.h -- C ABI of the native ASCII-PLY reader in libndnet_amd.so
 * (ndt-net_amd/csrc/ply_ingest.cpp): the parsing half of the reference's
 * CARLA_Seg.get_data_pcl (ndnet/datasets/CARLA_Seg.py:97-136), which reads a
 * scan with Python readlines + split + float() per token.
 *
 * Semantics (same as the reference):
 *   - the first `num_header_lines` lines are skipped (default 10 there);
 *   - every further line gives x, y, z = its first three tokens, parsed as
 *     decimal -> double (correctly rounded, as Python float()) and the class
 *     tag = its LAST token, parsed as an integer (Python int());
 *   - blank lines are skipped; a class tag > num_classes (or < 0), a line with fewer
 *     than four tokens or a malformed number is an error.
 * The random subsample and the one-hot encoding (CARLA_Seg.py:137-175) stay
 * in Python (ndnet.datasets.carla_seg), on numpy's global RNG as there.
 * Parsing runs on `threads` host threads (0 = hardware concurrency), each on
 * a newline-aligned byte range of the memory-mapped file.
 */
#ifndef NDNET_INGEST_H_
#define NDNET_INGEST_H_
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NDNET_PLY_ERR_IO (-30)     /* open / map failure */
#define NDNET_PLY_ERR_PARSE (-31)  /* malformed line; *n_out = its 0-based data-line index */
#define NDNET_PLY_ERR_CLASS (-32)  /* class tag > num_classes; *n_out = the data-line index */
#define NDNET_PLY_ERR_CAP (-33)    /* more data lines than `capacity`; *n_out = the count */

/* Counts the data lines (after the header) of `path` into *n_out. */
int ndnet_ply_count(const char *path, int num_header_lines, uint64_t *n_out);

/* Parses up to `capacity` data lines: xyz[i*3..] (double), cls[i] (uint16).
 * *n_out = the number of points on success. */
int ndnet_ply_read(const char *path, int num_header_lines, int num_classes, double *xyz, uint16_t *cls,
                   uint64_t capacity, uint64_t *n_out, int threads);

#ifdef __cplusplus
}
#endif
#endif /* NDNET_INGEST_H_ */
