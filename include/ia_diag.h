/* ia_diag.h — diagnostic entry points of libia.so (NOT part of the reference boundary).
 * Used by tools/screen_bench (kernel A/B timing and rocprofv3 PMC runs outside any
 * Python/torch process) to drive the matcher's stages one at a time.  Same conventions
 * as ia.h: device pointers, void* hipStream_t, 0 / IA_E_* return codes. */
#ifndef IA_DIAG_H
#define IA_DIAG_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* bytes of the screen's candidate buffer for M queries over nrows DB rows */
size_t ia_diag_cand_bytes(int M, long nrows);
/* rows of the fp32 query buffer qp (IA_DP floats each) a screen of M queries reads */
int ia_diag_qp_rows(int M);
/* fp64 queries (M x IA_DP) -> MFMA-ordered fp32 qp + |q - c|^2 */
int ia_diag_query_rows(const double *q64, int M, const double *center, float *qp, double *nq,
                       void *stream);
/* one screen launch; variant bits 0-3: 0 = queries in VGPRs, 1 = queries in LDS,
 * 2 = pipelined epilogue, 3 = 3-deep prefetch, 4/5 = L2-hot diagnostics,
 * 6 = segment-minimum screen (default matcher);
 * bits 4-7: cap on query tiles per wave (0 = default) */
int ia_diag_screen(const float *db, long nrows, const float *qp, int M, void *cand,
                   int variant, void *stream);

/* split-f16 screen (the default matcher's stage 1): query rows in both
 * forms (qp as ia_diag_query_rows, q16 = ia_diag_qp_rows(M) x 256 B, zeroed by the caller;
 * amax from ia_db_build), and one split-f16 screen launch (ia_diag_screen16) -> segment
 * minima (screen units).  Its flags select the form (0 = the default shape rule): bits 0-3
 * cap on query tiles per wave, 0x100 per-wave form, 0x200 no pipelined epilogue, 0x400
 * fragment prefetch, 0x800 pipelined epilogue at 3 tiles, 0x1000 spanning form (0x2000 /
 * 0x8000 its no-copy diagnostics), 0x4000 uneven shares, 0x10000 double-buffered fragment
 * registers, 0x20000 non-temporal DB stream, 0x40000 balanced shares, 0x80000 chain-balanced
 * stages.  Every form writes bitwise the same minima (tests/test_gpu_split16.py). */
int ia_diag_query_rows16(const double *q64, int M, const double *center, const float *amax,
                         float *qp, void *q16, double *nq, void *stream);
/* select the exact matcher's screen for this process (overrides IA_MATCH_ALG): 0 per-lane
 * top-K (f32), 1 segment minima (f32 MFMA), 2 segment minima (split-f16 MFMA, default);
 * returns the previous value (a negative alg only queries it). */
int ia_diag_set_match_alg(int alg);
/* exact stage form for this process: 0 one workgroup per query (k_rescore), 1 the work list
 * (k_select / k_items / k_gather), -1 the default (work list above 2^20 rows or when the
 * per-pixel tail runs separately); other values leave it; returns the previous value */
int ia_diag_set_rescore_mode(int mode);
/* HIP-graph capture of ia_synth_level's wave loop for this process (overrides IA_GRAPH):
 * 0 off, 1 levels of <= 2^18 rows, 2 every single-GPU level; other values leave it;
 * returns the previous value */
int ia_diag_set_graph_mode(int mode);
int ia_diag_screen16(const float *db, long nrows, const void *q16, int M, float *segmin,
                     int maxnq, void *stream);

#ifdef __cplusplus
}
#endif
#endif
