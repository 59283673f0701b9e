/* ia_diag.h — diagnostic entry points of libia.so (NOT part of the reference boundary).
 * Used by tools/screen_bench (kernel timing and rocprofv3 PMC runs outside any
 * Python/torch process) and by the tests to drive the matcher's stages one at a time.
 * Same conventions as ia.h: device pointers, void* hipStream_t, 0 / IA_E_* return codes. */
#ifndef IA_DIAG_H
#define IA_DIAG_H

#include <stddef.h>

#include "ia.h"

#ifdef __cplusplus
extern "C" {
#endif

/* rows of the query buffers (qp: IA_DP floats, q16: 256 B each) a screen of M queries
 * reads; the caller zeroes them */
int ia_diag_qp_rows(int M);
/* fp64 queries (M x IA_DP) -> the fp32 re-screen rows qp, the split-f16 screen rows q16
 * and |q - c|^2 (amax from ia_db_build) */
int ia_diag_query_rows16(const double *q64, int M, const double *center, const float *amax,
                         float *qp, void *q16, double *nq, void *stream);
/* one split-f16 screen launch (the exact matcher's stage 1) -> segment
 * minima segmin[M][nseg] (screen units; nseg = ia_db_rows_padded / segment rows) */
int ia_diag_screen16(const void *db, long nrows, const void *q16, int M, float *segmin,
                     void *stream);
/* the matcher's stage order of rows [row0, row0 + nrows) of a level W wide with Himg
 * scanlines per A' image (ia_internal.h StageMap): out = {W (0: linear chunks), strips per
 * scanline, 128-row stages per chunk}.  With strips, chunk c is the 128-px column strip
 * c % strips of stages-per-chunk consecutive scanlines and a segment is 4 consecutive stages
 * of a chunk; linear: chunk c = rows [c ch, (c + 1) ch). */
int ia_diag_stage_map(long row0, long nrows, int W, int Himg, int *out);
/* the row-form screen over rows [row0, row0 + nrows) of src's level in the product's stage
 * order (the same minima as the image form, bit for bit) */
int ia_diag_screen16_rows(const IaSrcLevel *src, long row0, long nrows, const void *db,
                          const void *q16, int M, float *segmin, void *stream);
/* the same screen streaming the DB's image form (ia_db_build_image) of rows
 * [row0, row0 + nrows) of src: the same minima bit for bit */
int ia_diag_screen16_image(const IaSrcLevel *src, long row0, long nrows, const void *dbi,
                           const void *q16, int M, float *segmin, void *stream);
/* the rotated (R16) screen of M fp64 query rows (IA_DP doubles each) over rows
 * [row0, row0 + nrows) of src's rotated DB (ia_db_build_rot with rot, amax {A, A_skip}):
 * the R16 query rows into q16 (qrows of 256 B, zeroed by the caller), nq[m] = |q'|^2,
 * nsk[m] = |kappa_skip|^2, then segmin[M][nseg] in the product's stage order (screen units) */
int ia_diag_screen16r(const IaSrcLevel *src, long row0, long nrows, const void *dbr, const float *rot,
                      const float *amax, const double *center, const double *q64, int M, void *q16,
                      double *nq, double *nsk, float *segmin, void *stream);
/* exact stage form for this process: 0 one workgroup per query (k_rescore), 1 the work list
 * (k_select / k_items / k_gather), -1 the default (work list above 2^20 rows); other values
 * leave it; returns the previous value */
int ia_diag_set_rescore_mode(int mode);
/* ia_db_build form for this process: 1 [default] the LDS-tiled kernels where the level's
 * width and row0 are multiples of 32, 0 always the per-row gather kernels (same bytes);
 * other values leave it; returns the previous value */
int ia_diag_set_db_build_form(int tiled);
/* pyramid_reduce form for this process: stream 1 = the one-pass k_pyr_wave where the
 * coefficients are a halving (default), 0 = the tiled k_pyr_reduce / two-kernel path only;
 * oh is unused.  Returns the previous stream flag. */
int ia_diag_set_pyr_form(int stream, int oh);
/* HIP-graph capture of ia_synth_level's wave loop for this process (overrides IA_GRAPH):
 * 0 off, 1 levels of <= 2^18 rows, 2 every single-GPU level; other values leave it;
 * returns the previous value */
int ia_diag_set_graph_mode(int mode);
/* the fused per-wave kernel (k_xwave: exact stage, device-side exchange, per-pixel tail and
 * the next wave's query rows in one launch) for this process: 2 [default, IA_XWAVE] wherever
 * it applies, with its strip form k_xstrip (fp64 windows) on strip-order image-form levels;
 * 1 k_xwave only; 0 the separate kernels (k_query_wave, k_rescore / work list,
 * k_peer_finish); other values leave it; returns the previous value */
int ia_diag_set_xwave(int on);
/* the split-f16 screen's stage schedule for this process (IA_SCREEN_SCHED): 0 tile-major,
 * 1 chain-major pipelined (same minima); returns the previous value, -1 leaves it */
int ia_diag_set_screen_sched(int sched);
/* strip-order image-form levels: the producer / consumer screen k_screen16p (1, default;
 * IA_SCREEN_PC) or k_screen16i (0); same minima; returns the previous value, -1 leaves it */
int ia_diag_set_screen_pc(int on);
/* the rotated screen's form for this process (IA_R16_FORM): 1 [default] the wave-owned
 * k_screen16w (queries staged in LDS, DB tiles in each wave's registers), 0 the block form
 * k_screen16r (DB staged through LDS); same minima; returns the previous value */
int ia_diag_set_r16_form(int form);
/* ia_db_build_image without rows: the fused one-pass build k_img_build (1, default;
 * IA_IMG_FUSED) or the range + bound + pad + norm-pass kernels (0); same bytes and amax */
int ia_diag_set_img_fused(int on);
/* k_screen16p stage stamps into buf (device, 16 waves x 256 u64: blocks 0 and 300, per
 * stage < 64 four s_memtime values; see ia_screen16.hip pc_stamp), NULL turns them off */
int ia_diag_screen_trace(void *buf);

/* 3-channel matching (ia_color3.hip): IA_COLOR16 (1 the split-f16 screen + exact stage, 0 the
 * exhaustive fp64 search; returns the previous value), the exact stage's counters since the
 * last call ([candidate 32-row tiles rescored, queries that scanned every tile]; the first call
 * starts counting), and the screen of M queries (M x 165) over an ia_db3_build buffer: per
 * (query, 32-row tile) the minimum screen value unscaled (M x ntiles, ntiles = ceil(nrows /
 * 32)), eps3 and |q'|^2 per query */
int ia_diag_set_color16(int on);
int ia_diag_color16_stats(unsigned long long *out);
int ia_diag_screen3(const void *db3, long nrows, const double *q165, int M, double *e, double *eps,
                    double *qn);
/* with IA_XW_TRACE=<level tag>: the fused kernel's phase stamps of that level (100 MHz
 * s_memrealtime) for waves < 4096 and the first 8 pixels of each, 12 stamps per pixel:
 * {start, ticket, e*, candidates, re-screen, rescore | coherence, winner, exchange,
 * update, neighbour, end}; 4096 x 8 x 16 u64 (slots 11-15: wave-level stamps of the re-screen, coherence and rescore) */
int ia_diag_xwave_trace(unsigned long long *out);

/* the sharded synthesis path in ONE process: level a (a->comm = NULL, a->db unused) with
 * its database split into n shards {db, row0, nrows, amax} (each ia_db_build'ed from its
 * row range, in row order, covering all N_total rows); per wave every shard's exact stage
 * runs here in turn and k_finish reduces their records as after the cross-rank exchange.
 * The product's multi-rank reduction on one GPU, for tests. */
typedef struct {
    const void *db;
    long row0, nrows;
    const float *amax;
    const void *dbi;    /* NULL or the shard's image form */
} IaShardDb;
int ia_diag_synth_level_shards(const IaSynthArgs *a, const IaShardDb *shards, int n,
                               void *stream);

/* the device-side exchange's protocol alone (ia.h ia_peer_*): nwaves waves of M queries,
 * every rank publishing a known record per (wave, query); *bad = the number of (wave,
 * query) whose collected records or minimum differ from the expected ones.  Every rank
 * of the exchange calls it at once. */
int ia_diag_peer_stress(void *comm, int nwaves, int M, int *bad, void *stream);
/* with IA_PEER_TRACE=1 at ia_peer_create: per epoch < 1024 and query < 8 of the exact
 * stage's exchange {own distance, own row, collected distance, collected row} (1024 x 8 x 4
 * doubles) */
int ia_diag_peer_trace(void *comm, double *out);

/* R16c (3-channel rotated screen): A_skip of a rotated DB (fp32); one screen of M given query
 * rows (M x 165) -> tile minima in unscaled units e[M][ntiles], eps[M] (the exact stage's
 * bound), qn[M] = |q'|^2 */
int ia_diag_db3_askip(const void *dbr, long nrows, float *out);
int ia_diag_screen3r(const void *db3, const void *dbr, const float *rot, long nrows, const double *q165, int M,
                     double *e, double *eps, double *qn);

#ifdef __cplusplus
}
#endif
#endif
