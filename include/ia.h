/* ia.h — C-ABI of the MI355X-native Image Analogies synthesis core (libia.so).
 *
 * Drop-in boundary for the reference's hot path (rubychen0611/image-analogies-python,
 * SURVEY.md §8(b)).  Every entry point below names the reference interface it
 * replaces.  Conventions:
 *   - all array arguments are caller-owned DEVICE memory (row-major, element counts);
 *     the library never allocates or frees caller memory; scratch comes in through a
 *     `workspace` pointer sized by the matching *_workspace_bytes() query;
 *   - `stream` is a hipStream_t passed as void* (no HIP/torch types in the ABI); work is
 *     enqueued stream-ordered and the call returns without synchronising unless noted;
 *   - return 0 on success, <0 on error (IA_E_*); ia_last_error() gives the message
 *     (thread-local).  The Python host layer raises on any non-zero return.
 *   - numerics: fp64 everywhere the reference computes in fp64, in the reference's
 *     operation order (numpy pairwise-8 sums, no FMA contraction); the matcher screens with
 *     split-f16 MFMA (a filter with a proven error bound), re-screens the candidates in
 *     fp32 and rescores them in fp64, so indices and distances are exact.
 */
#ifndef IA_H
#define IA_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define IA_OK 0
#define IA_E_ARG (-1)       /* bad argument / shape                      */
#define IA_E_HIP (-2)       /* HIP runtime error                         */
#define IA_E_COMM (-3)      /* RCCL error                                */
#define IA_E_UNSUPPORTED (-4)
#define IA_E_TIMEOUT (-5)   /* device-side exchange: another rank's records never came */
#define IA_E_SCHED (-6)     /* device schedule fault: a neighbouring pixel's decision wait
                               timed out inside the fused per-wave kernel (never a peer) */

#define IA_D 55             /* feature length, 1 channel: 9 + 25 + 9 + 12          */
#define IA_DP 56            /* padded row: 55 features + squared norm slot         */

const char *ia_last_error(void);
int ia_version(void);

/* One pyramid level pair of the A / A' database (algorithms.py:50-70 inputs).
 * A_sm/A_lg: A at levels l-1 (A_hs x A_ws) and l (Ah x Aw), fp64.
 * Ap_sm/Ap_lg: nAp A' images stacked contiguously with the same shapes. */
typedef struct {
    const double *A_sm, *A_lg, *Ap_sm, *Ap_lg;
    int A_hs, A_ws, Ah, Aw, nAp;
} IaSrcLevel;

/* ---- a1/a2: img_preprocess.py:6-13 convert_to_YIQ (+ image_analogies.py:32-50 scale).
 * src: npix x 3 interleaved, dtype 0=uint8, 1=float32, 2=float64; x = src / div.
 * yiq (npix x 3, nullable) and y (npix, nullable) receive the einsum result. */
int ia_rgb_to_yiq(const void *src, int src_dtype, long npix, double div, double *yiq,
                  double *y, void *stream);
/* img_preprocess.py:16-22 convert_to_RGB: in npix x 3 -> out npix x 3. */
int ia_yiq_to_rgb(const double *in, long npix, double *out, void *stream);
/* the colour image of a level before plt.imsave (image_analogies.py:216-217, 255-258), npix
 * pixels -> out (npix x 3 fp64): yiq non-NULL (convert): RGB of (bp, yiq[.., 1], yiq[.., 2])
 * clipped to [0, 1]; else the source colour of every pixel, ap[((im * ah + s_r) * aw + s_c)
 * * C + c] (nAp x ah x aw x C, C = 1 repeated over RGB, or 3) */
int ia_color_output(const double *bp, const double *yiq, const int32_t *s, const int32_t *im, const double *ap,
                    int ah, int aw, int C, long npix, double *out, void *stream);
/* scale only (convert=False path, image_analogies.py:51-56): out = src / div. */
int ia_scale_to_f64(const void *src, int src_dtype, long n, double div, double *out,
                    void *stream);
/* a3/a4: img_preprocess.py:25-44.  mode 0: y = a*x (compress_values);
 * mode 1: y = a*(x - m) + b (remap_luminance with a = s_B/s_A). */
int ia_axpb_f64(const double *x, long n, int mode, double a, double m, double b,
                double *y, void *stream);

/* ---- a5: one skimage pyramid_reduce step (img_preprocess.py:56).
 * src H x W -> dst h x w (h = ceil(H/2), w = ceil(W/2)); coef = (sx, tx, sy, ty) of
 * skimage's estimated AffineTransform; taps = (w0, w1, w2, w3).
 * workspace: ia_pyr_workspace_bytes(H, W). */
size_t ia_pyr_workspace_bytes(int H, int W);
int ia_pyr_reduce_f64(const double *src, int H, int W, double *dst, int h, int w,
                      const double coef[4], const double taps[4], void *workspace,
                      void *stream);

/* deterministic mean of n doubles (used for the screening centre). */
size_t ia_mean_workspace_bytes(long n);
int ia_mean_f64(const double *x, long n, double *out, void *workspace, void *stream);
/* unbiased variance of x[0..n): out[0] = sum (x - mean)^2 / (n - 1), out[1] = mean (two
 * passes; workspace of ia_mean_workspace_bytes(n)) */
int ia_var_f64(const double *x, long n, double *out, void *workspace, void *stream);

/* ---- a9: algorithms.py:11-47 compute_feature_array, one level, 1 channel.
 * out: (h*w) x (full ? 34 : 21) fp64. */
int ia_level_features_f64(const double *sm, int hs, int ws, const double *lg, int h, int w,
                          int full, double *out, void *stream);

/* ---- a10: algorithms.py:50-70 create_index — the screening database for rows
 * [row0, row0 + nrows) of As[level] (= A full | A'_i half): each row (a - center, k < 55;
 * |a - center|^2 at k = 55) scaled by powers of two and split into f16 pairs x = x_h + x_l
 * (DESIGN.md §4b), stored per 32-row tile as 7 contiguous 1 KiB register groups (224 B per
 * row): the MFMA screen's operand, and the exact stage's fp32 re-screen input (x_h + x_l
 * is exact in fp32).  Rows are padded to ia_db_rows_padded(nrows) (whole chunks of
 * ia_db_chunk_rows, a multiple of 4 chunks) by repeating the last real row.  amax (device,
 * 1 float) receives A >= max_row |a - center|, bounded from the value ranges of the level's
 * four images (max with its prior value: zero it first). */
long ia_db_rows_padded(long nrows);
/* bytes of the db buffer ia_db_build fills: 224 B per padded row */
size_t ia_db_bytes(long nrows);
int ia_db_chunk_rows(long nrows);
/* the chunk target (chunks per database, 4 .. 512; default 512) from which every database's
 * chunking (ia_db_chunk_rows, the padded row counts, workspace sizes) derives; returns the
 * previous one (any value outside the range only queries).  Per calling host thread: a
 * database must be built, sized and synthesised under the same target by the same thread;
 * other threads keep their own target (default 512).  synthesize_batch_dev uses
 * max(64, 512 / K) for a batch of K jobs (longer chunks, the same results). */
long ia_set_chunk_target(long chunks);
int ia_db_build(const IaSrcLevel *src, long row0, long nrows, const double *center,
                void *db, float *amax, void *stream);
/* the DB's image form: each pixel's split-f16 pair once, in images padded by
 * reflection, plus the rows' norm slots — 59 MB instead of 940 MB at the c4 finest level; the
 * screen builds its stages from it in LDS and the exact stage re-screens from it.  Applies when the level width and row0 are
 * multiples of 128 and the rows fill whole chunks: ia_db_image_bytes returns 0 otherwise.
 * db (nullable): the row form from ia_db_build, whose amax and norm slots are then reused;
 * with db NULL the image form is built alone (amax as ia_db_build computes it: zero it
 * first) and the matcher runs from it alone — screen and exact stage, no 224-B rows.
 * center must be constant over k < 34 and over k >= 34 (as ia_center_fill makes it). */
size_t ia_db_image_bytes(const IaSrcLevel *src, long row0, long nrows);
int ia_db_build_image(const IaSrcLevel *src, long row0, long nrows, const double *center,
                      const void *db, float *amax, void *dbi, void *stream);
/* per-dimension screening centre: k < 34 -> mA, k >= 34 -> mAp (host scalars). */
int ia_center_fill(double *center, double mA, double mAp, void *stream);

/* ---- §8(f)1: approximate matcher (config matcher='lsh', the reference's
 * output/freud-crop-filt-lsh.jpg variant; no reference code exists for it).  E2LSH over
 * the centred DB rows: L tables of k hashes h = floor((p . a' + b) / w); proj is
 * L*k rows of IA_DP floats on device (p in elements 0..54, b in element 55).
 * mem: ia_lsh_bytes(nrows, L) bytes of device memory, filled by ia_lsh_build from rows
 * [row0, row0 + nrows) of the level (fp32 of a - center, gathered from the pyramids).  A query returns the exact-distance (fp64) best of up to 32 rows
 * per table bucket it falls in (lexicographic (distance, row) minimum; an empty bucket
 * contributes the 4 entries around its position in the sorted table). */
typedef struct {
    void *mem;
    const float *proj;
    int L, k;
    float w;
} IaLsh;
size_t ia_lsh_bytes(long nrows, int L);
int ia_lsh_build(const IaSrcLevel *src, long row0, long nrows, const double *center,
                 const IaLsh *lsh, void *stream);
/* bucket keys are masked to ia_lsh_bits(nrows) = ceil(log2(nrows)) + 1 bits (<= 30). */
int ia_lsh_bits(long nrows);

/* ---- a11: algorithms.py:73-75 best_approximate_match, batched: exact 1-NN of M
 * fp64 queries (M x 55, row stride IA_DP) over the DB rows built above (split-f16 MFMA
 * screen, fp32 re-screen of the candidate segments, fp64 rescore from the src pyramids).  Outputs idx (global row, int64) and the fp64
 * distance (pairwise-8 sum of squares, the oracle's value).  lsh (nullable): use the
 * approximate LSH matcher over the same rows instead. */
typedef struct {
    IaSrcLevel src;
    const void *db;            /* ia_db_build output (NULL with dbi: image form only) */
    long row0, nrows;          /* this shard's global row range            */
    const double *center;      /* 55 (device)                              */
    const float *amax;         /* device scalar from ia_db_build           */
    const double *q64;         /* M x IA_DP queries (device)               */
    int M;
    int64_t *idx;              /* out M                                    */
    double *dist;              /* out M                                    */
    void *workspace;
    const IaLsh *lsh;          /* NULL: exact matcher                      */
    const void *dbi;           /* NULL, or ia_db_build_image output: the screen and the exact
                                  stage read the image form instead of the rows (same results) */
} IaMatchArgs;
size_t ia_match_workspace_bytes(int M, long nrows);
int ia_match_batch(const IaMatchArgs *a, void *stream);

/* ---- a13/a14: per-pixel helpers of algorithms.py:92-135 on device.
 * ia_coherence_pick: argmin over n candidate rows of sqrt(pairwise8((a - q)^2)),
 *   first minimum -> *out (device int32).  rows: n x 55, q: 55.
 * ia_wdist_batch: out[i] = s*s, s = sqrt(pairwise8(((a_i - q_i) * w)^2)). */
int ia_coherence_pick(const double *rows, int n, const double *q, int32_t *out,
                      void *stream);
int ia_wdist_batch(const double *a, const double *q, const double *w, int n, double *out,
                   void *stream);

/* ---- the rotated split-f16 database (R16; replaces the screen's 11 MFMAs
 * per 32x32 tile by 4 at P = 3).  Per level (shard): ia_db_cov -> the 55 x 55 covariance of ~64 k
 * sampled centred rows (fp64, cov[0 .. 56*56) row-major, stride 56; the rest of the buffer,
 * ia_db_cov_bytes() in all, is scratch); the caller takes its eigenvectors (host; any basis
 * orthonormal to fp64 precision keeps the matcher exact: the bound adapts to the components'
 * order) and passes rot = V rounded to fp32, rot[k * 56 + j]
 * = V[k][j] with the components j by decreasing variance, in a buffer of 13,312 B (zero
 * padded).  ia_db_build_rot then writes the rotated split rows (128 B per padded row at
 * P = 3), after them per 512-row segment A_skip,j (fp32, the max over the segment's rows of
 * the norm of components P..54) and a byte c_j with A_skip c_j / 255 >= A_skip,j (the exact
 * stage's per-segment bound), ia_db_rot_bytes in all; and amax[0] = A (as ia_db_build),
 * amax[1] = A_skip (max over all rows; zero it first).  ia_db_rot_applies: 1 where the synthesis
 * can use it (every level of the fused per-wave kernel, strip-order or not).
 * Precondition, checked (IA_E_ARG otherwise; one 12 KB read-back of rot per call): with V_f
 * the fp32 matrix passed, ||V_f^T V_f - I||_F <= 2 sqrt(55) 2^-24, the non-orthogonality the
 * screen's bound budgets (an fp32 eigh result or a perturbed basis fails it). */
int ia_db_rot_applies(const IaSrcLevel *src, long row0, long nrows);
/* the build's R16 form: components carried as split pairs (P), K-slots per row (16 per MFMA) */
int ia_db_rot_components(void);
/* resources (LDS bytes per workgroup, VGPRs per lane) of a sharded level's screen (which 0:
 * the rotated k_screen16r, 1: k_screen16i) and of the fused strip kernel (rot 1: R16 form)
 * that waits for other ranks: the forward-progress rule of DESIGN.md §7
 * (image_analogies.residency_ok) */
int ia_screen_resources(int which, int *lds, int *vgprs);
int ia_fused_resources(int rot, int *lds, int *vgprs);
int ia_db_rot_slots(void);
/* the A^2 coefficient E2 of the screen's bound eps_R = u (360 A|q'| + E2 A^2) + 2^-9 1.01
 * A_skip |q'_skip| (90 for the 16x16x32 MFMA form, 60 for 32x32x16) */
double ia_db_rot_eps_a2(void);
size_t ia_db_rot_bytes(long nrows);
size_t ia_db_cov_bytes(void);
int ia_db_cov(const IaSrcLevel *src, long row0, long nrows, const double *center, double *cov,
              void *stream);
int ia_db_build_rot(const IaSrcLevel *src, long row0, long nrows, const double *center,
                    const float *rot, float *amax, void *dbr, void *stream);

/* ---- 3-channel matching (config.py:29-42 num_ch = 3: convert=False on colour images) ----
 * Images are h x w x 3 fp64, channel-interleaved; IaSrcLevel / IaSynthArgs keep their
 * meaning with every image pointer 3-channel.  Feature rows have 165 values (the reference's
 * extract_patches_2d windows flattened (row, col, channel)); distances follow numpy's
 * pairwise summation for n = 165.
 * ia_db3_build: the materialised fp64 rows [A full | A'_i half] (168 doubles per row,
 *   ia_db3_bytes) of rows [row0, row0 + nrows).
 * ia_level_features3_f64: compute_feature_array (algorithms.py:11-47) of one level pair,
 *   h*w x 102 (full) or x 63 (half).
 * ia_synth_level3: one level on one GPU with the exact matcher (the split-f16 MFMA screen
 *   k_screen3 and an exact fp64 rescore of its candidate tiles in the oracle's order;
 *   IA_COLOR16=0: exhaustive fp64 search of the materialised rows), the coherence / kappa
 *   tail and the 3-channel B' update; a->db = ia_db3_build output over all rows; workspace
 *   of ia_synth3_workspace_bytes.
 * ia_synth_levels3: n consecutive 3-channel levels at once, pipelined as ia_synth_levels
 *   (one stream per level, wave t of level j behind the waves of level j-1 its coarse
 *   windows read); the same results as n ia_synth_level3 calls in order. */
size_t ia_db3_bytes(long nrows);
int ia_db3_build(const IaSrcLevel *src, long row0, long nrows, double *db3, void *stream);
int ia_level_features3_f64(const double *sm, int hs, int ws, const double *lg, int h, int w,
                           int full, double *out, void *stream);
size_t ia_synth3_workspace_bytes(int H, int W, long nrows);
/* the per-pixel API for 165-dim rows: exact 1-NN of M queries (M x 165) over the
 * materialised rows (workspace of ia_match3_workspace_bytes), the coherence argmin over n
 * <= 64 candidate rows (n x 165) and weighted distances (n pairs of 165-dim rows) */
size_t ia_match3_workspace_bytes(int M, long nrows);
int ia_match3_batch(const double *db3, long nrows, const double *q165, int M, int64_t *idx,
                    double *dist, void *workspace, void *stream);
int ia_coherence_pick3(const double *rows, int n, const double *q, int32_t *out, void *stream);
int ia_wdist3_batch(const double *a, const double *q, const double *w, int n, double *out,
                    void *stream);

/* ---- a12-a15: image_analogies.py:130-220 — synthesize one pyramid level on device,
 * skewed wavefront t = x + 3y (exactly the scanline semantics).
 * B_sm/B_lg: B at levels l-1 (B_hs x B_ws) and l (H x W); Bp_sm: B' level l-1;
 * Bp_lg: B' level l (in: init, out: result); s: H*W*2 int32 (row, col) in A';
 * im: H*W int32 A' image number.  weights: 55 fp64 (config.py:68-79);
 * kappa_factor = 1 + 2**(level - max_levels) * k.
 * comm: NULL (single GPU) or an ia_comm_init() communicator — the DB rows are then
 * sharded (row0/nrows of this rank, N_total overall) and each wave exchanges the per-rank
 * (dist, idx, weighted dist) winners with one RCCL all-gather (exact matcher only). */
typedef struct {
    IaSrcLevel src;
    const void *db; long row0, nrows, N_total;
    const double *center; const float *amax;
    const double *B_sm, *B_lg; int B_hs, B_ws, H, W;
    const double *Bp_sm; double *Bp_lg;
    const double *weights; double kappa_factor;
    int32_t *s, *im;
    void *workspace;
    void *comm;
    const IaLsh *lsh;   /* NULL: exact matcher; else LSH tables of this shard's rows */
    /* IA_SYNTH_EAGER: never capture the wave loop into a HIP graph.  Capture is off by
     * default (a graph's instantiation costs more than it saves on every c4 level); the
     * environment variable IA_GRAPH=1 captures levels of <= 2^18 rows on one GPU, =2 every
     * single-GPU level.
     * IA_SYNTH_PROF: while a profile is open (ia_prof_begin), record HIP events around every
     * screen launch and the matcher statistics under `tag` (no synchronisation; read back
     * by ia_prof_end).  Launches inside a captured graph are not timed. */
    int flags;
    int tag;
    /* optional debug outputs (image_analogies.py:141-159, 222-253; both or neither):
     * dbg_px: H*W x 7 int32 {p_app row, col, p_coh row, col, r* row, col, has coherence
     * candidate}; dbg_dist: H*W x 2 fp64 {d_app, d_coh} (zeros without a candidate) */
    int32_t *dbg_px;
    double *dbg_dist;
    const void *dbi;    /* NULL, or this shard's ia_db_build_image output (the matcher reads
                           it instead of the rows; db may then be NULL; same results) */
    /* NULL, or this shard's rotated database (ia_db_build_rot) and its rotation: on levels
     * where the fused per-wave kernel runs (one GPU or the device-side exchange) the screen
     * then streams it (4 MFMAs per tile instead of 11) and the exact stage
     * takes its bound; amax must then hold 2 floats {A, A_skip}.  Same results. */
    const void *dbr;
    const float *rot;
} IaSynthArgs;
/* the resources of ia_screen_resources / ia_fused_resources per level, from its IaSynthArgs as ia_synth_level would run it (the fused
 * kernel's form k_xstrip / k_xwave image / rows, or k_peer_finish without the fused kernel,
 * and the screen: k_screen16r where the level has the rotated DB, else the 4-wave split-f16
 * screen of its DB form): out = {waiting kernel LDS bytes, VGPRs, screen LDS bytes, VGPRs} */
int ia_level_resources(const IaSynthArgs *a, int *out);
#define IA_SYNTH_EAGER 1
#define IA_SYNTH_PROF 2
size_t ia_synth_workspace_bytes(int H, int W, long nrows, int nranks);
int ia_synth_level(const IaSynthArgs *a, void *stream);
int ia_synth_level3(const IaSynthArgs *a, void *stream);
/* after ia_synth_level3 / ia_synth_levels3 of these levels: synchronises the stream and returns
 * IA_E_SCHED if a wait for a neighbouring pixel's decision timed out in the fused colour tail */
int ia_synth3_status(const IaSynthArgs *levels, int n, void *stream);
int ia_synth_levels3(const IaSynthArgs *levels, int n, void *stream);
/* the rotated split screen for 3-channel rows (R16c): after ia_db3_build, the
 * caller takes the principal directions V of the level's centred rows (165 x 165, columns by
 * decreasing variance; any V orthonormal to fp64 precision keeps the matcher exact: checked,
 * ||V_f^T V_f - I||_F <= 2 sqrt(165) 2^-24 or IA_E_ARG) and passes them rounded to fp32
 * rot[k * 168 + j] = V[k][j] (ia_db3_rot_floats floats); ia_db3_build_rot writes the rotated
 * split tiles (352 B per row: ia_db3_rot_components components as f16 pairs, the rest as f16)
 * and A_skip into dbr (ia_db3_rot_bytes).  IaSynthArgs.dbr / .rot then select the R16c screen
 * in ia_synth_level3 / ia_synth_levels3 (11 MFMAs per 32 x 32 tile instead of 33). */
size_t ia_db3_rot_bytes(long nrows);
int ia_db3_rot_components(void);
int ia_db3_rot_floats(void);
int ia_db3_build_rot(const double *db3, long nrows, const float *rot, void *dbr, void *stream);
/* the matrix whose eigenvectors rot3_build takes: the 165 x 165 covariance (fp64, cov[a * 168
 * + b]) of ~64 k rows of an ia_db3_build buffer sampled every max(1, nrows / 65536) rows,
 * centred at their mean; cov holds ia_db3_cov_bytes() (the rest is scratch) */
size_t ia_db3_cov_bytes(void);
int ia_db3_cov(const double *db3, long nrows, double *cov, void *stream);
/* n consecutive levels (coarse to fine: levels[j].Bp_sm == levels[j-1].Bp_lg) at once, with
 * the same results as n ia_synth_level calls in order: each level runs on its own stream
 * and wave t of level j waits only for the waves of level j-1 its 3x3 coarse windows read
 * (coarse pixel (y/2 + 1, x/2 + 1) and before), so the levels overlap and the critical
 * path is about the finest level's waves.  Sharded levels need one communicator each. */
int ia_synth_levels(const IaSynthArgs *levels, int n, void *stream);
/* K independent jobs of identical shapes (the multi_script batch, multi_script.py:13-32;
 * SURVEY §8(e) config 5), n consecutive levels each: levels[j * K + k] is level j of job k,
 * every job with its own inputs, DB, workspace and outputs.  Each wave of each level is ONE
 * screen launch and ONE fused-kernel launch for all K jobs (grid y = job), so K jobs cost
 * about one job's launch latency; results equal K separate ia_synth_levels calls.  Exact
 * matcher on one GPU only (comm and lsh NULL), 1 <= K <= 128. */
int ia_synth_levels_batch(const IaSynthArgs *levels, int n, int K, void *stream);
/* after ia_synth_level(s) calls on `stream`: synchronises the stream and returns IA_E_SCHED if
 * a wait for a neighbouring pixel's decision inside the fused per-wave kernel timed out, or
 * IA_E_TIMEOUT if another rank's records on a device-side exchange never came: the results
 * are then wrong.  The reference has no such wait (image_analogies.py:161-220 is one
 * thread); this is the device schedule's own integrity check. */
int ia_synth_status(const IaSynthArgs *levels, int n, void *stream);
/* the same check for every fused level run on this device since the last clear (the level
 * workspaces may be gone): synchronises the device; IA_E_SCHED if any neighbour wait timed
 * out.  clear != 0 resets the sticky word.  Peer timeouts: ia_peer_status. */
int ia_sched_status(int clear);

/* profiling of ia_synth_level calls flagged IA_SYNTH_PROF (process-wide, thread-safe):
 * ia_prof_begin opens a profile (the caller has synchronised); ia_prof_end synchronises the
 * device and writes IA_PROF_FIELDS doubles per recorded level call, in call order:
 * {tag, DB rows, (query, row) pairs, screen ms over the timed launches, #timed screen
 * launches, #rows rescored in fp64, #candidate segments, #full scans, microseconds waited
 * for other ranks' records summed over the level's pixels (device-side exchange), the same
 * for the upper neighbour's decision (fused per-wave kernel), jobs per launch (a batch:
 * ia_synth_levels_batch; the pairs count all of them)}; returns the number of records
 * (<0: error). */
#define IA_PROF_FIELDS 11
int ia_prof_begin(void);
/* create the event pool up front (2 events per wave of every profiled level call of the
 * profile), so that no event is created inside a timed region */
int ia_prof_prepare(long nevents);
int ia_prof_end(double *out, int maxrec);
/* after ia_prof_end: record rec's screen launches one by one (ms from the HIP events, M
 * the launch's query count); returns the number of timed launches */
int ia_prof_launches(int rec, float *ms, int *M, int max);
/* the same record's per-wave spacing from a third event after each wave's exact stage:
 * tail_ms[i] = end of screen i -> end of its exact-stage / fused kernel, gap_ms[i] = that
 * -> the start of screen i + 1 on the level's stream (0 for the last wave) */
int ia_prof_waves(int rec, float *tail_ms, float *gap_ms, int max);
/* destroy the calling host thread's graph-capture stream and last executable graph */
int ia_release_thread_resources(void);

/* ---- multi-GPU: RCCL communicator over xGMI, one process per GPU. */
int ia_comm_unique_id(uint8_t out[128]);
int ia_comm_init(const uint8_t uid[128], int nranks, int rank, void **comm);
int ia_comm_destroy(void *comm);
int ia_comm_nranks(void *comm);
/* The device-side form of the same per-wave exchange (no RCCL call per wave): each rank
 * owns a receive box (2 x nranks x mcap x 24 B of uncached device memory; mcap >= the most
 * queries of any wave of the levels it serves), shared by IPC handle.  Per wave the exact
 * stage's kernel writes its shard's (distance, row) winner into every rank's box, and a
 * small finish kernel reads all ranks' winners from its own and finishes the pixel
 * (DESIGN.md §7).  Usable wherever a
 * communicator is (IaSynthArgs.comm, one per concurrently sharded level); destroyed by
 * ia_comm_destroy.  Protocol: ia_peer_create on every rank -> exchange the 64-byte handles
 * (rank order) -> ia_peer_connect -> a barrier -> ia_peer_check (a handshake wave; every
 * rank at once).  ia_peer_status: IA_E_COMM if any wait of this rank timed out (10 s).
 * ia_peer_mem_kind: 0 uncached, 1 fine-grained, 2 plain device memory. */
int ia_peer_create(int nranks, int rank, int mcap, void **comm, uint8_t handle[64]);
int ia_peer_connect(void *comm, const uint8_t *handles);
int ia_peer_check(void *comm, void *stream);
int ia_peer_status(void *comm);
int ia_peer_mem_kind(void *comm);

#ifdef __cplusplus
}
#endif
#endif /* IA_H */
