// ia_internal.h — declarations shared between libia.so translation units.
#pragma once
#include "ia_common.h"

#include <atomic>

namespace ia {

// ---- the rotations' precondition ----------------------------------------------
// The R16 / R16c bounds charge the fp32 rotation's non-orthogonality as
// 2 ||V_f V_f^T - I|| A|q'| <= 2 (2 sqrt(n) u) A|q'| (u = 2^-24): true for the fp32 rounding of a
// basis orthonormal to fp64 precision, not for any matrix.  The public builders check it: the
// n x n rotation rot[k * ld + j] (device memory, ordered on st) read back once per level, and
// ||V_f^T V_f - I||_F (>= the spectral norm, which equals ||V_f V_f^T - I||'s) <= 2 sqrt(n) u.
int rot_check_orthonormal(const float *rot, int n, int ld, hipStream_t st, const char *who);

// ---- database chunking (shared by ia_db_build, the screen and the exact stage) ------
// A screen workgroup owns one chunk of ch rows (32-row tiles, 4-tile stages).  ch is
// chosen so a DB produces ~DB_TARGET_CHUNKS chunks (one per screen slot at 2 blocks per
// CU: measured 4-10 % faster than 1024 at 0.5-1 M rows, equal at 4.19 M rows;
// profiles/r01_screen_bench_shard_sizes.txt, r01_chunks_ab_end.txt).  The chunk count is
// rounded up to a multiple of 4 (the exact stage reads the segment minima as float4).
#ifndef IA_DB_TARGET_CHUNKS
#define IA_DB_TARGET_CHUNKS 512
#endif
constexpr long DB_TARGET_CHUNKS = IA_DB_TARGET_CHUNKS;
// the chunk target in force (ia_set_chunk_target): a batch of K DBs screened in one launch
// asks for fewer, longer chunks per DB (the workgroups of K DBs fill the GPU anyway).
// Per host thread: a batch's target never reaches another thread's DB builds and syntheses
// (every DB is built, sized and synthesised by one thread; one host thread per GPU stream)
extern thread_local long g_db_chunk_target;
constexpr int DB_CHUNK_MAX = 8192;     // 64 tiles
constexpr int DB_SEG_MAX = 512;        // rows per segment (one minimum per query)

static inline int db_chunk_rows(long nrows) {
    const long target = g_db_chunk_target;
    const long want = (nrows + target * 128 - 1) / (target * 128);
    long tpw = 1;   // 128-row units, a power of two in [1, 64]
    while (tpw < want && tpw < DB_CHUNK_MAX / 128) tpw <<= 1;
    return (int)(128 * tpw);
}
static inline long db_nchunks(long nrows) {
    const long ch = db_chunk_rows(nrows);
    return ((nrows + ch - 1) / ch + 3) / 4 * 4;
}
static inline long db_rows_padded(long nrows) { return db_nchunks(nrows) * db_chunk_rows(nrows); }
// the DB buffer: npad split-f16 rows (112 halves = 224 B each, ia_split16.h), the screen's
// MFMA operand and the exact stage's re-screen input
static inline size_t db_bytes(long nrows) { return (size_t)db_rows_padded(nrows) * 224; }
// segment-minimum matcher: one running minimum per (query, segment) of min(ch, 512) rows
// (a whole number of 4-tile stages; <= 16 segments per chunk)
static inline int db_seg_rows(long nrows) {
    const int ch = db_chunk_rows(nrows);
    return ch < DB_SEG_MAX ? ch : DB_SEG_MAX;
}
static inline long db_nsegs(long nrows) { return db_rows_padded(nrows) / db_seg_rows(nrows); }

// ---- the matcher's order of a DB's rows: chunks, stages, segments -------
// A screen workgroup owns a chunk of ch rows and walks it in 128-row stages; a segment (one
// minimum per query) is seg_rows / 128 consecutive stages of one chunk.  Two orders:
//   linear  chunk c = rows [c ch, (c + 1) ch), stage s = its rows 128 s ...;
//   strips  (a level whose shard is whole scanlines of width W % 128 == 0, with every chunk's
//           ch / 128 scanlines inside one A' image): chunk c is the 128-pixel column strip
//           c % (W / 128) of ch / 128 consecutive scanlines, stage s its scanline s.  The
//           image-form screen then walks down the strip and reloads one window row per
//           stage instead of the whole window (IA_DB_STRIPS, default 1).
// Every kernel that maps a segment or a stage back to rows uses stage_lrow.
struct StageMap {
    int W;        // 0: linear; else the level width (strips)
    int nstrip;   // W / 128
    int sc;       // stages per chunk (ch / 128)
};
// (chunks, stages and segments come in powers of two; row indices of a level's shard stay
// below 2^31 wherever these run: 32-bit arithmetic, shifts instead of 64-bit divisions)
__host__ __device__ __forceinline__ long stage_lrow(const StageMap &m, long chunk, int s) {
    if (m.W == 0) return (chunk * m.sc + s) * 128L;
    const unsigned c = (unsigned)chunk, yb = c / (unsigned)m.nstrip, sx = c - yb * (unsigned)m.nstrip;
    return ((long)yb * m.sc + s) * (long)m.W + (long)sx * 128;
}
// local row of element k (0 <= k < seg_rows) of segment seg
__host__ __device__ __forceinline__ long seg_lrow(const StageMap &m, long seg, int seg_rows, long k) {
    const int lspc = __builtin_ctz((unsigned)(m.sc * 128 / seg_rows));   // log2 segments per chunk
    const long chunk = seg >> lspc;
    const int s = (int)(seg - (chunk << lspc)) * (seg_rows >> 7) + (int)(k >> 7);
    return stage_lrow(m, chunk, s) + (k & 127);
}
// the segment holding local row lrow (the inverse of seg_lrow; stages are 128 aligned rows, so
// every 64-aligned run of 64 rows lies in one segment)
__host__ __device__ __forceinline__ long seg_of_lrow(const StageMap &m, long lrow, int seg_rows) {
    const int lspc = __builtin_ctz((unsigned)(m.sc * 128 / seg_rows));
    const int lsst = __builtin_ctz((unsigned)(seg_rows >> 7));   // log2 stages per segment
    if (m.W == 0) return lrow / seg_rows;
    const long y = lrow / m.W;
    const int x = (int)(lrow - y * m.W);
    const long yb = y / m.sc;
    const int s = (int)(y - yb * m.sc);
    const long chunk = yb * m.nstrip + (x >> 7);
    return (chunk << lspc) + (s >> lsst);
}
static inline bool db_strips_enabled() {
    static const int v = env_int("IA_DB_STRIPS", 1);
    return v != 0;
}

// ---- the image form of a level's DB (ia_db_build_image) ---------------
// A row's 55 features are pixels of its neighbourhood, so the screen can stage 128-row
// stages (128 pixels of one scanline) from the images instead of from 224-B rows: every
// pixel's split-f16 pair (hi | lo << 16) stored once, the images padded by reflection
// (IMG_PX columns, IMG_PY rows on each side) so every window row is one contiguous run.
// Buffer: [A fine][A coarse][norm slots of the rows][for each A' image: fine, coarse][scratch
// of the build], each section 256-B aligned.  Applies when the level width and row0 are multiples of 128 and
// the rows fill whole chunks (no padding rows): see img_db_applies.
constexpr int IMG_PX = 4, IMG_PY = 2;
struct ImgDb {
    gptr<const uint32_t> fa, ca, norm, ap;   // ap: A' image 0's fine section
    int W, Wp, Wcp;                         // width, padded fine / coarse widths
    long fsz, csz, apstride, apc;           // padded image sizes (u32), A' image stride,
                                            // offset of an A' image's coarse section
    long hw, row0;                          // rows per image, global row of local row 0
    long scr;                               // byte offset of the build's scratch section
};
constexpr size_t IMG_SCRATCH = 1024 * 8 * sizeof(double);   // ia_db_build_image's amax partials
static inline bool img_db_applies(int W, long row0, long nrows) {
    return W % 128 == 0 && row0 % 128 == 0 && db_rows_padded(nrows) == nrows &&
           row0 + nrows < (1L << 31);   // win_src's 32-bit row arithmetic
}
static inline size_t img_align(size_t b) { return (b + 255) / 256 * 256; }
// the image-form buffer of rows [row0, row0 + nrows) of a level with fine images H x W and
// coarse images hs x ws: its bytes (nAp A' images) and, with dbi, the section pointers.
// False when the image form does not apply.
static inline bool img_db_layout(int H, int W, int hs, int ws, int nAp, long row0, long nrows,
                                 const void *dbi, ImgDb &v, size_t *bytes) {
    if (!img_db_applies(W, row0, nrows)) return false;
    v.W = W; v.Wp = W + 2 * IMG_PX; v.Wcp = ws + 2 * IMG_PX;
    v.fsz = (long)(H + 2 * IMG_PY) * v.Wp;
    v.csz = (long)(hs + 2 * IMG_PY) * v.Wcp;
    v.hw = (long)H * W;
    v.row0 = row0;
    const size_t fb = img_align(v.fsz * 4), cb = img_align(v.csz * 4), nb = img_align(nrows * 4);
    v.apstride = (long)((fb + cb) / 4);
    v.apc = (long)(fb / 4);
    v.scr = (long)(fb + cb + nb + (size_t)nAp * (fb + cb));
    if (bytes) *bytes = (size_t)v.scr + IMG_SCRATCH;
    const char *p = reinterpret_cast<const char *>(dbi);
    v.fa = reinterpret_cast<const uint32_t *>(p);
    v.ca = reinterpret_cast<const uint32_t *>(p + fb);
    v.norm = reinterpret_cast<const uint32_t *>(p + fb + cb);
    v.ap = reinterpret_cast<const uint32_t *>(p + fb + cb + nb);
    return true;
}

// the stage order of rows [row0, row0 + nrows) of a level W wide with Himg scanlines per
// A' image: strips where they apply (and are enabled), else linear
static inline StageMap db_stage_map(long row0, long nrows, int W, int Himg) {
    const int ch = db_chunk_rows(nrows);
    StageMap m{0, 1, ch / 128};
    if (!db_strips_enabled() || W <= 0 || W % 128 != 0 || row0 % W != 0 || nrows % W != 0 ||
        db_rows_padded(nrows) != nrows)
        return m;
    const long lines = nrows / W, sc = ch / 128;
    if (lines % sc != 0 || (row0 / W) % sc != 0 || Himg % sc != 0) return m;
    m.W = W;
    m.nstrip = W / 128;
    return m;
}

struct Best {            // exact winner of a (query, shard): fp64 distance + global row
    double d;
    long long idx;
};
struct ShardRec {        // what a rank contributes per query to the cross-rank exchange
    double d;            // its shard's exact winner: distance, global row,
    long long idx;
    double wd;           // and that row's weighted (kappa) distance to the query
    double pad;
};
struct WItem {           // one (query, candidate segment) of the work-list exact stage
    int q, seg;
    float twoR;          // the re-screen's norm-slot factor 2^R
    double trow;         // the query's fp32 re-screen threshold (units of sa)
};
struct QSel {            // per-query record of k_select: re-screen threshold, items
    double trow;
    int base, count;
};

// query rows allocated for Mmax queries: the screen reads whole groups of query tiles
// (T = ceil(M/32) tiles in ceil(T/11) equal groups, so at most groups - 1 padding tiles)
static inline int qrows_alloc(int Mmax) {
    const int T = (Mmax + 31) / 32;
    return (T + (T + 10) / 11) * 32;
}

// Device-side exchange of a sharded level (ia_comm.hip, ia_finish.h): every rank owns a
// receive box in uncached device memory, IPC-mapped into every other rank's process.  Per
// wave each rank writes its (distance, row) winner of query q straight into every rank's
// box as three 8-byte granules {epoch << 32 | 32-bit payload} (the data carries its own
// flag, so a reader needs no fence), and reads the G ranks' granules of q from its own
// box until all carry the wave's epoch.  Two slots (epoch parity): a rank can be at most
// one wave ahead of a slower one's reads (its next record needs the slower rank's next
// record first).
constexpr int IA_PEER_MAX = 16;
struct PeerView {
    gptr<unsigned long long> box[IA_PEER_MAX];   // box[g]: rank g's receive box (box[rank]: own)
    gptr<unsigned int> err;                      // this rank's timeout word (0: fine)
    gptr<double> trace;                          // diagnostic (nullable): ia_diag_peer_trace
    int nranks, rank, mcap;                 // nranks 0: not a peer exchange
    unsigned int epoch;                     // this wave's tag (>= 1, one per wave)
};
// granules per (slot, source rank, query) cell: 3 for the (distance, row) records of
// k_rescore<3>, 7 for the fused per-wave kernel's {distance, row, weighted distance, A'
// value} (ia_xwave.hip); cells are 64 B
constexpr int PEER_CELL = 8;
static inline size_t peer_box_words(int nranks, int mcap) { return (size_t)2 * nranks * mcap * PEER_CELL; }

// the level state one wave of the per-pixel tail updates (ia_finish.h)
struct FinishArgs {
    int t, y_lo, W;
    long N_total;
    gptr<const double> weights;
    double kappa_factor;
    gptr<double> Bp_lg;
    gptr<int32_t> s, im;
    gptr<int32_t> dbg_px;     // nullable: 7 int32 per pixel (ia.h IaSynthArgs)
    gptr<double> dbg_dist;    // nullable: 2 doubles per pixel
    // sharded DB (nullable otherwise): the exact stage writes each query's ShardRec and
    // its coherence pick (CohSel, ia_finish.h) here instead of finishing the pixel
    gptr<ShardRec> shard_out;
    gptr<void> coh_out;
    // sharded DB with the device-side exchange (px.nranks > 0): the exact stage publishes
    // its shard's winner, collects every rank's, and finishes the pixel in the same kernel
    PeerView px{};
};

// one job of a batch of identical-shape jobs sharing each wave's launches (the multi_script
// workload, ia_synth_levels_batch): its own images, DB, query buffers (by wave parity),
// outputs and control words; the screen and k_xwave take job blockIdx.y's pointers from a
// device table of these
struct XJob {
    gptr<const double> A_sm, A_lg, Ap_sm, Ap_lg;   // DbSrc images
    gptr<const uint32_t> fa, ca, norm, ap;          // image-form DB sections (ImgDb)
    gptr<const void> db;                            // split-f16 rows
    gptr<float> segmin;
    gptr<double> q64[2];
    gptr<float> qp[2];
    gptr<double> nq[2];
    gptr<_Float16> q16[2];
    gptr<const float> amax;
    gptr<const double> center;
    gptr<const double> B_sm, B_lg, Bp_sm;
    gptr<double> Bp_lg;
    gptr<const double> weights;
    double kappa_factor;
    gptr<int32_t> s, im, dbg_px;
    gptr<double> dbg_dist;
    gptr<unsigned long long> dbox;
    gptr<unsigned int> ctl;                         // tickets[2], error word
    gptr<const void> dbr;                           // R16 rotated DB (nullable)
    gptr<const float> rot;                          // R16 rotation (nullable)
    gptr<const unsigned char> askc;                 // R16 per-segment skip codes (nullable)
};
constexpr int IA_BATCH_MAX = 128;

// one launch of the fused per-wave kernel k_xwave (ia_xwave.hip): wave t's exact stage,
// exchange (f.px) and per-pixel tail, and wave t + 1's query rows
struct XArgs {
    DbSrc src;
    ImgDb im;                     // image-form DB (IMG) ...
    gptr<const void> db;          // ... or the split-f16 rows (half8)
    long row0, nrows, nseg;
    int seg_rows;
    StageMap smap;                // segment -> rows
    gptr<const float> segmin;     // [M][nseg], this wave's screen
    gptr<const double> q64;       // this wave's query rows (M)
    gptr<const float> qp;
    gptr<const double> nq;
    gptr<const float> amax;
    gptr<const double> center;
    gptr<double> q64n;            // wave t + 1's query rows (M_n), written here
    gptr<float> qpn;
    gptr<double> nqn;
    gptr<_Float16> q16n;
    ImgPair B, Bp;                // B / B' at levels l - 1, l (the query's features)
    int H, M, y_lo_n, M_n;        // wave t: M pixels from f.y_lo; wave t + 1: M_n from y_lo_n
    gptr<unsigned long long> dbox;  // decision granules, 2 per row
    gptr<unsigned int> tickets;   // [2]: this launch uses tickets[t & 1]
    gptr<unsigned int> err;       // set when a wait for a neighbour's decision times out
    gptr<unsigned long long> stats;  // nullable: rows rescored, candidate segments, full scans
    FinishArgs f;                 // t, y_lo, W, ..., px (sharded DB: the device-side exchange)
    gptr<const XJob> jobs;        // nullable: a batch, job blockIdx.y's pointers override these
    gptr<unsigned long long> trace;  // diagnostic (nullable): phase stamps, XW_TRACE_* below
    gptr<const float> rot;        // R16 level (k_xstrip only, nullable): the rotation; q16n rows in
                                  // the R16 layout, q64 slot 55 = |kappa_skip|^2, amax[1] = A_skip
    gptr<const unsigned char> askc;  // R16 level: per-segment skip codes (r16_askc, ia_rot16.h)
};
// k_xwave phase stamps (IA_XW_TRACE=<level tag>, ia_diag_xwave_trace): s_memrealtime (100
// MHz) at XW_TRACE_N - 1 points of the pixels with ticket < XW_TRACE_PX of waves < XW_TRACE_T;
// slot XW_TRACE_N - 1 holds the pixel's candidate segment count (k_xstrip)
constexpr int XW_TRACE_N = 17, XW_TRACE_PX = 512, XW_TRACE_T = 4096;
// form: XW_ROWS (split-f16 rows), XW_IMG (image-form windows, fp32 re-screen), XW_STRIP
// (strip-order image form: k_xstrip, fp64 windows; xstrip_applies)
constexpr int XW_ROWS = 0, XW_IMG = 1, XW_STRIP = 2;
bool xstrip_applies(const DbSrc &src);
int launch_xwave(const XArgs &a, int nblocks, int form, hipStream_t st, int njobs = 1);

// matcher statistics (profiling only): per-query counters are spread over STATS_SLOTS
// cache lines so that the atomics of a wave's M queries do not serialise on one address;
// the host sums the slots.
constexpr int STATS_SLOTS = 64, STATS_LINE = 8;
constexpr size_t STATS_BYTES = (size_t)STATS_SLOTS * STATS_LINE * sizeof(unsigned long long);
__device__ __forceinline__ unsigned long long *stats_slot(unsigned long long *s, int q) {
    return s + (q & (STATS_SLOTS - 1)) * STATS_LINE;
}

// the exact matcher's scratch (match_scratch_bytes): a 256-B head (the work list's counter),
// then the segment minima [M][nseg]
constexpr size_t MATCH_HEAD = 256;
static inline float *match_segmin(void *scratch) {
    return reinterpret_cast<float *>(reinterpret_cast<char *>(scratch) + MATCH_HEAD);
}
// the exact stage's form for this process (ia_diag_set_rescore_mode): 0 per-query
// workgroups, 1 the work list, -1 default
int exact_stage_mode();

// ---- launchers ------------------------------------------------------------------
// query rows of wave t: q64 (fp64 features), qp (fp32 rows of the exact stage's
// re-screen), nq = |q - c|^2 and q16 (the split-f16 screen operand, Q16_ROW half8 each)
int launch_query_wave(const ImgPair &B, const ImgPair &Bp, int t, int y_lo, int M,
                      const double *center, double *q64, float *qp, double *nq,
                      const float *amax, _Float16 *q16, hipStream_t st, const float *rot = nullptr);
// the rotated split-f16 screen (R16, ia_screen16r.hip, ia_rot16.h) of M queries (q16 in the
// R16 layout) over a rotated DB (ia_db_build_rot) -> segmin[M][db_nsegs(nrows)], the same
// units as launch_screen16; jobs: a batch (each job's dbr, q16[parity], segmin)
int launch_screen16r(const void *dbr, long nrows, const StageMap &sm, const _Float16 *q16, int M,
                     float *segmin, hipStream_t st, const XJob *jobs = nullptr, int njobs = 1, int parity = 0);
// amax = max(amax, the split scale's bound of a level's four value ranges) (ia_features.hip);
// part: DBB_BLOCKS x 8 doubles of scratch
int launch_db_amax(const IaSrcLevel *src, const DbSrc &d, const double *center, float *amax,
                   double *part, hipStream_t st);
int launch_query_rows(const double *qin, int M, const double *center, float *qp, double *nq,
                      const float *amax, _Float16 *q16, hipStream_t st);
// the split-f16 segment screen (ia_screen16.hip) of M queries over the DB ->
// segmin[M][db_nsegs(nrows)] (screen units); q16 holds qrows_alloc(M) rows
// img (nullable): the DB's image form (ImgDb, whole chunks) streamed instead of the rows
// (same minima, bit for bit)
// jobs (nullable): a batch of njobs identical-shape jobs in one launch (grid y = job; each
// job's DB sections, q16[parity] and segmin from its table entry).  sharded: a level whose
// fused kernels wait for other ranks: never the producer / consumer screen there (its
// one-per-CU blocks need ~94 KB of a CU's LDS, which waiting workgroups can hold for as long
// as another rank needs: measured, 2 ranks sharing one GPU timed out on c4)
int launch_screen16(const void *db, const ImgDb *img, long nrows, const StageMap &sm,
                    const _Float16 *q16, int M, float *segmin, hipStream_t st,
                    const XJob *jobs = nullptr, int njobs = 1, int parity = 0, bool sharded = false);
// the whole exact matcher (screen + exact stage); scratch of match_scratch_bytes(M, nrows).
// stats (nullable): rows rescored, candidate segments, full scans.
size_t match_scratch_bytes(int qrows, long nrows);
// ev0 / ev1 (nullable) are recorded on st immediately before / after the screen launch.
// fin (nullable, single shard only): the exact stage also runs the per-pixel tail of the
// wave (coherence, kappa, B'/s/im update) in the same kernel.
// dbi (nullable): the DB's image form for the screen (ia_db_build_image)
int launch_match(const DbSrc &src, long row0, long nrows, const void *db, const void *dbi,
                 const float *qp, const _Float16 *q16, int M, const double *q64, const double *nq,
                 const float *amax, void *scratch, Best *best, unsigned long long *stats,
                 hipStream_t st,
                 hipEvent_t ev0 = nullptr, hipEvent_t ev1 = nullptr,
                 const FinishArgs *fin = nullptr);
// approximate matcher (ia_lsh.hip): best[M] from the LSH buckets of each query
int launch_lsh_match(const IaLsh *lsh, const DbSrc &src, long row0, long nrows, int M,
                     const double *q64, const double *center, Best *best,
                     unsigned long long *stats, hipStream_t st);

}  // namespace ia
