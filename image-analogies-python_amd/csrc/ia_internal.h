// ia_internal.h — declarations shared between libia.so translation units.
#pragma once
#include "ia_common.h"

namespace ia {

// ---- database chunking (shared by ia_db_build and the screen) -------------------
// A screen workgroup owns one chunk of CH rows: 4 waves x (CH/4) rows, 32-row tiles.
// CH is chosen so a DB produces ~target_chunks(N) chunks (512 by default).
constexpr int SCREEN_K = 4;            // candidates kept per (query, chunk)
// ~chunks per database: IA_TARGET_CHUNKS (read once per process; default 512; a tuning knob for tools/screen_bench — the DB build and the screen must agree on it)
int target_chunks(long nrows);

// tiles per wave: a power of two in [1, 64] (so screen segments divide it)
static inline int db_chunk_rows(long nrows) {
    const long tc = target_chunks(nrows);
    const long want = (nrows + tc * 128 - 1) / (tc * 128);
    long tpw = 1;
    while (tpw < want && tpw < 64) tpw <<= 1;
    return (int)(128 * tpw);
}
static inline long db_nchunks(long nrows) {
    const long ch = db_chunk_rows(nrows);
    return (nrows + ch - 1) / ch;
}
static inline long db_rows_padded(long nrows) { return db_nchunks(nrows) * db_chunk_rows(nrows); }
// one DB buffer = the fp32 screening rows (npad x IA_DP floats, fragment-major) followed
// by their split-f16 copy (npad x 112 halves, ia_split16.h): 2 x 224 B per padded row
static inline size_t db_bytes(long nrows) { return (size_t)db_rows_padded(nrows) * IA_DP * 4 * 2; }
template <typename T>
static inline T *db16_of(T *db, long nrows) {
    return db + (size_t)db_rows_padded(nrows) * IA_DP * 4 / sizeof(T);
}
// segment-minimum matcher: one running minimum per (query, segment) of <= seg_rows_max()
// rows (IA_SEG_MAX, read once per process: 512 [default] or 256)
int seg_rows_max();
static inline int db_seg_rows(long nrows) {
    const int rpw = db_chunk_rows(nrows) / 4, cap = seg_rows_max();
    return rpw < cap ? rpw : cap;
}
static inline long db_nsegs(long nrows) { return db_rows_padded(nrows) / db_seg_rows(nrows); }

struct Cand {            // one screen candidate: fp32 screen value + local row
    float e;
    int idx;
};
struct Best {            // exact winner of a (query, shard): fp64 distance + global row
    double d;
    long long idx;
};
struct WItem {           // one (query, candidate segment) of the work-list exact stage
    int q, seg;
    double trow;         // the query's fp32 re-screen threshold
};
struct QSel {            // per-query record of k_select: re-screen threshold, items
    double trow;
    int base, count;
};

// query-group split of M queries (32-query tiles, NQ tiles per group)
struct QSplit {
    int nq, groups, rows_pad;
};
// T = ceil(M/32) query tiles in groups of nq <= maxnq tiles: fewest padded tiles, then
// the largest nq (fewest re-reads of the database).
static inline QSplit qsplit(int M, int maxnq) {
    const int T = (M + 31) / 32;
    QSplit s;
    if (T <= maxnq) {
        s.nq = T; s.groups = 1;
    } else {
        int bestnq = maxnq, bestpad = 1 << 30;
        for (int nq = maxnq; nq >= 2; --nq) {
            int pad = (T + nq - 1) / nq * nq;
            if (pad < bestpad) { bestpad = pad; bestnq = nq; }
        }
        s.nq = bestnq; s.groups = (T + bestnq - 1) / bestnq;
    }
    s.rows_pad = s.nq * s.groups * 32;
    return s;
}
constexpr int MAX_NQ = 6;
// query rows allocated for Mmax queries: the screens read up to 2 * MAX_NQ padding tiles
static inline int qrows_alloc(int Mmax) { return ((Mmax + 31) / 32 + 2 * MAX_NQ) * 32; }

// the level state one wave of the per-pixel tail updates (ia_finish.h)
struct FinishArgs {
    int t, y_lo, W;
    long N_total;
    const double *weights;
    double kappa_factor;
    double *Bp_lg;
    int32_t *s, *im;
};

// matcher statistics (profiling only): per-query counters are spread over STATS_SLOTS
// cache lines so that the atomics of a wave's M queries do not serialise on one address;
// the host sums the slots.
constexpr int STATS_SLOTS = 64, STATS_LINE = 8;
constexpr size_t STATS_BYTES = (size_t)STATS_SLOTS * STATS_LINE * sizeof(unsigned long long);
__device__ __forceinline__ unsigned long long *stats_slot(unsigned long long *s, int q) {
    return s + (q & (STATS_SLOTS - 1)) * STATS_LINE;
}

// ---- launchers ------------------------------------------------------------------
// q16 (nullable): the split-f16 query rows (Q16_ROW half8 each, ia_split16.h)
int launch_query_wave(const ImgPair &B, const ImgPair &Bp, int t, int y_lo, int M,
                      const double *center, double *q64, float *qp, double *nq,
                      const float *amax, _Float16 *q16, hipStream_t st);
int launch_query_rows(const double *qin, int M, const double *center, float *qp, double *nq,
                      const float *amax, _Float16 *q16, hipStream_t st);
// screen of M queries (qp) against nrows DB rows -> cand[M][nchunks][SCREEN_K]
// variant 0: queries in VGPRs (<= 3 tiles/wave); 1: queries in LDS (<= 6 tiles/wave)
int launch_screen(const float *db, long nrows, const float *qp, int M, Cand *cand,
                  hipStream_t st);
int launch_screen_v(const float *db, long nrows, const float *qp, int M, Cand *cand,
                    int variant, hipStream_t st);
// exact rescore of the screen's candidates -> best[M]; stats[0..2] += (#cand, #overflow
// chunks, #full scans) when stats != nullptr
int launch_merge(const DbSrc &src, long row0, long nrows, const Cand *cand, int M,
                 const double *q64, const double *nq, const float *amax, Best *best,
                 unsigned long long *stats, hipStream_t st);
// the whole exact matcher (screen + exact stage) with the selected algorithm
// (IA_MATCH_ALG: 1 segment minima [default], 0 per-lane top-K); scratch of
// match_scratch_bytes(qrows_alloc(M), nrows).  stats (segment alg): rows rescored,
// candidate segments, full scans.
size_t match_scratch_bytes(int qrows, long nrows);
// ev0 / ev1 (nullable) are recorded on st immediately before / after the screen launch.
// fin (nullable, single shard only): the exact stage also runs the per-pixel tail of the
// wave (coherence, kappa, B'/s/im update) in the same kernel.
int launch_match(const DbSrc &src, long row0, long nrows, const float *db, const float *qp,
                 const _Float16 *q16, int M, const double *q64, const double *nq,
                 const float *amax, void *scratch, Best *best, unsigned long long *stats,
                 hipStream_t st,
                 hipEvent_t ev0 = nullptr, hipEvent_t ev1 = nullptr,
                 const FinishArgs *fin = nullptr);
int fuse_finish();    // IA_FUSE_FINISH: 0 off, 1 levels <= 2^20 rows, 2 on [default]
int match_alg();      // IA_MATCH_ALG (default 2: segment minima, split-f16 screen)
// q16 != nullptr: the split-f16 screen (k_screen_h16) over db16_of(db)
int launch_screen_seg(const float *db, long nrows, const float *qp, int M, float *segmin,
                      int maxnq, hipStream_t st, const _Float16 *q16 = nullptr);
int screen_variant();
// split-f16 segment screen (ia_screen16.hip) over db16_of(db): flags bits 0-3 cap on
// query tiles per wave (0 = shape rule), bit 8 per-wave kernel (no LDS sharing), bit 9 no
// pipelined epilogue, bit 10 fragment-prefetch form, bit 11 keep the epilogue at
// NQ = 3, bit 12 spanning form (bits 13 / 15: its no-copy diagnostics), bit 14 uneven
// query shares, bit 16 double-buffered fragment registers,
// bit 17 non-temporal DB stream, bit 18 balanced query shares, bit 19
// chain-balanced stages (9..11 query tiles)
int launch_screen16(const float *db, long nrows, const _Float16 *q16, int M, float *segmin,
                    int flags, hipStream_t st);
// approximate matcher (ia_lsh.hip): best[M] from the LSH buckets of each query
int launch_lsh_match(const IaLsh *lsh, const DbSrc &src, long row0, long nrows, int M,
                     const double *q64, const double *center, Best *best,
                     unsigned long long *stats, hipStream_t st);

}  // namespace ia
