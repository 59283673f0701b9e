// ia_match.hip — the exact brute-force matcher (the hot path).
//
// best_approximate_match (algorithms.py:73-75, FLANN kd-tree in the reference) becomes an
// EXACT 1-NN over the level database As[level] in two stages:
//
//  1. the split-f16 MFMA screen (ia_screen16.hip): for every (query, 512-row segment) the
//     minimum of the screen value e(r) = |a'|^2 - 2 a'.q' (a' = a - c, q' = q - c, c the
//     screening centre), in units of sa * sq; no per-row state, branch free;
//  2. the exact stage (this file): e* = the minimum over all segments; every segment whose
//     minimum is within Tseg = e* + 2 eps16 is re-screened row by row in fp32 (VALU, from
//     the same split-f16 rows, x = x_h + x_l exactly in fp32), and every row within
//     Trow = e* + eps16 + eps_q is rescored in fp64
//     in the oracle's exact operation order (numpy pairwise-8, no FMA contraction),
//     gathering its 55 features from the fp64 pyramids; ties break to the lowest row
//     (np.argmin).  eps16 / eps_q bound the screen / re-screen error for ANY summation
//     order, so the oracle's winner is always rescored: the result is
//     bit-identical to the oracle's brute force for any input.
//
// Two forms of the exact stage: k_rescore (one workgroup per query; levels <= 2^20 rows)
// and the work list k_select -> k_items -> k_gather (larger levels, where a query with many
// candidate segments would serialise k_rescore).  On a single shard the last kernel also
// runs the per-pixel tail of the synthesis step (ia_finish.h).
#include "ia_exact.h"
#include "ia_finish.h"

#include <float.h>

namespace ia {

// (thresholds, re-screen and window helpers: ia_exact.h)

// The end of the exact stage for query q once its winner win (distance bd) is known, by
// the block's waves 0 and 1 (all threads call it; every wave reaches the barriers).
// MODE 0: best[q] only (written by the caller); 1 (one shard): wave 1 picks the coherence
// candidate while wave 0 weighs the winner, then wave 0 finishes the pixel (ia_finish.h),
// saving a launch and a round trip per wave; 2 (sharded DB): the same two picks, written
// out (ShardRec, CohSel) for k_finish after the cross-rank exchange.
// have_cs: the coherence pick is already in *cs (k_rescore's fifth wave): only the weight.
template <int MODE>
__device__ __forceinline__ void exact_tail(const DbSrc &src, int q, long long win, double bd,
                                           const FinishArgs &fa, const double *qs, CohSel *cs,
                                           bool have_cs = false) {
    if (MODE == 0) return;
    __syncthreads();
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    double d_app = 0.0;
    if (MODE == 3) {
        // device-side exchange: wave 0 hands this shard's winner to every rank's receive box
        // (ia_finish.h peer_publish); k_peer_finish (ia_synth.hip), the next launch,
        // collects every rank's and finishes the pixel.  Nothing here waits on another
        // rank, so this kernel's large workgroups never hold CUs while they wait.
        // (win / bd come from LDS words lane 0 of wave 0 wrote just before the call: only
        // that lane's copy is certain, and every publishing lane needs it)
        bd = __shfl(bd, 0);
        win = __shfl(win, 0);
        if (wv == 0) peer_publish(fa.px, q, bd, win, lane);
        return;
    }
    if (wv == 1 && !have_cs) {
        const CohSel c = coh_pick(src, q, fa, qs, lane);
        if (lane == 0) *cs = c;
    } else if (wv == 0) {
        d_app = app_wdist(src, win, fa, qs, lane);
    }
    if (MODE == 1) {
        if (!have_cs) __syncthreads();
        if (wv == 0) finish_apply(src, win, q, fa, *cs, d_app, lane);
    } else {
        if (!have_cs) __syncthreads();
        if (wv == 0 && lane == 0) {
            fa.shard_out[q] = ShardRec{bd, win, d_app, 0.0};
            reinterpret_cast<CohSel *>(fa.coh_out.get())[q] = *cs;
        }
    }
}

// The fifth wave (FIFTH, MODE 1-3): picks the coherence candidate during the row loop
// instead of in the tail.  k_rescore needs ~250 VGPRs (2 waves per SIMD, 8 per CU), so a
// 5-wave workgroup leaves room for one per CU (256 resident) and 4-wave ones for two
// (512).  A wave of more than 256 queries (c4's plateau: 342) runs 4-wave, in one round
// instead of two; smaller waves keep the fifth wave's overlap (profiles/r02_ab_fifth.txt).
// (Forcing 3 waves per SIMD spills ~110 VGPRs: r02_ab_rescore_occ.)
constexpr int RESCORE_FIFTH_MAX_M = 256;
constexpr int rescore_threads(int mode, bool fifth) { return mode != 0 && mode != 3 && fifth ? 320 : 256; }

// Exact stage, one workgroup per query: waves 0-3 screen and rescore, then the pixel tail
// (MODE 1-3: exact_tail; with IA_RESCORE_FIFTH a fifth wave picks the coherence candidate
// during the row loop, since it needs only s / im of earlier waves).
template <int MODE, bool IMG, bool FIFTH>
__global__ __launch_bounds__(rescore_threads(MODE, FIFTH), IMG ? 2 : 1) void k_rescore(
        DbSrc src, long row0, long nrows, long nseg, int seg_rows, StageMap sm,
        const float *__restrict__ segmin, const half8 *__restrict__ db, ImgDb im,
        const float *__restrict__ qp, const double *__restrict__ q64,
        const double *__restrict__ nq, const float *__restrict__ amax, Best *__restrict__ best,
        unsigned long long *stats, FinishArgs fa) {
    __shared__ int slist[RESCORE_SEGCAP];
    __shared__ long long win;
    __shared__ double wind;
    __shared__ CohSel cs;
    __shared__ int scount;
    __shared__ float redf[4];
    __shared__ double redd[4];
    __shared__ long long redi[4];
    __shared__ double qs[IA_DP];
    __shared__ float qf[IA_DP];
    __shared__ unsigned int nresc;
    __shared__ long rlist[RESCORE_ROWCAP];
    __shared__ int rcount;
    __shared__ __attribute__((aligned(16))) char wins[IMG ? 4 * WIN_B : 16];   // one window per wave

    const int q = blockIdx.x;
    const int tid = threadIdx.x;
    const bool ex = tid < 256;               // the exact stage's waves
    // every independent load in one round trip: the query rows, its norm, the DB bound and
    // the segment minima (the LDS stores of the query come after all of them are issued)
    double qsv = 0.0;
    float qfv = 0.f;
    if (tid < IA_DP) {
        qsv = q64[(long)q * IA_DP + tid];
        qfv = qp[(long)q * IA_DP + tid];
    }
    const double nqq = nq[vidx(q)];
    const float am = amax[vidx(0)];
    const long n4 = nseg / 4;
    const float4 *sq4 = reinterpret_cast<const float4 *>(segmin + (long)q * nseg);
    float4 v[RESCORE_REG];
    segmin_load(sq4, n4, v);
    if (tid == 0) { scount = 0; nresc = 0; rcount = 0; }
    const float emin = segmin_scan(sq4, n4, v, redf);
    if (tid < IA_DP) {                       // read after the selection's barrier
        qs[tid] = qsv;
        qf[tid] = qfv;
    }
    double Tseg, Trow;
    bool force_full;
    rescore_thresholds(emin, am, nqq, Tseg, Trow, force_full);
    const float twoR = ldexpf(1.f, split16_db_scale(am).R);
    segmin_select(sq4, n4, v, Tseg, slist, &scount);
    __syncthreads();
    const int ns = scount;
    const bool full = ns > RESCORE_SEGCAP || force_full;
    const long nscan = full ? nseg : ns;

    double bd = INFINITY;
    long long bi = 0x7fffffffffffffffLL;
    unsigned int mine = 0;
    // rows within Trow go to a list rescored one per thread after the re-screen (one round
    // of feature gathers); a list overflow is rescored in place
    const long nrs = ex ? nscan * seg_rows : 0;
    auto take = [&](long lr, float e) {     // lr: local row
        if (lr < nrows && (double)e <= Trow) {
            ++mine;
            const int pos = atomicAdd(&rcount, 1);
            if (pos < RESCORE_ROWCAP) rlist[pos] = lr;
            else best_update(bd, bi, row_dist2(src, row0 + lr, qs), row0 + lr);
        }
    };
    if constexpr (IMG) {
        // image form: wave w re-screens the 128-row stage k0 = base + 128 w of each 512-row
        // step from its own LDS window (no block barrier: the fifth wave is free meanwhile);
        // the next step's window loads fly while this one is re-screened
        const int wv = tid >> 6, lane = tid & 63;
        char *wb = wins + (wv & 3) * WIN_B;
        auto stage_row = [&](long k0) {
            const long seg = full ? k0 / seg_rows : slist[k0 / seg_rows];
            return seg_lrow(sm, seg, seg_rows, k0 % seg_rows);
        };
        piece_t pc[WIN_PPL];
        long k0 = 128L * wv, lrow = 0;
        if (k0 < nrs) {
            lrow = stage_row(k0);
            win_load(im, lrow, lane, pc);
        }
        for (; k0 < nrs; k0 += RESCORE_RPT * 256) {
            wave_lds_sync();                // the previous window's reads are done
            win_store(wb, lane, pc);
            wave_lds_sync();
            long lnext = 0;
            if (k0 + RESCORE_RPT * 256 < nrs) {
                lnext = stage_row(k0 + RESCORE_RPT * 256);
                win_load(im, lnext, lane, pc);
            }
            float e0, e1;
            rescreen_win2(wb, lane, qf, twoR, e0, e1);
            take(lrow + lane, e0);
            take(lrow + lane + 64, e1);
            lrow = lnext;
        }
    } else {
        // rows of the candidate segments, RESCORE_RPT per thread per step with all their DB
        // loads issued together (seg_rows <= 512 = RESCORE_RPT * 256: one step per segment)
        for (long base = 0; base < nrs; base += RESCORE_RPT * 256) {
            float e[RESCORE_RPT];
            long lr[RESCORE_RPT];
#pragma unroll
            for (int u = 0; u < RESCORE_RPT; ++u) {
                const long k = base + u * 256 + tid;
                const long seg = k < nrs ? (full ? k / seg_rows : slist[k / seg_rows]) : 0;
                lr[u] = k < nrs ? seg_lrow(sm, seg, seg_rows, k % seg_rows) : nrows;
                // out-of-range rows read row 0 and are discarded below
                half8 g0[DB16_GROUPS], g1[DB16_GROUPS];
                load_row16(db, lr[u] < nrows ? lr[u] : 0, g0, g1);
                e[u] = rescreen16(g0, g1, qf, twoR);
            }
#pragma unroll
            for (int u = 0; u < RESCORE_RPT; ++u) take(lr[u], e[u]);
        }
    }
    if (MODE != 0 && !ex) {                  // the fifth wave: coherence pick
        const CohSel c = coh_pick(src, q, fa, qs, tid & 63);
        if ((tid & 63) == 0) cs = c;
    }
    __syncthreads();
    if (ex) {
        const int nl = rcount < RESCORE_ROWCAP ? rcount : RESCORE_ROWCAP;
        for (int i = tid; i < nl; i += 256)
            best_update(bd, bi, row_dist2(src, row0 + rlist[i], qs), row0 + rlist[i]);
    }
    for (int o = 32; o > 0; o >>= 1) {
        const double od = __shfl_xor(bd, o);
        const long long oi = __shfl_xor(bi, o);
        best_update(bd, bi, od, oi);
    }
    if (mine) atomicAdd(&nresc, mine);
    if ((tid & 63) == 0 && ex) { redd[tid >> 6] = bd; redi[tid >> 6] = bi; }
    __syncthreads();
    if (tid == 0) {
        for (int w = 1; w < 4; ++w) best_update(bd, bi, redd[w], redi[w]);
        best[q] = Best{bd, bi};
        win = bi;
        wind = bd;
        if (stats) {
            unsigned long long *sl = stats_slot(stats, q);
            atomicAdd(&sl[0], (unsigned long long)nresc);
            atomicAdd(&sl[1], (unsigned long long)ns);
            atomicAdd(&sl[2], full ? 1ULL : 0ULL);
        }
    }
    exact_tail<MODE>(src, q, win, wind, fa, qs, &cs, FIFTH && MODE != 0 && MODE != 3);
}

// ---------------------------------------------------------------------------------
// Work-list exact stage: the same thresholds and the same rows as
// k_rescore, but the candidate segments of all queries become items of one list, so a
// query with many candidate segments spreads over many workgroups instead of serialising
// in one (k_rescore's time is that of its heaviest query).
//   k_select  one workgroup per query: e*, thresholds, candidate segments -> items
//   k_items   one workgroup per item (grid-stride): fp32 re-screen of the segment's rows,
//             exact rescore of those <= Trow -> the item's (distance, row) minimum
//   k_gather  one wave per query: the lexicographic minimum over its items [+ the
//             per-pixel tail]; also empties the list for the next call
// ---------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_select(long nseg, const float *__restrict__ segmin,
                                                const double *__restrict__ nq,
                                                const float *__restrict__ amax, int *ctr,
                                                WItem *__restrict__ items, QSel *__restrict__ sel,
                                                unsigned long long *stats) {
    __shared__ int slist[RESCORE_SEGCAP];
    __shared__ int scount, sbase;
    __shared__ float redf[4];
    const int q = blockIdx.x;
    const int tid = threadIdx.x;
    const double nqq = nq[vidx(q)];          // one round trip for all independent loads
    const float am = amax[vidx(0)];
    const long n4 = nseg / 4;
    const float4 *sq4 = reinterpret_cast<const float4 *>(segmin + (long)q * nseg);
    float4 v[RESCORE_REG];
    segmin_load(sq4, n4, v);
    if (tid == 0) scount = 0;
    const float emin = segmin_scan(sq4, n4, v, redf);
    double Tseg, Trow;
    bool force_full;
    rescore_thresholds(emin, am, nqq, Tseg, Trow, force_full);
    segmin_select(sq4, n4, v, Tseg, slist, &scount);
    __syncthreads();
    const int ns = scount;
    const bool full = ns > RESCORE_SEGCAP || force_full;
    const int cnt = full ? (int)nseg : ns;
    if (tid == 0) {
        sbase = atomicAdd(ctr, cnt);
        sel[q] = QSel{Trow, sbase, cnt};
        if (stats) {
            unsigned long long *sl = stats_slot(stats, q);
            atomicAdd(&sl[1], (unsigned long long)ns);
            atomicAdd(&sl[2], full ? 1ULL : 0ULL);
        }
    }
    __syncthreads();
    const int base = sbase;
    const float twoR = ldexpf(1.f, split16_db_scale(am).R);
    for (int i = tid; i < cnt; i += 256) items[base + i] = WItem{q, full ? i : slist[i], twoR, Trow};
}

template <bool IMG>
__global__ __launch_bounds__(256, IMG ? 2 : 1) void k_items(DbSrc src, long row0, long nrows, int seg_rows,
                                               StageMap sm,
                                               const WItem *__restrict__ items,
                                               const int *__restrict__ ctr,
                                               const half8 *__restrict__ db, ImgDb im,
                                               const float *__restrict__ qp,
                                               const double *__restrict__ q64,
                                               Best *__restrict__ ibest,
                                               unsigned long long *stats) {
    __shared__ double qs[IA_DP];
    __shared__ float qf[IA_DP];
    __shared__ double redd[4];
    __shared__ long long redi[4];
    __shared__ int plist[RESCORE_RPT * 256];
    __shared__ int pcount;
    __shared__ __attribute__((aligned(16))) char wins[IMG ? 4 * WIN_B : 16];   // one window per wave
    const int n = *ctr;
    const int tid = threadIdx.x;
    const int wv = tid >> 6, lane = tid & 63;
    for (int it = blockIdx.x; it < n; it += gridDim.x) {
        const WItem w = items[it];
        // this thread's rows of the segment (row form) or its wave's window (image form: wave
        // wv takes the segment's 128-row stage wv), issued before the query is staged so that
        // the two round trips overlap
        half8 x0[IMG ? 1 : RESCORE_RPT][DB16_GROUPS], x1[IMG ? 1 : RESCORE_RPT][DB16_GROUPS];
        long lr[RESCORE_RPT];
        piece_t pc[WIN_PPL];
        const bool wstage = IMG && wv * 128 < seg_rows;
        if constexpr (IMG) {
            if (wstage) win_load(im, seg_lrow(sm, w.seg, seg_rows, wv * 128), lane, pc);
        } else {
#pragma unroll
            for (int u = 0; u < RESCORE_RPT; ++u) {
                const int k = u * 256 + tid;
                lr[u] = k < seg_rows ? seg_lrow(sm, w.seg, seg_rows, k) : nrows;
                load_row16(db, lr[u] < nrows ? lr[u] : 0, x0[u], x1[u]);
            }
        }
        __syncthreads();                       // the previous item's LDS reads are done
        if (tid < IA_DP) {
            qs[tid] = q64[(long)w.q * IA_DP + tid];
            qf[tid] = qp[(long)w.q * IA_DP + tid];
        }
        if (tid == 0) pcount = 0;
        if (wstage) win_store(wins + wv * WIN_B, lane, pc);
        __syncthreads();
        // fp32 re-screen; rows within Trow go to one list, rescored one per thread below
        // (a single round of feature gathers, however the passing rows fall over lanes)
        if constexpr (IMG) {
            if (wstage) {
                float e0, e1;
                rescreen_win2(wins + wv * WIN_B, lane, qf, w.twoR, e0, e1);
                if ((double)e0 <= w.trow) plist[atomicAdd(&pcount, 1)] = wv * 128 + lane;
                if ((double)e1 <= w.trow) plist[atomicAdd(&pcount, 1)] = wv * 128 + lane + 64;
            }
        } else {
#pragma unroll
            for (int u = 0; u < RESCORE_RPT; ++u) {
                const float acc = rescreen16(x0[u], x1[u], qf, w.twoR);
                if (lr[u] < nrows && (double)acc <= w.trow) plist[atomicAdd(&pcount, 1)] = u * 256 + tid;
            }
        }
        __syncthreads();
        const int np = pcount;
        double bd = INFINITY;
        long long bi = 0x7fffffffffffffffLL;
        for (int i = tid; i < np; i += 256) {
            const long row = row0 + seg_lrow(sm, w.seg, seg_rows, plist[i]);
            best_update(bd, bi, row_dist2(src, row, qs), row);
        }
        for (int o = 32; o > 0; o >>= 1) {
            const double od = __shfl_xor(bd, o);
            const long long oi = __shfl_xor(bi, o);
            best_update(bd, bi, od, oi);
        }
        if ((tid & 63) == 0) { redd[tid >> 6] = bd; redi[tid >> 6] = bi; }
        __syncthreads();
        if (tid == 0) {
            for (int v = 1; v < 4; ++v) best_update(bd, bi, redd[v], redi[v]);
            ibest[it] = Best{bd, bi};
            if (stats) atomicAdd(&stats_slot(stats, w.q)[0], (unsigned long long)np);
        }
    }
}

// one wave per query reduces its items (lexicographic (distance, row) minimum); MODE as
// exact_tail (1, 2: a second wave picks the coherence candidate meanwhile)
template <int MODE>
__global__ __launch_bounds__(128) void k_gather(DbSrc src, const QSel *__restrict__ sel,
                                                const Best *__restrict__ ibest, int *ctr,
                                                Best *__restrict__ best, FinishArgs fa,
                                                const double *__restrict__ q64) {
    __shared__ double qs[IA_DP];
    __shared__ CohSel cs;
    __shared__ long long win;
    __shared__ double wind;
    const int m = blockIdx.x;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (MODE != 0 && threadIdx.x < IA_DP) qs[threadIdx.x] = q64[(long)m * IA_DP + threadIdx.x];
    double bd = INFINITY;
    long long bi = 0x7fffffffffffffffLL;
    if (wv == 0) {
        const QSel r = sel[m];
        for (int i = lane; i < r.count; i += 64) {
            const Best b = ibest[r.base + i];
            best_update(bd, bi, b.d, b.idx);
        }
        for (int o = 32; o > 0; o >>= 1) {
            const double od = __shfl_xor(bd, o);
            const long long oi = __shfl_xor(bi, o);
            best_update(bd, bi, od, oi);
        }
        if (m == 0 && lane == 0) *ctr = 0;   // every k_items block has read it
        if (lane == 0) {
            if (MODE == 0 || MODE == 3) best[m] = Best{bd, bi};
            win = bi;
            wind = bd;
        }
    }
    if (MODE != 0) {
        __syncthreads();
        exact_tail<MODE>(src, m, win, wind, fa, qs, &cs);
    }
}

// 0: per-query k_rescore, 1: work list, -1: default (see launch_match); settable through
// ia_diag_set_rescore_mode
static std::atomic<int> g_rescore_mode{env_int("IA_RESCORE", -1)};
static int rescore_mode() { return g_rescore_mode.load(std::memory_order_relaxed); }
int exact_stage_mode() { return rescore_mode(); }

// matcher scratch: [list counter | segment minima | items | item winners | per-query
// records]; the counter sits at a fixed offset (it carries over between calls, emptied by
// k_gather)
static constexpr size_t WL_HEAD = MATCH_HEAD;
struct SegWs {
    int *ctr;
    float *segmin;
    WItem *items;
    Best *ibest;
    QSel *sel;
};
static SegWs seg_ws(void *scratch, int M, long nrows) {
    char *p = reinterpret_cast<char *>(scratch);
    const size_t n = (size_t)M * db_nsegs(nrows);
    SegWs w;
    w.ctr = reinterpret_cast<int *>(p);
    w.segmin = reinterpret_cast<float *>(p + WL_HEAD);
    w.items = reinterpret_cast<WItem *>(p + WL_HEAD + align_up(n * sizeof(float), 256));
    w.ibest = reinterpret_cast<Best *>(reinterpret_cast<char *>(w.items) + align_up(n * sizeof(WItem), 256));
    w.sel = reinterpret_cast<QSel *>(reinterpret_cast<char *>(w.ibest) + align_up(n * sizeof(Best), 256));
    return w;
}
size_t match_scratch_bytes(int qrows, long nrows) {
    const size_t n = (size_t)qrows * db_nsegs(nrows);
    return WL_HEAD + align_up(n * sizeof(float), 256) + align_up(n * sizeof(WItem), 256) +
           align_up(n * sizeof(Best), 256) + align_up((size_t)qrows * sizeof(QSel), 256);
}

int launch_match(const DbSrc &src, long row0, long nrows, const void *dbv, const void *dbi,
                 const float *qp, const _Float16 *q16, int M, const double *q64, const double *nq,
                 const float *amax, void *scratch, Best *best, unsigned long long *stats,
                 hipStream_t st, hipEvent_t ev0, hipEvent_t ev1, const FinishArgs *fin) {
    int rc;
    IA_ARG(q16, "launch_match: no split-f16 query rows");
    const half8 *db = reinterpret_cast<const half8 *>(dbv);
    ImgDb img{};
    IA_ARG(!dbi || img_db_layout(src.A.h, src.A.w, src.A.hs, src.A.ws, 1, row0, nrows, dbi, img, nullptr),
           "launch_match: an image-form DB for a level it does not apply to");
    IA_ARG(db || dbi, "launch_match: no DB (row form or image form)");
    const SegWs ws = seg_ws(scratch, M, nrows);
    if (ev0) IA_HIP(hipEventRecord(ev0, st));
    const StageMap sm = db_stage_map(row0, nrows, src.A.w, src.A.h);
    // (the unfused matcher also serves sharded levels whose tails wait for other ranks: the
    // 4-wave screen here, never the one-block-per-CU producer / consumer form)
    if ((rc = launch_screen16(db, dbi ? &img : nullptr, nrows, sm, q16, M, ws.segmin, st, nullptr, 1, 0,
                              true)))
        return rc;
    if (ev1) IA_HIP(hipEventRecord(ev1, st));
    const FinishArgs fa = fin ? *fin : FinishArgs{};
    const int rm = rescore_mode();
    // the exact stage re-screens from the image form whenever there is one (the row form
    // need not exist then)
    const bool im = dbi != nullptr;
    // default: k_rescore (one workgroup per query, with or without the fused tail; a
    // sharded rank's 0.5 M-row shard: 13.9 vs 19.9 us per wave, profiles/r01_shard_sim_g8.txt),
    // except on row-form levels above 2^20 rows, where its per-query serialisation costs
    // most and the work list wins.  On the image form k_rescore wins at every size (c4's
    // 4.19 M-row finest level: 1637-1643 vs 1667-1669 ms/step, profiles/r02_ab_rescore.txt)
    const int mode = !fin ? 0 : fin->shard_out ? 2 : fin->px.nranks ? 3 : 1;
    if (rm == 1 || (rm < 0 && !im && nrows > (1L << 20))) {
        const long nseg = db_nsegs(nrows);
        k_select<<<M, 256, 0, st>>>(nseg, ws.segmin, nq, amax, ws.ctr, ws.items, ws.sel, stats);
        IA_LAUNCH_CHECK("k_select");
        const int grid = 2 * M + 64;
        if (im)
            k_items<true><<<grid, 256, 0, st>>>(src, row0, nrows, db_seg_rows(nrows), sm, ws.items, ws.ctr,
                                                db, img, qp, q64, ws.ibest, stats);
        else
            k_items<false><<<grid, 256, 0, st>>>(src, row0, nrows, db_seg_rows(nrows), sm, ws.items, ws.ctr,
                                                 db, img, qp, q64, ws.ibest, stats);
        IA_LAUNCH_CHECK("k_items");
        if (mode == 3)
            k_gather<3><<<M, 128, 0, st>>>(src, ws.sel, ws.ibest, ws.ctr, best, fa, q64);
        else if (mode == 2)
            k_gather<2><<<M, 128, 0, st>>>(src, ws.sel, ws.ibest, ws.ctr, best, fa, q64);
        else if (mode == 1)
            k_gather<1><<<M, 128, 0, st>>>(src, ws.sel, ws.ibest, ws.ctr, best, fa, q64);
        else
            k_gather<0><<<M, 64, 0, st>>>(src, ws.sel, ws.ibest, ws.ctr, best, fa, q64);
        IA_LAUNCH_CHECK("k_gather");
        return IA_OK;
    }
#define IA_RESCORE_LAUNCH(MD, IM, F)                                                            \
    k_rescore<MD, IM, F><<<M, rescore_threads(MD, F), 0, st>>>(src, row0, nrows, db_nsegs(nrows), \
                                                               db_seg_rows(nrows), sm, ws.segmin, db, \
                                                               img, qp, q64, nq, amax, best, stats, fa)
#define IA_RESCORE_CASE(MD, IM)                                                                  \
    do {                                                                                         \
        if (MD != 0 && MD != 3 && M <= RESCORE_FIFTH_MAX_M) IA_RESCORE_LAUNCH(MD, IM, true);                \
        else IA_RESCORE_LAUNCH(MD, IM, false);                                                   \
    } while (0)
    if (im) {
        if (mode == 3) IA_RESCORE_CASE(3, true);
        else if (mode == 2) IA_RESCORE_CASE(2, true);
        else if (mode == 1) IA_RESCORE_CASE(1, true);
        else IA_RESCORE_CASE(0, true);
    } else {
        if (mode == 3) IA_RESCORE_CASE(3, false);
        else if (mode == 2) IA_RESCORE_CASE(2, false);
        else if (mode == 1) IA_RESCORE_CASE(1, false);
        else IA_RESCORE_CASE(0, false);
    }
#undef IA_RESCORE_LAUNCH
#undef IA_RESCORE_CASE
    IA_LAUNCH_CHECK("k_rescore");
    return IA_OK;
}

__global__ void k_split_best(const Best *b, int M, int64_t *idx, double *dist) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= M) return;
    if (idx) idx[i] = b[i].idx;
    if (dist) dist[i] = b[i].d;
}

// ---------------------------------------------------------------------------------
// per-pixel API helpers (algorithms.py:92-135)
// ---------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_coherence_pick(const double *rows, int n,
                                                       const double *q, int32_t *out) {
    double bd = INFINITY;
    long long bi = 0x7fffffffffffffffLL;
    for (int i = threadIdx.x; i < n; i += 64) {
        Pw55 pw;
#pragma unroll
        for (int k = 0; k < IA_D; ++k) {
            const double x = rows[(long)i * IA_D + k] - q[k];
            pw.feed(k, x * x);
        }
        best_update(bd, bi, sqrt(pw.res), i);
    }
    for (int o = 32; o > 0; o >>= 1) {
        const double od = __shfl_xor(bd, o);
        const long long oi = __shfl_xor(bi, o);
        best_update(bd, bi, od, oi);
    }
    if (threadIdx.x == 0) out[0] = (int32_t)bi;
}

__global__ void k_wdist(const double *a, const double *q, const double *w, int n,
                        double *out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Pw55 pw;
#pragma unroll
    for (int k = 0; k < IA_D; ++k) {
        const double x = (a[(long)i * IA_D + k] - q[(long)i * IA_D + k]) * w[k];
        pw.feed(k, x * x);
    }
    const double s = sqrt(pw.res);
    out[i] = s * s;
}

}  // namespace ia

using namespace ia;

extern "C" {

static constexpr int MATCH_BATCH = 384;

size_t ia_match_workspace_bytes(int M, long nrows) {
    const int mb = M < MATCH_BATCH ? M : MATCH_BATCH;
    const int qr = qrows_alloc(mb);
    size_t b = 0;
    b += align_up((size_t)qr * IA_DP * sizeof(float), 256);                        // qp
    b += align_up((size_t)qr * Q16_ROW * sizeof(half8), 256);                      // q16
    b += align_up((size_t)qr * sizeof(double), 256);                               // nq
    b += align_up(match_scratch_bytes(qr, nrows), 256);                           // screen out
    b += align_up((size_t)qr * sizeof(Best), 256);                                 // best
    return b;
}

int ia_match_batch(const IaMatchArgs *a, void *stream) {
    IA_ARG(a && (a->db || a->dbi || a->lsh) && a->q64 && a->center && a->amax && a->workspace &&
               a->M >= 0 && a->nrows > 0,
           "ia_match_batch: bad args");
    if (a->M == 0) return IA_OK;
    hipStream_t st = S(stream);
    const int mb = a->M < MATCH_BATCH ? a->M : MATCH_BATCH;
    const int qr = qrows_alloc(mb);
    char *w = reinterpret_cast<char *>(a->workspace);
    float *qp = reinterpret_cast<float *>(w);
    w += align_up((size_t)qr * IA_DP * sizeof(float), 256);
    _Float16 *q16 = reinterpret_cast<_Float16 *>(w);
    w += align_up((size_t)qr * Q16_ROW * sizeof(half8), 256);
    double *nq = reinterpret_cast<double *>(w);
    w += align_up((size_t)qr * sizeof(double), 256);
    void *scratch = w;
    w += align_up(match_scratch_bytes(qr, a->nrows), 256);
    Best *best = reinterpret_cast<Best *>(w);
    IA_HIP(hipMemsetAsync(qp, 0, (size_t)qr * IA_DP * sizeof(float), st));
    IA_HIP(hipMemsetAsync(q16, 0, (size_t)qr * Q16_ROW * sizeof(half8), st));
    IA_HIP(hipMemsetAsync(scratch, 0, WL_HEAD, st));   // empty work list
    const DbSrc src = make_dbsrc(a->src);
    for (int m0 = 0; m0 < a->M; m0 += MATCH_BATCH) {
        const int M = a->M - m0 < MATCH_BATCH ? a->M - m0 : MATCH_BATCH;
        const double *q = a->q64 + (long)m0 * IA_DP;
        int rc;
        if (a->lsh) {
            if ((rc = launch_lsh_match(a->lsh, src, a->row0, a->nrows, M, q, a->center, best,
                                       nullptr, st)))
                return rc;
        } else {
            if ((rc = launch_query_rows(q, M, a->center, qp, nq, a->amax, q16, st))) return rc;
            if ((rc = launch_match(src, a->row0, a->nrows, a->db, a->dbi, qp, q16, M, q, nq,
                                   a->amax, scratch, best, nullptr, st)))
                return rc;
        }
        k_split_best<<<(M + 255) / 256, 256, 0, st>>>(best, M, a->idx ? a->idx + m0 : nullptr,
                                                      a->dist ? a->dist + m0 : nullptr);
        IA_LAUNCH_CHECK("k_split_best");
    }
    return IA_OK;
}

int ia_coherence_pick(const double *rows, int n, const double *q, int32_t *out, void *stream) {
    IA_ARG(rows && q && out && n > 0, "ia_coherence_pick: bad args");
    k_coherence_pick<<<1, 64, 0, S(stream)>>>(rows, n, q, out);
    IA_LAUNCH_CHECK("k_coherence_pick");
    return IA_OK;
}

int ia_wdist_batch(const double *a, const double *q, const double *w, int n, double *out,
                   void *stream) {
    IA_ARG(a && q && w && out && n >= 0, "ia_wdist_batch: bad args");
    if (n == 0) return IA_OK;
    k_wdist<<<(n + 63) / 64, 64, 0, S(stream)>>>(a, q, w, n, out);
    IA_LAUNCH_CHECK("k_wdist");
    return IA_OK;
}

}  // extern "C"

// ---- diagnostic entry points (include/ia_diag.h) ----------------------------------
#include "../../include/ia_diag.h"

extern "C" {

int ia_diag_qp_rows(int M) { return qrows_alloc(M); }

int ia_diag_query_rows16(const double *q64, int M, const double *center, const float *amax,
                         float *qp, void *q16, double *nq, void *stream) {
    IA_ARG(q64 && center && amax && qp && q16 && nq && M > 0, "ia_diag_query_rows16: bad args");
    return launch_query_rows(q64, M, center, qp, nq, amax, reinterpret_cast<_Float16 *>(q16),
                             S(stream));
}

int ia_diag_set_rescore_mode(int mode) {
    const int prev = rescore_mode();
    if (mode >= -1 && mode <= 1) g_rescore_mode.store(mode);
    return prev;
}

int ia_diag_screen16(const void *db, long nrows, const void *q16, int M, float *segmin,
                     void *stream) {
    IA_ARG(db && q16 && segmin && M > 0 && nrows > 0, "ia_diag_screen16: bad args");
    return launch_screen16(db, nullptr, nrows, StageMap{0, 1, db_chunk_rows(nrows) / 128},
                           reinterpret_cast<const _Float16 *>(q16), M, segmin, S(stream));
}

int ia_diag_stage_map(long row0, long nrows, int W, int Himg, int *out) {
    IA_ARG(out && nrows > 0 && row0 >= 0, "ia_diag_stage_map: bad args");
    const StageMap m = db_stage_map(row0, nrows, W, Himg);
    out[0] = m.W;
    out[1] = m.nstrip;
    out[2] = m.sc;
    return IA_OK;
}

int ia_diag_screen16_rows(const IaSrcLevel *src, long row0, long nrows, const void *db,
                          const void *q16, int M, float *segmin, void *stream) {
    IA_ARG(src && db && q16 && segmin && M > 0 && nrows > 0, "ia_diag_screen16_rows: bad args");
    return launch_screen16(db, nullptr, nrows, db_stage_map(row0, nrows, src->Aw, src->Ah),
                           reinterpret_cast<const _Float16 *>(q16), M, segmin, S(stream));
}

int ia_diag_screen16_image(const IaSrcLevel *src, long row0, long nrows, const void *dbi,
                           const void *q16, int M, float *segmin, void *stream) {
    IA_ARG(src && dbi && q16 && segmin && M > 0 && nrows > 0, "ia_diag_screen16_image: bad args");
    ImgDb img;
    IA_ARG(img_db_layout(src->Ah, src->Aw, src->A_hs, src->A_ws, src->nAp, row0, nrows, dbi, img, nullptr),
           "ia_diag_screen16_image: the image form does not apply to this level");
    return launch_screen16(nullptr, &img, nrows, db_stage_map(row0, nrows, src->Aw, src->Ah),
                           reinterpret_cast<const _Float16 *>(q16), M, segmin, S(stream));
}

}  // extern "C"
