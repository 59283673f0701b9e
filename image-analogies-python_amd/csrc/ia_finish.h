// ia_finish.h — per-pixel tail of one synthesis step (image_analogies.py:169-217), shared
// by k_finish (ia_synth.hip; after the cross-rank exchange) and the fused single-GPU
// exact stage k_rescore<true> (ia_match.hip).
#pragma once
#include "ia_internal.h"

namespace ia {

// the coherence candidate of one query pixel (coh_pick)
struct CohSel {
    long long wix;       // winning candidate's DB row
    int wr, wc, wim;     // its pixel and A' image
    int rr, rc;          // r*: the B' pixel whose source it continues
    int valid;           // 0: no candidate (first pixel of the level, or none in range)
    double dcoh;         // its weighted distance to the query
};

__device__ __forceinline__ void fin_best(double &bd, long long &bi, double d, long long i) {
    if (d < bd || (d == bd && i < bi)) { bd = d; bi = i; }
}

// Coherence half of the tail, executed by ONE 64-lane wave for query pixel m of wave t
// (query in qs, LDS): best_coherence_match (algorithms.py:92-130) over the causal 3x5
// window (lanes 0..14 = the reference's product(rows, cols) order) and the weighted
// distance of its winner (algorithms.py:133-135).  Needs only s / im of earlier waves.
// Result valid in every lane.
__device__ __forceinline__ CohSel coh_pick(const DbSrc &src, int m, const FinishArgs &f,
                                           const double *qs, int lane) {
    CohSel r{0, 0, 0, 0, 0, 0, 0, 0.0};
    const int y = f.y_lo + m, x = f.t - 3 * y;
    if (y == 0 && x == 0) return r;
    const int W = f.W;
    const int Ah = src.A.h, Aw = src.A.w;
    double cd = INFINITY;
    long long cl = 0x7fffffffffffffffLL;
    long cix = -1;
    int cr = 0, cc = 0, cim = 0;
    if (lane < 15) {
        const int rr = y - 2 + lane / 5, rc = x - 2 + lane % 5;
        if (rr >= 0 && rc >= 0 && rc < W && (rr < y || rc < x)) {
            const long sidx = (long)rr * W + rc;
            const int sr = f.s[2 * sidx] + y - rr, sc = f.s[2 * sidx + 1] + x - rc;
            if (sr >= 0 && sr < Ah && sc >= 0 && sc < Aw) {
                const int simg = f.im[sidx];
                cix = ((long)Ah * simg + sr) * Aw + sc;
                cr = sr; cc = sc; cim = simg;
                cd = sqrt(row_dist2(src, cix, qs));
                cl = lane;
            }
        }
    }
    double bd = cd;
    long long bl = cl;
    for (int o = 32; o > 0; o >>= 1) {
        const double od = __shfl_xor(bd, o);
        const long long ol = __shfl_xor(bl, o);
        fin_best(bd, bl, od, ol);
    }
    if (bl == 0x7fffffffffffffffLL) return r;
    const int win = (int)bl;
    r.wix = __shfl(cix, win);
    r.wr = __shfl(cr, win);
    r.wc = __shfl(cc, win);
    r.wim = __shfl(cim, win);
    r.rr = y - 2 + win / 5;
    r.rc = x - 2 + win % 5;
    r.valid = 1;
    double d = 0.0;
    if (lane == 1) d = row_wdist(src, r.wix, qs, f.weights);
    r.dcoh = __shfl(d, 1);
    return r;
}

// Weighted distance of the exact-match winner app (algorithms.py:133-135) for the kappa
// test: one gather round by lane 0, valid in every lane.  Runs beside coh_pick (another
// wave), so the tail's critical path is max(exact winner + 1 round, coh_pick's 2 rounds).
__device__ __forceinline__ long long app_clamp(long long app, const FinishArgs &f) {
    return (app < 0 || app >= f.N_total) ? 0 : app;   // unreachable: every search has a winner
}
__device__ __forceinline__ double app_wdist(const DbSrc &src, long long app, const FinishArgs &f,
                                            const double *qs, int lane) {
    double d = 0.0;
    if (lane == 0) d = row_wdist(src, app_clamp(app, f), qs, f.weights);
    return __shfl(d, 0);
}

// The rest of the tail: the kappa test (image_analogies.py:200-211) of the coherence
// candidate c against the exact-match winner app (weighted distance d_app, app_wdist), and
// the B' / s / im update (:213-217).  With the debug outputs (image_analogies.py:141-159,
// 222-240): per pixel {p_app row, col, p_coh row, col, r* row, col, has coherence} and
// {d_app, d_coh} (zeros where there is no coherence candidate, as the reference).
__device__ __forceinline__ void finish_apply(const DbSrc &src, long long app, int m,
                                             const FinishArgs &f, const CohSel &c, double d_app,
                                             int lane) {
    const int y = f.y_lo + m, x = f.t - 3 * y;
    const int W = f.W;
    const int Aw = src.A.w;
    const long hw = src.hw;
    app = app_clamp(app, f);
    long img = app / hw;
    long rem = app - img * hw;
    int pr = (int)(rem / Aw), pc = (int)(rem - (long)(rem / Aw) * Aw);
    if (c.valid && c.dcoh <= d_app * f.kappa_factor) {
        pr = c.wr; pc = c.wc; img = c.wim;
    }
    if (lane == 0) {
        const long q = (long)y * W + x;
        if (f.dbg_px) {
            int32_t *o = f.dbg_px + 7 * q;
            o[0] = (int32_t)(rem / Aw);
            o[1] = (int32_t)(rem - (long)(rem / Aw) * Aw);
            o[2] = c.valid ? c.wr : 0;
            o[3] = c.valid ? c.wc : 0;
            o[4] = c.valid ? c.rr : 0;
            o[5] = c.valid ? c.rc : 0;
            o[6] = c.valid;
            f.dbg_dist[2 * q] = c.valid ? d_app : 0.0;
            f.dbg_dist[2 * q + 1] = c.valid ? c.dcoh : 0.0;
        }
        f.Bp_lg[q] = src.Ap.lg[img * hw + (long)pr * Aw + pc];
        f.s[2 * q] = pr;
        f.s[2 * q + 1] = pc;
        f.im[q] = (int32_t)img;
    }
}

// The tail kernels run coh_pick on one wave and app_wdist + finish_apply on another.
// (Picking the coherence candidate ahead, on a side stream beside the screen, measured 5 %
// slower on c4: the per-wave cross-stream event waits cost more than the two gather rounds
// they hide.)

}  // namespace ia
