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

// ---- device-side exchange of a sharded level (PeerView, ia_internal.h) ----------------
// granules of (slot, source rank, query) in a receive box
__device__ __forceinline__ unsigned long long *peer_cell(unsigned long long *box, const PeerView &p,
                                                         int src, int q) {
    return box + (((long)(p.epoch & 1) * p.nranks + src) * p.mcap + q) * PEER_CELL;
}
// rank g's box pointer (selects over the kernel argument, not an indexed private copy)
__device__ __forceinline__ unsigned long long *peer_box(const PeerView &p, int g) {
    unsigned long long *box = p.box[0];
#pragma unroll
    for (int k = 1; k < IA_PEER_MAX; ++k) box = g == k ? p.box[k].get() : box;
    return box;
}
// lanes g < nranks of one wave: this rank's winner of query q into rank g's box (system-
// scope 8-byte stores: each granule arrives whole, over xGMI for a peer GPU's box)
__device__ __forceinline__ void peer_publish(const PeerView &p, int q, double d, long long row,
                                             int lane) {
    if (lane >= p.nranks) return;
    unsigned long long *dst = peer_cell(peer_box(p, lane), p, p.rank, q);
    const unsigned long long tag = (unsigned long long)p.epoch << 32;
    const unsigned long long bits = (unsigned long long)__double_as_longlong(d);
    __hip_atomic_store(dst, tag | (bits & 0xffffffffULL), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(dst + 1, tag | (bits >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(dst + 2, tag | (unsigned long long)(unsigned int)row, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
}
// 10 s at the 100 MHz real-time counter: a peer that never publishes (a dead rank, or
// memory the peer's stores do not reach) sets the error word instead of hanging the GPU;
// once it is set every later wait of this rank gives up at once (ia_peer_status reports it)
constexpr unsigned long long PEER_TIMEOUT_TICKS = 1000000000ULL;
// one whole wave: lane g < nranks reads rank g's granules of query q from this rank's box
// until all three carry this wave's epoch; then the lexicographic (distance, row) minimum
// over the ranks, valid in every lane.  bd / bi: this rank's own winner (uniform) on entry;
// kept as the result on timeout (false; the error word is then set).
__device__ __forceinline__ bool peer_collect(const PeerView &p, int q, int lane, double &bd,
                                             long long &bi, unsigned long long *raw = nullptr) {
    const bool mine = lane < p.nranks;
    const unsigned long long *src = peer_cell(peer_box(p, p.rank), p, mine ? lane : 0, q);
    unsigned long long g0 = 0, g1 = 0, g2 = 0;
    bool dead = __hip_atomic_load(p.err.get(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    bool ok;
    for (;;) {
        ok = true;
        if (mine) {
            g0 = __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            g1 = __hip_atomic_load(src + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            g2 = __hip_atomic_load(src + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            ok = (unsigned)(g0 >> 32) == p.epoch && (unsigned)(g1 >> 32) == p.epoch &&
                 (unsigned)(g2 >> 32) == p.epoch;
        }
        if (__all(ok) || dead) break;
        if (__builtin_amdgcn_s_memrealtime() - t0 > PEER_TIMEOUT_TICKS) {
            if (lane == 0) __hip_atomic_fetch_or(p.err.get(), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            dead = true;
            break;
        }
        __builtin_amdgcn_s_sleep(1);
    }
    if (raw && lane < 2) { raw[3 * lane] = g0; raw[3 * lane + 1] = g1; raw[3 * lane + 2] = g2; }
    if (dead) return false;
    double d = INFINITY;
    long long i = 0x7fffffffffffffffLL;
    if (mine) {
        d = __longlong_as_double((long long)(((g1 & 0xffffffffULL) << 32) | (g0 & 0xffffffffULL)));
        i = (long long)(g2 & 0xffffffffULL);
    }
    for (int o = 32; o > 0; o >>= 1) {
        const double od = __shfl_xor(d, o);
        const long long oi = __shfl_xor(i, o);
        fin_best(d, i, od, oi);
    }
    bd = d;
    bi = i;
    return true;
}

// ---- the fused per-wave kernel's records (k_xwave, ia_xwave.hip) ---------------------
// one rank's exact winner of one query: distance, global row, the row's weighted (kappa)
// distance to the query and its A' value (the B' value it would write)
struct XRec {
    double d;
    long long i;
    double wd, val;
};
__device__ __forceinline__ void xrec_take(XRec &b, const XRec &o) {
    if (o.d < b.d || (o.d == b.d && o.i < b.i)) b = o;
}
// lexicographic (distance, row) minimum over the wave, valid in every lane
__device__ __forceinline__ XRec xrec_wave_min(XRec b) {
    for (int o = 32; o > 0; o >>= 1) {
        const XRec x{__shfl_xor(b.d, o), __shfl_xor(b.i, o), __shfl_xor(b.wd, o), __shfl_xor(b.val, o)};
        xrec_take(b, x);
    }
    return b;
}
// lanes g < nranks: this rank's record of query q into rank g's box, 7 granules
// {epoch << 32 | 32-bit payload} (d lo/hi, row, wd lo/hi, val lo/hi); rows < 2^32 (checked
// on the host)
__device__ __forceinline__ void peer_publish_rec(const PeerView &p, int q, const XRec &r, int lane) {
    if (lane >= p.nranks) return;
    unsigned long long *dst = peer_cell(peer_box(p, lane), p, p.rank, q);
    const unsigned long long tag = (unsigned long long)p.epoch << 32;
    const unsigned long long bd = (unsigned long long)__double_as_longlong(r.d);
    const unsigned long long bw = (unsigned long long)__double_as_longlong(r.wd);
    const unsigned long long bv = (unsigned long long)__double_as_longlong(r.val);
    auto put = [&](int k, unsigned long long v) {
        __hip_atomic_store(dst + k, tag | v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    };
    put(0, bd & 0xffffffffULL);
    put(1, bd >> 32);
    put(2, (unsigned long long)(unsigned int)r.i);
    put(3, bw & 0xffffffffULL);
    put(4, bw >> 32);
    put(5, bv & 0xffffffffULL);
    put(6, bv >> 32);
}
// one whole wave: lane g < nranks polls rank g's record of query q in this rank's box until
// all 7 granules carry this wave's epoch; r = the lexicographic minimum over the ranks
// (valid in every lane).  On timeout (or an earlier one on this exchange) r is left as the
// caller's own record and false is returned (the error word is set).
__device__ __forceinline__ bool peer_collect_rec(const PeerView &p, int q, int lane, XRec &r) {
    const bool mine = lane < p.nranks;
    const unsigned long long *src = peer_cell(peer_box(p, p.rank), p, mine ? lane : 0, q);
    unsigned long long g0 = 0, g1 = 0, g2 = 0, g3 = 0, g4 = 0, g5 = 0, g6 = 0;
    bool dead = __hip_atomic_load(p.err.get(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    auto ld = [&](int k) { return __hip_atomic_load(src + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); };
    auto tagged = [&](unsigned long long v) { return (unsigned)(v >> 32) == p.epoch; };
    for (;;) {
        bool ok = true;
        if (mine) {
            g0 = ld(0); g1 = ld(1); g2 = ld(2); g3 = ld(3); g4 = ld(4); g5 = ld(5); g6 = ld(6);
            ok = tagged(g0) && tagged(g1) && tagged(g2) && tagged(g3) && tagged(g4) && tagged(g5) &&
                 tagged(g6);
        }
        if (__all(ok) || dead) break;
        if (__builtin_amdgcn_s_memrealtime() - t0 > PEER_TIMEOUT_TICKS) {
            if (lane == 0) __hip_atomic_fetch_or(p.err.get(), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            dead = true;
            break;
        }
        __builtin_amdgcn_s_sleep(1);
    }
    if (dead) return false;
    auto dbl = [](unsigned long long lo, unsigned long long hi) {
        return __longlong_as_double((long long)(((hi & 0xffffffffULL) << 32) | (lo & 0xffffffffULL)));
    };
    XRec x{INFINITY, 0x7fffffffffffffffLL, 0.0, 0.0};
    if (mine) x = XRec{dbl(g0, g1), (long long)(g2 & 0xffffffffULL), dbl(g3, g4), dbl(g5, g6)};
    r = xrec_wave_min(x);
    return true;
}

// The tail kernels run coh_pick on one wave and app_wdist + finish_apply on another.
// (Picking the coherence candidate ahead, on a side stream beside the screen, measured 5 %
// slower on c4: the per-wave cross-stream event waits cost more than the two gather rounds
// they hide.)

}  // namespace ia
