// ia_xwave.hip — everything a wave needs after its screen, in ONE launch (SURVEY §8(a) rows
// a11-a15, §8(e)).
//
// The reference's pixel loop (image_analogies.py:161-220) does, per pixel: query build
// (:166-168), approximate match (:175, algorithms.py:73-75), coherence match (:193,
// algorithms.py:92-130), two weighted distances and the kappa test (:200-211), and the
// B'/s/im update (:213-220).  On the wavefront t = x + 3y the screen (ia_screen16.hip) is
// the only step with real arithmetic; every other step is a few dependent memory round
// trips, and as separate launches (query build, exact stage, exchange + finish) they cost
// more per wave than the screen itself once the DB is sharded over 8 GPUs.  k_xwave runs
// them all for wave t, one 4-wave workgroup per pixel:
//
//   1. exact stage: e* over the pixel's segment minima, candidate segments, fp32 re-screen
//      of their rows (4 waves in parallel), fp64 rescore of the rows within the bound
//      (lane-parallel gathers, numpy's pairwise order from LDS), the lexicographic winner
//      with its weighted distance and A' value;
//   2. meanwhile wave 1 picks the coherence candidate (best_coherence_match: the 15
//      causal window positions gathered lane-parallel, sqrt distances, first minimum);
//   3. sharded DB: the winner goes to every rank's receive box and every rank's winner of
//      this pixel is collected from this rank's box (PeerView, ia_finish.h), nothing waits
//      before this workgroup has published;
//   4. kappa test and the B'/s/im (+ debug) update; the new B' value is published as two
//      tagged 8-byte granules (the decision box, one entry per row);
//   5. the query row of the SAME row in wave t + 1, pixel (y, x + 1): of its 55 features only
//      two can come from wave t — this pixel (y, x) and the upper neighbour's (y - 1, x + 3)
//      (the only wave-t pixels inside its causal windows, reflections included) — so they
//      come from this workgroup's registers and from the neighbour's decision granules;
//      every other feature is read from memory (earlier waves, the coarse level, B).
//
// Workgroups take their pixel from a ticket counter, so a workgroup only ever waits for
// the decision of a lower ticket (dispatched earlier), and it publishes its own record
// and decision before any wait: no wait can hold a slot another workgroup needs to make
// the awaited progress (forward progress).
#include "ia_exact.h"
#include "ia_finish.h"
#include "../../include/ia_diag.h"

#include <climits>

namespace ia {

// address of feature k (0..54) of pixel (r, c) of a pair X (full: k < 34) | Y (half:
// k >= 34), the layout of emit_feature (ia_common.h), and its sample (rr, cc) in that
// feature's image
__device__ __forceinline__ const double *feat_addr(const ImgPair &X, const ImgPair &Y, int r, int c,
                                                   int k, int &rr, int &cc) {
    const bool yk = k >= 34;
    const int kk = yk ? k - 34 : k;
    const bool coarse = kk < 9;
    const int t = coarse ? kk : kk - 9;
    // select between field VALUES (selecting between the structs would take their address:
    // a local ImgPair would then live in scratch memory)
    const int xh = coarse ? X.hs : X.h, yh = coarse ? Y.hs : Y.h;
    const int xw = coarse ? X.ws : X.w, yw = coarse ? Y.ws : Y.w;
    const double *xb = coarse ? X.sm : X.lg, *yb = coarse ? Y.sm : Y.lg;
    const int h = yk ? yh : xh;
    const int w = yk ? yw : xw;
    const double *base = yk ? yb : xb;
    const int r0 = coarse ? (r >> 1) + t / 3 - 1 : r + t / 5 - 2;
    const int c0 = coarse ? (c >> 1) + t % 3 - 1 : c + t % 5 - 2;
    rr = symi2(r0, h);
    cc = symi2(c0, w);
    return base + (long)rr * w + cc;
}
// image, row and column of global DB row g (< 2^31: the fused kernel's host check)
__device__ __forceinline__ void row_pos(long g, long hw, int w, int &img, int &r, int &c) {
    const unsigned u = (unsigned)g, im = u / (unsigned)hw, rem = u - im * (unsigned)hw;
    img = (int)im;
    r = (int)(rem / (unsigned)w);
    c = (int)(rem - (unsigned)r * (unsigned)w);
}

// lane's double at p into the wave's LDS words lo[lane], hi[lane] by two 4-byte DMA copies
// (global_load_lds: the gather is in flight without holding registers; the wave waits with
// s_waitcnt vmcnt(0) before reading the words).  lo / hi must be wave-uniform.
__device__ __forceinline__ void dma_f64(const double *p, bool on, unsigned *lo, unsigned *hi) {
    if (on) {
        __builtin_amdgcn_global_load_lds((const void *)p, (void *)lo, 4, 0, 0);
        __builtin_amdgcn_global_load_lds((const void *)(reinterpret_cast<const char *>(p) + 4), (void *)hi, 4, 0, 0);
    }
}
__device__ __forceinline__ double lds_f64(const unsigned *lo, const unsigned *hi, int l) {
    return __longlong_as_double((long long)(((unsigned long long)hi[l] << 32) | lo[l]));
}

// numpy pairwise_sum of v[0..54] (Pw55's order, ia_common.h) from LDS
__device__ __forceinline__ double pw55_lds(const double *v) {
    double r[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = v[j];
#pragma unroll 1
    for (int k = 8; k < 48; k += 8) {
#pragma unroll
        for (int j = 0; j < 8; ++j) r[j] += v[k + j];
    }
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
#pragma unroll
    for (int k = 48; k < IA_D; ++k) res += v[k];
    return res;
}

// (XArgs: ia_internal.h)

// the record of one DB row rescored by one thread (the row list's overflow: never on the
// measured configs; out of line so that its 55-load gathers do not inflate the common path)
__device__ __attribute__((noinline)) XRec row_rec(DbSrc src, long g, const double *qs,
                                                  const double *wts) {
    return XRec{row_dist2(src, g, qs), g, row_wdist(src, g, qs, wts), src.Ap.lg[g]};
}

constexpr int XW_ROWCAP = 256;   // rows within Trow rescored lane-parallel (the rest in place)
constexpr int XW_RPW = 4;        // rows per rescoring wave and batch
constexpr int XW_NCOH = 15;      // coherence window positions (3 x 5, algorithms.py:101-102)
constexpr size_t XW_STAGE_B = (size_t)4 * XW_RPW * IA_DP * 8 * 2;   // 4 waves x (x^2, (x w)^2)
constexpr size_t XW_RAW_B = (size_t)4 * XW_RPW * 128 * 4;            // 4 waves x rows' lo / hi words
constexpr int XW_COH_DMA = 2 + 2 * XW_NCOH;                          // coherence copies per lane

__device__ __forceinline__ unsigned long long dgran(unsigned int tag, unsigned int bits) {
    return ((unsigned long long)tag << 32) | bits;
}

// a batch's job J (blockIdx.y) in place of the launch's pointers; b = wave t's parity
__device__ __forceinline__ void xjob_apply(XArgs &a, const XJob &J, int b) {
    a.src.A.sm = J.A_sm; a.src.A.lg = J.A_lg; a.src.Ap.sm = J.Ap_sm; a.src.Ap.lg = J.Ap_lg;
    a.im.fa = J.fa; a.im.ca = J.ca; a.im.norm = J.norm; a.im.ap = J.ap;
    a.db = J.db;
    a.segmin = J.segmin;
    a.q64 = J.q64[b]; a.qp = J.qp[b]; a.nq = J.nq[b];
    a.q64n = J.q64[b ^ 1]; a.qpn = J.qp[b ^ 1]; a.nqn = J.nq[b ^ 1]; a.q16n = J.q16[b ^ 1];
    a.amax = J.amax;
    a.center = J.center;
    a.B.sm = J.B_sm; a.B.lg = J.B_lg; a.Bp.sm = J.Bp_sm; a.Bp.lg = J.Bp_lg;
    a.dbox = J.dbox;
    a.tickets = J.ctl;
    a.err = J.ctl + 2;
    a.f.weights = J.weights;
    a.f.kappa_factor = J.kappa_factor;
    a.f.Bp_lg = J.Bp_lg;
    a.f.s = J.s; a.f.im = J.im; a.f.dbg_px = J.dbg_px; a.f.dbg_dist = J.dbg_dist;
}

// BATCH: a0.jobs holds a batch's pointers; the block copies the launch arguments into LDS
// once and overrides them with its job's (a private copy of the arguments would live in
// scratch memory), then reads them from there
template <bool IMG, bool BATCH>
__global__ __launch_bounds__(256, 3) void k_xwave(XArgs a0) {
    __shared__ __attribute__((aligned(16))) char sa_raw[BATCH ? sizeof(XArgs) : 16];
    XArgs &sa = *reinterpret_cast<XArgs *>(sa_raw);
    if constexpr (BATCH) {
        static_assert(sizeof(XArgs) % 8 == 0, "XArgs copied as 8-byte words");
        const unsigned long long *w0 = reinterpret_cast<const unsigned long long *>(&a0);
        unsigned long long *w1 = reinterpret_cast<unsigned long long *>(&sa);
        for (int w = threadIdx.x; w < (int)(sizeof(XArgs) / 8); w += 256) w1[w] = w0[w];
        __syncthreads();
        if (threadIdx.x == 0) xjob_apply(sa, a0.jobs[blockIdx.y], a0.f.t & 1);
        __syncthreads();
    }
    const XArgs &a = BATCH ? sa : a0;
    constexpr size_t POOL = IMG ? (size_t)4 * WIN_SLOT : 0;
    constexpr size_t RESB = XW_STAGE_B + XW_RAW_B;
    __shared__ __attribute__((aligned(16))) char pool[POOL > RESB ? POOL : RESB];
    __shared__ double cx[XW_NCOH][IA_DP], cw[XW_NCOH][IA_DP];
    __shared__ double qs[IA_DP], wts[IA_DP];
    __shared__ float qf[IA_DP];
    __shared__ int slist[RESCORE_SEGCAP];
    __shared__ long rlist[XW_ROWCAP];
    __shared__ int tk, scount, rcount;
    __shared__ unsigned int nresc;
    __shared__ float redf[4];
    __shared__ XRec wbest[4];
    __shared__ CohSel cs;
    __shared__ double csval;
    // wave 1's coherence candidates (broadcast to the wave's gathers) and their A' values;
    // wave 0's next-query features and centre (LDS-DMA words)
    __shared__ long long ccix[XW_NCOH];
    __shared__ unsigned cvw[2][64];
    __shared__ unsigned nxw[4][64];
    __shared__ int cpos[XW_NCOH][3];

    // wv must be provably uniform: the LDS-DMA destinations derived from it go into M0 (a
    // per-lane value would turn each copy into a 64-iteration waterfall loop)
    const int tid = threadIdx.x, lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const FinishArgs &f = a.f;
    const DbSrc &src = a.src;
    const int t = f.t, W = f.W;
    const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
    if (tid == 0) tk = (int)atomicAdd(&a.tickets[t & 1], 1u);
    __syncthreads();
    const int i = tk;
    // diagnostic phase stamps (thread 0 of the first pixels)
    unsigned long long *trace =
        (a.trace && i < XW_TRACE_PX && t < XW_TRACE_T) ? a.trace + ((long)t * XW_TRACE_PX + i) * XW_TRACE_N : nullptr;
    auto stamp = [&](int k) {
        if (trace && tid == 0) trace[k] = __builtin_amdgcn_s_memrealtime();
    };
    auto wstamp = [&](int k) {   // lane 0 of any wave
        if (trace && lane == 0) trace[k] = __builtin_amdgcn_s_memrealtime();
    };
    if (trace && tid == 0) trace[0] = t_start;
    stamp(1);
    // the counter of launch t + 1 was launch t - 1's: empty it for the next launch
    if (i == 0 && tid == 0) __hip_atomic_store(&a.tickets[(t + 1) & 1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int y = f.y_lo + i, x = t - 3 * y;
    const bool cur = i < a.M;                                    // pixel (y, x) is in wave t
    const bool nxt = y >= a.y_lo_n && y < a.y_lo_n + a.M_n;       // (y, x + 1) is in wave t + 1

    // wave 0: the next query's features that do not depend on wave t, issued first
    // (copied into LDS by DMA, consumed only at the end: their wait never delays the exact
    // stage)
    const float amx = a.amax[vidx(0)];
    int pdep = 0;
    if (wv == 0 && nxt) {
        int rr = 0, cc = 0;
        const double *p = feat_addr(a.B, a.Bp, y, x + 1, lane < IA_D ? lane : 0, rr, cc);
        // 1: this pixel's new value, 2: the upper neighbour's
        pdep = lane < 43 || lane >= IA_D ? 0 : (rr == y && cc == x) ? 1 : (rr == y - 1 && cc == x + 3) ? 2 : 0;
        dma_f64(p, lane < IA_D && pdep == 0, nxw[0], nxw[1]);
        dma_f64(a.center + (lane < IA_D ? lane : 0), lane < IA_D, nxw[2], nxw[3]);
    }

    double own = 0.0;            // this pixel's new B' value (wave 0)
    if (cur) {
        // ---- 1. loads of one round trip: query, norm, bound, segment minima, coherence window
        double qsv = 0.0, wk = 0.0;
        float qfv = 0.f;
        if (tid < IA_DP) {
            qsv = a.q64[(long)i * IA_DP + tid];
            qfv = a.qp[(long)i * IA_DP + tid];
            wk = tid < IA_D ? f.weights[tid] : 0.0;
        }
        const double nqq = a.nq[vidx(i)];
        const float am = amx;
        const long n4 = a.nseg / 4;
        const float4 *sq4 = reinterpret_cast<const float4 *>(a.segmin + (long)i * a.nseg);
        float4 v[RESCORE_REG];
        segmin_load(sq4, n4, v);
        // wave 1, lane l < 15: s / im of coherence window position l (algorithms.py:101-119),
        // issued now, used after e*
        const int rr0 = y - 2 + lane / 5, rc0 = x - 2 + lane % 5;
        const bool cpos_ok = wv == 1 && lane < XW_NCOH && rr0 >= 0 && rc0 >= 0 && rc0 < W &&
                             (rr0 < y || rc0 < x);
        int s_r = 0, s_c = 0, s_i = 0;
        if (cpos_ok) {
            const long sidx = (long)rr0 * W + rc0;
            s_r = f.s[2 * sidx];
            s_c = f.s[2 * sidx + 1];
            s_i = f.im[sidx];
        }
        if (tid == 0) { scount = 0; nresc = 0; rcount = 0; }
        const float emin = segmin_scan(sq4, n4, v, redf);
        stamp(2);
        if (tid < IA_DP) {
            qs[tid] = qsv;
            qf[tid] = qfv;
            wts[tid] = wk;
        }
        double Tseg, Trow;
        bool force_full;
        rescore_thresholds(emin, am, nqq, Tseg, Trow, force_full);
        const float twoR = ldexpf(1.f, split16_db_scale(am).R);
        segmin_select(sq4, n4, v, Tseg, slist, &scount);
        __syncthreads();
        stamp(3);
        const int ns = scount;
        const bool full = ns > RESCORE_SEGCAP || force_full;
        const long nscan = full ? a.nseg : ns;
        const long nrs = nscan * a.seg_rows;
        const int lseg = __builtin_ctz((unsigned)a.seg_rows);
        // wave 1: the coherence candidates (p_r = s(r) + q - r inside A'); an invalid one gets
        // position (0, 0, 0) so that its (unused) copies read valid memory
        if (wv == 1) {
            if (lane < XW_NCOH) {
                const int sr = s_r + y - rr0, sc = s_c + x - rc0;
                const bool ok = cpos_ok && sr >= 0 && sr < src.A.h && sc >= 0 && sc < src.A.w;
                ccix[lane] = ok ? ((long)src.A.h * s_i + sr) * src.A.w + sc : -1;
                cpos[lane][0] = ok ? sr : 0; cpos[lane][1] = ok ? sc : 0; cpos[lane][2] = ok ? s_i : 0;
            }
            wave_lds_sync();
        }
        // wave 1: the candidates' A' values and all their features requested at once by LDS
        // DMA (candidate c's lo / hi words in cx / cw): EXACTLY XW_COH_DMA copies, none
        // skipped, so that a window copied in before them is waited for with vmcnt
        // (loads return in order)
        auto coh_issue = [&]() {
            const long long cl = lane < XW_NCOH ? ccix[lane] : -1;
            dma_f64(src.Ap.lg + (cl >= 0 ? cl : 0), true, cvw[0], cvw[1]);
            unsigned *clo = reinterpret_cast<unsigned *>(&cx[0][0]);
            unsigned *chi = reinterpret_cast<unsigned *>(&cw[0][0]);
#pragma unroll 1
            for (int c = 0; c < XW_NCOH; ++c) {
                ImgPair ap = src.Ap;
                ap.sm += (long)cpos[c][2] * src.hws;
                ap.lg += (long)cpos[c][2] * src.hw;
                int rr, cc;
                const double *fp = feat_addr(src.A, ap, cpos[c][0], cpos[c][1], lane < IA_D ? lane : 0, rr, cc);
                dma_f64(fp, true, clo + c * 64, chi + c * 64);
            }
            wstamp(13);
        };

        // ---- 2. fp32 re-screen of the candidate segments' rows; rows within Trow to the
        // list (overflow rows rescored in place: never on the measured configs)
        unsigned int mine = 0;
        XRec ob{INFINITY, LLONG_MAX, 0.0, 0.0};
        auto take = [&](long lr, float e) {
            if (lr < a.nrows && (double)e <= Trow) {
                ++mine;
                const int pos = atomicAdd(&rcount, 1);
                if (pos < XW_ROWCAP) {
                    rlist[pos] = lr;
                } else {
                    const long g = a.row0 + lr;
                    xrec_take(ob, row_rec(src, g, qs, wts));
                }
            }
        };
        auto stage_row = [&](long k) {   // local row of re-screen element k (a stage's first)
            const long seg = full ? (k >> lseg) : slist[k >> lseg];
            return seg_lrow(a.smap, seg, a.seg_rows, k & (a.seg_rows - 1));
        };
        if constexpr (IMG) {
            // stage j of each 512-row step to wave j, its window copied into LDS by DMA: one
            // round trip per step (more than one candidate segment per query is rare); wave 1
            // copies its first window before the coherence gathers and waits for that alone
            char *wb = pool + wv * WIN_SLOT;
            long k0 = 128L * wv, lr = 0;
            if (k0 < nrs) {
                lr = stage_row(k0);
                win_dma(a.im, lr, lane, wb);
            }
            if (wv == 1) {
                asm volatile("" ::: "memory");   // the window's copies are issued first
                coh_issue();
                asm volatile("s_waitcnt vmcnt(%0)" :: "n"(XW_COH_DMA) : "memory");
                __builtin_amdgcn_wave_barrier();
            } else {
                win_dma_wait();
            }
            if (wv == 0) wstamp(11);
            while (k0 < nrs) {
                float e0, e1;
                rescreen_win2(wb, lane, qf, twoR, e0, e1);
                take(lr + lane, e0);
                take(lr + lane + 64, e1);
                k0 += 512;
                if (k0 >= nrs) break;
                wave_lds_sync();   // every lane is done reading the slot
                lr = stage_row(k0);
                win_dma(a.im, lr, lane, wb);
                win_dma_wait();
            }
        } else {
            // row form: one row per thread per step (224-B split rows), waves 0, 2, 3 (wave 1's
            // in-order loads would wait behind its coherence gathers)
            if (wv == 1) coh_issue();
            const int rt = (wv == 0 ? 0 : wv - 1) * 64 + lane;
            for (long k = rt; wv != 1 && k < nrs; k += 192) {
                const long seg = full ? (k >> lseg) : slist[k >> lseg];
                const long lr = seg_lrow(a.smap, seg, a.seg_rows, k & (a.seg_rows - 1));
                half8 g0[DB16_GROUPS], g1[DB16_GROUPS];
                load_row16(reinterpret_cast<const half8 *>(a.db), lr < a.nrows ? lr : 0, g0, g1);
                take(lr, rescreen16(g0, g1, qf, twoR));
            }
        }
        if (wv == 0) wstamp(12);
        if (mine) atomicAdd(&nresc, mine);
        __syncthreads();   // the row list is complete; the windows are free
        stamp(4);

        // ---- 3. fp64 rescore of the listed rows (waves 2, 3, 0 in turn, XW_RPW rows per
        // batch: lane k copies feature k of each row into LDS by DMA, the squares go through
        // LDS, lane j sums row j in numpy's order) | wave 1: the coherence pick
        const int nl = rcount < XW_ROWCAP ? rcount : XW_ROWCAP;
        XRec b = ob;
        if (wv != 1) {
            const int rk = wv == 2 ? 0 : (wv == 3 ? 1 : 2);
            double *rx = reinterpret_cast<double *>(pool) + (size_t)wv * XW_RPW * IA_DP * 2;
            unsigned *rw = reinterpret_cast<unsigned *>(pool + XW_STAGE_B) + wv * XW_RPW * 128;
            for (int base = rk * XW_RPW; base < nl; base += 3 * XW_RPW) {
                // lane j < XW_RPW locates row base + j once
                int li = 0, lr_ = 0, lc = 0;
                long lg = 0;
                if (lane < XW_RPW && base + lane < nl) {
                    lg = a.row0 + rlist[base + lane];
                    row_pos(lg, src.hw, src.A.w, li, lr_, lc);
                }
                wave_lds_sync();   // the previous batch is done with rx and rw
#pragma unroll 1
                for (int j = 0; j < XW_RPW && base + j < nl; ++j) {
                    const int ri = __shfl(li, j), rr = __shfl(lr_, j), rc = __shfl(lc, j);
                    const long rg = __shfl(lg, j);
                    ImgPair ap = src.Ap;
                    ap.sm += (long)ri * src.hws;
                    ap.lg += (long)ri * src.hw;
                    int r2, c2;
                    const double *fp = feat_addr(src.A, ap, rr, rc, lane < IA_D ? lane : 0, r2, c2);
                    dma_f64(lane == IA_D ? src.Ap.lg + rg : fp, true, rw + j * 128, rw + j * 128 + 64);
                }
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                wave_lds_sync();
                const double ql = lane < IA_D ? qs[lane] : 0.0, wl = lane < IA_D ? wts[lane] : 0.0;
#pragma unroll 1
                for (int j = 0; j < XW_RPW && base + j < nl; ++j) {
                    const double g = lds_f64(rw + j * 128, rw + j * 128 + 64, lane);
                    if (lane < IA_D) {
                        const double xx = g - ql;
                        const double xw = xx * wl;
                        rx[j * IA_DP + lane] = xx * xx;
                        rx[(XW_RPW + j) * IA_DP + lane] = xw * xw;
                    } else if (lane == IA_D) {
                        rx[j * IA_DP + IA_D] = g;   // the row's A' value (slot 55)
                    }
                }
                wave_lds_sync();
                if (lane < XW_RPW && base + lane < nl) {
                    const double d = pw55_lds(rx + lane * IA_DP);
                    const double s = sqrt(pw55_lds(rx + (XW_RPW + lane) * IA_DP));
                    xrec_take(b, XRec{d, lg, s * s, rx[lane * IA_DP + IA_D]});
                }
            }
        } else {
            // best_coherence_match (algorithms.py:92-130) + the winner's compute_distance
            // (:133-135): the candidates' features, copied in before the re-screen; squares
            // written over the words from the last candidate down (candidate c's squares
            // only cover the words of candidates >= c, already read)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            wave_lds_sync();
            const long long cix = lane < XW_NCOH ? ccix[lane] : -1;
            const double cvl = cix >= 0 ? lds_f64(cvw[0], cvw[1], lane) : 0.0;
            const double ql = lane < IA_D ? qs[lane] : 0.0, wl = lane < IA_D ? wts[lane] : 0.0;
            const unsigned *clo = reinterpret_cast<const unsigned *>(&cx[0][0]);
            const unsigned *chi = reinterpret_cast<const unsigned *>(&cw[0][0]);
#pragma unroll 1
            for (int c = XW_NCOH - 1; c >= 0; --c) {
                const double g = lds_f64(clo + c * 64, chi + c * 64, lane);
                wave_lds_sync();   // every lane has candidate c's words
                if (lane < IA_D) {
                    const double xx = g - ql;
                    const double xw = xx * wl;
                    cx[c][lane] = xx * xx;
                    cw[c][lane] = xw * xw;
                }
            }
            wave_lds_sync();
            double cd = INFINITY, cwd = 0.0;
            long long cl = LLONG_MAX;
            if (lane < XW_NCOH && cix >= 0) {
                cd = sqrt(pw55_lds(cx[lane]));
                const double s = sqrt(pw55_lds(cw[lane]));
                cwd = s * s;
                cl = lane;
            }
            double bd = cd;
            long long bl = cl;
            for (int o = 32; o > 0; o >>= 1) {
                const double od = __shfl_xor(bd, o);
                const long long ol = __shfl_xor(bl, o);
                fin_best(bd, bl, od, ol);
            }
            const int win = bl == LLONG_MAX ? 0 : (int)bl;
            const long long wix = ccix[win];
            const int wr = cpos[win][0], wc = cpos[win][1], wim = cpos[win][2];
            const double wd = __shfl(cwd, win), wval = __shfl(cvl, win);
            wstamp(15);
            if (lane == 0) {
                cs = bl == LLONG_MAX ? CohSel{0, 0, 0, 0, 0, 0, 0, 0.0}
                                     : CohSel{wix, wr, wc, wim, y - 2 + win / 5, x - 2 + win % 5, 1, wd};
                csval = wval;
            }
        }
        stamp(5);
        if (wv == 2) wstamp(14);
        b = xrec_wave_min(b);
        if (lane == 0) wbest[wv] = b;
        __syncthreads();
        stamp(6);
        if (wv != 0) return;

        // ---- 4. this rank's winner; sharded DB: publish it, collect every rank's
        XRec lb = wbest[0];
#pragma unroll
        for (int w = 1; w < 4; ++w) xrec_take(lb, wbest[w]);
        XRec gb = lb;
        unsigned long long waited = 0;
        if (f.px.nranks > 0) {
            peer_publish_rec(f.px, i, lb, lane);
            const unsigned long long w0 = __builtin_amdgcn_s_memrealtime();
            if (!peer_collect_rec(f.px, i, lane, gb)) gb = lb;
            waited = __builtin_amdgcn_s_memrealtime() - w0;
        }
        stamp(7);
        if (a.stats && lane == 0) {
            unsigned long long *sl = stats_slot(a.stats, i);
            atomicAdd(&sl[0], (unsigned long long)nresc);
            atomicAdd(&sl[1], (unsigned long long)ns);
            atomicAdd(&sl[2], full ? 1ULL : 0ULL);
            atomicAdd(&sl[3], waited);
        }
        // ---- kappa test and update (image_analogies.py:200-220; finish_apply's rules)
        const CohSel c = cs;
        const long long app = (gb.i < 0 || gb.i >= f.N_total) ? 0 : gb.i;
        int im0, ar, ac;
        row_pos(app, src.hw, src.A.w, im0, ar, ac);
        long img = im0;
        int pr = ar, pc = ac;
        double val = gb.val;
        if (c.valid && c.dcoh <= gb.wd * f.kappa_factor) {
            pr = c.wr; pc = c.wc; img = c.wim;
            val = csval;
        }
        own = val;
        if (lane == 0) {
            const long q = (long)y * W + x;
            if (f.dbg_px) {
                int32_t *o = f.dbg_px + 7 * q;
                o[0] = ar; o[1] = ac;
                o[2] = c.valid ? c.wr : 0;
                o[3] = c.valid ? c.wc : 0;
                o[4] = c.valid ? c.rr : 0;
                o[5] = c.valid ? c.rc : 0;
                o[6] = c.valid;
                f.dbg_dist[2 * q] = c.valid ? gb.wd : 0.0;
                f.dbg_dist[2 * q + 1] = c.valid ? c.dcoh : 0.0;
            }
            f.Bp_lg[q] = val;
            f.s[2 * q] = pr;
            f.s[2 * q + 1] = pc;
            f.im[q] = (int32_t)img;
            // the decision for the lower neighbour's next query (step 5)
            const unsigned long long bits = (unsigned long long)__double_as_longlong(val);
            unsigned long long *d = a.dbox + 2 * (long)y;
            __hip_atomic_store(d, dgran(t + 1, (unsigned int)bits), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(d + 1, dgran(t + 1, (unsigned int)(bits >> 32)), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    stamp(8);
    if (wv != 0 || !nxt) return;

    // ---- 5. the query row of (y, x + 1) for wave t + 1 (k_query_wave's arithmetic)
    const int dep = pdep;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the prefetched words have landed
    wave_lds_sync();
    const double pv = lane < IA_D ? lds_f64(nxw[0], nxw[1], lane) : 0.0;
    const double pc0 = lane < IA_D ? lds_f64(nxw[2], nxw[3], lane) : 0.0;
    double nb = 0.0;
    if (__any(dep == 2)) {   // the upper neighbour (ticket i - 1) decided (y - 1, x + 3)
        const unsigned long long *d = a.dbox + 2 * (long)(y - 1);
        unsigned long long g0 = 0, g1 = 0;
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        auto waited = [&]() {
            if (a.stats && lane == 0)
                atomicAdd(&stats_slot(a.stats, i)[4], __builtin_amdgcn_s_memrealtime() - t0);
        };
        for (;;) {
            g0 = __hip_atomic_load(d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            g1 = __hip_atomic_load(d + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if ((unsigned)(g0 >> 32) == (unsigned)(t + 1) && (unsigned)(g1 >> 32) == (unsigned)(t + 1)) break;
            if (__builtin_amdgcn_s_memrealtime() - t0 > PEER_TIMEOUT_TICKS) {
                if (lane == 0) atomicOr(a.err, 1u);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        waited();
        nb = __longlong_as_double((long long)(((g1 & 0xffffffffULL) << 32) | (g0 & 0xffffffffULL)));
    }
    stamp(9);
    const double vq = dep == 1 ? own : (dep == 2 ? nb : pv);
    const double ncen = pc0;
    const int m = y - a.y_lo_n;
    double d = 0.0;
    if (lane < IA_D) {
        a.q64n[(long)m * IA_DP + lane] = vq;
        d = vq - ncen;
        a.qpn[(long)m * IA_DP + perm56(lane)] = -2.0f * (float)d;
    } else if (lane == IA_D) {
        a.q64n[(long)m * IA_DP + IA_D] = 0.0;
        a.qpn[(long)m * IA_DP + perm56(IA_D)] = 1.0f;
    }
    double d2 = d * d;
    for (int o = 32; o > 0; o >>= 1) d2 += __shfl_xor(d2, o);   // same sum in every lane
    if (lane == 0) a.nqn[m] = d2;
    split16_write_query(a.q16n + (long)m * Q16_ROW * 8, lane, d, d2, amx);
    stamp(10);
}

int launch_xwave(const XArgs &a, int nblocks, bool img, hipStream_t st, int njobs) {
    if (nblocks <= 0) return IA_OK;
    IA_ARG(njobs >= 1 && njobs <= IA_BATCH_MAX && (njobs == 1 || a.jobs), "launch_xwave: bad batch");
    const dim3 grid((unsigned)nblocks, (unsigned)njobs);
    if (njobs > 1) {
        if (img) k_xwave<true, true><<<grid, 256, 0, st>>>(a);
        else k_xwave<false, true><<<grid, 256, 0, st>>>(a);
    } else {
        if (img) k_xwave<true, false><<<grid, 256, 0, st>>>(a);
        else k_xwave<false, false><<<grid, 256, 0, st>>>(a);
    }
    IA_LAUNCH_CHECK("k_xwave");
    return IA_OK;
}

}  // namespace ia
