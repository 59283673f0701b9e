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
#include "ia_rot16.h"
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
// feat_addr for a pair whose two images share their dimensions (A and an A' image: the
// exact stage's rows and the coherence candidates), from VALUES: the base pointers and the
// fine / coarse dimensions arrive as uniform scalars, so the per-lane choice is a select of
// registers.  (feat_addr's per-lane choice between two fields of the argument structs
// compiled to per-lane loads from the kernel-argument memory and a vmcnt(0) wait, which also
// waited for every copy the wave had in flight: ~1 us before wave 1's first coherence copy)
__device__ __forceinline__ const double *feat_addr_v(const double *xs, const double *xl, const double *ys,
                                                     const double *yl, int h, int w, int hs, int ws, int r,
                                                     int c, int k, int &rr, int &cc) {
    const bool yk = k >= 34;
    const int kk = yk ? k - 34 : k;
    const bool coarse = kk < 9;
    const int t = coarse ? kk : kk - 9;
    const int hh = coarse ? hs : h, ww = coarse ? ws : w;
    const double *base = yk ? (coarse ? ys : yl) : (coarse ? xs : xl);
    const int r0 = coarse ? (r >> 1) + t / 3 - 1 : r + t / 5 - 2;
    const int c0 = coarse ? (c >> 1) + t % 3 - 1 : c + t % 5 - 2;
    rr = symi2(r0, hh);
    cc = symi2(c0, ww);
    return base + (long)rr * ww + cc;
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
// s_waitcnt vmcnt(0) before reading the words).  lo / hi must be wave-uniform.  Every lane
// copies (p must be valid in every lane; `on` only documents which words are used): a copy
// inside a divergent branch makes the join wait for it, so each copy would cost a round trip
__device__ __forceinline__ void dma_f64(const double *p, bool on, unsigned *lo, unsigned *hi) {
    (void)on;
    __builtin_amdgcn_global_load_lds((const void *)p, (void *)lo, 4, 0, 0);
    __builtin_amdgcn_global_load_lds((const void *)(reinterpret_cast<const char *>(p) + 4), (void *)hi, 4, 0, 0);
}
__device__ __forceinline__ double lds_f64(const unsigned *lo, const unsigned *hi, int l) {
    return __longlong_as_double((long long)(((unsigned long long)hi[l] << 32) | lo[l]));
}

// lexicographic (d, i) minimum over the 16 lanes of each row by DPP row rotations (8, 4, 2, 1):
// every lane of a row ends with its row's minimum (fin_best's order: the lowest i on ties)
__device__ __forceinline__ void rowmin16_lex(double &bd, long long &bl) {
    auto step = [&](auto ctrl) {
        constexpr int C = decltype(ctrl)::value;
        const long long db = __double_as_longlong(bd);
        const int dlo = __builtin_amdgcn_update_dpp((int)db, (int)db, C, 0xf, 0xf, false);
        const int dhi = __builtin_amdgcn_update_dpp((int)(db >> 32), (int)(db >> 32), C, 0xf, 0xf, false);
        const int ilo = __builtin_amdgcn_update_dpp((int)bl, (int)bl, C, 0xf, 0xf, false);
        const int ihi = __builtin_amdgcn_update_dpp((int)(bl >> 32), (int)(bl >> 32), C, 0xf, 0xf, false);
        const double od = __longlong_as_double((long long)(((unsigned long long)(unsigned)dhi << 32) | (unsigned)dlo));
        const long long ol = (long long)(((unsigned long long)(unsigned)ihi << 32) | (unsigned)ilo);
        fin_best(bd, bl, od, ol);
    };
    step(std::integral_constant<int, 0x128>{});   // row_ror:8
    step(std::integral_constant<int, 0x124>{});   // row_ror:4
    step(std::integral_constant<int, 0x122>{});   // row_ror:2
    step(std::integral_constant<int, 0x121>{});   // row_ror:1
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
    a.rot = J.rot;
    a.askc = J.askc;
}

// a workgroup barrier that orders LDS only: __syncthreads() also waits for every global load
// the wave has in flight (its release fence), which would make a barrier wait for a wave's
// prefetches
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// ---- the wave's tail, shared by k_xwave and k_xstrip ------------------------------------
// phase stamp k of a traced pixel (thread 0)
__device__ __forceinline__ void xw_stamp(unsigned long long *trace, int k) {
    if (trace && threadIdx.x == 0) trace[k] = __builtin_amdgcn_s_memrealtime();
}

// step 4 (wave 0, every lane): lb is this rank's winner for pixel (y, x) (ticket i); a
// sharded DB publishes it and collects every rank's; then the kappa test against the
// coherence pick c (A' value cval) and the B'/s/im (+ debug) update, and the decision
// granules for the lower neighbour's next query.  Returns the pixel's new B' value.
__device__ __forceinline__ double xw_finish(const XArgs &a, int i, int y, int x, int lane, const XRec &lb,
                                            const CohSel &c, double cval, unsigned int nresc, int ns,
                                            bool full, unsigned long long *trace) {
    const FinishArgs &f = a.f;
    const DbSrc &src = a.src;
    const int t = f.t, W = f.W;
    XRec gb = lb;
    unsigned long long waited = 0;
    if (f.px.nranks > 0) {
        peer_publish_rec(f.px, i, lb, lane);
        const unsigned long long w0 = __builtin_amdgcn_s_memrealtime();
        if (!peer_collect_rec(f.px, i, lane, gb)) gb = lb;
        waited = __builtin_amdgcn_s_memrealtime() - w0;
    }
    xw_stamp(trace, 7);
    if (a.stats && lane == 0) {
        unsigned long long *sl = stats_slot(a.stats, i);
        atomicAdd(&sl[0], (unsigned long long)nresc);
        atomicAdd(&sl[1], (unsigned long long)ns);
        atomicAdd(&sl[2], full ? 1ULL : 0ULL);
        atomicAdd(&sl[3], waited);
    }
    // ---- kappa test and update (image_analogies.py:200-220; finish_apply's rules)
    const long long app = (gb.i < 0 || gb.i >= f.N_total) ? 0 : gb.i;
    int im0, ar, ac;
    row_pos(app, src.hw, src.A.w, im0, ar, ac);
    long img = im0;
    int pr = ar, pc = ac;
    double val = gb.val;
    if (c.valid && c.dcoh <= gb.wd * f.kappa_factor) {
        pr = c.wr; pc = c.wc; img = c.wim;
        val = cval;
    }
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
    return val;
}

// step 5 (wave 0): the query row of (y, x + 1) for wave t + 1 (k_query_wave's arithmetic):
// the prefetched features (nxw, LDS-DMA words), this pixel's new value own (dep 1) or the
// upper neighbour's decision (dep 2, ticket i - 1 of this launch)
// rotl (nullable): an R16 level's rotation in LDS (k_xstrip<.., true>): the query row in the
// R16 layout (ia_rot16.h) and q64 slot 55 = |kappa_skip|^2; dq: 64 doubles of LDS scratch
__device__ __forceinline__ void xw_next_query(const XArgs &a, int i, int y, int x, int lane, int dep, double own,
                                              float amx, const unsigned (*nxw)[64],
                                              unsigned long long *trace, const float *rotl = nullptr,
                                              double *dq = nullptr) {
    const int t = a.f.t;
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
    xw_stamp(trace, 9);
    const double vq = dep == 1 ? own : (dep == 2 ? nb : pv);
    const double ncen = pc0;
    const int m = y - a.y_lo_n;
    double d = 0.0;
    if (lane < IA_D) {
        a.q64n[(long)m * IA_DP + lane] = vq;
        d = vq - ncen;
        a.qpn[(long)m * IA_DP + perm56(lane)] = -2.0f * (float)d;
    } else if (lane == IA_D) {
        if (!rotl) a.q64n[(long)m * IA_DP + IA_D] = 0.0;
        a.qpn[(long)m * IA_DP + perm56(IA_D)] = 1.0f;
    }
    double d2 = d * d;
    for (int o = 32; o > 0; o >>= 1) d2 += __shfl_xor(d2, o);   // same sum in every lane
    if (lane == 0) a.nqn[m] = d2;
    if (rotl) {
        const double s2 = r16_write_query(a.q16n + (long)m * Q16_ROW * 8, lane, d, d2, amx, rotl, dq);
        if (lane == 0) a.q64n[(long)m * IA_DP + IA_D] = s2;
    } else {
        split16_write_query(a.q16n + (long)m * Q16_ROW * 8, lane, d, d2, amx);
    }
    xw_stamp(trace, 10);
}

// BATCH: a0.jobs holds a batch's pointers; the block copies the launch arguments into LDS
// once and overrides them with its job's (a private copy of the arguments would live in
// scratch memory), then reads them from there
#ifndef IA_XWAVE_OCC
#define IA_XWAVE_OCC 2   // workgroups per CU k_xwave is built for (3: 168 VGPRs and 240-448 B of spills, c1 +8 %, c3 +11 %)
#endif
template <bool IMG, bool BATCH>
__global__ __launch_bounds__(256, IA_XWAVE_OCC) void k_xwave(XArgs a0) {
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
    // (rows of IA_DP + 1 doubles: lane c's pairwise sum over cx[c] then hits distinct banks)
    __shared__ double cx[XW_NCOH][IA_DP + 1], cw[XW_NCOH][IA_DP + 1];
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
    // an R16 level (a.rot): wave 0 copies the rotation into the pool once the exact stage is
    // done with it, for the next query row (as k_xstrip), 64 doubles of scratch after it
    static_assert(R16_ROT_B + 64 * 8 <= (POOL > RESB ? POOL : RESB), "the rotation fits the pool");
    float *const rotl = reinterpret_cast<float *>(pool);
    double *const dq = reinterpret_cast<double *>(pool + R16_ROT_B);
    auto rot_dma = [&]() {   // wave 0: 13 x 1 KiB, waited in xw_next_query (vmcnt(0))
#pragma unroll
        for (int pc = 0; pc < R16_ROT_FLOATS / 256; ++pc)
            __builtin_amdgcn_global_load_lds((const void *)(a.rot.get() + pc * 256 + lane * 4),
                                             (void *)(rotl + pc * 256), 16, 0, 0);
    };
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
        // (B and B' share their dimensions: feat_addr_v, no argument loads before the copies)
        const double *p = feat_addr_v(a.B.sm, a.B.lg, a.Bp.sm, a.Bp.lg, a.B.h, a.B.w, a.B.hs, a.B.ws, y, x + 1,
                                      lane < IA_D ? lane : 0, rr, cc);
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
        const double nskq = a.rot ? a.q64[(long)i * IA_DP + IA_D] : 0.0;
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
        // an R16 level (a.rot): the screen's bound eps_R (|kappa_skip|^2 in q64 slot 55)
        if (a.rot) r16_thresholds_rows(emin, am, a.amax[vidx(1)], nqq, nskq, Tseg, Trow, force_full);
        else rescore_thresholds(emin, am, nqq, Tseg, Trow, force_full);
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
        // cm: the candidates whose features are copied and scored.  The row form skips the
        // invalid ones and every repeat of an earlier candidate (same A' pixel: the same
        // distance at a higher index, never the first minimum; c5's finest level: 5.5 distinct
        // of 11.9 valid per pixel); the window form copies all 15 (its vmcnt count is fixed)
        unsigned cm = (1u << XW_NCOH) - 1;
        int c_r = 0, c_c = 0, c_i = 0;   // wave 1, lane c: candidate c's A' row, column, image
        // wave 1: the candidates' A' values and all their features requested at once by LDS
        // DMA (candidate c's lo / hi words in cx / cw); the window form: EXACTLY XW_COH_DMA
        // copies, none skipped, so that a window copied in before them is waited for with
        // vmcnt (loads return in order)
        auto coh_issue = [&]() {
            const long long cl = lane < XW_NCOH ? ccix[lane] : -1;
            dma_f64(src.Ap.lg + (cl >= 0 ? cl : 0), true, cvw[0], cvw[1]);
            unsigned *clo = reinterpret_cast<unsigned *>(&cx[0][0]);
            unsigned *chi = reinterpret_cast<unsigned *>(&cw[0][0]);
            // (the positions broadcast from wave 1's registers: no LDS round trip per candidate;
            // the images' bases and dimensions as scalars: feat_addr_v)
            const double *As = src.A.sm, *Al = src.A.lg, *Ps = src.Ap.sm, *Pl = src.Ap.lg;
            const int fh = src.A.h, fw = src.A.w, chh = src.A.hs, cww = src.A.ws;
            const long hws = src.hws, hw = src.hw;
#pragma unroll 1
            for (unsigned m = cm; m; m &= m - 1) {
                const int c = __builtin_ctz(m);
                const int pr = __builtin_amdgcn_readlane(c_r, c), pc = __builtin_amdgcn_readlane(c_c, c);
                const int pi = __builtin_amdgcn_readlane(c_i, c);
                int rr, cc;
                const double *fp = feat_addr_v(As, Al, Ps + (long)pi * hws, Pl + (long)pi * hw, fh, fw, chh, cww,
                                               pr, pc, lane < IA_D ? lane : 0, rr, cc);
                dma_f64(fp, true, clo + c * 64, chi + c * 64);
            }
            wstamp(13);
        };

        if (wv == 1) {
            long long mine = -1;
            if (lane < XW_NCOH) {
                const int sr = s_r + y - rr0, sc = s_c + x - rc0;
                const bool ok = cpos_ok && sr >= 0 && sr < src.A.h && sc >= 0 && sc < src.A.w;
                mine = ok ? ((long)src.A.h * s_i + sr) * src.A.w + sc : -1;
                ccix[lane] = mine;
                c_r = ok ? sr : 0; c_c = ok ? sc : 0; c_i = ok ? s_i : 0;
                cpos[lane][0] = c_r; cpos[lane][1] = c_c; cpos[lane][2] = c_i;
            }
            if constexpr (!IMG) {
                // (lane j's value by readlane: a scalar broadcast, not an LDS round trip)
                bool keep = mine >= 0;
                const int mlo = (int)mine, mhi = (int)(mine >> 32);
#pragma unroll
                for (int j = 0; j < XW_NCOH - 1; ++j) {
                    const long long o = (long long)(((unsigned long long)(unsigned)__builtin_amdgcn_readlane(mhi, j) << 32) |
                                                    (unsigned)__builtin_amdgcn_readlane(mlo, j));
                    keep = keep && !(j < lane && o == mine);
                }
                cm = (unsigned)__builtin_amdgcn_readfirstlane((unsigned)__ballot(keep && lane < XW_NCOH));
            }
            wave_lds_sync();
        }
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
                load_row16(reinterpret_cast<const half8 *>(a.db.get()), lr < a.nrows ? lr : 0, g0, g1);
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
                    int r2, c2;
                    const double *fp = feat_addr_v(src.A.sm, src.A.lg, src.Ap.sm + (long)ri * src.hws,
                                                   src.Ap.lg + (long)ri * src.hw, src.A.h, src.A.w, src.A.hs,
                                                   src.A.ws, rr, rc, lane < IA_D ? lane : 0, r2, c2);
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
            const long long cix = lane < XW_NCOH && ((cm >> lane) & 1u) ? ccix[lane] : -1;
            const double cvl = cix >= 0 ? lds_f64(cvw[0], cvw[1], lane) : 0.0;
            const double ql = lane < IA_D ? qs[lane] : 0.0, wl = lane < IA_D ? wts[lane] : 0.0;
            const unsigned *clo = reinterpret_cast<const unsigned *>(&cx[0][0]);
            const unsigned *chi = reinterpret_cast<const unsigned *>(&cw[0][0]);
            // (four candidates per LDS round trip, highest first: a chunk's squares only cover
            // words of candidates it or an earlier chunk has read)
#pragma unroll 1
            for (unsigned rem = cm; rem;) {
                int ci[4];
                double gv[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    ci[u] = -1;
                    gv[u] = 0.0;
                    if (rem) {
                        const int c = 31 - __builtin_clz(rem);
                        rem &= ~(1u << c);
                        ci[u] = c;
                        gv[u] = lds_f64(clo + c * 64, chi + c * 64, lane);
                    }
                }
                wave_lds_sync();   // every lane has the chunk's words
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    if (ci[u] >= 0 && lane < IA_D) {
                        const double xx = gv[u] - ql;
                        const double xw = xx * wl;
                        cx[ci[u]][lane] = xx * xx;
                        cw[ci[u]][lane] = xw * xw;
                    }
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
            // the first minimum over lanes 0..14 (row 0 of the wave): DPP rotations within the
            // row (no LDS round trip per step); every lane of row 0 ends with it
            double bd = cd;
            long long bl = cl;
            rowmin16_lex(bd, bl);
            bl = (long long)(((unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)(bl >> 32), 0) << 32) |
                             (unsigned)__builtin_amdgcn_readlane((int)bl, 0));
            const int win = bl == LLONG_MAX ? 0 : (int)bl;
            const long long wix = ccix[win];
            const int wr = cpos[win][0], wc = cpos[win][1], wim = cpos[win][2];
            auto lane_f64 = [&](double v) {   // v of lane win (uniform)
                const long long b = __double_as_longlong(v);
                return __longlong_as_double((long long)(((unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)(b >> 32), win) << 32) |
                                                        (unsigned)__builtin_amdgcn_readlane((int)b, win)));
            };
            const double wd = lane_f64(cwd), wval = lane_f64(cvl);
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
        if (a.rot && nxt) rot_dma();   // the pool is free: the rotation lands meanwhile

        // ---- 4. this rank's winner; sharded DB: publish it, collect every rank's; tail
        XRec lb = wbest[0];
#pragma unroll
        for (int w = 1; w < 4; ++w) xrec_take(lb, wbest[w]);
        own = xw_finish(a, i, y, x, lane, lb, cs, csval, nresc, ns, full, trace);
    }
    stamp(8);
    if (wv != 0 || !nxt) return;
    if (a.rot && !cur) rot_dma();   // (a pixel of wave t + 1 only: the pool was never used)
    // ---- 5. the query row of (y, x + 1) for wave t + 1 (an R16 level: the rotated row, the
    // rotation staged in the pool)
    xw_next_query(a, i, y, x, lane, pdep, own, amx, nxw, trace, a.rot ? rotl : nullptr, a.rot ? dq : nullptr);
}

// ---- strip-order image-form levels: the exact stage from fp64 windows (k_xstrip) ---------
// A candidate segment of a strip-order level (StageMap W > 0, ia_internal.h) is nst =
// seg_rows / 128 consecutive scanlines y0 .. y0 + nst - 1 of one 128-pixel column strip
// [x0, x0 + 128) of one A' image.  Every fp64 sample its rows' features read
// (algorithms.py:11-47) lies in four windows of the level's pyramids, held in LDS as the
// REFLECTED images (symi2 applied when they are filled), so that pixel (y, x)'s 55 samples
// sit at compile-time offsets from two per-pixel bases:
//   A fine    rows y0 - 2 .. y0 + 5, cols x0 - 4 .. x0 + 131   (8 x 136)
//   A' fine   rows y0 - 2 .. y0 + 3, the same cols             (6 x 136)
//   A, A' coarse rows y0/2 - 1 .. y0/2 + 2, cols x0/2 - 2 .. x0/2 + 65   (4 x 68 each)
// 19.6 KB, copied by DMA as 16-B pieces in ONE round trip; a piece with a column outside
// the image (strips at the image's left / right edge) is copied from a clamped address and
// rewritten by its own thread, after the wait, with its two reflected values (loaded in the
// same round trip).  Every row of the segment is then rescored in fp64 from LDS in the
// oracle's operation order (row_dist2), two rows per thread: no fp32 re-screen and no
// per-row gathers.  The exact minimum over every row of the candidate segments is the
// oracle's winner (the segments hold every row whose screen value is within Tseg, DESIGN.md
// §4b).  The winner's weighted distance and A' value come from the same windows; the
// coherence pick (wave 1) computes from its own LDS-DMA gathers while the first windows are
// in flight.
constexpr int XS_FW = 136, XS_CW = 68;                       // window columns (doubles)
constexpr int XS_FA = 0, XS_FP = XS_FA + 8 * XS_FW;          // window offsets (doubles)
constexpr int XS_CA = XS_FP + 6 * XS_FW, XS_CP = XS_CA + 4 * XS_CW;
constexpr int XS_DBL = XS_CP + 4 * XS_CW;                    // 2448 doubles, 19584 B
constexpr int XS_PIECES = XS_DBL / 2;                        // 16-B pieces
constexpr int XS_DMA = (XS_PIECES + 191) / 192;              // 7 copies per thread of waves 0, 2, 3
constexpr int XS_LDS_B = XS_DMA * 192 * 16;                  // 21504 B (the tail: dummy copies)
constexpr int XS_CST = 65;                                   // coherence samples per candidate (banks)

bool xstrip_applies(const DbSrc &src) {
    return src.A.w >= 128 && src.A.w % 2 == 0 && src.A.ws * 2 == src.A.w && src.A.h >= 1 && src.A.hs >= 1;
}

struct XsWin {
    const double *fa, *fp, *ca, *cp;   // A and the segment's A' image, fine and coarse
    long g0;                           // global row of the segment's first pixel (y0, x0)
    int y0, x0, nst;
};
__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }
__device__ __forceinline__ XsWin xs_window(const XArgs &a, long seg) {
    const DbSrc &src = a.src;
    XsWin w;
    w.g0 = a.row0 + seg_lrow(a.smap, seg, a.seg_rows, 0);
    int img;
    row_pos(w.g0, src.hw, src.A.w, img, w.y0, w.x0);
    w.nst = a.seg_rows >> 7;
    w.fa = src.A.lg;
    w.ca = src.A.sm;
    w.fp = src.Ap.lg + (long)img * src.hw;
    w.cp = src.Ap.sm + (long)img * src.hws;
    return w;
}
// window bases of pixel (y, x) (fine, coarse); its feature k sits at base + xs_koff(k)
__device__ __forceinline__ int xs_fbase(const XsWin &w, int y, int x) { return (y - w.y0 + 2) * XS_FW + (x - w.x0 + 4); }
__device__ __forceinline__ int xs_cbase(const XsWin &w, int y, int x) {
    return ((y >> 1) - (w.y0 >> 1) + 1) * XS_CW + ((x >> 1) - (w.x0 >> 1) + 2);
}
__host__ __device__ constexpr bool xs_coarse(int k) { return k < 9 || (k >= 34 && k < 43); }
__host__ __device__ constexpr int xs_koff(int k) {
    return k < 9 ? XS_CA + (k / 3 - 1) * XS_CW + (k % 3 - 1)
         : k < 34 ? XS_FA + ((k - 9) / 5 - 2) * XS_FW + ((k - 9) % 5 - 2)
         : k < 43 ? XS_CP + ((k - 34) / 3 - 1) * XS_CW + ((k - 34) % 3 - 1)
         : XS_FP + ((k - 43) / 5 - 2) * XS_FW + ((k - 43) % 5 - 2);
}

// thread t = 64 r + lane of DMA wave r (waves 0, 2, 3: wave 1 computes the coherence pick
// meanwhile) copies pieces p = 192 j + t to byte 16 p of win: the source row of
// window row r (reflected; rows no pixel of a shorter segment reads are clamped to one that
// exists) and the piece's first column C (clamped for the copy; edge pieces also load their
// two reflected values into fx for xs_fix)
struct XsFix {
    double v[XS_DMA][2];
    unsigned mask;
};
// piece p's source: its (reflected) image row, first column C (maybe outside the image) and
// the image width
__device__ __forceinline__ const double *xs_piece(const XsWin &w, const ImgPair &A, int p, int &C, int &iw) {
    constexpr int FP = XS_FW / 2, CP = XS_CW / 2;   // pieces per window row
    const double *img = w.fa;
    int sr = 0;
    iw = A.w;
    C = 0;
    if (p < 8 * FP) {
        const int r = p / FP;
        sr = symi2(min(w.y0 - 2 + r, w.y0 + w.nst + 1), A.h);
        C = w.x0 - 4 + 2 * (p - r * FP);
    } else if ((p -= 8 * FP) < 6 * FP) {
        const int r = p / FP;
        img = w.fp;
        sr = symi2(min(w.y0 - 2 + r, w.y0 + w.nst - 1), A.h);
        C = w.x0 - 4 + 2 * (p - r * FP);
    } else if ((p -= 6 * FP) < 8 * CP) {
        const int r = p / CP;
        img = r < 4 ? w.ca : w.cp;
        iw = A.ws;
        sr = symi2(min((w.y0 >> 1) - 1 + (r & 3), ((w.y0 + w.nst - 1) >> 1) + 1), A.hs);
        C = (w.x0 >> 1) - 2 + 2 * (p - r * CP);
    }
    return img + (long)sr * iw;
}
__device__ __forceinline__ void xs_dma(const XsWin &w, const ImgPair &A, char *win, int dr, int lane, XsFix &fx) {
    asm volatile("" : "+v"(lane));   // the piece addresses are computed here, not hoisted
    fx.mask = 0;
#pragma unroll
    for (int j = 0; j < XS_DMA; ++j) {
        const int p = 192 * j + 64 * dr + lane;
        int C, iw;
        const double *row = xs_piece(w, A, p, C, iw);
        __builtin_amdgcn_global_load_lds((const void *)(row + clampi(C, 0, iw - 2)),
                                         (void *)(win + (192 * j + 64 * dr) * 16), 16, 0, 0);
        if (C < 0 || C + 1 >= iw) {
            fx.mask |= 1u << j;
            fx.v[j][0] = row[symi2(clampi(C, -2, iw + 1), iw)];
            fx.v[j][1] = row[symi2(clampi(C + 1, -2, iw + 1), iw)];
        }
    }
}
// the next candidate segment's windows staged in registers while the current one is
// rescored (all 256 threads, pieces 256 j + tid: two reflected 8-B loads each, issued
// unconditionally), stored into the windows after the last reads of the current one
constexpr int XS_PRE = (XS_PIECES + 255) / 256;   // 5
struct XsPre {
    double v[XS_PRE][2];
};
__device__ __forceinline__ void xs_pre_load(const XsWin &w, const ImgPair &A, int tid, XsPre &pr) {
#pragma unroll
    for (int j = 0; j < XS_PRE; ++j) {
        const int p = 256 * j + tid;
        int C, iw;
        const double *row = xs_piece(w, A, p < XS_PIECES ? p : XS_PIECES - 1, C, iw);
        pr.v[j][0] = row[symi2(clampi(C, -2, iw + 1), iw)];
        pr.v[j][1] = row[symi2(clampi(C + 1, -2, iw + 1), iw)];
    }
}
__device__ __forceinline__ void xs_pre_store(const XsPre &pr, char *win, int tid) {
#pragma unroll
    for (int j = 0; j < XS_PRE; ++j) {
        const int p = 256 * j + tid;
        if (p < XS_PIECES) {
            double *d = reinterpret_cast<double *>(win + p * 16);
            d[0] = pr.v[j][0];
            d[1] = pr.v[j][1];
        }
    }
}
// after this thread's copies landed: its edge pieces get their reflected values
__device__ __forceinline__ void xs_fix(const XsFix &fx, char *win, int t) {
#pragma unroll
    for (int j = 0; j < XS_DMA; ++j)
        if (fx.mask & (1u << j)) {
            double *d = reinterpret_cast<double *>(win + (192 * j + t) * 16);
            d[0] = fx.v[j][0];
            d[1] = fx.v[j][1];
        }
}
template <int K0, int K1, typename F>
__device__ __forceinline__ void xs_for(F &&f) {
    if constexpr (K0 < K1) {
        f(std::integral_constant<int, K0>{});
        xs_for<K0 + 1, K1>(f);
    }
}
// row_dist2 of two pixels (window bases f*, c*) from the windows: numpy's pairwise order,
// the query from LDS; groups of 11 features in flight (z carried through asm: every load
// of a group follows the previous group's)
__device__ __forceinline__ void xs_dist2(const double *win, int f0, int c0, int f1, int c1, const double *qs,
                                         double &d0, double &d1) {
    Pw55 a, b;
    // the bases pass through asm (integers: the LDS address space stays known), so no
    // address is hoisted out of the caller's loop
    asm volatile("" : "+v"(f0), "+v"(c0), "+v"(f1), "+v"(c1));
    xs_for<0, IA_D>([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        constexpr int o = xs_koff(k);
        const int b0 = xs_coarse(k) ? c0 : f0, b1 = xs_coarse(k) ? c1 : f1;
        const double q = qs[k];
        const double x0 = win[b0 + o] - q, x1 = win[b1 + o] - q;
        a.feed(k, x0 * x0);
        b.feed(k, x1 * x1);
    });
    d0 = a.res;
    d1 = b.res;
    // the sums are finished HERE: sunk past the caller's barrier, every loaded value would
    // stay live across it (the next window's copies overwrite the LDS they came from)
    asm volatile("" :: "v"(d0), "v"(d1));
}

// row_dist2 of the vertically adjacent pixels (y, x) and (y + 1, x), y - y0 even (window bases
// fb, cb of (y, x)): the coarse samples of both are the same (y / 2 == (y + 1) / 2) and
// pixel (y + 1)'s fine rows are pixel y's shifted by one, so the shared loads are done once
// (65 window loads for the two rows instead of 110)
__device__ __forceinline__ void xs_dist_pair(const double *win, int fb, int cb, const double *qs,
                                             double &d0, double &d1) {
    Pw55 a, b;
    asm volatile("" : "+v"(fb), "+v"(cb));
    xs_for<0, IA_D>([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        constexpr int o = xs_koff(k);
        const double q = qs[k];
        if constexpr (xs_coarse(k)) {
            const double x = win[cb + o] - q;
            a.feed(k, x * x);
            b.feed(k, x * x);
        } else {
            const double x0 = win[fb + o] - q, x1 = win[fb + XS_FW + o] - q;
            a.feed(k, x0 * x0);
            b.feed(k, x1 * x1);
        }
    });
    d0 = a.res;
    d1 = b.res;
    asm volatile("" :: "v"(d0), "v"(d1));   // finished here (as xs_dist2)
}

// numpy's pairwise sum (Pw55's order) of term k held by lane k (k < 55), every lane
__device__ __forceinline__ double pw55_lanes(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = (int)b, hi = (int)(b >> 32);
    auto at = [&](int k) {
        return __longlong_as_double((long long)(((unsigned long long)(unsigned)__builtin_amdgcn_readlane(hi, k) << 32) |
                                                (unsigned)__builtin_amdgcn_readlane(lo, k)));
    };
    double r[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = at(j);
#pragma unroll
    for (int k = 8; k < 48; k += 8) {
#pragma unroll
        for (int j = 0; j < 8; ++j) r[j] += at(k + j);
    }
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
#pragma unroll
    for (int k = 48; k < IA_D; ++k) res += at(k);
    return res;
}

// ---- k_xstrip's segment-minima phase on waves 0, 2, 3 only (192 threads; wave 1 picks the
// coherence candidate meanwhile and never waits for this phase): thread t3 holds the float4s
// t3 + 192 j of the query's minima in registers (XS_REG of them: c4's 8192 segments on one
// GPU), the rest are streamed.  Same e* and candidate set as segmin_* over 256 threads.
constexpr int XS_REG = 11;
template <int XR>
__device__ __forceinline__ void seg3_load(const float4 *sq4, long n4, int t3, float4 (&v)[XR]) {
#pragma unroll
    for (int j = 0; j < XR; ++j) {
        const long i = t3 + (long)j * 192;
        const float4 x = sq4[i < n4 ? i : 0];   // unconditional (a valid index past the end)
        v[j] = i < n4 ? x : make_float4(FLT_MAX, FLT_MAX, FLT_MAX, FLT_MAX);
    }
}
template <int XR>
__device__ __forceinline__ float seg3_wave_min(const float4 *sq4, long n4, int t3, const float4 (&v)[XR]) {
    float emin = FLT_MAX;
#pragma unroll
    for (int j = 0; j < XR; ++j) emin = fminf(emin, fminf(fminf(v[j].x, v[j].y), fminf(v[j].z, v[j].w)));
    for (long i = t3 + (long)XR * 192; i < n4; i += 192) {
        const float4 x = sq4[i];
        emin = fminf(emin, fminf(fminf(x.x, x.y), fminf(x.z, x.w)));
    }
    for (int o = 32; o > 0; o >>= 1) emin = fminf(emin, __shfl_xor(emin, o));
    return emin;
}
template <int XR>
__device__ __forceinline__ void seg3_select(const float4 *sq4, long n4, int t3, const float4 (&v)[XR],
                                            double Tseg, int *slist, int *scount) {
    static_assert(XR * 4 <= 64, "one 64-bit mask");
    unsigned long long m = 0;
#pragma unroll
    for (int j = 0; j < XR; ++j) {
        m |= (unsigned long long)((double)v[j].x <= Tseg) << (4 * j);
        m |= (unsigned long long)((double)v[j].y <= Tseg) << (4 * j + 1);
        m |= (unsigned long long)((double)v[j].z <= Tseg) << (4 * j + 2);
        m |= (unsigned long long)((double)v[j].w <= Tseg) << (4 * j + 3);
    }
    if (m) {
        int pos = atomicAdd(scount, __builtin_popcountll(m));
        while (m) {
            const int b = __builtin_ctzll(m);
            m &= m - 1;
            if (pos < RESCORE_SEGCAP) slist[pos] = 4 * (t3 + (b >> 2) * 192) + (b & 3);
            ++pos;
        }
    }
    for (long i = t3 + (long)XR * 192; i < n4; i += 192) {
        const float4 x = sq4[i];
        unsigned mt = ((double)x.x <= Tseg ? 1u : 0u) | ((double)x.y <= Tseg ? 2u : 0u) |
                      ((double)x.z <= Tseg ? 4u : 0u) | ((double)x.w <= Tseg ? 8u : 0u);
        if (mt) {
            int pos = atomicAdd(scount, __builtin_popcount(mt));
            while (mt) {
                const int b = __builtin_ctz(mt);
                mt &= mt - 1;
                if (pos < RESCORE_SEGCAP) slist[pos] = (int)(4 * i + b);
                ++pos;
            }
        }
    }
}
// R16 levels: the same phases with the per-segment skip bound (ia_rot16.h r16_kseg): cv[j] holds
// the codes of the 4 segments of v[j] (one byte each, r16_askc); the reduction takes
// min fl32(m + Kf c) and the selection m <= T0 + K c
template <int XR>
__device__ __forceinline__ void seg3_load_codes(const unsigned *ac4, long n4, int t3, unsigned (&cv)[XR]) {
#pragma unroll
    for (int j = 0; j < XR; ++j) {
        const long i = t3 + (long)j * 192;
        cv[j] = ac4[i < n4 ? i : 0];
    }
}
__device__ __forceinline__ float seg_uval(float m, unsigned c, int b, float Kf) {
    return fmaf(Kf, (float)((c >> (8 * b)) & 255u), m);
}
template <int XR>
__device__ __forceinline__ float seg3_wave_umin(const float4 *sq4, const unsigned *ac4, long n4, int t3,
                                                const float4 (&v)[XR], const unsigned (&cv)[XR], float Kf) {
    float u = FLT_MAX;
#pragma unroll
    for (int j = 0; j < XR; ++j)
        u = fminf(u, fminf(fminf(seg_uval(v[j].x, cv[j], 0, Kf), seg_uval(v[j].y, cv[j], 1, Kf)),
                           fminf(seg_uval(v[j].z, cv[j], 2, Kf), seg_uval(v[j].w, cv[j], 3, Kf))));
    for (long i = t3 + (long)XR * 192; i < n4; i += 192) {
        const float4 x = sq4[i];
        const unsigned c = ac4[i];
        u = fminf(u, fminf(fminf(seg_uval(x.x, c, 0, Kf), seg_uval(x.y, c, 1, Kf)),
                           fminf(seg_uval(x.z, c, 2, Kf), seg_uval(x.w, c, 3, Kf))));
    }
    for (int o = 32; o > 0; o >>= 1) u = fminf(u, __shfl_xor(u, o));
    return u;
}
__device__ __forceinline__ unsigned seg_sel4(const float4 &x, unsigned c, double T0, double K) {
    return ((double)x.x <= fma(K, (double)(c & 255u), T0) ? 1u : 0u) |
           ((double)x.y <= fma(K, (double)((c >> 8) & 255u), T0) ? 2u : 0u) |
           ((double)x.z <= fma(K, (double)((c >> 16) & 255u), T0) ? 4u : 0u) |
           ((double)x.w <= fma(K, (double)(c >> 24), T0) ? 8u : 0u);
}
template <int XR>
__device__ __forceinline__ void seg3_select_codes(const float4 *sq4, const unsigned *ac4, long n4, int t3,
                                                  const float4 (&v)[XR], const unsigned (&cv)[XR],
                                                  double T0, double K, int *slist, int *scount) {
    unsigned long long m = 0;
#pragma unroll
    for (int j = 0; j < XR; ++j) m |= (unsigned long long)seg_sel4(v[j], cv[j], T0, K) << (4 * j);
    if (m) {
        int pos = atomicAdd(scount, __builtin_popcountll(m));
        while (m) {
            const int b = __builtin_ctzll(m);
            m &= m - 1;
            if (pos < RESCORE_SEGCAP) slist[pos] = 4 * (t3 + (b >> 2) * 192) + (b & 3);
            ++pos;
        }
    }
    for (long i = t3 + (long)XR * 192; i < n4; i += 192) {
        unsigned mt = seg_sel4(sq4[i], ac4[i], T0, K);
        if (mt) {
            int pos = atomicAdd(scount, __builtin_popcount(mt));
            while (mt) {
                const int b = __builtin_ctz(mt);
                mt &= mt - 1;
                if (pos < RESCORE_SEGCAP) slist[pos] = (int)(4 * i + b);
                ++pos;
            }
        }
    }
}
// a barrier of waves 0, 2 and 3 only (an LDS counter; wave 1 never takes part): generation g
// releases when all three have arrived for the g-th time
__device__ __forceinline__ void sync3(unsigned *cnt, unsigned g, int lane) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (lane == 0) __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < 3u * g)
        __builtin_amdgcn_s_sleep(1);
    asm volatile("" ::: "memory");
}

// ROT: an R16 level (ia_rot16.h): the exact stage's bound eps_R, and the next query row
// rotated (the rotation copied into LDS by wave 0 at the start)
// workgroups per CU the batch form (k_xstrip<true>) is built for (A/B builds)
#ifndef IA_XSTRIP_BOCC
#define IA_XSTRIP_BOCC 4
#endif
#ifndef IA_XSTRIP_BREG
#define IA_XSTRIP_BREG 2   // float4s of segment minima per thread in registers, batch form
#endif
template <bool BATCH, bool ROT>
__global__ __launch_bounds__(256, BATCH ? IA_XSTRIP_BOCC : 3) void k_xstrip(XArgs a0) {
    __shared__ __attribute__((aligned(16))) char sa_raw[BATCH ? sizeof(XArgs) : 16];
    XArgs &sa = *reinterpret_cast<XArgs *>(sa_raw);
    if constexpr (BATCH) {
        const unsigned long long *w0 = reinterpret_cast<const unsigned long long *>(&a0);
        unsigned long long *w1 = reinterpret_cast<unsigned long long *>(&sa);
        for (int w = threadIdx.x; w < (int)(sizeof(XArgs) / 8); w += 256) w1[w] = w0[w];
        __syncthreads();
        if (threadIdx.x == 0) xjob_apply(sa, a0.jobs[blockIdx.y], a0.f.t & 1);
        __syncthreads();
    }
    const XArgs &a = BATCH ? sa : a0;
    __shared__ __attribute__((aligned(16))) char win[XS_LDS_B];
    __shared__ double cxd[XW_NCOH * XS_CST];   // candidate c's samples at c * XS_CST
    __shared__ double cval[XW_NCOH];
    __shared__ double qs[IA_DP], wts[IA_DP];
    __shared__ double cwt[2 * IA_DP];   // the coherence lanes' factors: 1 (distance), weights
    __shared__ int slist[RESCORE_SEGCAP];
    __shared__ int tk, scount, sfull;
    __shared__ unsigned bar3;
    __shared__ float redf[4];
    __shared__ double bds[4], bwd[4], bvl[4];
    __shared__ long long bis[4];
    __shared__ CohSel cs;
    __shared__ double csval;
    __shared__ long long ccix[XW_NCOH];
    __shared__ int cpos[XW_NCOH][3];
    __shared__ unsigned nxw[4][64];
    // ROT: wave 0 copies the rotation into win once the rescore is done with it (no LDS of
    // its own: the fused kernel's LDS decides how many of its workgroups a CU holds beside
    // a screen block), with 64 doubles of scratch after it
    static_assert(R16_ROT_B + 64 * 8 <= XS_LDS_B, "the rotation fits the window buffer");
    float *const rotl = reinterpret_cast<float *>(win);
    double *const dq = reinterpret_cast<double *>(win + R16_ROT_B);

    const int tid = threadIdx.x, lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const FinishArgs &f = a.f;
    const DbSrc &src = a.src;
    const int t = f.t, W = f.W;
    const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
    auto rot_dma = [&]() {   // wave 0: 13 x 1 KiB, waited in xw_next_query (vmcnt(0))
#pragma unroll
        for (int pc = 0; pc < R16_ROT_FLOATS / 256; ++pc)
            __builtin_amdgcn_global_load_lds((const void *)(a.rot.get() + pc * 256 + lane * 4),
                                             (void *)(rotl + pc * 256), 16, 0, 0);
    };
    if (tid == 0) {
        tk = (int)atomicAdd(&a.tickets[t & 1], 1u);
        bar3 = 0;
        scount = 0;
    }
    __syncthreads();
    const int i = tk;
    unsigned long long *trace =
        (a.trace && i < XW_TRACE_PX && t < XW_TRACE_T) ? a.trace + ((long)t * XW_TRACE_PX + i) * XW_TRACE_N : nullptr;
    auto wstamp = [&](int k) {   // lane 0 of any wave
        if (trace && lane == 0) trace[k] = __builtin_amdgcn_s_memrealtime();
    };
    if (trace && tid == 0) trace[0] = t_start;
    xw_stamp(trace, 1);
    if (i == 0 && tid == 0) __hip_atomic_store(&a.tickets[(t + 1) & 1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int y = f.y_lo + i, x = t - 3 * y;
    const bool cur = i < a.M;
    const bool nxt = y >= a.y_lo_n && y < a.y_lo_n + a.M_n;

    // wave 0: the next query's features that do not depend on wave t (as k_xwave)
    const float amx = a.amax[vidx(0)];
    int pdep = 0;
    if (wv == 0 && nxt) {
        int rr = 0, cc = 0;
        // (B and B' share their dimensions: feat_addr_v, no argument loads before the copies)
        const double *p = feat_addr_v(a.B.sm, a.B.lg, a.Bp.sm, a.Bp.lg, a.B.h, a.B.w, a.B.hs, a.B.ws, y, x + 1,
                                      lane < IA_D ? lane : 0, rr, cc);
        pdep = lane < 43 || lane >= IA_D ? 0 : (rr == y && cc == x) ? 1 : (rr == y - 1 && cc == x + 3) ? 2 : 0;
        dma_f64(p, lane < IA_D && pdep == 0, nxw[0], nxw[1]);
        dma_f64(a.center + (lane < IA_D ? lane : 0), lane < IA_D, nxw[2], nxw[3]);
    }

    double own = 0.0;
    if (cur) {
        // ---- 1. one round trip each: waves 0, 2, 3 the query norm, bound and segment minima
        // (e* and the candidate segments among themselves, sync3); wave 1 the query, weights
        // and the coherence window's s / im, then the coherence gathers and pick, without
        // waiting for the others until the first windows have landed
        const int t3 = (wv == 0 ? 0 : wv - 1) * 64 + lane;   // waves 0, 2, 3
        const int ql = lane < IA_DP ? lane : 0;
        const double qsv = a.q64[(long)i * IA_DP + ql];
        const double wk0 = f.weights[lane < IA_D ? lane : 0];
        const double wk = lane < IA_D ? wk0 : 0.0;
        const double nqq = a.nq[vidx(i)];
        const double nsk = ROT ? a.q64[(long)i * IA_DP + IA_D] : 0.0;
        const float am = amx, ask = ROT ? a.amax[vidx(1)] : 0.f;
        const long n4 = a.nseg / 4;
        const float4 *sq4 = reinterpret_cast<const float4 *>(a.segmin + (long)i * a.nseg);
        // (the batch form holds fewer float4s of minima in registers: a c5 job's 512 segments
        // fit in 2 per thread, and the freed VGPRs buy a fourth workgroup per CU)
        constexpr int XR = BATCH ? IA_XSTRIP_BREG : XS_REG;
        float4 v[XR];
        unsigned sgc[XR];
        const unsigned *ac4 = ROT ? reinterpret_cast<const unsigned *>(a.askc.get()) : nullptr;
        if (wv != 1) {
            seg3_load(sq4, n4, t3, v);
            if constexpr (ROT) seg3_load_codes(ac4, n4, t3, sgc);
        }
        const int rr0 = y - 2 + lane / 5, rc0 = x - 2 + lane % 5;
        const bool cpos_ok = wv == 1 && lane < XW_NCOH && rr0 >= 0 && rc0 >= 0 && rc0 < W &&
                             (rr0 < y || rc0 < x);
        // unconditional loads (a valid index for the other lanes): a load inside a divergent
        // branch joins through a copy that waits for it
        const long sidx = cpos_ok ? (long)rr0 * W + rc0 : 0;
        const int s_r = f.s[2 * sidx], s_c = f.s[2 * sidx + 1], s_i = f.im[sidx];
        // the loads above stay in this round trip (not sunk to their first use, after the
        // segment minima's wait: one more round trip on wave 1's path)
        asm volatile("" ::: "memory");
        // R16: K of the per-segment skip bound, and Kf = K rounded up to fp32
        double Kd = 0.0;
        if constexpr (ROT) Kd = r16_kseg(am, ask, nqq, nsk);
        if (wv != 1) {
            float ewv;
            if constexpr (ROT) {
                float Kf = (float)Kd;
                if ((double)Kf < Kd) Kf = nextafterf(Kf, INFINITY);
                ewv = seg3_wave_umin(sq4, ac4, n4, t3, v, sgc, Kf);
            } else {
                ewv = seg3_wave_min(sq4, n4, t3, v);
            }
            if (lane == 0) redf[wv] = ewv;
        }
        if (wv == 1) wstamp(14);
        // ---- wave 1: the coherence candidates (best_coherence_match, algorithms.py:92-130:
        // p_r = s(r) + q - r inside A'): lane k loads sample k of each into registers now
        // (plain loads: cheap to issue, so the e* barrier does not wait for them); they are
        // transposed through LDS and picked after the selection, while waves 0, 2, 3 copy
        // the first windows
        double cv[XW_NCOH], cvl = 0.0;
        if (wv == 1) {
            int sr = s_r + y - rr0, sc = s_c + x - rc0;
            const bool ok = cpos_ok && sr >= 0 && sr < src.A.h && sc >= 0 && sc < src.A.w;
            sr = ok ? sr : 0;
            sc = ok ? sc : 0;
            const int si = ok ? s_i : 0;
            const long cix = ((long)src.A.h * si + sr) * src.A.w + sc;
            cvl = src.Ap.lg[cix];   // every lane (valid index); stored to LDS after the selection
            if (lane < XW_NCOH) {
                ccix[lane] = ok ? cix : -1;
                cpos[lane][0] = sr; cpos[lane][1] = sc; cpos[lane][2] = si;
            }
            // lane k's feature (emit_feature's order): its plane (A / A', fine / coarse) as a
            // base pointer, image stride, row stride and coordinate shift, and its offset from
            // the candidate's pixel in that plane, once; per candidate a few integer ops
            const int k = lane < IA_D ? lane : 0;
            const bool yk = k >= 34;
            const int kk = yk ? k - 34 : k;
            const bool co = kk < 9;
            const int t = co ? kk : kk - 9;
            const int dy = co ? t / 3 - 1 : t / 5 - 2, dx = co ? t % 3 - 1 : t % 5 - 2;
            // the fields as VALUES first (through asm): a per-lane select between struct
            // fields became a per-lane address into the kernel arguments, i.e. a vector load
            // and one more round trip
            int Ah = src.A.h, Ahs = src.A.hs, Aw2 = src.A.w, Aws = src.A.ws;
            int hw = (int)src.hw, hws = (int)src.hws;   // < 2^31 (image sizes)
            const double *pAl = src.A.lg, *pAs = src.A.sm, *pPl = src.Ap.lg, *pPs = src.Ap.sm;
            asm volatile("" : "+v"(Ah), "+v"(Ahs), "+v"(Aw2), "+v"(Aws), "+v"(hw), "+v"(hws));
            asm volatile("" : "+v"(pAl), "+v"(pAs), "+v"(pPl), "+v"(pPs));
            const int ih = co ? Ahs : Ah, iw = co ? Aws : Aw2;
            const int sh = co ? 1 : 0;
            const int istr = yk ? (co ? hws : hw) : 0;
            const double *lb0 = yk ? (co ? pPs : pPl) : (co ? pAs : pAl);
            const int offk = dy * iw + dx;
#pragma unroll
            for (int c = 0; c < XW_NCOH; ++c) {
                const int r = __builtin_amdgcn_readlane(sr, c), cc = __builtin_amdgcn_readlane(sc, c);
                const int im = __builtin_amdgcn_readlane(si, c);
                const int rs = r >> sh, cs2 = cc >> sh;
                int off = rs * iw + cs2 + offk;
                // fewer than 2 pixels from an edge of the fine image (uniform test): the
                // reflected sample instead
                if (!(r >= 2 && r + 2 < src.A.h && cc >= 2 && cc + 2 < src.A.w))
                    off = symi2(rs + dy, ih) * iw + symi2(cs2 + dx, iw);
                // a global load (the laundered pointer lost its address space: a flat load
                // would also count in lgkmcnt, so every LDS wait would wait for it)
                typedef const __attribute__((address_space(1))) double gdouble;
                cv[c] = *(gdouble *)(lb0 + ((long)im * istr + off));
            }
            wstamp(13);
        }
        if (wv == 1 && lane < IA_DP) {   // read by the others after the first full barrier
            qs[lane] = qsv;
            wts[lane] = wk;
            cwt[lane] = 1.0;
            cwt[IA_DP + lane] = wk;
        }
        int ns = 0;
        bool full = false;
        if (wv != 1) {
            sync3(&bar3, 1, lane);   // e* (waves 0, 2, 3)
            const float emin = fminf(redf[0], fminf(redf[2], redf[3]));
            xw_stamp(trace, 2);
            double Tseg, Trow;
            bool force_full;
            if constexpr (ROT) {
                r16_tseg0(emin, am, nqq, Tseg, force_full);   // emin: min (m + Kf c)
                seg3_select_codes(sq4, ac4, n4, t3, v, sgc, Tseg, Kd, slist, &scount);
            } else {
                rescore_thresholds(emin, am, nqq, Tseg, Trow, force_full);
                seg3_select(sq4, n4, t3, v, Tseg, slist, &scount);
            }
            sync3(&bar3, 2, lane);
            xw_stamp(trace, 3);
            ns = scount;
            full = ns > RESCORE_SEGCAP || force_full;
            if (tid == 0) sfull = full ? 1 : 0;
            if (trace && tid == 0) trace[XW_TRACE_N - 1] = (unsigned long long)(full ? a.nseg : ns);
        }

        auto coherence = [&]() {
#pragma unroll
            for (int c = 0; c < XW_NCOH; ++c) cxd[c * XS_CST + lane] = cv[c];
            if (lane < XW_NCOH) cval[lane] = cvl;
            wave_lds_sync();
            const int c = (lane & 31) < XW_NCOH ? (lane & 31) : XW_NCOH - 1;
            const bool wl = lane >= 32;
            // groups of 11 features in flight (as xs_dist2); the factor from a table, not a
            // per-lane select (which spilled)
            int co = c * XS_CST, qo = 0, wo = wl ? IA_DP : 0;
            asm volatile("" : "+v"(co), "+v"(qo), "+v"(wo));
            Pw55 pw;
#pragma unroll
            for (int k = 0; k < IA_D; ++k) {
                const double xx = (cxd[co + k] - qs[qo + k]) * cwt[wo + k];
                pw.feed(k, xx * xx);
                if (k % 11 == 10) asm volatile("" : "+v"(co), "+v"(qo), "+v"(wo) : "v"(xx));
            }
            const double r = sqrt(pw.res);
            asm volatile("" :: "v"(r));   // computed here, not sunk past the caller's barrier
            const bool valid = (lane & 31) < XW_NCOH && ccix[c] >= 0;
            double bd = valid && !wl ? r : INFINITY;
            long long bl = valid && !wl ? c : LLONG_MAX;
            const double cwd = r * r;
            for (int o = 32; o > 0; o >>= 1) {
                const double od = __shfl_xor(bd, o);
                const long long ol = __shfl_xor(bl, o);
                fin_best(bd, bl, od, ol);
            }
            const int wn = bl == LLONG_MAX ? 0 : (int)bl;
            const double wd = __shfl(cwd, 32 + wn);
            const double wval = cval[wn];
            wstamp(15);
            if (lane == 0) {
                cs = bl == LLONG_MAX ? CohSel{0, 0, 0, 0, 0, 0, 0, 0.0}
                                     : CohSel{ccix[wn], cpos[wn][0], cpos[wn][1], cpos[wn][2],
                                              y - 2 + wn / 5, x - 2 + wn % 5, 1, wd};
                csval = wval;
            }
        };

        // ---- 2. every row of the candidate segments, rescored in fp64 from the windows
        double bd = INFINITY;
        long long bi = LLONG_MAX;
        const int Aw = src.A.w;
        // the first segment's windows are requested before wave 1 computes the coherence
        // pick (its gathers landed meanwhile)
        // the first listed segment's windows are requested while wave 1 picks the coherence
        // candidate
        XsWin w{};
        XsFix fx;
        const int dr = wv == 0 ? 0 : wv - 1;   // DMA rank of waves 0, 2, 3
        long nit = full ? a.nseg : ns;          // (wave 1: after the barrier below)
        if (wv != 1 && nit > 0) {
            w = xs_window(a, full ? 0 : slist[0]);
            xs_dma(w, src.A, win, dr, lane, fx);
        }
        if (wv == 1) {
            coherence();
        } else if (nit > 0) {
            win_dma_wait();
            xs_fix(fx, win, 64 * dr + lane);
        }
        __syncthreads();   // the first windows complete; the selection visible to wave 1
        if (wv == 1) {
            ns = scount;
            full = sfull != 0;
            nit = full ? a.nseg : ns;
            if (nit > 0) w = xs_window(a, full ? 0 : slist[0]);
        }
        const long nscan = nit;
        // segments after the first: their windows are loaded into registers while the one
        // before is rescored, and stored after its last read (one LDS window, no DMA wait)
        XsPre pre;
        XsWin wn{};
        for (long si = 0; si < nit; ++si) {
            if (si > 0) {
                __syncthreads();   // every row of the last segment is read before the stores
                xs_pre_store(pre, win, tid);
                w = wn;
                __syncthreads();   // the windows are complete
            }
            if (si + 1 < nit) {
                wn = xs_window(a, full ? si + 1 : slist[si + 1]);
                xs_pre_load(wn, src.A, tid, pre);
            }
            if (si == 0) {
                xw_stamp(trace, 4);
                if (wv == 0) wstamp(11);
            }
            const double *wdb = reinterpret_cast<const double *>(win);
            if (w.nst == 4) {
                // 512 rows: thread tid takes pixels (y0 + 2p, x) and (y0 + 2p + 1, x),
                // x = x0 + (tid & 127), p = tid >> 7
                const int px = w.x0 + (tid & 127), py = w.y0 + 2 * (tid >> 7);
                double d0, d1;
                xs_dist_pair(wdb, xs_fbase(w, py, px), xs_cbase(w, py, px), qs, d0, d1);
                const long g = w.g0 + (long)(2 * (tid >> 7)) * Aw + (tid & 127);
                fin_best(bd, bi, d0, g);
                fin_best(bd, bi, d1, g + Aw);
            } else {
                // rows k = tid, tid + 256 of the segment (k & (seg_rows - 1): the rows past a
                // shorter segment recompute a real row and are not taken)
                const int k0 = tid & (a.seg_rows - 1), k1 = (tid + 256) & (a.seg_rows - 1);
                const int y0 = w.y0 + (k0 >> 7), x0 = w.x0 + (k0 & 127);
                const int y1 = w.y0 + (k1 >> 7), x1 = w.x0 + (k1 & 127);
                double d0, d1;
                xs_dist2(wdb, xs_fbase(w, y0, x0), xs_cbase(w, y0, x0), xs_fbase(w, y1, x1), xs_cbase(w, y1, x1),
                         qs, d0, d1);
                if (tid < a.seg_rows) fin_best(bd, bi, d0, w.g0 + (long)(k0 >> 7) * Aw + (k0 & 127));
                if (tid + 256 < a.seg_rows) fin_best(bd, bi, d1, w.g0 + (long)(k1 >> 7) * Aw + (k1 & 127));
            }
            if (si == 0 && wv == 0) wstamp(12);
        }
        for (int o = 32; o > 0; o >>= 1) {
            const double od = __shfl_xor(bd, o);
            const long long oi = __shfl_xor(bi, o);
            fin_best(bd, bi, od, oi);
        }
        // ---- 3. each wave's best row: its weighted distance (algorithms.py:133-135) and A'
        // value, from the windows when it is a row of the last segment (always with one
        // candidate segment), else gathered; the four waves in parallel, before the barrier
        XRec wb{bd, bi, 0.0, 0.0};
        if (bi != LLONG_MAX) {
            const long rel = bi - w.g0;
            const long ry = rel >= 0 ? rel / Aw : -1, rx = rel - ry * Aw;
            double sq = 0.0;
            if (rel >= 0 && ry < w.nst && rx < 128) {
                const int py = w.y0 + (int)ry, px = w.x0 + (int)rx;
                const int fb = xs_fbase(w, py, px), cb = xs_cbase(w, py, px);
                const double *wdb = reinterpret_cast<const double *>(win);
                if (lane < IA_D) {
                    const double xw = (wdb[(xs_coarse(lane) ? cb : fb) + xs_koff(lane)] - qs[lane]) * wts[lane];
                    sq = xw * xw;
                }
                wb.val = wdb[XS_FP + fb];
            } else {
                ImgPair ap;
                int r, c;
                src.locate(bi, ap, r, c);
                int rr, cc;
                const double *fp = feat_addr(src.A, ap, r, c, lane < IA_D ? lane : 0, rr, cc);
                if (lane < IA_D) {
                    const double xw = (*fp - qs[lane]) * wts[lane];
                    sq = xw * xw;
                }
                wb.val = src.Ap.lg[bi];
            }
            const double sw = sqrt(pw55_lanes(sq));
            wb.wd = sw * sw;
        }
        if (lane == 0) { bds[wv] = wb.d; bis[wv] = wb.i; bwd[wv] = wb.wd; bvl[wv] = wb.val; }
        __syncthreads();   // the block's winner; the coherence pick is in cs
        xw_stamp(trace, 5);
        if (wv != 0) return;
        if constexpr (ROT) {   // win is free: the rotation for the next query lands meanwhile
            if (nxt) rot_dma();
        }
        XRec lb{INFINITY, LLONG_MAX, 0.0, 0.0};
#pragma unroll
        for (int k = 0; k < 4; ++k) xrec_take(lb, XRec{bds[k], bis[k], bwd[k], bvl[k]});
        xw_stamp(trace, 6);
        own = xw_finish(a, i, y, x, lane, lb, cs, csval, (unsigned int)(nscan * a.seg_rows), ns, full, trace);
    }
    xw_stamp(trace, 8);
    if (wv != 0 || !nxt) return;
    if constexpr (ROT) {
        if (!cur) rot_dma();   // (a pixel of wave t + 1 only: win was never used)
    }
    xw_next_query(a, i, y, x, lane, pdep, own, amx, nxw, trace, ROT ? rotl : nullptr, ROT ? dq : nullptr);
}

}  // namespace ia

/* the fused strip kernel's resources (DESIGN.md §7 forward-progress rule): rot 1 the R16
 * form; LDS bytes per workgroup, VGPRs per lane */
extern "C" int ia_fused_resources(int rot, int *lds, int *vgprs) {
    IA_ARG(lds && vgprs, "ia_fused_resources: bad args");
    hipFuncAttributes at{};
    if (rot) IA_HIP(hipFuncGetAttributes(&at, reinterpret_cast<const void *>(&ia::k_xstrip<false, true>)));
    else IA_HIP(hipFuncGetAttributes(&at, reinterpret_cast<const void *>(&ia::k_xstrip<false, false>)));
    *lds = (int)at.sharedSizeBytes;
    *vgprs = at.numRegs;
    return IA_OK;
}

namespace ia {

// the one-job fused kernel of a form (launch_xwave): k_xstrip<false, rot> (XW_STRIP),
// k_xwave<true / false, false> (XW_IMG / XW_ROWS)
int xwave_attributes(int form, bool rot, hipFuncAttributes *at) {
    const void *f = form == XW_STRIP ? (rot ? reinterpret_cast<const void *>(&k_xstrip<false, true>)
                                            : reinterpret_cast<const void *>(&k_xstrip<false, false>))
                    : form == XW_IMG ? reinterpret_cast<const void *>(&k_xwave<true, false>)
                                     : reinterpret_cast<const void *>(&k_xwave<false, false>);
    IA_HIP(hipFuncGetAttributes(at, f));
    return IA_OK;
}

int launch_xwave(const XArgs &a, int nblocks, int form, hipStream_t st, int njobs) {
    if (nblocks <= 0) return IA_OK;
    IA_ARG(njobs >= 1 && njobs <= IA_BATCH_MAX && (njobs == 1 || a.jobs), "launch_xwave: bad batch");
    IA_ARG(form != XW_STRIP || (a.smap.W > 0 && xstrip_applies(a.src) && a.seg_rows >= 128 && a.seg_rows <= 512),
           "launch_xwave: the strip form needs a strip-order image-form level");
    const dim3 grid((unsigned)nblocks, (unsigned)njobs);
    const bool b = njobs > 1;
    if (form == XW_STRIP) {
        if (a.rot) {
            if (b) k_xstrip<true, true><<<grid, 256, 0, st>>>(a);
            else k_xstrip<false, true><<<grid, 256, 0, st>>>(a);
        } else {
            if (b) k_xstrip<true, false><<<grid, 256, 0, st>>>(a);
            else k_xstrip<false, false><<<grid, 256, 0, st>>>(a);
        }
    } else if (form == XW_IMG) {
        if (b) k_xwave<true, true><<<grid, 256, 0, st>>>(a);
        else k_xwave<true, false><<<grid, 256, 0, st>>>(a);
    } else {
        if (b) k_xwave<false, true><<<grid, 256, 0, st>>>(a);
        else k_xwave<false, false><<<grid, 256, 0, st>>>(a);
    }
    IA_LAUNCH_CHECK("k_xwave");
    return IA_OK;
}

}  // namespace ia
