// ia_synth.hip — per-level B' synthesis on device.
//
// The reference visits B' pixels in scanline order (image_analogies.py:161-162) and each
// query reads only causal B' samples: rows y-2, y-1 (cols x-2..x+2) and row y (cols
// x-2, x-1) of the fine level through symmetric padding, plus s/im of the same causal
// window for coherence.  Every such sample (including reflected border samples, which
// stay inside rows y-2..y+1 and cols x-2..x+2) satisfies: written before q in scanline
// order  <=>  its wave index x' + 3y' < x + 3y.  So processing the skewed wavefronts
// t = x + 3y in increasing t, each wave fully in parallel, reads exactly the values the
// scanline loop reads (DESIGN.md gives the case analysis; tests/test_oracle.py checks it
// exhaustively for small H, W).  Per wave:
//   k_query_wave  -> q64 / qp / q16 / nq        (ia_features.hip)
//   k_screen16    -> segment minima             (ia_screen16.hip, split-f16 MFMA)
//   k_rescore or k_select/k_items/k_gather -> the exact winner (ia_match.hip, fp64);
//                    on one GPU the same kernel runs the per-pixel tail (ia_finish.h)
//   sharded DB: RCCL all-gather of the per-rank winners, then
//   k_finish      -> coherence, kappa test, B'/s/im update (this file)
#include "ia_finish.h"
#include "ia_split16.h"
#include "ia_rot16.h"
#include "../../include/ia_diag.h"

#include <cstdio>
#include <cstdlib>
#include <functional>
#include <mutex>
#include <vector>

#include <rccl/rccl.h>

namespace ia {

// Sticky schedule-error word of this device: every level's done() folds its fused kernel's
// error word (a neighbour-decision wait that timed out) into it on the level's stream, so
// callers that skip the per-call ia_synth_status (bench.py's timed steps) check once at the
// end with ia_sched_status.  Vector stores only.
__device__ unsigned int g_sched_err;

__global__ __launch_bounds__(64) void k_err_sticky(const unsigned int *__restrict__ ctl,
                                                   const XJob *__restrict__ jt, int K) {
    for (int k = threadIdx.x; k < K; k += 64) {
        const unsigned int e = jt ? jt[k].ctl[2] : ctl[2];
        if (e) g_sched_err = 1u;
    }
}

// Sharded DB, after the cross-rank exchange: one wave per query pixel takes the
// lexicographic (distance, row) minimum over the ranks' ShardRec (lane g = rank g), whose
// weighted distance the owning rank already computed, and finishes the pixel with the
// coherence pick its own exact stage stored (every rank holds the same replicated state,
// so the picks agree; ia_finish.h).  No feature gathers here.
__global__ __launch_bounds__(64) void k_finish(DbSrc src, const ShardRec *__restrict__ rec_all,
                                               const CohSel *__restrict__ coh, int nranks, int M,
                                               FinishArgs f) {
    const int m = blockIdx.x;
    const int lane = threadIdx.x;
    double d = INFINITY, wd = 0.0;
    long long idx = 0x7fffffffffffffffLL;
    for (int g = lane; g < nranks; g += 64) {
        const ShardRec r = rec_all[(long)g * M + m];
        if (r.d < d || (r.d == d && r.idx < idx)) { d = r.d; idx = r.idx; wd = r.wd; }
    }
    for (int o = 32; o > 0; o >>= 1) {
        const double od = __shfl_xor(d, o), owd = __shfl_xor(wd, o);
        const long long oi = __shfl_xor(idx, o);
        if (od < d || (od == d && oi < idx)) { d = od; idx = oi; wd = owd; }
    }
    finish_apply(src, idx, m, f, coh[m], wd, lane);
}

// Sharded DB, the other tail form (IA_SHARD_TAIL=0): the exact stage writes only its
// shard's (distance, row); after the exchange wave 1 picks the coherence candidate while
// wave 0 reduces the ranks' winners and weighs the global one, then finishes the pixel
__global__ __launch_bounds__(128) void k_finish_gather(DbSrc src, const Best *__restrict__ best_all,
                                                       int nranks, int M, FinishArgs f,
                                                       const double *__restrict__ q64) {
    __shared__ double qs[IA_DP];
    __shared__ CohSel cs;
    const int m = blockIdx.x;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    // the query and (wave 0) the first 8 ranks' winners in one memory round trip
    const double qv = threadIdx.x < IA_DP ? q64[(long)m * IA_DP + threadIdx.x] : 0.0;
    constexpr int NB0 = 8;
    Best b0[NB0];
    if (wv == 0) {
#pragma unroll
        for (int g = 0; g < NB0; ++g)
            b0[g] = g < nranks ? best_all[(long)g * M + m] : Best{INFINITY, 0x7fffffffffffffffLL};
    }
    if (threadIdx.x < IA_DP) qs[threadIdx.x] = qv;
    __syncthreads();
    double ad = INFINITY;
    long long app = 0x7fffffffffffffffLL;
    if (wv == 1) {
        const CohSel c = coh_pick(src, m, f, qs, lane);
        if (lane == 0) cs = c;
    } else {
#pragma unroll
        for (int g = 0; g < NB0; ++g) fin_best(ad, app, b0[g].d, b0[g].idx);
        for (int g = NB0; g < nranks; ++g) {
            const Best b = best_all[(long)g * M + m];
            fin_best(ad, app, b.d, b.idx);
        }
    }
    const double d_app = wv == 0 ? app_wdist(src, app, f, qs, lane) : 0.0;
    __syncthreads();
    if (wv == 0) finish_apply(src, app, m, f, cs, d_app, lane);
}

// Sharded DB over the device-side exchange: the exact stage published this shard's winner
// (k_rescore<3> / k_gather<3>, which also left it in best[m]); wave 0 collects every
// rank's from this rank's receive box and weighs the global winner while wave 1 picks the
// coherence candidate, then wave 0 finishes the pixel.  The waits live in these small
// 2-wave workgroups, not in the exact stage's 4-wave, 250-VGPR ones: ranks sharing a GPU,
// or a rank's other streams, keep room to run the kernels the waits depend on (the fused
// form deadlocked two ranks on one GPU).  On timeout the shard's own winner.
__global__ __launch_bounds__(128) void k_peer_finish(DbSrc src, const Best *__restrict__ best,
                                                     FinishArgs f, const double *__restrict__ q64) {
    __shared__ double qs[IA_DP];
    __shared__ CohSel cs;
    const int m = blockIdx.x;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const double qv = threadIdx.x < IA_DP ? q64[(long)m * IA_DP + threadIdx.x] : 0.0;
    const Best own = best[m];
    if (threadIdx.x < IA_DP) qs[threadIdx.x] = qv;
    __syncthreads();
    double gd = own.d;
    long long gw = own.idx;
    if (wv == 1) {
        const CohSel c = coh_pick(src, m, f, qs, lane);
        if (lane == 0) cs = c;
    } else {
        const bool tron = f.px.trace && m < 8 && f.px.epoch < 1024;
        unsigned long long *tr = tron ? reinterpret_cast<unsigned long long *>(f.px.trace.get()) +
                                            ((long)f.px.epoch * 8 + m) * 12
                                      : nullptr;
        peer_collect(f.px, m, lane, gd, gw, tr ? tr + 4 : nullptr);
        if (tr && lane == 0) {
            tr[0] = __double_as_longlong(own.d); tr[1] = own.idx;
            tr[2] = __double_as_longlong(gd); tr[3] = gw;
        }
    }
    const double d_app = wv == 0 ? app_wdist(src, gw, f, qs, lane) : 0.0;
    __syncthreads();
    if (wv == 0) finish_apply(src, gw, m, f, cs, d_app, lane);
}

// LSH matcher (one shard): wave 1 picks the coherence candidate while wave 0 weighs the
// LSH winner, then wave 0 finishes the pixel (ia_finish.h)
__global__ __launch_bounds__(128) void k_lsh_tail(DbSrc src, const Best *__restrict__ best, int M,
                                                  FinishArgs f, const double *__restrict__ q64) {
    __shared__ double qs[IA_DP];
    __shared__ CohSel cs;
    const int m = blockIdx.x;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (threadIdx.x < IA_DP) qs[threadIdx.x] = q64[(long)m * IA_DP + threadIdx.x];
    __syncthreads();
    const long long app = best[m].idx;
    if (wv == 1) {
        const CohSel c = coh_pick(src, m, f, qs, lane);
        if (lane == 0) cs = c;
    }
    const double d_app = wv == 0 ? app_wdist(src, app, f, qs, lane) : 0.0;
    __syncthreads();
    if (wv == 0) finish_apply(src, app, m, f, cs, d_app, lane);
}

// -------------------------------- workspace ----------------------------------------
struct SynthWs {
    double *q64;
    float *qp;
    _Float16 *q16;
    double *nq;
    void *scratch;           // screen output (candidates or segment minima)
    Best *best_local;
    ShardRec *rec_local;     // sharded DB: this rank's records, then all ranks'
    ShardRec *rec_all;
    CohSel *coh;
    unsigned long long *stats;
    // the fused per-wave kernel (k_xwave): the query rows of odd waves (even waves use
    // q64 / qp / q16 / nq), the decision granules (2 per row) and the control words
    // {tickets[2], error}
    double *q64b;
    float *qpb;
    _Float16 *q16b;
    double *nqb;
    unsigned long long *dbox;
    unsigned int *ctl;
    XJob *jtab;              // a batch's job table (ia_synth_levels_batch, job 0's workspace)
};
constexpr int XW_CTL_ERR = 2;

static inline int wave_max_queries(int H, int W) {
    const int byw = (W + 2) / 3;   // ceil(W/3)
    return (H < byw ? H : byw) + 1;
}

static size_t carve(SynthWs *ws, char *base, int H, int W, long nrows, int nranks) {
    const int Mmax = wave_max_queries(H, W);
    const int qr = qrows_alloc(Mmax);
    size_t off = 0;
    auto take = [&](size_t bytes) { size_t o = off; off += align_up(bytes, 256); return base ? base + o : nullptr; };
    SynthWs w;
    w.q64 = (double *)take((size_t)Mmax * IA_DP * sizeof(double));
    w.qp = (float *)take((size_t)qr * IA_DP * sizeof(float));
    w.q16 = (_Float16 *)take((size_t)qr * Q16_ROW * 16);
    w.nq = (double *)take((size_t)qr * sizeof(double));
    w.scratch = take(match_scratch_bytes(qr, nrows));
    w.best_local = (Best *)take((size_t)Mmax * sizeof(Best));
    w.rec_local = (ShardRec *)take((size_t)Mmax * sizeof(ShardRec));
    w.rec_all = (ShardRec *)take((size_t)Mmax * nranks * sizeof(ShardRec));
    w.coh = (CohSel *)take((size_t)Mmax * sizeof(CohSel));
    w.stats = (unsigned long long *)take(STATS_BYTES);
    w.q64b = (double *)take((size_t)Mmax * IA_DP * sizeof(double));
    w.qpb = (float *)take((size_t)qr * IA_DP * sizeof(float));
    w.q16b = (_Float16 *)take((size_t)qr * Q16_ROW * 16);
    w.nqb = (double *)take((size_t)qr * sizeof(double));
    w.dbox = (unsigned long long *)take((size_t)H * 2 * sizeof(unsigned long long));
    w.ctl = (unsigned int *)take(256);
    w.jtab = (XJob *)take((size_t)IA_BATCH_MAX * sizeof(XJob));
    if (ws) *ws = w;
    return off;
}

// executable graphs stay alive until their launch has completed (destroyed lazily at the
// next capture, after an event wait; ia_release_thread_resources frees them)
struct GraphKeeper {
    hipStream_t cap = nullptr;
    hipGraphExec_t exec = nullptr;
    hipEvent_t done = nullptr;
    hipError_t retire() {
        if (!exec) return hipSuccess;
        hipError_t e = hipEventSynchronize(done);
        if (e == hipSuccess) e = hipGraphExecDestroy(exec);
        exec = nullptr;
        return e;
    }
    hipError_t hold(hipGraphExec_t x, hipStream_t st) {
        exec = x;
        if (!done) {
            hipError_t e = hipEventCreateWithFlags(&done, hipEventDisableTiming);
            if (e != hipSuccess) return e;
        }
        return hipEventRecord(done, st);
    }
};
static thread_local GraphKeeper g_graphs;

// ---- profiling (IA_SYNTH_PROF): HIP events around every screen launch and the matcher
// statistics, collected WITHOUT synchronising: events come from a process-wide pool and
// the statistics are copied stream-ordered into pinned host memory; ia_prof_end()
// synchronises once and reads everything back.  So a profiled level runs the same
// launches with no host round trip (bench.py profiles its timed steps this way).
struct ProfRec {
    int tag;
    int jobs;                // jobs batched into each launch
    long nrows;
    double pairs;
    size_t ev0;
    int nscreen, timed;
    unsigned long long *hstats;
    std::vector<int> M;      // queries of each screen launch, in launch order
};
struct ProfCollector {
    std::mutex mu;
    bool active = false;
    std::vector<hipEvent_t> ev;
    size_t next = 0;
    std::vector<ProfRec> recs;
    std::vector<unsigned long long *> pinned;
    size_t pinned_next = 0;
};
// never destroyed: the HIP runtime may be torn down before static destructors run
static ProfCollector *const g_prof = new ProfCollector;

static bool prof_active() {
    std::lock_guard<std::mutex> l(g_prof->mu);
    return g_prof->active;
}

// events [*ev0, *ev0 + nev) and one pinned statistics buffer for one level call
static int prof_reserve(size_t nev, size_t *ev0, unsigned long long **hstats) {
    std::lock_guard<std::mutex> l(g_prof->mu);
    while (g_prof->ev.size() < g_prof->next + nev) {
        hipEvent_t e;
        IA_HIP(hipEventCreate(&e));
        g_prof->ev.push_back(e);
    }
    *ev0 = g_prof->next;
    g_prof->next += nev;
    if (g_prof->pinned_next == g_prof->pinned.size()) {
        void *p = nullptr;
        IA_HIP(hipHostMalloc(&p, STATS_BYTES, hipHostMallocDefault));
        g_prof->pinned.push_back(reinterpret_cast<unsigned long long *>(p));
    }
    *hstats = g_prof->pinned[g_prof->pinned_next++];
    return IA_OK;
}

static hipEvent_t prof_event(size_t i) {
    std::lock_guard<std::mutex> l(g_prof->mu);
    return g_prof->ev[i];
}

static void prof_push(const ProfRec &r) {
    std::lock_guard<std::mutex> l(g_prof->mu);
    g_prof->recs.push_back(r);
}

// measured (tools/level_times.py, profiles/r01_level_times_graph.txt): eager launches beat
// a captured graph on every c4 level once instantiation is counted, so capture is opt-in
// (settable through ia_diag_set_graph_mode)
static std::atomic<int> g_graph_mode{env_int("IA_GRAPH", 0)};
static int graph_mode() { return g_graph_mode.load(std::memory_order_relaxed); }

int xwave_attributes(int form, bool rot, hipFuncAttributes *at);
int release_pipe3();
int screen16_attributes(bool img, hipFuncAttributes *at);
int screen_resources_r16(hipFuncAttributes *at);
int comm_allgather(void *comm, const void *send, void *recv, size_t bytes, hipStream_t st);
int comm_nranks(void *comm);
PeerView comm_peer_wave(void *comm);
int comm_peer_mcap(void *comm);

// sharded tail form (IA_SHARD_TAIL): 0 [default] the exchange carries (distance, row) and
// k_finish_gather does the coherence pick and the weighting after it; 1 the exact stage
// prepares the tail (ShardRec, CohSel) and k_finish only reduces.  Measured on the
// simulated G = 8 rank (`tools/gpu.sh abknob ... -- python tools/shard_sim.py 8`, one box): finest level 335 vs 361 ms, pipelined
// step 415 vs 450 ms, so 0
static int shard_tail() {
    static const int v = env_int("IA_SHARD_TAIL", 0);
    return v;
}

// the fused per-wave kernel (k_xwave, ia_xwave.hip): after each screen ONE launch runs the
// exact stage, the device-side exchange, the per-pixel tail and the next wave's query rows
// (IA_XWAVE / ia_diag_set_xwave: 2 [default] wherever it applies, with k_xstrip on
// strip-order image-form levels; 1 k_xwave only; 0 the separate kernels)
static std::atomic<int> g_xwave{env_int("IA_XWAVE", 2)};
static int xwave_on() { return g_xwave.load(std::memory_order_relaxed); }

// diagnostic: k_xwave phase stamps of the level tagged IA_XW_TRACE (one process-wide buffer)
static unsigned long long *g_xw_trace = nullptr;
static unsigned long long *xw_trace(int tag) {
    static const int want = env_int("IA_XW_TRACE", -1);
    if (want < 0 || tag != want) return nullptr;
    if (!g_xw_trace) {
        const size_t n = (size_t)XW_TRACE_T * XW_TRACE_PX * XW_TRACE_N * sizeof(unsigned long long);
        if (hipMalloc(&g_xw_trace, n) != hipSuccess) { g_xw_trace = nullptr; return nullptr; }
        (void)hipMemset(g_xw_trace, 0, n);
    }
    return g_xw_trace;
}

static int check_args(const IaSynthArgs *a) {
    IA_ARG(a && (a->db || a->dbi || a->lsh) && a->center && a->amax && a->B_sm && a->B_lg && a->Bp_sm && a->Bp_lg &&
               a->weights && a->s && a->im && a->workspace,
           "ia_synth_level: null argument");
    IA_ARG(a->H > 0 && a->W > 0 && a->nrows > 0 && a->row0 >= 0 &&
               a->row0 + a->nrows <= a->N_total,
           "ia_synth_level: bad sizes");
    IA_ARG(a->N_total == (long)a->src.nAp * a->src.Ah * a->src.Aw, "ia_synth_level: N_total mismatch");
    IA_ARG(a->B_hs == (a->H + 1) / 2 && a->B_ws == (a->W + 1) / 2, "ia_synth_level: B level shapes");
    IA_ARG(a->src.A_hs == (a->src.Ah + 1) / 2 && a->src.A_ws == (a->src.Aw + 1) / 2,
           "ia_synth_level: A level shapes");
    IA_ARG(!a->dbg_px == !a->dbg_dist, "ia_synth_level: debug outputs come in pairs");
    IA_ARG(comm_nranks(a->comm) >= 1, "ia_synth_level: bad communicator");
    IA_ARG(!(a->lsh && a->comm), "ia_synth_level: the LSH matcher runs unsharded (comm must be NULL)");
    return IA_OK;
}

// One level's synthesis state: init() on its stream, then wave(t) for t = 0..nw-1 in order
// (each enqueues that wave's launches), then done().
struct LevelRun {
    const IaSynthArgs *a = nullptr;
    const IaShardDb *sim = nullptr;   // diagnostic: nsim DB shards in this process
    int nsim = 0;
    SynthWs ws{};
    DbSrc src{};
    ImgPair B{}, Bp{};
    int H = 0, W = 0, nw = 0, nranks = 1;
    bool prof = false, timed = false, fused = false, peer = false, xw = false;
    // a batch of K identical-shape jobs (ia_synth_levels_batch): this run is job 0 and owns
    // the launches; part[k - 1] holds job k's state (member runs record no profile)
    int K = 1;
    bool member = false;
    // R16 (ia_rot16.h): the rotated DB and rotation given, on a strip-order level of the fused
    // kernel: the rotated screen, rotated query rows and k_xstrip's R16 bound
    bool r16 = false;
    std::vector<LevelRun> part;
    size_t ev0 = 0;
    unsigned long long *hstats = nullptr;
    double pairs = 0.0;
    int nscreen = 0;
    std::vector<int> Ms;

    int init(const IaSynthArgs *args, hipStream_t st) {
        a = args;
        int rc = check_args(a);
        if (rc) return rc;
        nranks = a->comm ? comm_nranks(a->comm) : (sim ? nsim : 1);
        H = a->H; W = a->W;
        nw = (W - 1) + 3 * (H - 1) + 1;
        long rows_ws = a->nrows;
        for (int r = 0; r < nsim; ++r) rows_ws = sim[r].nrows > rows_ws ? sim[r].nrows : rows_ws;
        carve(&ws, reinterpret_cast<char *>(a->workspace), H, W, rows_ws, nranks);
        const int Mmax = wave_max_queries(H, W);
        IA_HIP(hipMemsetAsync(ws.qp, 0, (size_t)qrows_alloc(Mmax) * IA_DP * sizeof(float), st));
        IA_HIP(hipMemsetAsync(ws.q16, 0, (size_t)qrows_alloc(Mmax) * Q16_ROW * 16, st));
        IA_HIP(hipMemsetAsync(ws.stats, 0, STATS_BYTES, st));
        IA_HIP(hipMemsetAsync(ws.scratch, 0, 256, st));   // the exact stage's empty work list
        src = make_dbsrc(a->src);
        B = ImgPair{a->B_sm, a->B_lg, a->B_hs, a->B_ws, H, W};
        Bp = ImgPair{a->Bp_sm, a->Bp_lg, a->B_hs, a->B_ws, H, W};
        prof = !member && (a->flags & IA_SYNTH_PROF) && prof_active();
        timed = prof;
        if (prof && (rc = prof_reserve(3 * (size_t)nw, &ev0, &hstats))) return rc;
        // fused tail (one launch + one round trip less per wave): on a single shard the exact
        // stage's last kernel (k_rescore, or k_gather of the work list) runs the pixel tail;
        // on a sharded DB it prepares the tail (coherence pick, the winner's weighted
        // distance) before the exchange
        fused = !a->comm && !a->lsh && !sim;
        // sharded level over the device-side exchange: the exact stage's kernel publishes,
        // k_peer_finish collects and finishes each pixel (no RCCL call)
        peer = a->comm && comm_peer_mcap(a->comm) > 0;
        IA_ARG(!peer || comm_peer_mcap(a->comm) >= Mmax,
               "ia_synth_level: the peer exchange's box holds fewer queries than a wave");
        IA_ARG(!peer || a->N_total < (1L << 32),
               "ia_synth_level: the peer exchange carries 32-bit rows (N_total >= 2^32)");
        // one launch per wave after the screen (k_xwave) wherever the exact matcher runs
        // on one GPU or over the device-side exchange (not the LSH matcher, the RCCL
        // exchange, the in-process shard simulation or a forced work list)
        xw = xwave_on() && !a->lsh && !sim && (!a->comm || peer) && exact_stage_mode() != 1;
        // (any form of the fused kernel: k_xstrip on strip-order levels, k_xwave elsewhere)
        r16 = xw && a->dbr && a->rot;
        IA_HIP(hipMemsetAsync(ws.ctl, 0, 256, st));   // tickets, error word (ia_synth_status)
        if (xw) {
            IA_HIP(hipMemsetAsync(ws.qpb, 0, (size_t)qrows_alloc(Mmax) * IA_DP * sizeof(float), st));
            IA_HIP(hipMemsetAsync(ws.q16b, 0, (size_t)qrows_alloc(Mmax) * Q16_ROW * 16, st));
            IA_HIP(hipMemsetAsync(ws.dbox, 0, (size_t)H * 2 * sizeof(unsigned long long), st));
        }
        return IA_OK;
    }

    // wave t: pixels y in [y_lo, y_hi], x = t - 3y
    static void wave_rows(int H, int W, int t, int &y_lo, int &M) {
        const int lo_num = t - (W - 1);
        y_lo = lo_num > 0 ? (lo_num + 2) / 3 : 0;
        const int y_hi = t / 3 < H - 1 ? t / 3 : H - 1;
        M = y_hi - y_lo + 1;
    }

    int wave(int t, hipStream_t sq) {
        int y_lo, M;
        wave_rows(H, W, t, y_lo, M);
        if (M <= 0) return IA_OK;
        int rc;
        if (sim) return sim_wave(t, y_lo, M, sq);
        if (xw) return xw_wave(t, y_lo, M, sq);
        if ((rc = launch_query_wave(B, Bp, t, y_lo, M, a->center, ws.q64, ws.qp, ws.nq, a->amax,
                                    ws.q16, sq)))
            return rc;
        hipEvent_t e0 = timed ? prof_event(ev0 + 3 * nscreen) : nullptr;
        hipEvent_t e1 = timed ? prof_event(ev0 + 3 * nscreen + 1) : nullptr;
        FinishArgs fa{t, y_lo, W, a->N_total, a->weights, a->kappa_factor, a->Bp_lg, a->s,
                      a->im, a->dbg_px, a->dbg_dist,
                      a->comm && !peer && shard_tail() ? ws.rec_local : nullptr,
                      a->comm && !peer && shard_tail() ? ws.coh : nullptr};
        if (peer) fa.px = comm_peer_wave(a->comm);
        if (a->lsh) {   // approximate matcher: the events bracket the LSH query kernel
            if (e0) IA_HIP(hipEventRecord(e0, sq));
            if ((rc = launch_lsh_match(a->lsh, src, a->row0, a->nrows, M, ws.q64, a->center,
                                       ws.best_local, prof ? ws.stats : nullptr, sq)))
                return rc;
            if (e1) IA_HIP(hipEventRecord(e1, sq));
        } else if ((rc = launch_match(src, a->row0, a->nrows, a->db, a->dbi, ws.qp, ws.q16, M, ws.q64, ws.nq,
                                      a->amax, ws.scratch, ws.best_local,
                                      prof ? ws.stats : nullptr, sq, e0, e1,
                                      (fused || peer || (a->comm && shard_tail())) ? &fa : nullptr))) {
            return rc;
        }
        ++nscreen;
        pairs += (double)M * (double)a->nrows;
        if (prof) Ms.push_back(M);
        // diagnostic (IA_SYNC_EVERY=n): wait for the stream every n waves, bounding the
        // dispatches in flight (rocprofv3 --pmc runs of the whole bench crash otherwise)
        static const int sync_every = env_int("IA_SYNC_EVERY", 0);
        if (sync_every > 0 && t % sync_every == sync_every - 1) IA_HIP(hipStreamSynchronize(sq));
        // e2 of this wave: right after the exact stage (the unfused tails are not bracketed)
        if (timed) IA_HIP(hipEventRecord(prof_event(ev0 + 3 * (nscreen - 1) + 2), sq));
        if (fused) return IA_OK;   // the exact stage already ran the per-pixel tail
        if (peer) {                // collect the ranks' winners, finish the pixel
            k_peer_finish<<<M, 128, 0, sq>>>(src, ws.best_local, fa, ws.q64);
            IA_LAUNCH_CHECK("k_peer_finish");
            return IA_OK;
        }
        if (a->lsh) {   // one shard, LSH winners: the tail in k_lsh_finish form
            k_lsh_tail<<<M, 128, 0, sq>>>(src, ws.best_local, M, fa, ws.q64);
            IA_LAUNCH_CHECK("k_lsh_tail");
            return IA_OK;
        }
        // sharded DB: the exact stage left this rank's records and coherence picks; the
        // exchange (also with one rank: the same RCCL path, exercised by the tests), then
        // the finish
        if (!shard_tail()) {
            Best *all = reinterpret_cast<Best *>(ws.rec_all);
            if ((rc = comm_allgather(a->comm, ws.best_local, all, (size_t)M * sizeof(Best), sq)))
                return rc;
            k_finish_gather<<<M, 128, 0, sq>>>(src, all, nranks, M, fa, ws.q64);
            IA_LAUNCH_CHECK("k_finish_gather");
            return IA_OK;
        }
        if ((rc = comm_allgather(a->comm, ws.rec_local, ws.rec_all, (size_t)M * sizeof(ShardRec), sq)))
            return rc;
        k_finish<<<M, 64, 0, sq>>>(src, ws.rec_all, ws.coh, nranks, M, fa);
        IA_LAUNCH_CHECK("k_finish");
        return IA_OK;
    }

    // job k's table entry (the batched launches read their pointers from it)
    XJob job_entry() const {
        XJob J{};
        J.A_sm = a->src.A_sm; J.A_lg = a->src.A_lg; J.Ap_sm = a->src.Ap_sm; J.Ap_lg = a->src.Ap_lg;
        ImgDb img{};
        if (a->dbi)
            img_db_layout(src.A.h, src.A.w, src.A.hs, src.A.ws, 1, a->row0, a->nrows, a->dbi, img, nullptr);
        J.fa = img.fa; J.ca = img.ca; J.norm = img.norm; J.ap = img.ap;
        J.db = a->db;
        J.segmin = match_segmin(ws.scratch);
        J.q64[0] = ws.q64; J.q64[1] = ws.q64b;
        J.qp[0] = ws.qp; J.qp[1] = ws.qpb;
        J.nq[0] = ws.nq; J.nq[1] = ws.nqb;
        J.q16[0] = ws.q16; J.q16[1] = ws.q16b;
        J.amax = a->amax;
        J.center = a->center;
        J.B_sm = a->B_sm; J.B_lg = a->B_lg; J.Bp_sm = a->Bp_sm; J.Bp_lg = a->Bp_lg;
        J.weights = a->weights;
        J.kappa_factor = a->kappa_factor;
        J.s = a->s; J.im = a->im; J.dbg_px = a->dbg_px; J.dbg_dist = a->dbg_dist;
        J.dbox = ws.dbox;
        J.ctl = ws.ctl;
        J.dbr = r16 ? a->dbr : nullptr;
        J.askc = r16 ? r16_askc(a->dbr, a->nrows) : nullptr;
        J.rot = r16 ? a->rot : nullptr;
        return J;
    }

    // K jobs (args[0..K)) of identical shapes in one set of launches per wave; the job
    // table is staged through `pinned` (kept alive by the caller until the copy has run)
    int init_batch(const IaSynthArgs *args, int nj, hipStream_t st, XJob *pinned) {
        int rc = init(&args[0], st);
        if (rc || nj == 1) return rc;
        IA_ARG(nj <= IA_BATCH_MAX, "ia_synth_levels_batch: too many jobs in one batch");
        IA_ARG(xw, "ia_synth_levels_batch: batches run the exact matcher on one GPU (fused kernel)");
        // XJob carries no exchange view: K jobs would publish into one box (cells indexed by
        // query only) and advance its epoch once per wave for K jobs
        IA_ARG(!a->comm && !a->lsh,
               "ia_synth_levels_batch: a batch of K > 1 jobs takes neither a comm nor an LSH index");
        K = nj;
        part.resize(K - 1);
        for (int k = 1; k < K; ++k) {
            const IaSynthArgs &b = args[k];
            IA_ARG(b.H == a->H && b.W == a->W && b.nrows == a->nrows && b.N_total == a->N_total &&
                       b.row0 == a->row0 && b.B_hs == a->B_hs && b.B_ws == a->B_ws &&
                       b.src.Ah == a->src.Ah && b.src.Aw == a->src.Aw && b.src.A_hs == a->src.A_hs &&
                       b.src.A_ws == a->src.A_ws && b.src.nAp == a->src.nAp &&
                       !b.comm == !a->comm && !b.lsh == !a->lsh && !b.dbi == !a->dbi &&
                       !b.dbg_px == !a->dbg_px,
                   "ia_synth_levels_batch: the jobs of a batch must have identical shapes and forms");
            part[k - 1].member = true;
            if ((rc = part[k - 1].init(&b, st))) return rc;
            IA_ARG(part[k - 1].xw, "ia_synth_levels_batch: a job without the fused kernel");
            IA_ARG(part[k - 1].r16 == r16, "ia_synth_levels_batch: jobs with and without the rotated DB");
        }
        pinned[0] = job_entry();
        for (int k = 1; k < K; ++k) pinned[k] = part[k - 1].job_entry();
        IA_HIP(hipMemcpyAsync(ws.jtab, pinned, (size_t)K * sizeof(XJob), hipMemcpyHostToDevice, st));
        return IA_OK;
    }

    // wave t on the fused path: [wave 0's query rows,] the screen, then k_xwave (exact
    // stage, exchange, tail, and wave t + 1's query rows into the other buffer set)
    int xw_wave(int t, int y_lo, int M, hipStream_t sq) {
        int rc;
        double *q64s[2] = {ws.q64, ws.q64b};
        float *qps[2] = {ws.qp, ws.qpb};
        _Float16 *q16s[2] = {ws.q16, ws.q16b};
        double *nqs[2] = {ws.nq, ws.nqb};
        const int b = t & 1;
        if (t == 0 && (rc = launch_query_wave(B, Bp, 0, y_lo, M, a->center, q64s[0], qps[0], nqs[0],
                                              a->amax, q16s[0], sq, r16 ? a->rot : nullptr)))
            return rc;
        for (int k = 1; k < K && t == 0; ++k) {
            const LevelRun &p = part[k - 1];
            if ((rc = launch_query_wave(p.B, p.Bp, 0, y_lo, M, p.a->center, p.ws.q64, p.ws.qp, p.ws.nq,
                                        p.a->amax, p.ws.q16, sq, r16 ? p.a->rot : nullptr)))
                return rc;
        }
        const XJob *jt = K > 1 ? ws.jtab : nullptr;
        ImgDb img{};
        const bool im = a->dbi != nullptr;
        IA_ARG(!im || img_db_layout(src.A.h, src.A.w, src.A.hs, src.A.ws, 1, a->row0, a->nrows, a->dbi, img,
                                    nullptr),
               "ia_synth_level: an image-form DB for a level it does not apply to");
        IA_ARG(im || a->db, "ia_synth_level: no DB (row form or image form)");
        float *segmin = match_segmin(ws.scratch);
        hipEvent_t e0 = timed ? prof_event(ev0 + 3 * nscreen) : nullptr;
        hipEvent_t e1 = timed ? prof_event(ev0 + 3 * nscreen + 1) : nullptr;
        if (e0) IA_HIP(hipEventRecord(e0, sq));
        const StageMap sm = db_stage_map(a->row0, a->nrows, src.A.w, src.A.h);
        if (r16) {
            if ((rc = launch_screen16r(a->dbr, a->nrows, sm, q16s[b], M, segmin, sq, jt, K, b)))
                return rc;
        } else if ((rc = launch_screen16(a->db, im ? &img : nullptr, a->nrows, sm, q16s[b], M, segmin, sq, jt,
                                         K, b, a->comm != nullptr))) {
            return rc;
        }
        if (e1) IA_HIP(hipEventRecord(e1, sq));
        int y_lo_n = 0, M_n = 0;
        if (t + 1 < nw) wave_rows(H, W, t + 1, y_lo_n, M_n);
        XArgs x{};
        x.src = src;
        x.im = img;
        x.db = a->db;
        x.row0 = a->row0;
        x.nrows = a->nrows;
        x.nseg = db_nsegs(a->nrows);
        x.seg_rows = db_seg_rows(a->nrows);
        x.smap = sm;
        x.segmin = segmin;
        x.q64 = q64s[b]; x.qp = qps[b]; x.nq = nqs[b];
        x.amax = a->amax;
        x.center = a->center;
        x.q64n = q64s[b ^ 1]; x.qpn = qps[b ^ 1]; x.nqn = nqs[b ^ 1]; x.q16n = q16s[b ^ 1];
        x.B = B;
        x.Bp = Bp;
        x.H = H; x.M = M; x.y_lo_n = y_lo_n; x.M_n = M_n;
        x.dbox = ws.dbox;
        x.tickets = ws.ctl;
        x.err = ws.ctl + XW_CTL_ERR;
        x.stats = prof ? ws.stats : nullptr;
        x.f = FinishArgs{t, y_lo, W, a->N_total, a->weights, a->kappa_factor, a->Bp_lg, a->s,
                         a->im, a->dbg_px, a->dbg_dist, nullptr, nullptr};
        if (peer) x.f.px = comm_peer_wave(a->comm);
        x.jobs = jt;
        x.trace = xw_trace(a->tag);
        x.rot = r16 ? a->rot : nullptr;
        x.askc = r16 ? r16_askc(a->dbr, a->nrows) : nullptr;
        const int R = M > y_lo_n + M_n - y_lo ? M : y_lo_n + M_n - y_lo;
        const int form = !im ? XW_ROWS
                       : (xwave_on() == 2 && sm.W > 0 && xstrip_applies(src)) ? XW_STRIP : XW_IMG;
        if ((rc = launch_xwave(x, R, form, sq, K))) return rc;
        if (timed) IA_HIP(hipEventRecord(prof_event(ev0 + 3 * nscreen + 2), sq));
        ++nscreen;
        pairs += (double)M * (double)a->nrows * K;
        if (prof) Ms.push_back(M);
        static const int sync_every = env_int("IA_SYNC_EVERY", 0);
        if (sync_every > 0 && t % sync_every == sync_every - 1) IA_HIP(hipStreamSynchronize(sq));
        return IA_OK;
    }

    // diagnostic: the sharded path with every shard's exact stage run here, one after the
    // other, each writing its records straight into the all-ranks array; then k_finish
    int sim_wave(int t, int y_lo, int M, hipStream_t sq) {
        int rc;
        for (int r = 0; r < nsim; ++r) {
            if ((rc = launch_query_wave(B, Bp, t, y_lo, M, a->center, ws.q64, ws.qp, ws.nq,
                                        sim[r].amax, ws.q16, sq)))
                return rc;
            const FinishArgs fr{t, y_lo, W, a->N_total, a->weights, a->kappa_factor, a->Bp_lg,
                                a->s, a->im, a->dbg_px, a->dbg_dist, ws.rec_all + (long)r * M,
                                ws.coh};
            if ((rc = launch_match(src, sim[r].row0, sim[r].nrows, sim[r].db, sim[r].dbi, ws.qp, ws.q16, M,
                                   ws.q64, ws.nq, sim[r].amax, ws.scratch, ws.best_local, nullptr,
                                   sq, nullptr, nullptr, &fr)))
                return rc;
        }
        const FinishArgs fa{t, y_lo, W, a->N_total, a->weights, a->kappa_factor, a->Bp_lg, a->s,
                            a->im, a->dbg_px, a->dbg_dist, nullptr, nullptr};
        k_finish<<<M, 64, 0, sq>>>(src, ws.rec_all, ws.coh, nsim, M, fa);
        IA_LAUNCH_CHECK("k_finish");
        return IA_OK;
    }

    int done(hipStream_t st) {
        if (xw) {
            k_err_sticky<<<1, 64, 0, st>>>(ws.ctl, K > 1 ? ws.jtab : nullptr, K);
            IA_HIP(hipGetLastError());
        }
        if (prof) {   // read back by ia_prof_end (no synchronisation here)
            IA_HIP(hipMemcpyAsync(hstats, ws.stats, STATS_BYTES, hipMemcpyDeviceToHost, st));
            prof_push(ProfRec{a->tag, K, a->nrows, pairs, ev0, nscreen, timed ? 1 : 0, hstats,
                              std::move(Ms)});
        }
        return IA_OK;
    }
};

// ---- pipelined levels (ia_synth_levels) ---------------------------------------------
// Level l's wave t reads the coarse level l-1 only through the 3x3 coarse windows of its
// pixels: coarse pixels up to (y/2 + 1, x/2 + 1), i.e. coarse waves <= need(t) =
// max over the wave's pixels of min(x/2 + 1, W'-1) + 3 min(y/2 + 1, H'-1) (the mirror at
// the coarse level's far edges stays inside that box).  So level l may start as soon as
// level l-1 has finished need(0) and run concurrently behind it on its own stream: the
// step's critical path becomes ~ the finest level's waves instead of the sum of all
// levels' waves.  Levels wait on events recorded every PIPE_BLOCK waves of the level below.
// waves per recorded event (build-time IA_PIPE_BLOCK).  8 against 4, same boxes, two
// rounds: c1 14.73-15.07 vs 14.93-15.19, c3 69.2-70.7 vs 69.9-72.3, c4 734-743 vs 735-744
// ms/step; 2 is slower (c1 16.1), 16 mixed (profiles/r06_pipe_block_ab.txt)
#ifndef IA_PIPE_BLOCK
#define IA_PIPE_BLOCK 8
#endif
constexpr int PIPE_BLOCK = IA_PIPE_BLOCK;
// waves a coarse level is enqueued ahead of its need (IA_PIPE_AHEAD, default 16): every
// coarse wave enqueued before the finest level's first costs ~10 us of host time; same box,
// two passes: c1 16.22 / 16.30 (64), 15.99 / 15.95 (32), 15.24 / 15.12 (16), 15.55 / 15.72 (8)
// ms/step, c3 1 % better at 16-32, c4 unchanged (profiles/r06_pipe_ahead_sweep.txt)
static int pipe_ahead() {
    static const int v = env_int("IA_PIPE_AHEAD", 16);
    return v < 0 ? 0 : v;
}

static int coarse_need(const IaSynthArgs *a, int t) {
    int y_lo, M;
    LevelRun::wave_rows(a->H, a->W, t, y_lo, M);
    const int Hc = a->B_hs, Wc = a->B_ws;
    int need = 0;
    for (int y = y_lo; y < y_lo + M; ++y) {
        const int x = t - 3 * y;
        const int cy = y / 2 + 1 < Hc - 1 ? y / 2 + 1 : Hc - 1;
        const int cx = x / 2 + 1 < Wc - 1 ? x / 2 + 1 : Wc - 1;
        need = cx + 3 * cy > need ? cx + 3 * cy : need;
    }
    return need;
}

struct PipeRes {   // per host thread: the level streams and events of ia_synth_levels
    std::vector<hipStream_t> streams;   // levels 0 .. n-2 of a call (coarser): high priority
    hipStream_t plain = nullptr;        // level n-1 of a call (the finest): plain priority
    std::vector<hipEvent_t> events;
    size_t next_event = 0;
    // pinned staging of the batch job tables: reused after the previous call's copies ran
    void *pin = nullptr;
    size_t pin_bytes = 0;
    hipEvent_t staged = nullptr;
    bool staged_rec = false;
    hipEvent_t last = nullptr;          // the previous call's end (on its caller's stream)
    bool last_rec = false;
    hipError_t staging(size_t bytes, void **p) {
        hipError_t r = hipSuccess;
        if (!staged && (r = hipEventCreateWithFlags(&staged, hipEventDisableTiming)) != hipSuccess) return r;
        if (staged_rec && (r = hipEventSynchronize(staged)) != hipSuccess) return r;
        if (bytes > pin_bytes) {
            if (pin && (r = hipHostFree(pin)) != hipSuccess) return r;
            pin = nullptr;
            if ((r = hipHostMalloc(&pin, bytes, hipHostMallocDefault)) != hipSuccess) return r;
            pin_bytes = bytes;
        }
        staged_rec = true;
        *p = pin;
        return r;
    }
    hipError_t event(hipEvent_t *e) {
        if (next_event == events.size()) {
            hipEvent_t x;
            hipError_t r = hipEventCreateWithFlags(&x, hipEventDisableTiming);
            if (r != hipSuccess) return r;
            events.push_back(x);
        }
        *e = events[next_event++];
        return hipSuccess;
    }
};
static thread_local PipeRes g_pipe;

}  // namespace ia

using namespace ia;

extern "C" {

int ia_diag_xwave_trace(unsigned long long *out) {
    IA_ARG(out && g_xw_trace, "ia_diag_xwave_trace: no trace (IA_XW_TRACE=<level>)");
    IA_HIP(hipDeviceSynchronize());
    IA_HIP(hipMemcpy(out, g_xw_trace, (size_t)XW_TRACE_T * XW_TRACE_PX * XW_TRACE_N * 8,
                     hipMemcpyDeviceToHost));
    return IA_OK;
}

int ia_diag_set_xwave(int on) {
    const int prev = xwave_on();
    if (on >= 0 && on <= 2) g_xwave.store(on);
    return prev;
}

int ia_level_resources(const IaSynthArgs *a, int *out) {
    // the kernels this level launches per wave, decided as LevelRun::init / xw_wave decide:
    // out = {waiting kernel LDS bytes, VGPRs; screen LDS bytes, VGPRs} (the forward-progress
    // rule of DESIGN.md §7, per level: ADVICE r05)
    IA_ARG(a && out && a->nrows > 0, "ia_level_resources: bad args");
    const bool peer = a->comm && comm_peer_mcap(a->comm) > 0;
    const bool xw = xwave_on() && !a->lsh && (!a->comm || peer) && exact_stage_mode() != 1;
    const bool r16 = xw && a->dbr && a->rot;
    const bool im = a->dbi != nullptr;
    const DbSrc src = make_dbsrc(a->src);
    const StageMap sm = db_stage_map(a->row0, a->nrows, src.A.w, src.A.h);
    hipFuncAttributes f{}, sc{};
    int rc;
    if (xw) {
        const int form = !im ? XW_ROWS : (xwave_on() == 2 && sm.W > 0 && xstrip_applies(src)) ? XW_STRIP : XW_IMG;
        rc = xwave_attributes(form, r16, &f);
    } else {
        IA_HIP(hipFuncGetAttributes(&f, reinterpret_cast<const void *>(&k_peer_finish)));
        rc = IA_OK;
    }
    if (rc) return rc;
    rc = r16 ? screen_resources_r16(&sc) : screen16_attributes(im, &sc);
    if (rc) return rc;
    out[0] = (int)f.sharedSizeBytes;
    out[1] = f.numRegs;
    out[2] = (int)sc.sharedSizeBytes;
    out[3] = sc.numRegs;
    return IA_OK;
}

int ia_synth_status(const IaSynthArgs *levels, int n, void *stream) {
    IA_ARG(levels && n >= 1, "ia_synth_status: bad args");
    IA_HIP(hipStreamSynchronize(S(stream)));
    for (int j = 0; j < n; ++j) {
        const IaSynthArgs &a = levels[j];
        IA_ARG(a.workspace && a.H > 0 && a.W > 0 && a.nrows > 0, "ia_synth_status: bad level");
        SynthWs w;
        carve(&w, reinterpret_cast<char *>(a.workspace), a.H, a.W, a.nrows, comm_nranks(a.comm));
        unsigned int e = 0;
        IA_HIP(hipMemcpy(&e, w.ctl + XW_CTL_ERR, sizeof(e), hipMemcpyDeviceToHost));
        if (e) {
            set_error("ia_synth_status: a wait for a neighbouring pixel's decision timed out "
                      "(device schedule fault)");
            return IA_E_SCHED;
        }
        if (comm_peer_mcap(a.comm) > 0) {
            const int rc = ia_peer_status(a.comm);
            if (rc) return rc;
        }
    }
    return IA_OK;
}

int ia_sched_status(int clear) {
    IA_HIP(hipDeviceSynchronize());
    unsigned int e = 0;
    IA_HIP(hipMemcpyFromSymbol(&e, HIP_SYMBOL(g_sched_err), sizeof(e), 0, hipMemcpyDeviceToHost));
    if (clear && e) {
        const unsigned int z = 0;
        IA_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_sched_err), &z, sizeof(z), 0, hipMemcpyHostToDevice));
    }
    if (e) {
        set_error("ia_sched_status: a wait for a neighbouring pixel's decision timed out in some "
                  "level since the last clear (device schedule fault)");
        return IA_E_SCHED;
    }
    return IA_OK;
}

int ia_diag_set_graph_mode(int mode) {
    const int prev = graph_mode();
    if (mode >= 0 && mode <= 2) g_graph_mode.store(mode);
    return prev;
}

int ia_release_thread_resources(void) {
    IA_HIP(g_graphs.retire());
    IA_HIP(hipDeviceSynchronize());
    for (hipStream_t s : g_pipe.streams) IA_HIP(hipStreamDestroy(s));
    if (g_pipe.plain) IA_HIP(hipStreamDestroy(g_pipe.plain));
    g_pipe.plain = nullptr;
    for (hipEvent_t e : g_pipe.events) IA_HIP(hipEventDestroy(e));
    g_pipe.streams.clear();
    {
        const int rc = release_pipe3();
        if (rc) return rc;
    }
    g_pipe.events.clear();
    if (g_pipe.pin) IA_HIP(hipHostFree(g_pipe.pin));
    if (g_pipe.staged) IA_HIP(hipEventDestroy(g_pipe.staged));
    g_pipe.pin = nullptr;
    g_pipe.pin_bytes = 0;
    g_pipe.staged = nullptr;
    g_pipe.staged_rec = false;
    if (g_pipe.last) IA_HIP(hipEventDestroy(g_pipe.last));
    g_pipe.last = nullptr;
    g_pipe.last_rec = false;
    g_pipe.next_event = 0;
    if (g_graphs.cap) { IA_HIP(hipStreamDestroy(g_graphs.cap)); g_graphs.cap = nullptr; }
    if (g_graphs.done) { IA_HIP(hipEventDestroy(g_graphs.done)); g_graphs.done = nullptr; }
    return IA_OK;
}

int ia_prof_begin(void) {
    std::lock_guard<std::mutex> l(g_prof->mu);
    g_prof->active = true;
    g_prof->next = 0;
    g_prof->pinned_next = 0;
    g_prof->recs.clear();
    return IA_OK;
}

int ia_prof_prepare(long nevents) {
    std::lock_guard<std::mutex> l(g_prof->mu);
    while ((long)g_prof->ev.size() < nevents) {
        hipEvent_t e;
        IA_HIP(hipEventCreate(&e));
        g_prof->ev.push_back(e);
    }
    return IA_OK;
}

int ia_prof_launches(int rec, float *ms, int *M, int max) {
    std::lock_guard<std::mutex> l(g_prof->mu);
    IA_ARG(rec >= 0 && rec < (int)g_prof->recs.size(), "ia_prof_launches: no such record");
    const ProfRec &p = g_prof->recs[rec];
    const int n = p.timed ? p.nscreen : 0;
    for (int i = 0; i < n && i < max; ++i) {
        if (ms) IA_HIP(hipEventElapsedTime(&ms[i], g_prof->ev[p.ev0 + 3 * i], g_prof->ev[p.ev0 + 3 * i + 1]));
        if (M) M[i] = p.M[i];
    }
    return n;
}

int ia_prof_waves(int rec, float *tail_ms, float *gap_ms, int max) {
    std::lock_guard<std::mutex> l(g_prof->mu);
    IA_ARG(rec >= 0 && rec < (int)g_prof->recs.size(), "ia_prof_waves: no such record");
    const ProfRec &p = g_prof->recs[rec];
    const int n = p.timed ? p.nscreen : 0;
    for (int i = 0; i < n && i < max; ++i) {
        const size_t e = p.ev0 + 3 * i;
        if (tail_ms) IA_HIP(hipEventElapsedTime(&tail_ms[i], g_prof->ev[e + 1], g_prof->ev[e + 2]));
        if (gap_ms) {
            gap_ms[i] = 0.f;
            if (i + 1 < n) IA_HIP(hipEventElapsedTime(&gap_ms[i], g_prof->ev[e + 2], g_prof->ev[e + 3]));
        }
    }
    return n;
}

int ia_prof_end(double *out, int maxrec) {
    IA_HIP(hipDeviceSynchronize());
    std::lock_guard<std::mutex> l(g_prof->mu);
    g_prof->active = false;
    const int n = (int)g_prof->recs.size();
    for (int r = 0; r < n && r < maxrec && out; ++r) {
        const ProfRec &p = g_prof->recs[r];
        double ms = 0.0;
        for (int i = 0; p.timed && i < p.nscreen; ++i) {
            float e = 0.f;
            IA_HIP(hipEventElapsedTime(&e, g_prof->ev[p.ev0 + 3 * i], g_prof->ev[p.ev0 + 3 * i + 1]));
            ms += e;
        }
        unsigned long long st[STATS_LINE] = {};
        for (int sl = 0; sl < STATS_SLOTS; ++sl)
            for (int i = 0; i < STATS_LINE; ++i) st[i] += p.hstats[sl * STATS_LINE + i];
        double *o = out + (size_t)r * IA_PROF_FIELDS;
        o[0] = p.tag;
        o[1] = (double)p.nrows;
        o[2] = p.pairs;
        o[3] = p.timed ? ms : 0.0;
        o[4] = p.timed ? p.nscreen : 0;
        o[5] = (double)st[0];
        o[6] = (double)st[1];
        o[7] = (double)st[2];
        o[8] = (double)st[3] * 1e-2;   // 100 MHz ticks -> us
        o[9] = (double)st[4] * 1e-2;
        o[10] = p.jobs;
    }
    return n;
}

size_t ia_synth_workspace_bytes(int H, int W, long nrows, int nranks) {
    if (H <= 0 || W <= 0 || nrows <= 0 || nranks <= 0) return 0;
    return carve(nullptr, nullptr, H, W, nrows, nranks);
}

int ia_synth_level(const IaSynthArgs *a, void *stream) {
    hipStream_t st = S(stream);
    LevelRun run;
    int rc = run.init(a, st);
    if (rc) return rc;
    // HIP-graph capture of the whole wave loop (IA_GRAPH / ia_diag_set_graph_mode: 0 off
    // [default], 1 levels of <= 2^18 rows, 2 every single-GPU level).  Sharded levels stay
    // eager (RCCL calls per wave).  Launches inside a graph are not timed.
    const int gm = graph_mode();
    const bool use_graph = !a->comm && !(a->flags & IA_SYNTH_EAGER) &&
                           (gm == 2 || (gm == 1 && a->nrows <= (1L << 18)));
    if (!use_graph) {
        for (int t = 0; t < run.nw; ++t)
            if ((rc = run.wave(t, st))) return rc;
    } else {
        // capture on a private stream (the legacy default stream cannot capture)
        run.timed = false;
        IA_HIP(g_graphs.retire());
        if (!g_graphs.cap) IA_HIP(hipStreamCreateWithFlags(&g_graphs.cap, hipStreamNonBlocking));
        IA_HIP(hipStreamBeginCapture(g_graphs.cap, hipStreamCaptureModeThreadLocal));
        for (int t = 0; t < run.nw && !rc; ++t) rc = run.wave(t, g_graphs.cap);
        hipGraph_t graph = nullptr;
        const hipError_t ec = hipStreamEndCapture(g_graphs.cap, &graph);
        if (rc) { if (graph) (void)hipGraphDestroy(graph); return rc; }
        IA_HIP(ec);
        hipGraphExec_t exec = nullptr;
        const hipError_t ei = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
        (void)hipGraphDestroy(graph);
        IA_HIP(ei);
        IA_HIP(hipGraphLaunch(exec, st));
        IA_HIP(g_graphs.hold(exec, st));
    }
    return run.done(st);
}

int ia_diag_synth_level_shards(const IaSynthArgs *a, const IaShardDb *shards, int n,
                               void *stream) {
    IA_ARG(a && shards && n >= 1 && !a->comm && !a->lsh, "ia_diag_synth_level_shards: bad args");
    long total = 0;
    for (int r = 0; r < n; ++r) {
        IA_ARG((shards[r].db || shards[r].dbi) && shards[r].amax && shards[r].row0 == total && shards[r].nrows > 0,
               "ia_diag_synth_level_shards: shards must tile the rows in order");
        total += shards[r].nrows;
    }
    IA_ARG(total == a->N_total, "ia_diag_synth_level_shards: shards must cover the DB");
    hipStream_t st = S(stream);
    LevelRun run;
    run.sim = shards;
    run.nsim = n;
    int rc = run.init(a, st);
    if (rc) return rc;
    for (int t = 0; t < run.nw; ++t)
        if ((rc = run.wave(t, st))) return rc;
    return run.done(st);
}

// n consecutive levels of K identical-shape jobs (levels[j * K + k]: level j of job k)
static int synth_levels(const IaSynthArgs *levels, int n, int K, void *stream) {
    IA_ARG(levels && n >= 1 && n <= 64 && K >= 1 && K <= IA_BATCH_MAX, "ia_synth_levels: bad level count");
    auto lv = [&](int j) -> const IaSynthArgs & { return levels[(size_t)j * K]; };
    for (int j = 1; j < n; ++j)
        for (int k = 0; k < K; ++k)
            IA_ARG(levels[(size_t)j * K + k].Bp_sm == levels[(size_t)(j - 1) * K + k].Bp_lg &&
                       levels[(size_t)j * K + k].B_hs == levels[(size_t)(j - 1) * K + k].H &&
                       levels[(size_t)j * K + k].B_ws == levels[(size_t)(j - 1) * K + k].W,
                   "ia_synth_levels: levels must be consecutive (level j's coarse B' = level j-1's B')");
    hipStream_t st = S(stream);
    // one stream per level; coarser levels at high priority (IA_PIPE_PRIO, default 1) so
    // that they run ahead of the finest level instead of time-sharing with it.  Measured
    // (c4, one box, `tools/gpu.sh abknob`): one level at a time 1706-1713 ms/step; pipelined
    // with the coarse levels enqueued whole first at high priority 1641-1643 ms (the finest
    // level's plateau screens undisturbed: k_screen16<11> 400 vs 396 us); enqueued just
    // ahead of their need 1619-1621 ms but the plateau screens contended (414 us)
    static const int prio_on = env_int("IA_PIPE_PRIO", 1);
    // a call waits on the host for this thread's previous call to end (IA_PIPE_DRAIN,
    // default 1) before it enqueues anything.  Queued behind a running call, the coarse
    // levels' first packets (their waits on `start`) sit in the high-priority queues for the
    // whole of the previous call's finest level, and while they do the finest level's
    // launches run ~4x slower (c1 with no host sync between steps: 61 vs 15 ms/step, screens
    // 39 vs 9.4 us; IA_PIPE_PRIO=0 18 ms; profiles/r06_pipe_drain_ab.txt).  The host's other
    // per-call work (the level indexes) still overlaps the previous call
    static const int drain = env_int("IA_PIPE_DRAIN", 1);
    if (drain && g_pipe.last_rec) IA_HIP(hipEventSynchronize(g_pipe.last));
    // the pools grow as needed; the finest level always takes the plain-priority stream,
    // whatever n the first call had (a pool sized by a smaller first call used to hand a
    // later call's coarse level a plain stream and its finest a high-priority one)
    while ((int)g_pipe.streams.size() < n - 1) {
        int lo = 0, hi = 0;
        IA_HIP(hipDeviceGetStreamPriorityRange(&lo, &hi));
        hipStream_t s;
        if (prio_on)
            IA_HIP(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, hi));
        else
            IA_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        (void)lo;
        g_pipe.streams.push_back(s);
    }
    if (!g_pipe.plain) IA_HIP(hipStreamCreateWithFlags(&g_pipe.plain, hipStreamNonBlocking));
    auto level_stream = [&](int j) { return j == n - 1 ? g_pipe.plain : g_pipe.streams[j]; };
    g_pipe.next_event = 0;
    hipEvent_t start;
    IA_HIP(g_pipe.event(&start));
    IA_HIP(hipEventRecord(start, st));
    // the batch job tables go through a pinned host buffer kept by this thread (reused once
    // the previous call's copies have run)
    XJob *pinned = nullptr;
    if (K > 1) {
        IA_HIP(g_pipe.staging((size_t)n * K * sizeof(XJob), reinterpret_cast<void **>(&pinned)));
    }
    std::vector<LevelRun> run(n);
    std::vector<std::vector<hipEvent_t>> blk(n);   // blk[j][b]: level j done through block b
    std::vector<int> next(n, 0), waited(n, -1), need_max(n, 0);
    for (int j = 0; j < n; ++j) {
        hipStream_t sj = level_stream(j);
        IA_HIP(hipStreamWaitEvent(sj, start, 0));
        int rc = run[j].init_batch(&levels[(size_t)j * K], K, sj, pinned + (size_t)j * K);
        if (rc) return rc;
        blk[j].assign((run[j].nw + PIPE_BLOCK - 1) / PIPE_BLOCK, nullptr);
    }
    // enqueue level j through wave `target` (and the coarse waves it needs, first)
    // Levels whose DB is sharded over several ranks and exchanged over RCCL never overlap
    // one another: each one's first wave waits for the previous such level's last.  RCCL's
    // kernels wait in-kernel for the other ranks, and two communicators in flight on
    // different streams can deadlock when the waiting kernels hold the CUs the awaited
    // ones need.  The same held for the first device-side exchange, whose waits sat inside
    // the exact stage's 4-wave, 250-VGPR workgroups (two bench ranks on one GPU deadlocked
    // on c3 with the levels pipelined).  Its waits now live in k_peer_finish's small 2-wave
    // workgroups (c4: at most (171 + 342) x 2 waves of 152 VGPRs when two sharded levels
    // overlap, a quarter of a GPU's wave slots), so those levels overlap: 3 ranks sharing
    // one GPU with every c3 level sharded and overlapping complete, and the simulated
    // G = 8 rank gains 3.6 % (profiles/r02_shard_overlap.txt).  IA_SHARD_OVERLAP=0
    // serializes them too.
    // Ranks sharing ONE GPU (IA_SHARE_GPU=1, the tests' multi-rank mode) serialize them as
    // well: their waiting workgroups (k_xwave's, up to ~343 per level and rank) could then
    // fill the one GPU's slots while a third rank's awaited ones cannot start.
    static const int overlap = env_int("IA_SHARD_OVERLAP", 1) && !env_int("IA_SHARE_GPU", 0);
    auto multi_rank = [&](int j) {
        if (lv(j).comm == nullptr || lv(j).nrows >= lv(j).N_total) return false;
        return !(overlap && comm_peer_mcap(lv(j).comm) > 0);
    };
    std::function<int(int, int)> advance;
    advance = [&](int j, int target) -> int {
        hipStream_t sj = level_stream(j);
        if (target > run[j].nw - 1) target = run[j].nw - 1;
        if (next[j] == 0 && target >= 0 && multi_rank(j)) {
            for (int i = j - 1; i >= 0; --i) {
                if (!multi_rank(i)) continue;
                int rc = advance(i, run[i].nw - 1);
                if (rc) return rc;
                IA_HIP(hipStreamWaitEvent(sj, blk[i].back(), 0));
                break;
            }
        }
        while (next[j] <= target) {
            const int t = next[j];
            if (j > 0) {
                // on the fused path wave t's launch also builds wave t + 1's query rows
                int w = coarse_need(&lv(j), run[j].xw && t + 1 < run[j].nw ? t + 1 : t);
                need_max[j] = w > need_max[j] ? w : need_max[j];
                w = need_max[j];
                if (w > waited[j]) {
                    const int b = w / PIPE_BLOCK;
                    int rc = advance(j - 1, b * PIPE_BLOCK + PIPE_BLOCK - 1 + pipe_ahead());
                    if (rc) return rc;
                    IA_HIP(hipStreamWaitEvent(sj, blk[j - 1][b], 0));
                    waited[j] = b * PIPE_BLOCK + PIPE_BLOCK - 1;
                }
            }
            int rc = run[j].wave(t, sj);
            if (rc) return rc;
            if ((t + 1) % PIPE_BLOCK == 0 || t == run[j].nw - 1) {
                hipEvent_t e;
                IA_HIP(g_pipe.event(&e));
                IA_HIP(hipEventRecord(e, sj));
                blk[j][t / PIPE_BLOCK] = e;
            }
            ++next[j];
        }
        return IA_OK;
    };
    // enqueue order (IA_PIPE_ORDER): 0 [default] the finest level first, coarse waves just
    // ahead of their need; 1 every level whole, coarse to fine.  One host thread enqueues
    // ~10 us of launches per wave, so with 1 the finest level's first wave was enqueued only
    // after every coarse wave (c1: at +14 ms of a 27 ms traced step, tools/trace_queues.py).
    // Same box, round 6: c1 18.51 -> 16.30, c3 76.0 -> 71.3, c4 783.7 -> 750.8, c5 794 -> 786
    // ms/step (profiles/r06_pipe_order_ab.txt)
    static const int order = env_int("IA_PIPE_ORDER", 0);
    for (int i = 0; i < n; ++i) {
        const int j = order ? i : n - 1 - i;
        int rc = advance(j, run[j].nw - 1);
        if (rc) return rc;
    }
    for (int j = 0; j < n; ++j) {
        hipStream_t sj = level_stream(j);
        int rc = run[j].done(sj);
        if (rc) return rc;
        hipEvent_t e;
        IA_HIP(g_pipe.event(&e));
        IA_HIP(hipEventRecord(e, sj));
        IA_HIP(hipStreamWaitEvent(st, e, 0));
    }
    if (pinned) IA_HIP(hipEventRecord(g_pipe.staged, st));
    if (!g_pipe.last) IA_HIP(hipEventCreateWithFlags(&g_pipe.last, hipEventDisableTiming));
    IA_HIP(hipEventRecord(g_pipe.last, st));
    g_pipe.last_rec = true;
    return IA_OK;
}

int ia_synth_levels(const IaSynthArgs *levels, int n, void *stream) { return synth_levels(levels, n, 1, stream); }

int ia_synth_levels_batch(const IaSynthArgs *levels, int n, int K, void *stream) {
    return synth_levels(levels, n, K, stream);
}

}  // extern "C"
