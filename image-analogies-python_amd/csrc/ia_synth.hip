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
//   k_query_wave  -> q64 / qp / nq       (ia_features.hip)
//   k_screen_seg  -> segment minima     (ia_match.hip, MFMA)
//   k_rescore     -> best (this shard)   (ia_match.hip, exact fp64)
//   [RCCL all-gather of best over ranks when the DB is sharded]
//   k_finish      -> coherence, kappa test, B'/s/im update (this file)
#include "ia_internal.h"

#include <vector>

#include <rccl/rccl.h>

namespace ia {

__device__ __forceinline__ void best_upd(double &bd, long long &bi, double d, long long i) {
    if (d < bd || (d == bd && i < bi)) { bd = d; bi = i; }
}

// one wave per query pixel
__global__ __launch_bounds__(64) void k_finish(DbSrc src, const Best *__restrict__ best_all,
                                               int nranks, int M, int t, int y_lo, int W,
                                               long N_total,
                                               const double *__restrict__ q64,
                                               const double *__restrict__ weights,
                                               double kappa_factor,
                                               double *__restrict__ Bp_lg,
                                               int32_t *__restrict__ s,
                                               int32_t *__restrict__ im) {
    __shared__ double qs[IA_DP];
    const int m = blockIdx.x;
    const int y = y_lo + m, x = t - 3 * y;
    const int lane = threadIdx.x;
    if (lane < IA_DP) qs[lane] = q64[(long)m * IA_DP + lane];
    __syncthreads();

    // p_app: lexicographic (dist, row) minimum over the shards' exact winners
    double ad = INFINITY;
    long long app = 0x7fffffffffffffffLL;
    for (int g = 0; g < nranks; ++g) {
        const Best b = best_all[(long)g * M + m];
        best_upd(ad, app, b.d, b.idx);
    }
    const int Ah = src.A.h, Aw = src.A.w;
    const long hw = src.hw;
    if (app < 0 || app >= N_total) app = 0;   // unreachable: every merge has a winner
    long img = app / hw;
    long rem = app - img * hw;
    int pr = (int)(rem / Aw), pc = (int)(rem - (long)(rem / Aw) * Aw);

    if (y != 0 || x != 0) {
        // best_coherence_match (algorithms.py:92-130): lanes 0..14 = 3x5 causal window,
        // row-major = the reference's product(rows, cols) order
        double cd = INFINITY;
        long long cl = 0x7fffffffffffffffLL;
        long cix = -1;
        int cr = 0, cc = 0, cim = 0;
        if (lane < 15) {
            const int rr = y - 2 + lane / 5, rc = x - 2 + lane % 5;
            if (rr >= 0 && rc >= 0 && rc < W && (rr < y || rc < x)) {
                const long sidx = (long)rr * W + rc;
                const int sr = s[2 * sidx] + y - rr, sc = s[2 * sidx + 1] + x - rc;
                if (sr >= 0 && sr < Ah && sc >= 0 && sc < Aw) {
                    const int simg = im[sidx];
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
            best_upd(bd, bl, od, ol);
        }
        if (bl != 0x7fffffffffffffffLL) {
            const int win = (int)bl;
            const long wix = __shfl(cix, win);
            const int wr = __shfl(cr, win), wc = __shfl(cc, win), wim = __shfl(cim, win);
            // kappa test (image_analogies.py:200-211), lane 0: d_app, lane 1: d_coh
            double d = 0.0;   // one inlined copy of the gather (instruction-cache footprint)
            if (lane < 2) d = row_wdist(src, lane == 0 ? app : wix, qs, weights);
            const double d_app = __shfl(d, 0), d_coh = __shfl(d, 1);
            if (d_coh <= d_app * kappa_factor) {
                pr = wr; pc = wc; img = wim;
            }
        }
    }
    if (lane == 0) {
        const long q = (long)y * W + x;
        Bp_lg[q] = src.Ap.lg[img * hw + (long)pr * Aw + pc];
        s[2 * q] = pr;
        s[2 * q + 1] = pc;
        im[q] = (int32_t)img;
    }
}

// -------------------------------- workspace ----------------------------------------
struct SynthWs {
    double *q64;
    float *qp;
    double *nq;
    void *scratch;           // screen output (candidates or segment minima)
    Best *best_local;
    Best *best_all;
    unsigned long long *stats;
};

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
    w.nq = (double *)take((size_t)qr * sizeof(double));
    w.scratch = take(match_scratch_bytes(qr, nrows));
    w.best_local = (Best *)take((size_t)Mmax * sizeof(Best));
    w.best_all = (Best *)take((size_t)Mmax * nranks * sizeof(Best));
    w.stats = (unsigned long long *)take(8 * sizeof(unsigned long long));
    if (ws) *ws = w;
    return off;
}

struct EventPool {
    std::vector<hipEvent_t> ev;
    int get(size_t n) {
        while (ev.size() < n) {
            hipEvent_t e;
            if (hipEventCreate(&e) != hipSuccess) return -1;
            ev.push_back(e);
        }
        return 0;
    }
};
static thread_local EventPool g_events;

int comm_allgather_best(void *comm, const Best *send, Best *recv, int M, hipStream_t st);
int comm_nranks(void *comm);

}  // namespace ia

using namespace ia;

extern "C" {

size_t ia_synth_workspace_bytes(int H, int W, long nrows, int nranks) {
    if (H <= 0 || W <= 0 || nrows <= 0 || nranks <= 0) return 0;
    return carve(nullptr, nullptr, H, W, nrows, nranks);
}

int ia_synth_level(const IaSynthArgs *a, void *stream) {
    IA_ARG(a && a->db && a->center && a->amax && a->B_sm && a->B_lg && a->Bp_sm && a->Bp_lg &&
               a->weights && a->s && a->im && a->workspace,
           "ia_synth_level: null argument");
    IA_ARG(a->H > 0 && a->W > 0 && a->nrows > 0 && a->row0 >= 0 &&
               a->row0 + a->nrows <= a->N_total,
           "ia_synth_level: bad sizes");
    IA_ARG(a->N_total == (long)a->src.nAp * a->src.Ah * a->src.Aw, "ia_synth_level: N_total mismatch");
    IA_ARG(a->B_hs == (a->H + 1) / 2 && a->B_ws == (a->W + 1) / 2, "ia_synth_level: B level shapes");
    IA_ARG(a->src.A_hs == (a->src.Ah + 1) / 2 && a->src.A_ws == (a->src.Aw + 1) / 2,
           "ia_synth_level: A level shapes");
    const int nranks = a->comm ? comm_nranks(a->comm) : 1;
    IA_ARG(nranks >= 1, "ia_synth_level: bad communicator");
    hipStream_t st = S(stream);
    const int H = a->H, W = a->W;
    SynthWs ws;
    carve(&ws, reinterpret_cast<char *>(a->workspace), H, W, a->nrows, nranks);
    const int Mmax = wave_max_queries(H, W);
    IA_HIP(hipMemsetAsync(ws.qp, 0, (size_t)qrows_alloc(Mmax) * IA_DP * sizeof(float), st));
    IA_HIP(hipMemsetAsync(ws.stats, 0, 8 * sizeof(unsigned long long), st));

    const DbSrc src = make_dbsrc(a->src);
    const ImgPair B{a->B_sm, a->B_lg, a->B_hs, a->B_ws, H, W};
    const ImgPair Bp{a->Bp_sm, a->Bp_lg, a->B_hs, a->B_ws, H, W};
    const int nw = (W - 1) + 3 * (H - 1) + 1;
    const bool prof = a->prof != nullptr;
    if (prof && g_events.get(2 * (size_t)nw)) { set_error("hipEventCreate failed"); return IA_E_HIP; }
    double pairs = 0.0;
    int nscreen = 0;
    for (int t = 0; t < nw; ++t) {
        const int lo_num = t - (W - 1);
        const int y_lo = lo_num > 0 ? (lo_num + 2) / 3 : 0;
        const int y_hi = t / 3 < H - 1 ? t / 3 : H - 1;
        const int M = y_hi - y_lo + 1;
        if (M <= 0) continue;
        int rc;
        if ((rc = launch_query_wave(B, Bp, t, y_lo, M, a->center, ws.q64, ws.qp, ws.nq, st)))
            return rc;
        hipEvent_t e0 = prof ? g_events.ev[2 * nscreen] : nullptr;
        hipEvent_t e1 = prof ? g_events.ev[2 * nscreen + 1] : nullptr;
        if (a->lsh) {   // approximate matcher: the events bracket the LSH query kernel
            if (e0) IA_HIP(hipEventRecord(e0, st));
            if ((rc = launch_lsh_match(a->lsh, src, a->row0, a->nrows, M, ws.q64, a->center,
                                       ws.best_local, prof ? ws.stats : nullptr, st)))
                return rc;
            if (e1) IA_HIP(hipEventRecord(e1, st));
        } else if ((rc = launch_match(src, a->row0, a->nrows, a->db, ws.qp, M, ws.q64, ws.nq,
                                      a->amax, ws.scratch, ws.best_local,
                                      prof ? ws.stats : nullptr, st, e0, e1))) {
            return rc;
        }
        ++nscreen;
        pairs += (double)M * (double)a->nrows;
        const Best *ball = ws.best_local;
        if (a->comm) {   // also with one rank: the same RCCL path, exercised by the tests
            if ((rc = comm_allgather_best(a->comm, ws.best_local, ws.best_all, M, st))) return rc;
            ball = ws.best_all;
        }
        k_finish<<<M, 64, 0, st>>>(src, ball, nranks, M, t, y_lo, W, a->N_total, ws.q64, a->weights,
                                   a->kappa_factor, a->Bp_lg, a->s, a->im);
        IA_LAUNCH_CHECK("k_finish");
    }
    if (prof) {
        IA_HIP(hipStreamSynchronize(st));
        double ms = 0.0;
        for (int i = 0; i < nscreen; ++i) {
            float e = 0.f;
            IA_HIP(hipEventElapsedTime(&e, g_events.ev[2 * i], g_events.ev[2 * i + 1]));
            ms += e;
        }
        unsigned long long st_h[8];
        IA_HIP(hipMemcpy(st_h, ws.stats, sizeof(st_h), hipMemcpyDeviceToHost));
        a->prof[0] = ms;
        a->prof[1] = nscreen;
        a->prof[2] = pairs;
        a->prof[3] = (double)st_h[0];
        a->prof[4] = (double)st_h[1];
        a->prof[5] = (double)st_h[2];
    }
    return IA_OK;
}

}  // extern "C"
