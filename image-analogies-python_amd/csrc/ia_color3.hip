// ia_color3.hip — 3-channel matching (the reference's convert=False on colour images:
// config.py:29-42 num_ch = 3, algorithms.py:11-47 with channel-interleaved windows).
//
// Each feature row has 165 values: [A coarse 3x3x3 | A fine 5x5x3 | A' coarse 3x3x3 | A'
// fine first 12 pixels x 3], every window flattened (row, col, channel) as
// extract_patches_2d + flatten do.  Distances follow numpy's pairwise summation for n = 165
// (two halves of 80 and 85, 8 accumulators each, algorithms.py:74 / :126 / :135 through
// norm / add.reduce), so the matcher is exact against the oracle.
//
// The path is built for the reference's colour workloads (c1-c3 sizes): the database rows
// are materialised in fp64 (1,344 B per row) and searched exhaustively in fp64 — 32 rows x
// 8 queries per block step, both staged in LDS — with the lexicographic (distance, row)
// minimum, then the per-pixel tail (coherence over the causal 3x5 window, kappa test, B'
// update of all three channels) runs one 64-lane wave per pixel.  Single GPU, exact matcher.
#include "ia_common.h"
#include "ia_internal.h"

#include <algorithm>
#include <vector>

namespace ia {

constexpr int D3 = 165, D3P = 168;              // features, padded row stride (doubles)
constexpr int D3_FULL = 102, D3_HALF = 63;      // A full / A' half feature counts

// numpy pairwise sum of n = 165 values fed in order k = 0..164
struct Pw165 {
    double r[8];
    double h1, h2;
    __device__ __forceinline__ static double tree(const double *r) {
        return ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    }
    __device__ __forceinline__ void feed(int k, double v) {
        const int j = k < 80 ? k : k - 80;
        if (j < 8) r[j] = v;
        else if (j < 80) r[j & 7] += v;
        if (k == 79) h1 = tree(r);
        if (k == 159) h2 = tree(r);
        if (k >= 160) h2 += v;
    }
    __device__ __forceinline__ double result() const { return h1 + h2; }
};

// Pw165's sum of t[0..164] (the same accumulator order, the accumulators in registers: the
// struct's runtime-indexed r[] lives in scratch when its feeding loop is not unrolled)
__device__ __forceinline__ double pw165_sum(const double *t) {
    double h[2];
#pragma unroll
    for (int half = 0; half < 2; ++half) {
        const double *u = t + 80 * half;
        double r[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) r[j] = u[j];
#pragma unroll 1
        for (int i = 8; i < 80; i += 8)
#pragma unroll
            for (int j = 0; j < 8; ++j) r[j] += u[i + j];
        h[half] = Pw165::tree(r);
    }
#pragma unroll
    for (int k = 160; k < D3; ++k) h[1] += t[k];
    return h[0] + h[1];
}

struct Img3 {            // a channel-interleaved image (h x w x 3, fp64)
    const double *p;
    int h, w;
    __device__ __forceinline__ double at(int r, int c, int ch) const {
        return p[((long)symi2(r, h) * w + symi2(c, w)) * 3 + ch];
    }
};

// feature k (< 102: full window of the pair sm/lg; the half window keeps the first 63) of
// pixel (r, c): coarse 3x3x3 at (r/2, c/2), then fine 5x5x3 at (r, c)
__device__ __forceinline__ double feat3(const Img3 &sm, const Img3 &lg, int r, int c, int k) {
    if (k < 27) {
        const int t = k / 3, ch = k - 3 * t;
        return sm.at((r >> 1) + t / 3 - 1, (c >> 1) + t % 3 - 1, ch);
    }
    const int t = (k - 27) / 3, ch = (k - 27) - 3 * t;
    return lg.at(r + t / 5 - 2, c + t % 5 - 2, ch);
}

// one thread per (row, feature): the materialised database rows [A full | A'_img half]
__global__ __launch_bounds__(256) void k_db3_build(Img3 Asm, Img3 Alg, const double *Ap_sm,
                                                   const double *Ap_lg, long row0, long nrows,
                                                   double *__restrict__ db3) {
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i >= nrows * D3P) return;
    const long lr = i / D3P;
    const int k = (int)(i - lr * D3P);
    double v = 0.0;
    if (k < D3) {
        const long hw = (long)Alg.h * Alg.w;
        const long ix = row0 + lr;
        const long img = ix / hw;
        const long rem = ix - img * hw;
        const int r = (int)(rem / Alg.w), c = (int)(rem - (long)(rem / Alg.w) * Alg.w);
        if (k < D3_FULL) {
            v = feat3(Asm, Alg, r, c, k);
        } else {
            const Img3 psm{Ap_sm + img * (long)Asm.h * Asm.w * 3, Asm.h, Asm.w};
            const Img3 plg{Ap_lg + img * hw * 3, Alg.h, Alg.w};
            v = feat3(psm, plg, r, c, k - D3_FULL);
        }
    }
    db3[i] = v;
}

// compute_feature_array for one level pair (algorithms.py:11-47), 3 channels
__global__ __launch_bounds__(256) void k_level_features3(Img3 sm, Img3 lg, int nf,
                                                         double *__restrict__ out) {
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    const long n = (long)lg.h * lg.w;
    if (i >= n * nf) return;
    const long px = i / nf;
    const int k = (int)(i - px * nf);
    out[i] = feat3(sm, lg, (int)(px / lg.w), (int)(px - (px / lg.w) * lg.w), k);
}

// queries of wave t (y = y_lo + m, x = t - 3y): [B full | B' half], one block per pixel
__global__ __launch_bounds__(256) void k_query3(Img3 Bsm, Img3 Blg, Img3 Bpsm, Img3 Bplg, int t,
                                                int y_lo, double *__restrict__ q3) {
    const int m = blockIdx.x, k = threadIdx.x;
    const int y = y_lo + m, x = t - 3 * y;
    if (k >= D3P) return;
    double v = 0.0;
    if (k < D3_FULL) v = feat3(Bsm, Blg, y, x, k);
    else if (k < D3) v = feat3(Bpsm, Bplg, y, x, k - D3_FULL);
    q3[(long)m * D3P + k] = v;
}

// exhaustive fp64 search: a block takes 32 rows (staged in LDS) against every query, 8 at
// a time; thread (row tid / 8, query tid % 8) computes the oracle's distance; per query the
// block's lexicographic (distance, row) minimum -> part[query][block]
constexpr int M3_ROWS = 32, M3_Q = 8;
__global__ __launch_bounds__(256) void k_match3(const double *__restrict__ db3, long nrows, long row0,
                                                const double *__restrict__ q3, int M,
                                                Best *__restrict__ part) {
    __shared__ double rows[M3_ROWS * D3P];
    __shared__ double qs[M3_Q * D3P];
    __shared__ double cd[M3_Q][M3_ROWS];
    const long r0 = (long)blockIdx.x * M3_ROWS;
    const int nb = gridDim.x;
    for (int i = threadIdx.x; i < M3_ROWS * D3P; i += 256) {
        const long r = r0 + i / D3P;
        rows[i] = r < nrows ? db3[r0 * D3P + i] : 0.0;
    }
    const int rl = threadIdx.x >> 3, ql = threadIdx.x & 7;
    for (int q0 = 0; q0 < M; q0 += M3_Q) {
        __syncthreads();   // rows staged / the previous group's candidates consumed
        for (int i = threadIdx.x; i < M3_Q * D3P; i += 256) {
            const int q = q0 + i / D3P;
            qs[i] = q < M ? q3[(long)q0 * D3P + i] : 0.0;
        }
        __syncthreads();
        Pw165 pw;
        const double *a = rows + rl * D3P, *b = qs + ql * D3P;
#pragma unroll
        for (int k = 0; k < D3; ++k) {
            const double d = a[k] - b[k];
            pw.feed(k, d * d);
        }
        cd[ql][rl] = r0 + rl < nrows ? pw.result() : INFINITY;
        __syncthreads();
        if (threadIdx.x < M3_Q && q0 + threadIdx.x < M) {
            double bd = INFINITY;
            long long bi = 0x7fffffffffffffffLL;
            for (int r = 0; r < M3_ROWS; ++r) {
                const double d = cd[threadIdx.x][r];
                if (d < bd) { bd = d; bi = row0 + r0 + r; }   // rows ascending: first minimum
            }
            part[(long)(q0 + threadIdx.x) * nb + blockIdx.x] = Best{bd, bi};
        }
    }
}

__device__ __forceinline__ void best3(double &bd, long long &bi, double d, long long i) {
    if (d < bd || (d == bd && i < bi)) { bd = d; bi = i; }
}

// per query: the minimum over the blocks' partials (one block per query)
__global__ __launch_bounds__(256) void k_reduce3(const Best *__restrict__ part, int nb,
                                                 Best *__restrict__ best) {
    __shared__ double sd[4];
    __shared__ long long si[4];
    const Best *p = part + (long)blockIdx.x * nb;
    double bd = INFINITY;
    long long bi = 0x7fffffffffffffffLL;
    for (int i = threadIdx.x; i < nb; i += 256) best3(bd, bi, p[i].d, p[i].idx);
    for (int o = 32; o > 0; o >>= 1) {
        const double od = __shfl_xor(bd, o);
        const long long oi = __shfl_xor(bi, o);
        best3(bd, bi, od, oi);
    }
    if ((threadIdx.x & 63) == 0) { sd[threadIdx.x >> 6] = bd; si[threadIdx.x >> 6] = bi; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < 4; ++w) best3(bd, bi, sd[w], si[w]);
        best[blockIdx.x] = Best{bd, bi};
    }
}

struct Fin3 {
    const double *db3;       // rows of the level (row0 = 0: single GPU)
    const double *q3;
    const Best *best;
    const double *Ap_lg;     // nAp x Ah x Aw x 3
    int Ah, Aw;
    int t, y_lo, W;
    const double *weights;   // 165
    double kappa_factor;
    double *Bp_lg;           // H x W x 3
    int32_t *s, *im, *dbg_px;
    double *dbg_dist;
};

// distance of DB row ix to the query: plain (sqrt of the pairwise sum) or weighted (s*s,
// s = sqrt(pairwise(((a - q) w)^2)), algorithms.py:133-135)
__device__ __forceinline__ double row3_dist(const Fin3 &f, long ix, const double *q,
                                            const double *w) {
    const double *a = f.db3 + ix * D3P;
    Pw165 pw;
#pragma unroll 5
    for (int k = 0; k < D3; ++k) {
        const double d = w ? (a[k] - q[k]) * w[k] : a[k] - q[k];
        pw.feed(k, d * d);
    }
    const double s = sqrt(pw.result());
    return w ? s * s : s;
}

// the per-pixel tail (image_analogies.py:169-217 with best_coherence_match and
// compute_distance, algorithms.py:92-135), one 64-lane wave per pixel of the wave
__global__ __launch_bounds__(64) void k_finish3(Fin3 f) {
    const int m = blockIdx.x, lane = threadIdx.x;
    const int y = f.y_lo + m, x = f.t - 3 * y;
    const int W = f.W, Ah = f.Ah, Aw = f.Aw;
    const double *q = f.q3 + (long)m * D3P;
    const long long app = f.best[m].idx;
    const long hw = (long)Ah * Aw;
    // coherence candidates: lanes 0..14 = product(rows y-2..y, cols x-2..x+2), scanline-earlier
    double cd = INFINITY;
    long long cl = 0x7fffffffffffffffLL;
    long cix = -1;
    int cr = 0, cc = 0, cim = 0;
    const bool first = y == 0 && x == 0;
    if (!first && lane < 15) {
        const int rr = y - 2 + lane / 5, rc = x - 2 + lane % 5;
        if (rr >= 0 && rc >= 0 && rc < W && (rr < y || rc < x)) {
            const long sidx = (long)rr * W + rc;
            const int sr = f.s[2 * sidx] + y - rr, sc = f.s[2 * sidx + 1] + x - rc;
            if (sr >= 0 && sr < Ah && sc >= 0 && sc < Aw) {
                const int simg = f.im[sidx];
                cix = ((long)Ah * simg + sr) * Aw + sc;
                cr = sr; cc = sc; cim = simg;
                cd = row3_dist(f, cix, q, nullptr);
                cl = lane;
            }
        }
    }
    double bd = cd;
    long long bl = cl;
    for (int o = 32; o > 0; o >>= 1) {
        const double od = __shfl_xor(bd, o);
        const long long ol = __shfl_xor(bl, o);
        best3(bd, bl, od, ol);
    }
    const bool valid = bl != 0x7fffffffffffffffLL;
    const int win = valid ? (int)bl : 0;
    const long wix = __shfl(cix, win);
    const int wr = __shfl(cr, win), wc = __shfl(cc, win), wim = __shfl(cim, win);
    // the two weighted distances (lanes 0 and 1), then the kappa test and the update
    double dw = 0.0;
    if (valid && lane == 0) dw = row3_dist(f, app, q, f.weights);
    if (valid && lane == 1) dw = row3_dist(f, wix, q, f.weights);
    const double d_app = __shfl(dw, 0), d_coh = __shfl(dw, 1);
    long img = app / hw;
    long rem = app - img * hw;
    const int ar = (int)(rem / Aw), ac = (int)(rem - (long)(rem / Aw) * Aw);
    int pr = ar, pc = ac;
    if (valid && d_coh <= d_app * f.kappa_factor) { pr = wr; pc = wc; img = wim; }
    const long qpx = (long)y * W + x;
    if (lane < 3)
        f.Bp_lg[qpx * 3 + lane] = f.Ap_lg[((img * hw) + (long)pr * Aw + pc) * 3 + lane];
    if (lane == 0) {
        f.s[2 * qpx] = pr;
        f.s[2 * qpx + 1] = pc;
        f.im[qpx] = (int32_t)img;
        if (f.dbg_px) {
            int32_t *o = f.dbg_px + 7 * qpx;
            o[0] = ar;
            o[1] = ac;
            o[2] = valid ? wr : 0;
            o[3] = valid ? wc : 0;
            o[4] = valid ? y - 2 + win / 5 : 0;
            o[5] = valid ? x - 2 + win % 5 : 0;
            o[6] = valid;
            f.dbg_dist[2 * qpx] = valid ? d_app : 0.0;
            f.dbg_dist[2 * qpx + 1] = valid ? d_coh : 0.0;
        }
    }
}

// The per-pixel tail with the per-query reduction of k_match3's partials folded in, one
// 256-thread workgroup per pixel (k_finish3 took one wave and summed each distance serially
// from global memory).  The 15 coherence candidates' and the exact winner's rows are read
// once, lane-parallel over (row, feature); their plain and weighted squared terms go to LDS,
// and 31 threads sum one row each in numpy's pairwise order (Pw165): the same values as
// row3_dist.  The reduction of the partials is a lexicographic minimum, so its order does
// not matter.
__global__ __launch_bounds__(256) void k_finish3w(Fin3 f, const Best *__restrict__ part, int nb) {
    __shared__ double qs[D3P], wsh[D3P];
    __shared__ double tp[15][D3], tw[16][D3];   // plain terms (candidates), weighted (+ winner)
    __shared__ double sump[15], sumw[16];
    __shared__ long long rix[16];               // rows: candidates 0..14, winner 15 (-1: none)
    __shared__ int rpos[15][3];
    __shared__ double rd[4];
    __shared__ long long ri[4];
    const int m = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int y = f.y_lo + m, x = f.t - 3 * y;
    const int W = f.W, Ah = f.Ah, Aw = f.Aw;
    const long hw = (long)Ah * Aw;
    const bool first = y == 0 && x == 0;
    // the query, the weights, the partials' minimum and the candidates' rows: one round trip
    if (tid < D3P) {
        qs[tid] = f.q3[(long)m * D3P + tid];
        wsh[tid] = tid < D3 ? f.weights[tid] : 0.0;
    }
    double bd = INFINITY;
    long long bi = 0x7fffffffffffffffLL;
    for (int i = tid; i < nb; i += 256) best3(bd, bi, part[(long)m * nb + i].d, part[(long)m * nb + i].idx);
    for (int o = 32; o > 0; o >>= 1) {
        const double od = __shfl_xor(bd, o);
        const long long oi = __shfl_xor(bi, o);
        best3(bd, bi, od, oi);
    }
    if (lane == 0) { rd[wv] = bd; ri[wv] = bi; }
    if (tid < 15) {
        long long cix = -1;
        int cr = 0, cc = 0, cim = 0;
        if (!first) {
            const int rr = y - 2 + tid / 5, rc = x - 2 + tid % 5;
            if (rr >= 0 && rc >= 0 && rc < W && (rr < y || rc < x)) {
                const long sidx = (long)rr * W + rc;
                const int sr = f.s[2 * sidx] + y - rr, sc = f.s[2 * sidx + 1] + x - rc;
                if (sr >= 0 && sr < Ah && sc >= 0 && sc < Aw) {
                    const int simg = f.im[sidx];
                    cix = ((long)Ah * simg + sr) * Aw + sc;
                    cr = sr; cc = sc; cim = simg;
                }
            }
        }
        rix[tid] = cix;
        rpos[tid][0] = cr; rpos[tid][1] = cc; rpos[tid][2] = cim;
    }
    __syncthreads();
    if (tid == 0) {
        for (int w = 1; w < 4; ++w) best3(rd[0], ri[0], rd[w], ri[w]);
        rix[15] = ri[0];
    }
    __syncthreads();
    const long long app = rix[15];
    // the terms: (row j, feature k) pairs spread over the block, each row read once
    for (int e = tid; e < 16 * D3; e += 256) {
        const int j = e / D3, k = e - j * D3;
        const long long ix = rix[j];
        if (ix < 0) continue;
        const double d = f.db3[ix * D3P + k] - qs[k];
        const double dw = d * wsh[k];
        if (j < 15) tp[j][k] = d * d;
        tw[j][k] = dw * dw;
    }
    __syncthreads();
    if (tid < 31) {   // one row per thread, numpy's pairwise order
        const bool pl = tid < 15;
        const int j = pl ? tid : tid - 15;
        const double *t = pl ? tp[j] : tw[j];
        if (rix[j] >= 0) {
            const double sq = sqrt(pw165_sum(t));
            if (pl) sump[j] = sq; else sumw[j] = sq * sq;
        } else {
            if (pl) sump[j] = INFINITY; else sumw[j] = 0.0;
        }
    }
    __syncthreads();
    if (wv != 0) return;
    // coherence: the first minimum of the plain distances in (row, col) candidate order
    double cd = lane < 15 && rix[lane] >= 0 ? sump[lane] : INFINITY;
    long long cl = lane < 15 && rix[lane] >= 0 ? lane : 0x7fffffffffffffffLL;
    for (int o = 32; o > 0; o >>= 1) {
        const double od = __shfl_xor(cd, o);
        const long long ol = __shfl_xor(cl, o);
        best3(cd, cl, od, ol);
    }
    const bool valid = cl != 0x7fffffffffffffffLL;
    const int win = valid ? (int)cl : 0;
    const int wr = rpos[win][0], wc = rpos[win][1], wim = rpos[win][2];
    const double d_app = valid ? sumw[15] : 0.0, d_coh = valid ? sumw[win] : 0.0;
    long img = app / hw;
    long rem = app - img * hw;
    const int ar = (int)(rem / Aw), ac = (int)(rem - (long)(rem / Aw) * Aw);
    int pr = ar, pc = ac;
    if (valid && d_coh <= d_app * f.kappa_factor) { pr = wr; pc = wc; img = wim; }
    const long qpx = (long)y * W + x;
    if (lane < 3)
        f.Bp_lg[qpx * 3 + lane] = f.Ap_lg[((img * hw) + (long)pr * Aw + pc) * 3 + lane];
    if (lane == 0) {
        f.s[2 * qpx] = pr;
        f.s[2 * qpx + 1] = pc;
        f.im[qpx] = (int32_t)img;
        if (f.dbg_px) {
            int32_t *o = f.dbg_px + 7 * qpx;
            o[0] = ar;
            o[1] = ac;
            o[2] = valid ? wr : 0;
            o[3] = valid ? wc : 0;
            o[4] = valid ? y - 2 + win / 5 : 0;
            o[5] = valid ? x - 2 + win % 5 : 0;
            o[6] = valid;
            f.dbg_dist[2 * qpx] = valid ? d_app : 0.0;
            f.dbg_dist[2 * qpx + 1] = valid ? d_coh : 0.0;
        }
    }
}

// per-pixel API helpers (algorithms.py:92-135) for 165-dim rows: the coherence argmin over n
// candidate rows (first minimum of sqrt(pairwise((a - q)^2))) and weighted distances
__global__ void k_coherence_pick3(const double *__restrict__ rows, int n, const double *__restrict__ q,
                                  int32_t *out) {
    __shared__ double sd[64];
    const int i = threadIdx.x;
    double d = INFINITY;
    if (i < n) {
        Pw165 pw;
        for (int k = 0; k < D3; ++k) {
            const double x = rows[(long)i * D3 + k] - q[k];
            pw.feed(k, x * x);
        }
        d = sqrt(pw.result());
    }
    sd[i] = d;
    __syncthreads();
    if (i == 0) {
        int b = 0;
        for (int j = 1; j < n; ++j)
            if (sd[j] < sd[b]) b = j;
        out[0] = b;
    }
}

__global__ void k_wdist3(const double *__restrict__ a, const double *__restrict__ q,
                         const double *__restrict__ w, int n, double *__restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Pw165 pw;
    for (int k = 0; k < D3; ++k) {
        const double x = (a[(long)i * D3 + k] - q[(long)i * D3 + k]) * w[k];
        pw.feed(k, x * x);
    }
    const double s = sqrt(pw.result());
    out[i] = s * s;
}

__global__ void k_split_best3(const Best *__restrict__ b, int M, int64_t *idx, double *dist) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= M) return;
    if (idx) idx[i] = b[i].idx;
    if (dist) dist[i] = b[i].d;
}

static inline int max_wave(int H, int W) { return std::min(H, (W + 2) / 3) + 1; }
static inline int match3_blocks(long nrows) { return (int)((nrows + M3_ROWS - 1) / M3_ROWS); }

}  // namespace ia

using namespace ia;

extern "C" {

size_t ia_db3_bytes(long nrows) { return nrows > 0 ? (size_t)nrows * D3P * sizeof(double) : 0; }

int ia_db3_build(const IaSrcLevel *src, long row0, long nrows, double *db3, void *stream) {
    IA_ARG(src && db3 && nrows > 0 && row0 >= 0, "ia_db3_build: bad args");
    IA_ARG(row0 + nrows <= (long)src->nAp * src->Ah * src->Aw, "ia_db3_build: rows out of range");
    const Img3 Asm{src->A_sm, src->A_hs, src->A_ws}, Alg{src->A_lg, src->Ah, src->Aw};
    const long n = nrows * D3P;
    k_db3_build<<<(unsigned)((n + 255) / 256), 256, 0, S(stream)>>>(Asm, Alg, src->Ap_sm, src->Ap_lg,
                                                                   row0, nrows, db3);
    IA_LAUNCH_CHECK("k_db3_build");
    return IA_OK;
}

int ia_level_features3_f64(const double *sm, int hs, int ws, const double *lg, int h, int w,
                           int full, double *out, void *stream) {
    IA_ARG(sm && lg && out && hs > 0 && ws > 0 && h > 0 && w > 0, "ia_level_features3_f64: bad args");
    const int nf = full ? D3_FULL : D3_HALF;
    const long n = (long)h * w * nf;
    k_level_features3<<<(unsigned)((n + 255) / 256), 256, 0, S(stream)>>>(Img3{sm, hs, ws},
                                                                         Img3{lg, h, w}, nf, out);
    IA_LAUNCH_CHECK("k_level_features3");
    return IA_OK;
}

int ia_coherence_pick3(const double *rows, int n, const double *q, int32_t *out, void *stream) {
    IA_ARG(rows && q && out && n > 0 && n <= 64, "ia_coherence_pick3: bad args");
    k_coherence_pick3<<<1, 64, 0, S(stream)>>>(rows, n, q, out);
    IA_LAUNCH_CHECK("k_coherence_pick3");
    return IA_OK;
}

int ia_wdist3_batch(const double *a, const double *q, const double *w, int n, double *out,
                    void *stream) {
    IA_ARG(a && q && w && out && n > 0, "ia_wdist3_batch: bad args");
    k_wdist3<<<(n + 63) / 64, 64, 0, S(stream)>>>(a, q, w, n, out);
    IA_LAUNCH_CHECK("k_wdist3");
    return IA_OK;
}

size_t ia_match3_workspace_bytes(int M, long nrows) {
    return align_up((size_t)M * D3P * sizeof(double), 256) + align_up((size_t)M * sizeof(Best), 256) +
           align_up((size_t)M * match3_blocks(nrows) * sizeof(Best), 256);
}

int ia_match3_batch(const double *db3, long nrows, const double *q165, int M, int64_t *idx,
                    double *dist, void *workspace, void *stream) {
    IA_ARG(db3 && q165 && workspace && M > 0 && nrows > 0, "ia_match3_batch: bad args");
    hipStream_t st = S(stream);
    char *ws = reinterpret_cast<char *>(workspace);
    double *q3 = reinterpret_cast<double *>(ws);
    Best *best = reinterpret_cast<Best *>(ws + align_up((size_t)M * D3P * sizeof(double), 256));
    Best *part = reinterpret_cast<Best *>(reinterpret_cast<char *>(best) + align_up((size_t)M * sizeof(Best), 256));
    IA_HIP(hipMemsetAsync(q3, 0, (size_t)M * D3P * sizeof(double), st));
    IA_HIP(hipMemcpy2DAsync(q3, D3P * sizeof(double), q165, D3 * sizeof(double), D3 * sizeof(double),
                            M, hipMemcpyDeviceToDevice, st));
    const int nb = match3_blocks(nrows);
    k_match3<<<nb, 256, 0, st>>>(db3, nrows, 0, q3, M, part);
    k_reduce3<<<M, 256, 0, st>>>(part, nb, best);
    k_split_best3<<<(M + 255) / 256, 256, 0, st>>>(best, M, idx, dist);
    IA_LAUNCH_CHECK("ia_match3_batch");
    return IA_OK;
}

size_t ia_synth3_workspace_bytes(int H, int W, long nrows) {
    const size_t M = (size_t)max_wave(H, W);
    return align_up(M * D3P * sizeof(double), 256) + align_up(M * sizeof(Best), 256) +
           align_up(M * (size_t)match3_blocks(nrows) * sizeof(Best), 256);
}

int ia_synth_level3(const IaSynthArgs *a, void *stream) {
    IA_ARG(a && a->db && a->B_sm && a->B_lg && a->Bp_sm && a->Bp_lg && a->weights && a->s && a->im &&
               a->workspace && a->H > 0 && a->W > 0,
           "ia_synth_level3: bad args");
    IA_ARG(!a->comm && !a->lsh && a->row0 == 0 && a->nrows == (long)a->src.nAp * a->src.Ah * a->src.Aw,
           "ia_synth_level3: 3-channel matching runs unsharded with the exact matcher");
    IA_ARG(!a->dbg_px == !a->dbg_dist, "ia_synth_level3: debug outputs come in pairs");
    hipStream_t st = S(stream);
    const int H = a->H, W = a->W;
    const int Mmax = max_wave(H, W);
    char *ws = reinterpret_cast<char *>(a->workspace);
    double *q3 = reinterpret_cast<double *>(ws);
    Best *best = reinterpret_cast<Best *>(ws + align_up((size_t)Mmax * D3P * sizeof(double), 256));
    Best *part = reinterpret_cast<Best *>(reinterpret_cast<char *>(best) + align_up((size_t)Mmax * sizeof(Best), 256));
    const int nb = match3_blocks(a->nrows);
    const Img3 Bsm{a->B_sm, a->B_hs, a->B_ws}, Blg{a->B_lg, H, W};
    const Img3 Bpsm{a->Bp_sm, a->B_hs, a->B_ws}, Bplg{a->Bp_lg, H, W};
    Fin3 f{reinterpret_cast<const double *>(a->db), q3, best, a->src.Ap_lg, a->src.Ah, a->src.Aw,
           0, 0, W, a->weights, a->kappa_factor, a->Bp_lg, a->s, a->im, a->dbg_px, a->dbg_dist};
    const int nwaves = (W - 1) + 3 * (H - 1) + 1;
    for (int t = 0; t < nwaves; ++t) {
        const int y_lo = std::max(0, (t - (W - 1) + 2) / 3);
        const int y_hi = std::min(H - 1, t / 3);
        const int M = y_hi - y_lo + 1;
        if (M <= 0) continue;
        k_query3<<<M, 256, 0, st>>>(Bsm, Blg, Bpsm, Bplg, t, y_lo, q3);
        k_match3<<<nb, 256, 0, st>>>(f.db3, a->nrows, 0, q3, M, part);
        f.t = t;
        f.y_lo = y_lo;
        k_finish3w<<<M, 256, 0, st>>>(f, part, nb);
        IA_LAUNCH_CHECK("ia_synth_level3 wave");
    }
    return IA_OK;
}

}  // extern "C"
