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
#include "ia_split16.h"

#include <algorithm>
#include <atomic>
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

// ---- the split-f16 screen for 165-dim rows (IA_COLOR16=1) ---------------
// The screen value of row r and query j is e = |a'|^2 - 2 a'.q' over 166 slots (165
// centred features + the norm slot), carried as f16 pairs exactly like the luminance screen
// (ia_split16.h: the same scales sa, 2^R, sq): alpha = [sa a'_k, sa 2^-R |a'|^2], beta =
// [sq (-2 q'_k), sq 2^R], alpha . beta = sa sq e.  The 176 slots (166 + 10 zeros) are 11
// chunks of 16, each one v_mfma_f32_32x32x16_f16 per product: the 22 cross-term MFMAs
// (a_h q_l, a_l q_h) first, then the 11 main ones (a_h q_h, the norm slot in the last): 33
// per 32x32 tile.  The screen keeps the minimum per (query, 32-row tile); the exact stage
// (k_finish3w<true>) rescores in fp64 every row of the tiles whose minimum is within 2 eps3
// of the smallest (the error bound of DESIGN.md §4c).
constexpr int C16_CH = 11;                 // 16-slot chunks
constexpr int C16_GRP = 2 * C16_CH;        // half8 groups per lane and tile: (chunk, hi / lo)
constexpr int C16_TILE = C16_GRP * 64;     // half8 per 32-row (or 32-query) tile
constexpr int C3_NSLOT = 16 * C16_CH;      // 176
constexpr int C3_CAND = 64;                // candidate tiles listed per query (more: all)
typedef float floatx16 __attribute__((ext_vector_type(16)));

// lane (row / query l & 31, half h = l >> 5) of group (chunk c, part p) holds slots
// 16c + 8h .. +7: half8 index within a tile
__host__ __device__ constexpr int c16_at(int c, int p, int h, int j) { return (2 * c + p) * 64 + h * 32 + j; }

struct Col16Meta {                         // per database: centre, range keys, bound
    double center[D3P];
    unsigned long long rng[2 * D3P];       // order keys of min and of -max per feature
    unsigned int amax_bits;                // fp32 bits of A >= max row |a'| (atomicMax)
    unsigned int pad;
};

struct Db3View {                           // the ia_db3_build buffer: fp64 rows | split | meta
    double *rows;
    half8 *db16;
    Col16Meta *meta;
    long ntiles;
};
static inline size_t db3_rows_bytes(long nrows) { return align_up((size_t)nrows * D3P * sizeof(double), 256); }
__host__ __device__ inline long db3_tiles(long nrows) { return (nrows + 31) / 32; }
static inline size_t db3_split_bytes(long nrows) { return (size_t)db3_tiles(nrows) * C16_TILE * sizeof(half8); }
static inline Db3View db3_view(void *base, long nrows) {
    char *b = reinterpret_cast<char *>(base);
    Db3View v;
    v.rows = reinterpret_cast<double *>(b);
    v.db16 = reinterpret_cast<half8 *>(b + db3_rows_bytes(nrows));
    v.meta = reinterpret_cast<Col16Meta *>(b + db3_rows_bytes(nrows) + db3_split_bytes(nrows));
    v.ntiles = db3_tiles(nrows);
    return v;
}

__device__ __forceinline__ unsigned long long c3key(double x) {   // order-preserving key
    const unsigned long long b = (unsigned long long)__double_as_longlong(x);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ULL);
}
__device__ __forceinline__ double c3key_inv(unsigned long long k) {
    return __longlong_as_double((long long)((k >> 63) ? (k & 0x7fffffffffffffffULL) : ~k));
}

// per-feature range of the rows: thread k of a block scans RB rows of feature k
constexpr int C3_RB = 1024;
__global__ __launch_bounds__(D3P) void k_db3_range(const double *__restrict__ rows, long nrows,
                                                   Col16Meta *__restrict__ meta) {
    const int k = threadIdx.x;
    if (k >= D3) return;
    const long r0 = (long)blockIdx.x * C3_RB;
    const long r1 = r0 + C3_RB < nrows ? r0 + C3_RB : nrows;
    double lo = INFINITY, hi = -INFINITY;
    for (long r = r0; r < r1; ++r) {
        const double v = rows[r * D3P + k];
        lo = fmin(lo, v);
        hi = fmax(hi, v);
    }
    atomicMin(&meta->rng[2 * k], c3key(lo));
    atomicMin(&meta->rng[2 * k + 1], c3key(-hi));
}

// the centre (midrange) into LDS from the range keys
__device__ __forceinline__ void c3_center(const Col16Meta *meta, double *cs) {
    for (int k = threadIdx.x; k < D3P; k += blockDim.x)
        cs[k] = k < D3 ? 0.5 * (c3key_inv(meta->rng[2 * k]) - c3key_inv(meta->rng[2 * k + 1])) : 0.0;
}

__device__ __forceinline__ double c3_norm(const double *a, const double *cs) {
    double n = 0.0;
#pragma unroll 5
    for (int k = 0; k < D3; ++k) {
        const double d = a[k] - cs[k];
        n = fma(d, d, n);
    }
    return n;
}

// A: max over rows of |a'| rounded up to fp32 (one thread per row); block 0 stores the centre
__global__ __launch_bounds__(256) void k_db3_bound(const double *__restrict__ rows, long nrows,
                                                   Col16Meta *__restrict__ meta) {
    __shared__ double cs[D3P];
    __shared__ float red[4];
    c3_center(meta, cs);
    __syncthreads();
    if (blockIdx.x == 0)
        for (int k = threadIdx.x; k < D3P; k += 256) meta->center[k] = cs[k];
    const long r = (long)blockIdx.x * 256 + threadIdx.x;
    float a = 0.f;
    if (r < nrows) {
        const double n = c3_norm(rows + r * D3P, cs);
        a = (float)sqrt(n);
        if ((double)a * (double)a < n) a = nextafterf(a, INFINITY);
        a = nextafterf(a, INFINITY);   // the fp64 norm's own rounding
    }
    for (int o = 32; o > 0; o >>= 1) a = fmaxf(a, __shfl_xor(a, o));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = a;
    __syncthreads();
    if (threadIdx.x == 0)
        atomicMax(&meta->amax_bits, __float_as_uint(fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]))));
}

// the split rows, one thread per row (rows >= nrows repeat the last row): 22 half8 per row,
// lanes of consecutive rows writing consecutive 16 B
__global__ __launch_bounds__(256) void k_db3_split(const double *__restrict__ rows, long nrows,
                                                   const Col16Meta *__restrict__ meta,
                                                   half8 *__restrict__ db16) {
    __shared__ double cs[D3P];
    for (int k = threadIdx.x; k < D3P; k += 256) cs[k] = meta->center[k];
    __syncthreads();
    const long r = (long)blockIdx.x * 256 + threadIdx.x;
    if (r >= db3_tiles(nrows) * 32) return;
    const double *a = rows + (r < nrows ? r : nrows - 1) * D3P;
    const float amax = __uint_as_float(meta->amax_bits);
    const Split16Db sc = split16_db_scale(amax);
    const double nrm = c3_norm(a, cs);
    half8 *t = db16 + (r >> 5) * C16_TILE + (r & 31);
#pragma unroll 1
    for (int c = 0; c < C16_CH; ++c)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            half8 vh, vl;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const int k = 16 * c + 8 * h + e;
                double x = 0.0;
                if (k < D3) x = ldexp(a[k] - cs[k], sc.ea);
                else if (k == D3) x = ldexp((double)(float)nrm, sc.ea - sc.R);
                _Float16 xh, xl;
                split16d(x, xh, xl);
                vh[e] = xh;
                vl[e] = xl;
            }
            t[c16_at(c, 0, h, 0)] = vh;
            t[c16_at(c, 1, h, 0)] = vl;
        }
}

// the split operand of query m (q16) and |q'|^2 (qn) from thread k's feature v (256
// threads; m >= M: zero columns)
__device__ __forceinline__ void c3_query_split(int m, int M, int k, double v, const Col16Meta *meta,
                                               double *qn, _Float16 *q16, double *red) {
    _Float16 *qt = q16 + (long)(m >> 5) * C16_TILE * 8;
    const int col = m & 31;
    auto put = [&](int slot, _Float16 h, _Float16 l) {
        const int c = slot >> 4, hh = (slot >> 3) & 1, e = slot & 7;
        qt[c16_at(c, 0, hh, col) * 8 + e] = h;
        qt[c16_at(c, 1, hh, col) * 8 + e] = l;
    };
    if (m >= M) {
        if (k < C3_NSLOT) put(k, (_Float16)0.f, (_Float16)0.f);
        return;
    }
    const double d = k < D3 ? v - meta->center[k] : 0.0;
    double n = d * d;
    for (int o = 32; o > 0; o >>= 1) n += __shfl_xor(n, o);
    if ((k & 63) == 0) red[k >> 6] = n;
    __syncthreads();
    const double nq = (red[0] + red[1]) + (red[2] + red[3]);
    if (k == 0) qn[m] = nq;
    if (k < C3_NSLOT) {
        const Split16Db sc = split16_db_scale(__uint_as_float(meta->amax_bits));
        const int eq = split16_q_scale(nq, sc.R);
        double b = 0.0;
        if (k < D3) b = ldexp(-2.0 * d, eq);
        else if (k == D3) b = ldexp(1.0, eq + sc.R);
        _Float16 h, l;
        split16d(b, h, l);
        put(k, h, l);
    }
}

// queries of wave t for the split-f16 screen: the fp64 row (q3, as k_query3), |q'|^2 (qn)
// and the split operand (q16); blocks M .. Mpad-1 zero their query columns
__global__ __launch_bounds__(256) void k_query3s(Img3 Bsm, Img3 Blg, Img3 Bpsm, Img3 Bplg, int t,
                                                 int y_lo, int M, const Col16Meta *__restrict__ meta,
                                                 double *__restrict__ q3, double *__restrict__ qn,
                                                 _Float16 *__restrict__ q16) {
    __shared__ double red[4];
    const int m = blockIdx.x, k = threadIdx.x;
    double v = 0.0;
    if (m < M) {
        const int y = y_lo + m, x = t - 3 * y;
        if (k < D3_FULL) v = feat3(Bsm, Blg, y, x, k);
        else if (k < D3) v = feat3(Bpsm, Bplg, y, x, k - D3_FULL);
        if (k < D3P) q3[(long)m * D3P + k] = v;
    }
    c3_query_split(m, M, k, v, meta, qn, q16, red);
}

// diagnostic: the split operand of given queries (M x 165)
__global__ __launch_bounds__(256) void k_qsplit3(const double *__restrict__ q165, int M,
                                                 const Col16Meta *__restrict__ meta,
                                                 double *__restrict__ qn, _Float16 *__restrict__ q16) {
    __shared__ double red[4];
    const int m = blockIdx.x, k = threadIdx.x;
    const double v = m < M && k < D3 ? q165[(long)m * D3 + k] : 0.0;
    c3_query_split(m, M, k, v, meta, qn, q16, red);
}

// diagnostic: the screen's tile minima in unscaled units (e = s / (sa sq)), eps3 per query
__global__ void k_screen3_unscale(const float *__restrict__ smin, int M, int ntiles,
                                  const double *__restrict__ qn, const Col16Meta *__restrict__ meta,
                                  double *__restrict__ e, double *__restrict__ eps) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (long)M * ntiles) return;
    const int m = (int)(i / ntiles);
    const float amax = __uint_as_float(meta->amax_bits);
    const Split16Db sc = split16_db_scale(amax);
    const int eq = split16_q_scale(qn[m], sc.R);
    e[i] = ldexp((double)smin[i], -(sc.ea + eq));
    if (i % ntiles == 0) {
        constexpr double U32 = 5.9604644775390625e-08;
        const double A = (double)amax;
        eps[m] = U32 * (900.0 * A * sqrt(qn[m]) + 450.0 * A * A);
    }
}

// the screen: block (x, query group y) of 4 waves.  The group's query tiles (up to S3_QG)
// are staged in LDS once; each wave then walks row tiles t = (x tpw + i) 4 + wave, holding
// the tile's 22 operand groups in registers (the next tile's loaded while this one's chains
// run) against every staged query tile: 33 MFMAs per (row tile, query tile), and per query
// the minimum over the tile's 32 rows.  Each DB tile is read once per query group (round 4's
// first form read it once per query tile: 7 times per wave at the c3 size).
constexpr int S3_QG = 4;                  // query tiles per group (LDS: 4 x 22.5 KB)
__device__ __forceinline__ void s3_load(const half8 *db16, int t, int lane, half8 (&ah)[C16_CH],
                                        half8 (&al)[C16_CH]) {
    const half8 *db = db16 + (long)t * C16_TILE + lane;
#pragma unroll
    for (int c = 0; c < C16_CH; ++c) {
        ah[c] = db[(2 * c) * 64];
        al[c] = db[(2 * c + 1) * 64];
    }
}
__global__ __launch_bounds__(256, 1) void k_screen3(const half8 *__restrict__ db16, int ntiles,
                                                    const half8 *__restrict__ q16, int M, int tpw,
                                                    float *__restrict__ smin) {
    __shared__ half8 qsh[S3_QG * C16_TILE];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int qt0 = blockIdx.y * S3_QG;
    const int QT = (M + 31) / 32;
    const int nq = QT - qt0 < S3_QG ? QT - qt0 : S3_QG;
    for (int i = threadIdx.x; i < nq * C16_TILE; i += 256) qsh[i] = q16[(long)qt0 * C16_TILE + i];
    __syncthreads();
    const floatx16 zero = {};
    const int tb = blockIdx.x * tpw * 4 + wv;
    int t = tb;
    if (t >= ntiles) return;   // (after the only barrier)
    half8 ah[C16_CH], al[C16_CH], nh[C16_CH], nl[C16_CH];
    s3_load(db16, t, lane, ah, al);
    for (int it = 0; it < tpw; ++it, t += 4) {
        const int tn = t + 4;
        const bool more = it + 1 < tpw && tn < ntiles;
        if (more) s3_load(db16, tn, lane, nh, nl);
        for (int j = 0; j < nq; ++j) {
            const half8 *qb = qsh + j * C16_TILE + lane;
            floatx16 acc = zero;
#pragma unroll
            for (int c = 0; c < C16_CH; ++c) {
                acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[c], qb[(2 * c + 1) * 64], acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[c], qb[(2 * c) * 64], acc, 0, 0, 0);
            }
#pragma unroll
            for (int c = 0; c < C16_CH; ++c)
                acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[c], qb[(2 * c) * 64], acc, 0, 0, 0);
            float mn = acc[0];
#pragma unroll
            for (int i = 1; i < 16; ++i) mn = fminf(mn, acc[i]);
            mn = fminf(mn, __shfl_xor(mn, 32));
            const int q = (qt0 + j) * 32 + lane;
            if (lane < 32 && q < M) smin[(long)q * ntiles + t] = mn;
        }
        if (!more) break;
#pragma unroll
        for (int c = 0; c < C16_CH; ++c) {
            ah[c] = nh[c];
            al[c] = nl[c];
        }
    }
}

// grid of k_screen3: row tiles per wave so that about 512 workgroups cover the
// (row tile, query group) pairs
static inline dim3 screen3_grid(int ntiles, int M, int &tpw) {
    const int QG = ((M + 31) / 32 + S3_QG - 1) / S3_QG;
    tpw = (int)std::max(1L, ((long)ntiles * QG + 4L * 512 - 1) / (4L * 512));
    return dim3((unsigned)((ntiles + 4 * tpw - 1) / (4 * tpw)), (unsigned)QG);
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

// the exact stage's inputs on the split-f16 screen: per (query, row tile) minima, |q'|^2
struct Scr3 {
    const float *smin;       // M x ntiles
    int ntiles;
    long nrows;
    const double *qn;
    const Col16Meta *meta;
    unsigned long long *stats;   // [candidate tiles, full scans] (diagnostic, may be null)
};

// Thresholds of the colour exact stage: Tseg = e* + 2 eps3 in screen units,
// eps3 = u (900 A|q'| + 450 A^2); full scan when the norm slot nears the f16 floor
__device__ __forceinline__ double c3_tseg(float emin, float amax0, double nqq, bool &force_full) {
    constexpr double U32 = 5.9604644775390625e-08;
    const double A = (double)amax0;
    const Split16Db sc = split16_db_scale(amax0);
    const int eq = split16_q_scale(nqq, sc.R);
    const int e2 = sc.ea + eq;
    const double em = ldexp((double)emin, -e2);
    const double eps3 = U32 * (900.0 * A * sqrt(nqq) + 450.0 * A * A);
    const double slack = 1e-12 * (fabs(em) + nqq + A * A);
    force_full = eq + sc.R < -10;
    return ldexp(em + 2.0 * eps3 + slack, e2);
}

// The per-pixel tail, one 256-thread workgroup per pixel (k_finish3 took one wave and summed
// each distance serially from global memory).  The winner: SCR = false reduces k_match3's
// partials (a lexicographic minimum: order free); SCR = true is the exact stage of the
// split-f16 screen: e* over the query's tile minima, the tiles within the threshold, and
// every row of those tiles rescored in fp64 (terms lane-parallel into LDS, one thread per
// row summing them in numpy's pairwise order, Pw165), lexicographic (distance, row) minimum.
// Then the 15 coherence candidates' and the winner's rows are read once, lane-parallel over
// (row, feature); their plain and weighted squared terms go to LDS, and 31 threads sum one
// row each (Pw165): the same values as row3_dist.
template <bool SCR>
__global__ __launch_bounds__(256) void k_finish3w(Fin3 f, const Best *__restrict__ part, int nb, Scr3 sc) {
    __shared__ double qs[D3P], wsh[D3P];
    __shared__ double tt[32 * D3];              // exact-stage terms
    __shared__ double tp[15][D3], tw[16][D3];   // coherence rows: plain, weighted (+ winner)
    __shared__ double sump[15], sumw[16];
    __shared__ long long rix[16];               // rows: candidates 0..14, winner 15 (-1: none)
    __shared__ int rpos[15][3];
    __shared__ double rd[4];
    __shared__ long long ri[4];
    __shared__ float fmn[4];
    __shared__ int clist[C3_CAND], ccount;
    const int m = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int y = f.y_lo + m, x = f.t - 3 * y;
    const int W = f.W, Ah = f.Ah, Aw = f.Aw;
    const long hw = (long)Ah * Aw;
    const bool first = y == 0 && x == 0;
    // the query, the weights, the partials' minimum (or the tile minima's) and the
    // candidates' rows: one round trip
    if (tid < D3P) {
        qs[tid] = f.q3[(long)m * D3P + tid];
        wsh[tid] = tid < D3 ? f.weights[tid] : 0.0;
    }
    // the coherence candidates' rows (their s / im in the same round trip as the rest)
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
    double bd = INFINITY;
    long long bi = 0x7fffffffffffffffLL;
    bool coh_done = false;   // the coherence rows' sums (SCR: beside the first tile's)
    if constexpr (!SCR) {
        for (int i = tid; i < nb; i += 256) best3(bd, bi, part[(long)m * nb + i].d, part[(long)m * nb + i].idx);
    } else {
        const float *sm = sc.smin + (long)m * sc.ntiles;
        float mn = INFINITY;
        for (int i = tid; i < sc.ntiles; i += 256) mn = fminf(mn, sm[i]);
        for (int o = 32; o > 0; o >>= 1) mn = fminf(mn, __shfl_xor(mn, o));
        if (lane == 0) fmn[wv] = mn;
        if (tid == 0) ccount = 0;
        __syncthreads();
        mn = fminf(fminf(fmn[0], fmn[1]), fminf(fmn[2], fmn[3]));
        bool full;
        const double Tseg = c3_tseg(mn, __uint_as_float(sc.meta->amax_bits), sc.qn[m], full);
        if (!full)
            for (int i = tid; i < sc.ntiles; i += 256)
                if ((double)sm[i] <= Tseg) {
                    const int j = atomicAdd(&ccount, 1);
                    if (j < C3_CAND) clist[j] = i;
                }
        __syncthreads();
        const int nc = ccount;
        full = full || nc > C3_CAND;
        const int ntl = full ? sc.ntiles : nc;
        if (tid == 0 && sc.stats) {
            atomicAdd(&sc.stats[0], (unsigned long long)ntl);
            if (full) atomicAdd(&sc.stats[1], 1ull);
        }
        for (int b = 0; b < ntl; ++b) {
            const long r0 = (long)(full ? b : clist[b]) * 32;
            for (int e = tid; e < 32 * D3; e += 256) {
                const int j = e / D3, k = e - j * D3;
                const long r = r0 + j;
                if (r < sc.nrows) {
                    const double d = f.db3[r * D3P + k] - qs[k];
                    tt[e] = d * d;
                }
            }
            if (b == 0) {   // with the first tile: the coherence rows' terms
                for (int e = tid; e < 15 * D3; e += 256) {
                    const int j = e / D3, k = e - j * D3;
                    const long long ix = rix[j];
                    if (ix < 0) continue;
                    const double d = f.db3[ix * D3P + k] - qs[k];
                    const double dw = d * wsh[k];
                    tp[j][k] = d * d;
                    tw[j][k] = dw * dw;
                }
            }
            __syncthreads();
            if (tid < 32 && r0 + tid < sc.nrows) best3(bd, bi, pw165_sum(tt + tid * D3), r0 + tid);
            if (b == 0 && tid >= 64 && tid < 94) {   // their sums (wave 1), numpy's pairwise order
                const bool pl = tid < 79;
                const int j = pl ? tid - 64 : tid - 79;
                if (rix[j] >= 0) {
                    const double sq = sqrt(pw165_sum(pl ? tp[j] : tw[j]));
                    if (pl) sump[j] = sq; else sumw[j] = sq * sq;
                } else {
                    if (pl) sump[j] = INFINITY; else sumw[j] = 0.0;
                }
            }
            __syncthreads();
        }
        coh_done = ntl > 0;
    }
    for (int o = 32; o > 0; o >>= 1) {
        const double od = __shfl_xor(bd, o);
        const long long oi = __shfl_xor(bi, o);
        best3(bd, bi, od, oi);
    }
    if (lane == 0) { rd[wv] = bd; ri[wv] = bi; }
    __syncthreads();
    if (tid == 0) {
        for (int w = 1; w < 4; ++w) best3(rd[0], ri[0], rd[w], ri[w]);
        rix[15] = ri[0];
    }
    __syncthreads();
    const long long app = rix[15];
    // the terms: (row j, feature k) pairs spread over the block, each row read once (the
    // coherence rows only when not done beside the exact stage: the winner's alone then)
    const int j0 = coh_done ? 15 : 0;
    for (int e = tid; e < (16 - j0) * D3; e += 256) {
        const int j = j0 + e / D3, k = e - (j - j0) * D3;
        const long long ix = rix[j];
        if (ix < 0) continue;
        const double d = f.db3[ix * D3P + k] - qs[k];
        const double dw = d * wsh[k];
        if (j < 15) tp[j][k] = d * d;
        tw[j][k] = dw * dw;
    }
    __syncthreads();
    if (tid < 31 && (!coh_done || tid == 30)) {   // one row per thread, numpy's pairwise order
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

// IA_COLOR16 (ia_diag_set_color16): 1 the split-f16 screen + exact stage, 0 the exhaustive
// fp64 search (k_match3)
static std::atomic<int> g_color16{env_int("IA_COLOR16", 1)};
static unsigned long long *g_c3_stats = nullptr;   // diagnostic counters (ia_diag_color16_stats)

// the synthesis workspace: q3 | best | partials (fp64 search) | q16 | qn | tile minima
struct Ws3 {
    double *q3;
    Best *best, *part;
    half8 *q16;
    double *qn;
    float *smin;
};
static inline size_t ws3_layout(int H, int W, long nrows, char *base, Ws3 *w) {
    const size_t M = (size_t)max_wave(H, W), Mp = (M + 31) / 32 * 32;
    size_t o = 0;
    auto take = [&](size_t bytes) { char *p = base ? base + o : nullptr; o += align_up(bytes, 256); return p; };
    char *q3 = take(Mp * D3P * sizeof(double));
    char *best = take(M * sizeof(Best));
    char *part = take(M * (size_t)match3_blocks(nrows) * sizeof(Best));
    char *q16 = take(Mp / 32 * C16_TILE * sizeof(half8));
    char *qn = take(Mp * sizeof(double));
    char *smin = take(M * (size_t)db3_tiles(nrows) * sizeof(float));
    if (w) {
        w->q3 = reinterpret_cast<double *>(q3);
        w->best = reinterpret_cast<Best *>(best);
        w->part = reinterpret_cast<Best *>(part);
        w->q16 = reinterpret_cast<half8 *>(q16);
        w->qn = reinterpret_cast<double *>(qn);
        w->smin = reinterpret_cast<float *>(smin);
    }
    return o;
}

}  // namespace ia

using namespace ia;

extern "C" {

size_t ia_db3_bytes(long nrows) {
    return nrows > 0 ? db3_rows_bytes(nrows) + db3_split_bytes(nrows) + sizeof(Col16Meta) : 0;
}

int ia_db3_build(const IaSrcLevel *src, long row0, long nrows, double *db3, void *stream) {
    IA_ARG(src && db3 && nrows > 0 && row0 >= 0, "ia_db3_build: bad args");
    IA_ARG(row0 + nrows <= (long)src->nAp * src->Ah * src->Aw, "ia_db3_build: rows out of range");
    const Img3 Asm{src->A_sm, src->A_hs, src->A_ws}, Alg{src->A_lg, src->Ah, src->Aw};
    const long n = nrows * D3P;
    hipStream_t st = S(stream);
    k_db3_build<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(Asm, Alg, src->Ap_sm, src->Ap_lg,
                                                            row0, nrows, db3);
    // the split-f16 rows of the screen: range -> centre and bound -> split
    const Db3View v = db3_view(db3, nrows);
    IA_HIP(hipMemsetAsync(v.meta->rng, 0xff, sizeof(v.meta->rng), st));
    IA_HIP(hipMemsetAsync(&v.meta->amax_bits, 0, sizeof(unsigned int), st));
    k_db3_range<<<(unsigned)((nrows + C3_RB - 1) / C3_RB), D3P, 0, st>>>(v.rows, nrows, v.meta);
    k_db3_bound<<<(unsigned)((nrows + 255) / 256), 256, 0, st>>>(v.rows, nrows, v.meta);
    k_db3_split<<<(unsigned)((v.ntiles * 32 + 255) / 256), 256, 0, st>>>(v.rows, nrows, v.meta, v.db16);
    IA_LAUNCH_CHECK("ia_db3_build");
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

size_t ia_synth3_workspace_bytes(int H, int W, long nrows) { return ws3_layout(H, W, nrows, nullptr, nullptr); }

int ia_synth_level3(const IaSynthArgs *a, void *stream) {
    IA_ARG(a && a->db && a->B_sm && a->B_lg && a->Bp_sm && a->Bp_lg && a->weights && a->s && a->im &&
               a->workspace && a->H > 0 && a->W > 0,
           "ia_synth_level3: bad args");
    IA_ARG(!a->comm && !a->lsh && a->row0 == 0 && a->nrows == (long)a->src.nAp * a->src.Ah * a->src.Aw,
           "ia_synth_level3: 3-channel matching runs unsharded with the exact matcher");
    IA_ARG(!a->dbg_px == !a->dbg_dist, "ia_synth_level3: debug outputs come in pairs");
    hipStream_t st = S(stream);
    const int H = a->H, W = a->W;
    Ws3 w;
    ws3_layout(H, W, a->nrows, reinterpret_cast<char *>(a->workspace), &w);
    const int nb = match3_blocks(a->nrows);
    const Img3 Bsm{a->B_sm, a->B_hs, a->B_ws}, Blg{a->B_lg, H, W};
    const Img3 Bpsm{a->Bp_sm, a->B_hs, a->B_ws}, Bplg{a->Bp_lg, H, W};
    const Db3View v = db3_view(const_cast<void *>(a->db), a->nrows);
    Fin3 f{v.rows, w.q3, w.best, a->src.Ap_lg, a->src.Ah, a->src.Aw,
           0, 0, W, a->weights, a->kappa_factor, a->Bp_lg, a->s, a->im, a->dbg_px, a->dbg_dist};
    const bool split = g_color16.load(std::memory_order_relaxed) != 0;
    const int ntiles = (int)v.ntiles;
    const Scr3 sc{w.smin, ntiles, a->nrows, w.qn, v.meta, g_c3_stats};
    const int nwaves = (W - 1) + 3 * (H - 1) + 1;
    for (int t = 0; t < nwaves; ++t) {
        const int y_lo = std::max(0, (t - (W - 1) + 2) / 3);
        const int y_hi = std::min(H - 1, t / 3);
        const int M = y_hi - y_lo + 1;
        if (M <= 0) continue;
        f.t = t;
        f.y_lo = y_lo;
        if (split) {
            const int QT = (M + 31) / 32;
            int tpw;
            const dim3 grid = screen3_grid(ntiles, M, tpw);
            k_query3s<<<QT * 32, 256, 0, st>>>(Bsm, Blg, Bpsm, Bplg, t, y_lo, M, v.meta, w.q3, w.qn,
                                               reinterpret_cast<_Float16 *>(w.q16));
            k_screen3<<<grid, 256, 0, st>>>(v.db16, ntiles, w.q16, M, tpw, w.smin);
            k_finish3w<true><<<M, 256, 0, st>>>(f, nullptr, 0, sc);
        } else {
            k_query3<<<M, 256, 0, st>>>(Bsm, Blg, Bpsm, Bplg, t, y_lo, w.q3);
            k_match3<<<nb, 256, 0, st>>>(f.db3, a->nrows, 0, w.q3, M, w.part);
            k_finish3w<false><<<M, 256, 0, st>>>(f, w.part, nb, sc);
        }
        IA_LAUNCH_CHECK("ia_synth_level3 wave");
    }
    return IA_OK;
}

int ia_diag_screen3(const void *db3, long nrows, const double *q165, int M, double *e, double *eps,
                    double *qn) {
    IA_ARG(db3 && q165 && e && eps && qn && nrows > 0 && M > 0, "ia_diag_screen3: bad args");
    const Db3View v = db3_view(const_cast<void *>(db3), nrows);
    const int QT = (M + 31) / 32, ntiles = (int)v.ntiles;
    half8 *q16 = nullptr;
    float *smin = nullptr;
    IA_HIP(hipMalloc(&q16, (size_t)QT * C16_TILE * sizeof(half8)));
    IA_HIP(hipMalloc(&smin, (size_t)M * ntiles * sizeof(float)));
    k_qsplit3<<<QT * 32, 256>>>(q165, M, v.meta, qn, reinterpret_cast<_Float16 *>(q16));
    int tpw;
    k_screen3<<<screen3_grid(ntiles, M, tpw), 256>>>(v.db16, ntiles, q16, M, tpw, smin);
    const long n = (long)M * ntiles;
    k_screen3_unscale<<<(unsigned)((n + 255) / 256), 256>>>(smin, M, ntiles, qn, v.meta, e, eps);
    IA_LAUNCH_CHECK("ia_diag_screen3");
    IA_HIP(hipDeviceSynchronize());
    IA_HIP(hipFree(q16));
    IA_HIP(hipFree(smin));
    return IA_OK;
}

int ia_diag_set_color16(int on) {
    const int prev = g_color16.load();
    if (on == 0 || on == 1) g_color16.store(on);
    return prev;
}

// the colour exact stage's counters since the last call: [candidate tiles rescored, queries
// that scanned every tile]; the first call allocates them (and returns zeros)
int ia_diag_color16_stats(unsigned long long *out) {
    IA_ARG(out, "ia_diag_color16_stats: bad args");
    if (!g_c3_stats) {
        IA_HIP(hipMalloc(&g_c3_stats, 2 * sizeof(unsigned long long)));
        IA_HIP(hipMemset(g_c3_stats, 0, 2 * sizeof(unsigned long long)));
        out[0] = out[1] = 0;
        return IA_OK;
    }
    IA_HIP(hipDeviceSynchronize());
    IA_HIP(hipMemcpy(out, g_c3_stats, 2 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    IA_HIP(hipMemset(g_c3_stats, 0, 2 * sizeof(unsigned long long)));
    return IA_OK;
}

}  // extern "C"
