// ia_color3.hip — 3-channel matching (the reference's convert=False on colour images:
// config.py:29-42 num_ch = 3, algorithms.py:11-47 with channel-interleaved windows).
//
// Each feature row has 165 values: [A coarse 3x3x3 | A fine 5x5x3 | A' coarse 3x3x3 | A'
// fine first 12 pixels x 3], every window flattened (row, col, channel) as
// extract_patches_2d + flatten do.  Distances follow numpy's pairwise summation for n = 165
// (two halves of 80 and 85, 8 accumulators each, algorithms.py:74 / :126 / :135 through
// norm / add.reduce), so the matcher is exact against the oracle.
//
// Per level (ia_db3_build) the rows are materialised in fp64 (1,344 B per row: the exact
// stage's input) with the split-f16 screen operand (704 B per row) after them;
// ia_db3_build_rot adds the rotated split operand (R16c, 352 B per row, §4e).  Per wave: the
// query rows (k_query3s / k_query3r), the MFMA screen's minimum per (query, 32-row tile)
// (k_screen3: 33 MFMAs per 32x32 tile; k_screen3r: 11), then k_exact3: every row of the tiles
// within the bound rescored in fp64 in the oracle's order, the coherence pick over the causal
// 3x5 window, the kappa test and the B' update of all three channels, one 256-thread
// workgroup per pixel.  IA_COLOR16=0 keeps the exhaustive fp64 search (k_match3 +
// k_finish3w).  ia_synth_levels3 runs the levels pipelined.  Single GPU, exact matcher.
#include "ia_common.h"
#include "ia_internal.h"
#include "ia_split16.h"

#include <algorithm>
#include <atomic>
#include <cstring>
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
// (k_exact3) rescores in fp64 every row of the tiles whose minimum is within 2 eps3
// of the smallest (the error bound of DESIGN.md §4c).
constexpr int C16_CH = 11;                 // 16-slot chunks
constexpr int C16_GRP = 2 * C16_CH;        // half8 groups per lane and tile: (chunk, hi / lo)
constexpr int C16_TILE = C16_GRP * 64;     // half8 per 32-row (or 32-query) tile
constexpr int C3_NSLOT = 16 * C16_CH;      // 176
constexpr int C3_CAND = 64;                // candidate tiles listed per query (more: all)
constexpr int C3_REG = 8;                  // float4s of tile minima per thread in registers
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
// row stride of the tile minima (M x stride floats): whole float4s, read into registers by
// the exact stage in one round trip (the pad entries are never written nor read as minima)
__host__ __device__ constexpr int c3_stride(int ntiles) { return (ntiles + 3) & ~3; }
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
// (R16c: nsk, rmeta given, eps = r3_eps)
struct Rot3Meta;
__device__ double r3_eps_m(const Rot3Meta *rm, double A, double nqq, double nsk);
__global__ void k_screen3_unscale(const float *__restrict__ smin, int M, int ntiles,
                                  const double *__restrict__ qn, const Col16Meta *__restrict__ meta,
                                  double *__restrict__ e, double *__restrict__ eps,
                                  const double *__restrict__ nsk = nullptr, const Rot3Meta *rm = nullptr) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (long)M * ntiles) return;
    const int m = (int)(i / ntiles), tl = (int)(i - (long)m * ntiles);
    const float amax = __uint_as_float(meta->amax_bits);
    const Split16Db sc = split16_db_scale(amax);
    const int eq = split16_q_scale(qn[m], sc.R);
    e[i] = ldexp((double)smin[(long)m * c3_stride(ntiles) + tl], -(sc.ea + eq));
    if (i % ntiles == 0) {
        constexpr double U32 = 5.9604644775390625e-08;
        const double A = (double)amax;
        eps[m] = nsk ? r3_eps_m(rm, A, qn[m], nsk[m]) : U32 * (900.0 * A * sqrt(qn[m]) + 450.0 * A * A);
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
            if (lane < 32 && q < M) smin[(long)q * c3_stride(ntiles) + t] = mn;
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

// ---- the rotated split screen for 3-channel rows (R16c) -----------------
// As ia_rot16.h for D = 165: per level the principal directions V (165 x 165, fp32, host
// eigh of the centred rows' covariance), rows rho = V^T a', queries kappa = V^T q'; the top
// R3_P components keep f16 split pairs (three products), the other 162 one f16 product, the
// norm its split pair: 2P cross slots, norm_lo, 165 main slots, norm_hi, zeros -> 176 slots =
// 11 MFMAs per 32x32 tile (33 in k_screen3), 352 B per row (704).  Same scales and units as
// §4c; the bound adds the skipped components' dropped cross terms (A_skip, |kappa_skip|).
constexpr int R3_P = 3;
constexpr int R3_NL = 2 * R3_P, R3_M0 = R3_NL + 1, R3_NH = R3_M0 + D3;   // 6, 7, 172
constexpr int R3_SLOTS = (R3_NH + 16) / 16 * 16;                           // 176
constexpr int R3_MFMA = R3_SLOTS / 16;                                     // 11
constexpr int R3_TILE = R3_MFMA * 64;                                      // half8 per tile
constexpr int R3_LD = 168;                                                 // rot[k * R3_LD + j]
constexpr int R3_ROT_FLOATS = D3 * R3_LD;
static_assert(R3_MFMA == 11, "R16c: 11 MFMAs per tile at P = 3");
// half8 index of slot s of tile row (or query column) j, and its element s & 7
__host__ __device__ constexpr int r3_h8(int s, int j) { return (s >> 4) * 64 + ((s & 15) >> 3) * 32 + j; }

struct Rot3Meta {   // after the rotated tiles: A_skip (fp32 bits, rounded up; atomicMax)
    unsigned int askip_bits;
    unsigned int pad[63];
};
static inline size_t db3r_tiles_bytes(long nrows) { return align_up((size_t)db3_tiles(nrows) * R3_TILE * sizeof(half8), 256); }
static inline Rot3Meta *db3r_meta(void *dbr, long nrows) {
    return reinterpret_cast<Rot3Meta *>(reinterpret_cast<char *>(dbr) + db3r_tiles_bytes(nrows));
}

// the rotated tiles: one 256-thread block per 32-row tile (rows past nrows repeat the last);
// V and the tile's centred rows staged in LDS; thread (row r = tid & 31, g = tid >> 5) takes
// components j = g + 8i in fp64 from the fp32 V; then the split slots through an LDS stage
// (reusing the rows' space) into the tile layout, and A_skip = max ||fl32(rho_skip)||
__global__ __launch_bounds__(256, 1) void k_db3_rot(const double *__restrict__ rows, long nrows,
                                                    const Col16Meta *__restrict__ meta,
                                                    const float *__restrict__ rot, half8 *__restrict__ dbr,
                                                    Rot3Meta *__restrict__ rmeta) {
    __shared__ __attribute__((aligned(16))) float V[R3_ROT_FLOATS];      // 110,880 B
    __shared__ __attribute__((aligned(16))) double X[32 * D3];          // 42,240 B (odd row stride)
    __shared__ double skp[32][8];
    __shared__ double nrm[32];
    __shared__ float red[4];
    const int tid = threadIdx.x, r = tid & 31, g = tid >> 5;
    for (int i = tid; i < R3_ROT_FLOATS / 4; i += 256)
        reinterpret_cast<float4 *>(V)[i] = reinterpret_cast<const float4 *>(rot)[i];
    const long t = blockIdx.x;
    for (int i = tid; i < 32 * D3; i += 256) {
        const int rr = i / D3, k = i - rr * D3;
        const long row = t * 32 + rr < nrows ? t * 32 + rr : nrows - 1;
        X[i] = rows[row * D3P + k] - meta->center[k];
    }
    __syncthreads();
    constexpr int NJ = (D3 + 7) / 8;   // 21 components per thread
    double acc[NJ];
#pragma unroll
    for (int i = 0; i < NJ; ++i) acc[i] = 0.0;
    double n2 = 0.0;
    for (int k = 0; k < D3; ++k) {
        const double dk = X[r * D3 + k];
        if (g == 0) n2 += dk * dk;
#pragma unroll
        for (int i = 0; i < NJ; ++i) {
            const int j = g + 8 * i;
            if (j < D3) acc[i] = fma((double)V[k * R3_LD + j], dk, acc[i]);
        }
    }
    __syncthreads();   // every read of X done: it becomes the slot stage
    _Float16 *stage = reinterpret_cast<_Float16 *>(X);   // [32][R3_SLOTS]
    const Split16Db sc = split16_db_scale(__uint_as_float(meta->amax_bits));
    double sk = 0.0;
#pragma unroll
    for (int i = 0; i < NJ; ++i) {
        const int j = g + 8 * i;
        if (j >= D3) continue;
        const float r32 = (float)acc[i];
        if (j >= R3_P) sk += (double)r32 * (double)r32;
        _Float16 h, l;
        split16f(ldexpf(r32, sc.ea), h, l);
        stage[r * R3_SLOTS + R3_M0 + j] = h;
        if (j < R3_P) {
            stage[r * R3_SLOTS + 2 * j] = l;
            stage[r * R3_SLOTS + 2 * j + 1] = h;
        }
    }
    skp[r][g] = sk;
    if (g == 0) nrm[r] = n2;
    __syncthreads();
    float askip = 0.f;
    if (g == 0) {
        _Float16 nh, nl;
        split16f(ldexpf((float)nrm[r], sc.ea - sc.R), nh, nl);
        stage[r * R3_SLOTS + R3_NL] = nl;
        stage[r * R3_SLOTS + R3_NH] = nh;
        for (int z = R3_NH + 1; z < R3_SLOTS; ++z) stage[r * R3_SLOTS + z] = (_Float16)0.f;
        double s = 0.0;
        for (int q = 0; q < 8; ++q) s += skp[r][q];
        const double a = sqrt(s * (1.0 + 1e-12));
        askip = (float)a;
        if ((double)askip < a) askip = nextafterf(askip, INFINITY);
    }
    for (int o = 32; o > 0; o >>= 1) askip = fmaxf(askip, __shfl_xor(askip, o));
    if ((tid & 63) == 0) red[tid >> 6] = askip;
    __syncthreads();
    if (tid == 0)
        atomicMax(&rmeta->askip_bits, __float_as_uint(fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]))));
    // the tile layout: half8 (m, hh, j) = slots 16 m + 8 hh .. +7 of row j
    half8 *out = dbr + t * R3_TILE;
    for (int i = tid; i < R3_TILE; i += 256) {
        const int m = i >> 6, hh = (i >> 5) & 1, j = i & 31;
        out[i] = *reinterpret_cast<const half8 *>(&stage[j * R3_SLOTS + 16 * m + 8 * hh]);
    }
}

// ---- the covariance of a 3-channel level's rows (ia_db3_cov, rot3_build's matrix) -------
// ~64 k rows sampled every `step` (rot3_build's rows[::max(1, N // 65536)]), centred at their
// mean, fp64: column sums per sample slice, the mean, then per (16 output rows a, slice) the
// centred products with every column b, 32 sampled rows staged in LDS at a time; partials
// reduced in slice order (deterministic).  Any orthonormal basis keeps the matcher exact; the
// principal one of this matrix keeps its bound tight.
constexpr int C3C_SPLIT = 128, C3C_AB = 16, C3C_NA = (D3 + C3C_AB - 1) / C3C_AB, C3C_TR = 32;
__global__ __launch_bounds__(256) void k_db3_colsum(const double *__restrict__ rows, long step, long nsamp,
                                                    double *__restrict__ part) {
    __shared__ double X[C3C_TR][D3P];
    const int t = threadIdx.x, sl = blockIdx.x;
    const long i0 = nsamp * sl / C3C_SPLIT, i1 = nsamp * (sl + 1) / C3C_SPLIT;
    double acc = 0.0;
    for (long r0 = i0; r0 < i1; r0 += C3C_TR) {
        __syncthreads();
        for (int e = t; e < C3C_TR * D3P; e += 256) {
            const int rr = e / D3P, k = e - rr * D3P;
            const long i = r0 + rr;
            X[rr][k] = i < i1 ? rows[i * step * D3P + k] : 0.0;
        }
        __syncthreads();
        if (t < D3)
            for (int rr = 0; rr < C3C_TR; ++rr) acc += X[rr][t];
    }
    if (t < D3P) part[sl * D3P + t] = t < D3 ? acc : 0.0;
}
__global__ __launch_bounds__(256) void k_db3_mean(const double *__restrict__ part, long nsamp, double *__restrict__ mean) {
    const int t = threadIdx.x;
    if (t >= D3P) return;
    double acc = 0.0;
    for (int sl = 0; sl < C3C_SPLIT; ++sl) acc += part[sl * D3P + t];
    mean[t] = t < D3 ? acc / (double)nsamp : 0.0;
}
__global__ __launch_bounds__(256) void k_db3_cov(const double *__restrict__ rows, long step, long nsamp,
                                                 const double *__restrict__ mean, double *__restrict__ part) {
    __shared__ double X[C3C_TR][D3P];
    const int t = threadIdx.x, a0 = blockIdx.x * C3C_AB, sl = blockIdx.y;
    const long i0 = nsamp * sl / C3C_SPLIT, i1 = nsamp * (sl + 1) / C3C_SPLIT;
    double acc[C3C_AB];
#pragma unroll
    for (int j = 0; j < C3C_AB; ++j) acc[j] = 0.0;
    const double mu = t < D3 ? mean[t] : 0.0;
    for (long r0 = i0; r0 < i1; r0 += C3C_TR) {
        __syncthreads();
        for (int e = t; e < C3C_TR * D3P; e += 256) {
            const int rr = e / D3P, k = e - rr * D3P;
            const long i = r0 + rr;
            X[rr][k] = i < i1 && k < D3 ? rows[i * step * D3P + k] - mean[k] : 0.0;
        }
        __syncthreads();
        if (t < D3) {
            for (int rr = 0; rr < C3C_TR; ++rr) {
                const double xb = X[rr][t];
#pragma unroll
                for (int j = 0; j < C3C_AB; ++j) acc[j] += X[rr][a0 + j < D3 ? a0 + j : 0] * xb;
            }
        }
    }
    (void)mu;
    if (t < D3) {
#pragma unroll
        for (int j = 0; j < C3C_AB; ++j)
            if (a0 + j < D3) part[((long)sl * D3 + a0 + j) * D3P + t] = acc[j];
    }
}
__global__ __launch_bounds__(256) void k_db3_cov_reduce(const double *__restrict__ part, double *__restrict__ cov) {
    const int a = blockIdx.x, t = threadIdx.x;
    if (t >= D3P) return;
    double acc = 0.0;
    if (t < D3)
        for (int sl = 0; sl < C3C_SPLIT; ++sl) acc += part[((long)sl * D3 + a) * D3P + t];
    cov[(long)a * D3P + t] = acc;
}

// the R16c query operand of query m from thread k's centred feature d (256 threads):
// kappa_j = sum_k V[k][j] d_k (thread j, fp64 from the fp32 V in global memory), |q'|^2 ->
// qn, |kappa_skip|^2 -> nsk, the slots into the query tile (m >= M: zero columns)
__device__ __forceinline__ void r3_query(int m, int M, int k, double v, const Col16Meta *meta,
                                         const float *__restrict__ rot, double *qn, double *nsk,
                                         half8 *q16, double *ds, double *red) {
    _Float16 *qt = reinterpret_cast<_Float16 *>(q16 + (long)(m >> 5) * R3_TILE);
    const int col = m & 31;
    auto put = [&](int slot, _Float16 x) { qt[r3_h8(slot, col) * 8 + (slot & 7)] = x; };
    if (m >= M) {
        if (k < R3_SLOTS) put(k, (_Float16)0.f);
        return;
    }
    const double d = k < D3 ? v - meta->center[k] : 0.0;
    if (k < D3) ds[k] = d;
    double n = d * d;
    for (int o = 32; o > 0; o >>= 1) n += __shfl_xor(n, o);
    if ((k & 63) == 0) red[k >> 6] = n;
    __syncthreads();
    const double nq = (red[0] + red[1]) + (red[2] + red[3]);
    double kap = 0.0;
    if (k < D3) {
        double k0 = 0.0, k1 = 0.0, k2 = 0.0, k3 = 0.0;
        int i = 0;
        // unrolled: the loads of V (L2-resident) issue far ahead of their FMAs
#pragma unroll 10
        for (; i + 4 <= D3; i += 4) {
            k0 = fma((double)rot[(i + 0) * R3_LD + k], ds[i + 0], k0);
            k1 = fma((double)rot[(i + 1) * R3_LD + k], ds[i + 1], k1);
            k2 = fma((double)rot[(i + 2) * R3_LD + k], ds[i + 2], k2);
            k3 = fma((double)rot[(i + 3) * R3_LD + k], ds[i + 3], k3);
        }
        for (; i < D3; ++i) k0 = fma((double)rot[i * R3_LD + k], ds[i], k0);
        kap = (k0 + k1) + (k2 + k3);
    }
    double s2 = k >= R3_P && k < D3 ? kap * kap : 0.0;
    for (int o = 32; o > 0; o >>= 1) s2 += __shfl_xor(s2, o);
    __syncthreads();   // red reused
    if ((k & 63) == 0) red[k >> 6] = s2;
    __syncthreads();
    if (k == 0) {
        qn[m] = nq;
        nsk[m] = (red[0] + red[1]) + (red[2] + red[3]);
    }
    const Split16Db sc = split16_db_scale(__uint_as_float(meta->amax_bits));
    const int eq = split16_q_scale(nq, sc.R);
    if (k < D3) {
        _Float16 h, l;
        split16d(ldexp(-2.0 * kap, eq), h, l);
        put(R3_M0 + k, h);
        if (k < R3_P) {
            put(2 * k, h);
            put(2 * k + 1, l);
        }
    } else if (k == D3) {
        const _Float16 nn = (_Float16)ldexpf(1.f, eq + sc.R);
        put(R3_NL, nn);
        put(R3_NH, nn);
    } else if (R3_NH + (k - D3) < R3_SLOTS) {
        put(R3_NH + (k - D3), (_Float16)0.f);
    }
}

// queries of wave t for the R16c screen (as k_query3s; qin: caller-given rows, diagnostics)
__global__ __launch_bounds__(256) void k_query3r(Img3 Bsm, Img3 Blg, Img3 Bpsm, Img3 Bplg, int t,
                                                 int y_lo, int M, const Col16Meta *__restrict__ meta,
                                                 const float *__restrict__ rot, const double *__restrict__ qin,
                                                 double *__restrict__ q3, double *__restrict__ qn,
                                                 double *__restrict__ nsk, half8 *__restrict__ q16) {
    __shared__ double red[4];
    __shared__ double ds[D3];
    const int m = blockIdx.x, k = threadIdx.x;
    double v = 0.0;
    if (m < M) {
        if (qin) {
            v = k < D3 ? qin[(long)m * D3 + k] : 0.0;
        } else {
            const int y = y_lo + m, x = t - 3 * y;
            if (k < D3_FULL) v = feat3(Bsm, Blg, y, x, k);
            else if (k < D3) v = feat3(Bpsm, Bplg, y, x, k - D3_FULL);
            if (k < D3P) q3[(long)m * D3P + k] = v;
        }
    }
    r3_query(m, M, k, v, meta, rot, qn, nsk, q16, ds, red);
}

// the R16c screen: as k_screen3 with 11 operand groups per tile and 11 MFMAs per (row tile,
// query tile); up to 8 query tiles staged per workgroup (a c3 wave's 213 queries: one group,
// each DB tile read once per wave)
// 7 query tiles per group (a c3 wave's <= 213 queries: one group; LDS 77 KiB, two workgroups
// per CU: the grid's ~450 workgroups in one round instead of two)
constexpr int S3R_QG = 7;
__global__ __launch_bounds__(256, 2) void k_screen3r(const half8 *__restrict__ db16, int ntiles,
                                                     const half8 *__restrict__ q16, int M, int tpw,
                                                     float *__restrict__ smin) {
    __shared__ half8 qsh[S3R_QG * R3_TILE];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int qt0 = blockIdx.y * S3R_QG;
    const int QT = (M + 31) / 32;
    const int nq = QT - qt0 < S3R_QG ? QT - qt0 : S3R_QG;
    for (int i = threadIdx.x; i < nq * R3_TILE; i += 256) qsh[i] = q16[(long)qt0 * R3_TILE + i];
    __syncthreads();
    const floatx16 zero = {};
    int t = blockIdx.x * tpw * 4 + wv;
    if (t >= ntiles) return;   // (after the only barrier)
    half8 a[R3_MFMA], n[R3_MFMA];
#pragma unroll
    for (int c = 0; c < R3_MFMA; ++c) a[c] = db16[(long)t * R3_TILE + c * 64 + lane];
    for (int it = 0; it < tpw; ++it, t += 4) {
        const int tn = t + 4;
        const bool more = it + 1 < tpw && tn < ntiles;
        if (more)
#pragma unroll
            for (int c = 0; c < R3_MFMA; ++c) n[c] = db16[(long)tn * R3_TILE + c * 64 + lane];
        // two query tiles per pass: both tiles' 22 operand reads issued first, the two
        // accumulation chains interleaved (each MFMA's operand and the other chain's MFMA
        // cover one another's latency; one wave per SIMD here), then both folds
        for (int j = 0; j < nq; j += 2) {
            const int j1 = j + 1 < nq ? j + 1 : j;
            const half8 *qb0 = qsh + j * R3_TILE + lane, *qb1 = qsh + j1 * R3_TILE + lane;
            half8 b0[R3_MFMA], b1[R3_MFMA];
#pragma unroll
            for (int c = 0; c < R3_MFMA; ++c) {
                b0[c] = qb0[c * 64];
                b1[c] = qb1[c * 64];
            }
            floatx16 acc0 = zero, acc1 = zero;
#pragma unroll
            for (int c = 0; c < R3_MFMA; ++c) {
                acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[c], b0[c], acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[c], b1[c], acc1, 0, 0, 0);
            }
            float mn0 = acc0[0], mn1 = acc1[0];
#pragma unroll
            for (int i = 1; i < 16; ++i) {
                mn0 = fminf(mn0, acc0[i]);
                mn1 = fminf(mn1, acc1[i]);
            }
            mn0 = fminf(mn0, __shfl_xor(mn0, 32));
            mn1 = fminf(mn1, __shfl_xor(mn1, 32));
            const int q0 = (qt0 + j) * 32 + lane, q1 = (qt0 + j1) * 32 + lane;
            if (lane < 32 && q0 < M) smin[(long)q0 * c3_stride(ntiles) + t] = mn0;
            if (lane < 32 && j1 != j && q1 < M) smin[(long)q1 * c3_stride(ntiles) + t] = mn1;
        }
        if (!more) break;
#pragma unroll
        for (int c = 0; c < R3_MFMA; ++c) a[c] = n[c];
    }
}
static inline dim3 screen3r_grid(int ntiles, int M, int &tpw) {
    const int QG = ((M + 31) / 32 + S3R_QG - 1) / S3R_QG;
    tpw = (int)std::max(1L, ((long)ntiles * QG + 4L * 512 - 1) / (4L * 512));
    return dim3((unsigned)((ntiles + 4 * tpw - 1) / (4 * tpw)), (unsigned)QG);
}

// eps of the R16c screen: u (850 A|q'| + 60 A^2) + 2^-9 1.01 A_skip |kappa_skip|
__device__ __forceinline__ double r3_eps(double A, double nqq, double askip, double nsk) {
    constexpr double U32 = 5.9604644775390625e-08;
    return U32 * (850.0 * A * sqrt(nqq) + 60.0 * A * A) + 0x1p-9 * 1.01 * askip * sqrt(nsk);
}
__device__ double r3_eps_m(const Rot3Meta *rm, double A, double nqq, double nsk) {
    return r3_eps(A, nqq, (double)__uint_as_float(rm->askip_bits), nsk);
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
    const double *nsk;           // R16c: |kappa_skip|^2 per query (null: the split-f16 screen)
    const Rot3Meta *rmeta;       // R16c: A_skip
};

// Thresholds of the colour exact stage: Tseg = e* + 2 eps3 in screen units,
// eps3 = u (900 A|q'| + 450 A^2); full scan when the norm slot nears the f16 floor
// (R16c, nsk >= 0: eps3 = r3_eps)
__device__ __forceinline__ double c3_tseg(float emin, float amax0, double nqq, bool &force_full,
                                          float askip = 0.f, double nsk = -1.0) {
    constexpr double U32 = 5.9604644775390625e-08;
    const double A = (double)amax0;
    const Split16Db sc = split16_db_scale(amax0);
    const int eq = split16_q_scale(nqq, sc.R);
    const int e2 = sc.ea + eq;
    const double em = ldexp((double)emin, -e2);
    const double eps3 = nsk >= 0.0 ? r3_eps(A, nqq, (double)askip, nsk)
                                   : U32 * (900.0 * A * sqrt(nqq) + 450.0 * A * A);
    const double slack = 1e-12 * (fabs(em) + nqq + A * A);
    force_full = eq + sc.R < -10;
    return ldexp(em + 2.0 * eps3 + slack, e2);
}

// ---- the exact stage + tail of the screened colour paths (k_exact3) ----------------------
// 8 threads per row: thread part j of a row holds features k = j + 8 i (i < 21), i.e. exactly
// Pw165's accumulator j of both halves (i < 10: k < 80; 10 <= i < 20: 80 <= k < 160) and,
// for j < 5, the tail term k = 160 + j.  All 21 loads issue before any use (one round trip),
// the accumulators are summed in Pw165's order in registers, and the row's part 0 finishes the
// two trees and the tail from LDS: the same value as pw165_sum / row3_dist, with no 165-term
// serial sum and no (row, feature) term array.
constexpr int R8_N = 21;
struct Acc8 {
    double p1, p2, pt, w1, w2, wt;   // plain / weighted: half 1, half 2, tail term
};
// thread part j's accumulators of row `row` (global fp64 rows, D3P stride) against qs / ws (LDS)
__device__ __forceinline__ Acc8 acc8_row(const double *__restrict__ row, int j, const double *qs,
                                         const double *ws) {
    double x[R8_N];
#pragma unroll
    for (int i = 0; i < R8_N; ++i) {
        const int k = j + 8 * i;
        x[i] = row[k < D3 ? k : 0];   // unconditional: every load before any use
    }
    Acc8 a{};
#pragma unroll
    for (int i = 0; i < R8_N; ++i) {
        const int k = j + 8 * i;
        const double d = x[i] - qs[k < D3 ? k : 0];
        const double dw = d * ws[k < D3 ? k : 0];
        const double tp = d * d, tw = dw * dw;
        if (i == 0) { a.p1 = tp; a.w1 = tw; }
        else if (i < 10) { a.p1 += tp; a.w1 += tw; }
        else if (i == 10) { a.p2 = tp; a.w2 = tw; }
        else if (i < 20) { a.p2 += tp; a.w2 += tw; }
        else if (k < D3) { a.pt = tp; a.wt = tw; }
    }
    return a;
}
// part 0 of a row: Pw165's value from the 8 parts' accumulators (LDS, acc[0..7])
__device__ __forceinline__ double acc8_sum(const Acc8 *acc, bool weighted) {
    double r1[8], r2[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        r1[j] = weighted ? acc[j].w1 : acc[j].p1;
        r2[j] = weighted ? acc[j].w2 : acc[j].p2;
    }
    const double h1 = Pw165::tree(r1);
    double h2 = Pw165::tree(r2);
#pragma unroll
    for (int j = 0; j < D3 - 160; ++j) h2 += weighted ? acc[j].wt : acc[j].pt;
    return h1 + h2;
}

// The exact stage of the screened paths (k_screen3 / k_screen3r) and the per-pixel tail, one
// 256-thread workgroup per pixel: the query, weights, the coherence window's s / im and the
// query's tile minima (float4s in registers) in one round trip; e* and the tiles within the
// threshold; then per candidate tile its 32 rows, 8 threads each (acc8_row: plain and weighted
// sums, so the winner's weighted distance needs no second read), with the 15 coherence rows
// in the first tile's round trip; the lexicographic (distance, row) minimum carries its
// weighted distance; coherence pick, kappa test and the B' update as k_finish3w.
// FUSE (the R16c path, IA_C3_FUSE): the same launch also writes the query rows of wave t + 1
// (as k_query3r / r3_query; k_xwave's scheme): the workgroup of pixel (y, x)
// builds the row of (y, x + 1).  Of its 165 features only the B' samples of two pixels can
// come from wave t: this pixel (its new value, from LDS) and the upper neighbour (y - 1,
// x + 3) (its three new channels from six tagged 8-byte decision granules, dbox[8 (y - 1)
// ...]); the rest are loaded at the start.  Pixels take their index from a ticket counter, so a
// workgroup waits only for a lower ticket (dispatched earlier); extra workgroups (index >= M)
// build the first row of the rows that enter wave t + 1.  Query buffers alternate by wave parity.
struct Nx3 {
    Img3 Bsm, Blg, Bpsm, Bplg;
    int M, y_lo_n, M_n, H;
    const Col16Meta *meta;
    const float *rot;
    double *q3n, *qnn, *nskn;
    half8 *q16n;
    unsigned *tickets;            // [2]; tickets[t & 1] is this launch's
    unsigned *err;                // a decision wait timed out
    unsigned long long *dbox;     // 8 granules per row: channel c's bits at 2c (lo), 2c + 1 (hi)
};
constexpr unsigned long long C3_WAIT_TICKS = 1000000000ULL;   // 10 s of s_memrealtime
__device__ __forceinline__ unsigned long long c3_gran(unsigned tag, unsigned bits) {
    return ((unsigned long long)tag << 32) | bits;
}

template <bool FUSE>
__global__ __launch_bounds__(256) void k_exact3(Fin3 f, Scr3 sc, Nx3 nx) {
    __shared__ double qs[D3P], wsh[D3P];
    __shared__ double ownv[3], nbv[3], qred[4], qds[D3];
    __shared__ int tks, anydep;
    __shared__ Acc8 acc[32 * 8];                // a tile's rows (32 x 8 parts)
    __shared__ Acc8 cacc[15 * 8];               // the coherence rows
    __shared__ double sump[15], sumw[15];
    __shared__ long long rix[15];
    __shared__ int rpos[15][3];
    __shared__ double rd[4], rw[4];
    __shared__ long long ri[4];
    __shared__ float fmn[4];
    __shared__ int clist[C3_CAND], ccount;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    int m = blockIdx.x;
    if constexpr (FUSE) {
        if (tid == 0) {
            tks = (int)atomicAdd(&nx.tickets[f.t & 1], 1u);
            anydep = 0;
        }
        __syncthreads();
        m = tks;
        if (m == 0 && tid == 0) __hip_atomic_store(&nx.tickets[(f.t + 1) & 1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    const int ro = tid >> 3, j = tid & 7;
    const int y = f.y_lo + m, x = f.t - 3 * y;
    const int W = f.W, Ah = f.Ah, Aw = f.Aw;
    const long hw = (long)Ah * Aw;
    const bool first = y == 0 && x == 0;
    const bool cur = !FUSE || m < nx.M;
    const bool nxt = FUSE && y >= nx.y_lo_n && y < nx.y_lo_n + nx.M_n;
    // FUSE: feature tid of the next query (y, x + 1): loaded now unless it is a wave-t sample
    double nv = 0.0;
    int dep = 0, dch = 0;
    if (FUSE && nxt && tid < D3) {
        const int X = x + 1;
        if (tid < D3_FULL) {
            nv = feat3(nx.Bsm, nx.Blg, y, X, tid);
        } else if (tid < D3_FULL + 27) {
            nv = feat3(nx.Bpsm, nx.Bplg, y, X, tid - D3_FULL);
        } else {
            const int t2 = (tid - D3_FULL - 27) / 3;
            dch = (tid - D3_FULL - 27) - 3 * t2;
            const int rr = symi2(y + t2 / 5 - 2, nx.H), cc = symi2(X + t2 % 5 - 2, W);
            dep = (rr == y && cc == x) ? 1 : (rr == y - 1 && cc == x + 3) ? 2 : 0;
            if (dep == 0) nv = nx.Bplg.p[((long)rr * W + cc) * 3 + dch];
        }
        if (dep == 2) anydep = 1;
    }
    if (cur) {
    // ---- one round trip: query, weights, coherence s / im, tile minima
    if (tid < D3P) {
        qs[tid] = f.q3[(long)m * D3P + tid];
        wsh[tid] = tid < D3 ? f.weights[tid] : 0.0;
    }
    if (tid < 15) {
        long long cix = -1;
        int cr = 0, cc = 0, cim = 0;
        if (!first) {
            const int rr = y - 2 + tid / 5, rc = x - 2 + tid % 5;
            if (rr >= 0 && rc >= 0 && rc < W && (rr < y || rc < x)) {
                const long sidx = (long)rr * W + rc;
                const int sr = f.s[2 * sidx] + y - rr, scc = f.s[2 * sidx + 1] + x - rc;
                if (sr >= 0 && sr < Ah && scc >= 0 && scc < Aw) {
                    const int simg = f.im[sidx];
                    cix = ((long)Ah * simg + sr) * Aw + scc;
                    cr = sr; cc = scc; cim = simg;
                }
            }
        }
        rix[tid] = cix;
        rpos[tid][0] = cr; rpos[tid][1] = cc; rpos[tid][2] = cim;
    }
    const int stride = c3_stride(sc.ntiles);
    const float4 *sm4 = reinterpret_cast<const float4 *>(sc.smin + (long)m * stride);
    const int n4 = stride / 4;
    float4 v[C3_REG];
#pragma unroll
    for (int q = 0; q < C3_REG; ++q) {
        const int i = tid + 256 * q;
        v[q] = sm4[i < n4 ? i : 0];
    }
    auto masked = [&](float4 xx, int i) {   // +inf past the tiles (and the float4 pad)
        const int b = 4 * i;
        xx.x = b + 0 < sc.ntiles && i < n4 ? xx.x : INFINITY;
        xx.y = b + 1 < sc.ntiles && i < n4 ? xx.y : INFINITY;
        xx.z = b + 2 < sc.ntiles && i < n4 ? xx.z : INFINITY;
        xx.w = b + 3 < sc.ntiles && i < n4 ? xx.w : INFINITY;
        return xx;
    };
    float mn = INFINITY;
#pragma unroll
    for (int q = 0; q < C3_REG; ++q) {
        v[q] = masked(v[q], tid + 256 * q);
        mn = fminf(mn, fminf(fminf(v[q].x, v[q].y), fminf(v[q].z, v[q].w)));
    }
    for (int i = tid + 256 * C3_REG; i < n4; i += 256) {
        const float4 xx = masked(sm4[i], i);
        mn = fminf(mn, fminf(fminf(xx.x, xx.y), fminf(xx.z, xx.w)));
    }
    for (int o = 32; o > 0; o >>= 1) mn = fminf(mn, __shfl_xor(mn, o));
    if (lane == 0) fmn[wv] = mn;
    if (tid == 0) ccount = 0;
    __syncthreads();
    // ---- the candidate tiles
    mn = fminf(fminf(fmn[0], fmn[1]), fminf(fmn[2], fmn[3]));
    bool full;
    const float amax = __uint_as_float(sc.meta->amax_bits);
    const double Tseg = sc.nsk ? c3_tseg(mn, amax, sc.qn[m], full, __uint_as_float(sc.rmeta->askip_bits), sc.nsk[m])
                               : c3_tseg(mn, amax, sc.qn[m], full);
    if (!full) {
        auto pick = [&](float4 xx, int i) {
            const float e4[4] = {xx.x, xx.y, xx.z, xx.w};
#pragma unroll
            for (int e = 0; e < 4; ++e)
                if ((double)e4[e] <= Tseg) {
                    const int c = atomicAdd(&ccount, 1);
                    if (c < C3_CAND) clist[c] = 4 * i + e;
                }
        };
#pragma unroll
        for (int q = 0; q < C3_REG; ++q) pick(v[q], tid + 256 * q);
        for (int i = tid + 256 * C3_REG; i < n4; i += 256) pick(masked(sm4[i], i), i);
    }
    __syncthreads();
    const int nc = ccount;
    full = full || nc > C3_CAND;
    const int ntl = full ? sc.ntiles : nc;
    if (tid == 0 && sc.stats) {
        atomicAdd(&sc.stats[0], (unsigned long long)ntl);
        if (full) atomicAdd(&sc.stats[1], 1ull);
    }
    // ---- every row of the candidate tiles (and, with the first, the coherence rows)
    double bd = INFINITY, bw = 0.0;
    long long bi = 0x7fffffffffffffffLL;
    const int nit = ntl > 0 ? ntl : 1;
    for (int b = 0; b < nit; ++b) {
        Acc8 ta{}, ca{};
        const long r0 = ntl > 0 ? (long)(full ? b : clist[b]) * 32 : 0;
        const long r = r0 + ro < sc.nrows ? r0 + ro : sc.nrows - 1;   // (rows past nrows: not taken)
        if (ntl > 0) ta = acc8_row(f.db3 + r * D3P, j, qs, wsh);
        if (b == 0 && tid < 15 * 8) {
            const long long ix = rix[ro];
            ca = acc8_row(f.db3 + (ix >= 0 ? ix : 0) * D3P, j, qs, wsh);
        }
        acc[tid] = ta;
        if (b == 0 && tid < 15 * 8) cacc[tid] = ca;
        __syncthreads();
        if (j == 0 && ntl > 0 && r0 + ro < sc.nrows) {
            const double d = acc8_sum(acc + 8 * ro, false);
            if (d < bd || (d == bd && r0 + ro < bi)) {
                bd = d;
                bi = r0 + ro;
                const double sq = sqrt(acc8_sum(acc + 8 * ro, true));
                bw = sq * sq;
            }
        }
        if (b == 0 && j == 0 && tid < 15 * 8) {
            if (rix[ro] >= 0) {
                sump[ro] = sqrt(acc8_sum(cacc + 8 * ro, false));
                const double sq = sqrt(acc8_sum(cacc + 8 * ro, true));
                sumw[ro] = sq * sq;
            } else {
                sump[ro] = INFINITY;
                sumw[ro] = 0.0;
            }
        }
        __syncthreads();   // acc is refilled by the next tile
    }
    for (int o = 32; o > 0; o >>= 1) {
        const double od = __shfl_xor(bd, o), ow = __shfl_xor(bw, o);
        const long long oi = __shfl_xor(bi, o);
        if (od < bd || (od == bd && oi < bi)) { bd = od; bi = oi; bw = ow; }
    }
    if (lane == 0) { rd[wv] = bd; ri[wv] = bi; rw[wv] = bw; }
    __syncthreads();
    if (wv == 0) {
    double wd = rd[0], ww = rw[0];
    long long wi = ri[0];
#pragma unroll
    for (int w = 1; w < 4; ++w)
        if (rd[w] < wd || (rd[w] == wd && ri[w] < wi)) { wd = rd[w]; wi = ri[w]; ww = rw[w]; }
    const long long app = wi;
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
    const double d_app = valid ? ww : 0.0, d_coh = valid ? sumw[win] : 0.0;
    long img = app / hw;
    long rem = app - img * hw;
    const int ar = (int)(rem / Aw), ac = (int)(rem - (long)(rem / Aw) * Aw);
    int pr = ar, pc = ac;
    if (valid && d_coh <= d_app * f.kappa_factor) { pr = wr; pc = wc; img = wim; }
    const long qpx = (long)y * W + x;
    if (lane < 3) {
        const double val = f.Ap_lg[((img * hw) + (long)pr * Aw + pc) * 3 + lane];
        f.Bp_lg[qpx * 3 + lane] = val;
        if constexpr (FUSE) {
            // the decision for the lower neighbour's next query, and this pixel's own
            ownv[lane] = val;
            const unsigned long long bits = (unsigned long long)__double_as_longlong(val);
            unsigned long long *d = nx.dbox + 8 * (long)y + 2 * lane;
            __hip_atomic_store(d, c3_gran(f.t + 1, (unsigned)bits), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(d + 1, c3_gran(f.t + 1, (unsigned)(bits >> 32)), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
    }
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
    }   // wave 0
    }   // cur
    if constexpr (FUSE) {
        __syncthreads();   // ownv, anydep
        if (nxt) {
            if (anydep && tid == 0) {   // the upper neighbour (ticket m - 1) decided (y - 1, x + 3)
                const unsigned long long *d = nx.dbox + 8 * (long)(y - 1);
                const unsigned tag = (unsigned)(f.t + 1);
                const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
                for (;;) {
                    bool ok = true;
                    unsigned long long g[6];
#pragma unroll
                    for (int c = 0; c < 6; ++c) {
                        g[c] = __hip_atomic_load(d + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        ok = ok && (unsigned)(g[c] >> 32) == tag;
                    }
                    if (ok) {
#pragma unroll
                        for (int c = 0; c < 3; ++c)
                            nbv[c] = __longlong_as_double(
                                (long long)(((g[2 * c + 1] & 0xffffffffULL) << 32) | (g[2 * c] & 0xffffffffULL)));
                        break;
                    }
                    if (__builtin_amdgcn_s_memrealtime() - t0 > C3_WAIT_TICKS) {
                        atomicOr(nx.err, 1u);
                        nbv[0] = nbv[1] = nbv[2] = 0.0;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
            }
            __syncthreads();
            const double v = dep == 1 ? ownv[dch] : dep == 2 ? nbv[dch] : nv;
            const int mq = y - nx.y_lo_n;
            if (tid < D3P) nx.q3n[(long)mq * D3P + tid] = tid < D3 ? v : 0.0;
            r3_query(mq, nx.M_n, tid, v, nx.meta, nx.rot, nx.qnn, nx.nskn, nx.q16n, qds, qred);
        }
    }
}

// The per-pixel tail of the exhaustive fp64 search (IA_COLOR16=0), one 256-thread workgroup
// per pixel: the winner is the lexicographic minimum of k_match3's partials (order free); the
// 15 coherence candidates' and the winner's rows are read once, lane-parallel over (row,
// feature); their plain and weighted squared terms go to LDS, and 31 threads sum one row each
// (Pw165): the same values as row3_dist.
__global__ __launch_bounds__(256) void k_finish3w(Fin3 f, const Best *__restrict__ part, int nb) {
    __shared__ double qs[D3P], wsh[D3P];
    __shared__ double tp[15][D3], tw[16][D3];   // coherence rows: plain, weighted (+ winner)
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
    // the query, the weights, the partials' minimum and the
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
    for (int i = tid; i < nb; i += 256) best3(bd, bi, part[(long)m * nb + i].d, part[(long)m * nb + i].idx);
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

// IA_COLOR16 (ia_diag_set_color16): 1 the split-f16 screen + exact stage, 0 the exhaustive
// fp64 search (k_match3)
static std::atomic<int> g_color16{env_int("IA_COLOR16", 1)};
static unsigned long long *g_c3_stats = nullptr;   // diagnostic counters (ia_diag_color16_stats)

// the synthesis workspace: q3 | best | partials (fp64 search) | q16 | qn | tile minima, and for
// the fused R16c tail (k_exact3<true>) the odd waves' query set, the control words and the
// decision granules
struct Ws3 {
    double *q3;
    Best *best, *part;
    half8 *q16;              // the query tiles of either screen (C16_TILE >= R3_TILE)
    double *qn, *nsk;
    float *smin;
    double *q3b, *qnb, *nskb;
    half8 *q16b;
    unsigned *ctl;           // tickets[2], error word
    unsigned long long *dbox;
};
constexpr int C3_CTL_ERR = 2;
// the fused colour tail (k_exact3<true>: the next wave's query rows from the exact stage's
// launch; IA_C3_FUSE, default 1) on R16c levels
static inline bool c3_fuse() {
    static const int v = env_int("IA_C3_FUSE", 1);
    return v != 0;
}
static_assert(C16_TILE >= R3_TILE, "query tiles");
static inline size_t ws3_layout(int H, int W, long nrows, char *base, Ws3 *w) {
    const size_t M = (size_t)max_wave(H, W), Mp = (M + 31) / 32 * 32;
    size_t o = 0;
    auto take = [&](size_t bytes) { char *p = base ? base + o : nullptr; o += align_up(bytes, 256); return p; };
    char *q3 = take(Mp * D3P * sizeof(double));
    char *best = take(M * sizeof(Best));
    char *part = take(M * (size_t)match3_blocks(nrows) * sizeof(Best));
    char *q16 = take(Mp / 32 * C16_TILE * sizeof(half8));
    char *qn = take(Mp * sizeof(double));
    char *nsk = take(Mp * sizeof(double));
    char *smin = take(M * (size_t)c3_stride((int)db3_tiles(nrows)) * sizeof(float));
    char *q3b = take(Mp * D3P * sizeof(double));
    char *q16b = take(Mp / 32 * C16_TILE * sizeof(half8));
    char *qnb = take(Mp * sizeof(double));
    char *nskb = take(Mp * sizeof(double));
    char *ctl = take(256);
    char *dbox = take((size_t)H * 8 * sizeof(unsigned long long));
    if (w) {
        w->q3b = reinterpret_cast<double *>(q3b);
        w->q16b = reinterpret_cast<half8 *>(q16b);
        w->qnb = reinterpret_cast<double *>(qnb);
        w->nskb = reinterpret_cast<double *>(nskb);
        w->ctl = reinterpret_cast<unsigned *>(ctl);
        w->dbox = reinterpret_cast<unsigned long long *>(dbox);
        w->q3 = reinterpret_cast<double *>(q3);
        w->best = reinterpret_cast<Best *>(best);
        w->part = reinterpret_cast<Best *>(part);
        w->q16 = reinterpret_cast<half8 *>(q16);
        w->qn = reinterpret_cast<double *>(qn);
        w->nsk = reinterpret_cast<double *>(nsk);
        w->smin = reinterpret_cast<float *>(smin);
    }
    return o;
}

// one 3-channel level on one GPU: the wave loop of ia_synth_level3 (per wave: the query
// rows and split operand, the screen, the exact stage + tail; or the exhaustive fp64 search)
struct Level3 {
    const IaSynthArgs *a = nullptr;
    Ws3 w{};
    Db3View v{};
    Fin3 f{};
    Scr3 sc{};
    Img3 Bsm{}, Blg{}, Bpsm{}, Bplg{};
    int H = 0, W = 0, nw = 0, nb = 0, ntiles = 0;
    bool split = true, rot = false;   // rot: the R16c screen (a->dbr, a->rot: ia_db3_build_rot)
    bool fuse = false;                // rot with the fused tail (k_exact3<true>)
    const half8 *dbr = nullptr;
    int init(const IaSynthArgs *a_, hipStream_t st) {
        a = a_;
        IA_ARG(a && a->db && a->B_sm && a->B_lg && a->Bp_sm && a->Bp_lg && a->weights && a->s && a->im &&
                   a->workspace && a->H > 0 && a->W > 0,
               "ia_synth_level3: bad args");
        IA_ARG(!a->comm && !a->lsh && a->row0 == 0 && a->nrows == (long)a->src.nAp * a->src.Ah * a->src.Aw,
               "ia_synth_level3: 3-channel matching runs unsharded with the exact matcher");
        IA_ARG(!a->dbg_px == !a->dbg_dist, "ia_synth_level3: debug outputs come in pairs");
        H = a->H;
        W = a->W;
        ws3_layout(H, W, a->nrows, reinterpret_cast<char *>(a->workspace), &w);
        nb = match3_blocks(a->nrows);
        Bsm = Img3{a->B_sm, a->B_hs, a->B_ws};
        Blg = Img3{a->B_lg, H, W};
        Bpsm = Img3{a->Bp_sm, a->B_hs, a->B_ws};
        Bplg = Img3{a->Bp_lg, H, W};
        v = db3_view(const_cast<void *>(a->db), a->nrows);
        f = Fin3{v.rows, w.q3, w.best, a->src.Ap_lg, a->src.Ah, a->src.Aw,
                 0, 0, W, a->weights, a->kappa_factor, a->Bp_lg, a->s, a->im, a->dbg_px, a->dbg_dist};
        split = g_color16.load(std::memory_order_relaxed) != 0;
        ntiles = (int)v.ntiles;
        rot = split && a->dbr && a->rot;
        dbr = reinterpret_cast<const half8 *>(a->dbr);
        sc = Scr3{w.smin, ntiles, a->nrows, w.qn, v.meta, g_c3_stats, rot ? w.nsk : nullptr,
                  rot ? db3r_meta(const_cast<void *>(a->dbr), a->nrows) : nullptr};
        nw = (W - 1) + 3 * (H - 1) + 1;
        fuse = rot && c3_fuse();
        IA_HIP(hipMemsetAsync(w.ctl, 0, 256, st));
        if (fuse) IA_HIP(hipMemsetAsync(w.dbox, 0, (size_t)H * 8 * sizeof(unsigned long long), st));
        return IA_OK;
    }
    static void rows(int H, int W, int t, int &y_lo, int &M) {
        y_lo = std::max(0, (t - (W - 1) + 2) / 3);
        M = std::min(H - 1, t / 3) - y_lo + 1;
    }
    int wave(int t, hipStream_t st) {
        int y_lo, M;
        rows(H, W, t, y_lo, M);
        if (M <= 0) return IA_OK;
        f.t = t;
        f.y_lo = y_lo;
        if (fuse) {
            // wave t's query set b (wave 0's built here, the later ones by the previous wave's
            // k_exact3<true>), wave t + 1's into set b ^ 1
            const int b = t & 1;
            double *q3s[2] = {w.q3, w.q3b}, *qns[2] = {w.qn, w.qnb}, *nsks[2] = {w.nsk, w.nskb};
            half8 *q16s[2] = {w.q16, w.q16b};
            int tpw;
            const dim3 grid = screen3r_grid(ntiles, M, tpw);
            if (t == 0)
                k_query3r<<<(M + 31) / 32 * 32, 256, 0, st>>>(Bsm, Blg, Bpsm, Bplg, t, y_lo, M, v.meta, a->rot, nullptr,
                                                              q3s[0], qns[0], nsks[0], q16s[0]);
            k_screen3r<<<grid, 256, 0, st>>>(dbr, ntiles, q16s[b], M, tpw, w.smin);
            int y_lo_n = 0, M_n = 0;
            if (t + 1 < nw) rows(H, W, t + 1, y_lo_n, M_n);
            const Nx3 nx{Bsm, Blg, Bpsm, Bplg, M, y_lo_n, M_n, H, v.meta, a->rot, q3s[b ^ 1], qns[b ^ 1],
                         nsks[b ^ 1], q16s[b ^ 1], w.ctl, w.ctl + C3_CTL_ERR, w.dbox};
            Fin3 fb = f;
            fb.q3 = q3s[b];
            Scr3 sb = sc;
            sb.qn = qns[b];
            sb.nsk = nsks[b];
            const int R = std::max(M, M_n > 0 ? y_lo_n + M_n - y_lo : 0);
            k_exact3<true><<<R, 256, 0, st>>>(fb, sb, nx);
        } else if (rot) {
            const int QT = (M + 31) / 32;
            int tpw;
            const dim3 grid = screen3r_grid(ntiles, M, tpw);
            k_query3r<<<QT * 32, 256, 0, st>>>(Bsm, Blg, Bpsm, Bplg, t, y_lo, M, v.meta, a->rot, nullptr, w.q3,
                                               w.qn, w.nsk, w.q16);
            k_screen3r<<<grid, 256, 0, st>>>(dbr, ntiles, w.q16, M, tpw, w.smin);
            k_exact3<false><<<M, 256, 0, st>>>(f, sc, Nx3{});
        } else if (split) {
            const int QT = (M + 31) / 32;
            int tpw;
            const dim3 grid = screen3_grid(ntiles, M, tpw);
            k_query3s<<<QT * 32, 256, 0, st>>>(Bsm, Blg, Bpsm, Bplg, t, y_lo, M, v.meta, w.q3, w.qn,
                                               reinterpret_cast<_Float16 *>(w.q16));
            k_screen3<<<grid, 256, 0, st>>>(v.db16, ntiles, w.q16, M, tpw, w.smin);
            k_exact3<false><<<M, 256, 0, st>>>(f, sc, Nx3{});
        } else {
            k_query3<<<M, 256, 0, st>>>(Bsm, Blg, Bpsm, Bplg, t, y_lo, w.q3);
            k_match3<<<nb, 256, 0, st>>>(f.db3, a->nrows, 0, w.q3, M, w.part);
            k_finish3w<<<M, 256, 0, st>>>(f, w.part, nb);
        }
        IA_LAUNCH_CHECK("ia_synth_level3 wave");
        return IA_OK;
    }
};

// the coarse waves wave t of level a reads (ia_synth.hip coarse_need: the 3x3 coarse window
// of pixel (y, x) reaches (y/2 + 1, x/2 + 1), clamped to the coarse level)
static int c3_need(const IaSynthArgs &a, int t) {
    int y_lo, M;
    Level3::rows(a.H, a.W, t, y_lo, M);
    int need = 0;
    for (int y = y_lo; y < y_lo + M; ++y) {
        const int x = t - 3 * y;
        const int cy = std::min(y / 2 + 1, a.B_hs - 1), cx = std::min(x / 2 + 1, a.B_ws - 1);
        need = std::max(need, cx + 3 * cy);
    }
    return need;
}
// 8 against 4 at the c3 size, same box, A/B/A/B: 112.6 / 111.0 vs 113.8 / 112.6 ms per
// step, same checksum (profiles/r06_pipe_block_ab.txt)
#ifndef IA_C3_PIPE_BLOCK
#define IA_C3_PIPE_BLOCK 8
#endif
constexpr int C3_PIPE_BLOCK = IA_C3_PIPE_BLOCK;   // waves per recorded event (build-time)

struct Pipe3 {   // per host thread: the level streams and events of ia_synth_levels3
    std::vector<hipStream_t> hi;   // levels 0 .. n-2 of a call (the coarser ones): high priority
    hipStream_t plain = nullptr;   // level n-1 (the finest): plain priority
    std::vector<hipEvent_t> events;
    size_t next = 0;
    hipEvent_t last = nullptr;     // the previous call's end (IA_PIPE_DRAIN, ia_synth.hip)
    bool last_rec = false;
    // the streams of an n-level call: the pools grow as needed, and the finest level always
    // takes the plain stream whatever n the first call had
    hipError_t streams(int n, std::vector<hipStream_t> &out) {
        hipError_t r = hipSuccess;
        int lo = 0, pr = 0;
        if ((r = hipDeviceGetStreamPriorityRange(&lo, &pr)) != hipSuccess) return r;
        while ((int)hi.size() < n - 1) {
            hipStream_t s;
            if ((r = hipStreamCreateWithPriority(&s, hipStreamNonBlocking, pr)) != hipSuccess) return r;
            hi.push_back(s);
        }
        if (!plain && (r = hipStreamCreateWithFlags(&plain, hipStreamNonBlocking)) != hipSuccess) return r;
        out.assign(hi.begin(), hi.begin() + (n - 1));
        out.push_back(plain);
        return r;
    }
    hipError_t release() {
        hipError_t r = hipSuccess;
        for (hipStream_t s : hi)
            if (r == hipSuccess) r = hipStreamDestroy(s);
        if (plain && r == hipSuccess) r = hipStreamDestroy(plain);
        for (hipEvent_t e : events)
            if (r == hipSuccess) r = hipEventDestroy(e);
        if (last && r == hipSuccess) r = hipEventDestroy(last);
        last = nullptr;
        last_rec = false;
        hi.clear();
        plain = nullptr;
        events.clear();
        next = 0;
        return r;
    }
    hipError_t event(hipEvent_t *e) {
        if (next == events.size()) {
            hipEvent_t x;
            hipError_t r = hipEventCreateWithFlags(&x, hipEventDisableTiming);
            if (r != hipSuccess) return r;
            events.push_back(x);
        }
        *e = events[next++];
        return hipSuccess;
    }
};
static thread_local Pipe3 g_pipe3;
// ia_release_thread_resources (ia_synth.hip): this thread's colour pipeline streams and events
int release_pipe3() {
    IA_HIP(g_pipe3.release());
    return IA_OK;
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

size_t ia_db3_rot_bytes(long nrows) { return nrows > 0 ? db3r_tiles_bytes(nrows) + sizeof(Rot3Meta) : 0; }

size_t ia_db3_cov_bytes(void) {
    return (size_t)(D3 * D3P + D3P + C3C_SPLIT * D3P + (size_t)C3C_SPLIT * D3 * D3P) * sizeof(double);
}

int ia_db3_cov(const double *db3, long nrows, double *cov, void *stream) {
    IA_ARG(db3 && cov && nrows > 0, "ia_db3_cov: bad args");
    hipStream_t st = S(stream);
    const long step = nrows / 65536 > 1 ? nrows / 65536 : 1;
    const long nsamp = (nrows + step - 1) / step;
    double *mean = cov + D3 * D3P, *cpart = mean + D3P, *vpart = cpart + C3C_SPLIT * D3P;
    k_db3_colsum<<<C3C_SPLIT, 256, 0, st>>>(db3, step, nsamp, cpart);
    k_db3_mean<<<1, 256, 0, st>>>(cpart, nsamp, mean);
    k_db3_cov<<<dim3(C3C_NA, C3C_SPLIT), 256, 0, st>>>(db3, step, nsamp, mean, vpart);
    k_db3_cov_reduce<<<D3, 256, 0, st>>>(vpart, cov);
    IA_LAUNCH_CHECK("ia_db3_cov");
    return IA_OK;
}
int ia_db3_rot_components(void) { return R3_P; }
int ia_db3_rot_floats(void) { return R3_ROT_FLOATS; }

int ia_db3_build_rot(const double *db3, long nrows, const float *rot, void *dbr, void *stream) {
    IA_ARG(db3 && rot && dbr && nrows > 0, "ia_db3_build_rot: bad args");
    hipStream_t st = S(stream);
    {
        const int rc = rot_check_orthonormal(rot, D3, R3_LD, st, "ia_db3_build_rot");
        if (rc) return rc;
    }
    const Db3View v = db3_view(const_cast<double *>(db3), nrows);
    Rot3Meta *rm = db3r_meta(dbr, nrows);
    IA_HIP(hipMemsetAsync(rm, 0, sizeof(Rot3Meta), st));
    k_db3_rot<<<(unsigned)v.ntiles, 256, 0, st>>>(v.rows, nrows, v.meta, rot, reinterpret_cast<half8 *>(dbr), rm);
    IA_LAUNCH_CHECK("ia_db3_build_rot");
    return IA_OK;
}

/* diagnostics: A_skip of a rotated 3-channel DB and the R16c screen of M given query rows
 * (M x 165): tile minima in unscaled units e[M][ntiles], eps (r3_eps) and |q'|^2 per query */
int ia_diag_db3_askip(const void *dbr, long nrows, float *out) {
    IA_ARG(dbr && out && nrows > 0, "ia_diag_db3_askip: bad args");
    unsigned int b = 0;
    IA_HIP(hipMemcpy(&b, &db3r_meta(const_cast<void *>(dbr), nrows)->askip_bits, 4, hipMemcpyDeviceToHost));
    std::memcpy(out, &b, 4);
    return IA_OK;
}

int ia_synth3_status(const IaSynthArgs *levels, int n, void *stream) {
    IA_ARG(levels && n >= 1, "ia_synth3_status: bad args");
    IA_HIP(hipStreamSynchronize(S(stream)));
    for (int j = 0; j < n; ++j) {
        const IaSynthArgs &a = levels[j];
        IA_ARG(a.workspace && a.H > 0 && a.W > 0 && a.nrows > 0, "ia_synth3_status: bad level");
        Ws3 w{};
        ws3_layout(a.H, a.W, a.nrows, reinterpret_cast<char *>(a.workspace), &w);
        unsigned e = 0;
        IA_HIP(hipMemcpy(&e, w.ctl + C3_CTL_ERR, sizeof(e), hipMemcpyDeviceToHost));
        if (e) {
            set_error("ia_synth3_status: a wait for a neighbouring pixel's decision timed out "
                      "(device schedule fault)");
            return IA_E_SCHED;
        }
    }
    return IA_OK;
}

int ia_synth_level3(const IaSynthArgs *a, void *stream) {
    hipStream_t st = S(stream);
    Level3 run;
    int rc = run.init(a, st);
    if (rc) return rc;
    for (int t = 0; t < run.nw; ++t)
        if ((rc = run.wave(t, st))) return rc;
    return IA_OK;
}

/* n consecutive 3-channel levels, pipelined as ia_synth_levels (ia_synth.hip): one stream per
 * level (the coarser ones at high priority), level j's wave t launched behind an event of
 * level j - 1 covering the coarse waves its pixels read (c3_need). */
int ia_synth_levels3(const IaSynthArgs *levels, int n, void *stream) {
    IA_ARG(levels && n >= 1 && n <= 64, "ia_synth_levels3: bad level count");
    for (int j = 1; j < n; ++j)
        IA_ARG(levels[j].Bp_sm == levels[j - 1].Bp_lg && levels[j].B_hs == levels[j - 1].H &&
                   levels[j].B_ws == levels[j - 1].W,
               "ia_synth_levels3: levels must be consecutive (level j's coarse B' = level j-1's B')");
    hipStream_t st = S(stream);
    Pipe3 &P = g_pipe3;
    // the previous call of this thread ends first (IA_PIPE_DRAIN, default 1: packets queued
    // in the high-priority streams behind a running call slow its finest level, ia_synth.hip)
    static const int drain = env_int("IA_PIPE_DRAIN", 1);
    if (drain && P.last_rec) IA_HIP(hipEventSynchronize(P.last));
    std::vector<hipStream_t> ss;   // ss[j] runs level j: high priority but the finest
    IA_HIP(P.streams(n, ss));
    P.next = 0;
    hipEvent_t start;
    IA_HIP(P.event(&start));
    IA_HIP(hipEventRecord(start, st));
    std::vector<Level3> run(n);
    std::vector<std::vector<hipEvent_t>> blk(n);   // blk[j][b]: level j done through block b
    for (int j = 0; j < n; ++j) {
        IA_HIP(hipStreamWaitEvent(ss[j], start, 0));   // (init's memsets too: after the caller's work)
        int rc = run[j].init(&levels[j], ss[j]);
        if (rc) return rc;
        blk[j].assign((run[j].nw + C3_PIPE_BLOCK - 1) / C3_PIPE_BLOCK, nullptr);
    }
    // every level whole, coarse to fine: a level's waits name events already recorded
    for (int j = 0; j < n; ++j) {
        hipStream_t sj = ss[j];
        int waited = -1;
        for (int t = 0; t < run[j].nw; ++t) {
            if (j > 0) {
                // (the fused tail's launch of wave t also builds wave t + 1's query rows)
                const int w = c3_need(levels[j], run[j].fuse && t + 1 < run[j].nw ? t + 1 : t);
                if (w > waited) {
                    const int b = w / C3_PIPE_BLOCK;
                    IA_HIP(hipStreamWaitEvent(sj, blk[j - 1][b], 0));
                    waited = b * C3_PIPE_BLOCK + C3_PIPE_BLOCK - 1;
                }
            }
            int rc = run[j].wave(t, sj);
            if (rc) return rc;
            if ((t + 1) % C3_PIPE_BLOCK == 0 || t == run[j].nw - 1) {
                hipEvent_t e;
                IA_HIP(P.event(&e));
                IA_HIP(hipEventRecord(e, sj));
                blk[j][t / C3_PIPE_BLOCK] = e;
            }
        }
    }
    for (int j = 0; j < n; ++j) {
        hipEvent_t e;
        IA_HIP(P.event(&e));
        IA_HIP(hipEventRecord(e, ss[j]));
        IA_HIP(hipStreamWaitEvent(st, e, 0));
    }
    if (!P.last) IA_HIP(hipEventCreateWithFlags(&P.last, hipEventDisableTiming));
    IA_HIP(hipEventRecord(P.last, st));
    P.last_rec = true;
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
    IA_HIP(hipMalloc(&smin, (size_t)M * c3_stride(ntiles) * sizeof(float)));
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

int ia_diag_screen3r(const void *db3, const void *dbr, const float *rot, long nrows, const double *q165, int M,
                     double *e, double *eps, double *qn) {
    IA_ARG(db3 && dbr && rot && q165 && e && eps && qn && nrows > 0 && M > 0, "ia_diag_screen3r: bad args");
    const Db3View v = db3_view(const_cast<void *>(db3), nrows);
    const int QT = (M + 31) / 32, ntiles = (int)v.ntiles;
    half8 *q16 = nullptr;
    float *smin = nullptr;
    double *nsk = nullptr;
    IA_HIP(hipMalloc(&q16, (size_t)QT * R3_TILE * sizeof(half8)));
    IA_HIP(hipMalloc(&smin, (size_t)M * c3_stride(ntiles) * sizeof(float)));
    IA_HIP(hipMalloc(&nsk, (size_t)QT * 32 * sizeof(double)));
    const Img3 z{nullptr, 0, 0};
    k_query3r<<<QT * 32, 256>>>(z, z, z, z, 0, 0, M, v.meta, rot, q165, nullptr, qn, nsk, q16);
    int tpw;
    k_screen3r<<<screen3r_grid(ntiles, M, tpw), 256>>>(reinterpret_cast<const half8 *>(dbr), ntiles, q16, M, tpw,
                                                        smin);
    const long n = (long)M * ntiles;
    k_screen3_unscale<<<(unsigned)((n + 255) / 256), 256>>>(smin, M, ntiles, qn, v.meta, e, eps, nsk,
                                                            db3r_meta(const_cast<void *>(dbr), nrows));
    IA_LAUNCH_CHECK("ia_diag_screen3r");
    IA_HIP(hipDeviceSynchronize());
    IA_HIP(hipFree(q16));
    IA_HIP(hipFree(smin));
    IA_HIP(hipFree(nsk));
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
