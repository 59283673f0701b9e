// ia_features.hip — neighbourhood feature construction.
//   * compute_feature_array (algorithms.py:11-47) for the API,
//   * the screening database (algorithms.py:50-70 As[level]): centred rows with the
//     squared norm folded in as element 55, split into f16 pairs in the MFMA operand
//     order (ia_split16.h), 224 B per row,
//   * per-wave query rows (image_analogies.py:166-168: B full | B' half): fp64 for the
//     exact rescore, fp32 for the re-screen, split-f16 for the screen.
// Feature values are pure gathers (exact); centring, rounding and splitting only feed the
// screen and re-screen, whose error bounds are accounted for in ia_match.hip.
#include "ia_common.h"
#include "ia_internal.h"
#include "ia_split16.h"

namespace ia {

__global__ void k_level_features(ImgPair p, int full, double *out) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (long)p.h * p.w) return;
    const int r = (int)(i / p.w), c = (int)(i - (long)r * p.w);
    if (full) {
        double *o = out + i * 34;
        emit_pixel<true>(p, r, c, 0, [&](int k, double v) { o[k] = v; });
    } else {
        double *o = out + i * 21;
        emit_pixel<false>(p, r, c, 0, [&](int k, double v) { o[k] = v; });
    }
}

// MFMA operand order of element k = 2s + h: position h*28 + s (the fp32 query rows qp).
__device__ __forceinline__ int perm56(int k) { return (k & 1) * 28 + (k >> 1); }

// Centred row of DB row ix: my[k] = fl32(a_k - c_k) (k < 55), my[55] = fl32(|a - c|^2)
// (fp64 sum in feature order); returns |a - c| in fp32.
__device__ __forceinline__ float db_row(const DbSrc &src, long ix, const double *__restrict__ center,
                                        float *my) {
    ImgPair ap; int r, c;
    src.locate(ix, ap, r, c);
    double n2 = 0.0;
    emit_feature(src.A, ap, r, c, [&](int k, double v) {
        const double d = v - center[k];
        n2 += d * d;
        my[k] = (float)d;
    });
    my[55] = (float)n2;
    return (float)sqrt(n2);
}

// Pass 1: amax = max over rows of |a - c| (the split scale and the error bounds need it
// before any row is split).  One thread per row, a block max, one atomic per block.
__global__ __launch_bounds__(256) void k_db_norms(DbSrc src, long row0, long nrows,
                                                  const double *__restrict__ center, float *amax) {
    __shared__ float redmax[4];
    const long lr = (long)blockIdx.x * 256 + threadIdx.x;
    float nrm = 0.f;
    if (lr < nrows) {
        float my[IA_DP];
        nrm = db_row(src, row0 + lr, center, my);
    }
    for (int o = 32; o > 0; o >>= 1) nrm = fmaxf(nrm, __shfl_xor(nrm, o));
    if ((threadIdx.x & 63) == 0) redmax[threadIdx.x >> 6] = nrm;
    __syncthreads();
    if (threadIdx.x == 0) {
        const float m = fmaxf(fmaxf(redmax[0], redmax[1]), fmaxf(redmax[2], redmax[3]));
        atomicMax(reinterpret_cast<unsigned int *>(amax), __float_as_uint(m));
    }
}

// Pass 2: the split-f16 rows (ia_split16.h), written once.  One thread per row computes
// its 56 centred fp32 values into LDS (256 rows = 8 tiles per block); then lane (j, h) of
// each wave emits its 7 register groups of two tiles: half8 (tile, g, lane) at
// (tile * 7 + g) * 64 + lane, so each of the screen's 7 loads per tile is one contiguous
// 1 KiB wave access.  Padding rows (>= nrows) repeat row nrows - 1: their screen values
// are those of a real row, so the segment minima need no masking (the exact stage never
// rescores a row >= nrows).
__global__ __launch_bounds__(256) void k_db_build(DbSrc src, long row0, long nrows, long npad,
                                                  const double *__restrict__ center,
                                                  const float *__restrict__ amax,
                                                  half8 *__restrict__ db16) {
    constexpr int LD = IA_DP + 1;
    __shared__ float tile[256 * LD];
    const long base = (long)blockIdx.x * 256;
    const long lr = base + threadIdx.x;
    if (lr < npad) {
        float my[IA_DP];
        db_row(src, row0 + (lr < nrows ? lr : nrows - 1), center, my);
#pragma unroll
        for (int k = 0; k < IA_DP; ++k) tile[threadIdx.x * LD + k] = my[k];
    }
    __syncthreads();
    const Split16Db s = split16_db_scale(amax[0]);
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int j = lane & 31, h = lane >> 5;
    for (int tt = wv; tt < 8; tt += 4) {
        const long T = (base >> 5) + tt;
        if (T * 32 >= npad) break;
        const float *tr = tile + (tt * 32 + j) * LD;
        half8 *out = db16 + T * (DB16_GROUPS * 64) + lane;
#pragma unroll
        for (int g = 0; g < DB16_GROUPS; ++g) {
            int k0;
            bool hi;
            split16_db_group(h, g, k0, hi);
            half8 o;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const int k = k0 + e;
                const float v = k < 55 ? ldexpf(tr[k], s.ea) : ldexpf(tr[55], s.ea - s.R);
                _Float16 xh, xl;
                split16f(v, xh, xl);
                o[e] = hi ? xh : xl;
            }
            out[g * 64] = o;
        }
    }
}

__global__ void k_center_fill(double *c, double mA, double mAp) {
    const int k = threadIdx.x;
    if (k < IA_D) c[k] = k < 34 ? mA : mAp;
}

// Query rows for the pixels of wave t (y = y_lo + m, x = t - 3y):
// q64[m][k] (fp64 feature), qp[m][perm56(k)] = fp32(-2 (q_k - c_k)), qp[..55] = 1,
// nq[m] = |q - c|^2.  One 64-lane wave per query, lane = feature index.
__global__ __launch_bounds__(64) void k_query_wave(ImgPair B, ImgPair Bp, int t, int y_lo,
                                                   const double *__restrict__ center,
                                                   double *__restrict__ q64,
                                                   float *__restrict__ qp,
                                                   double *__restrict__ nq,
                                                   const float *__restrict__ amax,
                                                   _Float16 *__restrict__ q16) {
    const int m = blockIdx.x;
    const int y = y_lo + m, x = t - 3 * y;
    const int lane = threadIdx.x;
    double v = 0.0;
    // lane-parallel gather: each lane picks its own element of the 55
    if (lane < 34) {
        const bool coarse = lane < 9;
        const int tt = coarse ? lane : lane - 9;
        v = coarse ? B.sm[(long)symi2((y >> 1) + tt / 3 - 1, B.hs) * B.ws + symi2((x >> 1) + tt % 3 - 1, B.ws)]
                   : B.lg[(long)symi2(y + tt / 5 - 2, B.h) * B.w + symi2(x + tt % 5 - 2, B.w)];
    } else if (lane < 55) {
        const bool coarse = lane < 43;
        const int tt = coarse ? lane - 34 : lane - 43;
        v = coarse ? Bp.sm[(long)symi2((y >> 1) + tt / 3 - 1, Bp.hs) * Bp.ws + symi2((x >> 1) + tt % 3 - 1, Bp.ws)]
                   : Bp.lg[(long)symi2(y + tt / 5 - 2, Bp.h) * Bp.w + symi2(x + tt % 5 - 2, Bp.w)];
    }
    double d = 0.0;
    if (lane < 55) {
        q64[(long)m * IA_DP + lane] = v;
        d = v - center[lane];
        qp[(long)m * IA_DP + perm56(lane)] = -2.0f * (float)d;
    } else if (lane == 55) {
        q64[(long)m * IA_DP + 55] = 0.0;
        qp[(long)m * IA_DP + perm56(55)] = 1.0f;
    }
    double d2 = d * d;
    for (int o = 32; o > 0; o >>= 1) d2 += __shfl_xor(d2, o);   // same sum in every lane
    if (lane == 0) nq[m] = d2;
    if (q16) split16_write_query(q16 + (long)m * Q16_ROW * 8, lane, d, d2, amax[0]);
}

// Query rows from caller-provided fp64 features (ia_match_batch).
__global__ __launch_bounds__(64) void k_query_rows(const double *__restrict__ qin, int M,
                                                   const double *__restrict__ center,
                                                   float *__restrict__ qp,
                                                   double *__restrict__ nq,
                                                   const float *__restrict__ amax,
                                                   _Float16 *__restrict__ q16) {
    const int m = blockIdx.x;
    const int lane = threadIdx.x;
    double d = 0.0;
    if (lane < 55) {
        d = qin[(long)m * IA_DP + lane] - center[lane];
        qp[(long)m * IA_DP + perm56(lane)] = -2.0f * (float)d;
    } else if (lane == 55) {
        qp[(long)m * IA_DP + perm56(55)] = 1.0f;
    }
    double d2 = d * d;
    for (int o = 32; o > 0; o >>= 1) d2 += __shfl_xor(d2, o);   // same sum in every lane
    if (lane == 0) nq[m] = d2;
    if (q16) split16_write_query(q16 + (long)m * Q16_ROW * 8, lane, d, d2, amax[0]);
}

int launch_query_wave(const ImgPair &B, const ImgPair &Bp, int t, int y_lo, int M,
                      const double *center, double *q64, float *qp, double *nq,
                      const float *amax, _Float16 *q16, hipStream_t st) {
    k_query_wave<<<M, 64, 0, st>>>(B, Bp, t, y_lo, center, q64, qp, nq, amax, q16);
    IA_LAUNCH_CHECK("k_query_wave");
    return IA_OK;
}

int launch_query_rows(const double *qin, int M, const double *center, float *qp, double *nq,
                      const float *amax, _Float16 *q16, hipStream_t st) {
    k_query_rows<<<M, 64, 0, st>>>(qin, M, center, qp, nq, amax, q16);
    IA_LAUNCH_CHECK("k_query_rows");
    return IA_OK;
}

}  // namespace ia

using namespace ia;

extern "C" {

int ia_level_features_f64(const double *sm, int hs, int ws, const double *lg, int h, int w,
                          int full, double *out, void *stream) {
    IA_ARG(sm && lg && out && hs > 0 && ws > 0 && h > 0 && w > 0, "ia_level_features_f64: bad args");
    ImgPair p{sm, lg, hs, ws, h, w};
    long n = (long)h * w;
    k_level_features<<<(unsigned)((n + 255) / 256), 256, 0, S(stream)>>>(p, full, out);
    IA_LAUNCH_CHECK("k_level_features");
    return IA_OK;
}

int ia_db_chunk_rows(long nrows) { return db_chunk_rows(nrows); }
long ia_db_rows_padded(long nrows) { return db_rows_padded(nrows); }
size_t ia_db_bytes(long nrows) { return db_bytes(nrows); }

int ia_db_build(const IaSrcLevel *src, long row0, long nrows, const double *center,
                void *db, float *amax, void *stream) {
    IA_ARG(src && center && db && amax && nrows > 0 && row0 >= 0, "ia_db_build: bad args");
    IA_ARG(row0 + nrows <= (long)src->nAp * src->Ah * src->Aw, "ia_db_build: rows out of range");
    const long npad = db_rows_padded(nrows);
    DbSrc d = make_dbsrc(*src);
    k_db_norms<<<(unsigned)((nrows + 255) / 256), 256, 0, S(stream)>>>(d, row0, nrows, center, amax);
    IA_LAUNCH_CHECK("k_db_norms");
    k_db_build<<<(unsigned)((npad + 255) / 256), 256, 0, S(stream)>>>(d, row0, nrows, npad, center,
                                                                     amax, reinterpret_cast<half8 *>(db));
    IA_LAUNCH_CHECK("k_db_build");
    return IA_OK;
}

int ia_center_fill(double *center, double mA, double mAp, void *stream) {
    IA_ARG(center, "ia_center_fill: bad args");
    k_center_fill<<<1, 64, 0, S(stream)>>>(center, mA, mAp);
    IA_LAUNCH_CHECK("k_center_fill");
    return IA_OK;
}

}  // extern "C"
