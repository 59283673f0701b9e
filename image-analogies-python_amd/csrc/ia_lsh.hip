// ia_lsh.hip — LSH matcher (config c2 "LSH vs GPU brute force").
//
// The reference snapshot has no LSH code (only the artefact output/freud-crop-filt-lsh.jpg),
// so this is the build's own definition: E2LSH over the same centred rows a' = a - c the
// exact matcher screens.  L tables, each k concatenated hashes
//     h_i(x) = floor((p_i . x + b_i) / w),   p_i ~ N(0, I_55),  b_i ~ U[0, w)
// (projections drawn on the host with a seeded RandomState), combined into a 32-bit key
// per table.  Build: one pass over the fp32 DB computes L keys per row, then one hipCUB
// radix sort of (key, row) pairs per table.  Query (one wave per query): L keys, a binary
// search per table, and the exact fp64 distance (the oracle's pairwise-8 value) of up to
// LSH_CAP rows per bucket; the lexicographic (distance, row) minimum is returned.
// Approximate by construction: the exact matcher is the default.
#include "ia_internal.h"

#include <hipcub/hipcub.hpp>

namespace ia {

constexpr int LSH_MAXH = 64;     // L * k hashes per row (one lane each in the query)
constexpr int LSH_CAP = 32;      // rows examined per (query, table) bucket

__device__ __forceinline__ unsigned int lsh_mix(int h, int i) {
    return (unsigned int)h * (0x9E3779B1u + 2u * (unsigned int)i) + 0x7F4A7C15u * (unsigned int)i;
}

// keys_in[t][r] for rows r of the fragment-major DB (centred values, element 55 skipped)
__global__ __launch_bounds__(256) void k_lsh_keys(const float *__restrict__ db, long nrows,
                                                  long npad, const float *__restrict__ proj,
                                                  int L, int k, float w,
                                                  unsigned int *__restrict__ keys,
                                                  int *__restrict__ rows) {
    __shared__ float P[LSH_MAXH * IA_DP];
    for (int i = threadIdx.x; i < L * k * IA_DP; i += 256) P[i] = proj[i];
    __syncthreads();
    const long r = (long)blockIdx.x * 256 + threadIdx.x;
    if (r >= npad) return;
    float a[IA_DP];
    const float4 *t4 = reinterpret_cast<const float4 *>(db) + (r >> 5) * (32 * IA_DP / 4) + (r & 31);
#pragma unroll
    for (int hh = 0; hh < 2; ++hh)
#pragma unroll
        for (int v = 0; v < 7; ++v) {
            const float4 x = t4[v * 64 + hh * 32];
            a[2 * (4 * v + 0) + hh] = x.x;
            a[2 * (4 * v + 1) + hh] = x.y;
            a[2 * (4 * v + 2) + hh] = x.z;
            a[2 * (4 * v + 3) + hh] = x.w;
        }
    for (int t = 0; t < L; ++t) {
        unsigned int key = 0;
        for (int i = 0; i < k; ++i) {
            const float *p = P + (t * k + i) * IA_DP;
            float d = p[55];
#pragma unroll
            for (int e = 0; e < IA_D; ++e) d = fmaf(p[e], a[e], d);
            key += lsh_mix((int)floorf(d / w), i);
        }
        // rows past nrows (sentinels) get a key no query can produce
        keys[(long)t * npad + r] = r < nrows ? (key & 0x7fffffffu) : 0xffffffffu;
        rows[(long)t * npad + r] = (int)r;
    }
}

__device__ __forceinline__ long lower_bound_u32(const unsigned int *a, long n, unsigned int x) {
    long lo = 0, hi = n;
    while (lo < hi) {
        const long mid = (lo + hi) >> 1;
        if (a[mid] < x) lo = mid + 1; else hi = mid;
    }
    return lo;
}

__device__ __forceinline__ void lbest(double &bd, long long &bi, double d, long long i) {
    if (d < bd || (d == bd && i < bi)) { bd = d; bi = i; }
}

// one 64-lane wave per query
__global__ __launch_bounds__(64) void k_lsh_query(DbSrc src, long row0, long nrows, long npad,
                                                  const unsigned int *__restrict__ keys,
                                                  const int *__restrict__ rows,
                                                  const float *__restrict__ proj, int L, int k,
                                                  float w, const double *__restrict__ q64,
                                                  const double *__restrict__ center,
                                                  Best *__restrict__ best,
                                                  unsigned long long *stats) {
    __shared__ double qs[IA_DP];
    __shared__ float qc[IA_DP];
    __shared__ unsigned int hk[LSH_MAXH];
    __shared__ long lo_s[LSH_MAXH], hi_s[LSH_MAXH];
    const int q = blockIdx.x, lane = threadIdx.x;
    if (lane < IA_DP) {
        qs[lane] = q64[(long)q * IA_DP + lane];
        qc[lane] = lane < IA_D ? (float)(qs[lane] - center[lane]) : 0.f;
    }
    __syncthreads();
    if (lane < L * k) {
        const float *p = proj + lane * IA_DP;
        float d = p[55];
        for (int e = 0; e < IA_D; ++e) d = fmaf(p[e], qc[e], d);
        hk[lane] = lsh_mix((int)floorf(d / w), lane % k);
    }
    __syncthreads();
    if (lane < L) {
        unsigned int key = 0;
        for (int i = 0; i < k; ++i) key += hk[lane * k + i];
        key &= 0x7fffffffu;
        const unsigned int *kt = keys + (long)lane * npad;
        long lo = lower_bound_u32(kt, npad, key);
        long hi = lower_bound_u32(kt, npad, key + 1);
        if (lo == hi) {   // empty bucket: take the neighbouring entries of the sorted table
            lo = lo >= 2 ? lo - 2 : 0;
            hi = lo + 4 < nrows ? lo + 4 : nrows;
        }
        lo_s[lane] = lo;
        hi_s[lane] = hi - lo > LSH_CAP ? lo + LSH_CAP : hi;
    }
    __syncthreads();
    double bd = INFINITY;
    long long bi = 0x7fffffffffffffffLL;
    int ncand = 0;
    for (int t = 0; t < L; ++t) {
        const long lo = lo_s[t], n = hi_s[t] - lo_s[t];
        for (long c = lane; c < n; c += 64) {
            const int lr = rows[(long)t * npad + lo + c];
            if (lr < nrows) {
                lbest(bd, bi, row_dist2(src, row0 + lr, qs), row0 + lr);
                ++ncand;
            }
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        const double od = __shfl_xor(bd, o);
        const long long oi = __shfl_xor(bi, o);
        lbest(bd, bi, od, oi);
        ncand += __shfl_xor(ncand, o);
    }
    if (lane == 0) {
        best[q] = Best{bd, bi == 0x7fffffffffffffffLL ? row0 : bi};
        if (stats) atomicAdd(&stats[0], (unsigned long long)ncand);
    }
}

int launch_lsh_match(const IaLsh *lsh, const DbSrc &src, long row0, long nrows, int M,
                     const double *q64, const double *center, Best *best,
                     unsigned long long *stats, hipStream_t st) {
    const long npad = db_rows_padded(nrows);
    const char *m = reinterpret_cast<const char *>(lsh->mem);
    const unsigned int *keys = reinterpret_cast<const unsigned int *>(m);
    const int *rows = reinterpret_cast<const int *>(m + align_up((size_t)lsh->L * npad * 4, 256));
    k_lsh_query<<<M, 64, 0, st>>>(src, row0, nrows, npad, keys, rows, lsh->proj, lsh->L, lsh->k,
                                  lsh->w, q64, center, best, stats);
    IA_LAUNCH_CHECK("k_lsh_query");
    return IA_OK;
}

static size_t sort_temp_bytes(long npad) {
    size_t tb = 0;
    if (hipcub::DeviceRadixSort::SortPairs(nullptr, tb, (unsigned int *)nullptr,
                                           (unsigned int *)nullptr, (int *)nullptr,
                                           (int *)nullptr, (int)npad) != hipSuccess)
        return 0;
    return tb;
}

}  // namespace ia

using namespace ia;

extern "C" {

size_t ia_lsh_bytes(long nrows, int L) {
    if (nrows <= 0 || L <= 0) return 0;
    const long npad = db_rows_padded(nrows);
    const size_t tab = align_up((size_t)L * npad * 4, 256);
    return 4 * tab + align_up(sort_temp_bytes(npad), 256);
}

int ia_lsh_build(const float *db, long nrows, const IaLsh *lsh, void *stream) {
    IA_ARG(db && lsh && lsh->mem && lsh->proj && nrows > 0, "ia_lsh_build: bad args");
    IA_ARG(lsh->L >= 1 && lsh->k >= 1 && lsh->L * lsh->k <= LSH_MAXH && lsh->w > 0.f,
           "ia_lsh_build: need 1 <= L*k <= 64 and w > 0");
    IA_ARG(nrows < (1L << 31), "ia_lsh_build: too many rows");
    hipStream_t st = S(stream);
    const long npad = db_rows_padded(nrows);
    char *m = reinterpret_cast<char *>(lsh->mem);
    const size_t tab = align_up((size_t)lsh->L * npad * 4, 256);
    unsigned int *keys = reinterpret_cast<unsigned int *>(m);
    int *rows = reinterpret_cast<int *>(m + tab);
    unsigned int *keys_in = reinterpret_cast<unsigned int *>(m + 2 * tab);
    int *rows_in = reinterpret_cast<int *>(m + 3 * tab);
    void *tmp = m + 4 * tab;
    size_t tb = sort_temp_bytes(npad);
    IA_ARG(tb > 0, "ia_lsh_build: radix-sort size query failed");
    k_lsh_keys<<<(unsigned)((npad + 255) / 256), 256, 0, st>>>(db, nrows, npad, lsh->proj, lsh->L,
                                                             lsh->k, lsh->w, keys_in, rows_in);
    IA_LAUNCH_CHECK("k_lsh_keys");
    for (int t = 0; t < lsh->L; ++t) {
        IA_HIP(hipcub::DeviceRadixSort::SortPairs(tmp, tb, keys_in + (long)t * npad,
                                                  keys + (long)t * npad, rows_in + (long)t * npad,
                                                  rows + (long)t * npad, (int)npad, 0, 32, st));
    }
    return IA_OK;
}

}  // extern "C"
