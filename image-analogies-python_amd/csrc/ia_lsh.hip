// ia_lsh.hip — LSH matcher (config c2 "LSH vs GPU brute force").
//
// The reference snapshot has no LSH code (only the artefact output/freud-crop-filt-lsh.jpg),
// so this is the build's own definition: E2LSH over the same centred rows a' = a - c the
// exact matcher screens.  L tables, each k concatenated hashes
//     h_i(x) = floor((p_i . x + b_i) / w),   p_i ~ N(0, I_55),  b_i ~ U[0, w)
// (projections drawn on the host with a seeded RandomState), combined into a 32-bit key
// per table and masked to B = lsh_bits(nrows) bits (2^B >= 2 nrows buckets).  Build: one
// pass over the fp32 DB computes L keys per row, one hipCUB radix sort of (key, row)
// pairs per table, and a bucket directory start[t][0..2^B] (counting-sort offsets).
// The rows' centred fp32 values are gathered from the pyramids like the DB build's.
// Query (one wave per query): L keys, two directory loads per table, and the exact fp64
// distance (the oracle's pairwise-8 value) of up to LSH_CAP rows per bucket, spread over
// the wave's lanes; the lexicographic (distance, row) minimum is returned.
// Approximate by construction: the exact matcher is the default.
#include "ia_internal.h"

#include <hipcub/hipcub.hpp>

namespace ia {

constexpr int LSH_MAXH = 64;     // L * k hashes per row (one lane each in the query)
constexpr int LSH_CAP = 32;      // rows examined per (query, table) bucket

// key bits: ceil(log2(nrows)) + 1, in [2, 30]
static inline int lsh_bits(long nrows) {
    int b = 1;
    while (b < 29 && (1L << b) < nrows) ++b;
    return b + 1;
}

__device__ __forceinline__ unsigned int lsh_mix(int h, int i) {
    return (unsigned int)h * (0x9E3779B1u + 2u * (unsigned int)i) + 0x7F4A7C15u * (unsigned int)i;
}

// keys_in[t][r] for the local rows r of [row0, row0 + nrows): the centred fp32 values
// fl32(a_k - c_k) gathered from the pyramids (the rows the exact matcher screens)
__global__ __launch_bounds__(256) void k_lsh_keys(DbSrc src, long row0, long nrows, long npad,
                                                  const double *__restrict__ center,
                                                  const float *__restrict__ proj,
                                                  int L, int k, float w, int bits,
                                                  unsigned int *__restrict__ keys,
                                                  int *__restrict__ rows) {
    __shared__ float P[LSH_MAXH * IA_DP];
    for (int i = threadIdx.x; i < L * k * IA_DP; i += 256) P[i] = proj[i];
    __syncthreads();
    const long r = (long)blockIdx.x * 256 + threadIdx.x;
    if (r >= npad) return;
    float a[IA_DP];
    {
        ImgPair ap; int rr, cc;
        src.locate(row0 + (r < nrows ? r : nrows - 1), ap, rr, cc);
        emit_feature(src.A, ap, rr, cc, [&](int kk, double v) { a[kk] = (float)(v - center[kk]); });
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
        // rows past nrows (sentinels) get the key 2^bits, beyond every bucket
        const unsigned int mask = (1u << bits) - 1u;
        keys[(long)t * npad + r] = r < nrows ? (key & mask) : mask + 1u;
        rows[(long)t * npad + r] = (int)r;
    }
}

// bucket directory: start[t][b] = first sorted position with key >= b, b in [0, 2^bits]
__global__ __launch_bounds__(256) void k_lsh_dir(const unsigned int *__restrict__ keys, long npad,
                                                 int bits, int *__restrict__ start) {
    const int t = blockIdx.y;
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i >= npad) return;
    const unsigned int *kt = keys + (long)t * npad;
    int *st = start + (long)t * ((1L << bits) + 1);
    const long kp = i > 0 ? (long)kt[i - 1] : -1;
    const long kc = kt[i];
    for (long b = kp + 1; b <= kc; ++b) st[b] = (int)i;
    if (i == npad - 1)   // sentinels hold key 2^bits: nothing beyond
        for (long b = kc + 1; b <= (1L << bits); ++b) st[b] = (int)npad;
}

__device__ __forceinline__ void lbest(double &bd, long long &bi, double d, long long i) {
    if (d < bd || (d == bd && i < bi)) { bd = d; bi = i; }
}

// one 64-lane wave per query
__global__ __launch_bounds__(64) void k_lsh_query(DbSrc src, long row0, long nrows, long npad,
                                                  const int *__restrict__ start, int bits,
                                                  const int *__restrict__ rows,
                                                  const float *__restrict__ proj, int L, int k,
                                                  float w, const double *__restrict__ q64,
                                                  const double *__restrict__ center,
                                                  Best *__restrict__ best,
                                                  unsigned long long *stats) {
    __shared__ double qs[IA_DP];
    __shared__ float qc[IA_DP];
    __shared__ unsigned int hk[LSH_MAXH];
    __shared__ int lo_s[LSH_MAXH + 1], n_s[LSH_MAXH + 1];
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
        key &= (1u << bits) - 1u;
        const int *st = start + (long)lane * ((1L << bits) + 1);
        long lo = st[key], hi = st[key + 1];
        if (lo == hi) {   // empty bucket: take the neighbouring entries of the sorted table
            lo = lo >= 2 ? lo - 2 : 0;
            hi = lo + 4 < nrows ? lo + 4 : nrows;
        }
        lo_s[lane] = (int)lo;
        n_s[lane] = (int)(hi - lo > LSH_CAP ? LSH_CAP : hi - lo);
    }
    __syncthreads();
    if (lane == 0) {   // exclusive prefix of the per-table counts in n_s (in place)
        int acc = 0;
        for (int t = 0; t < L; ++t) { const int c = n_s[t]; n_s[t] = acc; acc += c; }
        n_s[L] = acc;
    }
    __syncthreads();
    const int total = n_s[L];
    double bd = INFINITY;
    long long bi = 0x7fffffffffffffffLL;
    int ncand = 0;
    int t = 0;
    for (int c = lane; c < total; c += 64) {   // candidates of all tables over the lanes
        while (n_s[t + 1] <= c) ++t;
        const int lr = rows[(long)t * npad + lo_s[t] + (c - n_s[t])];
        if (lr < nrows) {
            lbest(bd, bi, row_dist2(src, row0 + lr, qs), row0 + lr);
            ++ncand;
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
        if (stats) atomicAdd(&stats_slot(stats, q)[0], (unsigned long long)ncand);
    }
}

// device layout of IaLsh::mem: rows[L][npad] | start[L][2^bits + 1] | keys[L][npad] |
// keys_in[L][npad] | rows_in[L][npad] | sort temp (the last four only used by the build)
struct LshLayout {
    size_t rows, start, keys, keys_in, rows_in, tmp, total;
};
static size_t sort_temp_bytes(long npad, int bits);
static LshLayout lsh_layout(long nrows, int L) {
    const long npad = db_rows_padded(nrows);
    const int bits = lsh_bits(nrows);
    const size_t tab = align_up((size_t)L * npad * 4, 256);
    LshLayout y;
    y.rows = 0;
    y.start = tab;
    y.keys = y.start + align_up((size_t)L * ((1L << bits) + 1) * 4, 256);
    y.keys_in = y.keys + tab;
    y.rows_in = y.keys_in + tab;
    y.tmp = y.rows_in + tab;
    y.total = y.tmp + align_up(sort_temp_bytes(npad, bits), 256);
    return y;
}

int launch_lsh_match(const IaLsh *lsh, const DbSrc &src, long row0, long nrows, int M,
                     const double *q64, const double *center, Best *best,
                     unsigned long long *stats, hipStream_t st) {
    const long npad = db_rows_padded(nrows);
    const LshLayout y = lsh_layout(nrows, lsh->L);
    const char *m = reinterpret_cast<const char *>(lsh->mem);
    k_lsh_query<<<M, 64, 0, st>>>(src, row0, nrows, npad,
                                  reinterpret_cast<const int *>(m + y.start), lsh_bits(nrows),
                                  reinterpret_cast<const int *>(m + y.rows), lsh->proj, lsh->L,
                                  lsh->k, lsh->w, q64, center, best, stats);
    IA_LAUNCH_CHECK("k_lsh_query");
    return IA_OK;
}

static size_t sort_temp_bytes(long npad, int bits) {
    size_t tb = 0;
    if (hipcub::DeviceRadixSort::SortPairs(nullptr, tb, (unsigned int *)nullptr,
                                           (unsigned int *)nullptr, (int *)nullptr,
                                           (int *)nullptr, (int)npad, 0, bits + 1) != hipSuccess)
        return 0;
    return tb;
}

}  // namespace ia

using namespace ia;

extern "C" {

size_t ia_lsh_bytes(long nrows, int L) {
    if (nrows <= 0 || L <= 0) return 0;
    return lsh_layout(nrows, L).total;
}

int ia_lsh_bits(long nrows) { return nrows > 0 ? lsh_bits(nrows) : 0; }

int ia_lsh_build(const IaSrcLevel *src, long row0, long nrows, const double *center,
                 const IaLsh *lsh, void *stream) {
    IA_ARG(src && center && lsh && lsh->mem && lsh->proj && nrows > 0 && row0 >= 0,
           "ia_lsh_build: bad args");
    IA_ARG(lsh->L >= 1 && lsh->k >= 1 && lsh->L * lsh->k <= LSH_MAXH && lsh->w > 0.f,
           "ia_lsh_build: need 1 <= L*k <= 64 and w > 0");
    IA_ARG(nrows < (1L << 31), "ia_lsh_build: too many rows");
    hipStream_t st = S(stream);
    const long npad = db_rows_padded(nrows);
    const int bits = lsh_bits(nrows);
    const LshLayout y = lsh_layout(nrows, lsh->L);
    char *m = reinterpret_cast<char *>(lsh->mem);
    int *rows = reinterpret_cast<int *>(m + y.rows);
    int *start = reinterpret_cast<int *>(m + y.start);
    unsigned int *keys = reinterpret_cast<unsigned int *>(m + y.keys);
    unsigned int *keys_in = reinterpret_cast<unsigned int *>(m + y.keys_in);
    int *rows_in = reinterpret_cast<int *>(m + y.rows_in);
    void *tmp = m + y.tmp;
    size_t tb = sort_temp_bytes(npad, bits);
    IA_ARG(tb > 0, "ia_lsh_build: radix-sort size query failed");
    const unsigned nb = (unsigned)((npad + 255) / 256);
    k_lsh_keys<<<nb, 256, 0, st>>>(make_dbsrc(*src), row0, nrows, npad, center, lsh->proj,
                                   lsh->L, lsh->k, lsh->w, bits, keys_in, rows_in);
    IA_LAUNCH_CHECK("k_lsh_keys");
    for (int t = 0; t < lsh->L; ++t) {
        IA_HIP(hipcub::DeviceRadixSort::SortPairs(tmp, tb, keys_in + (long)t * npad,
                                                  keys + (long)t * npad, rows_in + (long)t * npad,
                                                  rows + (long)t * npad, (int)npad, 0, bits + 1,
                                                  st));
    }
    k_lsh_dir<<<dim3(nb, lsh->L), 256, 0, st>>>(keys, npad, bits, start);
    IA_LAUNCH_CHECK("k_lsh_dir");
    return IA_OK;
}

}  // extern "C"
