// ia_match.hip — the brute-force matcher (the hot kernel).
//
// best_approximate_match (algorithms.py:73-75, FLANN kd-tree in the reference) becomes
// an EXACT 1-NN over the level database As[level] in two stages:
//
//  1. k_screen (MFMA-bound): e(q, a) = |a'|^2 - 2 a'.q' with a' = a - c, q' = q - c
//     (c = screening centre), computed as ONE fp32 contraction of length 56 on
//     v_mfma_f32_32x32x2_f32: DB row = [a'_0..a'_54, |a'|^2], query = [-2q'_0..-2q'_54, 1].
//     Queries are the stationary operand (kept in VGPRs for the whole chunk), DB rows
//     stream through in 32-row tiles.  Accumulator lane = query, registers = 16 DB rows,
//     so each lane keeps its own top-K (K=4) of (e, row) over the rows it sees; the
//     block merges 8 such lists per query through LDS and writes SCREEN_K candidates per
//     (query, chunk).
//  2. k_merge (latency-bound, one workgroup per query): e + |q'|^2 approximates the true
//     distance D within eps_q = 70 u32 (2 Amax |q'| + Amax^2) (fp32 conversion of both
//     operands + a 56-term fma chain, worst case; Amax = max row |a'|).  Every row whose
//     D could be the minimum therefore has e <= e_min + 2 eps_q; all such rows are
//     re-scored in fp64 with the oracle's exact pairwise-8 sum, gathering the row's 55
//     features straight from the fp64 pyramids.  A chunk whose K-th candidate is itself
//     inside the window may have dropped candidates: it is re-scanned exactly.  Ties
//     break to the lowest row index (np.argmin).  The result is bit-identical to the
//     oracle's brute force for any input.
#include "ia_finish.h"
#include "ia_split16.h"

#include <float.h>

namespace ia {

typedef float floatx16 __attribute__((ext_vector_type(16)));

// K = 4 sorted insert of (v, idx), v < t[3] known (branch-free).
__device__ __forceinline__ void topk_insert(float (&t)[SCREEN_K], int (&ti)[SCREEN_K], float v,
                                            int idx) {
    const bool c0 = v < t[0], c1 = v < t[1], c2 = v < t[2];
    const float n3 = c2 ? t[2] : v;
    const int i3 = c2 ? ti[2] : idx;
    const float n2 = c1 ? t[1] : (c2 ? v : t[2]);
    const int i2 = c1 ? ti[1] : (c2 ? idx : ti[2]);
    const float n1 = c0 ? t[0] : (c1 ? v : t[1]);
    const int i1 = c0 ? ti[0] : (c1 ? idx : ti[1]);
    t[0] = c0 ? v : t[0];
    ti[0] = c0 ? idx : ti[0];
    t[1] = n1; ti[1] = i1;
    t[2] = n2; ti[2] = i2;
    t[3] = n3; ti[3] = i3;
}

constexpr int TILE_VEC = 32 * IA_DP / 4;   // float4s per 32-row DB tile

// One 32-row DB tile against NQ query tiles: 28*NQ MFMAs, then the per-lane top-K
// epilogue.  C[row i][col j] lands at lane (j, h), register r, i = (r&3) + 8(r>>2) + 4h.
// B operands come from registers (bval) or, with FROM_LDS, from ds_read_b128 of the
// staged query image (4 k-steps per read).
template <int NQ, bool FROM_LDS, typename BV>
__device__ __forceinline__ void screen_tile(const float4 (&a4)[7], BV &bval,
                                            const float4 *qsh, int lane,
                                            float (&te)[NQ][SCREEN_K], int (&ti)[NQ][SCREEN_K],
                                            int rbase) {
    floatx16 acc[NQ];
#pragma unroll
    for (int qt = 0; qt < NQ; ++qt)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[qt][r] = 0.f;
#pragma unroll
    for (int v = 0; v < 7; ++v) {
        const float av[4] = {a4[v].x, a4[v].y, a4[v].z, a4[v].w};
        float4 bl[NQ];
        if constexpr (FROM_LDS) {
#pragma unroll
            for (int qt = 0; qt < NQ; ++qt) bl[qt] = qsh[(qt * 7 + v) * 64 + lane];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int qt = 0; qt < NQ; ++qt) {
                float bv;
                if constexpr (FROM_LDS)
                    bv = u == 0 ? bl[qt].x : u == 1 ? bl[qt].y : u == 2 ? bl[qt].z : bl[qt].w;
                else
                    bv = bval(qt, v, u);
                acc[qt] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[u], bv, acc[qt], 0, 0, 0);
            }
    }
#pragma unroll
    for (int qt = 0; qt < NQ; ++qt) {
        float mn = acc[qt][0];
#pragma unroll
        for (int r = 1; r < 16; ++r) mn = fminf(mn, acc[qt][r]);
        if (mn < te[qt][SCREEN_K - 1]) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float x = acc[qt][r];
                if (x < te[qt][SCREEN_K - 1])
                    topk_insert(te[qt], ti[qt], x, rbase + (r & 3) + 8 * (r >> 2));
            }
        }
    }
}

// DB tiles are fragment-major (ia_features.hip k_db_build): float4 (tile, v, lane) holds
// lane (j, h)'s k-steps 4v..4v+3 of row tile*32 + j, so each of the 7 loads of a tile
// is one contiguous 1 KiB wave access.  p = tile base + lane.
__device__ __forceinline__ void load_tile(float4 (&a)[7], const float4 *p) {
#pragma unroll
    for (int v = 0; v < 7; ++v) a[v] = p[v * 64];
}

// first float4 of this lane in the tile containing DB row `row` (a multiple of 32)
__device__ __forceinline__ const float4 *tile_ptr(const float *db, long row, int lane) {
    return reinterpret_cast<const float4 *>(db) + (row >> 5) * TILE_VEC + lane;
}

// A wave's stream over its ntile DB tiles with an explicit two-buffer ping-pong (the
// loads of tile t+1 are in flight while tile t's 28*NQ MFMAs run; no register copies,
// so the compiler's counted vmcnt waits only for the tile being consumed).
template <int NQ, bool FROM_LDS, typename BV>
__device__ __forceinline__ void stream_tiles(const float4 *dp, int ntile, long stride, int rbase0, BV &bval,
                                             const float4 *qsh, int lane,
                                             float (&te)[NQ][SCREEN_K],
                                             int (&ti)[NQ][SCREEN_K]) {
    float4 b0[7], b1[7];
    load_tile(b0, dp);
    int tile = 0;
    for (; tile + 1 < ntile; tile += 2) {
        load_tile(b1, dp + (long)(tile + 1) * stride);
        screen_tile<NQ, FROM_LDS>(b0, bval, qsh, lane, te, ti, rbase0 + tile * 32);
        // unconditional (clamped) reload: a load under a branch makes the compiler's
        // waitcnt at the join conservative and stalls the next tile on it
        const int nxt = tile + 2 < ntile ? tile + 2 : ntile - 1;
        load_tile(b0, dp + (long)nxt * stride);
        screen_tile<NQ, FROM_LDS>(b1, bval, qsh, lane, te, ti, rbase0 + (tile + 1) * 32);
    }
    if (tile < ntile) screen_tile<NQ, FROM_LDS>(b0, bval, qsh, lane, te, ti, rbase0 + tile * 32);
}

// Three-buffer ring: tile t+2's loads are issued while tile t computes (prefetch
// distance two tiles), for when one tile of MFMA work does not cover HBM latency.
template <int NQ, bool FROM_LDS, typename BV>
__device__ __forceinline__ void stream_tiles3(const float4 *dp, int ntile, long stride, int rbase0, BV &bval,
                                              const float4 *qsh, int lane,
                                              float (&te)[NQ][SCREEN_K],
                                              int (&ti)[NQ][SCREEN_K]) {
    float4 b0[7], b1[7], b2[7];
    auto at = [&](int t) { return dp + (long)(t < ntile ? t : ntile - 1) * stride; };
    load_tile(b0, at(0));
    load_tile(b1, at(1));
    int tile = 0;
    for (; tile + 2 < ntile; tile += 3) {
        load_tile(b2, at(tile + 2));
        screen_tile<NQ, FROM_LDS>(b0, bval, qsh, lane, te, ti, rbase0 + tile * 32);
        load_tile(b0, at(tile + 3));
        screen_tile<NQ, FROM_LDS>(b1, bval, qsh, lane, te, ti, rbase0 + (tile + 1) * 32);
        load_tile(b1, at(tile + 4));
        screen_tile<NQ, FROM_LDS>(b2, bval, qsh, lane, te, ti, rbase0 + (tile + 2) * 32);
    }
    if (tile < ntile) screen_tile<NQ, FROM_LDS>(b0, bval, qsh, lane, te, ti, rbase0 + tile * 32);
    if (tile + 1 < ntile)
        screen_tile<NQ, FROM_LDS>(b1, bval, qsh, lane, te, ti, rbase0 + (tile + 1) * 32);
}

// grid: (nchunks rounded up to 8) x groups workgroups, XCD-aware: all query groups of a
// chunk share blockIdx % 8 (one XCD under round-robin dispatch) so the chunk's rows are
// fetched from HBM once and re-read from that XCD's L2.
template <int NQ, int MODE = 0>
__global__ __launch_bounds__(256) void k_screen(const float *__restrict__ db, int nchunks,
                                                int ch, const float *__restrict__ qp, int M,
                                                int groups, Cand *__restrict__ cand) {
    __shared__ float le[NQ * 32][8][SCREEN_K];
    __shared__ int li[NQ * 32][8][SCREEN_K];

    const int b = blockIdx.x;
    const int slot = b >> 3;
    const int chunk = (slot / groups) * 8 + (b & 7);
    const int group = slot - (slot / groups) * groups;
    if (chunk >= nchunks) return;

    const int tid = threadIdx.x;
    const int lane = tid & 63, wv = tid >> 6;
    const int j = lane & 31, h = lane >> 5;

    // stationary query fragments: lane (j, h) holds B[k = 2s + h][col j], s = 0..27
    float bq[NQ][28];
#pragma unroll
    for (int qt = 0; qt < NQ; ++qt) {
        const float4 *p = reinterpret_cast<const float4 *>(
            qp + (long)((group * NQ + qt) * 32 + j) * IA_DP + h * 28);
#pragma unroll
        for (int v = 0; v < 7; ++v) {
            const float4 x = p[v];
            bq[qt][4 * v] = x.x; bq[qt][4 * v + 1] = x.y;
            bq[qt][4 * v + 2] = x.z; bq[qt][4 * v + 3] = x.w;
        }
    }

    float te[NQ][SCREEN_K];
    int ti[NQ][SCREEN_K];
#pragma unroll
    for (int qt = 0; qt < NQ; ++qt)
#pragma unroll
        for (int k = 0; k < SCREEN_K; ++k) { te[qt][k] = FLT_MAX; ti[qt][k] = -1; }

    const int rows_per_wave = ch >> 2;
    const int ntile = rows_per_wave >> 5;
    const long row_begin = (long)chunk * ch + wv * rows_per_wave;
    // lane (j, h) streams DB row (tile*32 + j), elements k = 2s + h
    const float4 *dp = tile_ptr(db, row_begin, lane);
    const int rbase0 = (int)(row_begin - (long)chunk * ch) + 4 * h;
    auto bval = [&](int qt, int v, int u) { return bq[qt][4 * v + u]; };
    if constexpr (MODE == 0) stream_tiles<NQ, false>(dp, ntile, TILE_VEC, rbase0, bval, nullptr, lane, te, ti);
    else if constexpr (MODE == 1) stream_tiles3<NQ, false>(dp, ntile, TILE_VEC, rbase0, bval, nullptr, lane, te, ti);
    else if constexpr (MODE == 2) stream_tiles<NQ, false>(dp, ntile, 0, rbase0, bval, nullptr, lane, te, ti);
    else stream_tiles3<NQ, false>(dp, ntile, 0, rbase0, bval, nullptr, lane, te, ti);

    // merge the 8 per-lane lists of each query (4 waves x 2 row halves) through LDS
#pragma unroll
    for (int qt = 0; qt < NQ; ++qt)
#pragma unroll
        for (int k = 0; k < SCREEN_K; ++k) {
            le[qt * 32 + j][wv * 2 + h][k] = te[qt][k];
            li[qt * 32 + j][wv * 2 + h][k] = ti[qt][k];
        }
    __syncthreads();
    if (tid < NQ * 32) {
        const int qg = group * NQ * 32 + tid;
        if (qg < M) {
            float be[SCREEN_K];
            int bi[SCREEN_K];
#pragma unroll
            for (int k = 0; k < SCREEN_K; ++k) { be[k] = FLT_MAX; bi[k] = -1; }
            for (int l = 0; l < 8; ++l)
#pragma unroll
                for (int k = 0; k < SCREEN_K; ++k) {
                    const float v = le[tid][l][k];
                    if (v < be[SCREEN_K - 1]) topk_insert(be, bi, v, li[tid][l][k]);
                }
            Cand *o = cand + ((long)qg * nchunks + chunk) * SCREEN_K;
            const int cbase = chunk * ch;
#pragma unroll
            for (int k = 0; k < SCREEN_K; ++k) o[k] = Cand{be[k], bi[k] < 0 ? -1 : cbase + bi[k]};
        }
    }
}

// Variant with the query group staged once per block in LDS (shared by the 4 waves)
// instead of 28*NQ VGPRs per wave: B operands come from ds_read_b128 (4 k-steps per
// read), which frees registers for up to 6 query tiles per wave — fewer query groups,
// so each DB chunk is re-read fewer times and each A fragment feeds 28*NQ MFMAs.
template <int NQ>
__global__ __launch_bounds__(256, NQ <= 3 ? 2 : 1) void k_screen_lds(const float *__restrict__ db, int nchunks,
                                                    int ch, const float *__restrict__ qp, int M,
                                                    int groups, Cand *__restrict__ cand) {
    constexpr int QVEC = NQ * 7 * 64;                                  // float4s of queries
    constexpr int LBYTES = NQ * 32 * 8 * SCREEN_K * 8;                 // merge lists
    constexpr int SBYTES = (QVEC * 16 > LBYTES) ? QVEC * 16 : LBYTES;
    __shared__ __attribute__((aligned(16))) char smem[SBYTES];
    float4 *qsh = reinterpret_cast<float4 *>(smem);

    const int b = blockIdx.x;
    const int slot = b >> 3;
    const int chunk = (slot / groups) * 8 + (b & 7);
    const int group = slot - (slot / groups) * groups;
    if (chunk >= nchunks) return;

    const int tid = threadIdx.x;
    const int lane = tid & 63, wv = tid >> 6;
    const int j = lane & 31, h = lane >> 5;

    // stage B fragments: qsh[(qt*7 + v)*64 + lane] = B[k = 2(4v+u) + h][col j], u = 0..3
    for (int i = tid; i < QVEC; i += 256) {
        const int qt = i / 448, rem = i - qt * 448;
        const int v = rem >> 6, l = rem & 63;
        qsh[i] = *reinterpret_cast<const float4 *>(
            qp + (long)((group * NQ + qt) * 32 + (l & 31)) * IA_DP + (l >> 5) * 28 + 4 * v);
    }
    __syncthreads();

    float te[NQ][SCREEN_K];
    int ti[NQ][SCREEN_K];
#pragma unroll
    for (int qt = 0; qt < NQ; ++qt)
#pragma unroll
        for (int k = 0; k < SCREEN_K; ++k) { te[qt][k] = FLT_MAX; ti[qt][k] = -1; }

    const int rows_per_wave = ch >> 2;
    const int ntile = rows_per_wave >> 5;
    const long row_begin = (long)chunk * ch + wv * rows_per_wave;
    const float4 *dp = tile_ptr(db, row_begin, lane);
    const int rbase0 = (int)(row_begin - (long)chunk * ch) + 4 * h;
    auto bval = [](int, int, int) { return 0.f; };
    stream_tiles<NQ, true>(dp, ntile, TILE_VEC, rbase0, bval, qsh, lane, te, ti);

    __syncthreads();   // queries no longer needed: the LDS becomes the merge lists
    float(*le)[8][SCREEN_K] = reinterpret_cast<float(*)[8][SCREEN_K]>(smem);
    int(*li)[8][SCREEN_K] = reinterpret_cast<int(*)[8][SCREEN_K]>(smem + NQ * 32 * 8 * SCREEN_K * 4);
#pragma unroll
    for (int qt = 0; qt < NQ; ++qt)
#pragma unroll
        for (int k = 0; k < SCREEN_K; ++k) {
            le[qt * 32 + j][wv * 2 + h][k] = te[qt][k];
            li[qt * 32 + j][wv * 2 + h][k] = ti[qt][k];
        }
    __syncthreads();
    for (int t = tid; t < NQ * 32; t += 256) {
        const int qg = group * NQ * 32 + t;
        if (qg < M) {
            float be[SCREEN_K];
            int bi[SCREEN_K];
#pragma unroll
            for (int k = 0; k < SCREEN_K; ++k) { be[k] = FLT_MAX; bi[k] = -1; }
            for (int l = 0; l < 8; ++l)
#pragma unroll
                for (int k = 0; k < SCREEN_K; ++k) {
                    const float v = le[t][l][k];
                    if (v < be[SCREEN_K - 1]) topk_insert(be, bi, v, li[t][l][k]);
                }
            Cand *o = cand + ((long)qg * nchunks + chunk) * SCREEN_K;
            const int cbase = chunk * ch;
#pragma unroll
            for (int k = 0; k < SCREEN_K; ++k) o[k] = Cand{be[k], bi[k] < 0 ? -1 : cbase + bi[k]};
        }
    }
}

// ---- variant 2: software-pipelined screen --------------------------------------------
// Queries in LDS (as variant 1) plus two accumulator sets: while the 28*NQ MFMAs of tile
// t+1 run into one set, the wave reduces tile t's set (accvgpr reads + v_min3) in the
// issue gaps between them (sched_group_barrier interleave: 1 MFMA, 1 VALU), so the
// MFMA pipe no longer idles through each tile's epilogue.  The rare top-K insertion
// (some lane's tile minimum beats its K-th best) runs after the interleaved block.
template <int NQ>
__device__ __forceinline__ void mfma_tile_lds(const float4 (&a4)[7], const float4 *qsh, int lane,
                                              floatx16 (&acc)[NQ]) {
#pragma unroll
    for (int qt = 0; qt < NQ; ++qt)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[qt][r] = 0.f;
#pragma unroll
    for (int v = 0; v < 7; ++v) {
        const float av[4] = {a4[v].x, a4[v].y, a4[v].z, a4[v].w};
        float4 bl[NQ];
#pragma unroll
        for (int qt = 0; qt < NQ; ++qt) bl[qt] = qsh[(qt * 7 + v) * 64 + lane];
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int qt = 0; qt < NQ; ++qt) {
                const float bv = u == 0 ? bl[qt].x : u == 1 ? bl[qt].y : u == 2 ? bl[qt].z : bl[qt].w;
                acc[qt] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[u], bv, acc[qt], 0, 0, 0);
            }
    }
}

template <int NQ>
__device__ __forceinline__ void min_tile(const floatx16 (&acc)[NQ], float (&mn)[NQ]) {
#pragma unroll
    for (int qt = 0; qt < NQ; ++qt) {
        float m = fminf(acc[qt][0], acc[qt][1]);
#pragma unroll
        for (int r = 2; r < 16; r += 2) m = fminf(m, fminf(acc[qt][r], acc[qt][r + 1]));
        mn[qt] = m;
    }
}

template <int NQ>
__device__ __forceinline__ void interleave_mark() {
#pragma unroll
    for (int i = 0; i < 28 * NQ; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // 1 MFMA
        __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);   // 1 VALU
    }
}

template <int NQ>
__device__ __forceinline__ void insert_tile(const floatx16 (&acc)[NQ], const float (&mn)[NQ],
                                            float (&te)[NQ][SCREEN_K], int (&ti)[NQ][SCREEN_K],
                                            int rbase) {
#pragma unroll
    for (int qt = 0; qt < NQ; ++qt) {
        if (mn[qt] < te[qt][SCREEN_K - 1]) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float x = acc[qt][r];
                if (x < te[qt][SCREEN_K - 1])
                    topk_insert(te[qt], ti[qt], x, rbase + (r & 3) + 8 * (r >> 2));
            }
        }
    }
}

template <int NQ>
__global__ __launch_bounds__(256, 2) void k_screen_pipe(const float *__restrict__ db, int nchunks,
                                                        int ch, const float *__restrict__ qp,
                                                        int M, int groups,
                                                        Cand *__restrict__ cand) {
    constexpr int QVEC = NQ * 7 * 64;
    constexpr int LBYTES = NQ * 32 * 8 * SCREEN_K * 8;
    constexpr int SBYTES = (QVEC * 16 > LBYTES) ? QVEC * 16 : LBYTES;
    __shared__ __attribute__((aligned(16))) char smem[SBYTES];
    float4 *qsh = reinterpret_cast<float4 *>(smem);

    const int b = blockIdx.x;
    const int slot = b >> 3;
    const int chunk = (slot / groups) * 8 + (b & 7);
    const int group = slot - (slot / groups) * groups;
    if (chunk >= nchunks) return;

    const int tid = threadIdx.x;
    const int lane = tid & 63, wv = tid >> 6;
    const int j = lane & 31, h = lane >> 5;
    for (int i = tid; i < QVEC; i += 256) {
        const int qt = i / 448, rem = i - qt * 448;
        const int v = rem >> 6, l = rem & 63;
        qsh[i] = *reinterpret_cast<const float4 *>(
            qp + (long)((group * NQ + qt) * 32 + (l & 31)) * IA_DP + (l >> 5) * 28 + 4 * v);
    }
    __syncthreads();

    float te[NQ][SCREEN_K];
    int ti[NQ][SCREEN_K];
#pragma unroll
    for (int qt = 0; qt < NQ; ++qt)
#pragma unroll
        for (int k = 0; k < SCREEN_K; ++k) { te[qt][k] = FLT_MAX; ti[qt][k] = -1; }

    const int rows_per_wave = ch >> 2;
    const int n = rows_per_wave >> 5;
    const long row_begin = (long)chunk * ch + wv * rows_per_wave;
    const float4 *dp = tile_ptr(db, row_begin, lane);
    const int rbase0 = (int)(row_begin - (long)chunk * ch) + 4 * h;
    auto at = [&](int t) { return dp + (long)(t < n ? t : n - 1) * TILE_VEC; };

    float4 bufA[7], bufB[7];
    floatx16 accA[NQ], accB[NQ];
    float mn[NQ];
    load_tile(bufA, at(0));
    load_tile(bufB, at(1));
    mfma_tile_lds<NQ>(bufA, qsh, lane, accA);
    load_tile(bufA, at(2));
    for (int t = 0; t < n; t += 2) {
        // accA = tile t, bufB = tile t+1, bufA = tile t+2 (in flight)
        if (t + 1 < n) {
            mfma_tile_lds<NQ>(bufB, qsh, lane, accB);
            min_tile<NQ>(accA, mn);
            interleave_mark<NQ>();
        } else {
            min_tile<NQ>(accA, mn);
        }
        insert_tile<NQ>(accA, mn, te, ti, rbase0 + t * 32);
        load_tile(bufB, at(t + 3));
        if (t + 1 >= n) break;
        if (t + 2 < n) {
            mfma_tile_lds<NQ>(bufA, qsh, lane, accA);
            min_tile<NQ>(accB, mn);
            interleave_mark<NQ>();
        } else {
            min_tile<NQ>(accB, mn);
        }
        insert_tile<NQ>(accB, mn, te, ti, rbase0 + (t + 1) * 32);
        load_tile(bufA, at(t + 4));
    }

    __syncthreads();
    float(*le)[8][SCREEN_K] = reinterpret_cast<float(*)[8][SCREEN_K]>(smem);
    int(*li)[8][SCREEN_K] = reinterpret_cast<int(*)[8][SCREEN_K]>(smem + NQ * 32 * 8 * SCREEN_K * 4);
#pragma unroll
    for (int qt = 0; qt < NQ; ++qt)
#pragma unroll
        for (int k = 0; k < SCREEN_K; ++k) {
            le[qt * 32 + j][wv * 2 + h][k] = te[qt][k];
            li[qt * 32 + j][wv * 2 + h][k] = ti[qt][k];
        }
    __syncthreads();
    for (int t = tid; t < NQ * 32; t += 256) {
        const int qg = group * NQ * 32 + t;
        if (qg < M) {
            float be[SCREEN_K];
            int bi[SCREEN_K];
#pragma unroll
            for (int k = 0; k < SCREEN_K; ++k) { be[k] = FLT_MAX; bi[k] = -1; }
            for (int l = 0; l < 8; ++l)
#pragma unroll
                for (int k = 0; k < SCREEN_K; ++k) {
                    const float v = le[t][l][k];
                    if (v < be[SCREEN_K - 1]) topk_insert(be, bi, v, li[t][l][k]);
                }
            Cand *o = cand + ((long)qg * nchunks + chunk) * SCREEN_K;
            const int cbase = chunk * ch;
#pragma unroll
            for (int k = 0; k < SCREEN_K; ++k) o[k] = Cand{be[k], bi[k] < 0 ? -1 : cbase + bi[k]};
        }
    }
}

// Default screen: variant 0 (queries in VGPRs, <= 3 query tiles per wave) measured
// fastest on MI355X (tools/screen_bench, profiles/).  IA_SCREEN_VARIANT selects another
// for A/B runs (bits 0-3 kind, 4-7 tile cap).
int screen_variant() {
    static const int v = [] {
        const int x = env_int("IA_SCREEN_VARIANT", 0);
        return (x < 0 || (x & 15) > 3) ? 0 : x;
    }();
    return v;
}

int launch_screen_v(const float *db, long nrows, const float *qp, int M, Cand *cand, int variant,
                    hipStream_t st) {
    const int ch = db_chunk_rows(nrows);
    const long nchunks = db_nchunks(nrows);
    // kinds: 0 registers/2-deep, 1 LDS queries, 2 pipelined epilogue, 3 registers/3-deep;
    // diagnostic only: 4 / 5 = kinds 0 / 3 re-reading ONE tile per wave (L2-hot, wrong
    // results) to separate memory latency from issue limits.
    const int kind = variant & 15, nq_cap = (variant >> 4) & 15;
    int maxnq = (kind == 1) ? MAX_NQ : 3;
    if (kind == 3 || kind == 5) maxnq = 2;
    if (nq_cap > 0 && nq_cap < maxnq) maxnq = nq_cap;
    const QSplit qs = qsplit(M, maxnq);
    const long nblocks = ((nchunks + 7) / 8) * 8 * qs.groups;
    IA_ARG(nblocks < (1L << 31), "screen grid too large");
#define IA_SCREEN_CASE(K, N)                                                                  \
    case N:                                                                                   \
        K<N><<<(unsigned)nblocks, 256, 0, st>>>(db, (int)nchunks, ch, qp, M, qs.groups, cand); \
        break;
#define IA_SCREEN_CASE_M(N, MODE)                                                             \
    case N:                                                                                   \
        k_screen<N, MODE><<<(unsigned)nblocks, 256, 0, st>>>(db, (int)nchunks, ch, qp, M,     \
                                                             qs.groups, cand);                \
        break;
    if (kind == 0 || kind == 3 || kind == 4 || kind == 5) {
        const int mode = kind == 0 ? 0 : kind == 3 ? 1 : kind == 4 ? 2 : 3;
        if (mode == 0) {
            switch (qs.nq) {
                IA_SCREEN_CASE_M(1, 0)
                IA_SCREEN_CASE_M(2, 0)
                IA_SCREEN_CASE_M(3, 0)
                default: set_error("bad query split"); return IA_E_ARG;
            }
        } else if (mode == 1) {
            switch (qs.nq) {
                IA_SCREEN_CASE_M(1, 1)
                IA_SCREEN_CASE_M(2, 1)
                default: set_error("bad query split"); return IA_E_ARG;
            }
        } else if (mode == 2) {
            switch (qs.nq) {
                IA_SCREEN_CASE_M(1, 2)
                IA_SCREEN_CASE_M(2, 2)
                IA_SCREEN_CASE_M(3, 2)
                default: set_error("bad query split"); return IA_E_ARG;
            }
        } else {
            switch (qs.nq) {
                IA_SCREEN_CASE_M(1, 3)
                IA_SCREEN_CASE_M(2, 3)
                default: set_error("bad query split"); return IA_E_ARG;
            }
        }
#undef IA_SCREEN_CASE_M
    } else if (kind == 2) {
        switch (qs.nq) {
            IA_SCREEN_CASE(k_screen_pipe, 1)
            IA_SCREEN_CASE(k_screen_pipe, 2)
            IA_SCREEN_CASE(k_screen_pipe, 3)
            IA_SCREEN_CASE(k_screen_pipe, 4)
            default: set_error("bad query split"); return IA_E_ARG;
        }
    } else {
        switch (qs.nq) {
            IA_SCREEN_CASE(k_screen_lds, 1)
            IA_SCREEN_CASE(k_screen_lds, 2)
            IA_SCREEN_CASE(k_screen_lds, 3)
            IA_SCREEN_CASE(k_screen_lds, 4)
            IA_SCREEN_CASE(k_screen_lds, 5)
            IA_SCREEN_CASE(k_screen_lds, 6)
            default: set_error("bad query split"); return IA_E_ARG;
        }
    }
#undef IA_SCREEN_CASE
    IA_LAUNCH_CHECK("k_screen");
    return IA_OK;
}

int launch_screen(const float *db, long nrows, const float *qp, int M, Cand *cand,
                  hipStream_t st) {
    return launch_screen_v(db, nrows, qp, M, cand, screen_variant(), st);
}

// ---------------------------------------------------------------------------------
// exact merge / rescore: one 256-thread workgroup per query
// ---------------------------------------------------------------------------------
constexpr int MERGE_CAP = 2048;     // candidate rows held in LDS
constexpr int MERGE_OCAP = 256;     // overflow chunks held in LDS

__device__ __forceinline__ void best_update(double &bd, long long &bi, double d, long long i) {
    if (d < bd || (d == bd && i < bi)) { bd = d; bi = i; }
}

__global__ __launch_bounds__(256) void k_merge(DbSrc src, long row0, long nrows, int nchunks,
                                               int ch, const Cand *__restrict__ cand,
                                               const double *__restrict__ q64,
                                               const double *__restrict__ nq,
                                               const float *__restrict__ amax,
                                               Best *__restrict__ best,
                                               unsigned long long *stats) {
    __shared__ int clist[MERGE_CAP];
    __shared__ int olist[MERGE_OCAP];
    __shared__ int ccount, ocount;
    __shared__ float redf[4];
    __shared__ double redd[4];
    __shared__ long long redi[4];
    __shared__ double qs[IA_DP];

    const int q = blockIdx.x;
    const int tid = threadIdx.x;
    const Cand *cq = cand + (long)q * nchunks * SCREEN_K;
    if (tid < IA_DP) qs[tid] = q64[(long)q * IA_DP + tid];
    if (tid == 0) { ccount = 0; ocount = 0; }

    float emin = FLT_MAX;
    for (int c = tid; c < nchunks; c += 256) emin = fminf(emin, cq[(long)c * SCREEN_K].e);
    for (int o = 32; o > 0; o >>= 1) emin = fminf(emin, __shfl_xor(emin, o));
    if ((tid & 63) == 0) redf[tid >> 6] = emin;
    __syncthreads();
    emin = fminf(fminf(redf[0], redf[1]), fminf(redf[2], redf[3]));

    const double A = (double)amax[0];
    const double nqq = nq[q];
    const double eps = 70.0 * 5.9604644775390625e-08 * (2.0 * A * sqrt(nqq) + A * A);
    const double T = (double)emin + 2.0 * eps + 1e-12 * (fabs((double)emin) + nqq + A * A);

    for (int c = tid; c < nchunks; c += 256) {
        const Cand *e = cq + (long)c * SCREEN_K;
#pragma unroll
        for (int k = 0; k < SCREEN_K; ++k) {
            if ((double)e[k].e <= T && e[k].idx >= 0 && e[k].idx < nrows) {
                const int pos = atomicAdd(&ccount, 1);
                if (pos < MERGE_CAP) clist[pos] = e[k].idx;
            }
        }
        if ((double)e[SCREEN_K - 1].e <= T) {
            const int pos = atomicAdd(&ocount, 1);
            if (pos < MERGE_OCAP) olist[pos] = c;
        }
    }
    __syncthreads();
    const int nc = ccount, no = ocount;
    const bool full = nc > MERGE_CAP || no > MERGE_OCAP;

    double bd = INFINITY;
    long long bi = 0x7fffffffffffffffLL;
    if (full) {
        for (long lr = tid; lr < nrows; lr += 256)
            best_update(bd, bi, row_dist2(src, row0 + lr, qs), row0 + lr);
    } else {
        for (int i = tid; i < nc; i += 256) {
            const long ix = row0 + clist[i];
            best_update(bd, bi, row_dist2(src, ix, qs), ix);
        }
        for (int o = 0; o < no; ++o) {
            const long lo = (long)olist[o] * ch;
            const long hi = lo + ch < nrows ? lo + ch : nrows;
            for (long lr = lo + tid; lr < hi; lr += 256)
                best_update(bd, bi, row_dist2(src, row0 + lr, qs), row0 + lr);
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        const double od = __shfl_xor(bd, o);
        const long long oi = __shfl_xor(bi, o);
        best_update(bd, bi, od, oi);
    }
    if ((tid & 63) == 0) { redd[tid >> 6] = bd; redi[tid >> 6] = bi; }
    __syncthreads();
    if (tid == 0) {
        for (int w = 1; w < 4; ++w) best_update(bd, bi, redd[w], redi[w]);
        best[q] = Best{bd, bi};
        if (stats) {
            unsigned long long *sl = stats_slot(stats, q);
            atomicAdd(&sl[0], (unsigned long long)nc);
            atomicAdd(&sl[1], (unsigned long long)no);
            atomicAdd(&sl[2], full ? 1ULL : 0ULL);
        }
    }
}

int launch_merge(const DbSrc &src, long row0, long nrows, const Cand *cand, int M,
                 const double *q64, const double *nq, const float *amax, Best *best,
                 unsigned long long *stats, hipStream_t st) {
    const int ch = db_chunk_rows(nrows);
    const long nchunks = db_nchunks(nrows);
    k_merge<<<M, 256, 0, st>>>(src, row0, nrows, (int)nchunks, ch, cand, q64, nq, amax, best,
                               stats);
    IA_LAUNCH_CHECK("k_merge");
    return IA_OK;
}

// =================================================================================
// Segment-minimum matcher (default): the screen keeps NO per-row state, only the
// running minimum of e per (query, 512-row segment) — 8 v_min3 per 16 values, branch
// free — and the exact stage re-screens just the segments whose minimum lies inside the
// error window.  Exactness: the oracle's winner r_o has e(r_o) <= e* + 2 eps_q (e* the
// global minimum), so its segment's minimum is inside the window; inside a candidate
// segment a VALU fp32 recomputation e'(r) obeys the same bound, so every row with
// e'(r) <= e* + 2 eps_q (+ slack) is rescored in fp64 and r_o is among them.
// =================================================================================
// one workgroup's work: DB chunk `chunk` against query tiles [tile0, tile0 + NQ)
template <int NQ>
__device__ __forceinline__ void seg_body(const float *__restrict__ db, int chunk, int ch,
                                         int seg_rows, const float *__restrict__ qp, int M,
                                         int tile0, float *__restrict__ segmin, long nseg) {
    const int tid = threadIdx.x;
    const int lane = tid & 63, wv = tid >> 6;
    const int j = lane & 31, h = lane >> 5;

    float bq[NQ][28];
#pragma unroll
    for (int qt = 0; qt < NQ; ++qt) {
        const float4 *p = reinterpret_cast<const float4 *>(
            qp + (long)((tile0 + qt) * 32 + j) * IA_DP + h * 28);
#pragma unroll
        for (int v = 0; v < 7; ++v) {
            const float4 x = p[v];
            bq[qt][4 * v] = x.x; bq[qt][4 * v + 1] = x.y;
            bq[qt][4 * v + 2] = x.z; bq[qt][4 * v + 3] = x.w;
        }
    }
    const int rows_per_wave = ch >> 2;
    const int ntile = rows_per_wave >> 5;
    const int tps = seg_rows >> 5;                          // tiles per segment
    const long row_begin = (long)chunk * ch + wv * rows_per_wave;
    const long seg_begin = row_begin / seg_rows;
    const float4 *dp = tile_ptr(db, row_begin, lane);

    float mn[NQ];
#pragma unroll
    for (int qt = 0; qt < NQ; ++qt) mn[qt] = FLT_MAX;

    auto tile_min = [&](const float4 (&a4)[7]) {
        floatx16 acc[NQ];
#pragma unroll
        for (int qt = 0; qt < NQ; ++qt)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[qt][r] = 0.f;
#pragma unroll
        for (int v = 0; v < 7; ++v) {
            const float av[4] = {a4[v].x, a4[v].y, a4[v].z, a4[v].w};
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int qt = 0; qt < NQ; ++qt)
                    acc[qt] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[u], bq[qt][4 * v + u],
                                                                   acc[qt], 0, 0, 0);
        }
#pragma unroll
        for (int qt = 0; qt < NQ; ++qt) {
            float m = mn[qt];
#pragma unroll
            for (int r = 0; r < 16; r += 2) m = fminf(m, fminf(acc[qt][r], acc[qt][r + 1]));
            mn[qt] = m;
        }
    };
    auto flush = [&](int tile) {   // after the last tile of a segment
        const long seg = seg_begin + tile / tps;
#pragma unroll
        for (int qt = 0; qt < NQ; ++qt) {
            const float m = fminf(mn[qt], __shfl_xor(mn[qt], 32));
            const int qg = (tile0 + qt) * 32 + j;
            if (h == 0 && qg < M) segmin[(long)qg * nseg + seg] = m;
            mn[qt] = FLT_MAX;
        }
    };

    float4 b0[7], b1[7];
    load_tile(b0, dp);
    int tile = 0;
    for (; tile + 1 < ntile; tile += 2) {
        load_tile(b1, dp + (long)(tile + 1) * TILE_VEC);
        tile_min(b0);
        if ((tile + 1) % tps == 0) flush(tile);
        const int nxt = tile + 2 < ntile ? tile + 2 : ntile - 1;
        load_tile(b0, dp + (long)nxt * TILE_VEC);
        tile_min(b1);
        if ((tile + 2) % tps == 0) flush(tile + 1);
    }
    if (tile < ntile) {
        tile_min(b0);
        flush(tile);
    }
}

// grid: nchunks (rounded up to 8) x groups, XCD-aware as k_screen.  The first nA groups
// hold NQA query tiles, the rest NQB (< NQA) tiles, so a launch computes exactly
// ceil(M/32) tiles with the largest groups that split them evenly (measured on MI355X:
// 3-tile groups run ~15 % faster per tile than 2-tile ones, which beat 1-tile ones by
// ~25 %; tools/screen_bench, profiles/r01_screen_bench_split.txt).
template <int NQA, int NQB>
__global__ __launch_bounds__(256) void k_screen_seg(const float *__restrict__ db, int nchunks,
                                                    int ch, int seg_rows,
                                                    const float *__restrict__ qp, int M,
                                                    int groups, int nA,
                                                    float *__restrict__ segmin, long nseg) {
    const int b = blockIdx.x;
    const int slot = b >> 3;
    const int chunk = (slot / groups) * 8 + (b & 7);
    const int group = slot - (slot / groups) * groups;
    if (chunk >= nchunks) return;
    if (NQB > 0 && group >= nA)
        seg_body<(NQB > 0 ? NQB : 1)>(db, chunk, ch, seg_rows, qp, M,
                                      nA * NQA + (group - nA) * NQB, segmin, nseg);
    else
        seg_body<NQA>(db, chunk, ch, seg_rows, qp, M, group * NQA, segmin, nseg);
}

// Phase probes (tools/rescore_probe only: built with -DIA_PROBE into a separate library):
// lane 0 of every wave of the first 64 workgroups stores wall_clock64() at each mark
// (slot [block][wave][mark], 64 x 4 x 16).
#ifdef IA_PROBE
__device__ unsigned long long *g_probe;
#define IA_PROBE_MARK(i)                                                                    \
    do {                                                                                    \
        if ((threadIdx.x & 63) == 0 && blockIdx.x < 64 && g_probe)                           \
            g_probe[(blockIdx.x * 4 + (threadIdx.x >> 6)) * 16 + (i)] = wall_clock64();     \
    } while (0)
#else
#define IA_PROBE_MARK(i) \
    do {                 \
    } while (0)
#endif

// Thresholds of the exact stage from the minimum segment minimum emin:
// Tseg for segment minima (screen units), Trow for the fp32 VALU re-screen (unscaled).
// f32 screen: both e* + 2 eps.  Split-f16 screen (minima in units of sa * sq): e* = emin /
// (sa sq) exactly, Tseg = e* + 2 eps16, Trow = e* + eps16 + eps; force_full when the
// query's norm slot nears the f16 floor (|q'| > 2^24 Amax).
template <bool SPLIT>
__device__ __forceinline__ void rescore_thresholds(float emin, float amax0, double nqq,
                                                   double &Tseg, double &Trow, bool &force_full) {
    constexpr double U32 = 5.9604644775390625e-08;
    const double A = (double)amax0;
    const double eps = 70.0 * U32 * (2.0 * A * sqrt(nqq) + A * A);
    force_full = false;
    if (SPLIT) {
        const Split16Db sc = split16_db_scale(amax0);
        const int eq = split16_q_scale(nqq, sc.R);
        const int e2 = sc.ea + eq;
        const double em = ldexp((double)emin, -e2);
        const double eps16 = U32 * (300.0 * A * sqrt(nqq) + 50.0 * A * A);
        const double slack = 1e-12 * (fabs(em) + nqq + A * A);
        Tseg = ldexp(em + 2.0 * eps16 + slack, e2);
        Trow = em + eps16 + eps + slack;
        force_full = eq + sc.R < -10;
    } else {
        Tseg = Trow = (double)emin + 2.0 * eps + 1e-12 * (fabs((double)emin) + nqq + A * A);
    }
}

constexpr int RESCORE_SEGCAP = 1024;   // candidate segments held in LDS per query
constexpr int RESCORE_REG = 8;         // float4s of segment minima per thread kept in VGPRs
constexpr int RESCORE_RPT = 2;         // candidate rows per thread per step
constexpr int RESCORE_ROWCAP = 512;    // rows to rescore held in LDS per query

// Exact stage of the segment-minimum matcher: one 256-thread workgroup per query.
// FIN: single shard — wave 0 then runs the per-pixel tail of the synthesis step
// (ia_finish.h) on the winner, saving a launch and a round trip per wave.
template <bool FIN, bool SPLIT>
__global__ __launch_bounds__(256) void k_rescore(DbSrc src, long row0, long nrows, long nseg,
                                                 int seg_rows, const float *__restrict__ segmin,
                                                 const float *__restrict__ db,
                                                 const float *__restrict__ qp,
                                                 const double *__restrict__ q64,
                                                 const double *__restrict__ nq,
                                                 const float *__restrict__ amax,
                                                 Best *__restrict__ best,
                                                 unsigned long long *stats, FinishArgs fa,
                                                 int probe) {
    __shared__ int slist[RESCORE_SEGCAP];
    __shared__ long long win;
    __shared__ CohSel cs;
    __shared__ int scount;
    __shared__ float redf[4];
    __shared__ double redd[4];
    __shared__ long long redi[4];
    __shared__ double qs[IA_DP];
    __shared__ float qf[IA_DP];
    __shared__ unsigned int nresc;
    __shared__ long rlist[RESCORE_ROWCAP];
    __shared__ int rcount;

    const int q = blockIdx.x;
    const int tid = threadIdx.x;
    IA_PROBE_MARK(0);
    if (tid < IA_DP) {
        qs[tid] = q64[(long)q * IA_DP + tid];
        qf[tid] = qp[(long)q * IA_DP + tid];
    }
    if (tid == 0) { scount = 0; nresc = 0; rcount = 0; }
    const float *sq = segmin + (long)q * nseg;
    const double A = (double)amax[0];   // issued with the segment-minimum loads
    const double nqq = nq[q];

    // segment minima of this query: the first RESCORE_REG*256 float4s stay in registers
    // between the two passes (all loads of a pass in flight at once); nseg is a multiple
    // of 4 (>= 4 segments per chunk)
    const long n4 = nseg / 4;
    const float4 *sq4 = reinterpret_cast<const float4 *>(sq);
    float4 v[RESCORE_REG];
#pragma unroll
    for (int j = 0; j < RESCORE_REG; ++j) {
        const long i = tid + (long)j * 256;
        v[j] = i < n4 ? sq4[i] : make_float4(FLT_MAX, FLT_MAX, FLT_MAX, FLT_MAX);
    }
    float emin = FLT_MAX;
#pragma unroll
    for (int j = 0; j < RESCORE_REG; ++j)
        emin = fminf(emin, fminf(fminf(v[j].x, v[j].y), fminf(v[j].z, v[j].w)));
    for (long i = tid + (long)RESCORE_REG * 256; i < n4; i += 256) {
        const float4 x = sq4[i];
        emin = fminf(emin, fminf(fminf(x.x, x.y), fminf(x.z, x.w)));
    }
    for (int o = 32; o > 0; o >>= 1) emin = fminf(emin, __shfl_xor(emin, o));
    if ((tid & 63) == 0) redf[tid >> 6] = emin;
    IA_PROBE_MARK(1);
    __syncthreads();
    IA_PROBE_MARK(2);
    emin = fminf(fminf(redf[0], redf[1]), fminf(redf[2], redf[3]));

    double Tseg, Trow;
    bool force_full;
    rescore_thresholds<SPLIT>(emin, amax[0], nqq, Tseg, Trow, force_full);

    auto push = [&](float e, long s) {
        if ((double)e <= Tseg) {
            const int pos = atomicAdd(&scount, 1);
            if (pos < RESCORE_SEGCAP) slist[pos] = (int)s;
        }
    };
#pragma unroll
    for (int j = 0; j < RESCORE_REG; ++j) {
        const long i = tid + (long)j * 256;
        push(v[j].x, 4 * i);
        push(v[j].y, 4 * i + 1);
        push(v[j].z, 4 * i + 2);
        push(v[j].w, 4 * i + 3);
    }
    for (long i = tid + (long)RESCORE_REG * 256; i < n4; i += 256) {
        const float4 x = sq4[i];
        push(x.x, 4 * i);
        push(x.y, 4 * i + 1);
        push(x.z, 4 * i + 2);
        push(x.w, 4 * i + 3);
    }
    if (SPLIT && probe && stats) {
        // diagnostic (IA_PRUNE_PROBE): how many segments a coarser screen would leave to the
        // exact stage.  Coarse f16 forms, error bounds in unscaled units: a_h q_h (4 MFMAs)
        // eps4 = 2^-9 A|q'| + 2^-11 A^2, a_h (q_h + q_l) (8 MFMAs) eps8 = 2^-10 A|q'| + 2^-11 A^2
        // (+ 2^-8 relative and 2^-18 (2A|q'| + A^2) accumulation allowances); counts of
        // segments with minimum <= e* + 2 eps4, e* + 4 eps4, e* + 2 eps8.
        const Split16Db sc = split16_db_scale(amax[0]);
        const int e2 = sc.ea + split16_q_scale(nqq, sc.R);
        const double em = ldexp((double)emin, -e2);
        const double aq = A * sqrt(nqq), acc = 0x1p-18 * (2.0 * aq + A * A);
        const double e4 = (0x1p-9 * aq + 0x1p-11 * A * A) * (1.0 + 0x1p-8) + acc;
        const double e8 = (0x1p-10 * aq + 0x1p-11 * A * A) * (1.0 + 0x1p-8) + acc;
        const double t42 = ldexp(em + 2.0 * e4, e2), t44 = ldexp(em + 4.0 * e4, e2);
        const double t82 = ldexp(em + 2.0 * e8, e2);
        unsigned int c42 = 0, c44 = 0, c82 = 0;
        for (long i = tid; i < nseg; i += 256) {
            const double x = (double)sq[i];
            c42 += x <= t42; c44 += x <= t44; c82 += x <= t82;
        }
        for (int o = 32; o > 0; o >>= 1) {
            c42 += __shfl_xor(c42, o); c44 += __shfl_xor(c44, o); c82 += __shfl_xor(c82, o);
        }
        __shared__ unsigned int pc[3];
        if (tid == 0) { pc[0] = 0; pc[1] = 0; pc[2] = 0; }
        __syncthreads();
        if ((tid & 63) == 0) { atomicAdd(&pc[0], c42); atomicAdd(&pc[1], c44); atomicAdd(&pc[2], c82); }
        __syncthreads();
        if (tid == 0) {
            unsigned long long *sl = stats_slot(stats, q);
            atomicAdd(&sl[3], (unsigned long long)pc[0]);
            atomicAdd(&sl[4], (unsigned long long)pc[1]);
            atomicAdd(&sl[5], (unsigned long long)pc[2]);
            atomicMax(&sl[6], (unsigned long long)pc[0]);
        }
    }
    __syncthreads();
    IA_PROBE_MARK(3);
    const int ns = scount;
    const bool full = ns > RESCORE_SEGCAP || force_full;
    const long nscan = full ? nseg : ns;

    double bd = INFINITY;
    long long bi = 0x7fffffffffffffffLL;
    unsigned int mine = 0;
    // rows of the candidate segments, RESCORE_RPT per thread per step with all their DB
    // loads issued together (seg_rows <= 512 = RESCORE_RPT * 256: one step per segment)
    const long nrs = nscan * seg_rows;
    for (long base = 0; base < nrs; base += RESCORE_RPT * 256) {
        float e[RESCORE_RPT];
        long lr[RESCORE_RPT];
#pragma unroll
        for (int u = 0; u < RESCORE_RPT; ++u) {
            const long k = base + u * 256 + tid;
            const long seg = k < nrs ? (full ? k / seg_rows : slist[k / seg_rows]) : 0;
            lr[u] = k < nrs ? seg * seg_rows + k % seg_rows : nrows;
            // fp32 recomputation from the fragment-major DB (row lr = tile*32 + jj);
            // out-of-range rows read row 0 and are discarded below
            const long r = lr[u] < nrows ? lr[u] : 0;
            const float4 *t4 = reinterpret_cast<const float4 *>(db) + (r >> 5) * TILE_VEC + (r & 31);
            float acc = 0.f;
#pragma unroll
            for (int hh = 0; hh < 2; ++hh)
#pragma unroll
                for (int v = 0; v < 7; ++v) {
                    const float4 x = t4[v * 64 + hh * 32];
                    const float *qv = qf + hh * 28 + 4 * v;
                    acc = fmaf(x.x, qv[0], acc);
                    acc = fmaf(x.y, qv[1], acc);
                    acc = fmaf(x.z, qv[2], acc);
                    acc = fmaf(x.w, qv[3], acc);
                }
            e[u] = acc;
        }
        IA_PROBE_MARK(8);
        // rows within Trow go to a list rescored one per thread after the loop (one round
        // of feature gathers); a list overflow is rescored in place
#pragma unroll
        for (int u = 0; u < RESCORE_RPT; ++u) {
            if (lr[u] < nrows && (double)e[u] <= Trow) {
                ++mine;
                const int pos = atomicAdd(&rcount, 1);
                if (pos < RESCORE_ROWCAP) rlist[pos] = lr[u];
                else best_update(bd, bi, row_dist2(src, row0 + lr[u], qs), row0 + lr[u]);
            }
        }
    }
    __syncthreads();
    {
        const int nl = rcount < RESCORE_ROWCAP ? rcount : RESCORE_ROWCAP;
        for (int i = tid; i < nl; i += 256)
            best_update(bd, bi, row_dist2(src, row0 + rlist[i], qs), row0 + rlist[i]);
    }
    for (int o = 32; o > 0; o >>= 1) {
        const double od = __shfl_xor(bd, o);
        const long long oi = __shfl_xor(bi, o);
        best_update(bd, bi, od, oi);
    }
    if (mine) atomicAdd(&nresc, mine);
    if ((tid & 63) == 0) { redd[tid >> 6] = bd; redi[tid >> 6] = bi; }
    IA_PROBE_MARK(4);
    __syncthreads();
    IA_PROBE_MARK(5);
    if (tid == 0) {
        for (int w = 1; w < 4; ++w) best_update(bd, bi, redd[w], redi[w]);
        best[q] = Best{bd, bi};
        win = bi;
        if (stats) {
            unsigned long long *sl = stats_slot(stats, q);
            atomicAdd(&sl[0], (unsigned long long)nresc);
            atomicAdd(&sl[1], (unsigned long long)ns);
            atomicAdd(&sl[2], full ? 1ULL : 0ULL);
        }
    }
    if (FIN) {   // wave 1 picks the coherence candidate while wave 0 weighs the winner
        __syncthreads();
        const int wv = tid >> 6, lane = tid & 63;
        double d_app = 0.0;
        if (wv == 1) {
            const CohSel c = coh_pick(src, q, fa, qs, lane);
            if (lane == 0) cs = c;
        } else if (wv == 0) {
            d_app = app_wdist(src, win, fa, qs, lane);
        }
        __syncthreads();
        if (wv == 0) finish_apply(src, win, q, fa, cs, d_app, lane);
        IA_PROBE_MARK(6);
    }
}

// ---------------------------------------------------------------------------------
// Work-list exact stage: the same thresholds and the same rows as
// k_rescore, but the candidate segments of all queries become items of one list, so a
// query with many candidate segments spreads over many workgroups instead of serialising
// in one (k_rescore's time is that of its heaviest query).
//   k_select  one workgroup per query: e*, thresholds, candidate segments -> items
//   k_items   one workgroup per item (grid-stride): fp32 re-screen of the segment's rows,
//             exact rescore of those <= Trow -> the item's (distance, row) minimum
//   k_gather  one wave per query: the lexicographic minimum over its items [+ the
//             per-pixel tail]; also empties the list for the next call
// ---------------------------------------------------------------------------------
template <bool SPLIT>
__global__ __launch_bounds__(256) void k_select(long nseg, const float *__restrict__ segmin,
                                                const double *__restrict__ nq,
                                                const float *__restrict__ amax, int *ctr,
                                                WItem *__restrict__ items, QSel *__restrict__ sel,
                                                unsigned long long *stats) {
    __shared__ int slist[RESCORE_SEGCAP];
    __shared__ int scount, sbase;
    __shared__ float redf[4];
    const int q = blockIdx.x;
    const int tid = threadIdx.x;
    if (tid == 0) scount = 0;
    const float *sq = segmin + (long)q * nseg;
    const double nqq = nq[q];
    const long n4 = nseg / 4;
    const float4 *sq4 = reinterpret_cast<const float4 *>(sq);
    float4 v[RESCORE_REG];
#pragma unroll
    for (int j = 0; j < RESCORE_REG; ++j) {
        const long i = tid + (long)j * 256;
        v[j] = i < n4 ? sq4[i] : make_float4(FLT_MAX, FLT_MAX, FLT_MAX, FLT_MAX);
    }
    float emin = FLT_MAX;
#pragma unroll
    for (int j = 0; j < RESCORE_REG; ++j)
        emin = fminf(emin, fminf(fminf(v[j].x, v[j].y), fminf(v[j].z, v[j].w)));
    for (long i = tid + (long)RESCORE_REG * 256; i < n4; i += 256) {
        const float4 x = sq4[i];
        emin = fminf(emin, fminf(fminf(x.x, x.y), fminf(x.z, x.w)));
    }
    for (int o = 32; o > 0; o >>= 1) emin = fminf(emin, __shfl_xor(emin, o));
    if ((tid & 63) == 0) redf[tid >> 6] = emin;
    __syncthreads();
    emin = fminf(fminf(redf[0], redf[1]), fminf(redf[2], redf[3]));
    double Tseg, Trow;
    bool force_full;
    rescore_thresholds<SPLIT>(emin, amax[0], nqq, Tseg, Trow, force_full);
    auto push = [&](float e, long s) {
        if ((double)e <= Tseg) {
            const int pos = atomicAdd(&scount, 1);
            if (pos < RESCORE_SEGCAP) slist[pos] = (int)s;
        }
    };
#pragma unroll
    for (int j = 0; j < RESCORE_REG; ++j) {
        const long i = tid + (long)j * 256;
        push(v[j].x, 4 * i);
        push(v[j].y, 4 * i + 1);
        push(v[j].z, 4 * i + 2);
        push(v[j].w, 4 * i + 3);
    }
    for (long i = tid + (long)RESCORE_REG * 256; i < n4; i += 256) {
        const float4 x = sq4[i];
        push(x.x, 4 * i);
        push(x.y, 4 * i + 1);
        push(x.z, 4 * i + 2);
        push(x.w, 4 * i + 3);
    }
    __syncthreads();
    const int ns = scount;
    const bool full = ns > RESCORE_SEGCAP || force_full;
    const int cnt = full ? (int)nseg : ns;
    if (tid == 0) {
        sbase = atomicAdd(ctr, cnt);
        sel[q] = QSel{Trow, sbase, cnt};
        if (stats) {
            unsigned long long *sl = stats_slot(stats, q);
            atomicAdd(&sl[1], (unsigned long long)ns);
            atomicAdd(&sl[2], full ? 1ULL : 0ULL);
        }
    }
    __syncthreads();
    const int base = sbase;
    for (int i = tid; i < cnt; i += 256) items[base + i] = WItem{q, full ? i : slist[i], Trow};
}

__global__ __launch_bounds__(256) void k_items(DbSrc src, long row0, long nrows, int seg_rows,
                                               const WItem *__restrict__ items,
                                               const int *__restrict__ ctr,
                                               const float *__restrict__ db,
                                               const float *__restrict__ qp,
                                               const double *__restrict__ q64,
                                               Best *__restrict__ ibest,
                                               unsigned long long *stats) {
    __shared__ double qs[IA_DP];
    __shared__ float qf[IA_DP];
    __shared__ double redd[4];
    __shared__ long long redi[4];
    __shared__ int plist[RESCORE_RPT * 256];
    __shared__ int pcount;
    IA_PROBE_MARK(0);
    const int n = *ctr;
    const int tid = threadIdx.x;
    for (int it = blockIdx.x; it < n; it += gridDim.x) {
        const WItem w = items[it];
        // this thread's rows of the segment (fragment-major fp32 DB, as k_rescore), issued
        // before the query is staged so that the two round trips overlap
        float4 x[RESCORE_RPT][14];
        long lr[RESCORE_RPT];
#pragma unroll
        for (int u = 0; u < RESCORE_RPT; ++u) {
            const int k = u * 256 + tid;
            lr[u] = k < seg_rows ? (long)w.seg * seg_rows + k : nrows;
            const long r = lr[u] < nrows ? lr[u] : 0;
            const float4 *t4 = reinterpret_cast<const float4 *>(db) + (r >> 5) * TILE_VEC + (r & 31);
#pragma unroll
            for (int hh = 0; hh < 2; ++hh)
#pragma unroll
                for (int v = 0; v < 7; ++v) x[u][hh * 7 + v] = t4[v * 64 + hh * 32];
        }
        __syncthreads();                       // the previous item's LDS reads are done
        if (tid < IA_DP) {
            qs[tid] = q64[(long)w.q * IA_DP + tid];
            qf[tid] = qp[(long)w.q * IA_DP + tid];
        }
        if (tid == 0) pcount = 0;
        __syncthreads();
        IA_PROBE_MARK(1);
        // fp32 re-screen; rows within Trow go to one list, rescored one per thread below
        // (a single round of feature gathers, however the passing rows fall over lanes)
#pragma unroll
        for (int u = 0; u < RESCORE_RPT; ++u) {
            float acc = 0.f;
#pragma unroll
            for (int hh = 0; hh < 2; ++hh)
#pragma unroll
                for (int v = 0; v < 7; ++v) {
                    const float4 xv = x[u][hh * 7 + v];
                    const float *qv = qf + hh * 28 + 4 * v;
                    acc = fmaf(xv.x, qv[0], acc);
                    acc = fmaf(xv.y, qv[1], acc);
                    acc = fmaf(xv.z, qv[2], acc);
                    acc = fmaf(xv.w, qv[3], acc);
                }
            if (lr[u] < nrows && (double)acc <= w.trow) plist[atomicAdd(&pcount, 1)] = u * 256 + tid;
        }
        __syncthreads();
        IA_PROBE_MARK(2);
        const int np = pcount;
        double bd = INFINITY;
        long long bi = 0x7fffffffffffffffLL;
        for (int i = tid; i < np; i += 256) {
            const long row = row0 + (long)w.seg * seg_rows + plist[i];
            best_update(bd, bi, row_dist2(src, row, qs), row);
        }
        IA_PROBE_MARK(3);
        for (int o = 32; o > 0; o >>= 1) {
            const double od = __shfl_xor(bd, o);
            const long long oi = __shfl_xor(bi, o);
            best_update(bd, bi, od, oi);
        }
        if ((tid & 63) == 0) { redd[tid >> 6] = bd; redi[tid >> 6] = bi; }
        __syncthreads();
        IA_PROBE_MARK(4);
        if (tid == 0) {
            for (int wv = 1; wv < 4; ++wv) best_update(bd, bi, redd[wv], redi[wv]);
            ibest[it] = Best{bd, bi};
            if (stats) atomicAdd(&stats_slot(stats, w.q)[0], (unsigned long long)np);
        }
    }
}

// FIN: two waves — wave 1 picks the coherence candidate (two gather rounds that need only
// s / im of earlier waves) while wave 0 reduces the items; then wave 0 finishes the pixel
template <bool FIN>
__global__ __launch_bounds__(128) void k_gather(DbSrc src, const QSel *__restrict__ sel,
                                                const Best *__restrict__ ibest, int *ctr,
                                                Best *__restrict__ best, FinishArgs fa,
                                                const double *__restrict__ q64) {
    __shared__ double qs[IA_DP];
    __shared__ CohSel cs;
    const int m = blockIdx.x;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (FIN) {
        if (threadIdx.x < IA_DP) qs[threadIdx.x] = q64[(long)m * IA_DP + threadIdx.x];
        __syncthreads();
        if (wv == 1) {
            const CohSel c = coh_pick(src, m, fa, qs, lane);
            if (lane == 0) cs = c;
        }
    }
    double bd = INFINITY;
    long long bi = 0x7fffffffffffffffLL;
    if (wv == 0) {
        const QSel r = sel[m];
        for (int i = lane; i < r.count; i += 64) {
            const Best b = ibest[r.base + i];
            best_update(bd, bi, b.d, b.idx);
        }
        for (int o = 32; o > 0; o >>= 1) {
            const double od = __shfl_xor(bd, o);
            const long long oi = __shfl_xor(bi, o);
            best_update(bd, bi, od, oi);
        }
        if (m == 0 && lane == 0) *ctr = 0;   // every k_items block has read it
    }
    if (FIN) {
        const double d_app = wv == 0 ? app_wdist(src, bi, fa, qs, lane) : 0.0;
        __syncthreads();
        if (wv == 0) finish_apply(src, bi, m, fa, cs, d_app, lane);
    } else if (wv == 0 && lane == 0) {
        best[m] = Best{bd, bi};
    }
}

// 0: per-query k_rescore, 1: work list, -1: default (see launch_match); settable through
// ia_diag_set_rescore_mode
static std::atomic<int> g_rescore_mode{env_int("IA_RESCORE", -1)};
static int rescore_mode() { return g_rescore_mode.load(std::memory_order_relaxed); }

int fuse_finish() {
    static const int f = env_int("IA_FUSE_FINISH", 2);
    return f;
}

int launch_screen_seg(const float *db, long nrows, const float *qp, int M, float *segmin,
                      int maxnq, hipStream_t st, const _Float16 *q16) {
    if (q16) return launch_screen16(db, nrows, q16, M, segmin, maxnq, st);
    const int ch = db_chunk_rows(nrows);
    const long nchunks = db_nchunks(nrows);
    const int seg_rows = db_seg_rows(nrows);
    const long nseg = db_nsegs(nrows);
    const bool uniform = maxnq & 0x100;      // diagnostic: pad to whole groups of maxnq
    maxnq &= 0xff;
    const int T = (M + 31) / 32;
    int nqa, nqb, nA, groups;
    if (uniform || maxnq < 3 || T < 3) {
        nqa = T < maxnq ? T : maxnq;
        nqb = 0;
        groups = (T + nqa - 1) / nqa;
        nA = groups;
    } else {                                 // T = 3a + 2b with b in {0, 1, 2} minimal
        const int b = (3 - T % 3) % 3;
        nqa = 3;
        nqb = b ? 2 : 0;
        nA = (T - 2 * b) / 3;
        groups = nA + b;
        if (T == 4) { nqa = 2; nqb = 0; nA = 2; groups = 2; }
    }
    const long nblocks = ((nchunks + 7) / 8) * 8 * groups;
    IA_ARG(nblocks < (1L << 31), "screen grid too large");
#define IA_SEG_CASE(NA, NB)                                                                   \
    if (nqa == NA && nqb == NB) {                                                             \
        k_screen_seg<NA, NB><<<(unsigned)nblocks, 256, 0, st>>>(db, (int)nchunks, ch, seg_rows, \
                                                                qp, M, groups, nA, segmin,    \
                                                                nseg);                        \
        IA_LAUNCH_CHECK("k_screen_seg");                                                      \
        return IA_OK;                                                                         \
    }
    IA_SEG_CASE(1, 0)
    IA_SEG_CASE(2, 0)
    IA_SEG_CASE(3, 0)
    IA_SEG_CASE(3, 2)
#undef IA_SEG_CASE
    set_error("bad query split");
    return IA_E_ARG;
}

// 0 = per-lane top-K, 1 = segment minima (f32 MFMA), 2 = segment minima (split f16);
// settable through ia_diag_set_match_alg
static std::atomic<int> g_match_alg{[] {
    const int a = env_int("IA_MATCH_ALG", 2);
    return (a < 0 || a > 2) ? 2 : a;
}()};
int match_alg() { return g_match_alg.load(std::memory_order_relaxed); }

// segment matcher scratch: [list counter | segment minima | items | item winners | per-query
// records]; the counter sits at a fixed offset (it carries over between calls, emptied by
// k_gather)
static constexpr size_t WL_HEAD = 256;
struct SegWs {
    int *ctr;
    float *segmin;
    WItem *items;
    Best *ibest;
    QSel *sel;
};
static SegWs seg_ws(void *scratch, int M, long nrows) {
    char *p = reinterpret_cast<char *>(scratch);
    const size_t n = (size_t)M * db_nsegs(nrows);
    SegWs w;
    w.ctr = reinterpret_cast<int *>(p);
    w.segmin = reinterpret_cast<float *>(p + WL_HEAD);
    w.items = reinterpret_cast<WItem *>(p + WL_HEAD + align_up(n * sizeof(float), 256));
    w.ibest = reinterpret_cast<Best *>(reinterpret_cast<char *>(w.items) + align_up(n * sizeof(WItem), 256));
    w.sel = reinterpret_cast<QSel *>(reinterpret_cast<char *>(w.ibest) + align_up(n * sizeof(Best), 256));
    return w;
}
size_t match_scratch_bytes(int qrows, long nrows) {
    const size_t a = (size_t)qrows * db_nchunks(nrows) * SCREEN_K * sizeof(Cand);
    const size_t n = (size_t)qrows * db_nsegs(nrows);
    const size_t b = WL_HEAD + align_up(n * sizeof(float), 256) + align_up(n * sizeof(WItem), 256) +
                     align_up(n * sizeof(Best), 256) + align_up((size_t)qrows * sizeof(QSel), 256);
    return a > b ? a : b;
}

int launch_match(const DbSrc &src, long row0, long nrows, const float *db, const float *qp,
                 const _Float16 *q16, int M, const double *q64, const double *nq,
                 const float *amax, void *scratch, Best *best, unsigned long long *stats,
                 hipStream_t st, hipEvent_t ev0, hipEvent_t ev1, const FinishArgs *fin) {
    int rc;
    if (ev0) IA_HIP(hipEventRecord(ev0, st));
    IA_ARG(!fin || match_alg() >= 1, "launch_match: the fused tail needs the segment matcher");
    IA_ARG(match_alg() != 2 || q16, "launch_match: split-f16 screen without q16 rows");
    if (match_alg() == 0) {
        Cand *cand = reinterpret_cast<Cand *>(scratch);
        if ((rc = launch_screen(db, nrows, qp, M, cand, st))) return rc;
        if (ev1) IA_HIP(hipEventRecord(ev1, st));
        return launch_merge(src, row0, nrows, cand, M, q64, nq, amax, best, stats, st);
    }
    const SegWs ws = seg_ws(scratch, M, nrows);
    float *segmin = ws.segmin;
    const int nq_cap = (screen_variant() >> 4) & 15;
    const bool split = match_alg() == 2;
    // f32: up to 3 query tiles per wave (profiles/r01_screen_bench_split.txt); split f16:
    // the shape rule of launch_screen16
    const int cap = nq_cap > 0 && nq_cap <= 3 ? nq_cap : 3;
    if ((rc = launch_screen_seg(db, nrows, qp, M, segmin, split ? 0 : cap, st,
                                split ? q16 : nullptr)))
        return rc;
    if (ev1) IA_HIP(hipEventRecord(ev1, st));
    const FinishArgs fa = fin ? *fin : FinishArgs{};
    const int rm = rescore_mode();
    // default: the work list for levels above 2^20 rows (where k_rescore's per-query
    // serialisation costs most); k_rescore below, with or without the fused tail (a
    // sharded rank's 0.5 M-row shard: 13.9 vs 19.9 us per wave, profiles/r01_shard_sim_g8.txt)
    if (rm == 1 || (rm < 0 && nrows > (1L << 20))) {
        const long nseg = db_nsegs(nrows);
        if (split)
            k_select<true><<<M, 256, 0, st>>>(nseg, segmin, nq, amax, ws.ctr, ws.items, ws.sel, stats);
        else
            k_select<false><<<M, 256, 0, st>>>(nseg, segmin, nq, amax, ws.ctr, ws.items, ws.sel, stats);
        IA_LAUNCH_CHECK("k_select");
        const int grid = 2 * M + 64;
        k_items<<<grid, 256, 0, st>>>(src, row0, nrows, db_seg_rows(nrows), ws.items, ws.ctr, db, qp,
                                      q64, ws.ibest, stats);
        IA_LAUNCH_CHECK("k_items");
        if (fin)
            k_gather<true><<<M, 128, 0, st>>>(src, ws.sel, ws.ibest, ws.ctr, best, fa, q64);
        else
            k_gather<false><<<M, 64, 0, st>>>(src, ws.sel, ws.ibest, ws.ctr, best, fa, q64);
        IA_LAUNCH_CHECK("k_gather");
        return IA_OK;
    }
    static const int probe = env_int("IA_PRUNE_PROBE", 0);
#define IA_RESCORE(F, SP)                                                                      \
    k_rescore<F, SP><<<M, 256, 0, st>>>(src, row0, nrows, db_nsegs(nrows), db_seg_rows(nrows), \
                                        segmin, db, qp, q64, nq, amax, best, stats, fa, probe)
    if (fin && split) IA_RESCORE(true, true);
    else if (fin) IA_RESCORE(true, false);
    else if (split) IA_RESCORE(false, true);
    else IA_RESCORE(false, false);
#undef IA_RESCORE
    IA_LAUNCH_CHECK("k_rescore");
    return IA_OK;
}

__global__ void k_split_best(const Best *b, int M, int64_t *idx, double *dist) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= M) return;
    if (idx) idx[i] = b[i].idx;
    if (dist) dist[i] = b[i].d;
}

// ---------------------------------------------------------------------------------
// per-pixel API helpers (algorithms.py:92-135)
// ---------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_coherence_pick(const double *rows, int n,
                                                       const double *q, int32_t *out) {
    double bd = INFINITY;
    long long bi = 0x7fffffffffffffffLL;
    for (int i = threadIdx.x; i < n; i += 64) {
        Pw55 pw;
#pragma unroll
        for (int k = 0; k < IA_D; ++k) {
            const double x = rows[(long)i * IA_D + k] - q[k];
            pw.feed(k, x * x);
        }
        best_update(bd, bi, sqrt(pw.res), i);
    }
    for (int o = 32; o > 0; o >>= 1) {
        const double od = __shfl_xor(bd, o);
        const long long oi = __shfl_xor(bi, o);
        best_update(bd, bi, od, oi);
    }
    if (threadIdx.x == 0) out[0] = (int32_t)bi;
}

__global__ void k_wdist(const double *a, const double *q, const double *w, int n,
                        double *out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Pw55 pw;
#pragma unroll
    for (int k = 0; k < IA_D; ++k) {
        const double x = (a[(long)i * IA_D + k] - q[(long)i * IA_D + k]) * w[k];
        pw.feed(k, x * x);
    }
    const double s = sqrt(pw.res);
    out[i] = s * s;
}

}  // namespace ia

using namespace ia;

extern "C" {

static constexpr int MATCH_BATCH = 384;

size_t ia_match_workspace_bytes(int M, long nrows) {
    const int mb = M < MATCH_BATCH ? M : MATCH_BATCH;
    const int qr = qrows_alloc(mb);
    size_t b = 0;
    b += align_up((size_t)qr * IA_DP * sizeof(float), 256);                        // qp
    b += align_up((size_t)qr * Q16_ROW * sizeof(half8), 256);                      // q16
    b += align_up((size_t)qr * sizeof(double), 256);                               // nq
    b += align_up(match_scratch_bytes(qr, nrows), 256);                           // screen out
    b += align_up((size_t)qr * sizeof(Best), 256);                                 // best
    return b;
}

int ia_match_batch(const IaMatchArgs *a, void *stream) {
    IA_ARG(a && a->db && a->q64 && a->center && a->amax && a->workspace && a->M >= 0 &&
               a->nrows > 0,
           "ia_match_batch: bad args");
    if (a->M == 0) return IA_OK;
    hipStream_t st = S(stream);
    const int mb = a->M < MATCH_BATCH ? a->M : MATCH_BATCH;
    const int qr = qrows_alloc(mb);
    char *w = reinterpret_cast<char *>(a->workspace);
    float *qp = reinterpret_cast<float *>(w);
    w += align_up((size_t)qr * IA_DP * sizeof(float), 256);
    _Float16 *q16 = reinterpret_cast<_Float16 *>(w);
    w += align_up((size_t)qr * Q16_ROW * sizeof(half8), 256);
    double *nq = reinterpret_cast<double *>(w);
    w += align_up((size_t)qr * sizeof(double), 256);
    void *scratch = w;
    w += align_up(match_scratch_bytes(qr, a->nrows), 256);
    Best *best = reinterpret_cast<Best *>(w);
    IA_HIP(hipMemsetAsync(qp, 0, (size_t)qr * IA_DP * sizeof(float), st));
    IA_HIP(hipMemsetAsync(q16, 0, (size_t)qr * Q16_ROW * sizeof(half8), st));
    IA_HIP(hipMemsetAsync(scratch, 0, WL_HEAD, st));   // empty work list
    const DbSrc src = make_dbsrc(a->src);
    for (int m0 = 0; m0 < a->M; m0 += MATCH_BATCH) {
        const int M = a->M - m0 < MATCH_BATCH ? a->M - m0 : MATCH_BATCH;
        const double *q = a->q64 + (long)m0 * IA_DP;
        int rc;
        if (a->lsh) {
            if ((rc = launch_lsh_match(a->lsh, src, a->row0, a->nrows, M, q, a->center, best,
                                       nullptr, st)))
                return rc;
        } else {
            if ((rc = launch_query_rows(q, M, a->center, qp, nq, a->amax, q16, st))) return rc;
            if ((rc = launch_match(src, a->row0, a->nrows, a->db, qp, q16, M, q, nq, a->amax,
                                   scratch, best, nullptr, st)))
                return rc;
        }
        k_split_best<<<(M + 255) / 256, 256, 0, st>>>(best, M, a->idx ? a->idx + m0 : nullptr,
                                                      a->dist ? a->dist + m0 : nullptr);
        IA_LAUNCH_CHECK("k_split_best");
    }
    return IA_OK;
}

int ia_coherence_pick(const double *rows, int n, const double *q, int32_t *out, void *stream) {
    IA_ARG(rows && q && out && n > 0, "ia_coherence_pick: bad args");
    k_coherence_pick<<<1, 64, 0, S(stream)>>>(rows, n, q, out);
    IA_LAUNCH_CHECK("k_coherence_pick");
    return IA_OK;
}

int ia_wdist_batch(const double *a, const double *q, const double *w, int n, double *out,
                   void *stream) {
    IA_ARG(a && q && w && out && n >= 0, "ia_wdist_batch: bad args");
    if (n == 0) return IA_OK;
    k_wdist<<<(n + 63) / 64, 64, 0, S(stream)>>>(a, q, w, n, out);
    IA_LAUNCH_CHECK("k_wdist");
    return IA_OK;
}

}  // extern "C"

// ---- diagnostic entry points (include/ia_diag.h) ----------------------------------
#include "../../include/ia_diag.h"

extern "C" {

size_t ia_diag_cand_bytes(int M, long nrows) { return match_scratch_bytes(qrows_alloc(M), nrows); }

int ia_diag_qp_rows(int M) { return qrows_alloc(M); }

int ia_diag_query_rows(const double *q64, int M, const double *center, float *qp, double *nq,
                       void *stream) {
    IA_ARG(q64 && center && qp && nq && M > 0, "ia_diag_query_rows: bad args");
    return launch_query_rows(q64, M, center, qp, nq, nullptr, nullptr, S(stream));
}

int ia_diag_query_rows16(const double *q64, int M, const double *center, const float *amax,
                         float *qp, void *q16, double *nq, void *stream) {
    IA_ARG(q64 && center && amax && qp && q16 && nq && M > 0, "ia_diag_query_rows16: bad args");
    return launch_query_rows(q64, M, center, qp, nq, amax, reinterpret_cast<_Float16 *>(q16),
                             S(stream));
}

int ia_diag_set_match_alg(int alg) {
    const int prev = match_alg();
    if (alg >= 0 && alg <= 2) g_match_alg.store(alg);
    return prev;
}

int ia_diag_set_rescore_mode(int mode) {
    const int prev = rescore_mode();
    if (mode >= -1 && mode <= 1) g_rescore_mode.store(mode);
    return prev;
}

int ia_diag_screen16(const float *db, long nrows, const void *q16, int M, float *segmin,
                     int maxnq, void *stream) {
    IA_ARG(db && q16 && segmin && M > 0 && nrows > 0, "ia_diag_screen16: bad args");
    return launch_screen16(db, nrows, reinterpret_cast<const _Float16 *>(q16), M, segmin, maxnq,
                           S(stream));
}

int ia_diag_screen(const float *db, long nrows, const float *qp, int M, void *cand, int variant,
                   void *stream) {
    IA_ARG(db && qp && cand && M > 0 && nrows > 0 && (variant & 15) <= 6,
           "ia_diag_screen: bad args");
    if ((variant & 15) == 6) {   // segment-minimum screen (the default matcher's stage 1)
        const int cap = (variant >> 4) & 15;
        const int uniform = variant & 0x100;   // bit 8: pad to whole query groups
        return launch_screen_seg(db, nrows, qp, M, reinterpret_cast<float *>(cand),
                                 (cap > 0 && cap <= 3 ? cap : 3) | uniform, S(stream));
    }
    return launch_screen_v(db, nrows, qp, M, reinterpret_cast<Cand *>(cand), variant, S(stream));
}

}  // extern "C"

#ifdef IA_PROBE
// diagnostic: route the phase marks to buf (device, 64 x 4 x 16 uint64) or disable (NULL)
extern "C" int ia_probe_set(unsigned long long *buf) {
    IA_HIP(hipMemcpyToSymbol(HIP_SYMBOL(ia::g_probe), &buf, sizeof(buf)));
    return IA_OK;
}
#endif
