// ia_screen16.hip — the split-f16 segment screen (IA_MATCH_ALG=2, default).
//
// Stage 1 of the exact matcher (ia_match.hip): for every (query, DB segment of <= 512
// rows) the minimum of the screen value sa * sq_j * (|a'|^2 - 2 a'.q'), computed as 11
// v_mfma_f32_32x32x16_f16 per 32x32 (rows x queries) tile from the split-f16 operands of
// ia_split16.h.  Queries are the stationary operand (VGPRs), DB rows stream through.
// Padding rows of the DB's last chunk repeat its last real row (k_db_split), so the
// minima need no masking.  Built with -fno-honor-nans (the min-reductions need no NaN
// canonicalisation: inputs are finite by construction) and -amdgpu-mfma-vgpr-form (MFMA
// results in VGPRs: the reductions read them without v_accvgpr_read copies).
//
// Two forms:
//  * k_screen_h16 (per-wave): each wave streams its own quarter of a chunk straight into
//    VGPRs (fragment-major DB: one contiguous 1 KiB per load instruction).
//  * k_screen_h16s (shared, default): the block's 4 waves are WR row parts x WQ query
//    parts; 4-tile stages (28 KiB) are copied global -> LDS by global_load_lds_dwordx4 and
//    read back with ds_read_b128, so each DB byte from L2 feeds WQ waves.  PIPE: two
//    accumulator sets, the min-reduction of tile t runs beside the MFMAs of tile t+1.
#include "ia_internal.h"
#include "ia_split16.h"

#include <float.h>

namespace ia {

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int TILE_H8 = DB16_GROUPS * 64;            // half8 per 32-row tile (7 KiB)
constexpr int STAGE_TILES = 4;
constexpr int STAGE_H8 = STAGE_TILES * TILE_H8;      // 28 KiB

// 11 MFMAs of one 32-row tile against NQ query tiles (the first with a zero C operand)
template <int NQ>
__device__ __forceinline__ void tile_mfma(const half8 (&a)[DB16_GROUPS],
                                          const half8 (&bq)[NQ][Q16_GROUPS],
                                          floatx16 (&acc)[NQ]) {
    const floatx16 zero = {};
#pragma unroll
    for (int qt = 0; qt < NQ; ++qt)
        acc[qt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[0], bq[qt][0], zero, 0, 0, 0);
#pragma unroll
    for (int m = 1; m < Q16_GROUPS; ++m)
#pragma unroll
        for (int qt = 0; qt < NQ; ++qt)
            acc[qt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[m < 7 ? m : m - 7], bq[qt][m],
                                                             acc[qt], 0, 0, 0);
}

// running minimum over a tile: 8 v_min3_f32 per query tile, dependency depth 3
template <int NQ>
__device__ __forceinline__ void tile_min(const floatx16 (&acc)[NQ], float (&mn)[NQ]) {
#pragma unroll
    for (int qt = 0; qt < NQ; ++qt) {
        const floatx16 &x = acc[qt];
        const float t0 = fminf(fminf(x[0], x[1]), x[2]), t1 = fminf(fminf(x[3], x[4]), x[5]);
        const float t2 = fminf(fminf(x[6], x[7]), x[8]), t3 = fminf(fminf(x[9], x[10]), x[11]);
        const float t4 = fminf(fminf(x[12], x[13]), x[14]);
        const float u0 = fminf(fminf(t0, t1), t2), u1 = fminf(fminf(t3, t4), x[15]);
        mn[qt] = fminf(fminf(mn[qt], u0), u1);
    }
}

// end of a segment: the two lane halves hold different rows of the same queries
template <int NQ>
__device__ __forceinline__ void seg_flush(float (&mn)[NQ], int tile0, int j, int h, int M,
                                          float *__restrict__ segmin, long nseg, long seg) {
#pragma unroll
    for (int qt = 0; qt < NQ; ++qt) {
        const float m = fminf(mn[qt], __shfl_xor(mn[qt], 32));
        const int qg = (tile0 + qt) * 32 + j;
        if (h == 0 && qg < M) segmin[(long)qg * nseg + seg] = m;
        mn[qt] = FLT_MAX;
    }
}

template <int NQ>
__device__ __forceinline__ void load_queries(half8 (&bq)[NQ][Q16_GROUPS],
                                             const half8 *__restrict__ q16, int tile0, int j,
                                             int h) {
#pragma unroll
    for (int qt = 0; qt < NQ; ++qt) {
        const half8 *p = q16 + (long)((tile0 + qt) * 32 + j) * Q16_ROW + h * Q16_GROUPS;
#pragma unroll
        for (int m = 0; m < Q16_GROUPS; ++m) bq[qt][m] = p[m];
    }
}

// ---------------------------------------------------------------------------------
// per-wave form
// ---------------------------------------------------------------------------------
template <int NQ>
__device__ __forceinline__ void wave_body(const half8 *__restrict__ db16, int chunk, int ch,
                                          int seg_rows, const half8 *__restrict__ q16, int M,
                                          int tile0, float *__restrict__ segmin, long nseg) {
    const int tid = threadIdx.x;
    const int lane = tid & 63, wv = tid >> 6;
    const int j = lane & 31, h = lane >> 5;
    half8 bq[NQ][Q16_GROUPS];
    load_queries<NQ>(bq, q16, tile0, j, h);
    const int rows_per_wave = ch >> 2;
    const int ntile = rows_per_wave >> 5;
    const int tps = seg_rows >> 5;
    const long row_begin = (long)chunk * ch + wv * rows_per_wave;
    const long seg_begin = row_begin / seg_rows;
    const half8 *dp = db16 + (row_begin >> 5) * TILE_H8 + lane;
    float mn[NQ];
#pragma unroll
    for (int qt = 0; qt < NQ; ++qt) mn[qt] = FLT_MAX;
    auto load = [&](half8 (&a)[DB16_GROUPS], int tile) {
#pragma unroll
        for (int g = 0; g < DB16_GROUPS; ++g) a[g] = dp[(long)tile * TILE_H8 + g * 64];
    };
    auto step = [&](const half8 (&a)[DB16_GROUPS], int tile) {
        floatx16 acc[NQ];
        tile_mfma<NQ>(a, bq, acc);
        tile_min<NQ>(acc, mn);
        if ((tile + 1) % tps == 0) seg_flush<NQ>(mn, tile0, j, h, M, segmin, nseg, seg_begin + tile / tps);
    };
    half8 b0[DB16_GROUPS], b1[DB16_GROUPS];
    load(b0, 0);
    int tile = 0;
    for (; tile + 1 < ntile; tile += 2) {
        load(b1, tile + 1);
        step(b0, tile);
        load(b0, tile + 2 < ntile ? tile + 2 : ntile - 1);
        step(b1, tile + 1);
    }
    if (tile < ntile) step(b0, tile);
}

// grid: nchunks (rounded up to 8) x groups of NQ query tiles, XCD-aware (all groups of a
// chunk share blockIdx % 8, so the chunk is fetched from HBM once per launch)
template <int NQ>
__global__ __launch_bounds__(256) void k_screen_h16(const half8 *__restrict__ db16, int nchunks,
                                                    int ch, int seg_rows,
                                                    const half8 *__restrict__ q16, int M,
                                                    int groups, float *__restrict__ segmin,
                                                    long nseg) {
    const int b = blockIdx.x;
    const int slot = b >> 3;
    const int chunk = (slot / groups) * 8 + (b & 7);
    const int group = slot - (slot / groups) * groups;
    if (chunk >= nchunks) return;
    wave_body<NQ>(db16, chunk, ch, seg_rows, q16, M, group * NQ, segmin, nseg);
}

// ---------------------------------------------------------------------------------
// shared-tile form
// ---------------------------------------------------------------------------------
template <int NQ, int WQ, bool PIPE>
__global__ __launch_bounds__(256) void k_screen_h16s(const half8 *__restrict__ db16, int nchunks,
                                                     int ch, int seg_rows,
                                                     const half8 *__restrict__ q16, int M,
                                                     int groups, float *__restrict__ segmin,
                                                     long nseg) {
    constexpr int WR = 4 / WQ;
    constexpr int TPW = STAGE_TILES / WR;      // tiles per wave per stage (4, 2 or 1)
    static_assert(!PIPE || TPW % 2 == 0, "pipelined epilogue needs an even tile count");
    __shared__ half8 sbuf[2][STAGE_H8];
    const int b = blockIdx.x;
    const int slot = b >> 3;
    const int chunk = (slot / groups) * 8 + (b & 7);
    const int group = slot - (slot / groups) * groups;
    if (chunk >= nchunks) return;   // uniform over the block, before any barrier
    const int tid = threadIdx.x;
    const int lane = tid & 63, wv = tid >> 6;
    const int j = lane & 31, h = lane >> 5;
    const int wr = wv / WQ, wq = wv - (wv / WQ) * WQ;
    const int tile0 = (group * WQ + wq) * NQ;

    half8 bq[NQ][Q16_GROUPS];
    load_queries<NQ>(bq, q16, tile0, j, h);
    const int tpc = ch >> 5;                   // tiles per chunk (a multiple of 4)
    const int tpp = tpc / WR;                  // tiles per row part
    const int tps = seg_rows >> 5;             // tiles per segment (divides tpp)
    const int nstage = tpc / STAGE_TILES;
    const long ctile0 = (long)chunk * tpc;
    const long seg0 = (ctile0 + (long)wr * tpp) * 32 / seg_rows;

    // stage s holds virtual tiles 4s..4s+3; virtual tile v = part v % WR, index v / WR
    auto issue = [&](int s, int buf) {
#pragma unroll
        for (int k = 0; k < DB16_GROUPS; ++k) {
            const int idx = k * 256 + tid;
            const int tt = idx / TILE_H8, rem = idx - tt * TILE_H8;
            const int v = s * STAGE_TILES + tt;
            const long gt = ctile0 + (long)(v % WR) * tpp + v / WR;
            __builtin_amdgcn_global_load_lds((const void *)(db16 + gt * TILE_H8 + rem),
                                             (void *)&sbuf[buf][k * 256 + wv * 64], 16, 0, 0);
        }
    };
    auto read_tile = [&](half8 (&a)[DB16_GROUPS], const half8 *sb, int u) {
        const half8 *p = sb + (u * WR + wr) * TILE_H8 + lane;
#pragma unroll
        for (int g = 0; g < DB16_GROUPS; ++g) a[g] = p[g * 64];
    };

    float mn[NQ];
#pragma unroll
    for (int qt = 0; qt < NQ; ++qt) mn[qt] = FLT_MAX;
    auto close = [&](int i) {   // after tile i (index within the part) is folded into mn
        if ((i + 1) % tps == 0) seg_flush<NQ>(mn, tile0, j, h, M, segmin, nseg, seg0 + i / tps);
    };

    issue(0, 0);
    __syncthreads();
    if (!PIPE) {
        for (int s = 0; s < nstage; ++s) {
            if (s + 1 < nstage) issue(s + 1, (s + 1) & 1);
            const half8 *sb = sbuf[s & 1];
#pragma unroll
            for (int u = 0; u < TPW; ++u) {
                half8 a[DB16_GROUPS];
                read_tile(a, sb, u);
                floatx16 acc[NQ];
                tile_mfma<NQ>(a, bq, acc);
                tile_min<NQ>(acc, mn);
                close(s * TPW + u);
            }
            __syncthreads();   // stage s+1 landed (vmcnt(0)) and stage s is free again
        }
        return;
    }
    floatx16 accX[NQ], accY[NQ];   // tile pairs: X = even, Y = odd tile of the wave
    for (int s = 0; s < nstage; ++s) {
        if (s + 1 < nstage) issue(s + 1, (s + 1) & 1);
        const half8 *sb = sbuf[s & 1];
#pragma unroll
        for (int u = 0; u < TPW; u += 2) {
            const int i = s * TPW + u;
            half8 a[DB16_GROUPS];
            read_tile(a, sb, u);
            tile_mfma<NQ>(a, bq, accX);
            if (i > 0) {              // the previous pair's odd tile, beside these MFMAs
                tile_min<NQ>(accY, mn);
                close(i - 1);
            }
            read_tile(a, sb, u + 1);
            tile_mfma<NQ>(a, bq, accY);
            tile_min<NQ>(accX, mn);
            close(i);
        }
        __syncthreads();
    }
    tile_min<NQ>(accY, mn);
    close(nstage * TPW - 1);
}

static int h16_shared() {
    static int v = -1;
    if (v < 0) {
        const char *e = getenv("IA_H16S");   // 0: per-wave form
        v = e ? atoi(e) : 1;
    }
    return v;
}

int launch_screen16(const float *db, long nrows, const _Float16 *q16, int M, float *segmin,
                    int flags, hipStream_t st) {
    const int ch = db_chunk_rows(nrows);
    const long nchunks = db_nchunks(nrows);
    const int seg_rows = db_seg_rows(nrows);
    const long nseg = db_nsegs(nrows);
    const half8 *db16 = reinterpret_cast<const half8 *>(db16_of(db, nrows));
    const half8 *q = reinterpret_cast<const half8 *>(q16);
    const int T = (M + 31) / 32;
    const int cap = flags & 15;
    bool pipe = !(flags & 0x200);
    if (h16_shared() && !(flags & 0x100) && T >= 2) {
        // query tiles per block WQ x NQ: T >= 9 -> 4 x 3, 5..8 -> 4 x 2, 3..4 -> 4 x 1,
        // 2 -> 2 x 1 (fewest padded tiles, then the most sharing)
        int wq = 4, nq = T >= 9 ? 3 : (T >= 5 ? 2 : 1);
        if (T == 2) wq = 2;
        if (cap > 0 && cap < nq) nq = cap;
        // the pipelined epilogue's second accumulator set costs NQ = 3 its second wave per
        // SIMD (measured slower: profiles/r01_screen_bench_h16s.txt)
        if (nq == 3) pipe = false;
        const int g = (T + wq * nq - 1) / (wq * nq);
        const long nb = ((nchunks + 7) / 8) * 8 * g;
        IA_ARG(nb < (1L << 31), "screen grid too large");
        IA_ARG(g * wq * nq <= T + 2 * MAX_NQ, "screen: query tiles exceed the padded rows");
#define IA_H16S_CASE(NQ, WQ, P)                                                                 \
        if (nq == NQ && wq == WQ && pipe == P) {                                                \
            k_screen_h16s<NQ, WQ, P><<<(unsigned)nb, 256, 0, st>>>(db16, (int)nchunks, ch,      \
                                                                   seg_rows, q, M, g, segmin,   \
                                                                   nseg);                       \
            IA_LAUNCH_CHECK("k_screen_h16s");                                                   \
            return IA_OK;                                                                       \
        }
        IA_H16S_CASE(2, 4, true)
        IA_H16S_CASE(1, 4, true)
        IA_H16S_CASE(1, 2, true)
        IA_H16S_CASE(3, 4, false)
        IA_H16S_CASE(2, 4, false)
        IA_H16S_CASE(1, 4, false)
        IA_H16S_CASE(1, 2, false)
#undef IA_H16S_CASE
        set_error("launch_screen16: bad shared split");
        return IA_E_ARG;
    }
    // per-wave form: groups of nq <= 2 tiles (2 waves per SIMD; cap 3 for A/B)
    int nq = T < 2 ? T : 2;
    if (cap > 0) nq = cap < T ? cap : T;
    if (nq > 3) nq = 3;
    const int g = (T + nq - 1) / nq;
    const long nb = ((nchunks + 7) / 8) * 8 * g;
    IA_ARG(nb < (1L << 31), "screen grid too large");
    IA_ARG(g * nq <= T + 2 * MAX_NQ, "screen: query tiles exceed the padded rows");
#define IA_H16_CASE(NQ)                                                                          \
    if (nq == NQ) {                                                                              \
        k_screen_h16<NQ><<<(unsigned)nb, 256, 0, st>>>(db16, (int)nchunks, ch, seg_rows, q, M,  \
                                                       g, segmin, nseg);                         \
        IA_LAUNCH_CHECK("k_screen_h16");                                                         \
        return IA_OK;                                                                            \
    }
    IA_H16_CASE(1)
    IA_H16_CASE(2)
    IA_H16_CASE(3)
#undef IA_H16_CASE
    set_error("launch_screen16: bad split");
    return IA_E_ARG;
}

}  // namespace ia
