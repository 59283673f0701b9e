// ia_screen16.hip — the split-f16 segment screen (IA_MATCH_ALG=2, default).
//
// Stage 1 of the exact matcher (ia_match.hip): for every (query, DB segment of <= 512
// rows) the minimum of the screen value sa * sq_j * (|a'|^2 - 2 a'.q'), computed as 11
// v_mfma_f32_32x32x16_f16 per 32x32 (rows x queries) tile from the split-f16 operands of
// ia_split16.h (7 DB and 8 query register groups per lane).  Queries are the stationary operand (VGPRs), DB rows stream through.
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
#include <cstdlib>
#include <type_traits>

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
    for (int m = 1; m < MFMA16; ++m)
#pragma unroll
        for (int qt = 0; qt < NQ; ++qt)
            acc[qt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[mfma_a(m)], bq[qt][mfma_b(m)],
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
// MODE 0: plain; 1: pipelined epilogue (two accumulator sets); 3: double-buffered fragment
// registers (below); 2: fragment prefetch (the
// next tile's LDS groups re-read into each register group right after its last MFMA use,
// barrier at the start of each stage's last tile, two stages of global_load_lds in flight)
template <int NQ, int WQ, int MODE, bool NT = false>
__global__ __launch_bounds__(256, 2) void k_screen_h16s(const half8 *__restrict__ db16, int nchunks,
                                                     int ch, int seg_rows,
                                                     const half8 *__restrict__ q16, int M,
                                                     int groups, float *__restrict__ segmin,
                                                     long nseg) {
    constexpr int WR = 4 / WQ;
    constexpr int TPW = STAGE_TILES / WR;      // tiles per wave per stage (4, 2 or 1)
    static_assert(MODE != 1 || TPW % 2 == 0, "pipelined epilogue needs an even tile count");
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
                                             (void *)&sbuf[buf][k * 256 + wv * 64], 16, 0, NT ? 2 : 0);
        }
    };
    // every wave's global_load_lds of the next stage retired, then the barrier: the
    // compiler's own wait before __syncthreads() is not reliable here (hipcc 7.2 dropped it
    // in the loop of MODE 2, letting waves read a stage before it landed)
    auto stage_barrier = [&]() {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
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
    if (MODE == 3) {
        // double-buffered fragments: tile i+1's ds_reads go into the other register set
        // before tile i's MFMAs, so no tile starts on an LDS round trip; the barrier sits at
        // the start of each stage's last tile (stage s+1 landed, stage s fully read), after
        // which stage s+2's copies and the reads of stage s+1's first tile are issued
        static_assert(TPW % 2 == 0, "register double buffering needs an even tile count");
        half8 ra[DB16_GROUPS], rb[DB16_GROUPS];
        if (nstage > 1) issue(1, 1);
        stage_barrier();
        read_tile(ra, sbuf[0], 0);
        for (int s = 0; s < nstage; ++s) {
            const half8 *sb = sbuf[s & 1];
#pragma unroll
            for (int u = 0; u < TPW; ++u) {
                half8 (&cur)[DB16_GROUPS] = (u & 1) ? rb : ra;
                half8 (&nxt)[DB16_GROUPS] = (u & 1) ? ra : rb;
                if (u + 1 < TPW) {
                    read_tile(nxt, sb, u + 1);
                } else {
                    stage_barrier();
                    if (s + 2 < nstage) issue(s + 2, s & 1);
                    if (s + 1 < nstage) read_tile(nxt, sbuf[(s + 1) & 1], 0);
                }
                floatx16 acc[NQ];
                tile_mfma<NQ>(cur, bq, acc);
                tile_min<NQ>(acc, mn);
                close(s * TPW + u);
            }
        }
        return;
    }
    if (MODE == 2) {
        if (nstage > 1) issue(1, 1);
        stage_barrier();
        half8 a[DB16_GROUPS];
        read_tile(a, sbuf[0], 0);
        const floatx16 zero = {};
        for (int s = 0; s < nstage; ++s) {
            const half8 *sb = sbuf[s & 1];
#pragma unroll
            for (int u = 0; u < TPW; ++u) {
                const half8 *np;      // where the next tile's groups come from
                if (u + 1 < TPW) {
                    np = sb + ((u + 1) * WR + wr) * TILE_H8 + lane;
                } else {
                    // stage s+1 landed and every wave is done reading stage s-1's buffer
                    stage_barrier();
                    if (s + 2 < nstage) issue(s + 2, s & 1);
                    np = (s + 1 < nstage ? sbuf[(s + 1) & 1] + wr * TILE_H8 : sb) + lane;
                }
                floatx16 acc[NQ];
#pragma unroll
                for (int qt = 0; qt < NQ; ++qt)
                    acc[qt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[0], bq[qt][0], zero, 0, 0, 0);
#pragma unroll
                for (int m = 1; m < MFMA16; ++m) {
                    const int g = mfma_a(m);
#pragma unroll
                    for (int qt = 0; qt < NQ; ++qt)
                        acc[qt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[g], bq[qt][mfma_b(m)],
                                                                         acc[qt], 0, 0, 0);
                    if (m >= 4) a[g] = np[g * 64];   // last use of group g in this tile
                }
                tile_min<NQ>(acc, mn);
                close(s * TPW + u);
            }
        }
        return;
    }
    stage_barrier();
    if (MODE == 0) {
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
            stage_barrier();   // stage s+1 landed and stage s is free again
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
        stage_barrier();
    }
    tile_min<NQ>(accY, mn);
    close(nstage * TPW - 1);
}

// ---------------------------------------------------------------------------------
// spanning form (flag 0x1000): 512 threads = 2 row parts x 4 query parts, three stage
// buffers (84 KiB, one array).  Stage s+2 is copied while stage s is computed, and the
// barrier before stage s+1 waits only for stage s+1's copies: a counted vmcnt (loads retire
// in order, so later stores only make the wait stricter) and a raw s_barrier, since
// __syncthreads()' fence would also drain the copies still in flight
// (cdna_hip_programming.md, "Pipelining across barriers").  MODE 1 / 2 (diagnostics, flags
// 0x2000 / 0x8000): stage 0 only is copied and every stage re-reads it, with / without the
// per-stage barriers — the ceiling of the same instruction stream.
// ---------------------------------------------------------------------------------
constexpr int SPAN_WAVES = 8;
constexpr int SPAN_LOADS = STAGE_TILES * DB16_GROUPS;     // 1 KiB wave-loads per stage (28)

template <int NQ, int MODE>
__global__ __launch_bounds__(512) void k_screen_h16p(const half8 *__restrict__ db16, int nchunks,
                                                     int ch, int seg_rows,
                                                     const half8 *__restrict__ q16, int M,
                                                     int groups, float *__restrict__ segmin,
                                                     long nseg) {
    constexpr bool DRY = MODE != 0;
    constexpr int WQ = 4, WR = 2, TPW = STAGE_TILES / WR;
    __shared__ half8 sbuf[3 * STAGE_H8];
    const int b = blockIdx.x;
    const int slot = b >> 3;
    const int chunk = (slot / groups) * 8 + (b & 7);
    const int group = slot - (slot / groups) * groups;
    if (chunk >= nchunks) return;   // uniform over the block, before any barrier
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int j = lane & 31, h = lane >> 5;
    const int wr = wv >> 2, wq = wv & 3;
    const int tile0 = (group * WQ + wq) * NQ;

    half8 bq[NQ][Q16_GROUPS];
    load_queries<NQ>(bq, q16, tile0, j, h);
    const int tpc = ch >> 5;
    const int tpp = tpc / WR;
    const int tps = seg_rows >> 5;
    const int nstage = tpc / STAGE_TILES;
    const long ctile0 = (long)chunk * tpc;
    const long seg0 = (ctile0 + (long)wr * tpp) * 32 / seg_rows;

    // wave-load k (0..27) of stage s: group k % 7 of virtual tile k / 7 (part v % WR,
    // index v / WR); waves 0-3 issue 4 loads per stage, waves 4-7 issue 3
    auto issue = [&](int s, int buf) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int k = wv + i * SPAN_WAVES;
            if (k < SPAN_LOADS) {
                const int tt = k / DB16_GROUPS, g = k - tt * DB16_GROUPS;
                const int v = s * STAGE_TILES + tt;
                const long gt = ctile0 + (long)(v % WR) * tpp + v / WR;
                __builtin_amdgcn_global_load_lds((const void *)(db16 + gt * TILE_H8 + g * 64 + lane),
                                                 (void *)(sbuf + buf * STAGE_H8 + k * 64), 16, 0,
                                                 0);
            }
        }
    };
    // this wave's copies of the next stage retired (ahead: the next-but-one stage's copies,
    // issued later, may still be in flight)
    auto wait_stage = [&](bool ahead) {
        if (!ahead) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else if (wv < SPAN_LOADS - 3 * SPAN_WAVES) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
    };
    auto barrier = [&]() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };

    float mn[NQ];
#pragma unroll
    for (int qt = 0; qt < NQ; ++qt) mn[qt] = FLT_MAX;
    issue(0, 0);
    if (!DRY && nstage > 1) issue(1, 1);
    wait_stage(!DRY && nstage > 1);
    barrier();
    int buf = 0;
    for (int s = 0; s < nstage; ++s) {
        if (!DRY && s + 2 < nstage) issue(s + 2, buf == 0 ? 2 : buf - 1);
        const half8 *sb = sbuf + buf * STAGE_H8;
#pragma unroll
        for (int u = 0; u < TPW; ++u) {
            half8 a[DB16_GROUPS];
            const half8 *p = sb + (u * WR + wr) * TILE_H8 + lane;
#pragma unroll
            for (int g = 0; g < DB16_GROUPS; ++g) a[g] = p[g * 64];
            floatx16 acc[NQ];
            tile_mfma<NQ>(a, bq, acc);
            tile_min<NQ>(acc, mn);
            const int i = s * TPW + u;
            if ((i + 1) % tps == 0) seg_flush<NQ>(mn, tile0, j, h, M, segmin, nseg, seg0 + i / tps);
        }
        if (MODE != 2) {
            wait_stage(!DRY && s + 2 < nstage);
            barrier();
        }
        if (!DRY) buf = buf == 2 ? 0 : buf + 1;
    }
}

// ---------------------------------------------------------------------------------
// uneven-share form (flag 0x4000): a block's G (4..12) query tiles are split over its 4
// waves as evenly as possible (G = 11: 3 + 3 + 3 + 2; G = 6: 2 + 2 + 1 + 1) instead of
// padding every wave to the same count (M = 342: 11 tiles computed, not 12); which wave
// takes a short share rotates from block to block, so that the SIMDs of a CU (one wave
// of each resident block) carry equal work on average.  Each wave runs the plain stage
// loop at its own tile count; every wave copies its part of each stage and meets every
// barrier.
// ---------------------------------------------------------------------------------
template <int NQ>
__device__ __forceinline__ void uneven_body(const half8 *__restrict__ db16, half8 *sbuf,
                                            long ctile0, int nstage, int tps, long seg0,
                                            const half8 *__restrict__ q16, int M, int tile0,
                                            float *__restrict__ segmin, long nseg) {
    const int tid = threadIdx.x;
    const int lane = tid & 63, wv = tid >> 6;
    const int j = lane & 31, h = lane >> 5;
    half8 bq[NQ][Q16_GROUPS];
    load_queries<NQ>(bq, q16, tile0, j, h);
    // one row part: stage s = the 4 consecutive tiles 4s..4s+3, one contiguous 28 KiB
    auto issue = [&](int s, int buf) {
        const half8 *src = db16 + (ctile0 + (long)s * STAGE_TILES) * TILE_H8 + tid;
#pragma unroll
        for (int k = 0; k < DB16_GROUPS; ++k)
            __builtin_amdgcn_global_load_lds((const void *)(src + k * 256),
                                             (void *)(sbuf + buf * STAGE_H8 + k * 256 + wv * 64),
                                             16, 0, 0);
    };
    auto stage_barrier = [&]() {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    };
    float mn[NQ];
#pragma unroll
    for (int qt = 0; qt < NQ; ++qt) mn[qt] = FLT_MAX;
    issue(0, 0);
    stage_barrier();
    for (int s = 0; s < nstage; ++s) {
        if (s + 1 < nstage) issue(s + 1, (s + 1) & 1);
        const half8 *sb = sbuf + (s & 1) * STAGE_H8;
#pragma unroll
        for (int u = 0; u < STAGE_TILES; ++u) {
            half8 a[DB16_GROUPS];
            const half8 *p = sb + u * TILE_H8 + lane;
#pragma unroll
            for (int g = 0; g < DB16_GROUPS; ++g) a[g] = p[g * 64];
            floatx16 acc[NQ];
            tile_mfma<NQ>(a, bq, acc);
            tile_min<NQ>(acc, mn);
            const int i = s * STAGE_TILES + u;
            if ((i + 1) % tps == 0) seg_flush<NQ>(mn, tile0, j, h, M, segmin, nseg, seg0 + i / tps);
        }
        stage_barrier();
    }
}

// grid: nchunks (rounded up to 8) x groups; the T query tiles split over the groups as
// evenly as possible (each 4..12 tiles: the launcher takes groups = ceil(T / 12), T >= 4)
__global__ __launch_bounds__(256) void k_screen_h16u(const half8 *__restrict__ db16, int nchunks,
                                                     int ch, int seg_rows,
                                                     const half8 *__restrict__ q16, int M, int T,
                                                     int groups, float *__restrict__ segmin,
                                                     long nseg) {
    __shared__ half8 sbuf[2 * STAGE_H8];
    const int b = blockIdx.x;
    const int slot = b >> 3;
    const int chunk = (slot / groups) * 8 + (b & 7);
    const int group = slot - (slot / groups) * groups;
    if (chunk >= nchunks) return;
    const int tpc = ch >> 5;
    const long ctile0 = (long)chunk * tpc;
    const int per = T / groups, rem = T - per * groups;
    const int G = per + (group < rem ? 1 : 0);
    const int first = group * per + (group < rem ? group : rem);
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int r = (wv + slot) & 3;                 // share index, rotated per block
    const int base = G >> 2, extra = G & 3;
    const int nqw = base + (r < extra ? 1 : 0);
    const int tile0 = first + r * base + (r < extra ? r : extra);
    const int nstage = tpc / STAGE_TILES;
    const int tps = seg_rows >> 5;
    const long seg0 = ctile0 * 32 / seg_rows;
    if (nqw >= 3)
        uneven_body<3>(db16, sbuf, ctile0, nstage, tps, seg0, q16, M, tile0, segmin, nseg);
    else if (nqw == 2)
        uneven_body<2>(db16, sbuf, ctile0, nstage, tps, seg0, q16, M, tile0, segmin, nseg);
    else
        uneven_body<1>(db16, sbuf, ctile0, nstage, tps, seg0, q16, M, tile0, segmin, nseg);
}

// ---------------------------------------------------------------------------------
// balanced form (flag 0x40000): a block's G query tiles (4A <= G <= 4A + 4, A = 1, 2) as
// A tiles owned by each wave plus G - 4A extra tiles shared out by row quarters: in
// quarter r of the chunk, wave w also takes extra tile (w + r) & 3 when that index is
// below G - 4A.  Every (extra tile, quarter) is covered once and every wave carries
// A + (G - 4A) / 4 tiles of work, so M = 342 computes 11 tiles (not 12) with the SIMDs
// still evenly loaded (the uneven form above loses that balance).  Quarters hold whole
// segments (seg_rows = min(ch / 4, 512)), so the extra tile's minima close inside them;
// the next quarter's extra tile is prefetched into spare registers.
// ---------------------------------------------------------------------------------
template <int NQ, int NB>
__device__ __forceinline__ void tile_mfma_n(const half8 (&a)[DB16_GROUPS],
                                            const half8 (&bq)[NB][Q16_GROUPS],
                                            floatx16 (&acc)[NB]) {
    const floatx16 zero = {};
#pragma unroll
    for (int qt = 0; qt < NQ; ++qt)
        acc[qt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[0], bq[qt][0], zero, 0, 0, 0);
#pragma unroll
    for (int m = 1; m < MFMA16; ++m)
#pragma unroll
        for (int qt = 0; qt < NQ; ++qt)
            acc[qt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[mfma_a(m)], bq[qt][mfma_b(m)],
                                                             acc[qt], 0, 0, 0);
}
template <int NQ, int NB>
__device__ __forceinline__ void tile_min_n(const floatx16 (&acc)[NB], float (&mn)[NB]) {
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
template <int NQ, int NB>
__device__ __forceinline__ void seg_flush_n(float (&mn)[NB], const int (&qtile)[NB], int j, int h,
                                            int M, float *__restrict__ segmin, long nseg,
                                            long seg) {
#pragma unroll
    for (int qt = 0; qt < NQ; ++qt) {
        const float m = fminf(mn[qt], __shfl_xor(mn[qt], 32));
        const int qg = qtile[qt] * 32 + j;
        if (h == 0 && qg < M) segmin[(long)qg * nseg + seg] = m;
        mn[qt] = FLT_MAX;
    }
}

template <int A>
__global__ __launch_bounds__(256, 2) void k_screen_h16b(const half8 *__restrict__ db16, int nchunks,
                                                        int ch, int seg_rows,
                                                        const half8 *__restrict__ q16, int M,
                                                        int T, int groups,
                                                        float *__restrict__ segmin, long nseg) {
    constexpr int NB = A + 1;
    __shared__ half8 sbuf[2][STAGE_H8];
    const int b = blockIdx.x;
    const int slot = b >> 3;
    const int chunk = (slot / groups) * 8 + (b & 7);
    const int group = slot - (slot / groups) * groups;
    if (chunk >= nchunks) return;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int j = lane & 31, h = lane >> 5;
    const int per = T / groups, rem = T - per * groups;
    const int G = per + (group < rem ? 1 : 0);
    const int first = group * per + (group < rem ? group : rem);
    const int bx = G - 4 * A;                  // 0..4 extra tiles
    auto extra_of = [&](int qr) {
        const int e = (wv + qr) & 3;
        return e < bx ? first + 4 * A + e : -1;
    };
    auto load_tile = [&](half8 (&dst)[Q16_GROUPS], int t) {
        const half8 *p = q16 + (long)(t * 32 + j) * Q16_ROW + h * Q16_GROUPS;
#pragma unroll
        for (int m = 0; m < Q16_GROUPS; ++m) dst[m] = p[m];
    };
    int qtile[NB];
    half8 bq[NB][Q16_GROUPS];
#pragma unroll
    for (int k = 0; k < A; ++k) {
        qtile[k] = first + wv * A + k;
        load_tile(bq[k], qtile[k]);
    }
    half8 bn[Q16_GROUPS];
    int ecur = extra_of(0), enext = extra_of(1);
    if (ecur >= 0) load_tile(bq[A], ecur);
    if (enext >= 0) load_tile(bn, enext);
    qtile[A] = ecur;

    const int tpc = ch >> 5;
    const int tq = tpc >> 2;                   // tiles per row quarter
    const int tps = seg_rows >> 5;
    const int nstage = tpc / STAGE_TILES;
    const long ctile0 = (long)chunk * tpc;
    const long seg0 = ctile0 * 32 / seg_rows;
    auto issue = [&](int s, int buf) {
        const half8 *src = db16 + (ctile0 + (long)s * STAGE_TILES) * TILE_H8 + tid;
#pragma unroll
        for (int k = 0; k < DB16_GROUPS; ++k)
            __builtin_amdgcn_global_load_lds((const void *)(src + k * 256),
                                             (void *)&sbuf[buf][k * 256 + wv * 64], 16, 0, 2);
    };
    auto stage_barrier = [&]() {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    };
    float mn[NB];
#pragma unroll
    for (int qt = 0; qt < NB; ++qt) mn[qt] = FLT_MAX;
    issue(0, 0);
    stage_barrier();
    for (int s = 0; s < nstage; ++s) {
        if (s + 1 < nstage) issue(s + 1, (s + 1) & 1);
        const half8 *sb = sbuf[s & 1];
#pragma unroll
        for (int u = 0; u < STAGE_TILES; ++u) {
            const int i = s * STAGE_TILES + u;
            if (i > 0 && i % tq == 0) {        // next row quarter: rotate the extra tile
                const int qr = i / tq;
                ecur = enext;
                if (ecur >= 0) {
#pragma unroll
                    for (int m = 0; m < Q16_GROUPS; ++m) bq[A][m] = bn[m];
                }
                qtile[A] = ecur;
                enext = qr + 1 < 4 ? extra_of(qr + 1) : -1;
                if (enext >= 0) load_tile(bn, enext);
            }
            half8 a[DB16_GROUPS];
            const half8 *p = sb + u * TILE_H8 + lane;
#pragma unroll
            for (int g = 0; g < DB16_GROUPS; ++g) a[g] = p[g * 64];
            floatx16 acc[NB];
            const bool close = (i + 1) % tps == 0;
            if (ecur >= 0) {
                tile_mfma_n<NB, NB>(a, bq, acc);
                tile_min_n<NB, NB>(acc, mn);
                if (close) seg_flush_n<NB, NB>(mn, qtile, j, h, M, segmin, nseg, seg0 + i / tps);
            } else {
                tile_mfma_n<A, NB>(a, bq, acc);
                tile_min_n<A, NB>(acc, mn);
                if (close) seg_flush_n<A, NB>(mn, qtile, j, h, M, segmin, nseg, seg0 + i / tps);
            }
        }
        stage_barrier();
    }
}

// ---------------------------------------------------------------------------------
// chain-balanced form (default for G = 5..7 and 9..11 query tiles, flag 0x80000; one block
// per chunk holds all G of them):
// the 4G (query tile t, stage tile u) MFMA chains of a stage, in the order 4t + u, are
// cut into 4 runs of G, one per wave.  Every wave issues the same G chains per stage, so
// the per-stage barrier never waits for a lighter wave, and M = 342 computes 11 query
// tiles instead of 12 (M = 171: 6 instead of 8).  A query tile cut between two waves has its per-segment minimum
// combined through LDS (ordered-int ds_min, two copies alternating by segment); chunks
// need segments of whole stages (tps >= 4).
// ---------------------------------------------------------------------------------
__host__ __device__ constexpr int bal_t0(int G, int W) { return (G * W) / 4; }
__host__ __device__ constexpr int bal_ns(int G, int W) { return (G * W + G - 1) / 4 - (G * W) / 4 + 1; }
__host__ __device__ constexpr bool bal_on(int G, int W, int k, int u) {
    return 4 * (bal_t0(G, W) + k) + u >= G * W && 4 * (bal_t0(G, W) + k) + u < G * W + G;
}
__host__ __device__ constexpr bool bal_owner(int G, int W, int t) { return (4 * t) / G == W; }

template <int K, int N, typename F>
__device__ __forceinline__ void static_for(F &&f) {
    if constexpr (K < N) {
        f(std::integral_constant<int, K>{});
        static_for<K + 1, N>(f);
    }
}
__device__ __forceinline__ int fkey(float x) {
    const int b = __float_as_int(x);
    return b >= 0 ? b : b ^ 0x7fffffff;
}
__device__ __forceinline__ float fkey_inv(int b) { return __int_as_float(b >= 0 ? b : b ^ 0x7fffffff); }

template <int G, int W>
__device__ __forceinline__ void bal_body(const half8 *__restrict__ db16, half8 *sbuf, int *xred,
                                         long ctile0, int nstage, int tps, long seg0,
                                         const half8 *__restrict__ q16, int M,
                                         float *__restrict__ segmin, long nseg) {
    constexpr int T0 = bal_t0(G, W), NS = bal_ns(G, W);
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int j = lane & 31, h = lane >> 5;
    half8 bq[NS][Q16_GROUPS];
#pragma unroll
    for (int k = 0; k < NS; ++k) {
        const half8 *p = q16 + (long)((T0 + k) * 32 + j) * Q16_ROW + h * Q16_GROUPS;
#pragma unroll
        for (int m = 0; m < Q16_GROUPS; ++m) bq[k][m] = p[m];
    }
    auto issue = [&](int s, int buf) {
        const half8 *src = db16 + (ctile0 + (long)s * STAGE_TILES) * TILE_H8 + tid;
#pragma unroll
        for (int k = 0; k < DB16_GROUPS; ++k)
            __builtin_amdgcn_global_load_lds((const void *)(src + k * 256),
                                             (void *)(sbuf + buf * STAGE_H8 + k * 256 + W * 64),
                                             16, 0, 2);
    };
    auto stage_barrier = [&]() {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    };
    float mn[NS];
#pragma unroll
    for (int k = 0; k < NS; ++k) mn[k] = FLT_MAX;
    const floatx16 zero = {};
    issue(0, 0);
    stage_barrier();
    for (int s = 0; s < nstage; ++s) {
        if (s + 1 < nstage) issue(s + 1, (s + 1) & 1);
        const half8 *sb = sbuf + (s & 1) * STAGE_H8;
        static_for<0, STAGE_TILES>([&](auto uc) {
            constexpr int u = decltype(uc)::value;
            half8 a[DB16_GROUPS];
            const half8 *p = sb + u * TILE_H8 + lane;
#pragma unroll
            for (int g = 0; g < DB16_GROUPS; ++g) a[g] = p[g * 64];
            floatx16 acc[NS];
            static_for<0, NS>([&](auto kc) {
                constexpr int k = decltype(kc)::value;
                if constexpr (bal_on(G, W, k, u))
                    acc[k] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[0], bq[k][0], zero, 0, 0, 0);
            });
#pragma unroll
            for (int m = 1; m < MFMA16; ++m)
                static_for<0, NS>([&](auto kc) {
                    constexpr int k = decltype(kc)::value;
                    if constexpr (bal_on(G, W, k, u))
                        acc[k] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[mfma_a(m)], bq[k][mfma_b(m)],
                                                                         acc[k], 0, 0, 0);
                });
            static_for<0, NS>([&](auto kc) {
                constexpr int k = decltype(kc)::value;
                if constexpr (bal_on(G, W, k, u)) {
                    const floatx16 &x = acc[k];
                    const float t0 = fminf(fminf(x[0], x[1]), x[2]), t1 = fminf(fminf(x[3], x[4]), x[5]);
                    const float t2 = fminf(fminf(x[6], x[7]), x[8]), t3 = fminf(fminf(x[9], x[10]), x[11]);
                    const float t4 = fminf(fminf(x[12], x[13]), x[14]);
                    const float u0 = fminf(fminf(t0, t1), t2), u1 = fminf(fminf(t3, t4), x[15]);
                    mn[k] = fminf(fminf(mn[k], u0), u1);
                }
            });
        });
        const int done = (s + 1) * STAGE_TILES;
        const bool close = done % tps == 0;
        const int sg = done / tps - 1;                 // segment (within the chunk) just closed
        int *xr = xred + (sg & 1) * (G * 32);
        if (close) {
#pragma unroll
            for (int k = 0; k < NS; ++k) {
                const float m = fminf(mn[k], __shfl_xor(mn[k], 32));
                if (h == 0) atomicMin(&xr[(T0 + k) * 32 + j], fkey(m));
                mn[k] = FLT_MAX;
            }
        }
        stage_barrier();
        if (close) {
            static_for<0, NS>([&](auto kc) {
                constexpr int k = decltype(kc)::value;
                if constexpr (bal_owner(G, W, T0 + k)) {
                    if (h == 0) {
                        const int at = (T0 + k) * 32 + j;
                        const float m = fkey_inv(xr[at]);
                        xr[at] = 0x7fffffff;
                        const int qg = (T0 + k) * 32 + j;
                        if (qg < M) segmin[(long)qg * nseg + seg0 + sg] = m;
                    }
                }
            });
        }
    }
}

template <int G>
__global__ __launch_bounds__(256, 2) void k_screen_h16c(const half8 *__restrict__ db16, int nchunks,
                                                        int ch, int seg_rows,
                                                        const half8 *__restrict__ q16, int M,
                                                        float *__restrict__ segmin, long nseg) {
    __shared__ half8 sbuf[2 * STAGE_H8];
    __shared__ int xred[2 * G * 32];
    const int b = blockIdx.x;
    const int chunk = (b >> 3) * 8 + (b & 7);
    if (chunk >= nchunks) return;
    for (int i = threadIdx.x; i < 2 * G * 32; i += 256) xred[i] = 0x7fffffff;
    const int tpc = ch >> 5;
    const long ctile0 = (long)chunk * tpc;
    const int nstage = tpc / STAGE_TILES;
    const int tps = seg_rows >> 5;
    const long seg0 = ctile0 * 32 / seg_rows;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (wv == 0) bal_body<G, 0>(db16, sbuf, xred, ctile0, nstage, tps, seg0, q16, M, segmin, nseg);
    else if (wv == 1) bal_body<G, 1>(db16, sbuf, xred, ctile0, nstage, tps, seg0, q16, M, segmin, nseg);
    else if (wv == 2) bal_body<G, 2>(db16, sbuf, xred, ctile0, nstage, tps, seg0, q16, M, segmin, nseg);
    else bal_body<G, 3>(db16, sbuf, xred, ctile0, nstage, tps, seg0, q16, M, segmin, nseg);
}

static int h16_shared() {
    static const int v = env_int("IA_H16S", 1);   // 0: per-wave form
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
    if ((flags & 0x1000) && T >= 2) {   // spanning form (A/B)
        const int nq = T >= 9 ? 3 : (T >= 5 ? 2 : 1);
        const int g = (T + 4 * nq - 1) / (4 * nq);
        const long nb = ((nchunks + 7) / 8) * 8 * g;
        IA_ARG(nb < (1L << 31), "screen grid too large");
        IA_ARG(g * 4 * nq <= T + 2 * MAX_NQ, "screen: query tiles exceed the padded rows");
        const int md = (flags & 0x8000) ? 2 : ((flags & 0x2000) ? 1 : 0);
#define IA_H16P_CASE(NQ, MD)                                                                    \
        if (nq == NQ && md == MD) {                                                             \
            k_screen_h16p<NQ, MD><<<(unsigned)nb, 512, 0, st>>>(db16, (int)nchunks, ch, seg_rows, \
                                                               q, M, g, segmin, nseg);          \
            IA_LAUNCH_CHECK("k_screen_h16p");                                                   \
            return IA_OK;                                                                       \
        }
        IA_H16P_CASE(3, 0)
        IA_H16P_CASE(2, 0)
        IA_H16P_CASE(1, 0)
        IA_H16P_CASE(3, 1)
        IA_H16P_CASE(2, 1)
        IA_H16P_CASE(1, 1)
        IA_H16P_CASE(3, 2)
        IA_H16P_CASE(2, 2)
        IA_H16P_CASE(1, 2)
#undef IA_H16P_CASE
        set_error("launch_screen16: bad span split");
        return IA_E_ARG;
    }
    // chain-balanced form: the default for 1, 3, 5..7 and 9..11 query tiles (IA_SCREEN_BAL=0
    // turns it off; 4, 8 and 12 split evenly anyway; T = 3: 8-10 % faster than 4 x 1 tiles,
    // profiles/r01_screen_bench_h16c_t3.txt; T = 1: 15 % faster than the per-wave stream,
    // 6.6 TB/s; T = 2, 4, 8: no gain — A/B only, profiles/r01_screen_bench_h16c_t12.txt,
    // _t48.txt)
    static const int bal_env = env_int("IA_SCREEN_BAL", 1);
    const bool bal_t = T <= 11 && ((T != 2 && T != 4 && T != 8) || (flags & 0x80000));
    if (((flags & 0x80000) || (bal_env && flags == 0)) && bal_t &&
        seg_rows >= STAGE_TILES * 32) {   // segments of whole stages (tps >= 4)
        const long nb = ((nchunks + 7) / 8) * 8;
#define IA_H16C_CASE(GG)                                                                        \
        if (T == GG) {                                                                          \
            k_screen_h16c<GG><<<(unsigned)nb, 256, 0, st>>>(db16, (int)nchunks, ch, seg_rows, q, M, \
                                                             segmin, nseg);                     \
            IA_LAUNCH_CHECK("k_screen_h16c");                                                   \
            return IA_OK;                                                                       \
        }
        IA_H16C_CASE(1)
        IA_H16C_CASE(2)
        IA_H16C_CASE(3)
        IA_H16C_CASE(4)
        IA_H16C_CASE(5)
        IA_H16C_CASE(6)
        IA_H16C_CASE(7)
        IA_H16C_CASE(8)
        IA_H16C_CASE(9)
        IA_H16C_CASE(10)
        IA_H16C_CASE(11)
#undef IA_H16C_CASE
    }
    if ((flags & 0x40000) && T >= 4) {   // balanced shares (A/B)
        const int g = (T + 11) / 12;
        const int A = (T / g) / 4;
        if (A == 1 || A == 2) {
            const long nb = ((nchunks + 7) / 8) * 8 * g;
            IA_ARG(nb < (1L << 31), "screen grid too large");
            if (A == 1)
                k_screen_h16b<1><<<(unsigned)nb, 256, 0, st>>>(db16, (int)nchunks, ch, seg_rows, q, M,
                                                               T, g, segmin, nseg);
            else
                k_screen_h16b<2><<<(unsigned)nb, 256, 0, st>>>(db16, (int)nchunks, ch, seg_rows, q, M,
                                                               T, g, segmin, nseg);
            IA_LAUNCH_CHECK("k_screen_h16b");
            return IA_OK;
        }
    }
    if ((flags & 0x4000) && T >= 4) {   // uneven query shares (A/B)
        const int g = (T + 11) / 12;
        const long nb = ((nchunks + 7) / 8) * 8 * g;
        IA_ARG(nb < (1L << 31), "screen grid too large");
        k_screen_h16u<<<(unsigned)nb, 256, 0, st>>>(db16, (int)nchunks, ch, seg_rows, q, M, T, g,
                                                    segmin, nseg);
        IA_LAUNCH_CHECK("k_screen_h16u");
        return IA_OK;
    }
    bool pipe = !(flags & 0x200);
    const bool pf = flags & 0x400;    // fragment-prefetch form (A/B)
    if (h16_shared() && !(flags & 0x100) && T >= 2) {
        // query tiles per block WQ x NQ: T >= 9 -> 4 x 3, 5..8 -> 4 x 2, 3..4 -> 4 x 1,
        // 2 -> 2 x 1 (fewest padded tiles, then the most sharing)
        int wq = 4, nq = T >= 9 ? 3 : (T >= 5 ? 2 : 1);
        if (T == 2) wq = 2;
        if (cap > 0 && cap < nq) nq = cap;
        // the pipelined epilogue's second accumulator set costs NQ = 3 its second wave per
        // SIMD (measured slower: profiles/r01_screen_bench_h16s.txt)
        if (nq == 3 && !(flags & 0x800)) pipe = false;   // bit 11: keep it (A/B)
        const int g = (T + wq * nq - 1) / (wq * nq);
        const long nb = ((nchunks + 7) / 8) * 8 * g;
        IA_ARG(nb < (1L << 31), "screen grid too large");
        IA_ARG(g * wq * nq <= T + 2 * MAX_NQ, "screen: query tiles exceed the padded rows");
        const int mode = (flags & 0x10000) ? 3 : (pf ? 2 : (pipe ? 1 : 0));
        // bit 17 / IA_SCREEN_NT (default 1): the DB stream copied with non-temporal loads (it
        // is read once per launch and never fits the caches)
        static const int nt_env = env_int("IA_SCREEN_NT", 1);
        const bool nt = (flags & 0x20000) || nt_env;
#define IA_H16S_NT_CASE(NQ, WQ, MD)                                                             \
        if (nt && nq == NQ && wq == WQ && mode == MD) {                                         \
            k_screen_h16s<NQ, WQ, MD, true><<<(unsigned)nb, 256, 0, st>>>(db16, (int)nchunks, ch, \
                                                                          seg_rows, q, M, g,    \
                                                                          segmin, nseg);        \
            IA_LAUNCH_CHECK("k_screen_h16s");                                                   \
            return IA_OK;                                                                       \
        }
        IA_H16S_NT_CASE(3, 4, 0)
        IA_H16S_NT_CASE(2, 4, 1)
        IA_H16S_NT_CASE(1, 4, 1)
        IA_H16S_NT_CASE(1, 2, 1)
#undef IA_H16S_NT_CASE
#define IA_H16S_CASE(NQ, WQ, MD)                                                                \
        if (nq == NQ && wq == WQ && mode == MD) {                                               \
            k_screen_h16s<NQ, WQ, MD><<<(unsigned)nb, 256, 0, st>>>(db16, (int)nchunks, ch,     \
                                                                    seg_rows, q, M, g, segmin,  \
                                                                    nseg);                      \
            IA_LAUNCH_CHECK("k_screen_h16s");                                                   \
            return IA_OK;                                                                       \
        }
        IA_H16S_CASE(3, 4, 1)
        IA_H16S_CASE(2, 4, 1)
        IA_H16S_CASE(1, 4, 1)
        IA_H16S_CASE(1, 2, 1)
        IA_H16S_CASE(3, 4, 0)
        IA_H16S_CASE(2, 4, 0)
        IA_H16S_CASE(1, 4, 0)
        IA_H16S_CASE(1, 2, 0)
        IA_H16S_CASE(3, 4, 2)
        IA_H16S_CASE(2, 4, 2)
        IA_H16S_CASE(1, 4, 2)
        IA_H16S_CASE(1, 2, 2)
        IA_H16S_CASE(3, 4, 3)
        IA_H16S_CASE(2, 4, 3)
        IA_H16S_CASE(1, 4, 3)
        IA_H16S_CASE(1, 2, 3)
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
