// ia_screen16.hip — the split-f16 segment screen, stage 1 of the exact
// matcher (ia_match.hip).
//
// For every (query, DB segment of seg_rows <= 512 rows) the minimum of the screen value
// sa * sq_j * (|a'|^2 - 2 a'.q'), computed as 11 v_mfma_f32_32x32x16_f16 per 32x32 (rows x
// queries) tile from the split-f16 operands of ia_split16.h (7 DB and 8 query register
// groups per lane).  Queries are the stationary operand (VGPRs); DB rows stream through
// LDS in 4-tile stages (28 KiB, global_load_lds_dwordx4, non-temporal: the DB is read
// once per launch and never fits the caches), double-buffered with one barrier per stage,
// so each DB byte fetched feeds the block's 4 waves.
//
// Chain balance: one block holds G (1..11) query tiles.  The 4G (query tile t, stage tile
// u) MFMA chains of a stage, in the order 4t + u, are cut into 4 equal runs of G, one per
// wave: every wave issues the same MFMAs per stage, so the per-stage barrier never waits
// for a lighter wave, and M queries compute ceil(M/32) tiles (M = 342: 11, not 12).  A
// query tile cut between two waves combines its per-segment minimum through LDS
// (ordered-int ds_min).  Launches of more than 11 tiles split them into equal groups.
//
// Segment minima are staged in LDS for the whole chunk (ch / seg_rows <= 16 segments) and
// written once at the end as spc consecutive floats per query (segmin is query-major,
// [M][nseg], the exact stage's layout): full 64-B runs instead of one 4-B store per
// (query, segment) strided by nseg.
//
// Padding rows of the DB's last chunks repeat its last real row (k_db_build), so the
// minima need no masking.  Built with -fno-honor-nans (the min-reductions need no NaN
// canonicalisation: inputs are finite by construction) and -amdgpu-mfma-vgpr-form (MFMA
// results in VGPRs: the reductions read them without v_accvgpr_read copies).
#include "ia_imgwin.h"
#include "ia_split16.h"

#include <atomic>
#include <float.h>
#include <stdint.h>
#include <type_traits>

namespace ia {

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int TILE_H8 = DB16_GROUPS * 64;            // half8 per 32-row tile (7 KiB)
constexpr int STAGE_TILES = 4;
constexpr int STAGE_H8 = STAGE_TILES * TILE_H8;      // 28 KiB
constexpr int MAX_G = 11;                            // query tiles per block
constexpr int SPC_MAX = 16;                          // segments per chunk (8192 / 512)
static_assert(DB_CHUNK_MAX / DB_SEG_MAX == SPC_MAX, "LDS staging of the chunk's minima");

__host__ __device__ constexpr int bal_t0(int G, int W) { return (G * W) / 4; }
__host__ __device__ constexpr int bal_ns(int G, int W) { return (G * W + G - 1) / 4 - (G * W) / 4 + 1; }
__host__ __device__ constexpr bool bal_on(int G, int W, int k, int u) {
    return 4 * (bal_t0(G, W) + k) + u >= G * W && 4 * (bal_t0(G, W) + k) + u < G * W + G;
}

template <int K, int N, typename F>
__device__ __forceinline__ void static_for(F &&f) {
    if constexpr (K < N) {
        f(std::integral_constant<int, K>{});
        static_for<K + 1, N>(f);
    }
}
// order-preserving int key of a float (LDS integer min)
__device__ __forceinline__ int fkey(float x) {
    const int b = __float_as_int(x);
    return b >= 0 ? b : b ^ 0x7fffffff;
}
__device__ __forceinline__ float fkey_inv(int b) { return __int_as_float(b >= 0 ? b : b ^ 0x7fffffff); }

// wave W's MFMA chains of one 4-tile stage (operand sb in LDS) into its running minima
template <int G, int W, int NS>
__device__ __forceinline__ void stage_mfma(const half8 *sb, const half8 (&bq)[NS][Q16_GROUPS],
                                           float (&mn)[NS], int lane) {
    const floatx16 zero = {};
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
        // running minimum: 8 v_min3_f32 per accumulator, dependency depth 3
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
}

// ---- chain-major stage (IA_SCREEN_SCHED=1) -------------------------------------------
// The same chains as stage_mfma, but each (query tile, stage tile) chain runs its 11 MFMAs
// back to back into one of two ping-pong accumulators (a single accumulation chain of
// v_mfma_f32_32x32x16 issues at the full rate), its running-minimum fold is issued after the
// NEXT chain's first MFMA (the VALU overlaps that chain's MFMAs instead of waiting on the
// last result behind an s_nop), and the next stage tile's 7 operand reads are issued at the
// start of the current tile's last chain (two operand register sets), so no tile boundary
// waits on an LDS round trip.  Same products, same per-accumulator order, same minima.
template <int G, int W>
__host__ __device__ constexpr int ch_count() {
    int n = 0;
    for (int u = 0; u < STAGE_TILES; ++u)
        for (int k = 0; k < bal_ns(G, W); ++k) n += bal_on(G, W, k, u) ? 1 : 0;
    return n;
}
// (stage tile, chain slot) of wave W's c-th chain in tile-major order
template <int G, int W>
__host__ __device__ constexpr int ch_u(int c) {
    for (int u = 0; u < STAGE_TILES; ++u)
        for (int k = 0; k < bal_ns(G, W); ++k)
            if (bal_on(G, W, k, u) && c-- == 0) return u;
    return -1;
}
template <int G, int W>
__host__ __device__ constexpr int ch_k(int c) {
    for (int u = 0; u < STAGE_TILES; ++u)
        for (int k = 0; k < bal_ns(G, W); ++k)
            if (bal_on(G, W, k, u) && c-- == 0) return k;
    return -1;
}
// ordinal of chain c's stage tile among the wave's distinct tiles (its operand set parity)
template <int G, int W>
__host__ __device__ constexpr int ch_uo(int c) {
    int o = 0;
    for (int i = 1; i <= c; ++i) o += ch_u<G, W>(i) != ch_u<G, W>(i - 1) ? 1 : 0;
    return o;
}

__device__ __forceinline__ void fold_min(const floatx16 &x, float &mn) {
    const float t0 = fminf(fminf(x[0], x[1]), x[2]), t1 = fminf(fminf(x[3], x[4]), x[5]);
    const float t2 = fminf(fminf(x[6], x[7]), x[8]), t3 = fminf(fminf(x[9], x[10]), x[11]);
    const float t4 = fminf(fminf(x[12], x[13]), x[14]);
    const float u0 = fminf(fminf(t0, t1), t2), u1 = fminf(fminf(t3, t4), x[15]);
    mn = fminf(fminf(mn, u0), u1);
}

template <int G, int W, int NS, bool CM_PIN = false>
__device__ __forceinline__ void stage_mfma_cm(const half8 *sb, const half8 (&bq)[NS][Q16_GROUPS],
                                              float (&mn)[NS], int lane) {
    constexpr int NC = ch_count<G, W>();
    const floatx16 zero = {};
    half8 a[2][DB16_GROUPS];
    floatx16 acc[2];
    {
        const half8 *p = sb + ch_u<G, W>(0) * TILE_H8 + lane;
#pragma unroll
        for (int g = 0; g < DB16_GROUPS; ++g) a[0][g] = p[g * 64];
    }
    static_for<0, NC>([&](auto cc) {
        constexpr int c = decltype(cc)::value;
        constexpr int k = ch_k<G, W>(c), ab = ch_uo<G, W>(c) & 1, cb = c & 1;
        if constexpr (c + 1 < NC && ch_u<G, W>(c + 1) != ch_u<G, W>(c)) {
            // the next tile's operand, into the set no issued chain still reads
            const half8 *p = sb + ch_u<G, W>(c + 1) * TILE_H8 + lane;
#pragma unroll
            for (int g = 0; g < DB16_GROUPS; ++g) a[ab ^ 1][g] = p[g * 64];
        }
        acc[cb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[ab][0], bq[k][0], zero, 0, 0, 0);
        if constexpr (c > 0) fold_min(acc[cb ^ 1], mn[ch_k<G, W>(c - 1)]);
#pragma unroll
        for (int m = 1; m < MFMA16; ++m)
            acc[cb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[ab][mfma_a(m)], bq[k][mfma_b(m)], acc[cb],
                                                             0, 0, 0);
        if constexpr (CM_PIN) {
            // this chain's region: [operand reads,] MFMA, then the previous chain's fold two
            // VALU at a time between the next MFMAs (each pair well inside an MFMA's 32
            // cycles), then the rest of the chain
            if constexpr (c + 1 < NC && ch_u<G, W>(c + 1) != ch_u<G, W>(c))
                __builtin_amdgcn_sched_group_barrier(0x100, DB16_GROUPS, 0);   // DS reads
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            if constexpr (c > 0) {
                static_for<0, 4>([&](auto) {
                    __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                });
                __builtin_amdgcn_sched_group_barrier(0x008, MFMA16 - 5, 0);
            } else {
                __builtin_amdgcn_sched_group_barrier(0x008, MFMA16 - 1, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    });
    fold_min(acc[(NC - 1) & 1], mn[ch_k<G, W>(NC - 1)]);
}

template <int SCHED, int G, int W, int NS>
__device__ __forceinline__ void stage_run(const half8 *sb, const half8 (&bq)[NS][Q16_GROUPS],
                                          float (&mn)[NS], int lane) {
    if constexpr (SCHED == 1) stage_mfma_cm<G, W, NS>(sb, bq, mn, lane);
    else stage_mfma<G, W, NS>(sb, bq, mn, lane);
}

// after stage s: when it closes a segment, fold the wave's minima into smin[seg][G * 32]
template <int G, int W, int NS>
__device__ __forceinline__ void stage_close(int s, int tps, int *smin, float (&mn)[NS], int lane) {
    constexpr int T0 = bal_t0(G, W);
    const int done = (s + 1) * STAGE_TILES;
    if (done % tps == 0) {   // segment done / tps - 1 of the chunk closed
        int *sm = smin + (done / tps - 1) * (G * 32);
        const int j = lane & 31, h = lane >> 5;
#pragma unroll
        for (int k = 0; k < NS; ++k) {
            // the two lane halves hold different rows of the same queries
            const float m = fminf(mn[k], __shfl_xor(mn[k], 32));
            if (h == 0) atomicMin(&sm[(T0 + k) * 32 + j], fkey(m));
            mn[k] = FLT_MAX;
        }
    }
}

template <int G, int W, int NS>
__device__ __forceinline__ void load_queries(const half8 *__restrict__ q16, half8 (&bq)[NS][Q16_GROUPS],
                                             int lane) {
    constexpr int T0 = bal_t0(G, W);
    const int j = lane & 31, h = lane >> 5;
#pragma unroll
    for (int k = 0; k < NS; ++k) {
        const half8 *p = q16 + (long)((T0 + k) * 32 + j) * Q16_ROW + h * Q16_GROUPS;
#pragma unroll
        for (int m = 0; m < Q16_GROUPS; ++m) bq[k][m] = p[m];
    }
}

// a workgroup barrier ordering LDS only (no wait for global loads in flight)
__device__ __forceinline__ void lds_sync() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// every wave's copies of the next stage retired, then the barrier (the compiler's own wait
// before __syncthreads() does not cover global_load_lds)
__device__ __forceinline__ void copies_barrier() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
}

// row form: wave W's share of one chunk, the DB rows streamed into LDS stage by stage
template <int SCHED, int G, int W>
__device__ __forceinline__ void chain_body(const half8 *__restrict__ db16, half8 *sbuf, int *smin,
                                           const StageMap &sm, long chunk, int nstage, int tps,
                                           const half8 *__restrict__ q16) {
    constexpr int NS = bal_ns(G, W);
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    half8 bq[NS][Q16_GROUPS];
    load_queries<G, W, NS>(q16, bq, lane);
    auto issue = [&](int s, int buf) {
        const half8 *src = db16 + (stage_lrow(sm, chunk, s) >> 5) * TILE_H8 + tid;
#pragma unroll
        for (int k = 0; k < DB16_GROUPS; ++k)
            __builtin_amdgcn_global_load_lds((const void *)(src + k * 256),
                                             (void *)(sbuf + buf * STAGE_H8 + k * 256 + W * 64),
                                             16, 0, 2);
    };
    float mn[NS];
#pragma unroll
    for (int k = 0; k < NS; ++k) mn[k] = FLT_MAX;
    issue(0, 0);
    copies_barrier();
    for (int s = 0; s < nstage; ++s) {
        if (s + 1 < nstage) issue(s + 1, (s + 1) & 1);
        stage_run<SCHED, G, W, NS>(sbuf + (s & 1) * STAGE_H8, bq, mn, lane);
        stage_close<G, W, NS>(s, tps, smin, mn, lane);
        copies_barrier();   // stage s+1 landed and stage s is free again
    }
}

// image form (ia_internal.h ImgDb): a stage is 128 pixels of one scanline, built in LDS
// from image windows — fine rows y-2..y+2 of A and y-2..y of A' (34 x 16-B pieces each),
// coarse rows of both (18 pieces), the stage's 128 norm slots — 6.6 KB instead of 28 KB
// of rows; the window is expanded into the row form's operand layout in LDS, then the
// same MFMA stage runs.  Windows are double-buffered (the next one's copies fly during the
// expansion and MFMAs of this one); the operand is built and consumed between two barriers.
static_assert(WIN_PIECES <= 448, "waves 0-2 x two wave-instructions + wave 3 x one stage the window");
__host__ __device__ constexpr int grp_k0(int h, int g) {
    return h == 0 ? (g < 4 ? 8 * g : 8 * (g - 4)) : (g < 3 ? 32 + 8 * g : (g == 3 ? 24 : 32 + 8 * (g - 4)));
}
__host__ __device__ constexpr bool grp_hi(int h, int g) { return h == 0 ? g < 4 : g < 3; }

// expand groups [G0, G1) of this wave's operand slot (tile 2 (W >> 1) + lane / 32, row
// lane % 32, lane half W & 1) from window wb into the stage operand E: ds_read_u16 at
// compile-time offsets from two per-lane bases, one ds_write_b128 per group
template <int W, int G0, int G1>
__device__ __forceinline__ void expand_groups(const char *wb, half8 *E, int lane) {
    constexpr int H = W & 1;
    const int tile = 2 * (W >> 1) + (lane >> 5), j = lane & 31;
    const int px = 32 * tile + j;
    const char *bf = wb + px * 4, *bc = wb + (px >> 1) * 4;
    half8 *e = E + tile * TILE_H8 + H * 32 + j;
    static_for<G0, G1>([&](auto gc) {
        constexpr int g = decltype(gc)::value;
        constexpr int k0 = grp_k0(H, g);
        constexpr bool hi = grp_hi(H, g);
        half8 o;
        static_for<0, 8>([&](auto ec) {
            constexpr int k = k0 + decltype(ec)::value;
            constexpr int off = win_off(k) + (hi ? 0 : 2);
            const char *b = (k < 55 && win_coarse(k)) ? bc : bf;
            o[decltype(ec)::value] = *reinterpret_cast<const _Float16 *>(b + off);
        });
        e[g * 64] = o;
    });
}

// Per stage: expand the window into the operand (all waves), barrier, the row form's MFMA
// stage, barrier.  The window of the next stage is in flight meanwhile (two window
// buffers, one operand buffer: 63.7 KB of LDS, 2 blocks per CU, which overlap one block's
// expansion with the other's MFMAs).  Measured against a pipelined form (two operand
// buffers, the next stage expanded before this one's MFMAs, one barrier per stage, 81.8 KB):
// c4 1615-1635 vs 1650-1656 ms/step (`tools/gpu.sh ablib`, profiles/r02_image_form_ab.txt).
template <int SCHED, int G, int W>
__device__ __forceinline__ void img_body(const ImgDb &im, half8 *E, char *wbuf, int *smin,
                                         const StageMap &sm, long chunk, int nstage, int tps,
                                         const half8 *__restrict__ q16) {
    constexpr int NS = bal_ns(G, W);
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    half8 bq[NS][Q16_GROUPS];
    load_queries<G, W, NS>(q16, bq, lane);
    auto issue = [&](int s, int buf) {
        const WinSrc ws = win_src(im, stage_lrow(sm, chunk, s));
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            if (t == 1 && W == 3) continue;     // pieces 448.. are past the window
            const int i = (t * 4 + W) * 64 + lane;
            if (i < WIN_PIECES)
                __builtin_amdgcn_global_load_lds((const void *)win_piece(im, ws, i),
                                                 (void *)(wbuf + buf * WIN_B + (t * 4 + W) * 1024),
                                                 16, 0, 2);
        }
    };
    float mn[NS];
#pragma unroll
    for (int k = 0; k < NS; ++k) mn[k] = FLT_MAX;
    issue(0, 0);
    copies_barrier();
    for (int s = 0; s < nstage; ++s) {
        if (s + 1 < nstage) issue(s + 1, (s + 1) & 1);
        expand_groups<W, 0, DB16_GROUPS>(wbuf + (s & 1) * WIN_B, E, lane);
        __syncthreads();   // the stage operand is complete
        stage_run<SCHED, G, W, NS>(E, bq, mn, lane);
        stage_close<G, W, NS>(s, tps, smin, mn, lane);
        copies_barrier();   // the operand is consumed and window s + 1 has landed
    }
}

// ---- strips (StageMap with W > 0): the rolling window --------------------------------
// A chunk is one 128-pixel column strip walked down scanline by scanline, so consecutive
// stages' windows share all but one fine row of A and of A' (and all coarse rows every
// second stage).  The window rows live in LDS rings indexed by their padded image row
// (A fine 8 slots, A' fine 4, each coarse image 4, norm slots 2); per stage the block
// copies in the rows the next stage adds (<= 5 wave instructions, ~1.9 KB instead of the
// whole 6.6 KB window), so every image row is fetched about once per chunk.
constexpr int FROW_B = WF_PC * 16, CROW_B = WC_PC * 16;        // 544, 288 B per window row
constexpr int RW_FA = 0, RW_FP = RW_FA + 8 * FROW_B, RW_CA = RW_FP + 4 * FROW_B;
constexpr int RW_CP = RW_CA + 4 * CROW_B, RW_NM = RW_CP + 4 * CROW_B, RW_B = RW_NM + 2 * 512;

// window row job j of a stage at position w into the ring (one wave instruction; lanes past
// the row's pieces idle).  kind: 0 A fine, 1 A' fine, 2 A coarse, 3 A' coarse, 4 norms;
// r = the padded image row (fine / coarse) or unused (norms); nslot = the stage's norm slot
__device__ __forceinline__ void rw_load(const ImgDb &im, const WinSrc &w, char *ring, int kind, int r,
                                        int nslot, int lane) {
    const uint32_t *src;
    char *dst;
    int n;
    if (kind == 0) { src = im.fa + (long)r * im.Wp + w.x0; dst = ring + RW_FA + (r & 7) * FROW_B; n = WF_PC; }
    else if (kind == 1) { src = w.fp + (long)r * im.Wp + w.x0; dst = ring + RW_FP + (r & 3) * FROW_B; n = WF_PC; }
    else if (kind == 2) { src = im.ca + (long)r * im.Wcp + (w.x0 >> 1); dst = ring + RW_CA + (r & 3) * CROW_B; n = WC_PC; }
    else if (kind == 3) { src = w.cp + (long)r * im.Wcp + (w.x0 >> 1); dst = ring + RW_CP + (r & 3) * CROW_B; n = WC_PC; }
    else { src = im.norm + w.lrow; dst = ring + RW_NM + nslot * 512; n = 32; }
    if (lane < n) __builtin_amdgcn_global_load_lds((const void *)(src + 4 * lane), (void *)dst, 16, 0, 2);
}

// the operand slot of wave W (as expand_groups) from the rings of the stage at image row y
// (padded fine rows y .. y + 4 / y + 2, coarse rows c1 .. c1 + 2, norm slot ns)
template <int W>
__device__ __forceinline__ void expand_ring(const char *ring, int y, int ns, half8 *E, int lane) {
    constexpr int H = W & 1;
    const int tile = 2 * (W >> 1) + (lane >> 5), j = lane & 31;
    const int px = 32 * tile + j;
    const int c1 = (y >> 1) + 1;
    const char *fa[5], *fp[3], *ca[3], *cp[3];
#pragma unroll
    for (int r = 0; r < 5; ++r) fa[r] = ring + RW_FA + ((y + r) & 7) * FROW_B + px * 4;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        fp[r] = ring + RW_FP + ((y + r) & 3) * FROW_B + px * 4;
        ca[r] = ring + RW_CA + ((c1 + r) & 3) * CROW_B + (px >> 1) * 4;
        cp[r] = ring + RW_CP + ((c1 + r) & 3) * CROW_B + (px >> 1) * 4;
    }
    const char *nm = ring + RW_NM + ns * 512 + px * 4;
    half8 *e = E + tile * TILE_H8 + H * 32 + j;
    static_for<0, DB16_GROUPS>([&](auto gc) {
        constexpr int g = decltype(gc)::value;
        constexpr int k0 = grp_k0(H, g);
        constexpr int hb = grp_hi(H, g) ? 0 : 2;
        half8 o;
        static_for<0, 8>([&](auto ec) {
            constexpr int k = k0 + decltype(ec)::value;
            const char *b;
            if constexpr (k < 9) b = ca[k / 3] + (k % 3 + 3) * 4;
            else if constexpr (k < 34) b = fa[(k - 9) / 5] + ((k - 9) % 5 + 2) * 4;
            else if constexpr (k < 43) b = cp[(k - 34) / 3] + ((k - 34) % 3 + 3) * 4;
            else if constexpr (k < 55) b = fp[(k - 43) / 5] + ((k - 43) % 5 + 2) * 4;
            else b = nm;
            o[decltype(ec)::value] = *reinterpret_cast<const _Float16 *>(b + hb);
        });
        e[g * 64] = o;
    });
}

template <int SCHED, int G, int W>
__device__ __forceinline__ void strip_body(const ImgDb &im, half8 *E, char *ring, int *smin,
                                           const StageMap &sm, long chunk, int nstage, int tps,
                                           const half8 *__restrict__ q16) {
    constexpr int NS = bal_ns(G, W);
    const int lane = threadIdx.x & 63;
    half8 bq[NS][Q16_GROUPS];
    load_queries<G, W, NS>(q16, bq, lane);
    float mn[NS];
#pragma unroll
    for (int k = 0; k < NS; ++k) mn[k] = FLT_MAX;
    // stage 0: the whole window, 15 row jobs dealt over the 4 waves
    WinSrc w = win_src(im, stage_lrow(sm, chunk, 0));
    for (int j = W; j < 15; j += 4) {
        const int kind = j < 5 ? 0 : j < 8 ? 1 : j < 11 ? 2 : j < 14 ? 3 : 4;
        const int r = j < 5 ? w.y + j : j < 8 ? w.y + j - 5 : j < 11 ? (w.y >> 1) + 1 + j - 8
                                                                    : (w.y >> 1) + 1 + j - 11;
        rw_load(im, w, ring, kind, r, 0, lane);
    }
    copies_barrier();
    for (int s = 0; s < nstage; ++s) {
        const int y = w.y;
        if (s + 1 < nstage) {
            // the rows stage s + 1 adds (scanline y + 1 of the same image): slots stage s
            // does not read
            const WinSrc wn = win_src(im, stage_lrow(sm, chunk, s + 1));
            const bool cnew = (wn.y >> 1) != (y >> 1);
            if (W == 0) rw_load(im, wn, ring, 0, wn.y + 4, 0, lane);
            else if (W == 1) rw_load(im, wn, ring, 1, wn.y + 2, 0, lane);
            else if (W == 2) rw_load(im, wn, ring, 4, 0, (s + 1) & 1, lane);
            else if (cnew) {
                rw_load(im, wn, ring, 2, (wn.y >> 1) + 3, 0, lane);
                rw_load(im, wn, ring, 3, (wn.y >> 1) + 3, 0, lane);
            }
            w = wn;
        }
        expand_ring<W>(ring, y, s & 1, E, lane);
        __syncthreads();   // the stage operand is complete
        stage_run<SCHED, G, W, NS>(E, bq, mn, lane);
        stage_close<G, W, NS>(s, tps, smin, mn, lane);
        copies_barrier();  // the operand is consumed and stage s + 1's rows have landed
    }
}

// ---- strips, producer / consumer (IA_SCREEN_PC=1): k_screen16p -----------------------
// One 8-wave workgroup per CU.  Waves 0-3 (one per SIMD) only run MFMA stages: the same
// chains as strip_body (chain-major, the next stage tile's operand prefetched).  Waves 4-7
// (the other wave of each SIMD) expand stage s + 1's operand from the rings into the second
// operand buffer while the MFMA waves run stage s, so the matrix pipe never waits on an
// expansion: one barrier per stage hands the operand buffers over.  Window rows are copied
// three stages ahead and waited one stage later (a copy has a whole MFMA stage to land):
// rings of 8 slots per image (rows in use: 5 + 2 in flight for A fine, 3 + 2 for the others)
// and 4 norm slots.
#ifndef IA_PC_PIN
#define IA_PC_PIN 0
#endif
constexpr bool PC_PIN = IA_PC_PIN;   // k_screen16p pins its MFMA stage's schedule (CM_PIN)
#ifndef IA_PC_AHEAD
#define IA_PC_AHEAD 3
#endif
constexpr int PC_AHEAD = IA_PC_AHEAD;
// A/B build knob (diagnostic builds only; the product uses the default): IA_PC_PRIO raises
// the MFMA waves' issue priority (s_setprio)
#ifndef IA_PC_PRIO
#define IA_PC_PRIO 0
#endif
static_assert(PC_AHEAD == 2 || PC_AHEAD == 3, "ring depth");
constexpr int RP_FA = 0, RP_FP = RP_FA + 8 * FROW_B, RP_CA = RP_FP + 8 * FROW_B;
constexpr int RP_CP = RP_CA + 8 * CROW_B, RP_NM = RP_CP + 8 * CROW_B, RP_B = RP_NM + 4 * 512;

// one window row job into the 8-slot rings (as rw_load): kind 0 A fine, 1 A' fine, 2 A
// coarse, 3 A' coarse (padded image row r), 4 norms (slot nslot)
__device__ __forceinline__ void rp_load(const ImgDb &im, const WinSrc &w, char *ring, int kind, int r,
                                        int nslot, int lane) {
    const uint32_t *src;
    char *dst;
    int n;
    if (kind == 0) { src = im.fa + (long)r * im.Wp + w.x0; dst = ring + RP_FA + (r & 7) * FROW_B; n = WF_PC; }
    else if (kind == 1) { src = w.fp + (long)r * im.Wp + w.x0; dst = ring + RP_FP + (r & 7) * FROW_B; n = WF_PC; }
    else if (kind == 2) { src = im.ca + (long)r * im.Wcp + (w.x0 >> 1); dst = ring + RP_CA + (r & 7) * CROW_B; n = WC_PC; }
    else if (kind == 3) { src = w.cp + (long)r * im.Wcp + (w.x0 >> 1); dst = ring + RP_CP + (r & 7) * CROW_B; n = WC_PC; }
    else { src = im.norm + w.lrow; dst = ring + RP_NM + nslot * 512; n = 32; }
    if (lane < n) __builtin_amdgcn_global_load_lds((const void *)(src + 4 * lane), (void *)dst, 16, 0, 2);
}

// the rows stage w2 adds to stage w1 (one scanline down), expander X: exactly RP_N(X) copies
// (X 3 re-copies the current coarse rows when w2 starts none: identical bytes into the
// slots they already hold, so that every iteration waits on a fixed count)
__host__ __device__ constexpr int rp_n(int X) { return X == 3 ? 2 : 1; }
template <int X>
__device__ __forceinline__ void rp_rows(const ImgDb &im, const WinSrc &w1, const WinSrc &w2, char *ring,
                                        int nslot, int lane) {
    (void)w1;
    if constexpr (X == 0) rp_load(im, w2, ring, 0, w2.y + 4, 0, lane);
    else if constexpr (X == 1) rp_load(im, w2, ring, 1, w2.y + 2, 0, lane);
    else if constexpr (X == 2) rp_load(im, w2, ring, 4, 0, nslot, lane);
    else {
        rp_load(im, w2, ring, 2, (w2.y >> 1) + 3, 0, lane);
        rp_load(im, w2, ring, 3, (w2.y >> 1) + 3, 0, lane);
    }
}

// expand_ring over the 8-slot rings
template <int W>
__device__ __forceinline__ void rp_expand(const char *ring, int y, int ns, half8 *E, int lane) {
    constexpr int H = W & 1;
    const int tile = 2 * (W >> 1) + (lane >> 5), j = lane & 31;
    const int px = 32 * tile + j;
    const int c1 = (y >> 1) + 1;
    const char *fa[5], *fp[3], *ca[3], *cp[3];
#pragma unroll
    for (int r = 0; r < 5; ++r) fa[r] = ring + RP_FA + ((y + r) & 7) * FROW_B + px * 4;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        fp[r] = ring + RP_FP + ((y + r) & 7) * FROW_B + px * 4;
        ca[r] = ring + RP_CA + ((c1 + r) & 7) * CROW_B + (px >> 1) * 4;
        cp[r] = ring + RP_CP + ((c1 + r) & 7) * CROW_B + (px >> 1) * 4;
    }
    const char *nm = ring + RP_NM + ns * 512 + px * 4;
    half8 *e = E + tile * TILE_H8 + H * 32 + j;
    static_for<0, DB16_GROUPS>([&](auto gc) {
        constexpr int g = decltype(gc)::value;
        constexpr int k0 = grp_k0(H, g);
        constexpr int hb = grp_hi(H, g) ? 0 : 2;
        half8 o;
        static_for<0, 8>([&](auto ec) {
            constexpr int k = k0 + decltype(ec)::value;
            const char *b;
            if constexpr (k < 9) b = ca[k / 3] + (k % 3 + 3) * 4;
            else if constexpr (k < 34) b = fa[(k - 9) / 5] + ((k - 9) % 5 + 2) * 4;
            else if constexpr (k < 43) b = cp[(k - 34) / 3] + ((k - 34) % 3 + 3) * 4;
            else if constexpr (k < 55) b = fp[(k - 43) / 5] + ((k - 43) % 5 + 2) * 4;
            else b = nm;
            o[decltype(ec)::value] = *reinterpret_cast<const _Float16 *>(b + hb);
        });
        e[g * 64] = o;
    });
}

// stage timing of k_screen16p (ia_diag_screen_trace): blocks 0 and 300, every wave, per stage
// (< 64) four s_memtime stamps: MFMA waves {barrier arrival, departure, MFMAs issued, close
// done}; expanders {arrival, departure, copies issued + operand written, copies landed}
__device__ unsigned long long *g_pc_trace;
// (the stamps go to LDS, a wave-uniform address, and are copied out at the end: a global
// pointer held across the stage loop pushed G = 11 into spills)
__device__ __forceinline__ void pc_stamp(unsigned long long *tr, int s, int k) {
    if (tr && s < 64) tr[s * 4 + k] = __builtin_readcyclecounter();
}
static std::atomic<bool> g_pc_trace_on{false};   // host side: launch the TRACE instantiation

template <int G, int W>
__device__ __forceinline__ void pc_mfma(half8 *E, int *smin, int nstage, int tps,
                                        const half8 *__restrict__ q16, unsigned long long *tr) {
    constexpr int NS = bal_ns(G, W);
    const int lane = threadIdx.x & 63;
    half8 bq[NS][Q16_GROUPS];
    load_queries<G, W, NS>(q16, bq, lane);
    float mn[NS];
#pragma unroll
    for (int k = 0; k < NS; ++k) mn[k] = FLT_MAX;
    lds_sync();       // the expanders' first windows landed (their first barrier)
    for (int s = 0; s < nstage; ++s) {
        pc_stamp(tr, s, 0);
        lds_sync();   // barrier s: operand s is complete (and operand s - 1 free for s + 1)
        pc_stamp(tr, s, 1);
        stage_mfma_cm<G, W, NS, PC_PIN>(E + (s & 1) * STAGE_H8, bq, mn, lane);
        stage_close<G, W, NS>(s, tps, smin, mn, lane);
        pc_stamp(tr, s, 3);   // (no stamp between: the last fold's accumulator is live there)
    }
    lds_sync();       // the last stage's operand reads done (pairs with the expanders' last)
}

template <int X>
__device__ __forceinline__ void pc_expand(const ImgDb &im, half8 *E, char *ring, const StageMap &sm,
                                          long chunk, int nstage, unsigned long long *tr) {
    const int lane = threadIdx.x & 63;
    // stage 0's whole window, stages 1 and 2's new rows; wait for stages 0 and 1; operand 0
    const WinSrc w0 = win_src(im, stage_lrow(sm, chunk, 0));
    for (int j = X; j < 15; j += 4) {
        const int kind = j < 5 ? 0 : j < 8 ? 1 : j < 11 ? 2 : j < 14 ? 3 : 4;
        const int r = j < 5 ? w0.y + j : j < 8 ? w0.y + j - 5 : j < 11 ? (w0.y >> 1) + 1 + j - 8
                                                                      : (w0.y >> 1) + 1 + j - 11;
        rp_load(im, w0, ring, kind, r, 0, lane);
    }
    WinSrc wl = w0;                      // the last stage whose rows were requested
    int req = 0;
    for (int k = 1; k < PC_AHEAD && k < nstage; ++k) {
        const WinSrc wk = win_src(im, stage_lrow(sm, chunk, k));
        rp_rows<X>(im, wl, wk, ring, k & 3, lane);
        wl = wk;
        req = k;
    }
    if (PC_AHEAD == 3 && req == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(rp_n(X)) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lds_sync();   // every expander's copies of stages 0 and 1 landed
    rp_expand<X>(ring, w0.y, 0, E, lane);
    WinSrc wn = nstage > 1 ? win_src(im, stage_lrow(sm, chunk, 1)) : w0;   // the next to expand
    for (int s = 0; s < nstage; ++s) {
        // barrier s: operand s complete, stage s + 1's rows landed, operand (s + 1) & 1 free
        pc_stamp(tr, s, 0);
        lds_sync();
        pc_stamp(tr, s, 1);
        const bool more = s + PC_AHEAD < nstage;
        if (more) {
            const WinSrc w3 = win_src(im, stage_lrow(sm, chunk, s + PC_AHEAD));
            rp_rows<X>(im, wl, w3, ring, (s + PC_AHEAD) & 3, lane);
            wl = w3;
        }
        if (s + 1 < nstage) {
            rp_expand<X>(ring, wn.y, (s + 1) & 3, E + ((s + 1) & 1) * STAGE_H8, lane);
            if (s + 2 < nstage) wn = win_src(im, stage_lrow(sm, chunk, s + 2));
        }
        pc_stamp(tr, s, 2);
        // stage s + 2's rows (requested one iteration ago) land before barrier s + 1
        if (PC_AHEAD == 3 && more) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(rp_n(X)) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        pc_stamp(tr, s, 3);
    }
    lds_sync();
}

template <int G, bool TRACE = false>
__global__ __launch_bounds__(512, 1) void k_screen16p(ImgDb im, int nchunks, int ch, int seg_rows,
                                                      StageMap sm, const half8 *__restrict__ q16,
                                                      int M, int groups, float *__restrict__ segmin,
                                                      long nseg, const XJob *jobs, int parity) {
    __shared__ half8 E[2 * STAGE_H8];
    if (jobs) {   // batch: this job's image-form sections, query rows and minima
        const XJob &J = jobs[blockIdx.y];
        im.fa = J.fa; im.ca = J.ca; im.norm = J.norm; im.ap = J.ap;
        q16 = reinterpret_cast<const half8 *>(J.q16[parity].get());
        segmin = J.segmin;
    }
    __shared__ __attribute__((aligned(16))) char ring[RP_B];
    __shared__ int smin[SPC_MAX * G * 32];
    const int b = blockIdx.x;
    const int slot = b >> 3;
    const int chunk = (slot / groups) * 8 + (b & 7);
    const int group = slot - (slot / groups) * groups;
    if (chunk >= nchunks) return;   // uniform over the block, before any barrier
    const int spc = ch / seg_rows;
    for (int i = threadIdx.x; i < spc * G * 32; i += 512) smin[i] = 0x7fffffff;
    const int nstage = ch / (STAGE_TILES * 32);
    const int tps = seg_rows >> 5;
    const half8 *qg = q16 + (long)group * G * 32 * Q16_ROW;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // waves 0-3 and 4-7 pair up on the SIMDs (wave w and w + 4 share SIMD w % 4)
    // stage stamps (TRACE instantiation only): per wave 256 u64 in LDS, copied out below
    __shared__ unsigned long long trs[TRACE ? 8 * 256 : 1];
    unsigned long long *tr = TRACE && (b == 0 || b == 300) ? trs + wv * 256 : nullptr;
    if (IA_PC_PRIO && wv < 4) __builtin_amdgcn_s_setprio(IA_PC_PRIO);
    if (wv == 0) pc_mfma<G, 0>(E, smin, nstage, tps, qg, tr);
    else if (wv == 1) pc_mfma<G, 1>(E, smin, nstage, tps, qg, tr);
    else if (wv == 2) pc_mfma<G, 2>(E, smin, nstage, tps, qg, tr);
    else if (wv == 3) pc_mfma<G, 3>(E, smin, nstage, tps, qg, tr);
    else if (wv == 4) pc_expand<0>(im, E, ring, sm, chunk, nstage, tr);
    else if (wv == 5) pc_expand<1>(im, E, ring, sm, chunk, nstage, tr);
    else if (wv == 6) pc_expand<2>(im, E, ring, sm, chunk, nstage, tr);
    else pc_expand<3>(im, E, ring, sm, chunk, nstage, tr);
    __syncthreads();
    if (TRACE && (b == 0 || b == 300) && g_pc_trace)
        for (int i = threadIdx.x; i < 8 * 256; i += 512) g_pc_trace[(b == 0 ? 0 : 8 * 256) + i] = trs[i];
    const long seg0 = (long)chunk * spc;
    const int q0 = group * G * 32;
    for (int i = threadIdx.x; i < G * 32 * spc; i += 512) {
        const int ql = i / spc, sg = i - ql * spc;
        if (q0 + ql < M) segmin[(long)(q0 + ql) * nseg + seg0 + sg] = fkey_inv(smin[sg * (G * 32) + ql]);
    }
}

// grid: (nchunks rounded up to 8) x groups, XCD-aware: all groups of a chunk share
// blockIdx % 8 (one XCD under round-robin dispatch), so the chunk is fetched from HBM once
// per launch.  Group g holds query tiles [g G, g G + G).
template <int G, int SCHED>
__global__ __launch_bounds__(256, 2) void k_screen16(const half8 *__restrict__ db16, int nchunks,
                                                     int ch, int seg_rows, StageMap sm,
                                                     const half8 *__restrict__ q16, int M,
                                                     int groups, float *__restrict__ segmin,
                                                     long nseg, const XJob *jobs, int parity) {
    __shared__ half8 sbuf[2 * STAGE_H8];
    if (jobs) {   // batch: this job's DB, query rows and minima
        const XJob &J = jobs[blockIdx.y];
        db16 = reinterpret_cast<const half8 *>(J.db.get());
        q16 = reinterpret_cast<const half8 *>(J.q16[parity].get());
        segmin = J.segmin;
    }
    __shared__ int smin[SPC_MAX * G * 32];
    const int b = blockIdx.x;
    const int slot = b >> 3;
    const int chunk = (slot / groups) * 8 + (b & 7);
    const int group = slot - (slot / groups) * groups;
    if (chunk >= nchunks) return;   // uniform over the block, before any barrier
    const int spc = ch / seg_rows;
    for (int i = threadIdx.x; i < spc * G * 32; i += 256) smin[i] = 0x7fffffff;
    const int nstage = ch / (STAGE_TILES * 32);
    const int tps = seg_rows >> 5;
    const half8 *qg = q16 + (long)group * G * 32 * Q16_ROW;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (wv == 0) chain_body<SCHED, G, 0>(db16, sbuf, smin, sm, chunk, nstage, tps, qg);
    else if (wv == 1) chain_body<SCHED, G, 1>(db16, sbuf, smin, sm, chunk, nstage, tps, qg);
    else if (wv == 2) chain_body<SCHED, G, 2>(db16, sbuf, smin, sm, chunk, nstage, tps, qg);
    else chain_body<SCHED, G, 3>(db16, sbuf, smin, sm, chunk, nstage, tps, qg);
    __syncthreads();
    // the chunk's minima, spc consecutive segments per query
    const long seg0 = (long)chunk * spc;
    const int q0 = group * G * 32;
    for (int i = threadIdx.x; i < G * 32 * spc; i += 256) {
        const int ql = i / spc, s = i - ql * spc;
        if (q0 + ql < M) segmin[(long)(q0 + ql) * nseg + seg0 + s] = fkey_inv(smin[s * (G * 32) + ql]);
    }
}

template <int G, int SCHED>
__global__ __launch_bounds__(256, 2) void k_screen16i(ImgDb im, int nchunks, int ch, int seg_rows,
                                                      StageMap sm,
                                                      const half8 *__restrict__ q16, int M,
                                                      int groups, float *__restrict__ segmin,
                                                      long nseg, const XJob *jobs, int parity) {
    __shared__ half8 E[STAGE_H8];
    if (jobs) {   // batch: this job's image-form sections, query rows and minima
        const XJob &J = jobs[blockIdx.y];
        im.fa = J.fa; im.ca = J.ca; im.norm = J.norm; im.ap = J.ap;
        q16 = reinterpret_cast<const half8 *>(J.q16[parity].get());
        segmin = J.segmin;
    }
    static_assert(RW_B <= 2 * WIN_B, "the rings fit the window buffers");
    __shared__ __attribute__((aligned(16))) char wbuf[2 * WIN_B];
    __shared__ int smin[SPC_MAX * G * 32];
    const int b = blockIdx.x;
    const int slot = b >> 3;
    const int chunk = (slot / groups) * 8 + (b & 7);
    const int group = slot - (slot / groups) * groups;
    if (chunk >= nchunks) return;   // uniform over the block, before any barrier
    const int spc = ch / seg_rows;
    for (int i = threadIdx.x; i < spc * G * 32; i += 256) smin[i] = 0x7fffffff;
    const int nstage = ch / (STAGE_TILES * 32);
    const int tps = seg_rows >> 5;
    const half8 *qg = q16 + (long)group * G * 32 * Q16_ROW;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (sm.W > 0) {   // strips: the rolling window (wbuf holds the rings)
        if (wv == 0) strip_body<SCHED, G, 0>(im, E, wbuf, smin, sm, chunk, nstage, tps, qg);
        else if (wv == 1) strip_body<SCHED, G, 1>(im, E, wbuf, smin, sm, chunk, nstage, tps, qg);
        else if (wv == 2) strip_body<SCHED, G, 2>(im, E, wbuf, smin, sm, chunk, nstage, tps, qg);
        else strip_body<SCHED, G, 3>(im, E, wbuf, smin, sm, chunk, nstage, tps, qg);
    } else {
        if (wv == 0) img_body<SCHED, G, 0>(im, E, wbuf, smin, sm, chunk, nstage, tps, qg);
        else if (wv == 1) img_body<SCHED, G, 1>(im, E, wbuf, smin, sm, chunk, nstage, tps, qg);
        else if (wv == 2) img_body<SCHED, G, 2>(im, E, wbuf, smin, sm, chunk, nstage, tps, qg);
        else img_body<SCHED, G, 3>(im, E, wbuf, smin, sm, chunk, nstage, tps, qg);
    }
    __syncthreads();
    // the chunk's minima, spc consecutive segments per query (as k_screen16)
    const long seg0 = (long)chunk * spc;
    const int q0 = group * G * 32;
    for (int i = threadIdx.x; i < G * 32 * spc; i += 256) {
        const int ql = i / spc, sg = i - ql * spc;
        if (q0 + ql < M) segmin[(long)(q0 + ql) * nseg + seg0 + sg] = fkey_inv(smin[sg * (G * 32) + ql]);
    }
}

// query tiles per launch group: T tiles in ceil(T / 11) equal groups
static inline int screen_groups(int T) { return (T + MAX_G - 1) / MAX_G; }

// the stage's MFMA schedule (IA_SCREEN_SCHED / ia_diag_set_screen_sched): 0 tile-major (one
// accumulator per chain of the tile, folds after the tile), 1 chain-major pipelined
static std::atomic<int> g_screen_sched{-1};
static int screen_sched() {
    int v = g_screen_sched.load();
    if (v < 0) {
        v = env_int("IA_SCREEN_SCHED", 0) ? 1 : 0;
        g_screen_sched.store(v);
    }
    return v;
}
// strip-order image-form levels: the producer / consumer kernel k_screen16p (IA_SCREEN_PC /
// ia_diag_set_screen_pc: 1) or k_screen16i's 4-wave body (0)
static std::atomic<int> g_screen_pc{-1};
static int screen_pc() {
    int v = g_screen_pc.load();
    if (v < 0) {
        v = env_int("IA_SCREEN_PC", 1) ? 1 : 0;
        g_screen_pc.store(v);
    }
    return v;
}

int launch_screen16(const void *db, const ImgDb *img, long nrows, const StageMap &sm,
                    const _Float16 *q16, int M, float *segmin, hipStream_t st, const XJob *jobs,
                    int njobs, int parity, bool sharded) {
    const int ch = db_chunk_rows(nrows);
    const long nchunks = db_nchunks(nrows);
    const int seg_rows = db_seg_rows(nrows);
    const long nseg = db_nsegs(nrows);
    IA_ARG(M > 0 && ch % (STAGE_TILES * 32) == 0 && seg_rows % (STAGE_TILES * 32) == 0 &&
               ch / seg_rows <= SPC_MAX,
           "launch_screen16: bad chunking");
    IA_ARG(!img || db_rows_padded(nrows) == nrows, "launch_screen16: image form needs whole chunks");
    IA_ARG(sm.sc == ch / 128, "launch_screen16: stage map of another chunking");
    const half8 *db16 = reinterpret_cast<const half8 *>(db);
    const half8 *q = reinterpret_cast<const half8 *>(q16);
    const int T = (M + 31) / 32;
    const int groups = screen_groups(T);
    const int G = (T + groups - 1) / groups;
    const long nb = ((nchunks + 7) / 8) * 8 * groups;
    IA_ARG(nb < (1L << 31), "screen grid too large");
    IA_ARG(njobs >= 1 && njobs <= IA_BATCH_MAX && (njobs == 1 || jobs), "launch_screen16: bad batch");
    const dim3 grid((unsigned)nb, (unsigned)njobs);
    const int sched = screen_sched();
    // (not for a batch of jobs: its one-per-CU workgroups ran c5 19% slower than the 4-wave
    // screen, 7.59 vs 9.04 M px/s on one box, profiles/r04_ab_c5_screen_pc.txt)
    const bool pc = img && sm.W > 0 && !sharded && njobs == 1 && screen_pc();
#define IA_SCREEN16_SCHED(GG, SS)                                                               \
    if (img)                                                                                    \
        k_screen16i<GG, SS><<<grid, 256, 0, st>>>(*img, (int)nchunks, ch, seg_rows, sm, q, M,  \
                                                  groups, segmin, nseg, jobs, parity);          \
    else                                                                                        \
        k_screen16<GG, SS><<<grid, 256, 0, st>>>(db16, (int)nchunks, ch, seg_rows, sm, q, M,   \
                                                 groups, segmin, nseg, jobs, parity);
#define IA_SCREEN16_CASE(GG)                                                                    \
    case GG:                                                                                    \
        if (pc && (GG == 11 || GG == 4) && g_pc_trace_on.load())                                \
            k_screen16p<GG, (GG == 11 || GG == 4)><<<grid, 512, 0, st>>>(                       \
                *img, (int)nchunks, ch, seg_rows, sm, q, M, groups, segmin, nseg, jobs, parity);\
        else if (pc)                                                                            \
            k_screen16p<GG><<<grid, 512, 0, st>>>(*img, (int)nchunks, ch, seg_rows, sm, q, M,  \
                                                  groups, segmin, nseg, jobs, parity);          \
        else if (sched) { IA_SCREEN16_SCHED(GG, 1) } else { IA_SCREEN16_SCHED(GG, 0) }          \
        break;
    switch (G) {
        IA_SCREEN16_CASE(1)
        IA_SCREEN16_CASE(2)
        IA_SCREEN16_CASE(3)
        IA_SCREEN16_CASE(4)
        IA_SCREEN16_CASE(5)
        IA_SCREEN16_CASE(6)
        IA_SCREEN16_CASE(7)
        IA_SCREEN16_CASE(8)
        IA_SCREEN16_CASE(9)
        IA_SCREEN16_CASE(10)
        IA_SCREEN16_CASE(11)
        default: set_error("launch_screen16: bad query split"); return IA_E_ARG;
    }
#undef IA_SCREEN16_CASE
#undef IA_SCREEN16_SCHED
    IA_LAUNCH_CHECK("k_screen16");
    return IA_OK;
}

}  // namespace ia

namespace ia {
int screen16i_attributes(hipFuncAttributes *at) {
    IA_HIP(hipFuncGetAttributes(at, reinterpret_cast<const void *>(&k_screen16i<11, 0>)));
    return IA_OK;
}
// the 4-wave screen a sharded level launches (launch_screen16, sharded): the image form
// k_screen16i or the row form k_screen16, widest instance (G = 11)
int screen16_attributes(bool img, hipFuncAttributes *at) {
    if (img) return screen16i_attributes(at);
    IA_HIP(hipFuncGetAttributes(at, reinterpret_cast<const void *>(&k_screen16<11, 0>)));
    return IA_OK;
}
}  // namespace ia

extern "C" int ia_diag_set_screen_sched(int sched) {
    const int prev = ia::screen_sched();
    if (sched >= 0 && sched <= 1) ia::g_screen_sched.store(sched);
    return prev;
}

extern "C" int ia_diag_screen_trace(void *buf) {
    unsigned long long *p = reinterpret_cast<unsigned long long *>(buf);
    IA_HIP(hipMemcpyToSymbol(HIP_SYMBOL(ia::g_pc_trace), &p, sizeof(p), 0, hipMemcpyHostToDevice));
    ia::g_pc_trace_on.store(p != nullptr);
    return IA_OK;
}

extern "C" int ia_diag_set_screen_pc(int on) {
    const int prev = ia::screen_pc();
    if (on >= 0 && on <= 1) ia::g_screen_pc.store(on);
    return prev;
}

namespace ia {

}  // namespace ia
