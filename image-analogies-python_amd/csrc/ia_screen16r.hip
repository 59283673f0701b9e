// ia_screen16r.hip — the rotated split-f16 screen (R16, ia_rot16.h): the
// level's rotation (covariance of the centred rows, ia_db_cov; the eigenvectors are taken
// on the host), the rotated database (ia_db_build_rot: R16_ROW_B bytes per row, R16_MFMA
// operand groups per 32-row tile: 128 B and 4 at the default P = 3) and the screen
// k_screen16r: at P = 3 (the default, IA_R16_SHAPE = 16) two v_mfma_f32_16x16x32_f16 per
// 16 x 16 (rows x queries) block, else R16_MFMA v_mfma_f32_32x32x16_f16 per 32x32 tile (the
// split-f16 screen of ia_screen16.hip needs 11), same segment minima units, so the exact stage
// (k_xstrip) is unchanged apart from its bound (ia_rot16.h r16_eps, per shape).
//
// The screen's structure is the row form's of ia_screen16.hip (k_screen16): queries are the
// stationary MFMA B operand (half8 per query block and lane); the DB streams through LDS in
// 4-tile stages (16 KiB at P = 3, global_load_lds_dwordx4, non-temporal, a ring of 3 buffers,
// one LDS-only barrier per stage) and every byte fetched feeds the block's 4 waves; the
// stage's (query block, row block) chains are cut into 4 equal runs (chain balance), each
// chain's MFMAs run back to back and its running-minimum fold is taken a few chains later
// (no MFMA -> VALU hazard pads), interleaved with the later chains' MFMAs; minima staged in
// LDS 8 segments at a time.
#include "ia_internal.h"
#include "ia_rot16.h"

#include <float.h>
#include <type_traits>

namespace ia {
namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));
constexpr int STAGE_TILES = 4;
constexpr int STAGE_H8 = STAGE_TILES * R16_TILE_H8;   // 16 KiB (P = 3)
constexpr int MAX_G = 11;
constexpr int SPC_MAX = 16;
// stage buffers (r16_body) and blocks per CU the kernel is built for (A/B builds)
#ifndef IA_R16_RING
#define IA_R16_RING 2
#endif
#ifndef IA_R16_OCC
#define IA_R16_OCC 4
#endif
constexpr int R16_RING = IA_R16_RING;
// (Round 5's lab builds that skipped loads, barriers, folds or operand reads to time the
// kernel's floors broke the minima; they are not part of this source: every knob left here
// keeps the minima bit-identical, tests/test_gpu_rot16.py.)
#ifndef IA_R16_NTMIN
#define IA_R16_NTMIN 0   // segment minima written non-temporally (less dirty L2 at the kernel's end)
#endif
// the stage's instruction order: 1 pins each chain as MFMA, 2 VALU of the previous chain's
// fold, MFMA, ... (sched_group_barrier), 0 leaves it to the compiler
#ifndef IA_R16_PIN
#define IA_R16_PIN 1
#endif
#ifndef IA_R16_SPC
#define IA_R16_SPC 2
#endif
constexpr int SPC_STAGE = IA_R16_SPC;   // segments of minima staged in LDS at a time

// chain balance (as ia_screen16.hip): the 4G chains of a stage in the order 4t + u cut into
// 4 equal runs of G, one per wave
__host__ __device__ constexpr int bal_t0(int G, int W) { return (G * W) / 4; }
__host__ __device__ constexpr int bal_ns(int G, int W) { return (G * W + G - 1) / 4 - (G * W) / 4 + 1; }
__host__ __device__ constexpr bool bal_on(int G, int W, int k, int u) {
    return 4 * (bal_t0(G, W) + k) + u >= G * W && 4 * (bal_t0(G, W) + k) + u < G * W + G;
}
template <int G, int W>
__host__ __device__ constexpr int ch_count() {
    int n = 0;
    for (int u = 0; u < STAGE_TILES; ++u)
        for (int k = 0; k < bal_ns(G, W); ++k) n += bal_on(G, W, k, u) ? 1 : 0;
    return n;
}
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
template <int G, int W>
__host__ __device__ constexpr int ch_uo(int c) {
    int o = 0;
    for (int i = 1; i <= c; ++i) o += ch_u<G, W>(i) != ch_u<G, W>(i - 1) ? 1 : 0;
    return o;
}
// the first chain after chain c's tile run (the next tile's first chain), or -1
template <int G, int W>
__host__ __device__ constexpr int ch_next(int c) {
    for (int i = c + 1; i < ch_count<G, W>(); ++i)
        if (ch_u<G, W>(i) != ch_u<G, W>(c)) return i;
    return -1;
}
// chain c starts a tile run
template <int G, int W>
__host__ __device__ constexpr bool ch_first(int c) { return c == 0 || ch_u<G, W>(c) != ch_u<G, W>(c - 1); }
// when the next tile's operands are read from LDS: 1 at the first chain of the current tile's
// run (2-3 chains ahead), 0 at its last chain (one chain ahead)
#ifndef IA_R16_PF
#define IA_R16_PF 1
#endif
template <int G, int W>
__host__ __device__ constexpr bool ch_reads_next(int c) {
    return IA_R16_PF ? (ch_first<G, W>(c) && ch_next<G, W>(c) >= 0)
                     : (c + 1 < ch_count<G, W>() && ch_u<G, W>(c + 1) != ch_u<G, W>(c));
}
template <int K, int N, typename F>
__device__ __forceinline__ void sfor(F &&f) {
    if constexpr (K < N) {
        f(std::integral_constant<int, K>{});
        sfor<K + 1, N>(f);
    }
}
__device__ __forceinline__ int fkey(float x) {
    const int b = __float_as_int(x);
    return b >= 0 ? b : b ^ 0x7fffffff;
}
__device__ __forceinline__ float fkey_inv(int b) { return __int_as_float(b >= 0 ? b : b ^ 0x7fffffff); }
__device__ __forceinline__ void fold_min(const floatx16 &x, float &mn) {
    const float t0 = fminf(fminf(x[0], x[1]), x[2]), t1 = fminf(fminf(x[3], x[4]), x[5]);
    const float t2 = fminf(fminf(x[6], x[7]), x[8]), t3 = fminf(fminf(x[9], x[10]), x[11]);
    const float t4 = fminf(fminf(x[12], x[13]), x[14]);
    const float u0 = fminf(fminf(t0, t1), t2), u1 = fminf(fminf(t3, t4), x[15]);
    mn = fminf(fminf(mn, u0), u1);
}

// the chain whose accumulator chain c's MFMAs fold (IA_R16_LAG = 1: the previous chain, right
// after its last MFMA (the compiler pads the MFMA -> VALU hazard with s_nop); 2: the one before,
// with one more accumulator, far enough back that no pad is needed)
#ifndef IA_R16_LAG
#define IA_R16_LAG 2
#endif
constexpr int R16_NACC = IA_R16_LAG + 1;

// wave W's chains of one stage (operand sb in LDS), chain-major with two operand sets
template <int G, int W, int NS>
__device__ __forceinline__ void r16_stage(const half8 *sb, const half8 (&bq)[NS][R16_MFMA], float (&mn)[NS],
                                          int lane) {
    constexpr int NC = ch_count<G, W>();
    const floatx16 zero = {};
    half8 a[2][R16_MFMA];
    floatx16 acc[R16_NACC];
    {
        const half8 *p = sb + ch_u<G, W>(0) * R16_TILE_H8 + lane;
#pragma unroll
        for (int m = 0; m < R16_MFMA; ++m) a[0][m] = p[m * 64];
    }
    sfor<0, NC>([&](auto cc) {
        constexpr int c = decltype(cc)::value;
        constexpr int k = ch_k<G, W>(c), ab = ch_uo<G, W>(c) & 1, cb = c % R16_NACC;
        constexpr int cf = c - IA_R16_LAG, fb = (c + 1) % R16_NACC;   // the chain folded here
        if constexpr (ch_reads_next<G, W>(c)) {
            const half8 *p = sb + ch_u<G, W>(ch_next<G, W>(c)) * R16_TILE_H8 + lane;
#pragma unroll
            for (int m = 0; m < R16_MFMA; ++m) a[ab ^ 1][m] = p[m * 64];
        }
        acc[cb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[ab][0], bq[k][0], zero, 0, 0, 0);
        if constexpr (cf >= 0) fold_min(acc[fb], mn[ch_k<G, W>(cf)]);
#pragma unroll
        for (int m = 1; m < R16_MFMA; ++m)
            acc[cb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[ab][m], bq[k][m], acc[cb], 0, 0, 0);
        if constexpr (IA_R16_PIN) {
            // [the next tile's 5 operand reads,] MFMA 0, then the previous chain's fold two
            // VALU at a time between the remaining MFMAs
            if constexpr (ch_reads_next<G, W>(c))
                __builtin_amdgcn_sched_group_barrier(0x100, R16_MFMA, 0);   // DS reads
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);              // MFMA
            if constexpr (cf >= 0) {
                sfor<0, R16_MFMA - 1>([&](auto) {
                    __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);      // VALU
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);      // MFMA
                });
            } else {
                __builtin_amdgcn_sched_group_barrier(0x008, R16_MFMA - 1, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    });
    sfor<(NC > IA_R16_LAG ? NC - IA_R16_LAG : 0), NC>([&](auto cc) {
        constexpr int c = decltype(cc)::value;
        fold_min(acc[c % R16_NACC], mn[ch_k<G, W>(c)]);
    });
}

// ---- the 16x16x32 form (IA_R16_SHAPE = 16): v_mfma_f32_16x16x32_f16, 2 per 16x16 (rows x
// queries) block at K = 64 slots.  Same DB stages and LDS layout (a lane's 8 slots of a row are
// one half8 of the 32x32 layout), same units and minima.  Per stage 8 row blocks (v: tile v / 2,
// rows 16 (v % 2) ..) x 2G query blocks of 16; the 16 G chains (t, v), order 8t + v, are cut
// into 4 equal runs, one per wave (as bal_*), each run walked row-block-major so that a row
// block's two operand reads serve all its chains.  Output: lane l holds rows 4 (l / 16) .. + 3
// of query l % 16, folded per lane, reduced over the 4 lane groups at each segment close.
typedef float floatx4 __attribute__((ext_vector_type(4)));
template <int G, int W>
__host__ __device__ constexpr int c16_lo() { return 4 * G * W; }   // first chain of wave W
template <int G, int W>
__host__ __device__ constexpr int c16_t0() { return c16_lo<G, W>() / 8; }
template <int G, int W>
__host__ __device__ constexpr int c16_ns() { return (c16_lo<G, W>() + 4 * G - 1) / 8 - c16_t0<G, W>() + 1; }
template <int G, int W>
__host__ __device__ constexpr bool c16_on(int k, int v) {
    return 8 * (c16_t0<G, W>() + k) + v >= c16_lo<G, W>() && 8 * (c16_t0<G, W>() + k) + v < c16_lo<G, W>() + 4 * G;
}
template <int G, int W>
__host__ __device__ constexpr int c16_count() { return 4 * G; }
template <int G, int W>
__host__ __device__ constexpr int c16_v(int c) {
    for (int v = 0; v < 8; ++v)
        for (int k = 0; k < c16_ns<G, W>(); ++k)
            if (c16_on<G, W>(k, v) && c-- == 0) return v;
    return -1;
}
template <int G, int W>
__host__ __device__ constexpr int c16_k(int c) {
    for (int v = 0; v < 8; ++v)
        for (int k = 0; k < c16_ns<G, W>(); ++k)
            if (c16_on<G, W>(k, v) && c-- == 0) return k;
    return -1;
}
template <int G, int W>
__host__ __device__ constexpr int c16_vo(int c) {   // row blocks started before chain c
    int o = 0;
    for (int i = 1; i <= c; ++i) o += c16_v<G, W>(i) != c16_v<G, W>(i - 1) ? 1 : 0;
    return o;
}
template <int G, int W>
__host__ __device__ constexpr int c16_next(int c) {
    for (int i = c + 1; i < c16_count<G, W>(); ++i)
        if (c16_v<G, W>(i) != c16_v<G, W>(c)) return i;
    return -1;
}
template <int G, int W>
__host__ __device__ constexpr bool c16_first(int c) { return c == 0 || c16_v<G, W>(c) != c16_v<G, W>(c - 1); }
// half8 offset (in a stage) of lane l's operand of MFMA n for row block v: row 16 (v % 2) +
// l % 16 of tile v / 2, slots 32 n + 8 (l / 16) .. + 7 = 32x32 group 2n + (l / 16) / 2, half
// (l / 16) % 2
__device__ __forceinline__ int s16_aoff(int v, int n, int lane) {
    const int q = lane >> 4, r = lane & 15;
    return (v >> 1) * R16_TILE_H8 + ((2 * n + (q >> 1)) * 64 + (q & 1) * 32 + 16 * (v & 1) + r);
}
constexpr int S16_LAG = 3;   // chain c folds chain c - S16_LAG (no MFMA -> VALU pads)
constexpr int S16_NACC = S16_LAG + 1;

template <int G, int W, int NS>
__device__ __forceinline__ void r16_stage_s16(const half8 *sb, const half8 (&bq)[NS][2], float (&mn)[NS], int lane) {
    constexpr int NC = c16_count<G, W>();
    const floatx4 zero = {};
    half8 a[2][2];
    floatx4 acc[S16_NACC];
    a[0][0] = sb[s16_aoff(c16_v<G, W>(0), 0, lane)];
    a[0][1] = sb[s16_aoff(c16_v<G, W>(0), 1, lane)];
    sfor<0, NC>([&](auto cc) {
        constexpr int c = decltype(cc)::value;
        constexpr int k = c16_k<G, W>(c), ab = c16_vo<G, W>(c) & 1, cb = c % S16_NACC;
        constexpr int cf = c - S16_LAG, fb = (c + 1) % S16_NACC;
        constexpr bool rd = c16_first<G, W>(c) && c16_next<G, W>(c) >= 0;
        if constexpr (rd) {
            constexpr int vn = c16_v<G, W>(c16_next<G, W>(c));
            a[ab ^ 1][0] = sb[s16_aoff(vn, 0, lane)];
            a[ab ^ 1][1] = sb[s16_aoff(vn, 1, lane)];
        }
        acc[cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[ab][0], bq[k][0], zero, 0, 0, 0);
        if constexpr (cf >= 0) mn[c16_k<G, W>(cf)] = fminf(mn[c16_k<G, W>(cf)], fminf(acc[fb][0], acc[fb][1]));
        acc[cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[ab][1], bq[k][1], acc[cb], 0, 0, 0);
        if constexpr (cf >= 0) mn[c16_k<G, W>(cf)] = fminf(mn[c16_k<G, W>(cf)], fminf(acc[fb][2], acc[fb][3]));
        if constexpr (IA_R16_PIN) {
            if constexpr (rd) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);   // DS reads
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                     // MFMA
            if constexpr (cf >= 0) __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            if constexpr (cf >= 0) __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);
            __builtin_amdgcn_sched_barrier(0);
        }
    });
    sfor<(NC > S16_LAG ? NC - S16_LAG : 0), NC>([&](auto cc) {
        constexpr int c = decltype(cc)::value;
        const floatx4 &x = acc[c % S16_NACC];
        mn[c16_k<G, W>(c)] = fminf(fminf(mn[c16_k<G, W>(c)], fminf(x[0], x[1])), fminf(x[2], x[3]));
    });
}

// LDS integer min as inline asm: the compiler's waitcnt pass treats an LDS atomic as a store
// that may alias the DB stages' LDS-DMA destination and drains every stage in flight before
// it (s_waitcnt vmcnt(0) at each segment close); smin and the stage ring never overlap
__device__ __forceinline__ void lds_min_i32(int *p, int v) {
    typedef __attribute__((address_space(3))) int lds_int;
    const unsigned a = (unsigned)(unsigned long)(lds_int *)p;
    asm volatile("ds_min_i32 %0, %1" :: "v"(a), "v"(v) : "memory");
}

template <int G, int W, int NS>
__device__ __forceinline__ void r16_close(int s, int tps, int *smin, float (&mn)[NS], int lane) {
    constexpr int T0 = bal_t0(G, W);
    const int done = (s + 1) * STAGE_TILES;
    if (done % tps == 0) {
        int *sm = smin + ((done / tps - 1) % SPC_STAGE) * (G * 32);
        const int j = lane & 31, h = lane >> 5;
#pragma unroll
        for (int k = 0; k < NS; ++k) {
            const float m = fminf(mn[k], __shfl_xor(mn[k], 32));
            if (h == 0) lds_min_i32(&sm[(T0 + k) * 32 + j], fkey(m));
            mn[k] = FLT_MAX;
        }
    }
}
template <int G, int W, int NS>
__device__ __forceinline__ void r16_close_s16(int s, int tps, int *smin, float (&mn)[NS], int lane) {
    constexpr int T0 = c16_t0<G, W>();
    const int done = (s + 1) * STAGE_TILES;
    if (done % tps == 0) {
        int *sm = smin + ((done / tps - 1) % SPC_STAGE) * (G * 32);
#pragma unroll
        for (int k = 0; k < NS; ++k) {
            float m = fminf(mn[k], __shfl_xor(mn[k], 16));
            m = fminf(m, __shfl_xor(m, 32));
            if (lane < 16) lds_min_i32(&sm[(T0 + k) * 16 + lane], fkey(m));
            mn[k] = FLT_MAX;
        }
    }
}

// a workgroup barrier that orders LDS only: __syncthreads()'s release fence would also wait
// for every DB stage in flight (s_waitcnt vmcnt(0)), i.e. collapse the ring to one stage.
// The caller has waited for the DMA stages the others must see (vmcnt) before it.
__device__ __forceinline__ void stage_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// The DB stream needs ~60 KB in flight per CU to keep the MFMA pipe fed at HBM latency
// (11.6 B per cycle and CU at full rate), so stages land in a ring of R16_RING buffers,
// R16_RING - 1 stages ahead (2 blocks per CU: 80 KB in flight), and the chunk's segment
// minima are staged for SPC_STAGE segments at a time (flushed to segmin as soon as they
// close) to leave the LDS for the ring.

template <int G, int W>
__device__ __forceinline__ void r16_body(const half8 *__restrict__ db16, half8 *sbuf, int *smin,
                                         const StageMap &sm, long chunk, int s0, int nstage, int tps,
                                         const half8 *__restrict__ q16, float *__restrict__ segmin,
                                         long seg0, long nseg, int q0, int M) {
    constexpr int NS = R16_S16 ? c16_ns<G, W>() : bal_ns(G, W);
    constexpr int T0 = bal_t0(G, W);
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    half8 bq[NS][R16_S16 ? 2 : R16_MFMA];
    if constexpr (R16_S16) {
        // query block T + k, lane l: query 16 (T + k) + l % 16, slots 32 n + 8 (l / 16) .. + 7,
        // i.e. the half8 (l / 16) % 2 * R16_MFMA + 2n + (l / 16) / 2 of its q16 row
        const int q = lane >> 4, c = lane & 15;
#pragma unroll
        for (int k = 0; k < NS; ++k) {
            const half8 *p = q16 + (long)((c16_t0<G, W>() + k) * 16 + c) * Q16_ROW + (q & 1) * R16_MFMA + (q >> 1);
            bq[k][0] = p[0];
            bq[k][1] = p[2];
        }
    } else {
        const int j = lane & 31, h = lane >> 5;
#pragma unroll
        for (int k = 0; k < NS; ++k) {
            const half8 *p = q16 + (long)((T0 + k) * 32 + j) * Q16_ROW + h * R16_MFMA;
#pragma unroll
            for (int m = 0; m < R16_MFMA; ++m) bq[k][m] = p[m];
        }
    }
    // one stage = 4 consecutive tiles: 4 R16_MFMA wave-instructions of 1 KiB, R16_MFMA per wave
    auto issue = [&](int s) {
        const half8 *src = db16 + (stage_lrow(sm, chunk, s0 + s) >> 5) * R16_TILE_H8 + W * 64 + lane;
        half8 *dst = sbuf + (s % R16_RING) * STAGE_H8 + W * 64;
#pragma unroll
        for (int k = 0; k < R16_MFMA; ++k)
            __builtin_amdgcn_global_load_lds((const void *)(src + k * 256), (void *)(dst + k * 256), 16, 0, 2);
    };
    float mn[NS];
#pragma unroll
    for (int k = 0; k < NS; ++k) mn[k] = FLT_MAX;
    const int spc = nstage * STAGE_TILES / tps;
#pragma unroll
    for (int s = 0; s < R16_RING - 1; ++s)
        if (s < nstage) issue(s);
    // stage 0 landed (the later stages' loads may stay in flight)
    if (nstage > 1) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(R16_MFMA * (R16_RING - 2)) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    stage_barrier();
    for (int s = 0; s < nstage; ++s) {
        const bool more = s + R16_RING - 1 < nstage;
        if (more) issue(s + R16_RING - 1);   // into the buffer stage s - 1 used (consumed)
        if constexpr (R16_S16) {
            r16_stage_s16<G, W, NS>(sbuf + (s % R16_RING) * STAGE_H8, bq, mn, lane);
            r16_close_s16<G, W, NS>(s, tps, smin, mn, lane);
        } else {
            r16_stage<G, W, NS>(sbuf + (s % R16_RING) * STAGE_H8, bq, mn, lane);
            r16_close<G, W, NS>(s, tps, smin, mn, lane);
        }
        const int done = (s + 1) * STAGE_TILES;
        if (done % tps == 0) {
            const int sg = done / tps - 1;            // the segment this stage closed
            if (sg % SPC_STAGE == SPC_STAGE - 1 || sg == spc - 1) {
                stage_barrier();                      // every wave's minima of these segments
                const int base = sg - sg % SPC_STAGE, n = sg - base + 1;
                for (int i = tid; i < G * 32 * n; i += 256) {
                    const int ql = i / n, k = i - ql * n;
                    int *e = &smin[k * (G * 32) + ql];
                    if (q0 + ql < M) {
                        float *dst = segmin + ((long)(q0 + ql) * nseg + seg0 + base + k);
                        if constexpr (IA_R16_NTMIN) __builtin_nontemporal_store(fkey_inv(*e), dst);
                        else *dst = fkey_inv(*e);
                    }
                    *e = 0x7fffffff;                  // this thread's entries only: no barrier
                }
            }
        }
        // stage s + 1 landed: the R16_RING - 2 stages issued after it may stay in flight
        if (more) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(R16_MFMA * (R16_RING - 2)) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        stage_barrier();   // (every wave's reads of stage s done: its buffer is refilled next)
    }
}

// grid: (nchunks x split rounded up to 8) x groups, XCD-aware (all groups of a part share
// blockIdx % 8); part p = chunk p / split, its stages [(p % split) nstage / split, ...) (a
// whole number of segments: the screen's grid, 4 blocks per CU, independent of the DB's
// chunking); group g holds query tiles [g G, g G + G); grid y = job of a batch
template <int G>
__global__ __launch_bounds__(256, IA_R16_OCC) void k_screen16r(const half8 *__restrict__ db16, int nchunks, int ch,
                                                      int seg_rows, StageMap sm,
                                                      const half8 *__restrict__ q16, int M, int groups,
                                                      float *__restrict__ segmin, long nseg,
                                                      const XJob *jobs, int parity, int split) {
    __shared__ half8 sbuf[R16_RING * STAGE_H8];
    __shared__ int smin[SPC_STAGE * G * 32];
    if (jobs) {
        const XJob &J = jobs[blockIdx.y];
        db16 = reinterpret_cast<const half8 *>(J.dbr.get());
        q16 = reinterpret_cast<const half8 *>(J.q16[parity].get());
        segmin = J.segmin;
    }
    const int b = blockIdx.x;
    const int slot = b >> 3;
    const int part = (slot / groups) * 8 + (b & 7);
    const int group = slot - (slot / groups) * groups;
    if (part >= nchunks * split) return;   // uniform over the block, before any barrier
    const int lsp = __builtin_ctz((unsigned)split);
    const int chunk = part >> lsp, half = part & (split - 1);
    const int spc = ch / seg_rows;
    for (int i = threadIdx.x; i < SPC_STAGE * G * 32; i += 256) smin[i] = 0x7fffffff;
    const int nstage = (ch / (STAGE_TILES * 32)) >> lsp;
    const int tps = seg_rows >> 5;
    const half8 *qg = q16 + (long)group * G * 32 * Q16_ROW;
    const long seg0 = (long)chunk * spc + (long)half * (spc >> lsp);
    const int q0 = group * G * 32;
    const int s0 = half * nstage;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (wv == 0) r16_body<G, 0>(db16, sbuf, smin, sm, chunk, s0, nstage, tps, qg, segmin, seg0, nseg, q0, M);
    else if (wv == 1) r16_body<G, 1>(db16, sbuf, smin, sm, chunk, s0, nstage, tps, qg, segmin, seg0, nseg, q0, M);
    else if (wv == 2) r16_body<G, 2>(db16, sbuf, smin, sm, chunk, s0, nstage, tps, qg, segmin, seg0, nseg, q0, M);
    else r16_body<G, 3>(db16, sbuf, smin, sm, chunk, s0, nstage, tps, qg, segmin, seg0, nseg, q0, M);
}

// ---- the wave-owned form (IA_R16_FORM = 1): DB tiles straight into each wave's registers ----
// The block form above streams every DB byte through LDS (DMA ring, one barrier per 128-row
// stage) so that the block's 4 waves, each holding a quarter of the query blocks in VGPRs,
// share it.  Here the roles are swapped: the block's 8 waves share the QUERIES, staged once
// in LDS in MFMA operand order (2G blocks of 16 x 2 MFMAs x 64 lanes x half8: 44 KiB at
// G = 11), and each wave owns a contiguous run of DB tiles (32 rows, 4 KiB each) that it
// loads straight into its registers (4 x 16 B per lane, the 16x16x32 operands of its two row
// blocks), W_RING tiles in flight.  Per tile: every query block's two half8 read from LDS
// (ds_read_b128, conflict-free), 4 MFMAs (two 16-row blocks x two K = 32 steps), the lagged
// minimum fold.  No DB staging, no per-stage barrier: the waves never wait for each other
// until the block's end.  Segment minima: a wave closing a segment (or its run) reduces its
// lane groups and ds_min's the 16 values per query block into the block's LDS minima
// (waves sharing a segment combine there); after one barrier the block writes runs of spb
// consecutive segments per query.  Same products, same two-MFMA chain per (16 rows, 16
// queries) and the same minima as the block form, bit for bit.
#ifndef IA_R16W_RING
#define IA_R16W_RING 3
#endif
constexpr int W_RING = IA_R16W_RING;   // tiles in flight per wave
constexpr int W_WAVES = 8;             // waves per workgroup
#ifndef IA_R16W_SPB
#define IA_R16W_SPB 16
#endif
constexpr int W_SPB_MAX = IA_R16W_SPB;  // segments per workgroup (LDS minima)
constexpr int W_LAG = 2;               // query blocks between an MFMA pair and its fold

__device__ __forceinline__ void w_fold(const floatx4 &x, const floatx4 &y, float &mn) {
    mn = fminf(fminf(mn, fminf(x[0], x[1])), fminf(fminf(x[2], x[3]), fminf(fminf(y[0], y[1]), fminf(y[2], y[3]))));
}

// one tile (two 16-row blocks: a[0..1] = block 0 MFMA 0..1, a[2..3] = block 1) against the 2G
// query blocks of the LDS operand array qs[(k * 2 + n) * 64 + lane]
template <int NQB>
__device__ __forceinline__ void w_tile(const half8 (&a)[4], const half8 *qs, float (&mn)[NQB], int lane) {
    const floatx4 zero = {};
    half8 bq[2][2];
    floatx4 acc[W_LAG + 1][2];
    bq[0][0] = qs[lane];
    bq[0][1] = qs[64 + lane];
    sfor<0, NQB>([&](auto kk) {
        constexpr int k = decltype(kk)::value, cb = k % (W_LAG + 1), b = k & 1;
        if constexpr (k + 1 < NQB) {
            bq[b ^ 1][0] = qs[((k + 1) * 2) * 64 + lane];
            bq[b ^ 1][1] = qs[((k + 1) * 2 + 1) * 64 + lane];
        }
        acc[cb][0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[0], bq[b][0], zero, 0, 0, 0);
        acc[cb][1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[2], bq[b][0], zero, 0, 0, 0);
        acc[cb][0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[1], bq[b][1], acc[cb][0], 0, 0, 0);
        acc[cb][1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[3], bq[b][1], acc[cb][1], 0, 0, 0);
        if constexpr (k >= W_LAG) {
            constexpr int f = (k - W_LAG) % (W_LAG + 1);
            w_fold(acc[f][0], acc[f][1], mn[k - W_LAG]);
        }
    });
    sfor<(NQB > W_LAG ? NQB - W_LAG : 0), NQB>([&](auto kk) {
        constexpr int k = decltype(kk)::value;
        w_fold(acc[k % (W_LAG + 1)][0], acc[k % (W_LAG + 1)][1], mn[k]);
    });
}

// grid: (segment blocks rounded up to 8) x query groups, XCD-aware (the groups of a segment
// block share blockIdx % 8); grid y = job of a batch.  Block sbk covers segments
// [sbk spb, (sbk + 1) spb); wave w its tiles [w tpw, (w + 1) tpw) (tpw = spb tps / 8).
template <int G>
__global__ __launch_bounds__(512, 4) void k_screen16w(const half8 *__restrict__ db16, int nsb, int spb, int tps,
                                                      int seg_rows, StageMap sm, const half8 *__restrict__ q16,
                                                      int M, int groups, float *__restrict__ segmin, long nseg,
                                                      const XJob *jobs, int parity) {
    constexpr int NQB = 2 * G;
    __shared__ half8 qs[NQB * 2 * 64];
    __shared__ int smin[W_SPB_MAX * NQB * 16];
    if (jobs) {
        const XJob &J = jobs[blockIdx.y];
        db16 = reinterpret_cast<const half8 *>(J.dbr.get());
        q16 = reinterpret_cast<const half8 *>(J.q16[parity].get());
        segmin = J.segmin;
    }
    const int b = blockIdx.x;
    const int slot = b >> 3;
    const int sbk = (slot / groups) * 8 + (b & 7);
    const int group = slot - (slot / groups) * groups;
    if (sbk >= nsb) return;   // uniform over the block, before any barrier
    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    // the group's queries in operand order: block k, MFMA n, lane l -> query 16 k + l % 16,
    // half8 (l / 16) % 2 * R16_MFMA + 2 n + (l / 16) / 2 of its q16 row (as r16_body)
    const half8 *qg = q16 + (long)group * G * 32 * Q16_ROW;
    for (int i = tid; i < NQB * 128; i += 512) {
        const int k = i >> 7, n = (i >> 6) & 1, l = i & 63, lq = l >> 4;
        qs[i] = qg[(long)(k * 16 + (l & 15)) * Q16_ROW + (lq & 1) * R16_MFMA + (lq >> 1) + 2 * n];
    }
    for (int i = tid; i < spb * NQB * 16; i += 512) smin[i] = 0x7fffffff;
    __syncthreads();
    const long seg0 = (long)sbk * spb;
    const int tpw = spb * tps / W_WAVES;
    const int jw = wv * tpw;                       // the wave's first block-local tile
    const int lts = __builtin_ctz((unsigned)tps);  // log2 tiles per segment
    const int q = lane >> 4, r = lane & 15;
    const int o0 = (q >> 1) * 64 + (q & 1) * 32 + r;   // (v, n) -> o0 + n * 128 + v * 16
    // block-local tile j (clamped to the wave's last: the ring's overrun re-reads a line the
    // wave loads anyway) -> its half8 base
    auto tile = [&](int j) -> const half8 * {
        j = j < tpw ? j : tpw - 1;
        const int jj = jw + j;
        const long lrow = seg_lrow(sm, seg0 + (jj >> lts), seg_rows, (long)(jj & (tps - 1)) * 32);
        return db16 + (lrow >> 5) * R16_TILE_H8 + o0;
    };
    half8 a[W_RING][4];
    auto issue = [&](half8 (&d)[4], int j) {
        const half8 *t = tile(j);
        d[0] = __builtin_nontemporal_load(t);
        d[1] = __builtin_nontemporal_load(t + 128);
        d[2] = __builtin_nontemporal_load(t + 16);
        d[3] = __builtin_nontemporal_load(t + 144);
    };
    float mn[NQB];
#pragma unroll
    for (int k = 0; k < NQB; ++k) mn[k] = FLT_MAX;
    sfor<0, W_RING - 1>([&](auto ss) { issue(a[decltype(ss)::value], decltype(ss)::value); });
    for (int j0 = 0; j0 < tpw; j0 += W_RING) {
        sfor<0, W_RING>([&](auto ss) {
            constexpr int s = decltype(ss)::value;
            const int j = j0 + s;
            issue(a[(s + W_RING - 1) % W_RING], j + W_RING - 1);
            if (j < tpw) {
                w_tile<NQB>(a[s], qs, mn, lane);
                const int jj = jw + j;
                if (((jj + 1) & (tps - 1)) == 0 || j + 1 == tpw) {   // the wave leaves a segment
                    int *sm0 = smin + (jj >> lts) * (NQB * 16);
#pragma unroll
                    for (int k = 0; k < NQB; ++k) {
                        float m = fminf(mn[k], __shfl_xor(mn[k], 16));
                        m = fminf(m, __shfl_xor(m, 32));
                        if (lane < 16) lds_min_i32(&sm0[k * 16 + lane], fkey(m));
                        mn[k] = FLT_MAX;
                    }
                }
            }
        });
    }
    stage_barrier();   // every wave's minima in LDS
    const int q0 = group * G * 32;
    for (int i = tid; i < NQB * 16 * spb; i += 512) {
        const int ql = i / spb, k = i - ql * spb;
        if (q0 + ql < M) segmin[(long)(q0 + ql) * nseg + seg0 + k] = fkey_inv(smin[k * (NQB * 16) + ql]);
    }
}

// ---- the level's covariance (ia_db_cov): sampled rows, centred, fp64 -------------------
// Block b takes COV_ROWS sampled rows (row0 + i * step, i = b * COV_ROWS ...), their 55
// centred features into LDS, and the 1540 upper-triangle sums over them into its partial;
// k_db_cov_reduce adds the partials in block order (deterministic).
constexpr int COV_ROWS = 128, COV_PAIRS = 55 * 56 / 2, COV_BLOCKS = 256;
__global__ __launch_bounds__(256) void k_db_cov(DbSrc src, long row0, long nrows, long step, long nsamp,
                                                const double *__restrict__ center, double *__restrict__ part) {
    __shared__ double X[COV_ROWS][IA_DP];
    double acc[(COV_PAIRS + 255) / 256];
#pragma unroll
    for (int i = 0; i < (COV_PAIRS + 255) / 256; ++i) acc[i] = 0.0;
    for (long base = (long)blockIdx.x * COV_ROWS; base < nsamp; base += (long)gridDim.x * COV_ROWS) {
        __syncthreads();
        if (threadIdx.x < COV_ROWS) {
            const long i = base + threadIdx.x;
            double *x = X[threadIdx.x];
            if (i < nsamp) {
                ImgPair ap; int r, c;
                src.locate(row0 + i * step, ap, r, c);
                emit_feature(src.A, ap, r, c, [&](int k, double v) { x[k] = v - center[k]; });
            } else {
                for (int k = 0; k < IA_D; ++k) x[k] = 0.0;
            }
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < (COV_PAIRS + 255) / 256; ++i) {
            const int p = threadIdx.x + 256 * i;
            if (p < COV_PAIRS) {
                // pair p -> (a, b), a <= b: row-major upper triangle
                int a = 0, rem = p;
                while (rem >= 55 - a) { rem -= 55 - a; ++a; }
                const int bb = a + rem;
                double s = 0.0;
                for (int r = 0; r < COV_ROWS; ++r) s += X[r][a] * X[r][bb];
                acc[i] += s;
            }
        }
    }
#pragma unroll
    for (int i = 0; i < (COV_PAIRS + 255) / 256; ++i) {
        const int p = threadIdx.x + 256 * i;
        if (p < COV_PAIRS) part[(long)blockIdx.x * COV_PAIRS + p] = acc[i];
    }
}
__global__ __launch_bounds__(256) void k_db_cov_reduce(const double *__restrict__ part, int nb, double *__restrict__ cov) {
    for (int p = threadIdx.x; p < COV_PAIRS; p += 256) {
        double s = 0.0;
        for (int b = 0; b < nb; ++b) s += part[(long)b * COV_PAIRS + p];
        int a = 0, rem = p;
        while (rem >= 55 - a) { rem -= 55 - a; ++a; }
        const int bb = a + rem;
        cov[a * R16_LD + bb] = s;
        cov[bb * R16_LD + a] = s;
    }
}

// ---- the rotated database (ia_db_build_rot) ---------------------------------------------
// One thread per padded row (rows past nrows repeat the last real row): the 55 centred
// features (fp64), rho = V^T a' (fp64 from the fp32 rotation), the split-f16 slots of
// ia_rot16.h in the tile layout (10 half8 stores), and the skipped components' norm for
// amax[1] (A_skip, rounded up).  amax[0] (A, the split scale's bound) is computed first by
// the same range / bound kernels as every other form (launch_db_amax).
__global__ __launch_bounds__(256) void k_db_build_rot(DbSrc src, long row0, long nrows, long npad,
                                                      const double *__restrict__ center,
                                                      const float *__restrict__ rot, float *amax,
                                                      half8 *__restrict__ dbr, StageMap sm, int seg_rows,
                                                      unsigned *__restrict__ askseg) {
    __shared__ __attribute__((aligned(16))) float R[R16_LD * R16_LD];
    __shared__ float red[4];
    for (int i = threadIdx.x; i < R16_LD * R16_LD / 4; i += 256)
        reinterpret_cast<float4 *>(R)[i] = reinterpret_cast<const float4 *>(rot)[i];
    __syncthreads();
    const long p = (long)blockIdx.x * 256 + threadIdx.x;
    float askip = 0.f;
    if (p < npad) {
        const long r = row0 + (p < nrows ? p : nrows - 1);
        double d[IA_D];
        double n2 = 0.0;
        ImgPair ap; int rr, cc;
        src.locate(r, ap, rr, cc);
        emit_feature(src.A, ap, rr, cc, [&](int k, double v) {
            d[k] = v - center[k];
            n2 += d[k] * d[k];
        });
        const Split16Db sc = split16_db_scale(amax[0]);
        half8 o[2 * R16_MFMA];
        double sk = 0.0;
#pragma unroll
        for (int jb = 0; jb < R16_LD; jb += 4) {
            double k0 = 0.0, k1 = 0.0, k2 = 0.0, k3 = 0.0;
#pragma unroll
            for (int k = 0; k < IA_D; ++k) {
                const float4 v = *reinterpret_cast<const float4 *>(&R[k * R16_LD + jb]);
                k0 = fma((double)v.x, d[k], k0);
                k1 = fma((double)v.y, d[k], k1);
                k2 = fma((double)v.z, d[k], k2);
                k3 = fma((double)v.w, d[k], k3);
            }
            const double kk[4] = {k0, k1, k2, k3};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int j = jb + e;
                if (j >= IA_D) continue;
                const float r32 = (float)kk[e];
                if (j >= R16_P) sk += (double)r32 * (double)r32;
                _Float16 h, l;
                split16f(ldexpf(r32, sc.ea), h, l);
                const int s = R16_M0 + j;
                o[((s & 15) >> 3) * R16_MFMA + (s >> 4)][s & 7] = h;
                if (j < R16_P) {
                    const int s0 = 2 * j, s1 = 2 * j + 1;
                    o[((s0 & 15) >> 3) * R16_MFMA + (s0 >> 4)][s0 & 7] = l;
                    o[((s1 & 15) >> 3) * R16_MFMA + (s1 >> 4)][s1 & 7] = h;
                }
            }
        }
        _Float16 nh, nl;
        split16f(ldexpf((float)n2, sc.ea - sc.R), nh, nl);
        o[((R16_NL & 15) >> 3) * R16_MFMA + (R16_NL >> 4)][R16_NL & 7] = nl;
        o[((R16_NH & 15) >> 3) * R16_MFMA + (R16_NH >> 4)][R16_NH & 7] = nh;
#pragma unroll
        for (int z = R16_NH + 1; z < R16_SLOTS; ++z) o[((z & 15) >> 3) * R16_MFMA + (z >> 4)][z & 7] = (_Float16)0.f;
        half8 *t = dbr + (p >> 5) * R16_TILE_H8 + (p & 31);
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int m = 0; m < R16_MFMA; ++m) __builtin_nontemporal_store(o[h * R16_MFMA + m], t + m * 64 + h * 32);
        const double a = sqrt(sk * (1.0 + 1e-12));
        askip = (float)a;
        if ((double)askip < a) askip = nextafterf(askip, INFINITY);
    }
    for (int o = 32; o > 0; o >>= 1) askip = fmaxf(askip, __shfl_xor(askip, o));
    // the wave's 64 rows lie in one segment (64-aligned rows of one 128-row stage): its
    // A_skip,j (non-negative floats order like their bit patterns)
    const long pw = p - (threadIdx.x & 63);
    if ((threadIdx.x & 63) == 0 && pw < npad) atomicMax(askseg + seg_of_lrow(sm, pw, seg_rows), __float_as_uint(askip));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = askip;
    __syncthreads();
    if (threadIdx.x == 0) {
        const float m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
        // non-negative floats order like their bit patterns
        atomicMax(reinterpret_cast<unsigned int *>(amax + 1), __float_as_uint(m));
    }
}

// per segment j the code c_j = ceil(255 A_skip,j / A_skip) (so A_skip c_j / 255 >= A_skip,j,
// checked in fp64 and bumped), the exact stage's per-segment skip bound (r16_askc)
__global__ __launch_bounds__(256) void k_askseg_codes(const float *__restrict__ askseg, const float *__restrict__ amax,
                                                      long nseg, unsigned char *__restrict__ codes) {
    const long j = (long)blockIdx.x * 256 + threadIdx.x;
    if (j >= nseg) return;
    const double ag = (double)amax[1], aj = (double)askseg[j];
    int c = 0;
    if (ag > 0.0 && aj > 0.0) {
        c = (int)ceil(255.0 * aj / ag);
        c = c < 1 ? 1 : (c > 255 ? 255 : c);
        while (c < 255 && ag * c / 255.0 < aj) ++c;
    }
    codes[j] = (unsigned char)c;
}

// query rows of caller-provided fp64 features (q64 rows of IA_DP), R16 layout (diagnostics)
__global__ __launch_bounds__(64) void k_query_rows_r16(const double *__restrict__ qin,
                                                       const double *__restrict__ center,
                                                       const float *__restrict__ rot,
                                                       const float *__restrict__ amax,
                                                       double *__restrict__ nq, double *__restrict__ nsk,
                                                       _Float16 *__restrict__ q16) {
    __shared__ double dq[64];
    const int m = blockIdx.x, lane = threadIdx.x;
    const double d = lane < IA_D ? qin[(long)m * IA_DP + lane] - center[lane] : 0.0;
    double d2 = d * d;
    for (int o = 32; o > 0; o >>= 1) d2 += __shfl_xor(d2, o);
    const double s2 = r16_write_query(q16 + (long)m * Q16_ROW * 8, lane, d, d2, amax[0], rot, dq);
    if (lane == 0) {
        nq[m] = d2;
        nsk[m] = s2;
    }
}

}  // namespace

// the rotated screen's form (IA_R16_FORM / ia_diag_set_r16_form): 0 [default] the block form
// k_screen16r (DB staged through LDS), 1 the wave-owned form k_screen16w (queries in LDS, DB
// tiles in each wave's registers); the same minima.  Measured on c4 (same box, A/B/A/B): the
// wave form's launches 155 vs 159 us but the step 781-789 vs 777-781 ms; the block form at 4
// blocks per CU (ring 2) 758-763 ms, 148.5-148.9 us: the default
static std::atomic<int> g_r16_form{env_int("IA_R16_FORM", 0)};
static int r16_form() { return g_r16_form.load(std::memory_order_relaxed); }

int launch_screen16r(const void *dbr, long nrows, const StageMap &sm, const _Float16 *q16, int M,
                     float *segmin, hipStream_t st, const XJob *jobs, int njobs, int parity) {
    const int ch = db_chunk_rows(nrows);
    const long nchunks = db_nchunks(nrows);
    const int seg_rows = db_seg_rows(nrows);
    const long nseg = db_nsegs(nrows);
    IA_ARG(M > 0 && ch % (STAGE_TILES * 32) == 0 && seg_rows % (STAGE_TILES * 32) == 0 &&
               ch / seg_rows <= SPC_MAX,
           "launch_screen16r: bad chunking");
    IA_ARG(sm.sc == ch / 128, "launch_screen16r: stage map of another chunking");
    IA_ARG(njobs >= 1 && njobs <= IA_BATCH_MAX && (njobs == 1 || jobs), "launch_screen16r: bad batch");
    const half8 *db16 = reinterpret_cast<const half8 *>(dbr);
    const half8 *q = reinterpret_cast<const half8 *>(q16);
    const int T = (M + 31) / 32;
    const int groups = (T + MAX_G - 1) / MAX_G;
    const int G = (T + groups - 1) / groups;
    // block-form parts per chunk: a power of two dividing the chunk's segments, doubled while
    // the grid stays within one round of IA_R16_OCC blocks per CU (256 CUs)
    static const long cus = [] {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
            n = 256;
        return (long)n;
    }();
    const int spc = ch / seg_rows;
    int split = 1;
    while (2 * split <= spc && nchunks * 2 * split * groups * njobs <= cus * IA_R16_OCC) split *= 2;
    const long nb = ((nchunks * split + 7) / 8) * 8 * groups;
    IA_ARG(nb < (1L << 31), "screen grid too large");
    const dim3 grid((unsigned)nb, (unsigned)njobs);
    // the wave-owned form (k_screen16w): segments per workgroup spb, a power of two dividing
    // nseg with >= 1 tile per wave, doubled while ~2 workgroups per CU stay busy
    const int tps = seg_rows / 32;
    int spb = 1;
    while (spb * tps < W_WAVES) spb <<= 1;
    while (spb < W_SPB_MAX && nseg % (2L * spb) == 0 && (nseg / (2L * spb)) * groups * njobs >= 512) spb <<= 1;
    const bool wform = r16_form() == 1 && R16_S16 && nseg % spb == 0;
    const long nsb = nseg / spb;
    const dim3 gridw((unsigned)(((nsb + 7) / 8) * 8 * groups), (unsigned)njobs);
#define IA_R16_CASE(GG)                                                                             \
    case GG:                                                                                        \
        if (wform)                                                                                  \
            k_screen16w<GG><<<gridw, 512, 0, st>>>(db16, (int)nsb, spb, tps, seg_rows, sm, q, M,    \
                                                   groups, segmin, nseg, jobs, parity);             \
        else                                                                                        \
            k_screen16r<GG><<<grid, 256, 0, st>>>(db16, (int)nchunks, ch, seg_rows, sm, q, M,       \
                                                  groups, segmin, nseg, jobs, parity, split);       \
        break;
    switch (G) {
        IA_R16_CASE(1)
        IA_R16_CASE(2)
        IA_R16_CASE(3)
        IA_R16_CASE(4)
        IA_R16_CASE(5)
        IA_R16_CASE(6)
        IA_R16_CASE(7)
        IA_R16_CASE(8)
        IA_R16_CASE(9)
        IA_R16_CASE(10)
        IA_R16_CASE(11)
        default: set_error("launch_screen16r: bad query split"); return IA_E_ARG;
    }
#undef IA_R16_CASE
    IA_LAUNCH_CHECK("k_screen16r");
    return IA_OK;
}

int launch_query_rows_r16(const double *q64, int M, const double *center, const float *rot,
                          const float *amax, double *nq, double *nsk, _Float16 *q16, hipStream_t st) {
    k_query_rows_r16<<<M, 64, 0, st>>>(q64, center, rot, amax, nq, nsk, q16);
    IA_LAUNCH_CHECK("k_query_rows_r16");
    return IA_OK;
}

int launch_db_amax(const IaSrcLevel *src, const DbSrc &d, const double *center, float *amax,
                   double *part, hipStream_t st);
int screen16i_attributes(hipFuncAttributes *at);
// the rotated screen's widest instance (a sharded R16 level's screen)
int screen_resources_r16(hipFuncAttributes *at) {
    IA_HIP(hipFuncGetAttributes(at, reinterpret_cast<const void *>(&k_screen16r<11>)));
    return IA_OK;
}

}  // namespace ia

using namespace ia;

extern "C" {

int ia_db_rot_applies(const IaSrcLevel *src, long row0, long nrows) {
    // every level: the screen streams the rotated rows in the level's stage order (strips or
    // linear chunks); the fused kernel of either form takes the R16 bound
    if (!src || nrows <= 0 || row0 < 0) return 0;
    return row0 + nrows <= (long)src->nAp * src->Ah * src->Aw ? 1 : 0;
}

/* kernel resources of a sharded level's screen and fused kernel (the forward-progress rule
 * of DESIGN.md §7): which = 0 the rotated screen's widest instance k_screen16r<11>, 1 the
 * split-f16 4-wave k_screen16i<11> (the sharded screen without R16); LDS bytes per block and
 * VGPRs per lane (hipFuncGetAttributes) */
int ia_screen_resources(int which, int *lds, int *vgprs) {
    IA_ARG(lds && vgprs && (which == 0 || which == 1), "ia_screen_resources: bad args");
    hipFuncAttributes at{};
    if (which == 0) {
        IA_HIP(hipFuncGetAttributes(&at, reinterpret_cast<const void *>(&k_screen16r<11>)));
    } else {
        int rc = screen16i_attributes(&at);
        if (rc) return rc;
    }
    *lds = (int)at.sharedSizeBytes;
    *vgprs = at.numRegs;
    return IA_OK;
}

int ia_diag_set_r16_form(int form) {
    const int prev = r16_form();
    if (form == 0 || form == 1) g_r16_form.store(form);
    return prev;
}

int ia_db_rot_components(void) { return R16_P; }
int ia_db_rot_slots(void) { return R16_SLOTS; }
double ia_db_rot_eps_a2(void) { return R16_EPS_A2; }

size_t ia_db_rot_bytes(long nrows) { return nrows > 0 ? r16_askc_off(nrows) + img_align((size_t)db_nsegs(nrows)) : 0; }

size_t ia_db_cov_bytes(void) { return (size_t)(R16_LD * R16_LD + COV_BLOCKS * COV_PAIRS) * sizeof(double); }

int ia_db_cov(const IaSrcLevel *src, long row0, long nrows, const double *center, double *cov, void *stream) {
    IA_ARG(src && center && cov && nrows > 0 && row0 >= 0, "ia_db_cov: bad args");
    IA_ARG(row0 + nrows <= (long)src->nAp * src->Ah * src->Aw, "ia_db_cov: rows out of range");
    hipStream_t st = S(stream);
    const DbSrc d = make_dbsrc(*src);
    // ~64 k sampled rows, an odd step (no aliasing with the image width)
    const long step = (nrows / 65536) | 1;
    const long nsamp = (nrows + step - 1) / step;
    double *part = cov + R16_LD * R16_LD;
    const int nb = (int)std::min<long>(COV_BLOCKS, (nsamp + COV_ROWS - 1) / COV_ROWS);
    IA_HIP(hipMemsetAsync(cov, 0, (size_t)R16_LD * R16_LD * sizeof(double), st));
    k_db_cov<<<nb, 256, 0, st>>>(d, row0, nrows, step, nsamp, center, part);
    IA_LAUNCH_CHECK("k_db_cov");
    k_db_cov_reduce<<<1, 256, 0, st>>>(part, nb, cov);
    IA_LAUNCH_CHECK("k_db_cov_reduce");
    return IA_OK;
}

int ia_db_build_rot(const IaSrcLevel *src, long row0, long nrows, const double *center, const float *rot,
                    float *amax, void *dbr, void *stream) {
    IA_ARG(src && center && rot && amax && dbr && nrows > 0 && row0 >= 0, "ia_db_build_rot: bad args");
    IA_ARG(row0 + nrows <= (long)src->nAp * src->Ah * src->Aw, "ia_db_build_rot: rows out of range");
    IA_ARG(row0 + nrows < (1L << 31), "ia_db_build_rot: rows past 2^31");
    hipStream_t st = S(stream);
    {
        const int rc = rot_check_orthonormal(rot, IA_D, R16_LD, st, "ia_db_build_rot");
        if (rc) return rc;
    }
    const DbSrc d = make_dbsrc(*src);
    const long npad = db_rows_padded(nrows);
    IA_ARG(npad * (long)R16_ROW_B >= 1024L * 8 * 8, "ia_db_build_rot: too few rows for the bound's partials");
    // A (amax[0]) first: max with its prior value (the image form's, if built: the same bound)
    const int rc = launch_db_amax(src, d, center, amax, reinterpret_cast<double *>(dbr), st);
    if (rc) return rc;
    const StageMap sm = db_stage_map(row0, nrows, src->Aw, src->Ah);
    const long nseg = db_nsegs(nrows);
    char *tail = reinterpret_cast<char *>(dbr);
    unsigned *askseg = reinterpret_cast<unsigned *>(tail + r16_askseg_off(nrows));
    IA_HIP(hipMemsetAsync(askseg, 0, (size_t)nseg * 4, st));
    k_db_build_rot<<<(unsigned)((npad + 255) / 256), 256, 0, st>>>(d, row0, nrows, npad, center, rot, amax,
                                                                  reinterpret_cast<half8 *>(dbr), sm,
                                                                  db_seg_rows(nrows), askseg);
    IA_LAUNCH_CHECK("k_db_build_rot");
    k_askseg_codes<<<(unsigned)((nseg + 255) / 256), 256, 0, st>>>(
        reinterpret_cast<const float *>(askseg), amax, nseg,
        reinterpret_cast<unsigned char *>(tail + r16_askc_off(nrows)));
    IA_LAUNCH_CHECK("k_askseg_codes");
    return IA_OK;
}

/* diagnostics: one R16 screen of M fp64 query rows (IA_DP each) over a rotated DB ->
 * segmin[M][db_nsegs(nrows)] (screen units), nq[M], nsk[M]; q16: qrows_alloc(M) rows of
 * Q16_ROW half8, zeroed by the caller */
int ia_diag_screen16r(const IaSrcLevel *src, long row0, long nrows, const void *dbr, const float *rot,
                      const float *amax, const double *center, const double *q64, int M, void *q16,
                      double *nq, double *nsk, float *segmin, void *stream) {
    IA_ARG(src && dbr && rot && amax && center && q64 && q16 && nq && nsk && segmin && M > 0,
           "ia_diag_screen16r: bad args");
    hipStream_t st = S(stream);
    int rc = launch_query_rows_r16(q64, M, center, rot, amax, nq, nsk, reinterpret_cast<_Float16 *>(q16), st);
    if (rc) return rc;
    const StageMap sm = db_stage_map(row0, nrows, src->Aw, src->Ah);
    return launch_screen16r(dbr, nrows, sm, reinterpret_cast<const _Float16 *>(q16), M, segmin, st, nullptr, 1, 0);
}

}  // extern "C"
