// ia_exact.h — device helpers of the exact stage, shared by the
// per-query exact stage (ia_match.hip) and the fused per-wave kernel (ia_xwave.hip):
// thresholds from the segment minima, the fp32 re-screen of split-f16 rows and of staged
// image-form windows, and the window staging itself.
#pragma once
#include "ia_imgwin.h"
#include "ia_split16.h"

#include <float.h>

namespace ia {

constexpr int TILE_H8 = DB16_GROUPS * 64;  // half8 per 32-row tile of the split-f16 DB

__device__ __forceinline__ void best_update(double &bd, long long &bi, double d, long long i) {
    if (d < bd || (d == bd && i < bi)) { bd = d; bi = i; }
}

// Thresholds of the exact stage from the minimum segment minimum emin (screen units):
// Tseg for segment minima (screen units), Trow for the fp32 VALU re-screen (in units of
// sa, the re-screen's scale).  e* = emin / (sa sq) exactly; Tseg = e* + 2 eps16,
// Trow = e* + eps16 + eps_q (+ a 1e-12 relative allowance for the fp64 rounding of d and
// of the centring); force_full when the query's norm slot nears the f16 floor
// (|q'| > 2^24 Amax).  eps_q = 70 u (2 A|q'| + A^2) bounds the re-screen (§4): fp32
// conversions 2u on the 2A|q'| term and u on A^2, the split residual |x - x_h - x_l| <=
// 4u|x|, a 56-term fp32 chain in any order <= 56u (1 + O(u)): 62u + O(u^2) in all.
__device__ __forceinline__ void rescore_thresholds(float emin, float amax0, double nqq,
                                                   double &Tseg, double &Trow, bool &force_full) {
    constexpr double U32 = 5.9604644775390625e-08;
    const double A = (double)amax0;
    const double eps = 70.0 * U32 * (2.0 * A * sqrt(nqq) + A * A);
    const Split16Db sc = split16_db_scale(amax0);
    const int eq = split16_q_scale(nqq, sc.R);
    const int e2 = sc.ea + eq;
    const double em = ldexp((double)emin, -e2);
    const double eps16 = U32 * (300.0 * A * sqrt(nqq) + 50.0 * A * A);
    const double slack = 1e-12 * (fabs(em) + nqq + A * A);
    Tseg = ldexp(em + 2.0 * eps16 + slack, e2);
    Trow = ldexp(em + eps16 + eps + slack, sc.ea);
    force_full = eq + sc.R < -10;
}

// The 14 register groups of DB row r (split-f16, ia_split16.h): g0 = lane half 0, g1 = 1
__device__ __forceinline__ void load_row16(const half8 *__restrict__ db16, long r,
                                           half8 (&g0)[DB16_GROUPS], half8 (&g1)[DB16_GROUPS]) {
    const half8 *t = db16 + (r >> 5) * TILE_H8 + (r & 31);
#pragma unroll
    for (int g = 0; g < DB16_GROUPS; ++g) {
        g0[g] = t[g * 64];
        g1[g] = t[g * 64 + 32];
    }
}

// fp32 re-screen value of a row from its split record, in units of sa: the same 56-term
// dot product [a', |a'|^2] . [-2 q', 1] as the screen (qf: the fp32 query row, MFMA
// operand order perm56), each value reassembled exactly as x_h + x_l in fp32; the norm
// slot carries sa 2^-R |a'|^2, so its query factor is 2^R.  Any summation order (§4).
__device__ __forceinline__ float rescreen16(const half8 (&g0)[DB16_GROUPS],
                                            const half8 (&g1)[DB16_GROUPS], const float *qf,
                                            float twoR) {
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < IA_DP; ++k) {
        _Float16 hi, lo;
        if (k < 24) { hi = g0[k >> 3][k & 7]; lo = g0[4 + (k >> 3)][k & 7]; }
        else if (k < 32) { hi = g0[3][k & 7]; lo = g1[3][k & 7]; }
        else { hi = g1[(k - 32) >> 3][k & 7]; lo = g1[4 + ((k - 32) >> 3)][k & 7]; }
        const float x = (float)hi + (float)lo;
        acc = fmaf(x, k < 55 ? qf[(k & 1) * 28 + (k >> 1)] : twoR, acc);
    }
    return acc;
}

// the same re-screen values for pixels p and p + 64 of a staged image-form window
// (ia_imgwin.h): the same 56 terms x_h + x_l in the same order as rescreen16, so the same
// fp32 values; one pass over k for both (each query factor read once)
__device__ __forceinline__ float win_x(const char *bf, const char *bc, int k) {
    const uint32_t v = *reinterpret_cast<const uint32_t *>(((k < 55 && win_coarse(k)) ? bc : bf) + win_off(k));
    return (float)__builtin_bit_cast(_Float16, (uint16_t)(v & 0xffffu)) +
           (float)__builtin_bit_cast(_Float16, (uint16_t)(v >> 16));
}
// the window's terms walked row by row (rolled loops over the window's rows, constant
// column offsets inside): the same 56 terms in the same order as rescreen16, so the same fp32
// values, in a few hundred bytes of code instead of several KB (the fused per-wave kernel
// runs cold from the instruction cache every launch)
__device__ __forceinline__ void win_terms2(const char *r0, const char *r1, const float *qf, int k,
                                           float &a0, float &a1) {
    const uint32_t v0 = *reinterpret_cast<const uint32_t *>(r0);
    const uint32_t v1 = *reinterpret_cast<const uint32_t *>(r1);
    const float f = qf[(k & 1) * 28 + (k >> 1)];
    a0 = fmaf((float)__builtin_bit_cast(_Float16, (uint16_t)(v0 & 0xffffu)) +
              (float)__builtin_bit_cast(_Float16, (uint16_t)(v0 >> 16)), f, a0);
    a1 = fmaf((float)__builtin_bit_cast(_Float16, (uint16_t)(v1 & 0xffffu)) +
              (float)__builtin_bit_cast(_Float16, (uint16_t)(v1 >> 16)), f, a1);
}
__device__ __forceinline__ void rescreen_win2(const char *wb, int p, const float *qf, float twoR,
                                              float &e0, float &e1) {
    const char *bf0 = wb + 4 * p, *bc0 = wb + 4 * (p >> 1);
    const char *bf1 = bf0 + 256, *bc1 = bc0 + 128;
    float a0 = 0.f, a1 = 0.f;
    int k = 0;
    // coarse A (k 0..8), fine A (9..33), coarse A' (34..42), fine A' (43..54): win_off's rows
#pragma unroll 1
    for (int r = 0; r < 3; ++r) {
        const int o = WB_FINE + r * WC_PC * 16 + 12;
#pragma unroll
        for (int c = 0; c < 3; ++c, ++k) win_terms2(bc0 + o + 4 * c, bc1 + o + 4 * c, qf, k, a0, a1);
    }
#pragma unroll 1
    for (int r = 0; r < 5; ++r) {
        const int o = r * WF_PC * 16 + 8;
#pragma unroll
        for (int c = 0; c < 5; ++c, ++k) win_terms2(bf0 + o + 4 * c, bf1 + o + 4 * c, qf, k, a0, a1);
    }
#pragma unroll 1
    for (int r = 3; r < 6; ++r) {
        const int o = WB_FINE + r * WC_PC * 16 + 12;
#pragma unroll
        for (int c = 0; c < 3; ++c, ++k) win_terms2(bc0 + o + 4 * c, bc1 + o + 4 * c, qf, k, a0, a1);
    }
#pragma unroll 1
    for (int r = 5; r < 8; ++r) {
        const int o = r * WF_PC * 16 + 8;
        const int nc = r < 7 ? 5 : 2;
#pragma unroll
        for (int c = 0; c < 5; ++c, ++k)
            if (c < nc) win_terms2(bf0 + o + 4 * c, bf1 + o + 4 * c, qf, k, a0, a1);
    }
    // the norm slot (k = 55), query factor 2^R
    const uint32_t v0 = *reinterpret_cast<const uint32_t *>(bf0 + WB_FINE + WB_COARSE);
    const uint32_t v1 = *reinterpret_cast<const uint32_t *>(bf1 + WB_FINE + WB_COARSE);
    a0 = fmaf((float)__builtin_bit_cast(_Float16, (uint16_t)(v0 & 0xffffu)) +
              (float)__builtin_bit_cast(_Float16, (uint16_t)(v0 >> 16)), twoR, a0);
    a1 = fmaf((float)__builtin_bit_cast(_Float16, (uint16_t)(v1 & 0xffffu)) +
              (float)__builtin_bit_cast(_Float16, (uint16_t)(v1 >> 16)), twoR, a1);
    e0 = a0;
    e1 = a1;
}
static_assert(win_off(0) == WB_FINE + 12 && win_off(9) == 8 && win_off(34) == WB_FINE + 3 * WC_PC * 16 + 12 &&
                  win_off(43) == 5 * WF_PC * 16 + 8 && win_off(54) == 7 * WF_PC * 16 + 12 &&
                  win_off(55) == WB_FINE + WB_COARSE,
              "rescreen_win2 walks win_off's rows");

// this lane's pieces of the window of the stage at local row lrow (a wave stages a whole
// window: pieces lane + 64 j), loaded into registers / stored into the wave's LDS window
constexpr int WIN_PPL = (WIN_PIECES + 63) / 64;   // 7
// a 16-B window piece as a native vector (HIP's struct uint4 defeats scalar replacement:
// a uint4[7] kept across the re-screen loop lived in scratch memory)
typedef unsigned int piece_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void win_load(const ImgDb &im, long lrow, int lane, piece_t (&pc)[WIN_PPL]) {
    const WinSrc ws = win_src(im, lrow);
#pragma unroll
    for (int j = 0; j < WIN_PPL; ++j) {
        const int i = lane + 64 * j;
        if (i < WIN_PIECES) pc[j] = *reinterpret_cast<const piece_t *>(win_piece(im, ws, i));
    }
}
// the same window copied straight into LDS (global_load_lds, no registers): lane l of
// instruction j moves piece 64 j + l to wb + 16 (64 j + l); lanes past the window's last
// piece re-load piece 0 into the slot's tail, so the slot holds WIN_SLOT bytes.  The wave
// must wait (win_dma_wait) before reading it.
constexpr int WIN_SLOT = WIN_PPL * 1024;           // 7168
__device__ __forceinline__ void win_dma(const ImgDb &im, long lrow, int lane, char *wb) {
    asm volatile("" : "+v"(lane));   // the piece addresses are computed here, not hoisted
    const WinSrc ws = win_src(im, lrow);
#pragma unroll
    for (int j = 0; j < WIN_PPL; ++j) {
        const int i = lane + 64 * j;
        __builtin_amdgcn_global_load_lds((const void *)win_piece(im, ws, i < WIN_PIECES ? i : 0),
                                         (void *)(wb + j * 1024), 16, 0, 0);
    }
}
__device__ __forceinline__ void win_dma_wait() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}
__device__ __forceinline__ void win_store(char *wb, int lane, const piece_t (&pc)[WIN_PPL]) {
#pragma unroll
    for (int j = 0; j < WIN_PPL; ++j) {
        const int i = lane + 64 * j;
        if (i < WIN_PIECES) reinterpret_cast<piece_t *>(wb)[i] = pc[j];
    }
}
// the wave's own LDS writes are visible to all its lanes (LDS executes a wave's operations
// in order; this keeps the compiler from moving them)
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

constexpr int RESCORE_SEGCAP = 1024;   // candidate segments held in LDS per query
constexpr int RESCORE_REG = 8;         // float4s of segment minima per thread kept in VGPRs
constexpr int RESCORE_RPT = 2;         // candidate rows per thread per step
constexpr int RESCORE_ROWCAP = 512;    // rows to rescore held in LDS per query
static_assert(DB_SEG_MAX <= RESCORE_RPT * 256, "one re-screen step per segment");

// a uniform index the compiler must treat as per-lane: the load it feeds is a vector load
// issued in program order with the others (a scalar load of it would be scheduled after
// their wait: one more memory round trip)
__device__ __forceinline__ int vidx(int i) {
    asm volatile("" : "+v"(i));
    return i;
}

// e* of query q over its nseg segment minima (float4 reads, nseg a multiple of 4); the
// first RESCORE_REG float4s per thread stay in v[] for the selection pass
// (threads >= 256 of a block take no part but meet the barrier).  segmin_load issues the
// loads only, so the caller can put its other independent loads in the same round trip.
__device__ __forceinline__ void segmin_load(const float4 *sq4, long n4, float4 (&v)[RESCORE_REG]) {
    const int tid = threadIdx.x;
    const long lim = tid < 256 ? n4 : 0;
    // every load unconditional (a valid index past the end; the value replaced after): a
    // load inside a divergent branch makes the join wait for it, before the caller's next
    // loads are issued
#pragma unroll
    for (int j = 0; j < RESCORE_REG; ++j) {
        const long i = tid + (long)j * 256;
        const float4 x = sq4[i < n4 ? i : 0];
        v[j] = i < lim ? x : make_float4(FLT_MAX, FLT_MAX, FLT_MAX, FLT_MAX);
    }
}
// this wave's share of e* (valid in every lane), no barrier
__device__ __forceinline__ float segmin_wave_min(const float4 *sq4, long n4, const float4 (&v)[RESCORE_REG]) {
    const int tid = threadIdx.x;
    const long lim = tid < 256 ? n4 : 0;
    float emin = FLT_MAX;
#pragma unroll
    for (int j = 0; j < RESCORE_REG; ++j)
        emin = fminf(emin, fminf(fminf(v[j].x, v[j].y), fminf(v[j].z, v[j].w)));
    for (long i = tid + (long)RESCORE_REG * 256; i < lim; i += 256) {
        const float4 x = sq4[i];
        emin = fminf(emin, fminf(fminf(x.x, x.y), fminf(x.z, x.w)));
    }
    for (int o = 32; o > 0; o >>= 1) emin = fminf(emin, __shfl_xor(emin, o));
    return emin;
}
// the same with a segment holding the wave's minimum (the lowest such index): arg
__device__ __forceinline__ float segmin_wave_argmin(const float4 *sq4, long n4, const float4 (&v)[RESCORE_REG],
                                                    long &arg) {
    const int tid = threadIdx.x;
    const long lim = tid < 256 ? n4 : 0;
    float m = FLT_MAX;
    long a = LONG_MAX;
    auto take = [&](float x, long i) {
        if (x < m || (x == m && i < a)) { m = x; a = i; }
    };
#pragma unroll
    for (int j = 0; j < RESCORE_REG; ++j) {
        const long i = 4 * (tid + (long)j * 256);
        if (tid + (long)j * 256 < lim) {
            take(v[j].x, i); take(v[j].y, i + 1); take(v[j].z, i + 2); take(v[j].w, i + 3);
        }
    }
    for (long i = tid + (long)RESCORE_REG * 256; i < lim; i += 256) {
        const float4 x = sq4[i];
        take(x.x, 4 * i); take(x.y, 4 * i + 1); take(x.z, 4 * i + 2); take(x.w, 4 * i + 3);
    }
    // wave minimum by DPP (row shifts, then row broadcasts: lane 63 ends with it), then the
    // lane-local argmin of the lowest lane that holds it (any segment holding e* will do)
    float r = m;
#define IA_DPP_MIN(CTRL, ROWS) \
    r = fminf(r, __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(r), __float_as_int(r), CTRL, ROWS, 0xf, false)))
    IA_DPP_MIN(0x111, 0xf);   // row_shr:1
    IA_DPP_MIN(0x112, 0xf);   // row_shr:2
    IA_DPP_MIN(0x114, 0xf);   // row_shr:4
    IA_DPP_MIN(0x118, 0xf);   // row_shr:8
    IA_DPP_MIN(0x142, 0xa);   // row_bcast:15 (rows 1, 3)
    IA_DPP_MIN(0x143, 0xc);   // row_bcast:31 (rows 2, 3)
#undef IA_DPP_MIN
    const float wm = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(r), 63));
    const unsigned long long hit = __ballot(m == wm);
    const int src = hit ? __builtin_ctzll(hit) : 0;
    const long long aa = (long long)a;
    arg = (long)(((unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)(aa >> 32), src) << 32) |
                 (unsigned)__builtin_amdgcn_readlane((int)aa, src));
    return wm;
}
__device__ __forceinline__ float segmin_scan(const float4 *sq4, long n4, const float4 (&v)[RESCORE_REG],
                                             float *redf) {
    const int tid = threadIdx.x;
    const float emin = segmin_wave_min(sq4, n4, v);
    if ((tid & 63) == 0 && tid < 256) redf[tid >> 6] = emin;
    __syncthreads();
    return fminf(fminf(redf[0], redf[1]), fminf(redf[2], redf[3]));
}

// candidate segments (minimum <= Tseg) -> slist (LDS, first RESCORE_SEGCAP), count in *scount:
// a thread's register-held candidates as one bit mask and ONE atomic per thread (unrolled
// per-candidate atomics cost ~800 instructions of code); any order (the winner is a
// lexicographic minimum)
__device__ __forceinline__ void segmin_select(const float4 *sq4, long n4, const float4 (&v)[RESCORE_REG],
                                              double Tseg, int *slist, int *scount) {
    const int tid = threadIdx.x;
    if (tid >= 256) return;
    static_assert(RESCORE_REG * 4 <= 32, "one 32-bit mask");
    unsigned m = 0;
#pragma unroll
    for (int j = 0; j < RESCORE_REG; ++j) {
        m |= ((double)v[j].x <= Tseg ? 1u : 0u) << (4 * j);
        m |= ((double)v[j].y <= Tseg ? 1u : 0u) << (4 * j + 1);
        m |= ((double)v[j].z <= Tseg ? 1u : 0u) << (4 * j + 2);
        m |= ((double)v[j].w <= Tseg ? 1u : 0u) << (4 * j + 3);
    }
    if (m) {
        int pos = atomicAdd(scount, __builtin_popcount(m));
        while (m) {
            const int b = __builtin_ctz(m);
            m &= m - 1;
            if (pos < RESCORE_SEGCAP) slist[pos] = 4 * (tid + (b >> 2) * 256) + (b & 3);
            ++pos;
        }
    }
    for (long i = tid + (long)RESCORE_REG * 256; i < n4; i += 256) {
        const float4 x = sq4[i];
        unsigned mt = ((double)x.x <= Tseg ? 1u : 0u) | ((double)x.y <= Tseg ? 2u : 0u) |
                      ((double)x.z <= Tseg ? 4u : 0u) | ((double)x.w <= Tseg ? 8u : 0u);
        if (mt) {
            int pos = atomicAdd(scount, __builtin_popcount(mt));
            while (mt) {
                const int b = __builtin_ctz(mt);
                mt &= mt - 1;
                if (pos < RESCORE_SEGCAP) slist[pos] = (int)(4 * i + b);
                ++pos;
            }
        }
    }
}

}  // namespace ia
