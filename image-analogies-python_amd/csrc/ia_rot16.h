// ia_rot16.h — the rotated split-f16 screen ("R16").
//
// The split-f16 screen of ia_split16.h carries every one of the 56 products a'_k q'_k as
// three f16 products (a_h q_h + a_h q_l + a_l q_h): 11 v_mfma_f32_32x32x16_f16 per 32x32
// tile, 7 of them for the cross terms, which are ~2^-11 of the main terms.  Neighbourhood
// features of images are strongly correlated (c4's finest database: the top 3 principal
// directions hold 92.8 % of the centred rows' energy, the top 11 98.8 %), so in a rotated
// basis most components are small, and dropping their cross terms costs little:
//
//   rho = V^T a',  kappa = V^T q'   (V: 55 x 55, columns = principal directions of the
//                                    level's centred rows, fp32 entries, fp64 arithmetic)
//   a'.q' ~= rho . kappa            (V V^T = I up to its fp32 rounding: a bound term)
//
// The screen value e = |a'|^2 - 2 rho.kappa is then carried as
//   * the top R16_P components (IA_R16_P, default 3): split pairs, three products each;
//   * the other 55 - P: f16 hi parts only, one product each (error <= 2^-10 |rho_k kappa_k|,
//     summed by Cauchy-Schwarz into 2^-9 A_skip |q'_skip|, A_skip = max over rows of the
//     skipped components' norm, |q'_skip| the query's; both exact inputs of the bound);
//   * |a'|^2 (original coordinates): split pair times 2^R, as before.
// 2P + 1 + 55 + 1 slots rounded up to 16: P = 3 -> 64 slots = 4 MFMAs, 128 B per row (P = 11:
// 80 = 5 MFMAs).  Slot order (the accumulation bound of DESIGN.md §4d: the small terms first,
// the norm in the last MFMA):
//   slot   0 .. 2P-1   cross terms of component i = s/2:  DB a_l[i] | a_h[i]   query q_h[i] | q_l[i]
//   slot   R16_NL      DB norm_l                          query sq 2^R
//   slot   R16_M0 + k  DB a_h[k] (k < 55)                 query q_h[k]
//   slot   R16_NH      DB norm_h                          query sq 2^R
//   the rest           0                                  0
// Scales exactly as ia_split16.h (split16_db_scale / split16_q_scale): the screen minima
// are in the same units sa sq e, so the exact stage (k_xstrip) only widens its bound.
//
// Layouts.  MFMA m covers slots 16m .. 16m + 15; lane half h supplies slots 16m + 8h ..+7.
//   DB: per 32-row tile, R16_MFMA groups x 64 lanes x half8: group m, lane (h * 32 + row).
//   query: a q16 row (Q16_ROW = 16 half8), half8 index h * R16_MFMA + m.
#pragma once
#include "ia_internal.h"
#include "ia_split16.h"

namespace ia {

#ifndef IA_R16_P
#define IA_R16_P 3
#endif
constexpr int R16_P = IA_R16_P;                // components with cross terms
constexpr int R16_NL = 2 * R16_P;              // slot of the norm's lo part (after the cross terms)
constexpr int R16_M0 = R16_NL + 1;             // slot of main term 0
constexpr int R16_NH = R16_M0 + IA_D;          // slot of the norm's hi part (last used slot)
constexpr int R16_SLOTS = (R16_NH + 16) / 16 * 16;   // 80 (P = 11) / 64 (P = 3)
constexpr int R16_MFMA = R16_SLOTS / 16;       // MFMAs per 32x32 tile
constexpr int R16_TILE_H8 = R16_MFMA * 64;     // half8 per 32-row tile (4 KiB at P = 3)
constexpr int R16_ROW_B = R16_SLOTS * 2;       // 128 B per row at P = 3
constexpr int R16_LD = 56;                     // rot[k * R16_LD + j] = V[k][j] (fp32)
// the rotation buffer: 56 x 56 floats, padded to whole 1 KiB LDS-DMA pieces (13)
constexpr int R16_ROT_FLOATS = 13 * 256;
constexpr int R16_ROT_B = R16_ROT_FLOATS * 4;  // 13,312 B

// the rotated DB buffer (ia_db_rot_bytes): the rows (R16_ROW_B each, padded), then per
// segment A_skip,j (fp32, rounded up: max over the segment's rows of |fl32(rho_skip)|), then per
// segment the code c_j with A_skip c_j / 255 >= A_skip,j (u8; the exact stage's skip bound)
static inline size_t r16_askseg_off(long nrows) { return (size_t)db_rows_padded(nrows) * R16_ROW_B; }
static inline size_t r16_askc_off(long nrows) {
    return r16_askseg_off(nrows) + img_align((size_t)db_nsegs(nrows) * 4);
}
static inline const unsigned char *r16_askc(const void *dbr, long nrows) {
    return reinterpret_cast<const unsigned char *>(dbr) + r16_askc_off(nrows);
}
static_assert(R16_LD * R16_LD <= R16_ROT_FLOATS, "rotation buffer");

// f16 index of slot s inside a query row (h * 5 + m) * 8 + e
__host__ __device__ constexpr int r16_qpos(int s) {
    return (((s & 15) >> 3) * R16_MFMA + (s >> 4)) * 8 + (s & 7);
}
// half8 index (in a tile) and element of slot s of tile row j (0..31)
__host__ __device__ constexpr int r16_dgrp(int s, int j) { return (s >> 4) * 64 + ((s & 15) >> 3) * 32 + j; }

// The screen's MFMA shape (ia_screen16r.hip): 16 = two v_mfma_f32_16x16x32_f16 per 16x16 block
// (P = 3 only), 32 = R16_MFMA v_mfma_f32_32x32x16_f16 per 32x32 tile
#ifndef IA_R16_SHAPE
#define IA_R16_SHAPE 16
#endif
constexpr bool R16_S16 = IA_R16_SHAPE == 16 && R16_MFMA == 4;
// The bound of DESIGN.md §4d: |s(r) / (sa sq) + |q'|^2 - D(r)| <= eps_R with
//   eps_R = u (360 A|q'| + E2 A^2) + 2^-9 1.01 A_skip |q'_skip|,  u = 2^-24
// (representation 14u(2A|q'| + A^2), f16 flush <= u(28.5 A|q'| + 7.1 A^2), the fp32 rotation's
// non-orthogonality 2 |V_f V_f^T - I| A|q'| <= 30u A|q'|, the skipped components' dropped cross
// terms <= (2^-10 + 2^-21) |alpha_skip| |beta_skip|, and the accumulation: an MFMA adding K
// products to C costs <= 2Ku (|C_in| + sum |p|); 32x32x16 (K = 16), <= 5 MFMAs with the main
// mass in at most four: <= 32u(4 Y_dot + Y_norm + 5X) ~ u(256.4 A|q'| + 32.1 A^2), E2 = 60;
// 16x16x32 (K = 32), 2 MFMAs: <= 64u(2 Y_dot + Y_norm (1 + 2^-10) + 2X) ~ u(256.3 A|q'| + 64.2
// A^2), E2 = 90 (the A^2 terms sum to 85.4)).
constexpr double R16_EPS_A2 = R16_S16 ? 90.0 : 60.0;
__device__ __forceinline__ double r16_eps(double A, double nqq, double Askip, double nsk) {
    constexpr double U32 = 5.9604644775390625e-08;
    return U32 * (360.0 * A * sqrt(nqq) + R16_EPS_A2 * A * A) + 0x1p-9 * 1.01 * Askip * sqrt(nsk);
}

// the exact stage's segment threshold (and force_full) for an R16 screen, as
// rescore_thresholds (ia_exact.h) with eps_R for eps16
__device__ __forceinline__ void r16_thresholds(float emin, float amax0, float askip, double nqq, double nsk,
                                               double &Tseg, bool &force_full) {
    const double A = (double)amax0;
    const Split16Db sc = split16_db_scale(amax0);
    const int eq = split16_q_scale(nqq, sc.R);
    const int e2 = sc.ea + eq;
    const double em = ldexp((double)emin, -e2);
    const double eps = r16_eps(A, nqq, (double)askip, nsk);
    const double slack = 1e-12 * (fabs(em) + nqq + A * A);
    Tseg = ldexp(em + 2.0 * eps + slack, e2);
    force_full = eq + sc.R < -10;
}

// Per-segment skip bound (k_xstrip): segment j's rows have |rho_skip| <=
// A_skip,j <= A_skip c_j / 255 (r16_askc), so eps_j = eps_0 + K c_j with eps_0 = r16_eps(.., 0, ..)
// and K = 2^-9 1.01 |q'_skip| A_skip / 255.  The oracle winner r_o (segment o) has
// m_o - eps_o <= D(r_o) <= min_i (m_i + eps_i) =: U, so segment j is a candidate iff
// m_j <= U + eps_j = (U - eps_0) + 2 eps_0 + K c_j.  In screen units (2^e2): r16_kseg gives K
// before the minima are reduced; the reduction forms u = min_i fl32(m_i + Kf c_i) (Kf = K rounded
// up to fp32, so u >= min_i (m_i + K c_i) up to the rounding 2^-24 |u|, covered by 2^-23 |u|);
// r16_tseg0 gives T0 and the test is m_j <= T0 + K c_j.
__device__ __forceinline__ double r16_kseg(float amax0, float askip, double nqq, double nsk) {
    const Split16Db sc = split16_db_scale(amax0);
    const int e2 = sc.ea + split16_q_scale(nqq, sc.R);
    return ldexp(0x1p-9 * 1.01 * sqrt(nsk) * (double)askip / 255.0, e2);
}
__device__ __forceinline__ void r16_tseg0(float umin, float amax0, double nqq, double &T0, bool &force_full) {
    const double A = (double)amax0;
    const Split16Db sc = split16_db_scale(amax0);
    const int eq = split16_q_scale(nqq, sc.R);
    const int e2 = sc.ea + eq;
    const double em = ldexp((double)umin, -e2);
    const double eps0 = r16_eps(A, nqq, 0.0, 0.0);
    const double slack = 1e-12 * (fabs(em) + nqq + A * A) + 0x1p-23 * fabs(em);
    T0 = ldexp(em + 2.0 * eps0 + slack, e2);
    force_full = eq + sc.R < -10;
}

// the same for k_xwave's exact stage (non-strip levels), which re-screens the candidate
// segments' rows in fp32 (error eps_q = 70u (2A|q'| + A^2), ia_exact.h) before the fp64
// rescore: the oracle winner has e'(r_o) <= e* + eps_R + eps_q, so Trow (fp32 re-screen units,
// 2^ea) takes eps_R where the split-f16 form takes eps16
__device__ __forceinline__ void r16_thresholds_rows(float emin, float amax0, float askip, double nqq, double nsk,
                                                    double &Tseg, double &Trow, bool &force_full) {
    constexpr double U32 = 5.9604644775390625e-08;
    const double A = (double)amax0;
    const Split16Db sc = split16_db_scale(amax0);
    const int eq = split16_q_scale(nqq, sc.R);
    const int e2 = sc.ea + eq;
    const double em = ldexp((double)emin, -e2);
    const double eps = r16_eps(A, nqq, (double)askip, nsk);
    const double epsq = 70.0 * U32 * (2.0 * A * sqrt(nqq) + A * A);
    const double slack = 1e-12 * (fabs(em) + nqq + A * A);
    Tseg = ldexp(em + 2.0 * eps + slack, e2);
    Trow = ldexp(em + eps + epsq + slack, sc.ea);
    force_full = eq + sc.R < -10;
}

// lane-parallel query row (64 lanes): d = this lane's centred feature q'_k (lane k < 55),
// nq = |q'|^2 (every lane).  kappa_j = sum_k V[k][j] d_k in fp64 (lane j), split into the
// row's slots; returns |kappa_skip|^2 = sum_{j >= R16_P} kappa_j^2 (every lane).  rot: the
// fp32 rotation (global or LDS); dq: 64 doubles of wave-private LDS.
__device__ __forceinline__ double r16_write_query(_Float16 *row, int lane, double d, double nq, float amax,
                                                  const float *rot, double *dq) {
    dq[lane] = lane < IA_D ? d : 0.0;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    const int j = lane < IA_D ? lane : 0;
    double k0 = 0.0, k1 = 0.0, k2 = 0.0, k3 = 0.0;
#pragma unroll
    for (int k = 0; k < 52; k += 4) {
        k0 = fma((double)rot[(k + 0) * R16_LD + j], dq[k + 0], k0);
        k1 = fma((double)rot[(k + 1) * R16_LD + j], dq[k + 1], k1);
        k2 = fma((double)rot[(k + 2) * R16_LD + j], dq[k + 2], k2);
        k3 = fma((double)rot[(k + 3) * R16_LD + j], dq[k + 3], k3);
    }
    k0 = fma((double)rot[52 * R16_LD + j], dq[52], k0);
    k1 = fma((double)rot[53 * R16_LD + j], dq[53], k1);
    k2 = fma((double)rot[54 * R16_LD + j], dq[54], k2);
    const double kap = (k0 + k1) + (k2 + k3);
    double s2 = (lane >= R16_P && lane < IA_D) ? kap * kap : 0.0;
    for (int o = 32; o > 0; o >>= 1) s2 += __shfl_xor(s2, o);
    const Split16Db sc = split16_db_scale(amax);
    const int eq = split16_q_scale(nq, sc.R);
    if (lane < IA_D) {
        _Float16 h, l;
        split16d(ldexp(-2.0 * kap, eq), h, l);
        row[r16_qpos(R16_M0 + lane)] = h;
        if (lane < R16_P) {
            row[r16_qpos(2 * lane)] = h;
            row[r16_qpos(2 * lane + 1)] = l;
        }
    } else if (lane == IA_D) {
        const _Float16 n = (_Float16)ldexpf(1.f, eq + sc.R);
        row[r16_qpos(R16_NL)] = n;
        row[r16_qpos(R16_NH)] = n;
    } else if (lane > IA_D && R16_NH + (lane - IA_D) < R16_SLOTS) {
        row[r16_qpos(R16_NH + (lane - IA_D))] = (_Float16)0.f;   // the zero slots
    }
    return s2;
}

}  // namespace ia
