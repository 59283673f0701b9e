// ia_split16.h — the split-f16 form of the screening contraction.
//
// The screen value e = |a'|^2 - 2 a'.q' is a 56-term dot product of a DB row
// [a'_0..a'_54, |a'|^2] with a query [-2q'_0..-2q'_54, 1].  gfx950 runs f16 MFMA at 16x
// the f32 MFMA rate, so each operand x is carried as two f16 values, x = x_h + x_l
// (x_h = f16(x), x_l = f16(x - x_h)), and the product as a_h q_h + a_h q_l + a_l q_h
// (the a_l q_l term, ~2^-22 relative, is dropped): 21 groups of 8 products, packed into
// 11 v_mfma_f32_32x32x16_f16 per 32x32 tile with f32 accumulation (one 8-slot group zero).  Both operands are
// scaled by powers of two first (exact), so that every f16 value is far from the f16
// overflow and flush thresholds:
//   DB     alpha_k = sa * a'_k, alpha_55 = sa * 2^-R * |a'|^2,  sa = 2^ea
//   query  beta_k = sq * (-2 q'_k),  beta_55 = sq * 2^R,          sq = 2^eq (per query)
// so alpha . beta = sa * sq * e.  ea, R come from Amax = max row |a'| (ia_db_build),
// eq from |q'|; the exact stage (k_rescore) divides by sa * sq (exact).
//
// Lane layout of one MFMA (lane l: row/col l & 31, half h = l >> 5 supplies k-slots
// 8h..8h+7 of both operands).  Groups of 8 features: [8g, 8g+8).  The DB lane (row, h)
// holds 7 register groups G0..G6, the query lane (col, h) 8 groups Q0..Q7, and MFMA m
// multiplies G[MA[m]] by Q[MB[m]] (tables below):
//   h = 0: G0..G3 = a_h[0..31], G4..G6 = a_l[0..23]
//          Q0..Q3 = q_l[0..31], Q4..Q7 = q_h[0..31]
//   h = 1: G0..G2 = a_h[32..55], G3 = a_l[24..31], G4..G6 = a_l[32..55]
//          Q0..Q2 = q_l[32..55], Q3 = q_h[24..31], Q4..Q6 = q_h[32..55], Q7 = 0
//   m      0  1  2  3  4  5  6  7  8  9 10
//   MA     0  1  2  3  4  5  6  0  1  3  2
//   MB     0  1  2  3  4  5  6  4  5  7  6
// MFMAs 0-6 carry only cross terms (a_h q_l, a_l q_h: ~2^-11 of the main terms) and
// 7-10 the main terms a_h q_h (h = 1 adds a_l[24..31] x 0 at m = 9), with the norm slot
// (55) in the last one; the error bound of DESIGN.md §4b uses that order.  The query
// groups q_h[0..23] / q_h[32..55] serve both a cross and a main term, so a query tile
// costs 8 half8 = 32 VGPRs.
#pragma once
#include <hip/hip_runtime.h>

namespace ia {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));

constexpr int Q16_GROUPS = 8;                    // half8 groups per query lane half
constexpr int Q16_ROW = 2 * Q16_GROUPS;          // half8 per query row (256 B)
constexpr int DB16_GROUPS = 7;                   // half8 groups per DB lane half (224 B/row)
constexpr int MFMA16 = 11;                       // MFMAs per 32x32 tile
__host__ __device__ constexpr int mfma_a(int m) { return m < 7 ? m : (m == 9 ? 3 : (m == 10 ? 2 : m - 7)); }
__host__ __device__ constexpr int mfma_b(int m) { return m < 7 ? m : (m == 9 ? 7 : (m == 10 ? 6 : m - 3)); }

// DB scale exponents from amax = max row |a'| (fp32): sa * Amax in [2^13, 2^14),
// 2^R >= Amax, so |alpha_k| < 2^14 and alpha_55 <= 2^14.
struct Split16Db {
    int ea, R;
};
__device__ __forceinline__ Split16Db split16_db_scale(float amax) {
    int e = amax > 0.f ? ilogbf(amax) : 0;
    e = e < -60 ? -60 : (e > 60 ? 60 : e);
    return Split16Db{13 - e, e + 1};
}
// query scale exponent from nq = |q'|^2: 2 |q'| sq < 2^14 and sq 2^R <= 2^15.  The same
// function of the same fp64 nq runs in the query kernels and in k_rescore.
__device__ __forceinline__ int split16_q_scale(double nq, int R) {
    int eq = 15 - R;
    if (nq > 0.0) {
        const int e = ilogb(sqrt(nq));
        const int c = 12 - e;
        eq = c < eq ? c : eq;
    }
    return eq < -120 ? -120 : eq;
}

// MFMA operand order of element k = 2s + h: position h*28 + s (the fp32 query rows qp, the
// exact stage's re-screen operand).
__device__ __forceinline__ int perm56(int k) { return (k & 1) * 28 + (k >> 1); }

// x = h + l (+ the f16 rounding of l)
__device__ __forceinline__ void split16f(float x, _Float16 &h, _Float16 &l) {
    h = (_Float16)x;
    l = (_Float16)(x - (float)h);   // x - h is exact in f32
}
__device__ __forceinline__ void split16d(double x, _Float16 &h, _Float16 &l) {
    const float xf = (float)x;      // |x - xf| <= 2^-24 |x|: part of the 4u split budget
    h = (_Float16)xf;
    l = (_Float16)(float)(x - (double)h);  // x - h exact in f64
}

// DB register group g (0..6) of lane half h: features k0..k0+7, hi or lo part (table above)
__host__ __device__ __forceinline__ void split16_db_group(int h, int g, int &k0, bool &hi) {
    if (h == 0) { hi = g < 4; k0 = hi ? 8 * g : 8 * (g - 4); }
    else { hi = g < 3; k0 = hi ? 32 + 8 * g : (g == 3 ? 24 : 32 + 8 * (g - 4)); }
}

// query slots of feature k (0..55), as h * 8 + group: the hi value goes to one or two
// slots (hi1 = -1: none), the lo value to one; element = k & 7.
__device__ __forceinline__ void split16_q_slots(int k, int &lo, int &hi0, int &hi1) {
    if (k < 32) {
        lo = k >> 3; hi0 = 4 + (k >> 3); hi1 = k >= 24 ? Q16_GROUPS + 3 : -1;
    } else {
        const int g = (k - 32) >> 3;
        lo = Q16_GROUPS + g; hi0 = Q16_GROUPS + 4 + g; hi1 = -1;
    }
}

// lane k (0..63) of a query wave writes its feature's split values into the query's
// 8 x 2 half8 groups (d = q'_k in fp64, k < 55; slot 55 = sq 2^R; lanes 56..63 zero
// the h = 1 group 7).  nq = |q'|^2 (same value in every lane).
__device__ __forceinline__ void split16_write_query(_Float16 *row, int k, double d, double nq,
                                                    float amax) {
    const Split16Db s = split16_db_scale(amax);
    const int eq = split16_q_scale(nq, s.R);
    if (k < 56) {
        _Float16 h, l;
        if (k < 55) {
            split16d(ldexp(-2.0 * d, eq), h, l);
        } else {
            h = (_Float16)ldexpf(1.f, eq + s.R);
            l = (_Float16)0.f;
        }
        int lo, hi0, hi1;
        split16_q_slots(k, lo, hi0, hi1);
        const int e = k & 7;
        row[lo * 8 + e] = l;
        row[hi0 * 8 + e] = h;
        if (hi1 >= 0) row[hi1 * 8 + e] = h;
    } else {
        row[(Q16_GROUPS + 7) * 8 + (k & 7)] = (_Float16)0.f;
    }
}

}  // namespace ia
