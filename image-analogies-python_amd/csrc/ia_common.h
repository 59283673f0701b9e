// ia_common.h — internal helpers shared by the libia.so translation units.
// Device-side restatements of the reference's index maps and fp64 reductions, in the
// exact operation order of oracle/ia_oracle.py (compiled with -ffp-contract=off).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <atomic>
#include <cstdlib>
#include <string>

#include "../../include/ia.h"

namespace ia {

// integer from the environment (tuning / A/B knobs).  Callers keep the value in a
// function-local static (thread-safe initialisation) or a std::atomic when a diagnostic
// entry can change it: libia is called from several host threads at once (bench.py c5).
static inline int env_int(const char *name, int dflt) {
    const char *e = getenv(name);
    return e ? atoi(e) : dflt;
}


void set_error(const std::string &msg);
int hip_fail(hipError_t e, const char *what);

#define IA_HIP(call)                                              \
    do {                                                          \
        hipError_t e_ = (call);                                   \
        if (e_ != hipSuccess) return ::ia::hip_fail(e_, #call);   \
    } while (0)
#define IA_LAUNCH_CHECK(name) IA_HIP(hipGetLastError())
#define IA_ARG(cond, msg)                                         \
    do {                                                          \
        if (!(cond)) { ::ia::set_error(msg); return IA_E_ARG; }   \
    } while (0)

// A pointer into device (global) memory held in an argument struct.  On the device its
// value is typed addrspace(1), so every access through it compiles to a global load or
// store even when the struct itself was read from LDS or from a job table in memory
// (pointers loaded from memory are generic otherwise: FLAT accesses, which also count in
// lgkmcnt, so every LDS wait of the wave would wait for them too).  Same size and bits as
// T* on the host, where it is a plain pointer.
template <class T>
struct gptr {
#if defined(__HIP_DEVICE_COMPILE__)
    __attribute__((address_space(1))) T *p;
#else
    T *p;
#endif
    gptr() = default;
    __host__ __device__ gptr(T *q) : p((decltype(p))q) {}
    template <class U, class = decltype(static_cast<T *>((U *)nullptr))>
    __host__ __device__ gptr(const gptr<U> &o) : p((decltype(p))o.get()) {}
    __host__ __device__ operator T *() const { return (T *)p; }
    __host__ __device__ T *get() const { return (T *)p; }
    __host__ __device__ gptr &operator+=(long d) { p += d; return *this; }
    __host__ __device__ gptr &operator-=(long d) { p -= d; return *this; }
};
static_assert(sizeof(gptr<double>) == sizeof(double *), "gptr is a plain pointer");

static inline hipStream_t S(void *s) { return reinterpret_cast<hipStream_t>(s); }
static inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// ---------------------------------------------------------------------------------
// index maps
// ---------------------------------------------------------------------------------

// np.pad(..., 'symmetric') / ndimage 'reflect': period 2n, edge sample repeated.
__device__ __forceinline__ int symi(int i, int n) {
    if (i >= 0 && i < n) return i;
    int p = 2 * n;
    i %= p;
    if (i < 0) i += p;
    return i >= n ? p - 1 - i : i;
}

// symi for i in [-2, n + 1] and n >= 1 (the feature windows), branch-free: three
// selects (reflect low, high, low) equal the period-2n map on that range.  Keeping the
// gathers of a 55-feature row in one basic block lets all 55 loads issue before the
// first use (a branchy index map serialises them: one memory round trip per feature).
__device__ __forceinline__ int symi2(int i, int n) {
    i = i < 0 ? -1 - i : i;
    i = i >= n ? 2 * n - 1 - i : i;
    return i < 0 ? -1 - i : i;
}

// skimage _warp_fast mode 'R' (mirror about the edge sample).
__device__ __forceinline__ long mirrori(long c, long n) {
    long cmax = n - 1;
    if (c >= 0 && c <= cmax) return c;
    if (cmax == 0) return 0;
    if (c < 0) {
        long a = -c;
        return ((a / cmax) % 2 != 0) ? cmax - (a % cmax) : a % cmax;
    }
    return ((c / cmax) % 2 != 0) ? cmax - (c % cmax) : c % cmax;
}

// ---------------------------------------------------------------------------------
// features: [X full (3x3 coarse | 5x5 fine) | Y half (3x3 coarse | first 12 fine)]
// algorithms.py:11-47 (rows of As), :78-89 / image_analogies.py:167-168 (queries).
// Emits the 55 values in feature order through f(k, v).
// ---------------------------------------------------------------------------------
struct ImgPair {          // one image at levels l-1 (sm) and l (lg)
    gptr<const double> sm, lg;
    int hs, ws, h, w;
};

template <bool FULL, typename F>
__device__ __forceinline__ void emit_pixel(const ImgPair &p, int r, int c, int k0, F &&f) {
    const int rs = r >> 1, cs = c >> 1;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
        const int rr = symi2(rs + t / 3 - 1, p.hs), cc = symi2(cs + t % 3 - 1, p.ws);
        f(k0 + t, p.sm[(long)rr * p.ws + cc]);
    }
    constexpr int NF = FULL ? 25 : 12;
#pragma unroll
    for (int t = 0; t < NF; ++t) {
        const int rr = symi2(r + t / 5 - 2, p.h), cc = symi2(c + t % 5 - 2, p.w);
        f(k0 + 9 + t, p.lg[(long)rr * p.w + cc]);
    }
}

template <typename F>
__device__ __forceinline__ void emit_feature(const ImgPair &x, const ImgPair &y, int r, int c,
                                             F &&f) {
    emit_pixel<true>(x, r, c, 0, f);
    emit_pixel<false>(y, r, c, 34, f);
}

// A/A' database row ix -> (A, A'_img) pair and pixel (algorithms.py:63-67,
// img_preprocess.py:96-101 Ap_ix2px).
struct DbSrc {
    ImgPair A, Ap;        // Ap.sm/.lg point at image 0; image i is offset i * size
    long hw, hws;
    __device__ __forceinline__ void locate(long ix, ImgPair &ap, int &r, int &c) const {
        const long img = ix / hw;
        const long rem = ix - img * hw;
        r = (int)(rem / A.w);
        c = (int)(rem - (long)r * A.w);
        ap = Ap;
        ap.sm = Ap.sm + img * hws;
        ap.lg = Ap.lg + img * hw;
    }
};

static inline DbSrc make_dbsrc(const IaSrcLevel &s) {
    DbSrc d;
    d.A = ImgPair{s.A_sm, s.A_lg, s.A_hs, s.A_ws, s.Ah, s.Aw};
    d.Ap = ImgPair{s.Ap_sm, s.Ap_lg, s.A_hs, s.A_ws, s.Ah, s.Aw};
    d.hw = (long)s.Ah * s.Aw;
    d.hws = (long)s.A_hs * s.A_ws;
    return d;
}

// ---------------------------------------------------------------------------------
// numpy pairwise_sum for n = 55 (8 accumulators over k < 48, tree combine, then
// k = 48..54 sequential) fed in k order — identical to np.add.reduce(axis=1).
// ---------------------------------------------------------------------------------
struct Pw55 {
    double r[8];
    double res;
    __device__ __forceinline__ void feed(int k, double v) {
        if (k < 8) {
            r[k] = v;
        } else if (k < 48) {
            r[k & 7] += v;
        } else {
            if (k == 48) res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
            res += v;
        }
    }
};

// squared distance of DB row ix to query q (55, fp64): the oracle's brute-force value.
__device__ __forceinline__ double row_dist2(const DbSrc &src, long ix, const double *q) {
    ImgPair ap; int r, c;
    src.locate(ix, ap, r, c);
    Pw55 pw;
    emit_feature(src.A, ap, r, c, [&](int k, double v) {
        const double x = v - q[k];
        pw.feed(k, x * x);
    });
    return pw.res;
}

// weighted distance (algorithms.py:133-135 restated): s = sqrt(pw(((a-q)*w)^2)); s*s
__device__ __forceinline__ double row_wdist(const DbSrc &src, long ix, const double *q,
                                            const double *w) {
    ImgPair ap; int r, c;
    src.locate(ix, ap, r, c);
    Pw55 pw;
    emit_feature(src.A, ap, r, c, [&](int k, double v) {
        const double x = (v - q[k]) * w[k];
        pw.feed(k, x * x);
    });
    const double s = sqrt(pw.res);
    return s * s;
}

// order-preserving int64 key for doubles (atomic min/max on fp64)
__device__ __forceinline__ long long dkey(double x) {
    long long b = __double_as_longlong(x);
    return b >= 0 ? b : (b ^ 0x7fffffffffffffffLL);
}
__device__ __forceinline__ double dkey_inv(long long b) {
    return __longlong_as_double(b >= 0 ? b : (b ^ 0x7fffffffffffffffLL));
}

}  // namespace ia
