// ia_features.hip — neighbourhood feature construction.
//   * compute_feature_array (algorithms.py:11-47) for the API,
//   * the screening database (algorithms.py:50-70 As[level]): centred rows with the
//     squared norm folded in as element 55, split into f16 pairs in the MFMA operand
//     order (ia_split16.h), 224 B per row,
//   * per-wave query rows (image_analogies.py:166-168: B full | B' half): fp64 for the
//     exact rescore, fp32 for the re-screen, split-f16 for the screen.
// Feature values are pure gathers (exact); centring, rounding and splitting only feed the
// screen and re-screen, whose error bounds are accounted for in ia_match.hip.
#include "ia_common.h"
#include "ia_internal.h"

#include <cmath>
#include <cstdio>
#include <vector>
#include "ia_rot16.h"
#include "ia_split16.h"

namespace ia {

thread_local long g_db_chunk_target = DB_TARGET_CHUNKS;

// column a of V^T V - I: part[a] = sum over b of (sum_k V[k][a] V[k][b] - [a == b])^2 in fp64
// (one block per column a; threads over b: the row reads are coalesced)
constexpr int ROT_CHECK_NMAX = 192;
__global__ __launch_bounds__(256) void k_rot_gram(const float *__restrict__ rot, int n, int ld,
                                                  double *__restrict__ part) {
    __shared__ double col[ROT_CHECK_NMAX];
    __shared__ double red[4];
    const int a = blockIdx.x, tid = threadIdx.x;
    for (int k = tid; k < n; k += 256) col[k] = (double)rot[(long)k * ld + a];
    __syncthreads();
    double s = 0.0;
    for (int b = tid; b < n; b += 256) {
        double e = a == b ? -1.0 : 0.0;
        for (int k = 0; k < n; ++k) e += col[k] * (double)rot[(long)k * ld + b];
        s += e * e;
    }
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if ((tid & 63) == 0) red[tid >> 6] = s;
    __syncthreads();
    if (tid == 0) part[a] = (red[0] + red[1]) + (red[2] + red[3]);
}

// per host thread: the n column sums (device) and their host copy
struct RotCheckBuf {
    double *dev = nullptr;
    ~RotCheckBuf() {}   // (freed with the process: the HIP runtime may be gone at thread exit)
};
static thread_local RotCheckBuf g_rot_check;

int rot_check_orthonormal(const float *rot, int n, int ld, hipStream_t st, const char *who) {
    IA_ARG(n > 0 && n <= ROT_CHECK_NMAX && ld >= n, "rot_check_orthonormal: bad shape");
    if (!g_rot_check.dev) IA_HIP(hipMalloc(&g_rot_check.dev, ROT_CHECK_NMAX * sizeof(double)));
    // V^T V on the device (a per-level host loop of n^3 fp64 products cost 1.8 ms at n = 165,
    // the GPU idle meanwhile: 8 gaps per colour step, profiles/r06_colour_c3_trace.txt)
    k_rot_gram<<<n, 256, 0, st>>>(rot, n, ld, g_rot_check.dev);
    IA_LAUNCH_CHECK("k_rot_gram");
    double part[ROT_CHECK_NMAX];
    IA_HIP(hipMemcpyAsync(part, g_rot_check.dev, (size_t)n * sizeof(double), hipMemcpyDeviceToHost, st));
    IA_HIP(hipStreamSynchronize(st));
    double fro = 0.0;
    for (int a = 0; a < n; ++a) fro += part[a];
    const double budget = 2.0 * std::sqrt((double)n) * 0x1p-24;
    if (!(std::sqrt(fro) <= budget)) {
        char msg[256];
        std::snprintf(msg, sizeof msg,
                      "%s: the rotation is not orthonormal to fp32 rounding (||V^T V - I||_F = %.3g > %.3g = "
                      "2 sqrt(%d) 2^-24, the bound's budget; pass an fp64-orthonormal basis rounded to fp32)",
                      who, std::sqrt(fro), budget, n);
        set_error(msg);
        return IA_E_ARG;
    }
    return IA_OK;
}

__global__ void k_level_features(ImgPair p, int full, double *out) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (long)p.h * p.w) return;
    const int r = (int)(i / p.w), c = (int)(i - (long)r * p.w);
    if (full) {
        double *o = out + i * 34;
        emit_pixel<true>(p, r, c, 0, [&](int k, double v) { o[k] = v; });
    } else {
        double *o = out + i * 21;
        emit_pixel<false>(p, r, c, 0, [&](int k, double v) { o[k] = v; });
    }
}

// (perm56, the MFMA operand order of the fp32 query rows qp: ia_split16.h)

// Centred row of DB row ix: my[k] = fl32(a_k - c_k) (k < 55), my[55] = fl32(|a - c|^2)
// (fp64 sum in feature order).
__device__ __forceinline__ void db_row(const DbSrc &src, long ix, const double *__restrict__ center,
                                        float *my) {
    ImgPair ap; int r, c;
    src.locate(ix, ap, r, c);
    double n2 = 0.0;
    emit_feature(src.A, ap, r, c, [&](int k, double v) {
        const double d = v - center[k];
        n2 += d * d;
        my[k] = (float)d;
    });
    my[55] = (float)n2;
}

// ---- pass 1: the split scale's A >= max_row |a - c| (ia_split16.h) ---------
// Every feature k reads one of four images (k < 9 coarse A, < 34 fine A, < 43 coarse A',
// else fine A'), so |a - c|^2 <= sum_k max((hi_k - c_k)^2, (lo_k - c_k)^2) with [lo_k, hi_k]
// the value range of feature k's image.  The bound needs one streaming min / max pass over
// the level's images (no feature gathers) and holds for every row, shard and padding row;
// it is within a few tens of percent of the row maximum on image data (c4: 3.7 vs 2.87),
// which only widens the exact stage's thresholds by that factor.  Per-block partials go to
// the head of the db buffer (overwritten by pass 2).
constexpr int DBB_BLOCKS = 1024;   // partials: 64 KiB < the smallest db buffer (512 rows)
static_assert(IMG_SCRATCH >= DBB_BLOCKS * 8 * sizeof(double), "the image form's scratch holds the partials");

// Blocks are dealt to the four images in proportion to their sizes (image g gets blocks
// [first[g], first[g + 1])); each thread keeps 8 x 16 B loads in flight per step (a loop of
// single loads is latency-bound).
struct DbSpans {
    const double *x[4];
    long n[4];
    int first[5];
};

__global__ __launch_bounds__(256) void k_db_range(DbSpans sp, double *__restrict__ part) {
    __shared__ double red[4][2];
    int g = 0;
    while (g < 3 && (int)blockIdx.x >= sp.first[g + 1]) ++g;
    const int nb = sp.first[g + 1] - sp.first[g], lb = blockIdx.x - sp.first[g];
    const double *x = sp.x[g];
    const long n = sp.n[g];
    double lo = INFINITY, hi = -INFINITY;
    const long stride = (long)nb * 256;
    const double2 *x2 = reinterpret_cast<const double2 *>(x);
    const long n2 = reinterpret_cast<uintptr_t>(x) % 16 == 0 ? n / 2 : 0;
    long i = (long)lb * 256 + threadIdx.x;
    for (; i + 7 * stride < n2; i += 8 * stride) {
        double2 v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = x2[i + k * stride];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            lo = fmin(lo, fmin(v[k].x, v[k].y));
            hi = fmax(hi, fmax(v[k].x, v[k].y));
        }
    }
    for (; i < n2; i += stride) {
        const double2 v = x2[i];
        lo = fmin(lo, fmin(v.x, v.y));
        hi = fmax(hi, fmax(v.x, v.y));
    }
    for (long j = 2 * n2 + (long)lb * 256 + threadIdx.x; j < n; j += stride) {
        lo = fmin(lo, x[j]);
        hi = fmax(hi, x[j]);
    }
    for (int o = 32; o > 0; o >>= 1) {
        lo = fmin(lo, __shfl_xor(lo, o));
        hi = fmax(hi, __shfl_xor(hi, o));
    }
    const int wv = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { red[wv][0] = lo; red[wv][1] = hi; }
    __syncthreads();
    if (threadIdx.x < 8) {   // this block's partial: its image's range, +-inf for the others
        const int i8 = threadIdx.x, gi = i8 >> 1;
        double v = (i8 & 1) ? -INFINITY : INFINITY;
        if (gi == g)
            for (int w = 0; w < 4; ++w) v = (i8 & 1) ? fmax(v, red[w][1]) : fmin(v, red[w][0]);
        part[(long)blockIdx.x * 8 + i8] = v;
    }
}

// the split scale's bound from the four value ranges fin[2g] (lo), fin[2g + 1] (hi) of the
// images g (0 coarse A, 1 fine A, 2 coarse A', 3 fine A'): fl32 rounded up of sqrt(sum over
// features of the larger squared deviation of its image's range from the centre); the
// terms are summed in feature order by one thread (the same value in every caller)
__device__ __forceinline__ float db_bound_f(const double *fin, const double *__restrict__ center) {
    double b2 = 0.0;
    for (int k = 0; k < 55; ++k) {
        const int g = k < 9 ? 0 : (k < 34 ? 1 : (k < 43 ? 2 : 3));
        const double dl = fin[2 * g] - center[k], dh = fin[2 * g + 1] - center[k];
        b2 += fmax(dl * dl, dh * dh);
    }
    const double a = sqrt(b2 * (1.0 + 1e-12));
    float f = (float)a;
    if ((double)f < a) f = nextafterf(f, INFINITY);
    return f;
}

// one block of DBB_BLOCKS threads, one partial each: reduce, then amax = max(amax, fl32
// rounded up of sqrt(bound))
__global__ __launch_bounds__(1024) void k_db_bound(const double *__restrict__ part, int nb,
                                                   const double *__restrict__ center, float *amax) {
    __shared__ double red[16][8];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    double v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
        v[i] = (int)threadIdx.x < nb ? part[(long)threadIdx.x * 8 + i] : ((i & 1) ? -INFINITY : INFINITY);
#pragma unroll
    for (int i = 0; i < 8; ++i)
        for (int o = 32; o > 0; o >>= 1)
            v[i] = (i & 1) ? fmax(v[i], __shfl_xor(v[i], o)) : fmin(v[i], __shfl_xor(v[i], o));
    if (lane == 0)
#pragma unroll
        for (int i = 0; i < 8; ++i) red[wv][i] = v[i];
    __syncthreads();
    __shared__ double fin[8];
    if (threadIdx.x < 8) {
        const int i = threadIdx.x;
        double x = red[0][i];
        for (int w = 1; w < (int)(blockDim.x >> 6); ++w) x = (i & 1) ? fmax(x, red[w][i]) : fmin(x, red[w][i]);
        fin[i] = x;
    }
    __syncthreads();
    if (threadIdx.x == 0) amax[0] = fmaxf(amax[0], db_bound_f(fin, center));
}

// ---- tiled form (A width % 32 == 0, row0 % 32 == 0: every 32-row DB tile is 32 pixels of
// one scanline).  A block takes 8 tiles; each tile's feature windows (fine rows y-2..y+2 of
// A and y-2..y of A', coarse rows y/2-1..y/2+1 of both, 36 / 18 columns, symmetric index map
// applied on load) are staged in LDS by the tile's 32 threads (row pointers and reflected
// columns computed once, ~20 loads per thread), then every thread computes its row from LDS
// with constant offsets: no per-feature index arithmetic.  A
// tile past the last real row stages the last real tile instead, and its lanes take row
// nrows - 1 (the padding rule below).
constexpr int DBT_TILES = 8;                       // tiles per block (256 rows)
constexpr int WF = 36, WC = 18;                    // fine / coarse window columns
constexpr int WIN_FA = 0, WIN_FP = 5 * WF, WIN_CA = 8 * WF, WIN_CP = 8 * WF + 3 * WC;
constexpr int WIN = 8 * WF + 6 * WC;               // doubles per tile window (396)

struct DbWinCtx {
    int e;        // this thread's row within its staged tile (0..31)
    const double *w;
};

// stage the windows of tile group grp (tiles grp * 8 ..); returns this thread's window and row.
// Threads 32u .. 32u + 31 stage tile u: lane c loads columns c and c + 32 of its 8 fine rows
// and column c of its 6 coarse rows (row pointers and the reflected columns computed once).
__device__ __forceinline__ DbWinCtx db_stage(const DbSrc &src, long row0, long nrows, long grp,
                                             double *win) {
    const long tiles0 = grp * DBT_TILES;
    const long tlast = (nrows - 1) >> 5;
    const int tid = threadIdx.x;
    const int u = tid >> 5, c = tid & 31;
    const long te = min(tiles0 + u, tlast);
    const ImgPair &A = src.A;
    int img = 0, y = 0, x0 = 0;
    if (c == 0) {   // the tile's origin (64-bit divisions once per tile), broadcast below
        const long g = row0 + te * 32;
        const long im = g / src.hw;
        const long rem = g - im * src.hw;
        img = (int)im;
        y = (int)(rem / A.w);
        x0 = (int)(rem - (long)y * A.w);
    }
    img = __shfl(img, tid & 32);
    y = __shfl(y, tid & 32);
    x0 = __shfl(x0, tid & 32);
    const double *Apl = src.Ap.lg + (long)img * src.hw, *Aps = src.Ap.sm + (long)img * src.hws;
    // every load first (one basic block: they all issue before the first LDS store), with
    // clamped columns where the lane has nothing to stage; then the stores
    const int fc0 = symi2(x0 - 2 + c, A.w);
    const int fc1 = symi2(x0 - 2 + min(c + 32, WF - 1), A.w);
    const int cc = symi2((x0 >> 1) - 1 + min(c, WC - 1), A.ws);
    double vf[8][2], vc[6];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        const double *row = (r < 5 ? A.lg.get() : Apl) + (long)symi2(y - 2 + (r < 5 ? r : r - 5), A.h) * A.w;
        vf[r][0] = row[fc0];
        vf[r][1] = row[fc1];
    }
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        const long ro = (long)symi2((y >> 1) - 1 + r, A.hs) * A.ws + cc;
        vc[r] = A.sm[ro];
        vc[3 + r] = Aps[ro];
    }
    double *w = win + u * WIN;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        w[r * WF + c] = vf[r][0];   // WIN_FA rows 0..4 then WIN_FP rows 5..7 (contiguous)
        if (c + 32 < WF) w[r * WF + c + 32] = vf[r][1];
    }
    if (c < WC) {
#pragma unroll
        for (int r = 0; r < 6; ++r) w[WIN_CA + r * WC + c] = vc[r];   // WIN_CA then WIN_CP
    }
    __syncthreads();
    const long lr = (tiles0 + u) * 32 + c;
    const long er = lr < nrows ? lr : nrows - 1;
    return DbWinCtx{(int)(er - te * 32), w};
}

// the row's 55 features in emit_feature order from the staged window
template <typename F>
__device__ __forceinline__ void db_win_features(const DbWinCtx &c, F &&f) {
    const double *w = c.w;
    const int e = c.e, es = e >> 1;
#pragma unroll
    for (int t = 0; t < 9; ++t) f(t, w[WIN_CA + (t / 3) * WC + es + t % 3]);
#pragma unroll
    for (int t = 0; t < 25; ++t) f(9 + t, w[WIN_FA + (t / 5) * WF + e + t % 5]);
#pragma unroll
    for (int t = 0; t < 9; ++t) f(34 + t, w[WIN_CP + (t / 3) * WC + es + t % 3]);
#pragma unroll
    for (int t = 0; t < 12; ++t) f(43 + t, w[WIN_FP + (t / 5) * WF + e + t % 5]);
}

// Pass 2 (tiled): each thread splits its own row and writes its 14 half8 groups straight to
// the MFMA operand layout ((tile, g) blocks of 64 half8, lane = h * 32 + j): for each (g, h)
// the 32 rows of a tile write one contiguous 512 B run.
// NORM_ONLY (the image form without a row form): only the norm slot pair, to norm[row]
template <bool NORM_ONLY>
__global__ __launch_bounds__(256) void k_db_build_t(DbSrc src, long row0, long nrows,
                                                    const double *__restrict__ center,
                                                    const float *__restrict__ amax,
                                                    half8 *__restrict__ db16,
                                                    uint32_t *__restrict__ norm) {
    __shared__ double win[DBT_TILES * WIN];
    const DbWinCtx c = db_stage(src, row0, nrows, blockIdx.x, win);
    float my[IA_DP];
    double n2 = 0.0;
    db_win_features(c, [&](int k, double v) {
        const double d = v - center[k];
        n2 += d * d;
        my[k] = (float)d;
    });
    my[55] = (float)n2;
    const Split16Db s = split16_db_scale(amax[0]);
    if constexpr (NORM_ONLY) {   // the same pair as k_img_norm reads back from the row form
        const long lr = (long)blockIdx.x * 256 + threadIdx.x;
        _Float16 h, l;
        split16f(ldexpf(my[55], s.ea - s.R), h, l);
        if (lr < nrows)
            norm[lr] = (uint32_t)__builtin_bit_cast(uint16_t, h) | ((uint32_t)__builtin_bit_cast(uint16_t, l) << 16);
        return;
    }
    _Float16 xh[IA_DP], xl[IA_DP];
#pragma unroll
    for (int k = 0; k < IA_DP; ++k)
        split16f(k < 55 ? ldexpf(my[k], s.ea) : ldexpf(my[55], s.ea - s.R), xh[k], xl[k]);
    const long T = (long)blockIdx.x * DBT_TILES + (threadIdx.x >> 5);
    half8 *out = db16 + T * (DB16_GROUPS * 64) + (threadIdx.x & 31);
#pragma unroll
    for (int g = 0; g < DB16_GROUPS; ++g)      // consecutive stores: adjacent 512 B halves
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            int k0;
            bool hi;
            split16_db_group(h, g, k0, hi);
            half8 o;
#pragma unroll
            for (int e = 0; e < 8; ++e) o[e] = hi ? xh[k0 + e] : xl[k0 + e];
            __builtin_nontemporal_store(o, out + g * 64 + h * 32);   // read back by the screen only
        }
}

// ---- general form (any width / row offset): one thread gathers its row per feature ----
// Pass 2: the split-f16 rows (ia_split16.h), written once.  One thread per row computes
// its 56 centred fp32 values into LDS (256 rows = 8 tiles per block); then lane (j, h) of
// each wave emits its 7 register groups of two tiles: half8 (tile, g, lane) at
// (tile * 7 + g) * 64 + lane, so each of the screen's 7 loads per tile is one contiguous
// 1 KiB wave access.  Padding rows (>= nrows) repeat row nrows - 1: their screen values
// are those of a real row, so the segment minima need no masking (the exact stage never
// rescores a row >= nrows).
__global__ __launch_bounds__(256) void k_db_build(DbSrc src, long row0, long nrows, long npad,
                                                  const double *__restrict__ center,
                                                  const float *__restrict__ amax,
                                                  half8 *__restrict__ db16) {
    constexpr int LD = IA_DP + 1;
    __shared__ float tile[256 * LD];
    const long base = (long)blockIdx.x * 256;
    const long lr = base + threadIdx.x;
    if (lr < npad) {
        float my[IA_DP];
        db_row(src, row0 + (lr < nrows ? lr : nrows - 1), center, my);
#pragma unroll
        for (int k = 0; k < IA_DP; ++k) tile[threadIdx.x * LD + k] = my[k];
    }
    __syncthreads();
    const Split16Db s = split16_db_scale(amax[0]);
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int j = lane & 31, h = lane >> 5;
    for (int tt = wv; tt < 8; tt += 4) {
        const long T = (base >> 5) + tt;
        if (T * 32 >= npad) break;
        const float *tr = tile + (tt * 32 + j) * LD;
        half8 *out = db16 + T * (DB16_GROUPS * 64) + lane;
#pragma unroll
        for (int g = 0; g < DB16_GROUPS; ++g) {
            int k0;
            bool hi;
            split16_db_group(h, g, k0, hi);
            half8 o;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const int k = k0 + e;
                const float v = k < 55 ? ldexpf(tr[k], s.ea) : ldexpf(tr[55], s.ea - s.R);
                _Float16 xh, xl;
                split16f(v, xh, xl);
                o[e] = hi ? xh : xl;
            }
            out[g * 64] = o;
        }
    }
}

// ---- the image form of the DB (ia_db_build_image, ia_internal.h ImgDb) -----------------
// one thread per padded pixel: the split pair of sa * fl32(v - c) for the reflected pixel v
// (the same value k_db_build_t writes for every feature that reads this pixel)
__global__ __launch_bounds__(256) void k_img_pad(const double *__restrict__ img, int h, int w,
                                                 int wp, long n, const double *__restrict__ center,
                                                 int ck, const float *__restrict__ amax,
                                                 uint32_t *__restrict__ out) {
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const int r = (int)(i / wp), q = (int)(i - (long)r * wp);
    const double v = img[(long)symi(r - IMG_PY, h) * w + symi(q - IMG_PX, w)];
    const Split16Db s = split16_db_scale(amax[0]);
    _Float16 xh, xl;
    split16f(ldexpf((float)(v - center[ck]), s.ea), xh, xl);
    out[i] = (uint32_t)__builtin_bit_cast(uint16_t, xh) | ((uint32_t)__builtin_bit_cast(uint16_t, xl) << 16);
}

// ---- the image form in one pass over the images (IA_IMG_FUSED, default 1) -------------
// (1) k_db_range_at: the four value ranges as order-preserving keys, atomic-min'd into 8
//     words of the image form's scratch (lo, and hi negated; one memset of 0xff first).
// (2) k_img_build: every block first derives the split scale's bound from those 8 words
//     (db_bound_f, the same value k_db_bound computes) and amax = max(amax, bound) (block 0
//     stores it; every block uses the same value); then each thread walks one column of
//     IB_R scanlines of one A' image with the features' windows in registers (5 x 5 fine A,
//     3 x 5 fine A', 3 x 3 coarse of each; one new row per step), and writes
//       - the padded split pairs of its fine pixel of A (image 0 only) and of A', and of the
//         coarse pixel when its fine coordinates are even,
//       - the row's norm slot (the tiled build's fp64 sum in feature order, split: the same
//         bits as k_db_build_t<true>).
//     The pad margins (reflections outside the images) come from extra blocks, one thread
//     per margin pixel (k_img_pad's gather).
// One read of the images for the range, one for everything else (the two-read floor: the
// split scale needs the global bound before any value is split).
__device__ __forceinline__ unsigned long long okey(double x) {   // order-preserving key
    const unsigned long long b = (unsigned long long)__double_as_longlong(x);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ULL);
}
__device__ __forceinline__ double okey_inv(unsigned long long k) {
    return __longlong_as_double((long long)((k >> 63) ? (k & 0x7fffffffffffffffULL) : ~k));
}

__global__ __launch_bounds__(256) void k_db_range_at(DbSpans sp, unsigned long long *__restrict__ rng) {
    __shared__ double red[4][2];
    int g = 0;
    while (g < 3 && (int)blockIdx.x >= sp.first[g + 1]) ++g;
    const int nb = sp.first[g + 1] - sp.first[g], lb = blockIdx.x - sp.first[g];
    const double *x = sp.x[g];
    const long n = sp.n[g];
    double lo = INFINITY, hi = -INFINITY;
    const long stride = (long)nb * 256;
    const double2 *x2 = reinterpret_cast<const double2 *>(x);
    const long n2 = reinterpret_cast<uintptr_t>(x) % 16 == 0 ? n / 2 : 0;
    long i = (long)lb * 256 + threadIdx.x;
    for (; i + 7 * stride < n2; i += 8 * stride) {
        double2 v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = x2[i + k * stride];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            lo = fmin(lo, fmin(v[k].x, v[k].y));
            hi = fmax(hi, fmax(v[k].x, v[k].y));
        }
    }
    for (; i < n2; i += stride) {
        const double2 v = x2[i];
        lo = fmin(lo, fmin(v.x, v.y));
        hi = fmax(hi, fmax(v.x, v.y));
    }
    for (long j = 2 * n2 + (long)lb * 256 + threadIdx.x; j < n; j += stride) {
        lo = fmin(lo, x[j]);
        hi = fmax(hi, x[j]);
    }
    for (int o = 32; o > 0; o >>= 1) {
        lo = fmin(lo, __shfl_xor(lo, o));
        hi = fmax(hi, __shfl_xor(hi, o));
    }
    const int wv = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { red[wv][0] = lo; red[wv][1] = hi; }
    __syncthreads();
    if (threadIdx.x < 2) {
        double v = red[0][threadIdx.x];
        for (int w = 1; w < 4; ++w) v = threadIdx.x ? fmax(v, red[w][1]) : fmin(v, red[w][0]);
        atomicMin(&rng[2 * g + threadIdx.x], okey(threadIdx.x ? -v : v));
    }
}

constexpr int IB_R = 16;    // scanlines per thread
constexpr int IB_T = 128;   // threads (columns) per block

struct ImgBuild {
    const double *A_lg, *A_sm, *Ap_lg, *Ap_sm;   // A' image 0; image i at i * hw / hws
    int H, W, hs, ws, nAp;
    long hw, hws;
    ImgDb v;                                     // the output sections
    long row0, nrows;
    int tiles_x, tiles_y, main_blocks;           // main blocks: tiles_x * tiles_y * nAp
    long mf, mc;                                 // margin pixels per fine / coarse image
};

__device__ __forceinline__ uint32_t split_pair(double d, int ea) {
    _Float16 xh, xl;
    split16f(ldexpf((float)d, ea), xh, xl);
    return (uint32_t)__builtin_bit_cast(uint16_t, xh) | ((uint32_t)__builtin_bit_cast(uint16_t, xl) << 16);
}

// margin pixel m of a padded image (hh x ww source, wp padded width): its padded position
__device__ __forceinline__ void margin_pos(long m, int hh, int ww, int wp, int &r, int &q) {
    const long top = (long)IMG_PY * wp;
    if (m < top) { r = (int)(m / wp); q = (int)(m - (long)r * wp); return; }
    m -= top;
    if (m < top) { const int rr = (int)(m / wp); r = IMG_PY + hh + rr; q = (int)(m - (long)rr * wp); return; }
    m -= top;
    const int side = 2 * IMG_PX;   // per source row: PX left, PX right
    const int rr = (int)(m / side), c = (int)(m - (long)rr * side);
    r = IMG_PY + rr;
    q = c < IMG_PX ? c : ww + c;   // c - PX + PX + ww
}

// one main block's tile of k_img_build: column x of IB_R scanlines of A' image img.
// SQ (every centre of A's features equal, and of A''s: the product's centres): the windows
// hold the squared deviations, each computed once when its sample enters (the centre
// column's deviations kept for the pads); the norm sums them in the same order, so the bits
// equal the general form's (d = v - c_k; n2 += d * d per feature)
template <bool SQ>
__device__ __forceinline__ void img_tile(const ImgBuild &b, int blk, const double *cs, const Split16Db &sc) {
    const int img = blk / (b.tiles_x * b.tiles_y);
    const int t2 = blk - img * b.tiles_x * b.tiles_y;
    const int ty = t2 / b.tiles_x, tx = t2 - ty * b.tiles_x;
    const int x = tx * IB_T + threadIdx.x;
    const int y0 = ty * IB_R;
    const int H = b.H, W = b.W;
    const double *A = b.A_lg, *As = b.A_sm;
    const double *P = b.Ap_lg + (long)img * b.hw, *Ps = b.Ap_sm + (long)img * b.hws;
    uint32_t *fa = const_cast<uint32_t *>(b.v.fa.get()), *ca = const_cast<uint32_t *>(b.v.ca.get());
    uint32_t *fp = const_cast<uint32_t *>(b.v.ap.get()) + (long)img * b.v.apstride;
    uint32_t *cp = fp + b.v.apc;
    uint32_t *nm = const_cast<uint32_t *>(b.v.norm.get());
    const double cA = cs[0], cP = cs[34];
    int col[5], ccol[3];
#pragma unroll
    for (int d = 0; d < 5; ++d) col[d] = symi2(x + d - 2, W);
    const int cx = x >> 1;
#pragma unroll
    for (int d = 0; d < 3; ++d) ccol[d] = symi2(cx + d - 1, b.ws);
    // windows: fine A rows y-2..y+2, fine A' rows y-2..y, coarse rows cy-1..cy+1 (raw samples,
    // or with SQ their squared deviations); dv*: the centre column's deviations (SQ)
    double wa[5][5], wp[3][5], wca[3][3], wcp[3][3];
    double dva[5], dvp[3], dvca[3], dvcp[3];
    auto ldrow5 = [&](const double *im, int r, double c, double (&o)[5], double &dc) {
        const double *row = im + (long)symi2(r, H) * W;
#pragma unroll
        for (int d = 0; d < 5; ++d) {
            const double v = row[col[d]];
            if constexpr (SQ) {
                const double dd = v - c;
                o[d] = dd * dd;
                if (d == 2) dc = dd;
            } else {
                o[d] = v;
            }
        }
    };
    auto ldrow3 = [&](const double *im, int r, double c, double (&o)[3], double &dc) {
        const double *row = im + (long)symi2(r, b.hs) * b.ws;
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            const double v = row[ccol[d]];
            if constexpr (SQ) {
                const double dd = v - c;
                o[d] = dd * dd;
                if (d == 1) dc = dd;
            } else {
                o[d] = v;
            }
        }
    };
#pragma unroll
    for (int r = 0; r < 5; ++r) ldrow5(A, y0 - 2 + r, cA, wa[r], dva[r]);
#pragma unroll
    for (int r = 0; r < 3; ++r) ldrow5(P, y0 - 2 + r, cP, wp[r], dvp[r]);
    int cy = y0 >> 1;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        ldrow3(As, cy - 1 + r, cA, wca[r], dvca[r]);
        ldrow3(Ps, cy - 1 + r, cP, wcp[r], dvcp[r]);
    }
#pragma unroll
    for (int s = 0; s < IB_R; ++s) {
        const int y = y0 + s;
        if (s > 0) {   // slide one scanline down
#pragma unroll
            for (int r = 0; r < 4; ++r) {
#pragma unroll
                for (int d = 0; d < 5; ++d) wa[r][d] = wa[r + 1][d];
                dva[r] = dva[r + 1];
            }
            ldrow5(A, y + 2, cA, wa[4], dva[4]);
#pragma unroll
            for (int r = 0; r < 2; ++r) {
#pragma unroll
                for (int d = 0; d < 5; ++d) wp[r][d] = wp[r + 1][d];
                dvp[r] = dvp[r + 1];
            }
            ldrow5(P, y, cP, wp[2], dvp[2]);
            if ((y >> 1) != cy) {
                cy = y >> 1;
#pragma unroll
                for (int r = 0; r < 2; ++r) {
#pragma unroll
                    for (int d = 0; d < 3; ++d) { wca[r][d] = wca[r + 1][d]; wcp[r][d] = wcp[r + 1][d]; }
                    dvca[r] = dvca[r + 1];
                    dvcp[r] = dvcp[r + 1];
                }
                ldrow3(As, cy + 1, cA, wca[2], dvca[2]);
                ldrow3(Ps, cy + 1, cP, wcp[2], dvcp[2]);
            }
        }
        if (y >= H) break;
        // the norm slot: the tiled build's sum in feature order (db_win_features)
        double n2 = 0.0;
        auto term = [&](double w, int k) {
            if constexpr (SQ) {
                n2 += w;
            } else {
                const double d = w - cs[k];
                n2 += d * d;
            }
        };
#pragma unroll
        for (int t = 0; t < 9; ++t) term(wca[t / 3][t % 3], t);
#pragma unroll
        for (int t = 0; t < 25; ++t) term(wa[t / 5][t % 5], 9 + t);
#pragma unroll
        for (int t = 0; t < 9; ++t) term(wcp[t / 3][t % 3], 34 + t);
#pragma unroll
        for (int t = 0; t < 12; ++t) term(wp[t / 5][t % 5], 43 + t);
        const long g = (long)img * b.hw + (long)y * W + x;
        if (g >= b.row0 && g < b.row0 + b.nrows) {
            _Float16 h, l;
            split16f(ldexpf((float)n2, sc.ea - sc.R), h, l);
            nm[g - b.row0] = (uint32_t)__builtin_bit_cast(uint16_t, h) | ((uint32_t)__builtin_bit_cast(uint16_t, l) << 16);
        }
        // padded pixels: fine A (image 0), fine A', and the coarse ones at even coordinates
        const double da = SQ ? dva[2] : wa[2][2] - cA, dp = SQ ? dvp[2] : wp[2][2] - cP;
        const long pf = (long)(y + IMG_PY) * b.v.Wp + x + IMG_PX;
        if (img == 0) fa[pf] = split_pair(da, sc.ea);
        fp[pf] = split_pair(dp, sc.ea);
        if (!(y & 1) && !(x & 1)) {
            const double dca = SQ ? dvca[1] : wca[1][1] - cA, dcp = SQ ? dvcp[1] : wcp[1][1] - cP;
            const long pc = (long)(cy + IMG_PY) * b.v.Wcp + cx + IMG_PX;
            if (img == 0) ca[pc] = split_pair(dca, sc.ea);
            cp[pc] = split_pair(dcp, sc.ea);
        }
    }
}

__global__ __launch_bounds__(IB_T) void k_img_build(ImgBuild b, const double *__restrict__ center,
                                                    float *amax, const unsigned long long *__restrict__ rng) {
    __shared__ double cs[56];
    __shared__ float amx;
    __shared__ int uni_s;
    if (threadIdx.x < IA_D) cs[threadIdx.x] = center[threadIdx.x];
    if (threadIdx.x == 0) {
        int u = 1;
        for (int k = 1; k < IA_D; ++k) u &= center[k] == center[k < 34 ? 0 : 34];
        uni_s = u;
        double fin[8];
        for (int i = 0; i < 8; ++i) fin[i] = (i & 1) ? -okey_inv(rng[i]) : okey_inv(rng[i]);
        const float a = fmaxf(amax[0], db_bound_f(fin, center));
        amx = a;
        if (blockIdx.x == 0) amax[0] = a;
    }
    __syncthreads();
    const Split16Db sc = split16_db_scale(amx);
    const bool uni = uni_s != 0;
    const int blk = blockIdx.x;
    if (blk >= b.main_blocks) {   // margins: one thread per margin pixel of one padded image
        const long m = (long)(blk - b.main_blocks) * IB_T + threadIdx.x;
        // images: A fine, A coarse, then per A' image fine, coarse
        const long per = b.mf + b.mc;
        const long img = m / per;
        if (img > b.nAp) return;
        long mm = m - img * per;
        const bool coarse = mm >= b.mf;
        if (coarse) mm -= b.mf;
        const int hh = coarse ? b.hs : b.H, ww = coarse ? b.ws : b.W, wp = coarse ? b.v.Wcp : b.v.Wp;
        int r, q;
        margin_pos(mm, hh, ww, wp, r, q);
        const double *src = img == 0 ? (coarse ? b.A_sm : b.A_lg)
                                     : (coarse ? b.Ap_sm + (img - 1) * b.hws : b.Ap_lg + (img - 1) * b.hw);
        const uint32_t *o0 = img == 0 ? (coarse ? b.v.ca.get() : b.v.fa.get())
                                      : b.v.ap.get() + (img - 1) * b.v.apstride + (coarse ? b.v.apc : 0);
        uint32_t *out = const_cast<uint32_t *>(o0);
        const double v = src[(long)symi(r - IMG_PY, hh) * ww + symi(q - IMG_PX, ww)];
        const double c = cs[img == 0 ? 0 : 34];
        out[(long)r * wp + q] = split_pair(v - c, sc.ea);
        return;
    }
    if (uni) img_tile<true>(b, blk, cs, sc);
    else img_tile<false>(b, blk, cs, sc);
}

static std::atomic<int> g_img_fused{-1};
static int img_fused() {
    int v = g_img_fused.load();
    if (v < 0) {
        v = env_int("IA_IMG_FUSED", 1) ? 1 : 0;
        g_img_fused.store(v);
    }
    return v;
}

// the rows' norm-slot pairs, read back from the row form (feature 55: hi in lane half 1's
// group 2, lo in its group 6, element 7; ia_split16.h)
__global__ __launch_bounds__(256) void k_img_norm(const half8 *__restrict__ db16, long nrows,
                                                  uint32_t *__restrict__ norm) {
    const long r = (long)blockIdx.x * 256 + threadIdx.x;
    if (r >= nrows) return;
    const long T = r >> 5;
    const int j = (int)(r & 31);
    const _Float16 xh = db16[(T * DB16_GROUPS + 2) * 64 + 32 + j][7];
    const _Float16 xl = db16[(T * DB16_GROUPS + 6) * 64 + 32 + j][7];
    norm[r] = (uint32_t)__builtin_bit_cast(uint16_t, xh) | ((uint32_t)__builtin_bit_cast(uint16_t, xl) << 16);
}

__global__ void k_center_fill(double *c, double mA, double mAp) {
    const int k = threadIdx.x;
    if (k < IA_D) c[k] = k < 34 ? mA : mAp;
}

// Query rows for the pixels of wave t (y = y_lo + m, x = t - 3y):
// q64[m][k] (fp64 feature), qp[m][perm56(k)] = fp32(-2 (q_k - c_k)), qp[..55] = 1,
// nq[m] = |q - c|^2.  One 64-lane wave per query, lane = feature index.  rot (nullable): the
// level's R16 rotation (ia_rot16.h): q16 then holds the rotated split rows and q64[m][55]
// the query's skipped-component norm |kappa_skip|^2 (the exact stage's bound)
__global__ __launch_bounds__(64) void k_query_wave(ImgPair B, ImgPair Bp, int t, int y_lo,
                                                   const double *__restrict__ center,
                                                   double *__restrict__ q64,
                                                   float *__restrict__ qp,
                                                   double *__restrict__ nq,
                                                   const float *__restrict__ amax,
                                                   _Float16 *__restrict__ q16,
                                                   const float *__restrict__ rot) {
    __shared__ double dq[64];
    const int m = blockIdx.x;
    const int y = y_lo + m, x = t - 3 * y;
    const int lane = threadIdx.x;
    double v = 0.0;
    // lane-parallel gather: each lane picks its own element of the 55
    if (lane < 34) {
        const bool coarse = lane < 9;
        const int tt = coarse ? lane : lane - 9;
        v = coarse ? B.sm[(long)symi2((y >> 1) + tt / 3 - 1, B.hs) * B.ws + symi2((x >> 1) + tt % 3 - 1, B.ws)]
                   : B.lg[(long)symi2(y + tt / 5 - 2, B.h) * B.w + symi2(x + tt % 5 - 2, B.w)];
    } else if (lane < 55) {
        const bool coarse = lane < 43;
        const int tt = coarse ? lane - 34 : lane - 43;
        v = coarse ? Bp.sm[(long)symi2((y >> 1) + tt / 3 - 1, Bp.hs) * Bp.ws + symi2((x >> 1) + tt % 3 - 1, Bp.ws)]
                   : Bp.lg[(long)symi2(y + tt / 5 - 2, Bp.h) * Bp.w + symi2(x + tt % 5 - 2, Bp.w)];
    }
    double d = 0.0;
    if (lane < 55) {
        q64[(long)m * IA_DP + lane] = v;
        d = v - center[lane];
        qp[(long)m * IA_DP + perm56(lane)] = -2.0f * (float)d;
    } else if (lane == 55) {
        q64[(long)m * IA_DP + 55] = 0.0;
        qp[(long)m * IA_DP + perm56(55)] = 1.0f;
    }
    double d2 = d * d;
    for (int o = 32; o > 0; o >>= 1) d2 += __shfl_xor(d2, o);   // same sum in every lane
    if (lane == 0) nq[m] = d2;
    if (rot) {
        const double s2 = r16_write_query(q16 + (long)m * Q16_ROW * 8, lane, d, d2, amax[0], rot, dq);
        if (lane == 0) q64[(long)m * IA_DP + 55] = s2;
    } else if (q16) {
        split16_write_query(q16 + (long)m * Q16_ROW * 8, lane, d, d2, amax[0]);
    }
}

// Query rows from caller-provided fp64 features (ia_match_batch).
__global__ __launch_bounds__(64) void k_query_rows(const double *__restrict__ qin, int M,
                                                   const double *__restrict__ center,
                                                   float *__restrict__ qp,
                                                   double *__restrict__ nq,
                                                   const float *__restrict__ amax,
                                                   _Float16 *__restrict__ q16) {
    const int m = blockIdx.x;
    const int lane = threadIdx.x;
    double d = 0.0;
    if (lane < 55) {
        d = qin[(long)m * IA_DP + lane] - center[lane];
        qp[(long)m * IA_DP + perm56(lane)] = -2.0f * (float)d;
    } else if (lane == 55) {
        qp[(long)m * IA_DP + perm56(55)] = 1.0f;
    }
    double d2 = d * d;
    for (int o = 32; o > 0; o >>= 1) d2 += __shfl_xor(d2, o);   // same sum in every lane
    if (lane == 0) nq[m] = d2;
    if (q16) split16_write_query(q16 + (long)m * Q16_ROW * 8, lane, d, d2, amax[0]);
}

int launch_query_wave(const ImgPair &B, const ImgPair &Bp, int t, int y_lo, int M,
                      const double *center, double *q64, float *qp, double *nq,
                      const float *amax, _Float16 *q16, hipStream_t st, const float *rot) {
    k_query_wave<<<M, 64, 0, st>>>(B, Bp, t, y_lo, center, q64, qp, nq, amax, q16, rot);
    IA_LAUNCH_CHECK("k_query_wave");
    return IA_OK;
}

int launch_query_rows(const double *qin, int M, const double *center, float *qp, double *nq,
                      const float *amax, _Float16 *q16, hipStream_t st) {
    k_query_rows<<<M, 64, 0, st>>>(qin, M, center, qp, nq, amax, q16);
    IA_LAUNCH_CHECK("k_query_rows");
    return IA_OK;
}

}  // namespace ia

using namespace ia;

extern "C" {

int ia_level_features_f64(const double *sm, int hs, int ws, const double *lg, int h, int w,
                          int full, double *out, void *stream) {
    IA_ARG(sm && lg && out && hs > 0 && ws > 0 && h > 0 && w > 0, "ia_level_features_f64: bad args");
    ImgPair p{sm, lg, hs, ws, h, w};
    long n = (long)h * w;
    k_level_features<<<(unsigned)((n + 255) / 256), 256, 0, S(stream)>>>(p, full, out);
    IA_LAUNCH_CHECK("k_level_features");
    return IA_OK;
}

int ia_db_chunk_rows(long nrows) { return db_chunk_rows(nrows); }

long ia_set_chunk_target(long chunks) {
    const long prev = g_db_chunk_target;
    if (chunks >= 4 && chunks <= DB_TARGET_CHUNKS) g_db_chunk_target = chunks;
    return prev;
}
long ia_db_rows_padded(long nrows) { return db_rows_padded(nrows); }
size_t ia_db_bytes(long nrows) { return db_bytes(nrows); }

static int g_db_tiled = 1;   // ia_diag_set_db_build_form
int ia_diag_set_img_fused(int on) {
    const int prev = img_fused();
    if (on == 0 || on == 1) g_img_fused.store(on);
    return prev;
}

int ia_diag_set_db_build_form(int tiled) {
    const int prev = g_db_tiled;
    if (tiled == 0 || tiled == 1) g_db_tiled = tiled;
    return prev;
}

// amax = max(amax, the bound of the level's four value ranges): k_db_range partials (part:
// DBB_BLOCKS x 8 doubles of scratch), then k_db_bound
}  // extern "C"

int ia::launch_db_amax(const IaSrcLevel *src, const DbSrc &d, const double *center, float *amax,
                       double *part, hipStream_t st) {
    DbSpans sp;   // blocks per image in proportion to its size, at least one each
    sp.x[0] = src->A_sm; sp.n[0] = d.hws;
    sp.x[1] = src->A_lg; sp.n[1] = d.hw;
    sp.x[2] = src->Ap_sm; sp.n[2] = (long)src->nAp * d.hws;
    sp.x[3] = src->Ap_lg; sp.n[3] = (long)src->nAp * d.hw;
    const long tot = sp.n[0] + sp.n[1] + sp.n[2] + sp.n[3];
    sp.first[0] = 0;
    for (int g = 0; g < 4; ++g) {
        const long want = std::max<long>(1, (long)((double)(DBB_BLOCKS - 4) * sp.n[g] / tot));
        sp.first[g + 1] = sp.first[g] + (int)want;
    }
    k_db_range<<<sp.first[4], 256, 0, st>>>(sp, part);
    IA_LAUNCH_CHECK("k_db_range");
    k_db_bound<<<1, DBB_BLOCKS, 0, st>>>(part, sp.first[4], center, amax);
    IA_LAUNCH_CHECK("k_db_bound");
    return IA_OK;
}

extern "C" {

int ia_db_build(const IaSrcLevel *src, long row0, long nrows, const double *center,
                void *db, float *amax, void *stream) {
    IA_ARG(src && center && db && amax && nrows > 0 && row0 >= 0, "ia_db_build: bad args");
    IA_ARG(row0 + nrows <= (long)src->nAp * src->Ah * src->Aw, "ia_db_build: rows out of range");
    const long npad = db_rows_padded(nrows);
    DbSrc d = make_dbsrc(*src);
    int rc = launch_db_amax(src, d, center, amax, reinterpret_cast<double *>(db), S(stream));
    if (rc) return rc;   // partials: DBB_BLOCKS x 8 doubles, < db_bytes
    if (g_db_tiled && src->Aw % 32 == 0 && row0 % 32 == 0) {   // tiled form (npad is a multiple of 256)
        k_db_build_t<false><<<(unsigned)(npad / 256), 256, 0, S(stream)>>>(
            d, row0, nrows, center, amax, reinterpret_cast<half8 *>(db), nullptr);
        IA_LAUNCH_CHECK("k_db_build_t");
        return IA_OK;
    }
    k_db_build<<<(unsigned)((npad + 255) / 256), 256, 0, S(stream)>>>(d, row0, nrows, npad, center,
                                                                     amax, reinterpret_cast<half8 *>(db));
    IA_LAUNCH_CHECK("k_db_build");
    return IA_OK;
}

size_t ia_db_image_bytes(const IaSrcLevel *src, long row0, long nrows) {
    if (!src || nrows <= 0 || row0 < 0) return 0;
    ImgDb v;
    size_t b = 0;
    return img_db_layout(src->Ah, src->Aw, src->A_hs, src->A_ws, src->nAp, row0, nrows, nullptr, v,
                         &b) ? b : 0;
}

int ia_db_build_image(const IaSrcLevel *src, long row0, long nrows, const double *center,
                      const void *db, float *amax, void *dbi, void *stream) {
    IA_ARG(src && center && amax && dbi && nrows > 0 && row0 >= 0, "ia_db_build_image: bad args");
    IA_ARG(row0 + nrows <= (long)src->nAp * src->Ah * src->Aw, "ia_db_build_image: rows out of range");
    ImgDb v;
    IA_ARG(img_db_layout(src->Ah, src->Aw, src->A_hs, src->A_ws, src->nAp, row0, nrows, dbi, v, nullptr),
           "ia_db_build_image: the image form needs width and row0 multiples of 128 and whole chunks");
    hipStream_t st = S(stream);
    const DbSrc d = make_dbsrc(*src);
    if (!db && img_fused() && src->A_ws * 2 == src->Aw && src->A_hs == (src->Ah + 1) / 2) {
        // one pass for the ranges, one for the pads and the norm slots (k_img_build)
        unsigned long long *rng = reinterpret_cast<unsigned long long *>(reinterpret_cast<char *>(dbi) + v.scr);
        IA_HIP(hipMemsetAsync(rng, 0xff, 8 * sizeof(unsigned long long), st));
        DbSpans sp;
        sp.x[0] = src->A_sm; sp.n[0] = d.hws;
        sp.x[1] = src->A_lg; sp.n[1] = d.hw;
        sp.x[2] = src->Ap_sm; sp.n[2] = (long)src->nAp * d.hws;
        sp.x[3] = src->Ap_lg; sp.n[3] = (long)src->nAp * d.hw;
        const long tot = sp.n[0] + sp.n[1] + sp.n[2] + sp.n[3];
        sp.first[0] = 0;
        for (int g = 0; g < 4; ++g) {
            const long want = std::max<long>(1, (long)((double)(DBB_BLOCKS - 4) * sp.n[g] / tot));
            sp.first[g + 1] = sp.first[g] + (int)want;
        }
        k_db_range_at<<<sp.first[4], 256, 0, st>>>(sp, rng);
        IA_LAUNCH_CHECK("k_db_range_at");
        ImgBuild bb;
        bb.A_lg = src->A_lg; bb.A_sm = src->A_sm; bb.Ap_lg = src->Ap_lg; bb.Ap_sm = src->Ap_sm;
        bb.H = src->Ah; bb.W = src->Aw; bb.hs = src->A_hs; bb.ws = src->A_ws; bb.nAp = src->nAp;
        bb.hw = d.hw; bb.hws = d.hws;
        bb.v = v;
        bb.row0 = row0; bb.nrows = nrows;
        bb.tiles_x = src->Aw / IB_T;
        bb.tiles_y = (src->Ah + IB_R - 1) / IB_R;
        bb.main_blocks = bb.tiles_x * bb.tiles_y * src->nAp;
        bb.mf = 2L * IMG_PY * v.Wp + 2L * IMG_PX * src->Ah;
        bb.mc = 2L * IMG_PY * v.Wcp + 2L * IMG_PX * src->A_hs;
        const long mblocks = ((1 + src->nAp) * (bb.mf + bb.mc) + IB_T - 1) / IB_T;
        IA_ARG(src->Aw % IB_T == 0 && (long)bb.main_blocks + mblocks < (1L << 31),
               "ia_db_build_image: fused build shape");
        k_img_build<<<(unsigned)(bb.main_blocks + mblocks), IB_T, 0, st>>>(bb, center, amax, rng);
        IA_LAUNCH_CHECK("k_img_build");
        return IA_OK;
    }
    if (!db) {   // no row form: amax here, from the scratch section's partials
        const int rc = launch_db_amax(src, d, center, amax,
                                      reinterpret_cast<double *>(reinterpret_cast<char *>(dbi) + v.scr), st);
        if (rc) return rc;
    }
    auto pad = [&](const double *img, int h, int w, int wp, long n, int ck, const uint32_t *out) {
        k_img_pad<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(img, h, w, wp, n, center, ck, amax,
                                                              const_cast<uint32_t *>(out));
    };
    pad(src->A_lg, src->Ah, src->Aw, v.Wp, v.fsz, 0, v.fa);
    pad(src->A_sm, src->A_hs, src->A_ws, v.Wcp, v.csz, 0, v.ca);
    for (int i = 0; i < src->nAp; ++i) {
        const uint32_t *f = v.ap + (long)i * v.apstride;
        pad(src->Ap_lg + (long)i * src->Ah * src->Aw, src->Ah, src->Aw, v.Wp, v.fsz, 34, f);
        pad(src->Ap_sm + (long)i * src->A_hs * src->A_ws, src->A_hs, src->A_ws, v.Wcp, v.csz, 34,
            f + v.apc);
    }
    IA_LAUNCH_CHECK("k_img_pad");
    if (db) {
        k_img_norm<<<(unsigned)((nrows + 255) / 256), 256, 0, st>>>(reinterpret_cast<const half8 *>(db), nrows,
                                                                   const_cast<uint32_t *>(v.norm.get()));
        IA_LAUNCH_CHECK("k_img_norm");
    } else {     // nrows is a multiple of 512 here (whole chunks, ia_internal.h)
        k_db_build_t<true><<<(unsigned)(nrows / 256), 256, 0, st>>>(d, row0, nrows, center, amax, nullptr,
                                                                    const_cast<uint32_t *>(v.norm.get()));
        IA_LAUNCH_CHECK("k_db_build_t<norm>");
    }
    return IA_OK;
}

int ia_center_fill(double *center, double mA, double mAp, void *stream) {
    IA_ARG(center, "ia_center_fill: bad args");
    k_center_fill<<<1, 64, 0, S(stream)>>>(center, mA, mAp);
    IA_LAUNCH_CHECK("k_center_fill");
    return IA_OK;
}

}  // extern "C"
