// ia_preprocess.hip — HBM-bound preprocessing kernels:
//   YIQ conversion (img_preprocess.py:6-22) fused with the [0,1] scaling
//   (image_analogies.py:32-56), remap/compress affines (img_preprocess.py:25-44),
//   one skimage pyramid_reduce step (img_preprocess.py:56 -> skimage 0.18.3) as an
//   LDS-tiled separable blur + bilinear resample, and a deterministic mean.
// All fp64 arithmetic follows oracle/ia_oracle.py operation for operation; the build
// uses -ffp-contract=off so no multiply-add is fused.
#include "ia_common.h"

#include <mutex>

namespace ia {

thread_local std::string g_err;
void set_error(const std::string &msg) { g_err = msg; }
int hip_fail(hipError_t e, const char *what) {
    g_err = std::string(what) + ": " + hipGetErrorString(e);
    return IA_E_HIP;
}

template <typename T>
__device__ __forceinline__ double ld(const void *p, long i) {
    return (double)reinterpret_cast<const T *>(p)[i];
}

__device__ __forceinline__ double load_any(const void *p, int dt, long i) {
    return dt == 0 ? ld<uint8_t>(p, i) : (dt == 1 ? ld<float>(p, i) : ld<double>(p, i));
}

// einsum('ij,klj->kli', m, img): numpy's order for 3 terms is (m0*x0 + m2*x2) + m1*x1.
__global__ void k_rgb_to_yiq(const void *src, int dt, long npix, double div, double *yiq,
                             double *y) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= npix) return;
    const double x0 = load_any(src, dt, 3 * i) / div;
    const double x1 = load_any(src, dt, 3 * i + 1) / div;
    const double x2 = load_any(src, dt, 3 * i + 2) / div;
    const double Y = (0.299 * x0 + 0.114 * x2) + 0.587 * x1;
    if (y) y[i] = Y;
    if (yiq) {
        yiq[3 * i] = Y;
        yiq[3 * i + 1] = (0.596 * x0 + -0.321 * x2) + -0.275 * x1;
        yiq[3 * i + 2] = (0.212 * x0 + 0.311 * x2) + -0.523 * x1;
    }
}

__global__ void k_yiq_to_rgb(const double *in, long npix, double *out) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= npix) return;
    const double x0 = in[3 * i], x1 = in[3 * i + 1], x2 = in[3 * i + 2];
    out[3 * i] = (1. * x0 + 0.621 * x2) + 0.956 * x1;
    out[3 * i + 1] = (1. * x0 + -0.647 * x2) + -0.272 * x1;
    out[3 * i + 2] = (1. * x0 + 1.702 * x2) + -1.105 * x1;
}

// the colour image of a level (image_analogies.py:216-217, 255-258): convert, YIQ (B' as Y,
// B's I / Q) to RGB clipped to [0, 1] (np.clip); otherwise each pixel's source colour in the
// A' images (im, s), C channels (a luminance A' is repeated over RGB)
__global__ void k_color_output(const double *bp, const double *yiq, const int32_t *s, const int32_t *im,
                               const double *ap, long ah, long aw, int C, long npix, double *out) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= npix) return;
    if (yiq) {
        const double x0 = bp[i], x1 = yiq[3 * i + 1], x2 = yiq[3 * i + 2];
        const double r = (1. * x0 + 0.621 * x2) + 0.956 * x1;
        const double g = (1. * x0 + -0.647 * x2) + -0.272 * x1;
        const double b = (1. * x0 + 1.702 * x2) + -1.105 * x1;
        out[3 * i] = fmin(fmax(r, 0.0), 1.0);
        out[3 * i + 1] = fmin(fmax(g, 0.0), 1.0);
        out[3 * i + 2] = fmin(fmax(b, 0.0), 1.0);
    } else {
        const long p = ((long)im[i] * ah + s[2 * i]) * aw + s[2 * i + 1];
        for (int c = 0; c < 3; ++c) out[3 * i + c] = ap[p * C + (C == 1 ? 0 : c)];
    }
}

__global__ void k_scale(const void *src, int dt, long n, double div, double *out) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = load_any(src, dt, i) / div;
}

__global__ void k_axpb(const double *x, long n, int mode, double a, double m, double b,
                       double *y) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    y[i] = mode == 0 ? a * x[i] : a * (x[i] - m) + b;
}

// ---------------------------------------------------------------------------------
// Gaussian blur: scipy NI_Correlate1D (symmetric branch) along axis 0 then axis 1,
// mode 'reflect' (= symmetric index map), 7 taps.  One 64x16 output tile per block;
// the (16+6) x (64+6) input tile (reflected on load) is staged in LDS, the vertical
// pass result in LDS, then the horizontal pass writes the tile and block min/max.
// ---------------------------------------------------------------------------------
constexpr int BT_W = 64, BT_H = 16, BH = 3;
// min/max of the smoothed image (warp's clip range) as order-preserving int64 keys, spread
// over MM_SLOTS slots of one 128-B line each: k_blur's blocks hit 64 lines instead of two
// addresses (the serialised atomics made k_blur 0.6 TB/s), k_resample reduces the slots
constexpr int MM_SLOTS = 64, MM_STRIDE = 16;
static_assert(MM_SLOTS == 64, "k_resample reduces the slots with one wave");
constexpr int IN_W = BT_W + 2 * BH, IN_H = BT_H + 2 * BH;

__global__ __launch_bounds__(256) void k_blur(const double *__restrict__ src, int H, int W,
                                              double w0, double w1, double w2, double w3,
                                              double *__restrict__ out,
                                              unsigned long long *minmax) {
    __shared__ double tin[IN_H][IN_W + 1];
    __shared__ double tv[BT_H][IN_W + 1];
    __shared__ long long red[2][4];
    const int x0 = blockIdx.x * BT_W, y0 = blockIdx.y * BT_H;
    const int tid = threadIdx.x;
    for (int i = tid; i < IN_H * IN_W; i += 256) {
        const int ty = i / IN_W, tx = i - ty * IN_W;
        const int gy = symi(y0 - BH + ty, H), gx = symi(x0 - BH + tx, W);
        tin[ty][tx] = src[(long)gy * W + gx];
    }
    __syncthreads();
    for (int i = tid; i < BT_H * IN_W; i += 256) {
        const int ty = i / IN_W, tx = i - ty * IN_W;
        double acc = tin[ty + 3][tx] * w0;
        acc = acc + (tin[ty][tx] + tin[ty + 6][tx]) * w3;
        acc = acc + (tin[ty + 1][tx] + tin[ty + 5][tx]) * w2;
        acc = acc + (tin[ty + 2][tx] + tin[ty + 4][tx]) * w1;
        tv[ty][tx] = acc;
    }
    __syncthreads();
    long long kmin = 0x7fffffffffffffffLL, kmax = (long long)0x8000000000000000ULL;
    for (int i = tid; i < BT_H * BT_W; i += 256) {
        const int ty = i / BT_W, tx = i - ty * BT_W;
        const int gy = y0 + ty, gx = x0 + tx;
        if (gy < H && gx < W) {
            double acc = tv[ty][tx + 3] * w0;
            acc = acc + (tv[ty][tx] + tv[ty][tx + 6]) * w3;
            acc = acc + (tv[ty][tx + 1] + tv[ty][tx + 5]) * w2;
            acc = acc + (tv[ty][tx + 2] + tv[ty][tx + 4]) * w1;
            out[(long)gy * W + gx] = acc;
            const long long k = dkey(acc);
            kmin = k < kmin ? k : kmin;
            kmax = k > kmax ? k : kmax;
        }
    }
    // wave reduce then block reduce, one atomic pair per block
    for (int o = 32; o > 0; o >>= 1) {
        long long a = __shfl_xor(kmin, o), b = __shfl_xor(kmax, o);
        kmin = a < kmin ? a : kmin;
        kmax = b > kmax ? b : kmax;
    }
    if ((tid & 63) == 0) { red[0][tid >> 6] = kmin; red[1][tid >> 6] = kmax; }
    __syncthreads();
    if (tid == 0) {
        for (int i = 1; i < 4; ++i) {
            kmin = red[0][i] < kmin ? red[0][i] : kmin;
            kmax = red[1][i] > kmax ? red[1][i] : kmax;
        }
        unsigned long long *sl = minmax + ((blockIdx.x + blockIdx.y * gridDim.x) % MM_SLOTS) * MM_STRIDE;
        atomicMin(reinterpret_cast<long long *>(&sl[0]), kmin);
        atomicMax(reinterpret_cast<long long *>(&sl[1]), kmax);
    }
}

// skimage _warp_fast bilinear (order 1, mode 'reflect' = mirror) at src = s*dst + t,
// then warp()'s clip to [min, max] of its input.
__global__ __launch_bounds__(256) void k_resample(const double *__restrict__ sm, int H, int W,
                                                  double *__restrict__ dst, int h, int w,
                                                  double sx, double tx, double sy, double ty,
                                                  const unsigned long long *minmax) {
    __shared__ double clip[2];
    if (threadIdx.x < 64) {   // MM_SLOTS == 64: one slot per lane of wave 0
        long long kmin = (long long)minmax[threadIdx.x * MM_STRIDE];
        long long kmax = (long long)minmax[threadIdx.x * MM_STRIDE + 1];
        for (int o = 32; o > 0; o >>= 1) {
            const long long a = __shfl_xor(kmin, o), b = __shfl_xor(kmax, o);
            kmin = a < kmin ? a : kmin;
            kmax = b > kmax ? b : kmax;
        }
        if (threadIdx.x == 0) { clip[0] = dkey_inv(kmin); clip[1] = dkey_inv(kmax); }
    }
    __syncthreads();
    const int x = blockIdx.x * 64 + (threadIdx.x & 63);
    const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (x >= w || y >= h) return;
    const double c = (double)x * sx + tx;
    const double r = (double)y * sy + ty;
    const double fr = floor(r), fc = floor(c);
    const long minr = (long)fr, minc = (long)fc, maxr = (long)ceil(r), maxc = (long)ceil(c);
    const double dr = r - (double)minr, dc = c - (double)minc;
    const long r0 = mirrori(minr, H), r1 = mirrori(maxr, H);
    const long c0 = mirrori(minc, W), c1 = mirrori(maxc, W);
    const double tl = sm[r0 * W + c0], tr = sm[r0 * W + c1];
    const double bl = sm[r1 * W + c0], br = sm[r1 * W + c1];
    const double top = (1 - dc) * tl + dc * tr;
    const double bot = (1 - dc) * bl + dc * br;
    double v = (1 - dr) * top + dr * bot;
    const double lo = clip[0], hi = clip[1];
    v = v < lo ? lo : v;   // np.clip(out, min, max) (NaN-free inputs)
    v = v > hi ? hi : v;
    dst[(long)y * w + x] = v;
}

// ---------------------------------------------------------------------------------
// Fused pyramid_reduce: one output tile of PT_H x PT_W per block.  The block works out
// which blurred rows / cols its bilinear samples read (mirror-mapped floor / ceil of
// s * dst + t) plus the blurred pixels it OWNS for the clip range (the blurred rows
// [floor(r(y0)), floor(r(y0 + PT_H))) and likewise cols: the owned sets partition the
// image), blurs that region from an LDS-staged input tile (symmetric halo of 3, the
// k_blur operation order), resamples it (the k_resample order) and writes the UNCLIPPED
// value; the min / max of its owned blurred pixels go to the slots.  k_pyr_clip then
// clips to [min, max] of the whole blurred image (warp's clip), writing only the rare
// values outside it.  No fp64 intermediate image in HBM: input read once (+ halo from
// L2), output written once and read once.
// ---------------------------------------------------------------------------------
constexpr int PT_H = 16, PT_W = 32;                  // output tile
constexpr int PR_H = 2 * PT_H + 8, PR_W = 2 * PT_W + 8;   // max blurred region (rows, cols)

__device__ __forceinline__ int floor_i(double v) { return (int)floor(v); }
__device__ __forceinline__ int ceil_i(double v) { return (int)ceil(v); }

__global__ __launch_bounds__(256) void k_pyr_reduce(const double *__restrict__ src, int H, int W,
                                                    double *__restrict__ dst, int h, int w,
                                                    double sx, double tx, double sy, double ty,
                                                    double w0, double w1, double w2, double w3,
                                                    unsigned long long *minmax) {
    // one LDS region (28.7 KiB: up to 5 blocks per CU): the input tile, then the vertical
    // pass, then the blurred region; each pass holds its results in registers across the
    // barrier that frees the region for them
    __shared__ double buf[(PR_H + 6) * (PR_W + 6)];
    __shared__ int ext[8];
    __shared__ long long red[4][4];
    const int tid = threadIdx.x;
    const int y0 = blockIdx.y * PT_H, x0 = blockIdx.x * PT_W;
    const int y1 = min(y0 + PT_H, h), x1 = min(x0 + PT_W, w);
    if (tid < 8) ext[tid] = (tid & 1) ? -0x40000000 : 0x40000000;
    __syncthreads();
    // blurred region [R0, R1] x [C0, C1]: every mirrored sample row / col + the owned set
    if (tid < PT_H && y0 + tid < y1) {
        const double r = (double)(y0 + tid) * sy + ty;
        const int a = (int)mirrori(floor_i(r), H), b = (int)mirrori(ceil_i(r), H);
        atomicMin(&ext[0], min(a, b));
        atomicMax(&ext[1], max(a, b));
    } else if (tid >= 64 && tid < 64 + PT_W && x0 + tid - 64 < x1) {
        const double c = (double)(x0 + tid - 64) * sx + tx;
        const int a = (int)mirrori(floor_i(c), W), b = (int)mirrori(ceil_i(c), W);
        atomicMin(&ext[2], min(a, b));
        atomicMax(&ext[3], max(a, b));
    } else if (tid == 128) {
        const int o0 = blockIdx.y == 0 ? 0 : max(0, min(H, floor_i((double)y0 * sy + ty)));
        const int o1 = y1 == h ? H : max(0, min(H, floor_i((double)y1 * sy + ty)));
        ext[4] = o0; ext[5] = o1;
    } else if (tid == 192) {
        const int o0 = blockIdx.x == 0 ? 0 : max(0, min(W, floor_i((double)x0 * sx + tx)));
        const int o1 = x1 == w ? W : max(0, min(W, floor_i((double)x1 * sx + tx)));
        ext[6] = o0; ext[7] = o1;
    }
    __syncthreads();
    const int oR0 = ext[4], oR1 = ext[5], oC0 = ext[6], oC1 = ext[7];
    const int R0 = oR1 > oR0 ? min(ext[0], oR0) : ext[0];
    const int R1 = oR1 > oR0 ? max(ext[1], oR1 - 1) : ext[1];
    const int C0 = oC1 > oC0 ? min(ext[2], oC0) : ext[2];
    const int C1 = oC1 > oC0 ? max(ext[3], oC1 - 1) : ext[3];
    const int RH = R1 - R0 + 1, RW = C1 - C0 + 1;   // <= PR_H, PR_W (checked by the host)
    const int IW = RW + 6;
    // 2-D loops: 64 columns x 4 rows per step (tx0 + 64 cx, ty0 + 4 ry); the halo reflects
    // once on each side for images of >= 3 rows / cols (symi otherwise)
    const int tx0 = tid & 63, ty0 = tid >> 6;
    constexpr int NRY = (PR_H + 6 + 3) / 4, NCX = (PR_W + 6 + 63) / 64;
    const bool big = H >= 3 && W >= 3;
    double v[NRY][NCX];
    {   // every load first (clamped slots re-read a valid element), then the LDS stores: the
        // loads issue back to back instead of one memory round trip per loop iteration
        int gx[NCX];
#pragma unroll
        for (int cx = 0; cx < NCX; ++cx) {
            const int tx_ = min(tx0 + 64 * cx, IW - 1);
            gx[cx] = big ? symi2(C0 - 3 + tx_, W) : symi(C0 - 3 + tx_, W);
        }
#pragma unroll
        for (int ry = 0; ry < NRY; ++ry) {
            const int ty_ = min(ty0 + 4 * ry, RH + 5);
            const double *row = src + (long)(big ? symi2(R0 - 3 + ty_, H) : symi(R0 - 3 + ty_, H)) * W;
#pragma unroll
            for (int cx = 0; cx < NCX; ++cx) v[ry][cx] = row[gx[cx]];
        }
#pragma unroll
        for (int ry = 0; ry < NRY; ++ry)
#pragma unroll
            for (int cx = 0; cx < NCX; ++cx) {
                const int ty_ = ty0 + 4 * ry, tx_ = tx0 + 64 * cx;
                if (ty_ < RH + 6 && tx_ < IW) buf[ty_ * IW + tx_] = v[ry][cx];
            }
    }
    __syncthreads();
#pragma unroll
    for (int ry = 0; ry < NRY; ++ry)          // vertical pass (k_blur's order)
#pragma unroll
        for (int cx = 0; cx < NCX; ++cx) {
            const int ty_ = ty0 + 4 * ry, tx_ = tx0 + 64 * cx;
            if (ty_ < RH && tx_ < IW) {
                const double *c = buf + (ty_ + 3) * IW + tx_;
                double acc = c[0] * w0;
                acc = acc + (c[-3 * IW] + c[3 * IW]) * w3;
                acc = acc + (c[-2 * IW] + c[2 * IW]) * w2;
                acc = acc + (c[-IW] + c[IW]) * w1;
                v[ry][cx] = acc;
            }
        }
    __syncthreads();
#pragma unroll
    for (int ry = 0; ry < NRY; ++ry)
#pragma unroll
        for (int cx = 0; cx < NCX; ++cx) {
            const int ty_ = ty0 + 4 * ry, tx_ = tx0 + 64 * cx;
            if (ty_ < RH && tx_ < IW) buf[ty_ * IW + tx_] = v[ry][cx];
        }
    __syncthreads();
    long long kmin = 0x7fffffffffffffffLL, kmax = (long long)0x8000000000000000ULL;
#pragma unroll
    for (int ry = 0; ry < NRY; ++ry)          // horizontal pass, owned min / max
#pragma unroll
        for (int cx = 0; cx < NCX; ++cx) {
            const int ty_ = ty0 + 4 * ry, tx_ = tx0 + 64 * cx;
            if (ty_ < RH && tx_ < RW) {
                const double *c = buf + ty_ * IW + tx_ + 3;
                double acc = c[0] * w0;
                acc = acc + (c[-3] + c[3]) * w3;
                acc = acc + (c[-2] + c[2]) * w2;
                acc = acc + (c[-1] + c[1]) * w1;
                v[ry][cx] = acc;
                const int gy = R0 + ty_, gx = C0 + tx_;
                if (gy >= oR0 && gy < oR1 && gx >= oC0 && gx < oC1) {
                    const long long k = dkey(acc);
                    kmin = k < kmin ? k : kmin;
                    kmax = k > kmax ? k : kmax;
                }
            }
        }
    __syncthreads();
#pragma unroll
    for (int ry = 0; ry < NRY; ++ry)
#pragma unroll
        for (int cx = 0; cx < NCX; ++cx) {
            const int ty_ = ty0 + 4 * ry, tx_ = tx0 + 64 * cx;
            if (ty_ < RH && tx_ < RW) buf[ty_ * RW + tx_] = v[ry][cx];
        }
    __syncthreads();
    long long omin = 0x7fffffffffffffffLL, omax = (long long)0x8000000000000000ULL;
    {   // bilinear samples of the blurred region (k_resample's operation order), unclipped
        const int ox = x0 + (tid & 31), oy0 = y0 + (tid >> 5);
        if (ox < x1) {
            const double c = (double)ox * sx + tx;
            const double fc = floor(c);
            const long minc = (long)fc, maxc = (long)ceil(c);
            const double dc = c - (double)minc;
            const int c0 = (int)mirrori(minc, W) - C0, c1 = (int)mirrori(maxc, W) - C0;
            for (int oy = oy0; oy < y1; oy += 8) {
                const double r = (double)oy * sy + ty;
                const double fr = floor(r);
                const long minr = (long)fr, maxr = (long)ceil(r);
                const double dr = r - (double)minr;
                const int r0 = (int)mirrori(minr, H) - R0, r1 = (int)mirrori(maxr, H) - R0;
                const double tl = buf[r0 * RW + c0], tr = buf[r0 * RW + c1];
                const double bl = buf[r1 * RW + c0], br = buf[r1 * RW + c1];
                const double top = (1 - dc) * tl + dc * tr;
                const double bot = (1 - dc) * bl + dc * br;
                const double val = (1 - dr) * top + dr * bot;
                dst[(long)oy * w + ox] = val;
                const long long k = dkey(val);
                omin = k < omin ? k : omin;
                omax = k > omax ? k : omax;
            }
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        long long a = __shfl_xor(kmin, o), b = __shfl_xor(kmax, o);
        kmin = a < kmin ? a : kmin;
        kmax = b > kmax ? b : kmax;
        a = __shfl_xor(omin, o), b = __shfl_xor(omax, o);
        omin = a < omin ? a : omin;
        omax = b > omax ? b : omax;
    }
    if ((tid & 63) == 0) {
        red[0][tid >> 6] = kmin; red[1][tid >> 6] = kmax;
        red[2][tid >> 6] = omin; red[3][tid >> 6] = omax;
    }
    __syncthreads();
    if (tid == 0) {
        for (int i = 1; i < 4; ++i) {
            kmin = red[0][i] < kmin ? red[0][i] : kmin;
            kmax = red[1][i] > kmax ? red[1][i] : kmax;
            omin = red[2][i] < omin ? red[2][i] : omin;
            omax = red[3][i] > omax ? red[3][i] : omax;
        }
        unsigned long long *sl = minmax + ((blockIdx.x + blockIdx.y * gridDim.x) % MM_SLOTS) * MM_STRIDE;
        atomicMin(reinterpret_cast<long long *>(&sl[0]), kmin);
        atomicMax(reinterpret_cast<long long *>(&sl[1]), kmax);
        atomicMin(reinterpret_cast<long long *>(&sl[2]), omin);
        atomicMax(reinterpret_cast<long long *>(&sl[3]), omax);
    }
}

// ---------------------------------------------------------------------------------
// Wave pyramid_reduce (the halving case: 1.25 <= s <= 2 + 1e-9, 0 <= t < 1 in both
// directions, no sample outside the image — what skimage's fit gives for h = ceil(H/2); the
// host checks).  Each wave is independent (no LDS, no barrier): it owns <= PW_OW output
// columns and <= PW_OH output rows, one input column per lane (the blurred columns it needs
// plus 3 on each side: <= 64).  It loads every input row of its strip first (one memory
// round trip), then walks the blurred rows: vertical pass from registers, horizontal pass
// from the neighbour lanes (DPP wave shifts), and every output row as soon as its two
// sample rows are the current / previous blurred row (lane shuffles gather the two sample
// columns).  Operation orders are k_blur's and k_resample's.  Per wave: the min / max of
// its owned blurred pixels (coverage of the clip range, as k_pyr_reduce) and of its outputs
// -> part[wave][4] as keys; k_pyr_clip_p reduces them.  (An LDS-tiled strip form — 256
// columns per block, rows staged through LDS — ran at 24-33 us for 2048^2: LDS-bound.)
// ---------------------------------------------------------------------------------
constexpr int PW_OW = 28, PW_OH = 16;
constexpr int PW_NB = 2 * PW_OH + 2;         // blurred rows of a wave (s <= 2)

__device__ __forceinline__ double dpp_shr1(double x) {   // lane l <- lane l - 1
    const int2 v = __builtin_bit_cast(int2, x);
    return __builtin_bit_cast(double, make_int2(__builtin_amdgcn_update_dpp(0, v.x, 0x138, 0xf, 0xf, false),
                                                __builtin_amdgcn_update_dpp(0, v.y, 0x138, 0xf, 0xf, false)));
}
__device__ __forceinline__ double dpp_shl1(double x) {   // lane l <- lane l + 1
    const int2 v = __builtin_bit_cast(int2, x);
    return __builtin_bit_cast(double, make_int2(__builtin_amdgcn_update_dpp(0, v.x, 0x130, 0xf, 0xf, false),
                                                __builtin_amdgcn_update_dpp(0, v.y, 0x130, 0xf, 0xf, false)));
}

// AF: the exact halving map (host-checked for every output row and column: floor(y s + t)
// = 2y, ceil = 2y + 1, likewise x): output row j is emitted at blurred row 2j + 1 from the
// previous and current rows, and its samples sit in lanes 2j + 3 and 2j + 4 (one DPP shift),
// so the emission needs no per-row sample-row test and no lane shuffle.
template <bool AF>
__global__ __launch_bounds__(256) void k_pyr_wave(const double *__restrict__ src, int H, int W,
                                                  double *__restrict__ dst, int h, int w,
                                                  int nstrip, int nunit, double sx, double tx,
                                                  double sy, double ty, double w0, double w1,
                                                  double w2, double w3, long long *__restrict__ part) {
    const int lane = threadIdx.x & 63;
    const int unit = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (unit >= nunit) return;                // uniform over the wave; no barriers below
    const int ui = unit % nstrip, uj = unit / nstrip;
    const int x0 = ui * PW_OW, x1 = min(x0 + PW_OW, w);
    const int y0 = uj * PW_OH, y1 = min(y0 + PW_OH, h);
    // sample columns / rows are monotone and inside the image (host): the extremes are those
    // of the first and last output
    auto lo_of = [](double v) { return (int)floor(v); };
    auto hi_of = [](double v) { return (int)ceil(v); };
    const int oR0 = uj == 0 ? 0 : max(0, min(H, lo_of((double)y0 * sy + ty)));
    const int oR1 = y1 == h ? H : max(0, min(H, lo_of((double)y1 * sy + ty)));
    const int oC0 = ui == 0 ? 0 : max(0, min(W, lo_of((double)x0 * sx + tx)));
    const int oC1 = x1 == w ? W : max(0, min(W, lo_of((double)x1 * sx + tx)));
    const int sR0 = lo_of((double)y0 * sy + ty), sR1 = hi_of((double)(y1 - 1) * sy + ty);
    const int sC0 = lo_of((double)x0 * sx + tx), sC1 = hi_of((double)(x1 - 1) * sx + tx);
    const int BR0 = min(sR0, oR0), BR1 = max(sR1, oR1 - 1);
    const int BC0 = min(sC0, oC0), BC1 = max(sC1, oC1 - 1);
    const int NB = BR1 - BR0 + 1;            // <= PW_NB, BC1 - BC0 + 7 <= 64 (host: s <= 2)
    // this lane's input column (blurred column BC0 - 3 + lane), reflected (W >= 4)
    int cix = min(BC0 - 3 + lane, BC1 + 3);
    cix = cix < 0 ? -1 - cix : cix;
    cix = cix >= W ? 2 * W - 1 - cix : cix;
    const double *col = src + cix;
    const int bc = BC0 - 3 + lane;
    const bool hown = lane >= 3 && bc <= BC1 && bc >= oC0 && bc < oC1;
    // this lane's output column: x0 + lane (its sample lanes L0, L1), or with AF x0 + (lane
    // - 3) / 2 for the odd lanes 3 .. 2 (x1 - x0) + 1 (samples in this lane and the next)
    int L0 = 0, L1 = 0;
    double dc = 0.0;
    const int oj = AF ? (lane - 3) >> 1 : lane;
    const bool olane = AF ? (lane >= 3 && (lane & 1) && oj < x1 - x0) : lane < x1 - x0;
    if (olane) {
        const double c = (double)(x0 + oj) * sx + tx;
        const double fc = floor(c);
        L0 = (int)fc - BC0 + 3;
        L1 = (int)ceil(c) - BC0 + 3;
        dc = c - fc;
    }
    const double omdc = 1 - dc;
    // every input row first; rows past the wave's re-read its last one
    double I[PW_NB + 6];
#pragma unroll
    for (int i = 0; i < PW_NB + 6; ++i) {
        int r = BR0 - 3 + min(i, NB + 5);
        r = r < 0 ? -1 - r : r;
        r = r >= H ? 2 * H - 1 - r : r;
        I[i] = col[(long)r * W];
    }
    double bmin = INFINITY, bmax = -INFINITY, omin = INFINITY, omax = -INFINITY;
    double Bp = 0.0, Bc = 0.0;
    int yn = y0;                             // next output row
    double *out = dst + x0 + oj;
#pragma unroll
    for (int i = 0; i < PW_NB; ++i) {
        if (i < NB) {
            double v = I[i + 3] * w0;          // vertical pass (k_blur's order)
            v = v + (I[i] + I[i + 6]) * w3;
            v = v + (I[i + 1] + I[i + 5]) * w2;
            v = v + (I[i + 2] + I[i + 4]) * w1;
            const double m1 = dpp_shr1(v), m2 = dpp_shr1(m1), m3 = dpp_shr1(m2);
            const double p1 = dpp_shl1(v), p2 = dpp_shl1(p1), p3 = dpp_shl1(p2);
            double b = v * w0;                 // horizontal pass
            b = b + (m3 + p3) * w3;
            b = b + (m2 + p2) * w2;
            b = b + (m1 + p1) * w1;
            Bp = Bc;
            Bc = b;
            const int row = BR0 + i;
            if (hown && row >= oR0 && row < oR1) {
                bmin = fmin(bmin, b);
                bmax = fmax(bmax, b);
            }
            if (AF) {
                if ((i & 1) && y0 + (i >> 1) < y1) {  // output row y0 + i / 2, rows 2j and 2j + 1
                    const int y = y0 + (i >> 1);
                    const double r = (double)y * sy + ty;
                    const double dr = r - floor(r);
                    const double top = omdc * Bp + dc * dpp_shl1(Bp);
                    const double bot = omdc * Bc + dc * dpp_shl1(Bc);
                    const double val = (1 - dr) * top + dr * bot;
                    if (olane) {
                        out[(long)y * w] = val;
                        omin = fmin(omin, val);
                        omax = fmax(omax, val);
                    }
                }
            } else if (yn < y1) {
                const double r = (double)yn * sy + ty;
                const double fr = floor(r);
                const int r0 = (int)fr, r1 = (int)ceil(r);
                if (r1 == row) {               // both sample rows done (r0 = row or row - 1)
                    const double dr = r - fr;
                    const double T = r0 == row ? Bc : Bp;
                    const double tl = __shfl(T, L0), tr = __shfl(T, L1);
                    const double bl = __shfl(Bc, L0), br = __shfl(Bc, L1);
                    const double top = omdc * tl + dc * tr;
                    const double bot = omdc * bl + dc * br;
                    const double val = (1 - dr) * top + dr * bot;
                    if (olane) {
                        out[(long)yn * w] = val;
                        omin = fmin(omin, val);
                        omax = fmax(omax, val);
                    }
                    ++yn;
                }
            }
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        bmin = fmin(bmin, __shfl_xor(bmin, o));
        bmax = fmax(bmax, __shfl_xor(bmax, o));
        omin = fmin(omin, __shfl_xor(omin, o));
        omax = fmax(omax, __shfl_xor(omax, o));
    }
    if (lane < 4) {
        const double v = lane == 0 ? bmin : lane == 1 ? bmax : lane == 2 ? omin : omax;
        part[(long)unit * 4 + lane] = dkey(v);
    }
}

// warp's clip after k_pyr_wave: every block reduces the np wave partials (blurred min /
// max, output min / max keys) and returns when the outputs lie inside the blurred range (the
// usual case); otherwise the grid clips the level.  The partials come from fmin / fmax, so a
// zero bound may carry either sign; that never changes the level: a value is replaced only
// when it lies strictly outside [lo, hi], and with lo = 0 every blurred value, hence every
// bilinear sample (non-negative weights), is >= 0 (likewise hi = 0).
__global__ __launch_bounds__(256) void k_pyr_clip_p(double *__restrict__ dst, long n,
                                                    const long long *__restrict__ part, int np) {
    __shared__ long long red[4][4];
    __shared__ double clip[2];
    __shared__ int skip;
    const int tid = threadIdx.x;
    long long v[4] = {0x7fffffffffffffffLL, (long long)0x8000000000000000ULL,
                      0x7fffffffffffffffLL, (long long)0x8000000000000000ULL};
    for (int i = tid; i < np; i += 256) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const long long x = part[(long)i * 4 + k];
            v[k] = (k & 1) ? (x > v[k] ? x : v[k]) : (x < v[k] ? x : v[k]);
        }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        for (int o = 32; o > 0; o >>= 1) {
            const long long x = __shfl_xor(v[k], o);
            v[k] = (k & 1) ? (x > v[k] ? x : v[k]) : (x < v[k] ? x : v[k]);
        }
        if ((tid & 63) == 0) red[k][tid >> 6] = v[k];
    }
    __syncthreads();
    if (tid == 0) {
#pragma unroll
        for (int k = 0; k < 4; ++k)
            for (int i = 1; i < 4; ++i)
                v[k] = (k & 1) ? (red[k][i] > v[k] ? red[k][i] : v[k]) : (red[k][i] < v[k] ? red[k][i] : v[k]);
        clip[0] = dkey_inv(v[0]);
        clip[1] = dkey_inv(v[1]);
        skip = v[2] >= v[0] && v[3] <= v[1];
    }
    __syncthreads();
    if (skip) return;
    const double lo = clip[0], hi = clip[1];
    for (long i = (long)blockIdx.x * 256 + tid; i < n; i += (long)gridDim.x * 256) {
        const double x = dst[i];
        if (x < lo) dst[i] = lo;
        else if (x > hi) dst[i] = hi;
    }
}

// warp's clip of the resampled level to [min, max] of the blurred image (np.clip; only
// values outside the range, which bilinear weights can produce by rounding, are written).
// k_pyr_reduce also recorded the min / max of its outputs: when they lie inside the range
// (the usual case) every block returns without reading the level.
__global__ __launch_bounds__(256) void k_pyr_clip(double *__restrict__ dst, long n,
                                                  const unsigned long long *minmax) {
    __shared__ double clip[2];
    __shared__ int skip;
    if (threadIdx.x < 64) {
        long long kmin = (long long)minmax[threadIdx.x * MM_STRIDE];
        long long kmax = (long long)minmax[threadIdx.x * MM_STRIDE + 1];
        long long omin = (long long)minmax[threadIdx.x * MM_STRIDE + 2];
        long long omax = (long long)minmax[threadIdx.x * MM_STRIDE + 3];
        for (int o = 32; o > 0; o >>= 1) {
            long long a = __shfl_xor(kmin, o), b = __shfl_xor(kmax, o);
            kmin = a < kmin ? a : kmin;
            kmax = b > kmax ? b : kmax;
            a = __shfl_xor(omin, o), b = __shfl_xor(omax, o);
            omin = a < omin ? a : omin;
            omax = b > omax ? b : omax;
        }
        if (threadIdx.x == 0) {
            clip[0] = dkey_inv(kmin); clip[1] = dkey_inv(kmax);
            skip = omin >= kmin && omax <= kmax;
        }
    }
    __syncthreads();
    if (skip) return;
    const double lo = clip[0], hi = clip[1];
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
        const double v = dst[i];
        if (v < lo) dst[i] = lo;
        else if (v > hi) dst[i] = hi;
    }
}

__global__ void k_init_minmax(unsigned long long *mm) {   // <<<1, MM_SLOTS>>>
    mm[threadIdx.x * MM_STRIDE] = 0x7fffffffffffffffULL;       // blurred min / max
    mm[threadIdx.x * MM_STRIDE + 1] = 0x8000000000000000ULL;
    mm[threadIdx.x * MM_STRIDE + 2] = 0x7fffffffffffffffULL;   // output min / max (fused form)
    mm[threadIdx.x * MM_STRIDE + 3] = 0x8000000000000000ULL;
}

// deterministic two-pass mean: block partial sums (fixed order) then one block.
__global__ __launch_bounds__(256) void k_sum_partial(const double *x, long n, double *part) {
    __shared__ double s[256];
    double acc = 0.0;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256)
        acc += x[i];
    s[threadIdx.x] = acc;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) s[threadIdx.x] += s[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) part[blockIdx.x] = s[0];
}

__global__ __launch_bounds__(256) void k_sum_final(const double *part, int nb, long n,
                                                   double *out) {
    __shared__ double s[256];
    double acc = 0.0;
    for (int i = threadIdx.x; i < nb; i += 256) acc += part[i];
    s[threadIdx.x] = acc;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) s[threadIdx.x] += s[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) out[0] = s[0] / (double)n;
}

constexpr int MEAN_BLOCKS = 1024;

// sum of squared deviations from *mean (ia_var_f64's second pass), per block as k_sum_partial
__global__ __launch_bounds__(256) void k_sqdev_partial(const double *x, long n, const double *mean, double *part) {
    __shared__ double s[256];
    const double m = *mean;
    double acc = 0.0;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
        const double d = x[i] - m;
        acc += d * d;
    }
    s[threadIdx.x] = acc;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) s[threadIdx.x] += s[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) part[blockIdx.x] = s[0];
}

}  // namespace ia

using namespace ia;

extern "C" {

const char *ia_last_error(void) { return g_err.c_str(); }
int ia_version(void) { return 1; }

static inline unsigned nblk(long n, int b) { return (unsigned)((n + b - 1) / b); }

int ia_rgb_to_yiq(const void *src, int dt, long npix, double div, double *yiq, double *y,
                  void *stream) {
    IA_ARG(src && npix >= 0 && dt >= 0 && dt <= 2, "ia_rgb_to_yiq: bad args");
    if (npix == 0) return IA_OK;
    k_rgb_to_yiq<<<nblk(npix, 256), 256, 0, S(stream)>>>(src, dt, npix, div, yiq, y);
    IA_LAUNCH_CHECK("k_rgb_to_yiq");
    return IA_OK;
}

int ia_yiq_to_rgb(const double *in, long npix, double *out, void *stream) {
    IA_ARG(in && out && npix >= 0, "ia_yiq_to_rgb: bad args");
    if (npix == 0) return IA_OK;
    k_yiq_to_rgb<<<nblk(npix, 256), 256, 0, S(stream)>>>(in, npix, out);
    IA_LAUNCH_CHECK("k_yiq_to_rgb");
    return IA_OK;
}

int ia_color_output(const double *bp, const double *yiq, const int32_t *s, const int32_t *im, const double *ap,
                    int ah, int aw, int C, long npix, double *out, void *stream) {
    IA_ARG(out && npix >= 0 && ((bp && yiq) || (s && im && ap && ah > 0 && aw > 0 && (C == 1 || C == 3))),
           "ia_color_output: bad args");
    if (npix == 0) return IA_OK;
    k_color_output<<<nblk(npix, 256), 256, 0, S(stream)>>>(yiq ? bp : nullptr, yiq, s, im, ap, ah, aw, C, npix, out);
    IA_LAUNCH_CHECK("k_color_output");
    return IA_OK;
}

int ia_scale_to_f64(const void *src, int dt, long n, double div, double *out, void *stream) {
    IA_ARG(src && out && n >= 0 && dt >= 0 && dt <= 2, "ia_scale_to_f64: bad args");
    if (n == 0) return IA_OK;
    k_scale<<<nblk(n, 256), 256, 0, S(stream)>>>(src, dt, n, div, out);
    IA_LAUNCH_CHECK("k_scale");
    return IA_OK;
}

int ia_axpb_f64(const double *x, long n, int mode, double a, double m, double b, double *y,
                void *stream) {
    IA_ARG(x && y && n >= 0 && (mode == 0 || mode == 1), "ia_axpb_f64: bad args");
    if (n == 0) return IA_OK;
    k_axpb<<<nblk(n, 256), 256, 0, S(stream)>>>(x, n, mode, a, m, b, y);
    IA_LAUNCH_CHECK("k_axpb");
    return IA_OK;
}

// pyramid_reduce form (ia_diag_set_pyr_form): 1 the wave kernel where it applies (default),
// 0 the tiled fused kernel / two-kernel path only
static int g_pyr_stream = env_int("IA_PYR_STREAM", 1);
int ia_diag_set_pyr_form(int stream, int oh) {
    (void)oh;
    const int prev = g_pyr_stream;
    if (stream == 0 || stream == 1) g_pyr_stream = stream;
    return prev;
}
// k_pyr_wave's preconditions, in the device's own arithmetic (no FMA contraction here
// either): halving scales, every sample row / column of the first and last output inside
// the image (the maps are monotone), and a wave's blurred span within its 64 lanes
// the exact halving map k_pyr_wave<true> assumes: floor(v s + t) = 2v and ceil = 2v + 1 for
// every output row / column v (the device evaluates v * s + t the same way: no contraction)
static bool pyr_halving_exact(int n, double s, double t) {
    for (int v = 0; v < n; ++v) {
        const double c = (double)v * s + t;
        if (std::floor(c) != 2.0 * v || std::ceil(c) != 2.0 * v + 1) return false;
    }
    return true;
}
static bool pyr_wave_applies(int H, int W, int h, int w, const double coef[4]) {
    const double sx = coef[0], tx = coef[1], sy = coef[2], ty = coef[3];
    if (H < 4 || W < 4 || !(sx >= 1.25 && sx <= 2.0 + 1e-9 && sy >= 1.25 && sy <= 2.0 + 1e-9))
        return false;
    if (!(tx >= 0 && tx < 1.0 && ty >= 0 && ty < 1.0)) return false;
    const double cmax = (double)(w - 1) * sx + tx, rmax = (double)(h - 1) * sy + ty;
    if (std::ceil(cmax) > W - 1 || std::ceil(rmax) > H - 1) return false;
    // blurred columns of a wave: <= (PW_OW - 1) s + 2 sampled, PW_OW s + 1 owned
    return (PW_OW - 1) * sx + 2 + 6 <= 64 && PW_OW * sx + 1 + 6 <= 64 &&
           (PW_OH - 1) * sy + 2 <= PW_NB && PW_OH * sy + 1 <= PW_NB;
}

size_t ia_pyr_workspace_bytes(int H, int W) {
    return align_up((size_t)H * W * sizeof(double), 256) + MM_SLOTS * MM_STRIDE * 8;
}

int ia_pyr_reduce_f64(const double *src, int H, int W, double *dst, int h, int w,
                      const double coef[4], const double taps[4], void *workspace,
                      void *stream) {
    IA_ARG(src && dst && coef && taps && workspace && H > 0 && W > 0,
           "ia_pyr_reduce_f64: bad args");
    IA_ARG(h == (H + 1) / 2 && w == (W + 1) / 2, "ia_pyr_reduce_f64: dst must be ceil(H/2) x ceil(W/2)");
    double *sm = reinterpret_cast<double *>(workspace);
    unsigned long long *mm = reinterpret_cast<unsigned long long *>(
        reinterpret_cast<char *>(workspace) + align_up((size_t)H * W * sizeof(double), 256));
    hipStream_t st = S(stream);
    // fused form when every output tile's sample rows / cols fit the LDS region (skimage's
    // coefficients of a halving: s <= 2 up to rounding (its fit gives 2.0000000000000004),
    // 0 <= t < 1; the region has 8 spare rows / cols; anything else takes the two-kernel path)
    const bool fused = coef[0] > 0 && coef[0] <= 2.01 && coef[2] > 0 && coef[2] <= 2.01 &&
                       coef[1] >= 0 && coef[1] < 1.0 && coef[3] >= 0 && coef[3] < 1.0 &&
                       H >= 2 && W >= 2;
    if (g_pyr_stream && pyr_wave_applies(H, W, h, w, coef)) {
        const int nstrip = (w + PW_OW - 1) / PW_OW;
        const int nunit = nstrip * ((h + PW_OH - 1) / PW_OH);
        IA_ARG((size_t)nunit * 4 * sizeof(long long) <= ia_pyr_workspace_bytes(H, W),
               "ia_pyr_reduce_f64: workspace too small for the partials");
        long long *part = reinterpret_cast<long long *>(workspace);
        const unsigned grid = (unsigned)((nunit + 3) / 4);
        if (pyr_halving_exact(h, coef[2], coef[3]) && pyr_halving_exact(w, coef[0], coef[1]))
            k_pyr_wave<true><<<grid, 256, 0, st>>>(src, H, W, dst, h, w, nstrip, nunit, coef[0], coef[1],
                                                   coef[2], coef[3], taps[0], taps[1], taps[2], taps[3], part);
        else
            k_pyr_wave<false><<<grid, 256, 0, st>>>(src, H, W, dst, h, w, nstrip, nunit, coef[0], coef[1],
                                                    coef[2], coef[3], taps[0], taps[1], taps[2], taps[3], part);
        IA_LAUNCH_CHECK("k_pyr_wave");
        const long n = (long)h * w;
        k_pyr_clip_p<<<(unsigned)std::min<long>(nblk(n, 256), 64), 256, 0, st>>>(dst, n, part, nunit);
        IA_LAUNCH_CHECK("k_pyr_clip_p");
        return IA_OK;
    }
    k_init_minmax<<<1, MM_SLOTS, 0, st>>>(mm);
    IA_LAUNCH_CHECK("k_init_minmax");
    if (fused) {
        dim3 g(nblk(w, PT_W), nblk(h, PT_H));
        k_pyr_reduce<<<g, 256, 0, st>>>(src, H, W, dst, h, w, coef[0], coef[1], coef[2], coef[3],
                                        taps[0], taps[1], taps[2], taps[3], mm);
        IA_LAUNCH_CHECK("k_pyr_reduce");
        const long n = (long)h * w;
        k_pyr_clip<<<(unsigned)std::min<long>(nblk(n, 256), 1024), 256, 0, st>>>(dst, n, mm);
        IA_LAUNCH_CHECK("k_pyr_clip");
        return IA_OK;
    }
    dim3 g1(nblk(W, BT_W), nblk(H, BT_H));
    k_blur<<<g1, 256, 0, st>>>(src, H, W, taps[0], taps[1], taps[2], taps[3], sm, mm);
    IA_LAUNCH_CHECK("k_blur");
    dim3 g2(nblk(w, 64), nblk(h, 4));
    k_resample<<<g2, 256, 0, st>>>(sm, H, W, dst, h, w, coef[0], coef[1], coef[2], coef[3], mm);
    IA_LAUNCH_CHECK("k_resample");
    return IA_OK;
}

size_t ia_mean_workspace_bytes(long n) { (void)n; return MEAN_BLOCKS * sizeof(double); }

int ia_var_f64(const double *x, long n, double *out, void *workspace, void *stream) {
    // two passes: the mean into out[1], then sum (x - mean)^2 / (n - 1) into out[0]
    // (torch's unbiased var, up to rounding order)
    IA_ARG(x && out && workspace && n > 1, "ia_var_f64: bad args");
    double *part = reinterpret_cast<double *>(workspace);
    int nb = (int)std::min<long>(MEAN_BLOCKS, (n + 255) / 256);
    k_sum_partial<<<nb, 256, 0, S(stream)>>>(x, n, part);
    k_sum_final<<<1, 256, 0, S(stream)>>>(part, nb, n, out + 1);
    k_sqdev_partial<<<nb, 256, 0, S(stream)>>>(x, n, out + 1, part);
    k_sum_final<<<1, 256, 0, S(stream)>>>(part, nb, n - 1, out);
    IA_LAUNCH_CHECK("ia_var_f64");
    return IA_OK;
}

int ia_mean_f64(const double *x, long n, double *out, void *workspace, void *stream) {
    IA_ARG(x && out && workspace && n > 0, "ia_mean_f64: bad args");
    double *part = reinterpret_cast<double *>(workspace);
    int nb = (int)std::min<long>(MEAN_BLOCKS, (n + 255) / 256);
    k_sum_partial<<<nb, 256, 0, S(stream)>>>(x, n, part);
    IA_LAUNCH_CHECK("k_sum_partial");
    k_sum_final<<<1, 256, 0, S(stream)>>>(part, nb, n, out);
    IA_LAUNCH_CHECK("k_sum_final");
    return IA_OK;
}

}  // extern "C"
