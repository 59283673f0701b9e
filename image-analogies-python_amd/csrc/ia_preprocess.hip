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

__global__ void k_init_minmax(unsigned long long *mm) {   // <<<1, MM_SLOTS>>>
    mm[threadIdx.x * MM_STRIDE] = 0x7fffffffffffffffULL;
    mm[threadIdx.x * MM_STRIDE + 1] = 0x8000000000000000ULL;
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
    k_init_minmax<<<1, MM_SLOTS, 0, st>>>(mm);
    IA_LAUNCH_CHECK("k_init_minmax");
    dim3 g1(nblk(W, BT_W), nblk(H, BT_H));
    k_blur<<<g1, 256, 0, st>>>(src, H, W, taps[0], taps[1], taps[2], taps[3], sm, mm);
    IA_LAUNCH_CHECK("k_blur");
    dim3 g2(nblk(w, 64), nblk(h, 4));
    k_resample<<<g2, 256, 0, st>>>(sm, H, W, dst, h, w, coef[0], coef[1], coef[2], coef[3], mm);
    IA_LAUNCH_CHECK("k_resample");
    return IA_OK;
}

size_t ia_mean_workspace_bytes(long n) { (void)n; return MEAN_BLOCKS * sizeof(double); }

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
