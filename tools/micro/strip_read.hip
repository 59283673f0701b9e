// Read-bandwidth probe for the pyramid's access pattern (diagnostic, tools/micro):
// a 2048 x 2048 fp64 image read by 256-thread blocks in strips of C columns x R rows, each
// lane loading V consecutive doubles per row (all rows of the strip issued first), summed
// and written once per lane.  Prints GB/s per (C, R, V).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

template <int V, int R>
__global__ __launch_bounds__(256) void k_strip(const double *__restrict__ src, int W, int H,
                                               int cols, double *__restrict__ out) {
    const int x = blockIdx.x * cols + threadIdx.x * V;
    const int y0 = blockIdx.y * R;
    double acc = 0.0;
    if (threadIdx.x * V < cols && x < W) {
        double v[R][V];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const double *p = src + (long)min(y0 + r, H - 1) * W + x;
            if constexpr (V == 1) v[r][0] = p[0];
            else if constexpr (V == 2) { const double2 t = *reinterpret_cast<const double2 *>(p); v[r][0] = t.x; v[r][1] = t.y; }
            else { const double2 a = reinterpret_cast<const double2 *>(p)[0], b = reinterpret_cast<const double2 *>(p)[1];
                   v[r][0] = a.x; v[r][1] = a.y; v[r][2] = b.x; v[r][3] = b.y; }
        }
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int i = 0; i < V; ++i) acc += v[r][i];
    }
    out[(long)(blockIdx.y * gridDim.x + blockIdx.x) * 256 + threadIdx.x] = acc;
}

template <int V, int R>
static void run(const double *src, double *out, int cols) {
    const int W = 2048, H = 2048;
    dim3 g((W + cols - 1) / cols, H / R);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    std::vector<float> ts;
    for (int i = 0; i < 30; ++i) {
        hipEventRecord(a);
        k_strip<V, R><<<g, 256>>>(src, W, H, cols, out);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    const double us = ts[ts.size() / 2] * 1e3;
    printf("cols %4d rows %2d V %d: %7.1f us  %7.1f GB/s (blocks %d)\n", cols, R, V, us,
           8.0 * W * H / us / 1e3, g.x * g.y);
}

int main() {
    double *src, *out;
    hipMalloc(&src, 8L * 2048 * 2048);
    hipMalloc(&out, 8L * 2048 * 2048);
    hipMemset(src, 0, 8L * 2048 * 2048);
    run<1, 40>(src, out, 256);
    run<1, 16>(src, out, 256);
    run<2, 40>(src, out, 512);
    run<2, 16>(src, out, 512);
    run<4, 16>(src, out, 1024);
    run<4, 8>(src, out, 1024);
    run<1, 8>(src, out, 256);
    run<2, 8>(src, out, 512);
    hipFree(src);
    hipFree(out);
    return 0;
}
