// screen_setup.h — the c4 finest-level database and queries shared by the screen
// harnesses (screen_bench, screen_lab): A = A' smooth noise S x S -> S^2 split-f16 rows built
// with libia's own kernels; Mmax queries = perturbed database pixels.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "../include/ia.h"
#include "../include/ia_diag.h"

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                \
        }                                                                           \
    } while (0)
#define CI(x)                                                                       \
    do {                                                                            \
        int r_ = (x);                                                               \
        if (r_ != 0) { fprintf(stderr, "%s -> %d: %s\n", #x, r_, ia_last_error()); exit(1); } \
    } while (0)

static std::vector<int> parse_list(const char *s) {
    std::vector<int> v;
    std::string t(s);
    size_t p = 0;
    while (p < t.size()) {
        size_t q = t.find(',', p);
        if (q == std::string::npos) q = t.size();
        v.push_back((int)strtol(t.substr(p, q - p).c_str(), nullptr, 0));
        p = q + 1;
    }
    return v;
}

struct ScreenSetup {
    long N, npad, nseg;
    int ch, qrows;
    void *db, *q16;
    float *segmin;
    hipStream_t st;
    // host copies of the level (for harness-side layouts): fine A, A' (H x W), coarse
    // (hs x ws), the centre values and the split bound
    int H, W, hs, ws;
    std::vector<double> A, Ap, Asm, Apsm;
    double mA, mAp;
    float amax;
};

static void box_blur(std::vector<double> &img, int H, int W, int r) {
    std::vector<double> tmp(img.size());
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            double s = 0; int n = 0;
            for (int d = -r; d <= r; ++d) { int xx = x + d; if (xx >= 0 && xx < W) { s += img[(size_t)y * W + xx]; ++n; } }
            tmp[(size_t)y * W + x] = s / n;
        }
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            double s = 0; int n = 0;
            for (int d = -r; d <= r; ++d) { int yy = y + d; if (yy >= 0 && yy < H) { s += tmp[(size_t)yy * W + x]; ++n; } }
            img[(size_t)y * W + x] = s / n;
        }
}

static inline int symi(int i, int n) {
    int p = 2 * n; i %= p; if (i < 0) i += p; return i >= n ? p - 1 - i : i;
}

static ScreenSetup make_setup(int S, int Mmax) {
    const int H = S, W = S, hs = (H + 1) / 2, ws = (W + 1) / 2;
    std::mt19937_64 rng(1234);
    std::uniform_real_distribution<double> U(0, 1);
    std::vector<double> A((size_t)H * W), Ap;
    for (auto &x : A) x = U(rng);
    box_blur(A, H, W, 3); box_blur(A, H, W, 3);
    double mn = 1e9, mx = -1e9;
    for (double x : A) { mn = std::min(mn, x); mx = std::max(mx, x); }
    for (auto &x : A) x = (x - mn) / (mx - mn);
    Ap = A; box_blur(Ap, H, W, 2);

    hipStream_t st; CK(hipStreamCreate(&st));
    double *dA, *dAp, *dAs, *dAps, *dc, *dmean;
    CK(hipMalloc(&dA, sizeof(double) * H * W)); CK(hipMalloc(&dAp, sizeof(double) * H * W));
    CK(hipMalloc(&dAs, sizeof(double) * hs * ws)); CK(hipMalloc(&dAps, sizeof(double) * hs * ws));
    CK(hipMalloc(&dc, sizeof(double) * 64)); CK(hipMalloc(&dmean, sizeof(double) * 2));
    CK(hipMemcpy(dA, A.data(), sizeof(double) * H * W, hipMemcpyHostToDevice));
    CK(hipMemcpy(dAp, Ap.data(), sizeof(double) * H * W, hipMemcpyHostToDevice));
    void *pws; CK(hipMalloc(&pws, ia_pyr_workspace_bytes(H, W)));
    const double coef[4] = {2.0, 0.5, 2.0, 0.5};
    const double taps[4] = {0.598, 0.194, 0.0066, 0.00002};
    CI(ia_pyr_reduce_f64(dA, H, W, dAs, hs, ws, coef, taps, pws, st));
    CI(ia_pyr_reduce_f64(dAp, H, W, dAps, hs, ws, coef, taps, pws, st));
    void *mws; CK(hipMalloc(&mws, ia_mean_workspace_bytes((long)H * W)));
    CI(ia_mean_f64(dA, (long)H * W, dmean, mws, st));
    CI(ia_mean_f64(dAp, (long)H * W, dmean + 1, mws, st));
    double means[2]; CK(hipMemcpyAsync(means, dmean, 16, hipMemcpyDeviceToHost, st));
    CK(hipStreamSynchronize(st));
    CI(ia_center_fill(dc, means[0], means[1], st));
    IaSrcLevel src{dAs, dA, dAps, dAp, hs, ws, H, W, 1};
    const long N = (long)H * W;
    void *db; float *amax;
    CK(hipMalloc(&db, ia_db_bytes(N)));
    CK(hipMalloc(&amax, sizeof(float))); CK(hipMemset(amax, 0, sizeof(float)));
    CI(ia_db_build(&src, 0, N, dc, db, amax, st));

    // queries: perturbed features of random pixels (host gather from host copies)
    std::vector<double> Asm((size_t)hs * ws), Apsm((size_t)hs * ws);
    CK(hipMemcpy(Asm.data(), dAs, sizeof(double) * hs * ws, hipMemcpyDeviceToHost));
    CK(hipMemcpy(Apsm.data(), dAps, sizeof(double) * hs * ws, hipMemcpyDeviceToHost));
    std::vector<double> q((size_t)Mmax * IA_DP, 0.0);
    std::normal_distribution<double> G(0, 0.01);
    for (int m = 0; m < Mmax; ++m) {
        int r = (int)(U(rng) * H), c = (int)(U(rng) * W), k = 0;
        double *o = q.data() + (size_t)m * IA_DP;
        for (int t = 0; t < 9; ++t) o[k++] = Asm[(size_t)symi(r / 2 + t / 3 - 1, hs) * ws + symi(c / 2 + t % 3 - 1, ws)];
        for (int t = 0; t < 25; ++t) o[k++] = A[(size_t)symi(r + t / 5 - 2, H) * W + symi(c + t % 5 - 2, W)];
        for (int t = 0; t < 9; ++t) o[k++] = Apsm[(size_t)symi(r / 2 + t / 3 - 1, hs) * ws + symi(c / 2 + t % 3 - 1, ws)];
        for (int t = 0; t < 12; ++t) o[k++] = Ap[(size_t)symi(r + t / 5 - 2, H) * W + symi(c + t % 5 - 2, W)];
        for (int j = 0; j < 55; ++j) o[j] += G(rng);
    }
    double *dq, *dnq; float *qp;
    CK(hipMalloc(&dq, sizeof(double) * q.size()));
    CK(hipMemcpy(dq, q.data(), sizeof(double) * q.size(), hipMemcpyHostToDevice));
    const int qrows = ia_diag_qp_rows(Mmax);
    CK(hipMalloc(&qp, sizeof(float) * IA_DP * qrows)); CK(hipMemset(qp, 0, sizeof(float) * IA_DP * qrows));
    CK(hipMalloc(&dnq, sizeof(double) * qrows));
    void *q16;
    CK(hipMalloc(&q16, (size_t)256 * qrows)); CK(hipMemset(q16, 0, (size_t)256 * qrows));
    CI(ia_diag_query_rows16(dq, Mmax, dc, amax, qp, q16, dnq, st));
    const long npad = ia_db_rows_padded(N);
    const int ch = ia_db_chunk_rows(N);
    const long nseg = npad / (ch < 512 ? ch : 512);
    float *segmin;
    CK(hipMalloc(&segmin, sizeof(float) * (size_t)qrows * nseg));
    float amax_h; CK(hipMemcpy(&amax_h, amax, sizeof(float), hipMemcpyDeviceToHost));
    return ScreenSetup{N, npad, nseg, ch, qrows, db, q16, segmin, st, H, W, hs, ws,
                       A, Ap, Asm, Apsm, means[0], means[1], amax_h};
}
