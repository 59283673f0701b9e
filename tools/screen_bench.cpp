// screen_bench — standalone A/B timing of the matcher's MFMA screen (no Python / torch),
// also the process rocprofv3 --pmc runs against (tools/README in DESIGN.md).
//
//   screen_bench [--A 2048] [--M 32,64,128,256,342] [--variants 0,1] [--reps 5]
//
// Builds the c4 finest-level database (A = A' smooth noise, 2048x2048 -> 4,194,304 rows)
// with libia's own kernels, makes M queries from perturbed database pixels and times
// ia_diag_screen per variant with HIP events.  Prints TFLOP/s of 2*55*M*N algorithmic
// flops, and checks that every variant returns identical candidates.
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
#ifdef IA_PROBE
extern "C" int ia_probe_set(unsigned long long *buf);
#endif

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

int main(int argc, char **argv) {
    int S = 2048, reps = 3, rounds = 5;
    std::vector<int> Ms = {32, 64, 128, 256, 342}, vars = {0, 1};
    for (int i = 1; i + 1 < argc; i += 2) {
        if (!strcmp(argv[i], "--A")) S = atoi(argv[i + 1]);
        else if (!strcmp(argv[i], "--M")) Ms = parse_list(argv[i + 1]);
        else if (!strcmp(argv[i], "--variants")) vars = parse_list(argv[i + 1]);
        else if (!strcmp(argv[i], "--reps")) reps = atoi(argv[i + 1]);
        else if (!strcmp(argv[i], "--rounds")) rounds = atoi(argv[i + 1]);
    }
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
    float *db, *amax;
    CK(hipMalloc(&db, ia_db_bytes(N)));
    CK(hipMalloc(&amax, sizeof(float))); CK(hipMemset(amax, 0, sizeof(float)));
    CI(ia_db_build(&src, 0, N, dc, db, amax, st));

    // queries: perturbed features of random pixels (host gather from host copies)
    std::vector<double> Asm((size_t)hs * ws), Apsm((size_t)hs * ws);
    CK(hipMemcpy(Asm.data(), dAs, sizeof(double) * hs * ws, hipMemcpyDeviceToHost));
    CK(hipMemcpy(Apsm.data(), dAps, sizeof(double) * hs * ws, hipMemcpyDeviceToHost));
    int Mmax = 0; for (int m : Ms) Mmax = std::max(Mmax, m);
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
    // variant 7 (bits 4-7 cap, bit 8 uniform): the split-f16 screen
    auto screen = [&](int M, void *out, int v) {
        if ((v & 15) == 7)
            CI(ia_diag_screen16(db, N, q16, M, reinterpret_cast<float *>(out), ((v >> 4) & 15) | (v & 0xfff00), st));
        else
            CI(ia_diag_screen(db, N, qp, M, out, v, st));
    };
#ifdef IA_PROBE
    {   // rescore_probe: phase timestamps of the exact stage (k_rescore) for M queries
        unsigned long long *probe;
        const int NS = 64 * 4 * 16;
        CK(hipMalloc(&probe, NS * 8));
        const int M = Ms.back();
        void *mw; CK(hipMalloc(&mw, ia_match_workspace_bytes(M, N)));
        int64_t *idx; double *dist;
        CK(hipMalloc(&idx, 8 * M)); CK(hipMalloc(&dist, 8 * M));
        IaMatchArgs a{};
        a.src = src; a.db = db; a.row0 = 0; a.nrows = N; a.center = dc; a.amax = amax;
        a.q64 = dq; a.M = M; a.idx = idx; a.dist = dist; a.workspace = mw; a.lsh = nullptr;
        for (int rep = 0; rep < reps + 1; ++rep) {
            CK(hipMemset(probe, 0, NS * 8));
            CI(ia_probe_set(probe));
            CI(ia_match_batch(&a, st));
            CK(hipStreamSynchronize(st));
            CI(ia_probe_set(nullptr));
            std::vector<unsigned long long> h(NS);
            CK(hipMemcpy(h.data(), probe, h.size() * 8, hipMemcpyDeviceToHost));
            if (rep == 0) continue;   // warm-up
            const int nb = M < 64 ? M : 64;
            unsigned long long t0 = ~0ULL;
            for (int b = 0; b < nb; ++b) if (h[b * 64]) t0 = std::min(t0, h[b * 64]);
            printf("M=%d rep %d: wall_clock64 @100 MHz; us after the block's wave-0 mark 0; "
                   "mean / max over %d blocks\n", M, rep, nb);
            for (int i = 1; i < 16; ++i) {
                printf("  mark %2d:", i);
                bool any = false;
                for (int w = 0; w < 4; ++w) {
                    double sum = 0, mx = 0; int n = 0;
                    for (int b = 0; b < nb; ++b) {
                        const unsigned long long x = h[(b * 4 + w) * 16 + i], s0 = h[b * 64];
                        if (!x || !s0) continue;
                        const double d = ((double)x - (double)s0) / 100.0;
                        sum += d; mx = std::max(mx, d); ++n;
                    }
                    if (n) { printf("  w%d %6.2f/%6.2f", w, sum / n, mx); any = true; }
                    else printf("  w%d      -/     -", w);
                }
                printf("%s\n", any ? "" : "  (unused)");
            }
            double sk = 0;
            for (int b = 0; b < nb; ++b) sk = std::max(sk, (h[b * 64] - t0) / 100.0);
            printf("  block start skew: %.2f us\n", sk);
        }
        return 0;
    }
#endif
    const size_t cb = ia_diag_cand_bytes(Mmax, N);
    char *cand, *cand_ref;
    CK(hipMalloc(&cand, cb)); CK(hipMalloc(&cand_ref, cb));
    std::vector<char> h1(cb), h2(cb);
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    printf("N=%ld rows, DB %.1f MB; %d interleaved rounds x %d reps per variant\n", N,
           N * IA_DP * 4 / 1e6, rounds, reps);
    for (int M : Ms) {
        std::vector<std::vector<float>> t(vars.size());
        for (size_t vi = 0; vi < vars.size(); ++vi)       // warm-up + result check
            screen(M, vi == 0 ? cand_ref : cand, vars[vi]);
        for (int rd = 0; rd < rounds; ++rd)
            for (size_t vi = 0; vi < vars.size(); ++vi) {
                char *out = vi == 0 ? cand_ref : cand;
                CK(hipEventRecord(e0, st));
                for (int r = 0; r < reps; ++r) screen(M, out, vars[vi]);
                CK(hipEventRecord(e1, st));
                CK(hipEventSynchronize(e1));
                float ms; CK(hipEventElapsedTime(&ms, e0, e1));
                t[vi].push_back(ms / reps);
            }
        for (size_t vi = 0; vi < vars.size(); ++vi) {
            std::vector<float> v = t[vi];
            std::sort(v.begin(), v.end());
            const float med = v[v.size() / 2], mn = v[0];
            const double tf = 2.0 * 55 * M * (double)N / (med * 1e-3) / 1e12;
            long diff = 0;
            if (vi > 0 && (vars[vi] & 15) == (vars[0] & 15)) {
                screen(M, cand_ref, vars[0]);
                screen(M, cand, vars[vi]);
                CK(hipStreamSynchronize(st));
                CK(hipMemcpy(h1.data(), cand_ref, cb, hipMemcpyDeviceToHost));
                CK(hipMemcpy(h2.data(), cand, cb, hipMemcpyDeviceToHost));
                const size_t used = (size_t)M * cb / ia_diag_qp_rows(Mmax);
                for (size_t i = 0; i < used && i < cb; ++i) diff += h1[i] != h2[i];
            }
            printf("variant 0x%03x M %4d  median %9.1f us  min %9.1f us  %6.1f TFLOP/s  %5.1f%% of 157.3  out-diff %ld\n",
                   vars[vi], M, med * 1e3, mn * 1e3, tf, 100 * tf / 157.3, diff);
        }
        fflush(stdout);
    }
    return 0;
}
