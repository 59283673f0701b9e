// screen_bench — standalone timing of the matcher's split-f16 MFMA screen (no Python /
// torch), also the process rocprofv3 --pmc runs against.
//
//   screen_bench [--A 2048] [--M 32,64,128,256,342] [--reps 5] [--rounds 5]
//
// Builds the c4 finest-level database (A = A' smooth noise, 2048x2048 -> 4,194,304 rows)
// with libia's own kernels, makes M queries from perturbed database pixels and times
// ia_diag_screen16 with HIP events.  Prints f16 TFLOP/s of 330*M*N algorithmic flops.
#include "screen_setup.h"

int main(int argc, char **argv) {
    int S = 2048, reps = 3, rounds = 5;
    std::vector<int> Ms = {32, 64, 128, 256, 342};
    for (int i = 1; i + 1 < argc; i += 2) {
        if (!strcmp(argv[i], "--A")) S = atoi(argv[i + 1]);
        else if (!strcmp(argv[i], "--M")) Ms = parse_list(argv[i + 1]);
        else if (!strcmp(argv[i], "--reps")) reps = atoi(argv[i + 1]);
        else if (!strcmp(argv[i], "--rounds")) rounds = atoi(argv[i + 1]);
    }
    int Mmax = 0; for (int m : Ms) Mmax = std::max(Mmax, m);
    const ScreenSetup su = make_setup(S, Mmax);
    const long N = su.N, npad = su.npad;
    void *db = su.db, *q16 = su.q16;
    float *segmin = su.segmin;
    hipStream_t st = su.st;
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    printf("N=%ld rows, split-f16 DB %.1f MB; %d rounds x %d reps\n", N, npad * 224 / 1e6, rounds, reps);
    for (int M : Ms) {
        CI(ia_diag_screen16(db, N, q16, M, segmin, st));   // warm-up
        std::vector<float> t;
        for (int rd = 0; rd < rounds; ++rd) {
            CK(hipEventRecord(e0, st));
            for (int r = 0; r < reps; ++r) CI(ia_diag_screen16(db, N, q16, M, segmin, st));
            CK(hipEventRecord(e1, st));
            CK(hipEventSynchronize(e1));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1));
            t.push_back(ms / reps);
        }
        std::sort(t.begin(), t.end());
        const float med = t[t.size() / 2], mn = t[0];
        // 330 f16 flop per (query, row) pair (3 split products x 55 features x 2)
        const double tf = 330.0 * M * (double)N / (med * 1e-3) / 1e12;
        const double peak = 4096.0 * 256 * 2.4e9 / 1e12;
        printf("screen M %4d  median %9.1f us  min %9.1f us  %7.1f TFLOP/s f16  %5.1f%% of %.0f\n",
               M, med * 1e3, mn * 1e3, tf, 100 * tf / peak, peak);
        fflush(stdout);
    }
    return 0;
}
