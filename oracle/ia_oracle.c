/* CPU ORACLE for the B' synthesis hot path — TEST INFRASTRUCTURE ONLY.
 *
 * C restatement of the reference's per-level synthesis loop
 * (image_analogies.py:130-220) with the exact brute-force matcher in place of FLANN
 * (algorithms.py:73-75; see oracle/ia_oracle.py for why), used by tests/ as the fast
 * checker for the HIP path and by bench.py's cpu_baseline leg.  Never linked into or
 * called by the product library.
 *
 * It follows oracle/ia_oracle.py operation for operation (and is checked against it
 * bit for bit in tests/test_oracle.py), for luminance (num_ch = 1, 55-dim rows) and colour
 * (num_ch = 3: config.py:29-42, 165-dim rows of (row, col, channel)-flattened windows):
 *   features      algorithms.py:11-47, 78-89   symmetric-padded 3x3 coarse + 5x5 fine
 *   brute force   algorithms.py:73-75 (exact) d = pairwise8( (a-q)*(a-q) ), first min
 *   coherence     algorithms.py:92-130         argmin sqrt(pairwise8(x*x)), first min
 *   kappa test    algorithms.py:133-135 + image_analogies.py:200-211
 *                 d = s*s, s = sqrt(pairwise8(((a-q)*w)^2)); coh iff d_coh <= d_app*f
 *   update        image_analogies.py:214-220
 * pairwise8 is numpy's pairwise_sum (8 accumulators for n <= 128, recursive halves
 * above).  Build: see oracle/Makefile (-O3 -ffp-contract=off: no FMA contraction; OpenMP
 * splits the 1-NN scan over rows, combined in row order).
 */
#include <math.h>
#ifdef _OPENMP
#include <omp.h>
#endif
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define NSM 3
#define NLG 5
#define NHALF 12

static double pairwise8(const double *a, long n) {
    if (n < 8) {
        double res = 0.;
        for (long i = 0; i < n; i++) res += a[i];
        return res;
    } else if (n <= 128) {
        double r[8];
        for (int j = 0; j < 8; j++) r[j] = a[j];
        long i;
        for (i = 8; i < n - (n % 8); i += 8)
            for (int j = 0; j < 8; j++) r[j] += a[i + j];
        double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; i++) res += a[i];
        return res;
    } else {
        long n2 = n / 2;
        n2 -= n2 % 8;
        return pairwise8(a, n2) + pairwise8(a + n2, n - n2);
    }
}

static inline long symi(long i, long n) {   /* np.pad 'symmetric' index map */
    long p = 2 * n;
    i %= p;
    if (i < 0) i += p;
    return i >= n ? p - 1 - i : i;
}

/* feature of pixel (r, c) of a C-channel image pair (channel-interleaved, C = 1 or 3):
 * [3x3 of sm at (r/2, c/2) | 5x5 (or the first 12 positions) of lg], each window flattened
 * (row, col, channel) as extract_patches_2d + flatten do (algorithms.py:20-31) */
static int pixel_feature(const double *sm, long hs, long ws, const double *lg, long h, long w,
                         long r, long c, int full, int C, double *out) {
    int k = 0;
    for (int dr = -1; dr <= 1; dr++)
        for (int dc = -1; dc <= 1; dc++)
            for (int ch = 0; ch < C; ch++)
                out[k++] = sm[(symi(r / 2 + dr, hs) * ws + symi(c / 2 + dc, ws)) * C + ch];
    int nfine = full ? NLG * NLG : NHALF;
    for (int t = 0; t < nfine; t++) {
        int dr = t / NLG - 2, dc = t % NLG - 2;
        for (int ch = 0; ch < C; ch++)
            out[k++] = lg[(symi(r + dr, h) * w + symi(c + dc, w)) * C + ch];
    }
    return k;
}

typedef struct {
    const double *A_sm, *A_lg;   /* A level l-1 (A_hs x A_ws), level l (Ah x Aw)        */
    const double *Ap_sm, *Ap_lg; /* nAp A' images stacked, same shapes as A             */
    int A_hs, A_ws, Ah, Aw, nAp;
    const double *B_sm, *B_lg;   /* B level l-1 (B_hs x B_ws), level l (H x W)          */
    int B_hs, B_ws, H, W;
    const double *Bp_sm;         /* B' level l-1 (already synthesized / init)           */
    double *Bp_lg;               /* B' level l, in: init values, out: synthesized       */
    const double *weights;       /* 55 Gaussian weights (config.py:68-79)               */
    double kappa_factor;         /* 1 + 2**(level-max_levels)*k                          */
    int32_t *s;                  /* out: H*W*2 source pixel (row, col) in A'            */
    int32_t *im;                 /* out: H*W source image number                        */
    long max_pixels;             /* <0: whole level; else stop after this many pixels   */
    int nch;                     /* channels (config.py:29-42 num_ch): 0 or 1, or 3     */
} IaOracleLevel;

#define D 55          /* luminance row length (the scan and batch entries below)         */
#define DMAX 165      /* 3 channels: 55 x 3                                              */
static inline int lch(const IaOracleLevel *L) { return L->nch > 1 ? L->nch : 1; }
int ia_oracle_threads(void);
static int g_threads_build(void) { int t = ia_oracle_threads(); return t > 0 ? t : 1; }

/* database row ix -> 55 C features (algorithms.py:63-67: [A full | A'_img half]) */
static void db_row(const IaOracleLevel *L, long ix, double *f) {
    const int C = lch(L);
    long hw = (long)L->Ah * L->Aw;
    long img = ix / hw, rem = ix - img * hw;
    long r = rem / L->Aw, c = rem % L->Aw;
    int k = pixel_feature(L->A_sm, L->A_hs, L->A_ws, L->A_lg, L->Ah, L->Aw, r, c, 1, C, f);
    pixel_feature(L->Ap_sm + img * (long)L->A_hs * L->A_ws * C, L->A_hs, L->A_ws,
                  L->Ap_lg + img * hw * C, L->Ah, L->Aw, r, c, 0, C, f + k);
}

double *ia_oracle_build_db(const IaOracleLevel *L) {
    const int Dd = 55 * lch(L);
    long N = (long)L->nAp * L->Ah * L->Aw;
    double *db = (double *)malloc(sizeof(double) * N * Dd);
    if (!db) return NULL;
#ifdef _OPENMP
#pragma omp parallel for num_threads(g_threads_build())
#endif
    for (long ix = 0; ix < N; ix++) db_row(L, ix, db + ix * Dd);
    return db;
}

void ia_oracle_free(void *p) { free(p); }

/* pairwise8((a - q)^2) for n = 55, written out: the same operations in the same order as
 * pairwise8 above (8 accumulators over k < 48, tree combine, k = 48..54 sequential), in a
 * form the compiler vectorises across the 8 accumulators (no reassociation: the sums are
 * element-wise vector adds). */
static inline double dist55(const double *a, const double *q) {
    double r[8];
    for (int j = 0; j < 8; j++) { double x = a[j] - q[j]; r[j] = x * x; }
    for (int i = 8; i < 48; i += 8)
        for (int j = 0; j < 8; j++) { double x = a[i + j] - q[i + j]; r[j] += x * x; }
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (int i = 48; i < D; i++) { double x = a[i] - q[i]; res += x * x; }
    return res;
}

/* pairwise8((a - q)^2) for n = 55 (dist55) or any n (165: numpy's halves of 80 and 85) */
static inline double distn(const double *a, const double *q, int n) {
    if (n == D) return dist55(a, q);
    double t[DMAX];
    for (int j = 0; j < n; j++) { double x = a[j] - q[j]; t[j] = x * x; }
    return pairwise8(t, n);
}

/* threads of the 1-NN scan (0 = OpenMP's default, i.e. OMP_NUM_THREADS) */
static int g_threads = 1;
void ia_oracle_set_threads(int n) { g_threads = n; }
int ia_oracle_threads(void) {
#ifdef _OPENMP
    return g_threads > 0 ? g_threads : omp_get_max_threads();
#else
    return 1;
#endif
}

/* first minimum over rows [lo, hi) */
static long nn_range(const double *db, long lo, long hi, const double *q, double *best_out) {
    double best = INFINITY;
    long bi = -1;
    for (long i = lo; i < hi; i++) {
        double d = dist55(db + i * D, q);
        if (d < best) { best = d; bi = i; }
    }
    *best_out = best;
    return bi;
}

/* exact 1-NN over db (N x 55): first minimum of pairwise8((a-q)^2).  With several
 * threads the rows are cut into contiguous blocks, each block's first minimum is taken,
 * and the blocks are combined in row order keeping the first strict minimum: the same
 * row as the serial scan, for any thread count. */
long ia_oracle_nn(const double *db, long N, const double *q, double *dmin_out) {
    int T = ia_oracle_threads();
    if (T > 64) T = 64;
    if (T <= 1 || N < 4096) {
        double best;
        long bi = nn_range(db, 0, N, q, &best);
        if (dmin_out) *dmin_out = best;
        return bi;
    }
    double bd[64];
    long bix[64];
#ifdef _OPENMP
#pragma omp parallel for num_threads(T) schedule(static, 1)
#endif
    for (int t = 0; t < T; t++)
        bix[t] = nn_range(db, N * t / T, N * (t + 1) / T, q, &bd[t]);
    double best = INFINITY;
    long bi = -1;
    for (int t = 0; t < T; t++)
        if (bix[t] >= 0 && bd[t] < best) { best = bd[t]; bi = bix[t]; }
    if (dmin_out) *dmin_out = best;
    return bi;
}

/* M queries (M x 55) at once: idx[m], dmin[m] (the bench's all-cores baseline and the
 * large-database fixtures parallelise over queries) */
void ia_oracle_nn_batch(const double *db, long N, const double *Q, long M, long *idx,
                        double *dmin) {
    int T = ia_oracle_threads();
#ifdef _OPENMP
#pragma omp parallel for num_threads(T > 0 ? T : 1) schedule(dynamic, 1)
#endif
    for (long m = 0; m < M; m++) {
        double d;
        idx[m] = nn_range(db, 0, N, Q + m * D, &d);
        dmin[m] = d;
    }
}

/* ---- exact 1-NN through a projection index (fixture generation only) ------------------
 *
 * The brute-force scan above is the reference-faithful matcher and the bench's CPU
 * baseline.  For full-size fixtures (c4's finest level: 1,048,576 queries x 4,194,304
 * rows) it is too slow, so the fixture scripts may use this index instead.  It returns
 * EXACTLY the brute force's answer: the lexicographic (d, row) minimum, d = dist55 of
 * the same row values in the same operation order, i.e. the first minimum of the scan.
 *
 * Pruning is by a lower bound that holds for every row: for orthonormal v_1..v_P,
 * |a - q|^2 >= sum_i ((a - q).v_i)^2 (Bessel).  Rows are sorted by their first
 * projection, so a query's candidates lie in one contiguous key window.  Rounding is
 * covered by margins: a computed n-term projection differs from the exact one by at most
 * gamma_n sum_k |a_k v_k| (gamma_n = n u / (1 - n u), u = 2^-53), so projection p uses the
 * margin delta_p = max(IX_DELTA, gamma_n (S_p + s_p)) with S_p the largest such sum over the
 * rows (taken at build time) and s_p the query's own (a fixed 1e-10 was argued
 * for 55 terms of |values| <= 1e3 only; 165-dim rows need the dimension in it), the
 * bound is shrunk by (1 - 1e-9) for the vectors' orthonormality error,
 * and a row is only skipped when its bound exceeds best * (1 + 1e-9) + 1e-300, while a
 * computed d differs from the exact |a - q|^2 by < 1e-13 relative.  So a row whose
 * computed d could equal or beat the best is never skipped (ties keep the lowest row).
 */
#define IX_PMAX 8
#define IX_DELTA 1e-10
#define IX_SLACK (1.0 + 1e-9)

typedef struct {
    long N;
    int P;                      /* projections used (1..IX_PMAX)                      */
    int dim;                    /* row length: 55 or 165                              */
    double v[IX_PMAX][DMAX];    /* orthonormal projection vectors                     */
    double smax[IX_PMAX];       /* max over rows of sum_k |a_k v_pk| (rounding margin) */
    long *orig;                 /* sorted position -> original row                    */
    double *proj;               /* N x P projections, sorted order                    */
    double *rows;               /* N x D rows, sorted order                           */
} IaOracleIndex;

static double dotn(const double *a, const double *v, int n) {
    double s = 0.;
    for (int k = 0; k < n; k++) s += a[k] * v[k];
    return s;
}
static double absdotn(const double *a, const double *v, int n) {
    double s = 0.;
    for (int k = 0; k < n; k++) s += fabs(a[k] * v[k]);
    return s;
}
/* gamma_n of an n-term sum (u = 2^-53), rounded up generously */
static double ix_gamma(int n) {
    const double nu = (double)(n + 1) * 0x1p-53;
    return 1.01 * nu / (1.0 - nu);
}

static const double *g_sort_key;
static int cmp_key(const void *x, const void *y) {
    double a = g_sort_key[*(const long *)x], b = g_sort_key[*(const long *)y];
    if (a < b) return -1;
    if (a > b) return 1;
    return *(const long *)x < *(const long *)y ? -1 : (*(const long *)x > *(const long *)y);
}

/* build the index over db (N x Dn, Dn = 55 or 165) with P orthonormal vectors V (P x Dn) */
IaOracleIndex *ia_oracle_index_build2(const double *db, long N, int Dn, const double *V, int P) {
    if (P < 1 || P > IX_PMAX || Dn < 1 || Dn > DMAX) return NULL;
    IaOracleIndex *ix = (IaOracleIndex *)calloc(1, sizeof(IaOracleIndex));
    if (!ix) return NULL;
    ix->N = N;
    ix->P = P;
    ix->dim = Dn;
    for (int p = 0; p < P; p++) memcpy(ix->v[p], V + (long)p * Dn, sizeof(double) * Dn);
    double *key = (double *)malloc(sizeof(double) * N);
    ix->orig = (long *)malloc(sizeof(long) * N);
    ix->proj = (double *)malloc(sizeof(double) * N * P);
    ix->rows = (double *)malloc(sizeof(double) * N * Dn);
    if (!key || !ix->orig || !ix->proj || !ix->rows) {
        free(key); free(ix->orig); free(ix->proj); free(ix->rows); free(ix);
        return NULL;
    }
#ifdef _OPENMP
#pragma omp parallel for num_threads(ia_oracle_threads())
#endif
    for (long i = 0; i < N; i++) { key[i] = dotn(db + i * Dn, ix->v[0], Dn); ix->orig[i] = i; }
    g_sort_key = key;
    qsort(ix->orig, N, sizeof(long), cmp_key);
#ifdef _OPENMP
#pragma omp parallel for num_threads(ia_oracle_threads())
#endif
    for (long s = 0; s < N; s++) {
        const double *a = db + ix->orig[s] * Dn;
        memcpy(ix->rows + s * Dn, a, sizeof(double) * Dn);
        for (int p = 0; p < P; p++) ix->proj[s * P + p] = dotn(a, ix->v[p], Dn);
    }
    for (int p = 0; p < P; p++) {
        double m = 0.;
        for (long i = 0; i < N; i++) {
            const double t = absdotn(db + i * Dn, ix->v[p], Dn);
            m = t > m ? t : m;
        }
        ix->smax[p] = m;
    }
    free(key);
    return ix;
}
IaOracleIndex *ia_oracle_index_build(const double *db, long N, const double *V, int P) {
    return ia_oracle_index_build2(db, N, D, V, P);
}

void ia_oracle_index_free(IaOracleIndex *ix) {
    if (!ix) return;
    free(ix->orig); free(ix->proj); free(ix->rows); free(ix);
}

/* lower bound of |a - q|^2 from the projections, rounding margins applied */
static inline double ix_bound(const double *pa, const double *pq, const double *dl, int P) {
    double lb = 0.;
    for (int p = 0; p < P; p++) {
        double g = fabs(pa[p] - pq[p]) - dl[p];
        if (g > 0.) lb += g * g;
    }
    return lb * (1.0 - 1e-9);
}

/* (d, row) lexicographic minimum over sorted positions [lo, hi), starting from (*bd, *bi) */
static void ix_scan(const IaOracleIndex *ix, long lo, long hi, const double *q, const double *pq,
                    const double *dl, double *bd, long *bi) {
    const int P = ix->P, Dn = ix->dim;
    double best = *bd;
    long bix = *bi;
    for (long s = lo; s < hi; s++) {
        if (ix_bound(ix->proj + s * P, pq, dl, P) > best * IX_SLACK + 1e-300) continue;
        double d = distn(ix->rows + s * Dn, q, Dn);
        long r = ix->orig[s];
        if (d < best || (d == best && r < bix)) { best = d; bix = r; }
    }
    *bd = best;
    *bi = bix;
}

/* first position with key >= x */
static long ix_lower(const IaOracleIndex *ix, double x) {
    long lo = 0, hi = ix->N;
    while (lo < hi) {
        long mid = (lo + hi) / 2;
        if (ix->proj[mid * ix->P] < x) lo = mid + 1; else hi = mid;
    }
    return lo;
}

/* exact 1-NN of q through the index; seeds (original rows, may be NULL) start the bound */
long ia_oracle_index_nn(const IaOracleIndex *ix, const double *db, const double *q,
                        const long *seeds, int nseeds, double *dmin_out) {
    const int P = ix->P, Dn = ix->dim;
    double pq[IX_PMAX], dl[IX_PMAX];
    const double gam = ix_gamma(Dn);
    for (int p = 0; p < P; p++) {
        pq[p] = dotn(q, ix->v[p], Dn);
        const double m = gam * (ix->smax[p] + absdotn(q, ix->v[p], Dn));
        dl[p] = m > IX_DELTA ? m : IX_DELTA;
    }
    double best = INFINITY;
    long bi = -1;
    for (int i = 0; i < nseeds; i++) {
        double d = distn(db + seeds[i] * Dn, q, Dn);
        if (d < best || (d == best && seeds[i] < bi)) { best = d; bi = seeds[i]; }
    }
    /* seed from the key neighbourhood too */
    long c = ix_lower(ix, pq[0]);
    long s0 = c - 256 < 0 ? 0 : c - 256, s1 = c + 256 > ix->N ? ix->N : c + 256;
    ix_scan(ix, s0, s1, q, pq, dl, &best, &bi);
    /* the key window that can hold a row with computed d <= best */
    double r = sqrt(best * IX_SLACK / (1.0 - 1e-9)) + 2 * dl[0];
    long lo = ix_lower(ix, pq[0] - r), hi = ix_lower(ix, pq[0] + r);
    while (hi < ix->N && ix->proj[hi * P] <= pq[0] + r) hi++;
    int T = ia_oracle_threads();
    if (T > 64) T = 64;
    if (T <= 1 || hi - lo < 8192) {
        ix_scan(ix, lo, hi, q, pq, dl, &best, &bi);
    } else {
        double bd[64];
        long bix[64];
#ifdef _OPENMP
#pragma omp parallel for num_threads(T) schedule(static, 1)
#endif
        for (int t = 0; t < T; t++) {
            bd[t] = best;
            bix[t] = bi;
            ix_scan(ix, lo + (hi - lo) * t / T, lo + (hi - lo) * (t + 1) / T, q, pq, dl, &bd[t], &bix[t]);
        }
        for (int t = 0; t < T; t++)
            if (bd[t] < best || (bd[t] == best && bix[t] < bi)) { best = bd[t]; bi = bix[t]; }
    }
    if (dmin_out) *dmin_out = best;
    return bi;
}

/* M independent queries through the index, parallel over queries */
void ia_oracle_index_nn_batch(const IaOracleIndex *ix, const double *db, const double *Q, long M,
                              long *idx, double *dmin) {
    int T = ia_oracle_threads();
    int saved = g_threads;
    g_threads = 1;   /* each query serial inside */
#ifdef _OPENMP
#pragma omp parallel for num_threads(T > 0 ? T : 1) schedule(dynamic, 1)
#endif
    for (long m = 0; m < M; m++) idx[m] = ia_oracle_index_nn(ix, db, Q + m * ix->dim, NULL, 0, &dmin[m]);
    g_threads = saved;
}

static double wdist(const double *a, const double *q, const double *w, int n) {
    double t[DMAX];
    for (int j = 0; j < n; j++) { double v = (a[j] - q[j]) * w[j]; t[j] = v * v; }
    double s = sqrt(pairwise8(t, n));
    return s * s;
}

/* exact 1-NN (first minimum) over any row length n, rows split over threads, combined in
 * row order (the 3-channel synthesis without an index) */
static long nn_n(const double *db, long N, int n, const double *q) {
    int T = ia_oracle_threads();
    if (T > 64) T = 64;
    if (T < 1 || N < 4096) T = 1;
    double bd[64];
    long bix[64];
#ifdef _OPENMP
#pragma omp parallel for num_threads(T) schedule(static, 1)
#endif
    for (int t = 0; t < T; t++) {
        double best = INFINITY;
        long bi = -1;
        for (long i = N * t / T; i < N * (t + 1) / T; i++) {
            double d = distn(db + i * n, q, n);
            if (d < best) { best = d; bi = i; }
        }
        bd[t] = best;
        bix[t] = bi;
    }
    double best = INFINITY;
    long bi = -1;
    for (int t = 0; t < T; t++)
        if (bix[t] >= 0 && bd[t] < best) { best = bd[t]; bi = bix[t]; }
    return bi;
}

/* exact 1-NN of M queries over rows of any length n (brute force; tests cross-check the
 * projection index of 165-dim rows against it) */
void ia_oracle_nn_n_batch(const double *db, long N, int n, const double *Q, long M, long *idx,
                          double *dmin) {
    for (long m = 0; m < M; m++) {
        idx[m] = nn_n(db, N, n, Q + m * n);
        dmin[m] = idx[m] >= 0 ? distn(db + idx[m] * n, Q + m * n, n) : INFINITY;
    }
}

/* image_analogies.py:161-220 for one level (db may be NULL: rows built on the fly).
 * Returns the number of pixels processed. */
long ia_oracle_synth_level_ix(const IaOracleLevel *L, const double *db, const IaOracleIndex *ix);
long ia_oracle_synth_level(const IaOracleLevel *L, const double *db) {
    return ia_oracle_synth_level_ix(L, db, NULL);
}

/* the same loop; with an index (ia_oracle_index_build over this db) the 1-NN goes through
 * ia_oracle_index_nn (the same row and distance as the scan), seeded with the coherence
 * candidates' rows */
long ia_oracle_synth_level_ix(const IaOracleLevel *L, const double *db, const IaOracleIndex *ix) {
    const long H = L->H, W = L->W, Ah = L->Ah, Aw = L->Aw;
    const long N = (long)L->nAp * Ah * Aw;
    double *own = NULL;
    if (!db) { own = ia_oracle_build_db(L); db = own; if (!db) return -1; }
    long npx = H * W;
    if (L->max_pixels >= 0 && L->max_pixels < npx) npx = L->max_pixels;
    const int C = lch(L), Dn = 55 * C;
    if (ix && ix->dim != Dn) return -2;
    double q[DMAX], x[DMAX], t[DMAX];
    for (long qi = 0; qi < npx; qi++) {
        long row = qi / W, col = qi % W;
        /* BBp_feat = [B_features[level][ix] | extract_pixel_feature(Bp pads, half)] */
        int k = pixel_feature(L->B_sm, L->B_hs, L->B_ws, L->B_lg, H, W, row, col, 1, C, q);
        pixel_feature(L->Bp_sm, L->B_hs, L->B_ws, L->Bp_lg, H, W, row, col, 0, C, q + k);
        long p_app_ix;
        if (ix) {
            long seeds[16];
            int ns = 0;
            for (long rr = row - 2 < 0 ? 0 : row - 2; rr <= row; rr++) {
                long cend = col + 3 < W ? col + 3 : W;
                for (long cc = col - 2 < 0 ? 0 : col - 2; cc < cend; cc++) {
                    long rix = rr * W + cc;
                    if (rix >= qi) continue;
                    long sr = L->s[2 * rix] + row - rr, sc = L->s[2 * rix + 1] + col - cc;
                    if (!(sr >= 0 && sr < Ah && sc >= 0 && sc < Aw)) continue;
                    seeds[ns++] = (Ah * (long)L->im[rix] + sr) * Aw + sc;
                }
            }
            p_app_ix = ia_oracle_index_nn(ix, db, q, seeds, ns, NULL);
        } else {
            p_app_ix = Dn == 55 ? ia_oracle_nn(db, N, q, NULL) : nn_n(db, N, Dn, q);
        }
        long hw = Ah * Aw;
        long i_app = p_app_ix / hw, rem = p_app_ix - i_app * hw;
        long pr_app = rem / Aw, pc_app = rem % Aw;
        long pr = pr_app, pc = pc_app, pi = i_app;
        if (qi > 0) {
            /* best_coherence_match (algorithms.py:92-130) */
            double bestd = INFINITY;
            long bsr = -1, bsc = -1, bim = 0, bix = -1;
            for (long rr = row - 2 < 0 ? 0 : row - 2; rr <= row; rr++) {
                long cend = col + 3 < W ? col + 3 : W;
                for (long cc = col - 2 < 0 ? 0 : col - 2; cc < cend; cc++) {
                    long rix = rr * W + cc;
                    if (rix >= qi) continue;
                    long sr = L->s[2 * rix] + row - rr, sc = L->s[2 * rix + 1] + col - cc;
                    if (!(sr >= 0 && sr < Ah && sc >= 0 && sc < Aw)) continue;
                    long img = L->im[rix];
                    long ix = (Ah * img + sr) * Aw + sc;
                    const double *a = db + ix * Dn;
                    for (int j = 0; j < Dn; j++) { x[j] = a[j] - q[j]; t[j] = x[j] * x[j]; }
                    double d = sqrt(pairwise8(t, Dn));
                    if (d < bestd) { bestd = d; bsr = sr; bsc = sc; bim = img; bix = ix; }
                }
            }
            if (bix >= 0) {
                double d_app = wdist(db + p_app_ix * Dn, q, L->weights, Dn);
                double d_coh = wdist(db + bix * Dn, q, L->weights, Dn);
                if (d_coh <= d_app * L->kappa_factor) { pr = bsr; pc = bsc; pi = bim; }
            }
        }
        for (int ch = 0; ch < C; ch++)   /* image_analogies.py:214: every channel */
            L->Bp_lg[(row * W + col) * C + ch] = L->Ap_lg[(pi * hw + pr * Aw + pc) * C + ch];
        L->s[2 * qi] = (int32_t)pr;
        L->s[2 * qi + 1] = (int32_t)pc;
        L->im[qi] = (int32_t)pi;
    }
    free(own);
    return npx;
}
