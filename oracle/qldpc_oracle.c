/*
 * qldpc_oracle.c — CPU restatement of the reference hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product package links, loads or
 * calls this file: only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg use it, as the checker / the CPU baseline.
 *
 * What it restates (file:line under /root/reference):
 *  - BP decoding: the reference calls the third-party `ldpc` package
 *    (`from ldpc import bp_decoder`, src/Decoders.py:47; constructed at
 *    src/Decoders.py:52,80-84 and src/Decoders_SpaceTime.py:207-213).  `ldpc` is
 *    not vendored and not installed; this is a restatement of the published
 *    ldpc 0.1.x `bp_decoder` Cython (bp_decoder.pyx: `bp_decode_log_prob_ratios`
 *    = "minimum_sum", `bp_decode_prob_ratios` = "product_sum") over Neal's
 *    `mod2sparse` lists: rows visited in ascending column order, columns in
 *    ascending row order, flooding schedule, stop when H·x == syndrome or at
 *    max_iter.  Parity of this part is UNPINNED by the reference (it has no
 *    tests or fixtures for BP); see DESIGN.md §Oracle.
 *  - Error sampling / syndromes / failure check: CodeSimulator_DataError
 *    (src/Simulators.py:89-168): per-qubit uniform u, 3-way split
 *    Z if u<pz, X if pz<=u<pz+px, Y if pz+px<=u<pz+px+py; s = H e mod 2;
 *    failure = any(H r) or any(L r) with r = e + decoding.
 *  - Shot RNG: the reference uses Python's MT19937 (`random.random()`),
 *    reseeded per forked worker and therefore not reproducible.  The engine's
 *    fused path draws u from Philox4x32-10 keyed by (seed, shot, qubit) with
 *    the same 53-bit construction as CPython's random.random()
 *    ((a>>5)*2^26 + (b>>6)) / 2^53; the "external uniforms" entry points take u
 *    from the caller (e.g. CPython's own random()) for bit-exact replays.
 *
 * T = double is the reference arithmetic; T = float is the engine's fast mode
 * in the same operation order (so the fp32 GPU kernel is checked bit-exactly
 * too).  Float mode replaces the 1e308 min-sum sentinel by FLT_MAX.
 */
#include <math.h>
#include <float.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define ORACLE_API __attribute__((visibility("default")))

/* ------------------------------------------------------------------ graph */
typedef struct {
    int m, n, E;
    const int32_t *row_ptr, *col_idx; /* CSR, columns ascending in a row      */
    int32_t *col_ptr, *col_edge;      /* CSC: edge ids (row-major), rows asc. */
    int32_t *edge_row;                /* row of each edge                     */
} graph_t;

static int graph_init(graph_t *g, int m, int n, const int32_t *row_ptr, const int32_t *col_idx) {
    g->m = m; g->n = n; g->E = row_ptr[m];
    g->row_ptr = row_ptr; g->col_idx = col_idx;
    g->col_ptr = (int32_t *)calloc((size_t)n + 1, sizeof(int32_t));
    g->col_edge = (int32_t *)malloc(sizeof(int32_t) * (size_t)(g->E ? g->E : 1));
    g->edge_row = (int32_t *)malloc(sizeof(int32_t) * (size_t)(g->E ? g->E : 1));
    if (!g->col_ptr || !g->col_edge || !g->edge_row) return -1;
    for (int e = 0; e < g->E; e++) g->col_ptr[col_idx[e] + 1]++;
    for (int j = 0; j < n; j++) g->col_ptr[j + 1] += g->col_ptr[j];
    int32_t *fill = (int32_t *)malloc(sizeof(int32_t) * (size_t)(n ? n : 1));
    memcpy(fill, g->col_ptr, sizeof(int32_t) * (size_t)n);
    for (int i = 0; i < m; i++)
        for (int e = row_ptr[i]; e < row_ptr[i + 1]; e++) {
            g->edge_row[e] = i;
            g->col_edge[fill[col_idx[e]]++] = e; /* rows visited ascending */
        }
    free(fill);
    return 0;
}

static void graph_free(graph_t *g) {
    free(g->col_ptr); free(g->col_edge); free(g->edge_row);
}

/* ------------------------------------------------------------- BP decoders */
typedef struct {
    int max_iter;
    int method;     /* 0 = product_sum, 1 = minimum_sum */
    double alpha;   /* ms_scaling_factor; 0 => 1 - 2^-iter   */
} bp_params_t;

#define DEFINE_BP(T, SUFFIX, SENTINEL)                                                          \
typedef struct {                                                                                \
    T *b2c, *c2b; int *sgn; T *prior; T *ratio; T *lpr; uint8_t *dec, *dsyn;                  \
} ws_##SUFFIX;                                                                                  \
                                                                                                \
static int ws_alloc_##SUFFIX(ws_##SUFFIX *w, const graph_t *g) {                                \
    size_t E = g->E ? g->E : 1;                                                                 \
    w->b2c = (T *)malloc(sizeof(T) * E); w->c2b = (T *)malloc(sizeof(T) * E);                  \
    w->sgn = (int *)malloc(sizeof(int) * E);                                                    \
    w->prior = (T *)malloc(sizeof(T) * (size_t)(g->n + 1));                                     \
    w->ratio = (T *)malloc(sizeof(T) * (size_t)(g->n + 1));                                     \
    w->lpr = (T *)malloc(sizeof(T) * (size_t)(g->n + 1));                                       \
    w->dec = (uint8_t *)malloc((size_t)g->n + 1); w->dsyn = (uint8_t *)malloc((size_t)g->m + 1);\
    return (w->b2c && w->c2b && w->sgn && w->prior && w->ratio && w->lpr && w->dec && w->dsyn) ? 0 : -1;\
}                                                                                               \
static void ws_free_##SUFFIX(ws_##SUFFIX *w) {                                                  \
    free(w->b2c); free(w->c2b); free(w->sgn); free(w->prior); free(w->ratio); free(w->lpr);    \
    free(w->dec); free(w->dsyn);                                                                \
}                                                                                               \
/* channel priors, computed in double with libm like the Cython code */                         \
static void ws_priors_##SUFFIX(ws_##SUFFIX *w, const graph_t *g, const double *p) {             \
    for (int j = 0; j < g->n; j++) {                                                            \
        w->prior[j] = (T)log((1.0 - p[j]) / p[j]);                                              \
        w->ratio[j] = (T)(p[j] / (1.0 - p[j]));                                                 \
    }                                                                                           \
}                                                                                               \
/* H x == synd ?  (mod2sparse_mulvec + compare) */                                             \
static int synd_equal_##SUFFIX(const graph_t *g, const uint8_t *x, const uint8_t *s, uint8_t *d) {\
    for (int i = 0; i < g->m; i++) {                                                            \
        uint8_t a = 0;                                                                          \
        for (int e = g->row_ptr[i]; e < g->row_ptr[i + 1]; e++) a ^= x[g->col_idx[e]];         \
        d[i] = a;                                                                               \
    }                                                                                           \
    for (int i = 0; i < g->m; i++) if (d[i] != (s[i] & 1)) return 0;                            \
    return 1;                                                                                   \
}                                                                                               \
/* ldpc bp_decode_log_prob_ratios (minimum_sum) */                                              \
static int bp_ms_##SUFFIX(const graph_t *g, const bp_params_t *P, ws_##SUFFIX *w,              \
                          const uint8_t *synd, int *iters_out) {                               \
    const int m = g->m, n = g->n;                                                               \
    for (int j = 0; j < n; j++)                                                                 \
        for (int k = g->col_ptr[j]; k < g->col_ptr[j + 1]; k++) w->b2c[g->col_edge[k]] = w->prior[j];\
    int it;                                                                                     \
    for (it = 1; it <= P->max_iter; it++) {                                                     \
        T alpha = (P->alpha == 0.0) ? (T)(1.0 - ldexp(1.0, -it)) : (T)P->alpha;                \
        for (int i = 0; i < m; i++) {                                                           \
            const int e0 = g->row_ptr[i], e1 = g->row_ptr[i + 1];                               \
            T temp = (T)(SENTINEL);                                                             \
            int sgn = (synd[i] & 1) ? 1 : 0;                                                    \
            for (int e = e0; e < e1; e++) {                                                     \
                w->c2b[e] = temp; w->sgn[e] = sgn;                                              \
                T a = fabs(w->b2c[e]);                                                          \
                if (a < temp) temp = a;                                                         \
                if (w->b2c[e] <= 0) sgn += 1;                                                   \
            }                                                                                   \
            temp = (T)(SENTINEL); sgn = 0;                                                      \
            for (int e = e1 - 1; e >= e0; e--) {                                                \
                if (temp < w->c2b[e]) w->c2b[e] = temp;                                         \
                w->sgn[e] += sgn;                                                               \
                w->c2b[e] *= ((w->sgn[e] & 1) ? -alpha : alpha);                                \
                T a = fabs(w->b2c[e]);                                                          \
                if (a < temp) temp = a;                                                         \
                if (w->b2c[e] <= 0) sgn += 1;                                                   \
            }                                                                                   \
        }                                                                                       \
        for (int j = 0; j < n; j++) {                                                           \
            const int k0 = g->col_ptr[j], k1 = g->col_ptr[j + 1];                               \
            T temp = w->prior[j];                                                               \
            for (int k = k0; k < k1; k++) {                                                     \
                int e = g->col_edge[k];                                                         \
                w->b2c[e] = temp; temp += w->c2b[e];                                            \
            }                                                                                   \
            w->lpr[j] = temp; /* log_prob_ratios[j], the OSD sort key */                        \
            w->dec[j] = (temp <= 0) ? 1 : 0;                                                    \
            temp = (T)0;                                                                        \
            for (int k = k1 - 1; k >= k0; k--) {                                                \
                int e = g->col_edge[k];                                                         \
                w->b2c[e] += temp; temp += w->c2b[e];                                           \
            }                                                                                   \
        }                                                                                       \
        if (synd_equal_##SUFFIX(g, w->dec, synd, w->dsyn)) { *iters_out = it; return 1; }       \
    }                                                                                           \
    *iters_out = P->max_iter;                                                                   \
    return 0;                                                                                   \
}                                                                                               \
/* ldpc bp_decode_prob_ratios (product_sum) */                                                  \
static int bp_ps_##SUFFIX(const graph_t *g, const bp_params_t *P, ws_##SUFFIX *w,              \
                          const uint8_t *synd, int *iters_out) {                               \
    const int m = g->m, n = g->n;                                                               \
    for (int j = 0; j < n; j++)                                                                 \
        for (int k = g->col_ptr[j]; k < g->col_ptr[j + 1]; k++) w->b2c[g->col_edge[k]] = w->ratio[j];\
    int it;                                                                                     \
    for (it = 1; it <= P->max_iter; it++) {                                                     \
        for (int i = 0; i < m; i++) {                                                           \
            const int e0 = g->row_ptr[i], e1 = g->row_ptr[i + 1];                               \
            T temp = (synd[i] & 1) ? (T)-1 : (T)1;                                              \
            for (int e = e0; e < e1; e++) {                                                     \
                w->c2b[e] = temp;                                                               \
                temp *= (T)2 / ((T)1 + w->b2c[e]) - (T)1;                                       \
            }                                                                                   \
            temp = (T)1;                                                                        \
            for (int e = e1 - 1; e >= e0; e--) {                                                \
                w->c2b[e] *= temp;                                                              \
                w->c2b[e] = ((T)1 - w->c2b[e]) / ((T)1 + w->c2b[e]);                            \
                temp *= (T)2 / ((T)1 + w->b2c[e]) - (T)1;                                       \
            }                                                                                   \
        }                                                                                       \
        for (int j = 0; j < n; j++) {                                                           \
            const int k0 = g->col_ptr[j], k1 = g->col_ptr[j + 1];                               \
            T temp = w->ratio[j];                                                               \
            for (int k = k0; k < k1; k++) {                                                     \
                int e = g->col_edge[k];                                                         \
                w->b2c[e] = temp; temp *= w->c2b[e];                                            \
                if (isnan(temp)) temp = (T)1;                                                   \
            }                                                                                   \
            w->dec[j] = (temp >= (T)1) ? 1 : 0;                                                 \
            /* ldpc bp_decode_prob_ratios: log_prob_ratios[j] = log(1 / temp) (OSD's sort key) */\
            w->lpr[j] = (T)log(1.0 / (double)temp);                                             \
            temp = (T)1;                                                                        \
            for (int k = k1 - 1; k >= k0; k--) {                                                \
                int e = g->col_edge[k];                                                         \
                w->b2c[e] *= temp; temp *= w->c2b[e];                                           \
                if (isnan(temp)) temp = (T)1;                                                   \
            }                                                                                   \
        }                                                                                       \
        if (synd_equal_##SUFFIX(g, w->dec, synd, w->dsyn)) { *iters_out = it; return 1; }       \
    }                                                                                           \
    *iters_out = P->max_iter;                                                                   \
    return 0;                                                                                   \
}                                                                                               \
static int bp_run_##SUFFIX(const graph_t *g, const bp_params_t *P, ws_##SUFFIX *w,             \
                           const uint8_t *synd, int *iters) {                                   \
    return P->method == 0 ? bp_ps_##SUFFIX(g, P, w, synd, iters) : bp_ms_##SUFFIX(g, P, w, synd, iters);\
}

DEFINE_BP(double, f64, 1e308)
DEFINE_BP(float, f32, FLT_MAX)

static int norm_max_iter(int max_iter, int n) { return max_iter > 0 ? max_iter : n; }

/*
 * Batch decode of external syndromes (the `bp_decoder.decode(synd)` contract,
 * src/Decoders.py:88-90).  synd: [B][m] 0/1 bytes; corr: [B][n] 0/1 bytes.
 * precision: 64 or 32.  Returns 0 on success.
 */
static int bp_decode_batch_impl(int m, int n, const int32_t *row_ptr, const int32_t *col_idx,
                                const double *channel_probs, int max_iter, int method, double alpha,
                                int precision, const uint8_t *synd, uint8_t *corr, int32_t *iters,
                                uint8_t *conv, double *post, int64_t B, int nthreads);

ORACLE_API int oracle_bp_decode_batch(int m, int n, const int32_t *row_ptr, const int32_t *col_idx,
                                      const double *channel_probs, int max_iter, int method, double alpha,
                                      int precision, const uint8_t *synd, uint8_t *corr, int32_t *iters,
                                      uint8_t *conv, int64_t B, int nthreads) {
    return bp_decode_batch_impl(m, n, row_ptr, col_idx, channel_probs, max_iter, method, alpha, precision,
                                synd, corr, iters, conv, NULL, B, nthreads);
}

/* The same plus post [B][n]: the final log_prob_ratios, the input of ldpc's OSD
 * (bposd_decoder.osd): min-sum's posterior sums, or product-sum's log(1 / ratio)
 * (method 0; ldpc's bp_decode_prob_ratios). */
ORACLE_API int oracle_bp_decode_batch_soft(int m, int n, const int32_t *row_ptr, const int32_t *col_idx,
                                           const double *channel_probs, int max_iter, double alpha,
                                           int precision, const uint8_t *synd, uint8_t *corr, int32_t *iters,
                                           uint8_t *conv, double *post, int64_t B, int nthreads) {
    return bp_decode_batch_impl(m, n, row_ptr, col_idx, channel_probs, max_iter, 1, alpha, precision,
                                synd, corr, iters, conv, post, B, nthreads);
}
ORACLE_API int oracle_bp_decode_batch_soft_method(int m, int n, const int32_t *row_ptr, const int32_t *col_idx,
                                                  const double *channel_probs, int max_iter, int method,
                                                  double alpha, int precision, const uint8_t *synd, uint8_t *corr,
                                                  int32_t *iters, uint8_t *conv, double *post, int64_t B,
                                                  int nthreads) {
    return bp_decode_batch_impl(m, n, row_ptr, col_idx, channel_probs, max_iter, method, alpha, precision,
                                synd, corr, iters, conv, post, B, nthreads);
}

static int bp_decode_batch_impl(int m, int n, const int32_t *row_ptr, const int32_t *col_idx,
                                const double *channel_probs, int max_iter, int method, double alpha,
                                int precision, const uint8_t *synd, uint8_t *corr, int32_t *iters,
                                uint8_t *conv, double *post, int64_t B, int nthreads) {
    graph_t g;
    if (graph_init(&g, m, n, row_ptr, col_idx)) return -1;
    bp_params_t P = {norm_max_iter(max_iter, n), method, alpha};
    int rc = 0;
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel num_threads(nthreads) reduction(| : rc)
#endif
    {
        int tid = 0, nth = 1;
#ifdef _OPENMP
        tid = omp_get_thread_num(); nth = omp_get_num_threads();
#endif
        if (precision == 32) {
            ws_f32 w; if (ws_alloc_f32(&w, &g)) rc |= 1; else {
                ws_priors_f32(&w, &g, channel_probs);
                for (int64_t b = tid; b < B; b += nth) {
                    int it; int c = bp_run_f32(&g, &P, &w, synd + b * m, &it);
                    memcpy(corr + b * n, w.dec, (size_t)n);
                    if (post) for (int j = 0; j < n; j++) post[b * n + j] = (double)w.lpr[j];
                    if (iters) iters[b] = it;
                    if (conv) conv[b] = (uint8_t)c;
                }
                ws_free_f32(&w);
            }
        } else {
            ws_f64 w; if (ws_alloc_f64(&w, &g)) rc |= 1; else {
                ws_priors_f64(&w, &g, channel_probs);
                for (int64_t b = tid; b < B; b += nth) {
                    int it; int c = bp_run_f64(&g, &P, &w, synd + b * m, &it);
                    memcpy(corr + b * n, w.dec, (size_t)n);
                    if (post) for (int j = 0; j < n; j++) post[b * n + j] = (double)w.lpr[j];
                    if (iters) iters[b] = it;
                    if (conv) conv[b] = (uint8_t)c;
                }
                ws_free_f64(&w);
            }
        }
    }
    graph_free(&g);
    return rc ? -1 : 0;
}

/* ------------------------------------------------------------ OSD (bposd) */
/*
 * ldpc 0.1 `bposd_decoder.osd` (the reference's BPOSD_Decoder, src/Decoders.py:26-41)
 * restated in C: the same algorithm, step for step, as oracle.py's osd_decode (pure
 * Python, small codes only), so that the n1600 OSD-E(10) candidates can be checked.
 *   1. stable ascending sort of the columns by the BP posteriors (log_prob_ratios);
 *   2. Neal's mod2sparse_decomp, "first" strategy, on that column order: for pivot i
 *      the first column at or after position i with a set bit in a row not yet used
 *      (rows scanned in index order), swapped into position i; that row becomes row i
 *      and is added to every later row with the pivot bit;
 *   3. OSD-0 by forward (recorded row additions) and back substitution;
 *   4. candidates: osd_e all 2^w inputs on the first w = min(order, n-rank) non-pivot
 *      columns in natural binary order; osd_cs weight-1 on every non-pivot column then
 *      weight-2 inside the first w; each solved the same way, the first of strictly
 *      smaller sum_{j: x_j=1} log(1/p_j) (summed in index order) wins.
 * Bit-vectors (rows as words over columns / over pivot positions) carry the same GF(2)
 * values as the byte loops of osd_decode; a column found empty in the remaining rows
 * stays empty (remaining rows are only ever added to remaining rows), so the pivot scan
 * skips it thereafter.  Parity of this against bposd itself is unpinned (absent).
 */
typedef struct {
    int m, n, MW, NW, rank, method, order;
    uint64_t *hrow;  /* [m][NW] H rows over columns  */
    uint64_t *hcol;  /* [n][MW] H columns over rows  */
    double *wts;     /* log(1/p_j)                   */
} osd_ctx_t;

#define BIT(v, i) (((v)[(i) >> 6] >> ((i) & 63)) & 1ull)
#define FLIP(v, i) ((v)[(i) >> 6] ^= 1ull << ((i) & 63))

static int osd_rank(int m, int NW, const uint64_t *hrow, int n) {
    uint64_t *A = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)m * NW + 8);
    if (!A) return -1;
    memcpy(A, hrow, sizeof(uint64_t) * (size_t)m * NW);
    int r = 0;
    for (int c = 0; c < n && r < m; c++) {
        int p = -1;
        for (int i = r; i < m; i++) if (BIT(A + (size_t)i * NW, c)) { p = i; break; }
        if (p < 0) continue;
        if (p != r) for (int w = 0; w < NW; w++) { uint64_t t = A[(size_t)p * NW + w]; A[(size_t)p * NW + w] = A[(size_t)r * NW + w]; A[(size_t)r * NW + w] = t; }
        for (int i = 0; i < m; i++)
            if (i != r && BIT(A + (size_t)i * NW, c))
                for (int w = 0; w < NW; w++) A[(size_t)i * NW + w] ^= A[(size_t)r * NW + w];
        r++;
    }
    free(A);
    return r;
}

static int osd_ctx_init(osd_ctx_t *C, int m, int n, const int32_t *rp, const int32_t *ci, const double *probs,
                        int method, int order) {
    C->m = m; C->n = n; C->MW = (m + 63) / 64; C->NW = (n + 63) / 64; C->method = method; C->order = order;
    C->hrow = (uint64_t *)calloc((size_t)m * C->NW + 1, sizeof(uint64_t));
    C->hcol = (uint64_t *)calloc((size_t)n * C->MW + 1, sizeof(uint64_t));
    C->wts = (double *)malloc(sizeof(double) * (size_t)(n + 1));
    if (!C->hrow || !C->hcol || !C->wts) return -1;
    for (int i = 0; i < m; i++)
        for (int e = rp[i]; e < rp[i + 1]; e++) {
            FLIP(C->hrow + (size_t)i * C->NW, ci[e]);
            FLIP(C->hcol + (size_t)ci[e] * C->MW, i);
        }
    for (int j = 0; j < n; j++) C->wts[j] = log(1.0 / probs[j]);
    C->rank = osd_rank(m, C->NW, C->hrow, n);
    return C->rank < 0 ? -1 : 0;
}

static void osd_ctx_free(osd_ctx_t *C) { free(C->hrow); free(C->hcol); free(C->wts); }

/* stable merge sort of idx by key ascending (`<`: -0 ties +0, as numpy's stable argsort) */
static void stable_argsort(const double *key, int32_t *idx, int32_t *tmp, int n) {
    for (int i = 0; i < n; i++) idx[i] = i;
    for (int wdt = 1; wdt < n; wdt *= 2)
        for (int lo = 0; lo < n; lo += 2 * wdt) {
            int mid = lo + wdt < n ? lo + wdt : n, hi = lo + 2 * wdt < n ? lo + 2 * wdt : n;
            int a = lo, b = mid, k = lo;
            while (a < mid && b < hi) tmp[k++] = (key[idx[b]] < key[idx[a]]) ? idx[b++] : idx[a++];
            while (a < mid) tmp[k++] = idx[a++];
            while (b < hi) tmp[k++] = idx[b++];
            memcpy(idx + lo, tmp + lo, sizeof(int32_t) * (size_t)(hi - lo));
        }
}

static int osd_decode_one(const osd_ctx_t *C, const uint8_t *synd, const double *post, uint8_t *osd0, uint8_t *osdw) {
    const int m = C->m, n = C->n, MW = C->MW, NW = C->NW, rank = C->rank;
    const int RW = (rank + 63) / 64 + 1;
    int32_t *cols = (int32_t *)malloc(sizeof(int32_t) * (size_t)(2 * n + 2 * m + 2 * rank + 4));
    uint64_t *Bm = (uint64_t *)malloc(sizeof(uint64_t) * ((size_t)m * NW + 1));
    uint64_t *tgt = (uint64_t *)calloc((size_t)rank * MW + 1, sizeof(uint64_t));
    uint64_t *U = (uint64_t *)calloc((size_t)rank * RW + 1, sizeof(uint64_t));
    uint64_t *g = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)(MW + 1));
    uint64_t *xp = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)RW);
    uint8_t *dead = (uint8_t *)calloc((size_t)n + 1, 1), *x = (uint8_t *)malloc((size_t)n + 1);
    if (!cols || !Bm || !tgt || !U || !g || !xp || !dead || !x) {
        free(cols); free(Bm); free(tgt); free(U); free(g); free(xp); free(dead); free(x);
        return -1;
    }
    int32_t *tmp = cols + n, *rows = tmp + n, *rinv = rows + m, *opr = rinv + m, *piv = opr + rank;
    stable_argsort(post, cols, tmp, n);
    for (int r = 0; r < m; r++) rows[r] = rinv[r] = r;
    memcpy(Bm, C->hrow, sizeof(uint64_t) * (size_t)m * NW);
    for (int i = 0; i < rank; i++) {
        int fk = -1, fr = -1;
        for (int k = i; k < n && fk < 0; k++) {
            const int c = cols[k];
            if (dead[c]) continue;
            for (int r = 0; r < m; r++)
                if (BIT(Bm + (size_t)r * NW, c) && rinv[r] >= i) { fk = k; fr = r; break; }
            if (fk < 0) dead[c] = 1;
        }
        if (fk < 0) break; /* cannot happen below rank */
        int32_t t = cols[fk]; cols[fk] = cols[i]; cols[i] = t;
        const int kr = rinv[fr];
        t = rows[kr]; rows[kr] = rows[i]; rows[i] = t;
        rinv[rows[kr]] = kr;
        rinv[rows[i]] = i;
        const int c = cols[i];
        for (int r2 = 0; r2 < m; r2++)
            if (BIT(Bm + (size_t)r2 * NW, c) && rinv[r2] > i) {
                FLIP(tgt + (size_t)i * MW, r2);
                for (int w = 0; w < NW; w++) Bm[(size_t)r2 * NW + w] ^= Bm[(size_t)fr * NW + w];
            }
        opr[i] = fr;
    }
    for (int i = 0; i < rank; i++) piv[i] = cols[i];
    for (int i = 0; i < rank; i++)  /* U[i][j] = Bm[rows[i], piv[j]] for j > i */
        for (int j = i + 1; j < rank; j++)
            if (BIT(Bm + (size_t)rows[i] * NW, piv[j])) FLIP(U + (size_t)i * RW, j);
    const int32_t *ht = cols + rank;
    const int k = n - rank;
    /* solve(g): forward over the recorded additions, back substitution over the pivots */
#define OSD_SOLVE()                                                                          \
    do {                                                                                     \
        for (int i = 0; i < rank; i++)                                                       \
            if (BIT(g, opr[i])) for (int w = 0; w < MW; w++) g[w] ^= tgt[(size_t)i * MW + w];\
        memset(xp, 0, sizeof(uint64_t) * (size_t)RW);                                       \
        for (int i = rank - 1; i >= 0; i--) {                                                \
            uint64_t acc = BIT(g, rows[i]);                                                  \
            const uint64_t *u = U + (size_t)i * RW;                                          \
            for (int w = (i + 1) >> 6; w < RW; w++) acc ^= (uint64_t)__builtin_parityll(u[w] & xp[w]);\
            if (acc & 1ull) FLIP(xp, i);                                                     \
        }                                                                                    \
        memset(x, 0, (size_t)n);                                                             \
        for (int i = 0; i < rank; i++) x[piv[i]] = (uint8_t)BIT(xp, i);                      \
    } while (0)
    memset(g, 0, sizeof(uint64_t) * (size_t)(MW + 1));
    for (int i = 0; i < m; i++) if (synd[i] & 1) FLIP(g, i);
    OSD_SOLVE();
    memcpy(osd0, x, (size_t)n);
    memcpy(osdw, x, (size_t)n);
    if (C->method != 0 && C->order != 0 && k > 0) {
        double best_w = 0.0;
        for (int j = 0; j < n; j++) if (osd0[j]) best_w += C->wts[j];
        const int w = C->order < k ? C->order : k;
        const long long ncand = C->method == 1 ? (1ll << w) : (long long)k + (long long)w * (w - 1) / 2;
        int a = 0, b = 1; /* osd_cs weight-2 pair cursor (i < j inside w) */
        for (long long l = 0; l < ncand; l++) {
            int in[24], nin = 0;
            if (C->method == 1) {
                for (int j = 0; j < w; j++) if ((l >> j) & 1) in[nin++] = j;
            } else if (l < k) {
                in[nin++] = (int)l;
            } else {
                in[nin++] = a; in[nin++] = b;
                if (++b >= w) { ++a; b = a + 1; }
            }
            memset(g, 0, sizeof(uint64_t) * (size_t)(MW + 1));
            for (int i = 0; i < m; i++) if (synd[i] & 1) FLIP(g, i);
            for (int t = 0; t < nin; t++)
                for (int q = 0; q < MW; q++) g[q] ^= C->hcol[(size_t)ht[in[t]] * MW + q];
            OSD_SOLVE();
            for (int t = 0; t < nin; t++) x[ht[in[t]]] = 1;
            double wx = 0.0;
            for (int j = 0; j < n; j++) if (x[j]) wx += C->wts[j];
            if (wx < best_w) { best_w = wx; memcpy(osdw, x, (size_t)n); }
        }
    }
#undef OSD_SOLVE
    free(cols); free(Bm); free(tgt); free(U); free(g); free(xp); free(dead); free(x);
    return 0;
}

/* Batch entry: synd [B][m], post [B][n] -> osd0 / osdw [B][n] (every syndrome decoded;
 * the caller applies bposd's "only when BP did not converge"). method 0/1/2 = osd_0/e/cs. */
ORACLE_API int oracle_osd_decode_batch(int m, int n, const int32_t *row_ptr, const int32_t *col_idx,
                                       const double *channel_probs, int method, int order, const uint8_t *synd,
                                       const double *post, uint8_t *osd0, uint8_t *osdw, int64_t B, int nthreads) {
    if (method == 1 && order > 24) return -1;
    osd_ctx_t C;
    if (osd_ctx_init(&C, m, n, row_ptr, col_idx, channel_probs, method, order)) { osd_ctx_free(&C); return -1; }
    int rc = 0;
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for num_threads(nthreads) schedule(dynamic, 1) reduction(| : rc)
#endif
    for (int64_t b = 0; b < B; b++)
        rc |= osd_decode_one(&C, synd + b * m, post + b * n, osd0 + b * n, osdw + b * n) ? 1 : 0;
    osd_ctx_free(&C);
    return rc ? -1 : 0;
}

/* ------------------------------------------------------------- Philox4x32 */
#define PHILOX_M0 0xD2511F53u
#define PHILOX_M1 0xCD9E8D57u
#define PHILOX_W0 0x9E3779B9u
#define PHILOX_W1 0xBB67AE85u

ORACLE_API void oracle_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
    uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3], k0 = key[0], k1 = key[1];
    for (int r = 0; r < 10; r++) {
        uint64_t p0 = (uint64_t)PHILOX_M0 * c0, p1 = (uint64_t)PHILOX_M1 * c2;
        uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        uint32_t n0 = hi1 ^ c1 ^ k0, n1 = lo1, n2 = hi0 ^ c3 ^ k1, n3 = lo0;
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
        k0 += PHILOX_W0; k1 += PHILOX_W1;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

/* Domain tag in counter word 3 for the data-error stream. */
#define QLDPC_STREAM_DATA 0x51D50001u

/* u for (seed, shot, qubit, stream): CPython random() 53-bit construction */
ORACLE_API double oracle_uniform(uint64_t seed, uint64_t shot, uint32_t qubit, uint32_t stream) {
    uint32_t ctr[4] = {qubit, (uint32_t)shot, (uint32_t)(shot >> 32), stream};
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    uint32_t o[4];
    oracle_philox4x32_10(ctr, key, o);
    return ((double)(o[0] >> 5) * 67108864.0 + (double)(o[1] >> 6)) * (1.0 / 9007199254740992.0);
}

/* src/Simulators.py:99-113 three-way split; returns bit0 = x, bit1 = z */
static inline int classify(double u, double t1, double t2, double t3) {
    if (u < t1) return 2;                 /* Z */
    if (t1 <= u && u < t2) return 1;      /* X */
    if (t2 <= u && u < t3) return 3;      /* Y */
    return 0;
}

/* ------------------------------------------------------------ MC shot loop */
typedef struct {
    int64_t shots, failures;
    int64_t sector_decodes[2], sector_iters[2], sector_nonconv[2], sector_fail[2];
} oracle_counters_t;

/*
 * Fused data-error shot loop (CodeSimulator_DataError._single_run,
 * src/Simulators.py:117-168).  Sector 0 = X errors decoded on hz (logical lz),
 * sector 1 = Z errors decoded on hx (logical lx).  logical_mode: 0 = 'X',
 * 1 = 'Z', 2 = 'Total'; sectors not needed by the mode are skipped (their
 * outcome cannot change the returned failure).  uniforms: NULL => Philox
 * stream, else [shot_count][n] doubles.  per-shot outputs optional.
 */
ORACLE_API int oracle_mc_run(int n,
                             int mx, const int32_t *hz_row_ptr, const int32_t *hz_col_idx,
                             int kx, const int32_t *lz_row_ptr, const int32_t *lz_col_idx,
                             const double *probs_x,
                             int mz, const int32_t *hx_row_ptr, const int32_t *hx_col_idx,
                             int kz, const int32_t *lx_row_ptr, const int32_t *lx_col_idx,
                             const double *probs_z,
                             int max_iter_x, int max_iter_z, int method, double alpha, int precision,
                             double px, double py, double pz, uint64_t seed, uint64_t shot_begin,
                             int64_t shot_count, int logical_mode, const double *uniforms,
                             oracle_counters_t *out, uint8_t *fail_out, uint8_t *err_out /*[S][n] bit0 x bit1 z*/,
                             uint8_t *corr_out /*[S][2][n]*/, int32_t *iters_out /*[S][2]*/,
                             int nthreads) {
    graph_t G[2];
    if (graph_init(&G[0], mx, n, hz_row_ptr, hz_col_idx)) return -1;
    if (graph_init(&G[1], mz, n, hx_row_ptr, hx_col_idx)) return -1;
    const int32_t *lrp[2] = {lz_row_ptr, lx_row_ptr}, *lci[2] = {lz_col_idx, lx_col_idx};
    const int kk[2] = {kx, kz};
    const double *pr[2] = {probs_x, probs_z};
    bp_params_t P[2] = {{norm_max_iter(max_iter_x, n), method, alpha}, {norm_max_iter(max_iter_z, n), method, alpha}};
    const int need[2] = {logical_mode != 1, logical_mode != 0};
    const double t1 = pz, t2 = pz + px, t3 = (pz + px) + py;
    oracle_counters_t tot;
    memset(&tot, 0, sizeof(tot));
    int rc = 0;
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel num_threads(nthreads) reduction(| : rc)
#endif
    {
        int tid = 0, nth = 1;
#ifdef _OPENMP
        tid = omp_get_thread_num(); nth = omp_get_num_threads();
#endif
        oracle_counters_t loc; memset(&loc, 0, sizeof(loc));
        ws_f64 w64[2]; ws_f32 w32[2];
        uint8_t *e = (uint8_t *)malloc((size_t)n), *s = (uint8_t *)malloc((size_t)(mx > mz ? mx : mz) + 1);
        uint8_t *r = (uint8_t *)malloc((size_t)n);
        for (int q = 0; q < 2; q++) {
            if (precision == 32) { if (ws_alloc_f32(&w32[q], &G[q])) rc |= 1; else ws_priors_f32(&w32[q], &G[q], pr[q]); }
            else { if (ws_alloc_f64(&w64[q], &G[q])) rc |= 1; else ws_priors_f64(&w64[q], &G[q], pr[q]); }
        }
        /* static contiguous partition of the shot range */
        int64_t lo = shot_count * tid / nth, hi = shot_count * (tid + 1) / nth;
        for (int64_t b = lo; b < hi && !rc; b++) {
            uint64_t shot = shot_begin + (uint64_t)b;
            uint8_t cls[1]; (void)cls;
            int fail_sec[2] = {0, 0};
            for (int q = 0; q < 2; q++) {
                if (!need[q]) continue;
                for (int j = 0; j < n; j++) {
                    double u = uniforms ? uniforms[b * n + j] : oracle_uniform(seed, shot, (uint32_t)j, QLDPC_STREAM_DATA);
                    int c = classify(u, t1, t2, t3);
                    e[j] = (uint8_t)((q == 0) ? (c & 1) : (c >> 1));
                    if (err_out) err_out[b * n + j] = (uint8_t)c;
                }
                const graph_t *g = &G[q];
                for (int i = 0; i < g->m; i++) {
                    uint8_t a = 0;
                    for (int k = g->row_ptr[i]; k < g->row_ptr[i + 1]; k++) a ^= e[g->col_idx[k]];
                    s[i] = a;
                }
                int it, conv;
                const uint8_t *dec;
                if (precision == 32) { conv = bp_run_f32(g, &P[q], &w32[q], s, &it); dec = w32[q].dec; }
                else { conv = bp_run_f64(g, &P[q], &w64[q], s, &it); dec = w64[q].dec; }
                for (int j = 0; j < n; j++) r[j] = e[j] ^ dec[j];
                int lf = 0;
                for (int l = 0; l < kk[q] && !lf; l++) {
                    uint8_t a = 0;
                    for (int k = lrp[q][l]; k < lrp[q][l + 1]; k++) a ^= r[lci[q][k]];
                    lf = a;
                }
                fail_sec[q] = (!conv) || lf;
                loc.sector_decodes[q]++; loc.sector_iters[q] += it; loc.sector_nonconv[q] += !conv;
                loc.sector_fail[q] += fail_sec[q];
                if (corr_out) memcpy(corr_out + (b * 2 + q) * n, dec, (size_t)n);
                if (iters_out) iters_out[b * 2 + q] = it;
            }
            int f = logical_mode == 0 ? fail_sec[0] : logical_mode == 1 ? fail_sec[1] : (fail_sec[0] || fail_sec[1]);
            loc.shots++; loc.failures += f;
            if (fail_out) fail_out[b] = (uint8_t)(fail_sec[0] | (fail_sec[1] << 1));
        }
        for (int q = 0; q < 2; q++) { if (precision == 32) ws_free_f32(&w32[q]); else ws_free_f64(&w64[q]); }
        free(e); free(s); free(r);
#ifdef _OPENMP
#pragma omp critical
#endif
        {
            tot.shots += loc.shots; tot.failures += loc.failures;
            for (int q = 0; q < 2; q++) {
                tot.sector_decodes[q] += loc.sector_decodes[q]; tot.sector_iters[q] += loc.sector_iters[q];
                tot.sector_nonconv[q] += loc.sector_nonconv[q]; tot.sector_fail[q] += loc.sector_fail[q];
            }
        }
    }
    graph_free(&G[0]); graph_free(&G[1]);
    if (out) *out = tot;
    return rc ? -1 : 0;
}

/* ------------------------------------------- phenomenological space-time */
#define QLDPC_STREAM_PHEN 0x51D50002u

/* GetSpaceTimeCheckMat(h, reps) as CSR (src/Decoders_SpaceTime.py:179-194):
 * row block i = [h | I] on column block i, [0 | I] on column block i-1. */
static int st_graph(int m, int n, const int32_t *rp, const int32_t *ci, int reps, int32_t **orp, int32_t **oci) {
    int w = n + m, E = 0;
    int32_t *r = (int32_t *)malloc(sizeof(int32_t) * ((size_t)reps * m + 1));
    int32_t *c = (int32_t *)malloc(sizeof(int32_t) * ((size_t)reps * (rp[m] + 2 * m) + 1));
    if (!r || !c) { free(r); free(c); return -1; }
    r[0] = 0;
    for (int i = 0; i < reps; i++)
        for (int a = 0; a < m; a++) {
            if (i > 0) c[E++] = (i - 1) * w + n + a;
            for (int e = rp[a]; e < rp[a + 1]; e++) c[E++] = i * w + ci[e];
            c[E++] = i * w + n + a;
            r[i * m + a + 1] = E;
        }
    *orp = r; *oci = c;
    return 0;
}

static void csr_mulvec(const int32_t *rp, const int32_t *ci, int m, const uint8_t *x, uint8_t *y) {
    for (int i = 0; i < m; i++) {
        uint8_t a = 0;
        for (int e = rp[i]; e < rp[i + 1]; e++) a ^= x[ci[e]];
        y[i] = a;
    }
}

/*
 * CodeSimulator_Phenon_SpaceTime._single_run (src/Simulators_SpaceTime.py:433-529)
 * for shot_count samples, with ST_BP_Decoder_syndrome as decoder1
 * (src/Decoders_SpaceTime.py:200-223) and BPDecoder as decoder2.  Sector 0 = X
 * errors (hz, lz), sector 1 = Z errors (hx, lx).  Per repetition the uniforms
 * are drawn in the reference's order: n data qubits (3-way split, :408-422),
 * m_x flips of the hx syndrome (Z sector, :425-427), m_z flips of the hz
 * syndrome (X sector, :429-431); uniform index ((r*reps + j)*P + p), P = n+m_x+m_z.
 * probs_st_*: [reps*(n+m)] ST priors; probs2_*: [n].  trace_out: per sample,
 * per noisy round the Z then X detector histories, then the final Z then X
 * syndromes (the arrays the decoders are handed).
 */
static int phenl_run_impl(int n,
                          int mz, const int32_t *hz_rp, const int32_t *hz_ci,
                          int kx, const int32_t *lz_rp, const int32_t *lz_ci,
                          int mx, const int32_t *hx_rp, const int32_t *hx_ci,
                          int kz, const int32_t *lx_rp, const int32_t *lx_ci,
                          const double *probs_st_x, const double *probs_st_z,
                          const double *probs2_x, const double *probs2_z,
                          int reps, int max_iter_st, int max_iter_2, int method, double alpha, int precision,
                          double px, double py, double pz, double q, uint64_t seed, uint64_t shot_begin,
                          int64_t shot_count, int num_rounds, int logical_mode, const double *uniforms,
                          oracle_counters_t *out, uint8_t *fail_out, uint8_t *trace_out, int nthreads,
                          int osd_method, int osd_order, int fm_max_iter);

ORACLE_API int oracle_phenl_run(int n,
                                int mz, const int32_t *hz_rp, const int32_t *hz_ci,
                                int kx, const int32_t *lz_rp, const int32_t *lz_ci,
                                int mx, const int32_t *hx_rp, const int32_t *hx_ci,
                                int kz, const int32_t *lx_rp, const int32_t *lx_ci,
                                const double *probs_st_x, const double *probs_st_z,
                                const double *probs2_x, const double *probs2_z,
                                int reps, int max_iter_st, int max_iter_2, int method, double alpha, int precision,
                                double px, double py, double pz, double q, uint64_t seed, uint64_t shot_begin,
                                int64_t shot_count, int num_rounds, int logical_mode, const double *uniforms,
                                oracle_counters_t *out, uint8_t *fail_out, uint8_t *trace_out, int nthreads) {
    return phenl_run_impl(n, mz, hz_rp, hz_ci, kx, lz_rp, lz_ci, mx, hx_rp, hx_ci, kz, lx_rp, lx_ci, probs_st_x,
                          probs_st_z, probs2_x, probs2_z, reps, max_iter_st, max_iter_2, method, alpha, precision, px,
                          py, pz, q, seed, shot_begin, shot_count, num_rounds, logical_mode, uniforms, out, fail_out,
                          trace_out, nthreads, -1, 0, -1);
}

/* The same with decoder2 = BPOSD_Decoder (src/Decoders.py:26-41; the Threshold notebook's
 * CodeFamilyPhenlThreshold final round): min-sum BP on the perfect round, then, when it did
 * not converge, the OSD restated above on its final log_prob_ratios (osd_method 0/1/2). */
ORACLE_API int oracle_phenl_run_osd(int n,
                                    int mz, const int32_t *hz_rp, const int32_t *hz_ci,
                                    int kx, const int32_t *lz_rp, const int32_t *lz_ci,
                                    int mx, const int32_t *hx_rp, const int32_t *hx_ci,
                                    int kz, const int32_t *lx_rp, const int32_t *lx_ci,
                                    const double *probs_st_x, const double *probs_st_z,
                                    const double *probs2_x, const double *probs2_z,
                                    int reps, int max_iter_st, int max_iter_2, double alpha, int precision,
                                    double px, double py, double pz, double q, uint64_t seed, uint64_t shot_begin,
                                    int64_t shot_count, int num_rounds, int logical_mode, const double *uniforms,
                                    oracle_counters_t *out, uint8_t *fail_out, uint8_t *trace_out, int nthreads,
                                    int osd_method, int osd_order) {
    if (osd_method < 0 || osd_method > 2) return -1;
    return phenl_run_impl(n, mz, hz_rp, hz_ci, kx, lz_rp, lz_ci, mx, hx_rp, hx_ci, kz, lx_rp, lx_ci, probs_st_x,
                          probs_st_z, probs2_x, probs2_z, reps, max_iter_st, max_iter_2, 1, alpha, precision, px,
                          py, pz, q, seed, shot_begin, shot_count, num_rounds, logical_mode, uniforms, out, fail_out,
                          trace_out, nthreads, osd_method, osd_order, -1);
}

/* The same with decoder1 = FirstMinBPDecoder (src/Decoders.py:49-74, the Single-Shot notebook's
 * CodeSimulator_Phenon decoder1): per noisy round, one-iteration min-sum BP on the running
 * detector vector while the residual weight does not grow, at most fm_max_iter accepted steps, the
 * xor of the accepted decisions folded like a BP decoding; a sector's "iterations" count the
 * accepted steps (no convergence notion: never counted non-converged).  decoder2: BP, or
 * BPOSD_Decoder when osd_method >= 0. */
ORACLE_API int oracle_phenl_run_firstmin(int n,
                                         int mz, const int32_t *hz_rp, const int32_t *hz_ci,
                                         int kx, const int32_t *lz_rp, const int32_t *lz_ci,
                                         int mx, const int32_t *hx_rp, const int32_t *hx_ci,
                                         int kz, const int32_t *lx_rp, const int32_t *lx_ci,
                                         const double *probs_st_x, const double *probs_st_z,
                                         const double *probs2_x, const double *probs2_z,
                                         int reps, int fm_max_iter, int max_iter_2, double alpha, int precision,
                                         double px, double py, double pz, double q, uint64_t seed,
                                         uint64_t shot_begin, int64_t shot_count, int num_rounds, int logical_mode,
                                         const double *uniforms, oracle_counters_t *out, uint8_t *fail_out,
                                         uint8_t *trace_out, int nthreads, int osd_method, int osd_order) {
    if (osd_method > 2 || fm_max_iter < 0) return -1;
    return phenl_run_impl(n, mz, hz_rp, hz_ci, kx, lz_rp, lz_ci, mx, hx_rp, hx_ci, kz, lx_rp, lx_ci, probs_st_x,
                          probs_st_z, probs2_x, probs2_z, reps, 1, max_iter_2, 1, alpha, precision, px, py, pz, q,
                          seed, shot_begin, shot_count, num_rounds, logical_mode, uniforms, out, fail_out, trace_out,
                          nthreads, osd_method < 0 ? -1 : osd_method, osd_order, fm_max_iter);
}

static int phenl_run_impl(int n,
                          int mz, const int32_t *hz_rp, const int32_t *hz_ci,
                          int kx, const int32_t *lz_rp, const int32_t *lz_ci,
                          int mx, const int32_t *hx_rp, const int32_t *hx_ci,
                          int kz, const int32_t *lx_rp, const int32_t *lx_ci,
                          const double *probs_st_x, const double *probs_st_z,
                          const double *probs2_x, const double *probs2_z,
                          int reps, int max_iter_st, int max_iter_2, int method, double alpha, int precision,
                          double px, double py, double pz, double q, uint64_t seed, uint64_t shot_begin,
                          int64_t shot_count, int num_rounds, int logical_mode, const double *uniforms,
                          oracle_counters_t *out, uint8_t *fail_out, uint8_t *trace_out, int nthreads,
                          int osd_method, int osd_order, int fm_max_iter) {
    const int m[2] = {mz, mx};
    const int32_t *hrp[2] = {hz_rp, hx_rp}, *hci[2] = {hz_ci, hx_ci};
    const int32_t *lrp[2] = {lz_rp, lx_rp}, *lci[2] = {lz_ci, lx_ci};
    const int kk[2] = {kx, kz};
    const double *pst[2] = {probs_st_x, probs_st_z}, *p2[2] = {probs2_x, probs2_z};
    graph_t G2[2], GS[2];
    int32_t *srp[2] = {0, 0}, *sci[2] = {0, 0};
    for (int s = 0; s < 2; s++) {
        if (graph_init(&G2[s], m[s], n, hrp[s], hci[s])) return -1;
        if (st_graph(m[s], n, hrp[s], hci[s], reps, &srp[s], &sci[s])) return -1;
        if (graph_init(&GS[s], reps * m[s], reps * (n + m[s]), srp[s], sci[s])) return -1;
    }
    /* ldpc's max_iter = 0 means the decoder's own n (ST: reps*(n+m) of that sector) */
    bp_params_t PSs[2] = {{norm_max_iter(max_iter_st, GS[0].n), method, alpha},
                          {norm_max_iter(max_iter_st, GS[1].n), method, alpha}};
    bp_params_t P2 = {norm_max_iter(max_iter_2, n), method, alpha};
    osd_ctx_t OC[2];
    memset(OC, 0, sizeof(OC));
    if (osd_method >= 0)
        for (int s = 0; s < 2; s++)
            if (osd_ctx_init(&OC[s], m[s], n, hrp[s], hci[s], p2[s], osd_method, osd_order)) return -1;
    const int need[2] = {logical_mode != 1, logical_mode != 0};
    const double t1 = pz, t2 = pz + px, t3 = (pz + px) + py;
    const int Pw = n + mx + mz;
    const int64_t nu = ((int64_t)(num_rounds - 1) * reps + 1) * Pw;
    const int64_t tlen = (int64_t)(num_rounds - 1) * reps * (mx + mz) + mx + mz;
    oracle_counters_t tot;
    memset(&tot, 0, sizeof(tot));
    int rc = 0;
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel num_threads(nthreads) reduction(| : rc)
#endif
    {
        int tid = 0, nth = 1;
#ifdef _OPENMP
        tid = omp_get_thread_num(); nth = omp_get_num_threads();
#endif
        oracle_counters_t loc; memset(&loc, 0, sizeof(loc));
        ws_f64 w64s[2], w64f[2]; ws_f32 w32s[2], w32f[2];
        int mm = mx > mz ? mx : mz;
        uint8_t *cur[2], *hist[2], *det = (uint8_t *)malloc((size_t)reps * mm + 1);
        uint8_t *ser[2], *syn = (uint8_t *)malloc((size_t)mm + 1), *chk = (uint8_t *)malloc((size_t)mm + 1);
        uint8_t *r = (uint8_t *)malloc((size_t)n);
        /* first-min decoder1: running detector vector, its residual, the accepted correction */
        const size_t nst = (size_t)reps * (n + mm);
        uint8_t *fcur = (uint8_t *)malloc((size_t)reps * mm + 1), *fns = (uint8_t *)malloc((size_t)reps * mm + 1);
        uint8_t *fcor = (uint8_t *)malloc(nst + 1);
        uint8_t *o0 = (uint8_t *)malloc((size_t)n), *ow = (uint8_t *)malloc((size_t)n);
        double *post = (double *)malloc(sizeof(double) * (size_t)n);
        for (int s = 0; s < 2; s++) {
            cur[s] = (uint8_t *)malloc((size_t)n);
            hist[s] = (uint8_t *)malloc((size_t)reps * m[s] + 1);
            ser[s] = (uint8_t *)malloc((size_t)m[s] + 1);
            if (precision == 32) {
                if (ws_alloc_f32(&w32s[s], &GS[s]) || ws_alloc_f32(&w32f[s], &G2[s])) rc |= 1;
                else { ws_priors_f32(&w32s[s], &GS[s], pst[s]); ws_priors_f32(&w32f[s], &G2[s], p2[s]); }
            } else {
                if (ws_alloc_f64(&w64s[s], &GS[s]) || ws_alloc_f64(&w64f[s], &G2[s])) rc |= 1;
                else { ws_priors_f64(&w64s[s], &GS[s], pst[s]); ws_priors_f64(&w64f[s], &G2[s], p2[s]); }
            }
        }
        int64_t lo = shot_count * tid / nth, hi = shot_count * (tid + 1) / nth;
        for (int64_t b = lo; b < hi && !rc; b++) {
            const uint64_t shot = shot_begin + (uint64_t)b;
            uint8_t *tr = trace_out ? trace_out + b * tlen : NULL;
#define U(idx) (uniforms ? uniforms[b * nu + (idx)] : oracle_uniform(seed, shot, (uint32_t)(idx), QLDPC_STREAM_PHEN))
            memset(cur[0], 0, (size_t)n); memset(cur[1], 0, (size_t)n);
            for (int rd = 0; rd + 1 < num_rounds; rd++) {
                for (int j = 0; j < reps; j++) {
                    const int64_t base = ((int64_t)rd * reps + j) * Pw;
                    for (int p = 0; p < n; p++) {
                        int c = classify(U(base + p), t1, t2, t3);
                        cur[0][p] ^= (uint8_t)(c & 1); cur[1][p] ^= (uint8_t)(c >> 1);
                    }
                    for (int i = 0; i < mx; i++) ser[1][i] = U(base + n + i) < q;
                    for (int i = 0; i < mz; i++) ser[0][i] = U(base + n + mx + i) < q;
                    for (int s = 0; s < 2; s++) {  /* synd = h_ext @ [cur | serr] */
                        csr_mulvec(hrp[s], hci[s], m[s], cur[s], syn);
                        for (int i = 0; i < m[s]; i++) hist[s][j * m[s] + i] = syn[i] ^ ser[s][i];
                    }
                }
                for (int s = 1; s >= 0; s--) {  /* decoder1_z then decoder1_x, :478-481 */
                    const int R = reps * m[s];
                    for (int k = 0; k < R; k++)  /* Z: consecutive differences; X: raw (quirk Q3) */
                        det[k] = (s == 1 && k >= m[s]) ? (uint8_t)(hist[s][k] ^ hist[s][k - m[s]]) : hist[s][k];
                    if (tr && need[s]) memcpy(tr, det, (size_t)R);  /* skipped sectors: bytes untouched */
                    if (tr) tr += R;
                    if (!need[s]) continue;
                    int it, conv; const uint8_t *e;
                    if (fm_max_iter >= 0) {  /* FirstMinBPDecoder.decode, src/Decoders.py:60-74 */
                        const int nS = GS[s].n;
                        const uint8_t *d;
                        int wc = 0, wn = 0, k = 0;
                        memcpy(fcur, det, (size_t)R); memset(fcor, 0, (size_t)nS);
                        for (int i = 0; i < R; i++) wc += fcur[i];
#define FM_STEP()                                                                                   \
    do {                                                                                            \
        if (precision == 32) { bp_run_f32(&GS[s], &PSs[s], &w32s[s], fcur, &it); d = w32s[s].dec; } \
        else { bp_run_f64(&GS[s], &PSs[s], &w64s[s], fcur, &it); d = w64s[s].dec; }                 \
        csr_mulvec(srp[s], sci[s], R, d, fns);                                                      \
        wn = 0;                                                                                     \
        for (int i = 0; i < R; i++) { fns[i] ^= fcur[i]; wn += fns[i]; }                            \
    } while (0)
                        FM_STEP();
                        while (wn <= wc && k < fm_max_iter) {
                            memcpy(fcur, fns, (size_t)R);
                            for (int p = 0; p < nS; p++) fcor[p] ^= d[p];
                            k++; wc = wn;
                            FM_STEP();
                        }
#undef FM_STEP
                        it = k; conv = 1; e = fcor;
                    } else if (precision == 32) { conv = bp_run_f32(&GS[s], &PSs[s], &w32s[s], det, &it); e = w32s[s].dec; }
                    else { conv = bp_run_f64(&GS[s], &PSs[s], &w64s[s], det, &it); e = w64s[s].dec; }
                    loc.sector_decodes[s]++; loc.sector_iters[s] += it; loc.sector_nonconv[s] += !conv;
                    const int w = n + m[s];
                    for (int i = 0; i < reps; i++)  /* fold, src/Decoders_SpaceTime.py:218-223 */
                        for (int p = 0; p < n; p++) cur[s][p] ^= e[i * w + p];
                }
            }
            {   /* final perfect round, :483-529 */
                const int64_t base = (int64_t)(num_rounds - 1) * reps * Pw;
                for (int p = 0; p < n; p++) {
                    int c = classify(U(base + p), t1, t2, t3);
                    cur[0][p] ^= (uint8_t)(c & 1); cur[1][p] ^= (uint8_t)(c >> 1);
                }
            }
            int fs[2] = {0, 0};
            for (int s = 1; s >= 0; s--) {
                csr_mulvec(hrp[s], hci[s], m[s], cur[s], syn);
                if (tr && need[s]) memcpy(tr, syn, (size_t)m[s]);
                if (tr) tr += m[s];
                if (!need[s]) continue;
                int it, conv; const uint8_t *e;
                if (precision == 32) { conv = bp_run_f32(&G2[s], &P2, &w32f[s], syn, &it); e = w32f[s].dec; }
                else { conv = bp_run_f64(&G2[s], &P2, &w64f[s], syn, &it); e = w64f[s].dec; }
                loc.sector_decodes[s]++; loc.sector_iters[s] += it; loc.sector_nonconv[s] += !conv;
                if (osd_method >= 0 && !conv) {  /* bposd_decoder: OSD on the final log_prob_ratios */
                    for (int p = 0; p < n; p++) post[p] = precision == 32 ? (double)w32f[s].lpr[p] : w64f[s].lpr[p];
                    if (osd_decode_one(&OC[s], syn, post, o0, ow)) rc |= 1;
                    e = ow;
                }
                for (int p = 0; p < n; p++) r[p] = cur[s][p] ^ e[p];
                csr_mulvec(hrp[s], hci[s], m[s], r, chk);
                int f = 0;
                for (int i = 0; i < m[s] && !f; i++) f = chk[i];
                for (int l = 0; l < kk[s] && !f; l++) {
                    uint8_t a = 0;
                    for (int k = lrp[s][l]; k < lrp[s][l + 1]; k++) a ^= r[lci[s][k]];
                    f = a;
                }
                fs[s] = f;
                loc.sector_fail[s] += f;
            }
#undef U
            int f = logical_mode == 0 ? fs[0] : logical_mode == 1 ? fs[1] : (fs[0] || fs[1]);
            loc.shots++; loc.failures += f;
            if (fail_out) fail_out[b] = (uint8_t)(fs[0] | (fs[1] << 1));
        }
        for (int s = 0; s < 2; s++) {
            if (precision == 32) { ws_free_f32(&w32s[s]); ws_free_f32(&w32f[s]); }
            else { ws_free_f64(&w64s[s]); ws_free_f64(&w64f[s]); }
            free(cur[s]); free(hist[s]); free(ser[s]);
        }
        free(det); free(syn); free(chk); free(r); free(o0); free(ow); free(post); free(fcur); free(fns); free(fcor);
#ifdef _OPENMP
#pragma omp critical
#endif
        {
            tot.shots += loc.shots; tot.failures += loc.failures;
            for (int s = 0; s < 2; s++) {
                tot.sector_decodes[s] += loc.sector_decodes[s]; tot.sector_iters[s] += loc.sector_iters[s];
                tot.sector_nonconv[s] += loc.sector_nonconv[s]; tot.sector_fail[s] += loc.sector_fail[s];
            }
        }
    }
    for (int s = 0; s < 2; s++) { graph_free(&G2[s]); graph_free(&GS[s]); free(srp[s]); free(sci[s]); }
    if (osd_method >= 0) { osd_ctx_free(&OC[0]); osd_ctx_free(&OC[1]); }
    if (out) *out = tot;
    return rc ? -1 : 0;
}
