/*
 * knn_compat.c -- knn_search_mpi_compat(): the neighbour lists the reference
 * MPI programs (mpi-knn-parallel_blocking.c / _non_blocking.c) actually
 * compute, bugs included, on the GPU engine.  Opt-in; the
 * default path (knn_search) has the serial semantics.
 *
 * What rank r of P holds after its loops (blk:81-244; nb:91-259 moves the
 * same data with Isend/Irecv + Wait):
 *   - R = floor(m / P) rows per rank; the remainder is dropped (blk:81);
 *   - step 0 folds its OWN block (blk:155-181 reads matrix[i], not the
 *     block just received), with real ids and labels (blk:107-108,176-177);
 *   - the first hop sends only R*n of the R*(n+2) doubles of the sender's
 *     matrix (count m/procs*n, blk:130,137,146): in the receiver's
 *     (n+2)-strided matrix_temp, rows below q = floor(R*n/(n+2)) arrive
 *     whole, row q gets its first R*n - q*(n+2) doubles (features only, up
 *     to n), later rows stay zero (fresh allocation, blk:82);
 *   - matrix_send copies only the n feature columns (blk:169,231), so every
 *     later block carries id 0 and label 0, and the truncation travels on;
 *   - iteration p = 0..P-2 (blk:187-244) folds the block that started on
 *     rank r-2-p: r-2, r-3, ..., r-P = r (its own block again, truncated);
 *     block r-1 is never seen.
 * Insertion is strict `<` then a stable distance-only qsort (blk:24-31,
 * 172-178), so equal distances keep scan order.  Here every visit gets
 * scan-order ids (own block: its real ids; visit p: m + p*R + row) so the
 * engine's (distance, id) order IS scan order; ids above m are then written
 * as idx 0 / label 0.  The vote (blk:252-270) is knn_classify(KNN_VOTE_MPI);
 * the reference's own vote writes class[-1] on these label-0 records (F6),
 * which knn_classify skips.
 *
 * All P ranks run one after another on device 0 (a parity/debug mode, not a
 * performance path).
 */
#include "knn_internal.h"

#include <hip/hip_runtime_api.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

static double compat_now(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

/* rows [b*R, (b+1)*R) of X as row-major R x n; truncated as received by
 * the first hop when `trunc` */
static void compat_rows(const double *X, size_t m, size_t n, int layout, size_t R, int b,
                        int trunc, double *dst)
{
    const size_t base = (size_t)b * R;
    for (size_t i = 0; i < R; i++)
        for (size_t j = 0; j < n; j++)
            dst[i * n + j] = layout == KNN_COLMAJOR ? X[(base + i) + j * m] : X[(base + i) * n + j];
    if (!trunc) return;
    const size_t sent = R * n, stride = n + 2;
    const size_t q = sent / stride;          /* whole rows received */
    for (size_t i = q; i < R; i++) {
        const size_t got = i == q ? sent - q * stride : 0;   /* doubles of row i received */
        for (size_t j = (got < n ? got : n); j < n; j++) dst[i * n + j] = 0.0;
    }
}

int knn_search_mpi_compat(const double *X, size_t m, size_t n, int layout, const double *labels,
                          int k, int procs, knn_neighbour_t *out)
{
    if (!X || !out || m == 0 || n == 0 || k <= 0 || procs < 2) return KNN_ERR_INVALID;
    if (layout != KNN_COLMAJOR && layout != KNN_ROWMAJOR) return KNN_ERR_INVALID;
    if (k > KNN_MAX_K) return KNN_ERR_UNSUPPORTED;
    const int P = procs;
    const size_t R = m / (size_t)P;
    if (R == 0) return KNN_ERR_INVALID;
    if (m + (size_t)P * R > (size_t)0x7fffffff) return KNN_ERR_UNSUPPORTED;   /* int ids */
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return KNN_ERR_NODEVICE;

    const size_t bytes = knn_block_bytes_dt(R, n, KNN_F64);
    const size_t moff = knn_block_meta_offset_dt(R, n, KNN_F64);
    int rc = KNN_OK;
    knn_ctx_t *ctx = NULL;
    void **blk = (void **)calloc((size_t)P, sizeof(void *));   /* [0] own, [1+p] visit p */
    double *h_rows = (double *)malloc(R * n * sizeof(double));
    double *d_rows = NULL, *d_meta = NULL;
    knn_neighbour_t *d_out = NULL;
    if (!blk || !h_rows) rc = KNN_ERR_NOMEM;
    if (!rc && hipSetDevice(0) != hipSuccess) rc = KNN_ERR_HIP;
    if (!rc && (hipMalloc((void **)&d_rows, R * n * sizeof(double)) != hipSuccess ||
                hipMalloc((void **)&d_meta, KNN_META_DOUBLES * sizeof(double)) != hipSuccess ||
                hipMalloc((void **)&d_out, R * (size_t)k * sizeof(knn_neighbour_t)) != hipSuccess))
        rc = KNN_ERR_NOMEM;
    for (int v = 0; v < P && !rc; v++)
        if (hipMalloc(&blk[v], bytes) != hipSuccess) rc = KNN_ERR_NOMEM;
    if (!rc) rc = knn_ctx_create_dt(&ctx, 0, R, n, R, k, KNN_F64);

    const double t0 = compat_now();
    for (int r = 0; r < P && !rc; r++) {
        /* pack the own block, then the P-1 truncated visits */
        double meta[KNN_META_DOUBLES];
        for (int v = 0; v < P && !rc; v++) {
            const int b = v == 0 ? r : ((r - 1 - v) % P + P) % P;
            compat_rows(X, m, n, layout, R, b, v > 0, h_rows);
            if (hipMemcpy(d_rows, h_rows, R * n * sizeof(double), hipMemcpyHostToDevice) != hipSuccess) {
                rc = KNN_ERR_HIP;
                break;
            }
            rc = knn_block_pack_dt(blk[v], KNN_F64, R, R, n, d_rows, KNN_F64, n, KNN_ROWMAJOR, NULL);
            double bm[KNN_META_DOUBLES];
            if (!rc && hipMemcpy(bm, (char *)blk[v] + moff, sizeof(bm), hipMemcpyDeviceToHost) != hipSuccess)
                rc = KNN_ERR_HIP;
            for (int i = 0; i < KNN_META_DOUBLES && !rc; i++)
                meta[i] = (v == 0 || bm[i] > meta[i]) ? bm[i] : meta[i];   /* the ring's max-reduce */
        }
        if (!rc && hipMemcpy(d_meta, meta, sizeof(meta), hipMemcpyHostToDevice) != hipSuccess)
            rc = KNN_ERR_HIP;
        if (!rc) rc = knn_ctx_begin(ctx, blk[0], R, (size_t)r * R, d_meta, NULL);
        for (int v = 0; v < P && !rc; v++)
            rc = knn_ctx_step(ctx, blk[v], R, v == 0 ? (size_t)r * R : m + (size_t)(v - 1) * R, NULL);
        size_t unresolved = 0;
        if (!rc) rc = knn_ctx_end(ctx, d_out, &unresolved, NULL);
        if (!rc && unresolved) {
            for (int v = 0; v < P && !rc; v++)
                rc = knn_ctx_rescan_step(ctx, blk[v], R, v == 0 ? (size_t)r * R : m + (size_t)(v - 1) * R,
                                         NULL);
            if (!rc) rc = knn_ctx_rescan_end(ctx, d_out, NULL);
        }
        knn_neighbour_t *o = out + (size_t)r * R * (size_t)k;
        if (!rc && hipMemcpy(o, d_out, R * (size_t)k * sizeof(knn_neighbour_t), hipMemcpyDeviceToHost) !=
                       hipSuccess)
            rc = KNN_ERR_HIP;
        /* ids above m came from forwarded blocks: id and label columns never
         * copied (blk:169,231) */
        for (size_t e = 0; e < R * (size_t)k && !rc; e++) {
            if (o[e].idx > (int32_t)m) {
                o[e].idx = 0;
                o[e].label = 0;
            } else if (o[e].idx > 0) {
                o[e].label = labels ? (int32_t)labels[o[e].idx - 1] : 0;
            } else {
                o[e].label = 0;
            }
        }
    }
    knn_set_last_search_seconds(compat_now() - t0);

    if (ctx) knn_ctx_destroy(ctx);
    for (int v = 0; blk && v < P; v++) hipFree(blk[v]);
    hipFree(d_rows);
    hipFree(d_meta);
    hipFree(d_out);
    free(blk);
    free(h_rows);
    return rc;
}
