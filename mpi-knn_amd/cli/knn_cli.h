/*
 * knn_cli.h -- shared driver of the three drop-in executables.
 *
 * They keep the reference CLI and stdout contract:
 *   knn-serial                         (serial:36-133)
 *   mpi-knn-parallel_blocking P T      (blk:50-278)
 *   mpi-knn-parallel_non_blocking P T  (nb:59-297)
 * The corpus is read from "mnist_train.mat" in the working directory
 * (serial:40, blk:65) unless KNN_MAT names another file; variables
 * train_X / train_labels (serial:47,52).  P selects the GPU count (one GPU
 * per reference rank); T (OpenMP threads) has no GPU meaning and is ignored.
 * KNN_MPI_COMPAT=1 makes the MPI mains print what the reference MPI
 * programs compute, bugs included (knn_search_mpi_compat).
 */
#ifndef KNN_CLI_H
#define KNN_CLI_H
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "knn.h"

#define NN 30   /* serial:8  */
#define MAXC 10 /* serial:9  */

typedef struct {
    double *X, *labels;
    size_t m, n, nl;
    knn_neighbour_t *nb;
    double seconds;
} cli_run_t;

static int cli_fail(const char *what, int rc)
{
    fprintf(stderr, "%s: %s\n", what, knn_strerror(rc));
    return 1;
}

/* load + search; returns 0 or a process exit code */
static int cli_search(cli_run_t *r, int ngpus, int compat)
{
    const char *path = getenv("KNN_MAT");
    if (!path || !*path) path = "mnist_train.mat";
    int rc = knn_load_mat(path, "train_X", "train_labels", &r->X, &r->m, &r->n, &r->labels, &r->nl);
    if (rc) return cli_fail(path, rc);
    if (r->nl != r->m) {
        fprintf(stderr, "%s: train_labels has %zu entries, train_X %zu rows\n", path, r->nl, r->m);
        return 1;
    }
    r->nb = (knn_neighbour_t *)malloc(r->m * NN * sizeof(knn_neighbour_t));
    if (!r->nb) return cli_fail("malloc", KNN_ERR_NOMEM);
    if (compat) {
        /* ngpus = the reference's procs; rows past procs*floor(m/procs) dropped */
        rc = knn_search_mpi_compat(r->X, r->m, r->n, KNN_COLMAJOR, r->labels, NN, ngpus, r->nb);
        if (rc) return cli_fail("knn_search_mpi_compat", rc);
        r->m = (r->m / (size_t)ngpus) * (size_t)ngpus;
    } else {
        rc = knn_search(r->X, r->m, r->n, KNN_COLMAJOR, r->labels, NN, ngpus, KNN_F64, r->nb);
        if (rc) return cli_fail("knn_search", rc);
    }
    r->seconds = knn_last_search_seconds();
    return 0;
}

static void cli_free(cli_run_t *r)
{
    knn_free(r->X);
    knn_free(r->labels);
    free(r->nb);
}

/* The MPI mains: per-rank block of rows [g*R, min(m,(g+1)*R)), R = ceil(m/P)
 * (the reference's floor(m/P) drops m mod P rows, blk:81), each printing its
 * own Matches with the MPI vote rule (blk:252-272). */
__attribute__((unused)) static int cli_mpi_main(int argc, char **argv, int nonblocking)
{
    if (argc < 3) {
        fprintf(stderr, "usage: %s <procs> <threads>\n", argv[0]);
        return 2;
    }
    int procs = atoi(argv[1]);
    if (procs < 1) procs = 1;
    cli_run_t r;
    memset(&r, 0, sizeof(r));
    const char *cenv = getenv("KNN_MPI_COMPAT");
    const int compat = cenv && cenv[0] == '1' && procs >= 2;
    int ec = cli_search(&r, procs, compat);
    if (ec) return ec;
    const size_t R = (r.m + procs - 1) / procs;   /* compat: r.m = procs*floor(m/procs) */
    int *pred = (int *)malloc(r.m * sizeof(int));
    size_t total = 0;
    int rc = pred ? knn_classify(r.nb, r.m, NN, MAXC, KNN_VOTE_MPI, r.labels, pred, &total)
                  : KNN_ERR_NOMEM;
    if (rc) { free(pred); cli_free(&r); return cli_fail("knn_classify", rc); }
    if (nonblocking) {
        for (int p = 0; p < procs - 1; p++)
            for (int g = 0; g < procs; g++)
                printf("%s\n", g == 0 ? "DONE" : (g == procs - 1 ? "done" : "DOne")); /* nb:208-226 */
    }
    for (int g = 0; g < procs; g++) {
        const size_t base = (size_t)g * R;
        if (base >= r.m) break;
        const size_t rows = base + R <= r.m ? R : r.m - base;
        size_t hit = 0;
        for (size_t i = base; i < base + rows; i++) hit += (pred[i] == r.labels[i]);
        printf(nonblocking ? "Matches%zu\n" : "Matches: %zu\n", hit); /* blk:272 / nb:290 */
    }
    free(pred);
    printf(nonblocking ? "Time :%f" : "KNN time: %f", r.seconds);  /* blk:273 / nb:292 */
    fflush(stdout);
    cli_free(&r);
    return 0;
}
#endif
