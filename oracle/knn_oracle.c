/*
 * knn_oracle.c -- CPU restatement of the reference all-kNN hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see knn_oracle.h): the parity checker for the
 * HIP engine and the "port" CPU baseline of bench.py.  Never linked into
 * libknn.  Build: oracle/Makefile (gcc -O2 -fopenmp -ffp-contract=off).
 *
 * Every function cites the reference lines it restates.
 */
#include "knn_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* serial:20-28 -- qsort comparator on distance only. */
static int orc_compare(const void *s1, const void *s2)
{
    double a = ((const orc_nb_t *)s1)->distance;
    double b = ((const orc_nb_t *)s2)->distance;
    if (a < b) return -1;
    else if (a == b) return 0;
    else return 1;
}

/* serial:76-85 -- S = S + pow(Da - Db, 2) sequentially over j.  pow(x,2)
 * compiles to a single mulsd at -O2, so the square is x*x
 * rounded once, then added: two roundings per feature, no FMA. */
static inline double orc_sqdist(const double *a, size_t sa,
                                const double *b, size_t sb, size_t n)
{
    double S = 0;
    for (size_t j = 0; j < n; j++) {
        double t = a[j * sa] - b[j * sb];
        double t2 = t * t;
        S = S + t2;
    }
    return S;
}

void orc_lists_init(orc_nb_t *lists, size_t nq, int k)
{
    /* serial:57-63 */
    for (size_t q = 0; q < nq * (size_t)k; q++) {
        lists[q].distance = INFINITY;
        lists[q].idx = 0;
        lists[q].label = 0;
    }
}

/* serial:86-91 restated: "overwrite slot NN-1, then stable sort" is the same
 * as inserting after every entry whose distance is <= d (glibc 2.35 qsort is
 * a stable merge sort at this size). */
static inline void orc_insert_stable(orc_nb_t *L, int k, double d, int32_t idx,
                                     int32_t label)
{
    int p = k - 1;
    while (p > 0 && L[p - 1].distance > d) {
        L[p] = L[p - 1];
        p--;
    }
    L[p].distance = d;
    L[p].idx = idx;
    L[p].label = label;
}

/* serial:86-91 verbatim semantics: overwrite the last slot and qsort. */
static inline void orc_insert_literal(orc_nb_t *L, int k, double d, int32_t idx,
                                      int32_t label)
{
    L[k - 1].distance = d;
    L[k - 1].idx = idx;
    L[k - 1].label = label;
    qsort(L, (size_t)k, sizeof(orc_nb_t), orc_compare);
}

/* Insertion ordered by (distance, idx): used where blocks may be visited out
 * of index order (the ring); equals orc_insert_stable for in-order scans. */
static inline void orc_insert_keyed(orc_nb_t *L, int k, double d, int32_t idx,
                                    int32_t label)
{
    int p = k - 1;
    while (p > 0 && (L[p - 1].distance > d ||
                     (L[p - 1].distance == d && L[p - 1].idx > idx))) {
        L[p] = L[p - 1];
        p--;
    }
    L[p].distance = d;
    L[p].idx = idx;
    L[p].label = label;
}

static inline int32_t orc_label_of(const double *labels, size_t row)
{
    return labels ? (int32_t)labels[row] : 0;
}

int orc_knn_rows(const double *X, size_t m, size_t n, int layout,
                 const double *labels, size_t q0, size_t nq, int k,
                 int literal, int nthreads, orc_nb_t *out)
{
    if (!X || !out || k <= 0 || q0 + nq > m) return 1;
    /* serial:82-83 reads column-major X[k + j*m]; the MPI variants pack
     * row-major rows (blk:100-109).  Either way S sums j = 0..n-1 in order,
     * so a row-major copy changes no rounding and keeps the loops cache
     * friendly. */
    const double *R = X;
    double *tmp = NULL;
    if (layout == ORC_COLMAJOR && n > 1) {
        tmp = (double *)malloc(m * n * sizeof(double));
        if (!tmp) return 2;
        for (size_t j = 0; j < n; j++)
            for (size_t i = 0; i < m; i++) tmp[i * n + j] = X[i + j * m];
        R = tmp;
    }
    orc_lists_init(out, nq, k);
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
    long long nqq = (long long)nq;
#pragma omp parallel for schedule(dynamic, 4)
    for (long long qq = 0; qq < nqq; qq++) {           /* serial:72 */
        size_t q = q0 + (size_t)qq;
        orc_nb_t *L = out + (size_t)qq * (size_t)k;
        const double *a = R + q * n;
        for (size_t i = 0; i < m; i++) {                /* serial:74 */
            double S = orc_sqdist(a, 1, R + i * n, 1, n);
            double d = sqrt(S);
            if ((d < L[k - 1].distance) && (d != 0)) {  /* serial:86 */
                if (literal)
                    orc_insert_literal(L, k, d, (int32_t)(i + 1),
                                       orc_label_of(labels, i));
                else
                    orc_insert_stable(L, k, d, (int32_t)(i + 1),
                                      orc_label_of(labels, i));
            }
        }
    }
    free(tmp);
    return 0;
}

/* orc_knn_rows on a row-major fp32 matrix: the same scan over the values
 * widened to double (exact), so it is orc_knn_rows of X.astype(float64)
 * without the 8-byte copy -- the checker of the fp32 path (KNN_F32: the
 * exact kNN of the fp32 points) at configs[4]'s 4M x 960, where that copy
 * would be 31 GB.  Queries: the rows listed in qidx (any order, one
 * thread each).  Stable insertion (serial:86-91). */
int orc_knn_rows_f32(const float *X, size_t m, size_t n, const int64_t *qidx, size_t nq, int k,
                     int nthreads, orc_nb_t *out)
{
    if (!X || !out || !qidx || k <= 0) return 1;
    for (size_t q = 0; q < nq; q++)
        if (qidx[q] < 0 || (size_t)qidx[q] >= m) return 1;
    orc_lists_init(out, nq, k);
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
    long long nqq = (long long)nq;
#pragma omp parallel
    {
        double *a = (double *)malloc(n * sizeof(double));
#pragma omp for schedule(dynamic, 1)
        for (long long qq = 0; qq < nqq; qq++) {        /* serial:72 */
            if (!a) continue;
            const size_t q = (size_t)qidx[qq];
            orc_nb_t *L = out + (size_t)qq * (size_t)k;
            for (size_t j = 0; j < n; j++) a[j] = (double)X[q * n + j];
            for (size_t i = 0; i < m; i++) {            /* serial:74 */
                const float *b = X + i * n;
                double S = 0;
                for (size_t j = 0; j < n; j++) {        /* serial:76-85 */
                    double t = a[j] - (double)b[j];
                    double t2 = t * t;
                    S = S + t2;
                }
                double d = sqrt(S);
                if ((d < L[k - 1].distance) && (d != 0)) /* serial:86 */
                    orc_insert_stable(L, k, d, (int32_t)(i + 1), 0);
            }
        }
        free(a);
    }
    return 0;
}

int orc_knn_block(const double *Q, size_t nq, size_t q_base,
                  const double *C, size_t nc, size_t c_base, size_t n,
                  const double *labels, int k, int nthreads, orc_nb_t *lists)
{
    if (!Q || !C || !lists || k <= 0) return 1;
    (void)q_base;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
    long long nqq = (long long)nq;
    /* blk:217-242: every local query against every row of the received
     * block; the candidate's id is its global 1-based row (blk:107,237). */
#pragma omp parallel for schedule(dynamic, 4)
    for (long long q = 0; q < nqq; q++) {
        orc_nb_t *L = lists + (size_t)q * (size_t)k;
        for (size_t i = 0; i < nc; i++) {
            double S = orc_sqdist(Q + (size_t)q * n, 1, C + i * n, 1, n);
            double d = sqrt(S);
            int32_t idx = (int32_t)(c_base + i + 1);
            if (d == 0) continue;
            if (d < L[k - 1].distance ||
                (d == L[k - 1].distance && idx < L[k - 1].idx))
                orc_insert_keyed(L, k, d, idx, orc_label_of(labels, c_base + i));
        }
    }
    return 0;
}

long orc_classify(const orc_nb_t *nb, size_t nq, size_t q0, int k, int nclasses,
                  int rule, const double *labels, int *pred)
{
    long matches = 0;
    int *cls = (int *)calloc((size_t)nclasses, sizeof(int));
    if (!cls) return -1;
    for (size_t q = 0; q < nq; q++) {                   /* serial:111 */
        const orc_nb_t *L = nb + q * (size_t)k;
        memset(cls, 0, (size_t)nclasses * sizeof(int)); /* serial:114 clear() */
        for (int i = 0; i < k; i++) {                   /* serial:116-119 */
            if (L[i].idx <= 0) continue;                /* empty slot (UB in ref) */
            int lab = (int)labels[L[i].idx - 1];
            if (lab >= 1 && lab <= nclasses) cls[lab - 1]++;
        }
        int most = 0;
        if (rule == ORC_VOTE_MAJORITY) {
            /* Not in the reference: a true majority whose ties go to the
             * tied label met first in neighbour order (SURVEY F7's 1742). */
            int best = 0;
            for (int j = 0; j < nclasses; j++)
                if (cls[j] > best) best = cls[j];
            for (int i = 0; i < k && best > 0; i++) {
                if (L[i].idx <= 0) continue;
                int lab = (int)labels[L[i].idx - 1];
                if (lab >= 1 && lab <= nclasses && cls[lab - 1] == best) {
                    most = lab;
                    break;
                }
            }
        } else {
            /* serial:121-124 / blk:263-266: `most` is compared as a count and
             * assigned a label.  Tie label: the nearest
             * neighbour's label (serial) or that label minus one (MPI). */
            int nn0 = (L[0].idx > 0) ? (int)labels[L[0].idx - 1] : 0;
            int tie = (rule == ORC_VOTE_MPI) ? nn0 - 1 : nn0;
            for (int j = 0; j < nclasses; j++)
                if (cls[j] > most || ((cls[j] == most) && ((j + 1) == tie)))
                    most = j + 1;
        }
        if (pred) pred[q] = most;
        if (most == labels[q0 + q]) matches++;          /* serial:126-127 */
    }
    free(cls);
    return matches;
}
