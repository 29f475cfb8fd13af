/*
 * knn_vote.c -- knn_classify(): the label vote + accuracy stage.
 *
 * Rule SERIAL restates serial:104-130 and rule MPI blk:252-270 / nb:269-288,
 * including their quirk: `most` is compared as a vote count but
 * assigned a label, and ties go to the nearest neighbour's label (SERIAL) or
 * to that label minus one (MPI, blk:265).  Rule MAJORITY is a true
 * majority with ties to the tied label met first in neighbour order (not in
 * the reference).  Host code: m*k small integers, negligible next to the
 * search, and the reference excludes it from its timer (serial:94-98).
 */
#include "knn.h"
#include "knn_internal.h"

#include <hip/hip_runtime_api.h>
#include <stdlib.h>
#include <string.h>

int knn_classify(const knn_neighbour_t *nb, size_t m, int k, int nclasses, int vote_rule,
                 const double *labels, int *pred, size_t *matches)
{
    if (!nb || !labels || k <= 0 || nclasses <= 0 || nclasses > 65536) return KNN_ERR_INVALID;
    if (vote_rule != KNN_VOTE_SERIAL && vote_rule != KNN_VOTE_MPI &&
        vote_rule != KNN_VOTE_MAJORITY)
        return KNN_ERR_INVALID;
    int *cls = (int *)calloc((size_t)nclasses, sizeof(int));
    if (!cls) return KNN_ERR_NOMEM;
    size_t hit = 0;
    for (size_t q = 0; q < m; q++) {
        const knn_neighbour_t *L = nb + q * (size_t)k;
        memset(cls, 0, (size_t)nclasses * sizeof(int));          /* serial:114 */
        for (int i = 0; i < k; i++) {                             /* serial:116-119 */
            if (L[i].idx <= 0) continue;                             /* empty slot */
            const int lab = (int)labels[L[i].idx - 1];
            if (lab >= 1 && lab <= nclasses) cls[lab - 1]++;      /* F6: no class[-1] */
        }
        int most = 0;
        if (vote_rule == KNN_VOTE_MAJORITY) {
            int best = 0;
            for (int j = 0; j < nclasses; j++)
                if (cls[j] > best) best = cls[j];
            for (int i = 0; i < k && best > 0; i++) {
                if (L[i].idx <= 0) continue;
                const int lab = (int)labels[L[i].idx - 1];
                if (lab >= 1 && lab <= nclasses && cls[lab - 1] == best) {
                    most = lab;
                    break;
                }
            }
        } else {
            const int nn0 = L[0].idx > 0 ? (int)labels[L[0].idx - 1] : 0;
            const int tie = vote_rule == KNN_VOTE_MPI ? nn0 - 1 : nn0;  /* blk:265 vs serial:123 */
            for (int j = 0; j < nclasses; j++)                          /* serial:121-124 */
                if (cls[j] > most || ((cls[j] == most) && ((j + 1) == tie))) most = j + 1;
        }
        if (pred) pred[q] = most;
        if (most == labels[q]) hit++;                             /* serial:126-127 */
    }
    free(cls);
    if (matches) *matches = hit;
    return KNN_OK;
}

/* The same stage on device-resident records (k_vote in knn_kernels.hip):
 * one wave per query, no host round trip between search and vote. */
int knn_classify_device(knn_neighbour_t *d_nb, size_t m, int k, int nclasses, int vote_rule,
                        const double *d_labels, size_t nlabels, size_t q_base, int *d_pred,
                        unsigned long long *d_matches, void *stream)
{
    if (!d_nb || !d_labels || k <= 0 || nclasses <= 0) return KNN_ERR_INVALID;
    if (vote_rule != KNN_VOTE_SERIAL && vote_rule != KNN_VOTE_MPI &&
        vote_rule != KNN_VOTE_MAJORITY)
        return KNN_ERR_INVALID;
    if (nclasses > KNN_VOTE_MAX_CLASSES) return KNN_ERR_UNSUPPORTED;
    return knn_launch_vote(d_nb, m, k, nclasses, vote_rule, d_labels, nlabels, q_base, d_pred,
                           d_matches, stream);
}
