/*
 * knn-serial -- drop-in for knn-serial.c (serial:36-133): load
 * mnist_train.mat, all-kNN (k = 30) on one MI355X, serial vote, and the
 * reference's three stdout lines.
 */
#include "knn_cli.h"

int main(int argc, char *argv[])
{
    (void)argc;
    (void)argv;
    cli_run_t r;
    memset(&r, 0, sizeof(r));
    printf("Number of Classes: %d\n", MAXC);                          /* serial:65 */
    int ec = cli_search(&r, 1, 0);
    if (ec) return ec;
    printf("Sorting done\nClock time = %f\n", r.seconds);             /* serial:98 */
    size_t matches = 0;
    int rc = knn_classify(r.nb, r.m, NN, MAXC, KNN_VOTE_SERIAL, r.labels, NULL, &matches);
    if (rc) { cli_free(&r); return cli_fail("knn_classify", rc); }
    printf("Matches: %zu\n", matches);                                 /* serial:130 */
    cli_free(&r);
    return 0;
}
