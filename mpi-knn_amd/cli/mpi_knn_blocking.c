/*
 * mpi-knn-parallel_blocking P T -- drop-in for mpi-knn-parallel_blocking.c
 * (blk:50-278): the block ring runs on P GPUs over RCCL (one GPU per
 * reference rank; T is ignored).  Prints each block's "Matches: %d" and
 * "KNN time: %f" like the reference (blk:272-273).
 */
#include "knn_cli.h"

int main(int argc, char **argv) { return cli_mpi_main(argc, argv, 0); }
