/*
 * mpi-knn-parallel_non_blocking P T -- drop-in for
 * mpi-knn-parallel_non_blocking.c (nb:59-297).  Same engine as the blocking
 * variant (the RCCL ring always overlaps the next hop with compute); keeps
 * this program's stdout: per-hop DONE/done/DOne (nb:208-226),
 * "Matches%d" (nb:290) and "Time :%f" (nb:292).
 */
#include "knn_cli.h"

int main(int argc, char **argv) { return cli_mpi_main(argc, argv, 1); }
