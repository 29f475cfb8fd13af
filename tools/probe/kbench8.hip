// kbench8 -- timing harness for k_dist_topk_i8 (not part of libknn).
// Builds the product kernel source and times product instantiations and
// template neighbours of them (staging depth NST, survivor buffer NB) with
// HIP events; the bounds array is reset to +inf before every launch, kept
// from the previous launch (converged), or taken as given (preset by the
// driver).  Driven by tools/probe/kbench8.py (data from the real engine).
// KB8_SRC: the kernel source (the product file, or an ablated copy made by
// tools/probe/ablate.py)
#ifndef KB8_SRC
#define KB8_SRC "../../mpi-knn_amd/csrc/knn_i8.hip"
#endif
#include KB8_SRC
#include <string.h>

#ifdef KB8_COUNT
// event counters of the "count" ablation (tools/probe/ablate.py): read
// into h[8], then zeroed
extern "C" int kb8_counts(unsigned long long *h)
{
    static const unsigned long long z[8] = {0};
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(kb8_cnt), sizeof(z)) != hipSuccess) return -1;
    return hipMemcpyToSymbol(HIP_SYMBOL(kb8_cnt), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif

#ifdef KB8_STAMP
// the stamp ablation's per-workgroup clocks: 4 words a workgroup
extern "C" int kb8_stamps(unsigned long long *h, int nwg)
{
    return hipMemcpyFromSymbol(h, HIP_SYMBOL(kb8_stamp), sizeof(unsigned long long) * 4 * nwg) == hipSuccess ? 0 : -1;
}
#endif

__global__ void kb8_fill_inf(double *p, int n)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = __builtin_inf();
}

// variant v: (NST, NB) = {0: (7, 8), 1: (8, 3), 2: (8, 4),
// 3: (7, 6), 4: (7, 4), 5: (8, 5) the 8-wave kernel, 6: the half-tile kernel} at the data's K-step bucket (sift 4,
// mnist 25)
template <int NKS, int NST, int NB>
static void kb8_go(dim3 grid, const void *qsh, size_t q_rows_pad, int nq, const void *csh, size_t c_rows_pad,
                   int nc, int rs, int nks, int ntiles, int nsplit, int nqb, double *part_d, int *part_i,
                   double *part_T, int nq_pad, double *qthr, int uj)
{
    knn_i8_blocks_t cb;   // one block: the whole corpus
    memset(&cb, 0, sizeof(cb));
    cb.nblk = 1;
    for (int b = 0; b < KNN_I8_MAXBLK; b++) {
        cb.ptr[b] = csh;
        cb.nptr[b] = (const char *)csh + c_rows_pad * (size_t)rs;
        cb.nc[b] = nc;
        cb.t0[b + 1] = ntiles;
    }
    cb.t0[0] = 0;
    hipLaunchKernelGGL(HIP_KERNEL_NAME(k_dist_topk_i8<KNN_I8_KL_S, NKS, 8, 2, NST, NB, 4>), grid, dim3(512), 0, 0,
                       (const signed char *)qsh, q_rows_pad, (size_t)0, nq, cb, c_rows_pad, rs, nks, ntiles,
                       nsplit, nqb, part_d, part_i, part_T, nq_pad, (unsigned long long *)qthr, uj,
                       (unsigned long long *)nullptr);
}

// the half-tile product kernel (4 waves, 64-row tiles, two workgroups a CU)
template <int NKS>
static void kb8_half(dim3 grid, const void *qsh, size_t q_rows_pad, int nq, const void *csh, size_t c_rows_pad,
                     int nc, int rs, int nks, int ntiles, int nsplit, int nqb, double *part_d, int *part_i,
                     double *part_T, int nq_pad, double *qthr, int uj)
{
    knn_i8_blocks_t cb;
    memset(&cb, 0, sizeof(cb));
    cb.nblk = 1;
    for (int b = 0; b < KNN_I8_MAXBLK; b++) {
        cb.ptr[b] = csh;
        cb.nptr[b] = (const char *)csh + c_rows_pad * (size_t)rs;
        cb.nc[b] = nc;
        cb.t0[b + 1] = ntiles;
    }
    cb.t0[0] = 0;
    hipLaunchKernelGGL(HIP_KERNEL_NAME(k_dist_topk_i8<KNN_I8_KL_S, NKS, 4, 2, 8, 5, 2>), grid, dim3(256), 0, 0,
                       (const signed char *)qsh, q_rows_pad, (size_t)0, nq, cb, c_rows_pad, rs, nks, ntiles,
                       nsplit, nqb, part_d, part_i, part_T, nq_pad, (unsigned long long *)qthr, uj,
                       (unsigned long long *)nullptr);
}

// average kernel ms over iters launches (after one warm-up); reset: 1 bounds
// to +inf before every launch, 0 only before the warm-up, 2 never
extern "C" float kbench8(int variant, const void *qsh, size_t q_rows_pad, int nq, const void *csh,
                         size_t c_rows_pad, int nc, int n, int k, int nsplit, double *part_d,
                         int *part_i, double *part_T, int nq_pad, double *qthr, int iters, int reset)
{
    const int rs = (int)knn_s8_rs((size_t)n), nks = rs / 32;
    const int nqb = (nq + 127) / 128, ntiles = (nc + 127) / 128;
    int uj = (k + 2) / 2 - 1, uj4 = (k + 4) / 4 - 1;   // as knn_launch_dist_i8
    const int no2 = uj > KNN_I8_KL_S - 1;   // as knn_launch_dist_i8
    if (uj > KNN_I8_KL_S - 1) uj = KNN_I8_KL_S - 1;
    uj |= uj4 << 8;
    if (no2) uj |= 1 << 16;
    if (nks > 25) return -1.f;
    const dim3 grid((unsigned)(nqb * nsplit));
    hipEvent_t e0, e1;
    if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) return -2.f;
    float total = 0.f;
    for (int it = 0; it <= iters; it++) {
        if (reset == 1 || (reset == 0 && it == 0))
            hipLaunchKernelGGL(kb8_fill_inf, dim3((nq_pad + 255) / 256), dim3(256), 0, 0, qthr, nq_pad);
        (void)hipEventRecord(e0, 0);
#define KB8(NKS, NST, NB) kb8_go<NKS, NST, NB>(grid, qsh, q_rows_pad, nq, csh, c_rows_pad, nc, rs, nks, ntiles, \
                                               nsplit, nqb, part_d, part_i, part_T, nq_pad, qthr, uj)
#define KB8V(NKS)                               \
    switch (variant) {                          \
    case 1: KB8(NKS, 8, 3); break;              \
    case 2: KB8(NKS, 8, 4); break;              \
    case 3: KB8(NKS, 7, 6); break;              \
    case 4: KB8(NKS, 7, 4); break;              \
    case 5: KB8(NKS, 8, 5); break;              \
    case 6:                                     \
        kb8_half<NKS>(grid, qsh, q_rows_pad, nq, csh, c_rows_pad, nc, rs, nks, ntiles, nsplit, nqb, part_d, \
                      part_i, part_T, nq_pad, qthr, uj);                                                 \
        break;                                  \
    default: KB8(NKS, 7, 8); break;             \
    }
        if (nks <= 4) {
            KB8V(4)
        } else {
            KB8V(25)
        }
#undef KB8V
#undef KB8
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (it) total += ms;
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return hipGetLastError() == hipSuccess ? total / iters : -2.f;
}
