// kbench8 -- tuning harness for k_dist_topk_i8 (not part of libknn).
// Builds the product kernel source with ablation variants (the ABL template
// argument; libknn instantiates ABL = 0 only) and times each launch with HIP
// events, qthr reset to +inf before every launch so each run filters alike.
// Driven by tools/probe/kbench8.py (data from the real engine).
#include "../../mpi-knn_amd/csrc/knn_i8.hip"

__global__ void kb8_fill_inf(double *p, int n)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = __builtin_inf();
}

template <int ABL>
static void kb8_launch(dim3 grid, hipStream_t s, const void *qsh, size_t q_rows_pad, int nq, const void *csh,
                       size_t c_rows_pad, int nc, int rs, int nks, int ntiles, int nsplit, int nqb,
                       double *part_d, int *part_i, double *part_T, int nq_pad, double *qthr, int uj, int nch)
{
    // the product's k <= 32 variants: sift (4 K-steps), mnist (25)
    if (nch == 1)
        hipLaunchKernelGGL(HIP_KERNEL_NAME(k_dist_topk_i8<KNN_I8_KL, 4, 8, 2, 7, 8, ABL>), grid, dim3(512), 0, s,
                           (const signed char *)qsh, q_rows_pad, (size_t)0, nq, (const signed char *)csh,
                           c_rows_pad, (size_t)0, nc, rs, nks, ntiles, nsplit, nqb, part_d, part_i, part_T,
                           nq_pad, (unsigned long long *)qthr, uj);
    else
        hipLaunchKernelGGL(HIP_KERNEL_NAME(k_dist_topk_i8<KNN_I8_KL, 25, 8, 2, 7, 8, ABL>), grid, dim3(512), 0, s,
                           (const signed char *)qsh, q_rows_pad, (size_t)0, nq, (const signed char *)csh,
                           c_rows_pad, (size_t)0, nc, rs, nks, ntiles, nsplit, nqb, part_d, part_i, part_T,
                           nq_pad, (unsigned long long *)qthr, uj);
}

// ABL 32 counters of the last launch: wave-tiles with survivors, insertion rounds
extern "C" void kbench8_counters(unsigned long long *out)
{
    hipMemcpyFromSymbol(out, HIP_SYMBOL(i8_dbg), sizeof(i8_dbg), 0, hipMemcpyDeviceToHost);
}
extern "C" void kbench8_reset()
{
    unsigned long long z[4] = {0, 0, 0, 0};
    hipMemcpyToSymbol(HIP_SYMBOL(i8_dbg), z, sizeof(z), 0, hipMemcpyHostToDevice);
}

// returns the average kernel ms over iters launches (after one warm-up)
extern "C" float kbench8(int abl, const void *qsh, size_t q_rows_pad, int nq, const void *csh,
                         size_t c_rows_pad, int nc, int n, int k, int nsplit, double *part_d,
                         int *part_i, double *part_T, int nq_pad, double *qthr, int iters, int reset)
{
    const int rs = (int)knn_s8_rs((size_t)n), nks = rs / 32, nch = (nks + 3) / 4;
    const int nqb = (nq + 127) / 128, ntiles = (nc + 127) / 128;
    int uj = (k + 2) / 2 - 1, uj4 = (k + 4) / 4 - 1;   // as knn_launch_dist_i8
    if (uj > KNN_I8_KL - 1) uj = KNN_I8_KL - 1;
    uj |= uj4 << 8;
    const dim3 grid((unsigned)(nqb * nsplit));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    float total = 0.f;
    for (int it = 0; it <= iters; it++) {
        if (reset == 1 || (reset == 0 && it == 0)) hipLaunchKernelGGL(kb8_fill_inf, dim3((nq_pad + 255) / 256), dim3(256), 0, 0, qthr, nq_pad);
        hipEventRecord(e0, 0);
#define KB(A) case A: kb8_launch<A>(grid, 0, qsh, q_rows_pad, nq, csh, c_rows_pad, nc, rs, nks, ntiles, nsplit, nqb, part_d, part_i, part_T, nq_pad, qthr, uj, nch); break;
        switch (abl) {
            KB(0) KB(1) KB(2) KB(4) KB(8) KB(16) KB(5) KB(32)
        default: return -1.f;
        }
#undef KB
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        float ms = 0.f;
        hipEventElapsedTime(&ms, e0, e1);
        if (it) total += ms;
    }
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    return hipGetLastError() == hipSuccess ? total / iters : -2.f;
}
