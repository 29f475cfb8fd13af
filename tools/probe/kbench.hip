// kbench: tuning harness for k_dist_topk (not part of libknn).
//  1. sustained fp64 MFMA rate (long loop) and the clock it holds;
//  2. k_dist_topk variants (ABL/EPI ablations, see knn_kernels.hip) on a 60000x784
//     integer corpus, timed with HIP events.
#include "../../mpi-knn_amd/csrc/knn_kernels.hip"
#include <cstdio>
#include <vector>
#include <cstdlib>
#include <cstring>
#define CK(x) do{hipError_t e_=(x); if(e_!=hipSuccess){printf("HIP %s @%d\n",hipGetErrorString(e_),__LINE__); exit(1);}}while(0)

__global__ void mfma_sustain(double* out, long long* clk, int iters, double x)
{
    dbl4 acc[4];
    for (int i = 0; i < 4; i++) acc[i] = (dbl4){0, 0, 0, 0};
    double a = x + threadIdx.x * 0.37, b = x - threadIdx.x * 0.11;
    long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int i = 0; i < 4; i++) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
    }
    long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    double s = 0; for (int i = 0; i < 4; i++) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) { clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = r1 - r0; }
}

__global__ void fill_int(double* X, size_t cnt, unsigned seed)
{
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i < cnt) {
        unsigned h = (unsigned)(i * 2654435761u) ^ seed; h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
        X[i] = (double)(h % 256u);
    }
}

template <int EPI, int ABL = 0>
float run(const double* blk, size_t rp, int m, int n, int nsplit, double* pd, int* pi, double* pT, int nq_pad, int reps,
          double* qthr = nullptr)
{
    const int np = (int)knn_n_pad(n);
    const int nqb = (m + KNN_TQ - 1) / KNN_TQ, ntiles = (m + KNN_TC - 1) / KNN_TC;
    const double* norms = blk + rp * np;
    const double* meta = norms + rp;
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    if (qthr) knn_launch_fill_inf(qthr, nq_pad, 0);
    hipLaunchKernelGGL(HIP_KERNEL_NAME(k_dist_topk<double, KNN_KL, KNN_KP, EPI, ABL>), dim3(nqb * nsplit), dim3(512), 0, 0,
                       blk, norms, (size_t)0, m, blk, norms, (size_t)0, m, n, np, ntiles, nsplit, nqb, meta, pd, pi, pT, nq_pad,
                           (unsigned long long*)qthr, 7 | (7 << 8), 0);
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; r++) {
        if (qthr) knn_launch_fill_inf(qthr, nq_pad, 0);
        hipLaunchKernelGGL(HIP_KERNEL_NAME(k_dist_topk<double, KNN_KL, KNN_KP, EPI, ABL>), dim3(nqb * nsplit), dim3(512), 0, 0,
                           blk, norms, (size_t)0, m, blk, norms, (size_t)0, m, n, np, ntiles, nsplit, nqb, meta, pd, pi, pT, nq_pad,
                           (unsigned long long*)qthr, 7 | (7 << 8), 0);
    }
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / reps;
}

int main(int argc, char** argv)
{
    // 1. sustained MFMA
    {
        int nb = 256 * 2, nt = 256, iters = 200000;
        double* o; long long* clk; CK(hipMalloc(&o, (size_t)nb * nt * 8)); CK(hipMalloc(&clk, nb * 16));
        hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
        mfma_sustain<<<nb, nt>>>(o, clk, 1000, 1.0);
        CK(hipEventRecord(e0)); mfma_sustain<<<nb, nt>>>(o, clk, iters, 1.0); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        std::vector<long long> h(nb * 2); CK(hipMemcpy(h.data(), clk, nb * 16, hipMemcpyDeviceToHost));
        double f = 0; for (int b = 0; b < nb; b++) f += (double)h[2 * b] / h[2 * b + 1] * 100.0; f /= nb;
        double fl = (double)nb * (nt / 64) * iters * 4 * 2048.0;
        printf("sustained mfma_f64: %.1f ms  %.2f TFLOP/s  in-kernel clock %.0f MHz\n", ms, fl / ms / 1e9, f);
    }
    int m = argc > 1 ? atoi(argv[1]) : 60000, n = 784;
    size_t rp = knn_rows_pad(m), np = knn_n_pad(n);
    double *src, *blk; CK(hipMalloc(&src, (size_t)m * n * 8)); CK(hipMalloc(&blk, (rp * np + rp + 8) * 8));
    fill_int<<<(unsigned)(((size_t)m * n + 255) / 256), 256>>>(src, (size_t)m * n, 1234u);
    if (knn_launch_pack(blk, KNN_F64, m, m, n, src, KNN_F64, m, KNN_COLMAJOR, 0)) { printf("pack failed\n"); return 1; }
    int nq_pad = (int)knn_round_up(m, KNN_TQ);
    double *pd, *pT; int* pi;
    CK(hipMalloc(&pd, (size_t)15 * nq_pad * 4 * KNN_KL * 8)); CK(hipMalloc(&pi, (size_t)15 * nq_pad * 4 * KNN_KL * 4));
    CK(hipMalloc(&pT, (size_t)15 * nq_pad * 8));
    const double flop = 2.0 * m * (double)m * n;
    double* qthr; CK(hipMalloc(&qthr, (size_t)nq_pad * 8));
    for (int rep = 0; rep < 2; rep++) {
        const int s = 6;
        const size_t pn = (size_t)s * nq_pad * 4 * KNN_KL;
        std::vector<double> h1(pn), h2(pn);
        run<1>(blk, rp, m, n, s, pd, pi, pT, nq_pad, 1);
        CK(hipMemcpy(h1.data(), pd, pn * 8, hipMemcpyDeviceToHost));
        run<1, 8192>(blk, rp, m, n, s, pd, pi, pT, nq_pad, 1);
        CK(hipMemcpy(h2.data(), pd, pn * 8, hipMemcpyDeviceToHost));
        const bool ok1 = !memcmp(h1.data(), h2.data(), pn * 8);
        float pq = run<1>(blk, rp, m, n, s, pd, pi, pT, nq_pad, 3, qthr);
        float l1 = run<1, 8192>(blk, rp, m, n, s, pd, pi, pT, nq_pad, 3, qthr);
        float p2n = run<0>(blk, rp, m, n, s, pd, pi, pT, nq_pad, 3, qthr);
        float l1n = run<0, 8192>(blk, rp, m, n, s, pd, pi, pT, nq_pad, 3, qthr);
        float a1 = run<0, 1>(blk, rp, m, n, s, pd, pi, pT, nq_pad, 3, qthr);
        printf("full %.2f ms (%.1f TF) | loaders-0-3 %.2f ms (%.1f TF, lists %s) | noEPI %.2f  noEPI+loaders-0-3 %.2f  no-glds %.2f\n",
               pq, flop / pq / 1e9, l1, flop / l1 / 1e9, ok1 ? "same" : "DIFF", p2n, l1n, a1);
    }
    for (int v = 0; v < 2; v++) {
        unsigned long long z[256] = {0};
        CK(hipMemcpyToSymbol(HIP_SYMBOL(knn_dbg_rounds), z, sizeof z));
        run<3>(blk, rp, m, n, 6, pd, pi, pT, nq_pad, 1, v ? qthr : nullptr);   // 2 launches counted
        CK(hipMemcpyFromSymbol(z, HIP_SYMBOL(knn_dbg_rounds), sizeof z));
        const int nqb = (m + KNN_TQ - 1) / KNN_TQ;
        double tot = 0;
        printf("%s: insertion rounds per wave by tile position:", v ? "shared-bound" : "own-bound");
        for (int i = 0; i < 80; i++) { double r = z[i] / 2.0 / (nqb * 6.0); tot += r; if (i < 8 || i % 10 == 0) printf(" [%d]%.2f", i, r); }
        printf("  total %.1f\n", tot);
    }
    return 0;
}
