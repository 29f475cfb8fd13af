// kbench16: ablations of the fp16-shadow k_dist_topk (H16 = 2, the mnist
// default) on a 60000x784 integer corpus, timed with HIP events.  Tuning
// harness only (not part of libknn); variants with ABL bits give wrong
// results by design (see the ABL comment in knn_kernels.hip).
#include "../../mpi-knn_amd/csrc/knn_kernels.hip"
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#define CK(x) do{hipError_t e_=(x); if(e_!=hipSuccess){printf("HIP %s @%d\n",hipGetErrorString(e_),__LINE__); exit(1);}}while(0)

__global__ void fill_int(double* X, size_t cnt, unsigned seed)
{
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i < cnt) {
        unsigned h = (unsigned)(i * 2654435761u) ^ seed; h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
        X[i] = (double)(h % 256u);
    }
}

struct Args { const double *sh, *norms, *meta; int m, n, nps, nsplit, nq_pad; double *pd, *pT, *qthr; int *pi; };

template <int EPI, int ABL>
float run(const Args& a, int reps)
{
    const int nqb = (a.m + KNN_TQ - 1) / KNN_TQ, ntiles = (a.m + KNN_TC - 1) / KNN_TC;
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    float tot = 0;
    for (int r = 0; r <= reps; r++) {
        if (a.qthr) knn_launch_fill_inf(a.qthr, a.nq_pad, 0);
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(HIP_KERNEL_NAME(k_dist_topk<double, KNN_KL, KNN_KP, EPI, ABL, 2>),
                           dim3(nqb * a.nsplit), dim3(512), 0, 0, a.sh, a.norms, (size_t)0, a.m, a.sh,
                           a.norms, (size_t)0, a.m, a.n, a.nps, ntiles, a.nsplit, nqb, a.meta, a.pd, a.pi,
                           a.pT, a.nq_pad, (unsigned long long*)a.qthr, 7 | (7 << 8), 0);
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        if (r) tot += ms;   // first launch is warmup
    }
    return tot / reps;
}

int main(int argc, char** argv)
{
    int m = argc > 1 ? atoi(argv[1]) : 60000, n = 784, s = argc > 2 ? atoi(argv[2]) : 6;
    size_t rp = knn_rows_pad(m), np = knn_n_pad(n), nps = knn_round_up(n, 64);
    double *src, *blk; CK(hipMalloc(&src, (size_t)m * n * 8)); CK(hipMalloc(&blk, (rp * np + rp + 8) * 8));
    fill_int<<<(unsigned)(((size_t)m * n + 255) / 256), 256>>>(src, (size_t)m * n, 1234u);
    if (knn_launch_pack(blk, KNN_F64, m, m, n, src, KNN_F64, m, KNN_COLMAJOR, 0)) { printf("pack failed\n"); return 1; }
    void* sh; CK(hipMalloc(&sh, rp * nps * 2 + 4096));
    if (knn_launch_shadow(sh, blk, KNN_F64, rp, n, 0)) { printf("shadow failed\n"); return 1; }
    Args a;
    a.sh = (const double*)sh; a.norms = blk + rp * np; a.meta = a.norms + rp;
    a.m = m; a.n = n; a.nps = (int)nps; a.nsplit = s; a.nq_pad = (int)knn_round_up(m, KNN_TQ);
    CK(hipMalloc(&a.pd, (size_t)s * a.nq_pad * 4 * KNN_KL * 8)); CK(hipMalloc(&a.pi, (size_t)s * a.nq_pad * 4 * KNN_KL * 4));
    CK(hipMalloc(&a.pT, (size_t)s * a.nq_pad * 8)); CK(hipMalloc(&a.qthr, (size_t)a.nq_pad * 8));
    const double flop = 2.0 * m * (double)m * n;
    // scheduling-only variants must leave the partial lists unchanged
    // (checked without the shared bound, whose timing makes lists vary)
    const size_t pn = (size_t)s * a.nq_pad * 4 * KNN_KL;
    std::vector<double> h0(pn), h1(pn);
    Args b = a; b.qthr = nullptr;
    run<1, 0>(b, 1); CK(hipMemcpy(h0.data(), a.pd, pn * 8, hipMemcpyDeviceToHost));
auto same = [&](float) { CK(hipMemcpy(h1.data(), a.pd, pn * 8, hipMemcpyDeviceToHost));
                             return memcmp(h0.data(), h1.data(), pn * 8) == 0 ? "same" : "DIFF"; };
#define SAME(ABLV) same(run<1, ABLV>(b, 1))
    float full = run<1, 0>(a, 5);
    printf("full        %.3f ms  %.1f TF\n", full, flop / full / 1e9);
    printf("noEPI       %.3f ms\n", run<0, 0>(a, 5));
    printf("prio47      %.3f ms  %s\n", run<1, 16>(a, 5), SAME(16));
    printf("seg-load    %.3f ms  %s\n", run<1, 2048>(a, 5), SAME(2048));
    printf("loaders03   %.3f ms  %s\n", run<1, 8192>(a, 5), SAME(8192));
    printf("L03+prio    %.3f ms  %s\n", run<1, 8192 | 16>(a, 5), SAME(8192 | 16));
    printf("L03+seg     %.3f ms  %s\n", run<1, 8192 | 2048>(a, 5), SAME(8192 | 2048));
    printf("prio+seg    %.3f ms  %s\n", run<1, 16 | 2048>(a, 5), SAME(16 | 2048));
    printf("all3        %.3f ms  %s\n", run<1, 8192 | 16 | 2048>(a, 5), SAME(8192 | 16 | 2048));
    printf("full again  %.3f ms\n", run<1, 0>(a, 5));
    return 0;
}
