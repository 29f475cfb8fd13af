// kbench32: tuning harness for the fp32 k_dist_topk on the SIFT shape
// (configs[3]: n = 128, k = 32 -> <float, 24, 64>), not part of libknn.
// Ablations as in kbench (ABL / EPI bits documented in knn_kernels.hip).
//   ./kbench32 [m]     (default 250000: ~1/16 of configs[3]'s pairs)
#include "../../mpi-knn_amd/csrc/knn_kernels.hip"
#include <cstdio>
#include <vector>
#include <cstdlib>
#define CK(x) do{hipError_t e_=(x); if(e_!=hipSuccess){printf("HIP %s @%d\n",hipGetErrorString(e_),__LINE__); exit(1);}}while(0)

__device__ unsigned hsh(unsigned a) { a ^= a >> 16; a *= 0x7feb352du; a ^= a >> 15; a *= 0x846ca68bu; a ^= a >> 16; return a; }

// SIFT-like: 1024 cluster centres in [0,160), noise ~ N(0, 25) (sum of 4
// uniforms), rounded and clipped to [0, 255]
__global__ void fill_sift(float* X, int m, int n)
{
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= (size_t)m * n) return;
    const unsigned row = (unsigned)(i / n), col = (unsigned)(i % n);
    const unsigned c = hsh(row * 2654435761u + 17u) % 1024u;
    const float centre = (float)(hsh(c * 131u + col * 7919u) % 160u);
    float u = 0.f;
    for (int t = 0; t < 4; t++) u += (float)(hsh((unsigned)i * 4u + t + 99u) & 0xffff) / 65536.f - 0.5f;
    float v = rintf(centre + u * 43.3f);
    X[i] = fminf(fmaxf(v, 0.f), 255.f);
}

constexpr int KL = KNN_KL_M, KP = KNN_KP_M;

template <int EPI, int ABL = 0>
float run(const float* blk, size_t rp, int m, int n, double* pd, int* pi, double* pT, int nq_pad, int reps,
          double* qthr)
{
    const int np = (int)knn_n_pad_dt(n, KNN_F32);
    const int nqb = (m + KNN_TQ - 1) / KNN_TQ, ntiles = (m + KNN_TC - 1) / KNN_TC;
    const float* norms = blk + rp * np;
    const double* meta = (const double*)(norms + rp);
    const int uj = 8 | (15 << 8);
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    float best = 1e30f;
    for (int r = 0; r <= reps; r++) {
        knn_launch_fill_inf(qthr, nq_pad, 0);
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(HIP_KERNEL_NAME(k_dist_topk<float, KL, KP, EPI, ABL>), dim3(nqb), dim3(512), 0, 0,
                           blk, norms, (size_t)0, m, blk, norms, (size_t)0, m, n, np, ntiles, 1, nqb, meta, pd, pi, pT,
                           nq_pad, (unsigned long long*)qthr, uj, 0);
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        if (r > 0 && ms < best) best = ms;
    }
    return best;
}

int main(int argc, char** argv)
{
    const int m = argc > 1 ? atoi(argv[1]) : 250000, n = 128;
    const size_t rp = knn_rows_pad(m), np = knn_n_pad_dt(n, KNN_F32);
    float* src; CK(hipMalloc(&src, (size_t)m * n * 4));
    void* blk; CK(hipMalloc(&blk, (rp * np + rp) * 4 + 64));
    fill_sift<<<(unsigned)(((size_t)m * n + 255) / 256), 256>>>(src, m, n);
    if (knn_launch_pack(blk, KNN_F32, m, m, n, src, KNN_F32, n, KNN_ROWMAJOR, 0)) { printf("pack failed\n"); return 1; }
    const int nq_pad = (int)knn_round_up(m, KNN_TQ);
    double *pd, *pT, *qthr; int* pi;
    CK(hipMalloc(&pd, (size_t)nq_pad * 4 * KL * 8)); CK(hipMalloc(&pi, (size_t)nq_pad * 4 * KL * 4));
    CK(hipMalloc(&pT, (size_t)nq_pad * 8)); CK(hipMalloc(&qthr, (size_t)nq_pad * 8));
    const float* b = (const float*)blk;
    const double flop = 2.0 * m * (double)m * n;
    auto pr = [&](const char* name, float ms) { printf("  %-34s %8.2f ms  %6.1f TF  %5.1f%% of 157.3\n", name, ms, flop / ms / 1e9, flop / ms / 1e9 / 1.573); };
    printf("k_dist_topk<float,%d,%d> m=%d n=%d (SIFT-like), best of 2\n", KL, KP, m, n);
    pr("full", run<1>(b, rp, m, n, pd, pi, pT, nq_pad, 2, qthr));
    pr("setprio waves 4-7 (ABL 16)", run<1, 16>(b, rp, m, n, pd, pi, pT, nq_pad, 2, qthr));
    pr("no epilogue insertion (EPI 0)", run<0>(b, rp, m, n, pd, pi, pT, nq_pad, 2, qthr));
    pr("no staging loads (ABL 1)", run<1, 1>(b, rp, m, n, pd, pi, pT, nq_pad, 2, qthr));
    pr("no chunk barrier (ABL 2)", run<1, 2>(b, rp, m, n, pd, pi, pT, nq_pad, 2, qthr));
    pr("EPI 0 + no loads", run<0, 1>(b, rp, m, n, pd, pi, pT, nq_pad, 2, qthr));
    pr("EPI 0 + no loads + no barrier", run<0, 3>(b, rp, m, n, pd, pi, pT, nq_pad, 2, qthr));
    pr("pairs order swapped (ABL 32)", run<1, 32>(b, rp, m, n, pd, pi, pT, nq_pad, 2, qthr));
    {
        unsigned long long z[256] = {0};
        CK(hipMemcpyToSymbol(HIP_SYMBOL(knn_dbg_rounds), z, sizeof z));
        run<3>(b, rp, m, n, pd, pi, pT, nq_pad, 0, qthr);
        CK(hipMemcpyFromSymbol(z, HIP_SYMBOL(knn_dbg_rounds), sizeof z));
        const int nqb = (m + KNN_TQ - 1) / KNN_TQ;
        double tot = 0;
        printf("  insertion rounds per wave by tile position:");
        for (int i = 0; i < 256; i++) { double r = z[i] / (double)nqb; tot += r; if (i < 6 || i % 50 == 0 || i == 255) printf(" [%d]%.2f", i, r); }
        printf("  total(first 255 + tail bucket) %.1f\n", tot);
    }
    return 0;
}
