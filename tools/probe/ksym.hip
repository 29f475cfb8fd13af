// ksym -- timing and coverage harness for the self-join's symmetric launch
// (not part of libknn).  Built by tools/probe/ablate.py sym
// from the product k_dist_topk_i8 with the sym patch; driven by
// tools/probe/ksym.py on real engine data (queries = corpus, one byte block).
//
//   S: every query against rows [0, 128 qa) -- the product kernel, one split
//      (its bounds seed the column filter)
//   prep: w(r) = min(floor(qthr[r]), dmax) - |r'|^2 into the block's init
//      words (zero and unread on long rows)
//   T: sy_mode 1 -- query blocks < qa against rows [128 qa, m), row direction
//      only; the others against the rows from their own on, and the column
//      direction on the tiles past their own block
//   scatter: the per-workgroup survivor regions into per-row buckets of cap
//      entries, key (d^2 << 32 | query)
#include KB8_SRC
#include <string.h>

__global__ void ksym_fill_inf(double *p, int n)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = __builtin_inf();
}

__global__ void ksym_prep(int *norms, size_t rows_pad, int m, int dmax, const unsigned long long *qthr)
{
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= m) return;
    const int pos = i8_norm_pos(r);
    const int nr = -(norms[pos] >> 5);
    const double b = __longlong_as_double((long long)qthr[r]);
    const int lim = b >= (double)dmax ? dmax : (int)b;
    norms[rows_pad + pos] = lim - nr;
}

__global__ void ksym_clear_iw(int *norms, size_t rows_pad, int m)
{
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r < m) norms[rows_pad + i8_norm_pos(r)] = 0;
}

__global__ void ksym_scatter(const uint4 *buf, const unsigned *wcnt, int wcap, unsigned *ccnt,
                             unsigned long long *cbuf, int cap)
{
    const int w = blockIdx.x;
    const int n = (int)min(wcnt[w], (unsigned)wcap);
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const uint4 e = buf[(size_t)w * wcap + i];
        if (e.y == 0u) continue;   // an exact duplicate (d^2 == 0)
        const unsigned sl = atomicAdd(ccnt + e.x, 1u);
        if ((int)sl < cap) cbuf[(size_t)e.x * cap + sl] = ((unsigned long long)e.y << 32) | e.z;
    }
}

template <int NKS>
static void ksym_launch(dim3 grid, const void *sh, size_t rows_pad, int nq, int nc, int rs, int nks, int ntiles,
                        int nsplit, int nqb, double *part_d, int *part_i, double *part_T, int nq_pad, double *qthr,
                        int uj, int mode, int qa, unsigned *wcnt, uint4 *buf, int wcap)
{
    knn_i8_blocks_t cb;
    memset(&cb, 0, sizeof(cb));
    cb.nblk = 1;
    for (int b = 0; b < KNN_I8_MAXBLK; b++) {
        cb.ptr[b] = sh;
        cb.nptr[b] = (const char *)sh + rows_pad * (size_t)rs;
        cb.nc[b] = nc;
        cb.t0[b + 1] = ntiles;
    }
    cb.t0[0] = 0;
    hipLaunchKernelGGL(HIP_KERNEL_NAME(k_dist_topk_i8<KNN_I8_KL_S, NKS, 4, 2, 8, 5, 2>), grid, dim3(256), 0, 0,
                       (const signed char *)sh, rows_pad, (size_t)0, nq, cb, rows_pad, rs, nks, ntiles, nsplit, nqb,
                       part_d, part_i, part_T, nq_pad, (unsigned long long *)qthr, uj, (unsigned long long *)nullptr,
                       mode, qa, wcnt, buf, wcap);
}

// ms[0..4] = S, prep, T, scatter, total (averages over iters after one
// warm-up); the buffers of the last iteration are left for the checker.
// qthr is reset to +inf before every iteration (a cold search).
extern "C" int ksym(const void *sh, size_t rows_pad, int m, int n, int k, int qa, int nsplit_s, int nsplit_t,
                    double *pd_s, int *pi_s, double *pT_s, double *pd_t, int *pi_t, double *pT_t, int nq_pad,
                    double *qthr, unsigned *wcnt, uint4 *wbuf, int wcap, unsigned *ccnt, unsigned long long *cbuf,
                    int cap, int iters, float *ms)
{
    const int rs = (int)knn_s8_rs((size_t)n), nks = rs / 32;
    if (nks <= 4 || nks > 25) return -1;   // long rows only (the init words carry w)
    const int nqb = (m + 127) / 128, ntiles = (m + 127) / 128;
    const int a_rows = 128 * qa < m ? 128 * qa : m;
    const int ntiles_a = (a_rows + 127) / 128;
    int uj = (k + 2) / 2 - 1, uj4 = (k + 4) / 4 - 1;
    const int no2 = uj > KNN_I8_KL_S - 1;
    if (uj > KNN_I8_KL_S - 1) uj = KNN_I8_KL_S - 1;
    uj |= uj4 << 8;
    if (no2) uj |= 1 << 16;
    const int dmax = rs * 65025 + 1;
    int *norms = (int *)((char *)sh + rows_pad * (size_t)rs);
    hipEvent_t ev[5];
    for (int i = 0; i < 5; i++)
        if (hipEventCreate(&ev[i]) != hipSuccess) return -2;
    for (int i = 0; i < 5; i++) ms[i] = 0.f;
    for (int it = 0; it <= iters; it++) {
        hipLaunchKernelGGL(ksym_fill_inf, dim3((nq_pad + 255) / 256), dim3(256), 0, 0, qthr, nq_pad);
        (void)hipMemsetAsync(ccnt, 0, sizeof(unsigned) * (size_t)m, 0);
        hipLaunchKernelGGL(ksym_clear_iw, dim3((m + 255) / 256), dim3(256), 0, 0, norms, rows_pad, m);
        (void)hipEventRecord(ev[0], 0);
        ksym_launch<25>(dim3((unsigned)(nqb * nsplit_s)), sh, rows_pad, m, a_rows, rs, nks, ntiles_a, nsplit_s, nqb,
                        pd_s, pi_s, pT_s, nq_pad, qthr, uj, 0, 0, wcnt, wbuf, wcap);
        (void)hipEventRecord(ev[1], 0);
        hipLaunchKernelGGL(ksym_prep, dim3((m + 255) / 256), dim3(256), 0, 0, norms, rows_pad, m, dmax,
                           (const unsigned long long *)qthr);
        (void)hipEventRecord(ev[2], 0);
        ksym_launch<25>(dim3((unsigned)(nqb * nsplit_t)), sh, rows_pad, m, m, rs, nks, ntiles, nsplit_t, nqb,
                        pd_t, pi_t, pT_t, nq_pad, qthr, uj, 1, qa, wcnt, wbuf, wcap);
        (void)hipEventRecord(ev[3], 0);
        hipLaunchKernelGGL(ksym_scatter, dim3((unsigned)(nqb * nsplit_t)), dim3(256), 0, 0, wbuf, wcnt, wcap, ccnt,
                           cbuf, cap);
        (void)hipEventRecord(ev[4], 0);
        if (hipEventSynchronize(ev[4]) != hipSuccess) return -3;
        if (it) {
            float t;
            for (int i = 0; i < 4; i++) {
                (void)hipEventElapsedTime(&t, ev[i], ev[i + 1]);
                ms[i] += t / iters;
            }
            (void)hipEventElapsedTime(&t, ev[0], ev[4]);
            ms[4] += t / iters;
        }
    }
    hipLaunchKernelGGL(ksym_clear_iw, dim3((m + 255) / 256), dim3(256), 0, 0, norms, rows_pad, m);
    (void)hipDeviceSynchronize();
    for (int i = 0; i < 5; i++) (void)hipEventDestroy(ev[i]);
    return hipGetLastError() == hipSuccess ? 0 : -4;
}
