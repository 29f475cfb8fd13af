// Probe (diagnostic, not part of libknn): does the int8 MFMA shape change the
// rate the chip sustains under load?  MI355X_MICROARCH.md DVFS item 7 reports
// bf16 16x16x32 loops delivering ~1.12-1.15x the FLOP/s of 32x32x16 loops at
// equal cycles per FLOP (the 16x16 shape holds a higher clock).  This is the
// int8 kernel's inner loop in both shapes, at the same LDS bytes per MFMA op:
//   s32: a wave = 32 queries x 2 m-blocks of 32 rows; per 32-byte K-step 2
//        ds_read_b128 (A fragments) + 2 v_mfma_i32_32x32x32_i8, the queries'
//        B fragments resident (25 K-steps x 4 VGPRs) -- k_dist_topk_i8's loop;
//   s16: the same 32 queries x 64 rows as 2 query groups of 16 x 4 m-tiles of
//        16; per 64-byte K-step 4 ds_read_b128 + 8 v_mfma_i32_16x16x64_i8,
//        each A fragment used by both query groups (13 K-steps x 2 x 4 VGPRs).
// 256-thread workgroups, two a CU (80 KB of LDS each), random bytes; the
// in-kernel clock is stamped (s_memtime / s_memrealtime) into a buffer of its
// own.  Prints TOPS and the clock per shape and repetition.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
#define LDSB 81920

template <int SHAPE>
__global__ __launch_bounds__(256, 2) void loop(const v4i *__restrict__ src, int *__restrict__ out, int iters,
                                               unsigned long long *__restrict__ stamps)
{
    __shared__ __attribute__((aligned(16))) char smem[LDSB];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    // random bytes into LDS
    for (int i = threadIdx.x; i < LDSB / 16; i += 256) ((v4i *)smem)[i] = src[(blockIdx.x * 977 + i) & 65535];
    // queries (B fragments) resident
    constexpr int NQ = SHAPE == 32 ? 25 : 26;
    v4i q[NQ];
#pragma unroll
    for (int s = 0; s < NQ; s++) q[s] = src[(blockIdx.x * 131 + threadIdx.x * 7 + s * 4099) & 65535];
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    int sink = 0;
    if constexpr (SHAPE == 32) {
        v16i acc[2];
        for (int b = 0; b < 2; b++) acc[b] = (v16i){0};
        for (int it = 0; it < iters; it++) {
#pragma unroll
            for (int s = 0; s < 25; s++) {
                // 2 KiB of A a K-step, rotating through 32 KiB (the ring's stage size x 4)
                const int base = ((it * 25 + s) & 15) * 2048 + wave * 256;
                v4i a0 = *(const v4i *)(smem + ((base + lane * 16) & (LDSB - 1)));
                v4i a1 = *(const v4i *)(smem + ((base + 1024 + lane * 16) & (LDSB - 1)));
                acc[0] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a0, q[s], acc[0], 0, 0, 0);
                acc[1] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a1, q[s], acc[1], 0, 0, 0);
            }
        }
        for (int b = 0; b < 2; b++)
            for (int i = 0; i < 16; i++) sink ^= acc[b][i];
    } else {
        v4i acc[8];
        for (int b = 0; b < 8; b++) acc[b] = (v4i){0, 0, 0, 0};
        for (int it = 0; it < iters; it++) {
#pragma unroll
            for (int s = 0; s < 13; s++) {
                // 4 KiB of A a 64-byte K-step (the same bytes per op as s32)
                const int base = ((it * 13 + s) & 7) * 4096 + wave * 256;
                v4i a[4];
#pragma unroll
                for (int m = 0; m < 4; m++) a[m] = *(const v4i *)(smem + ((base + 1024 * m + lane * 16) & (LDSB - 1)));
#pragma unroll
                for (int m = 0; m < 4; m++) {
                    acc[m] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[m], q[2 * s], acc[m], 0, 0, 0);
                    acc[4 + m] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[m], q[2 * s + 1], acc[4 + m], 0, 0, 0);
                }
            }
        }
        for (int b = 0; b < 8; b++)
            for (int i = 0; i < 4; i++) sink ^= acc[b][i];
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * 256 + threadIdx.x] = sink;
    if (threadIdx.x == 0) {
        stamps[2 * blockIdx.x] = t1 - t0;
        stamps[2 * blockIdx.x + 1] = r1 - r0;
    }
}

int main(int argc, char **argv)
{
    const int nwg = 512;
    const int iters = argc > 1 ? atoi(argv[1]) : 2000;
    std::vector<v4i> h(65536);
    srand(12345);
    for (auto &x : h) x = (v4i){rand(), rand(), rand(), rand()};
    v4i *d;
    int *o;
    unsigned long long *st;
    CK(hipMalloc(&d, 65536 * 16));
    CK(hipMalloc(&o, nwg * 256 * 4));
    CK(hipMalloc(&st, nwg * 16));
    CK(hipMemcpy(d, h.data(), 65536 * 16, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<unsigned long long> hs(2 * nwg);
    // ops a launch: per wave per iteration 25 x 2 x 32x32x32 = 50 x 65536 (s32),
    // 13 x 8 x 16x16x64 = 104 x 32768 (s16: 4% more, the 64-byte K padding)
    for (int rep = 0; rep < 3; rep++) {
        for (int shape : {32, 16}) {
            float ms = 0;
            // warm the clock up: a few launches back to back, then time one
            for (int w = 0; w < 3; w++) {
                if (shape == 32) loop<32><<<nwg, 256>>>(d, o, iters, st);
                else loop<16><<<nwg, 256>>>(d, o, iters, st);
            }
            CK(hipEventRecord(e0));
            if (shape == 32) loop<32><<<nwg, 256>>>(d, o, iters, st);
            else loop<16><<<nwg, 256>>>(d, o, iters, st);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            CK(hipEventElapsedTime(&ms, e0, e1));
            CK(hipMemcpy(hs.data(), st, 16 * nwg, hipMemcpyDeviceToHost));
            std::vector<double> clk;
            for (int b = 0; b < nwg; b++) clk.push_back((double)hs[2 * b] / (double)hs[2 * b + 1] * 100.0);
            std::sort(clk.begin(), clk.end());
            const double ops = (double)nwg * 4 * iters * (shape == 32 ? 50.0 * 65536.0 : 104.0 * 32768.0);
            const double useful = (double)nwg * 4 * iters * 50.0 * 65536.0;   // the 800-byte rows' ops
            printf("{\"shape\": %d, \"rep\": %d, \"ms\": %.3f, \"tops_issued\": %.1f, \"tops_useful\": %.1f, "
                   "\"clock_mhz_median\": %.0f}\n",
                   shape, rep, ms, ops / ms / 1e9, useful / ms / 1e9, clk[nwg / 2]);
        }
    }
    return 0;
}
