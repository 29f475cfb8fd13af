// knn_device.h -- device helpers shared by the kernel translation units
// (knn_kernels.hip: element / fp16 contraction; knn_i8.hip: int8 contraction).
#ifndef KNN_DEVICE_H
#define KNN_DEVICE_H
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "knn_internal.h"

typedef double dbl4 __attribute__((ext_vector_type(4)));
typedef double dbl2 __attribute__((ext_vector_type(2)));
typedef float flt4 __attribute__((ext_vector_type(4)));
#define LDS_AS __attribute__((address_space(3)))

static constexpr double KNN_INF = __builtin_inf();

// LDS-DMA issue as inline asm (guide: glds16_asm).  Written through
// __builtin_amdgcn_global_load_lds, the loads make hipcc's waitcnt pass treat
// every later LDS read as racing a pending FLAT access and emit lgkmcnt(0)
// ahead of each segment's first MFMA; hidden from it, their completion is
// counted by the kernel's own `s_waitcnt vmcnt(N)`.  M0 (the wave-uniform
// LDS destination) is written and restored inside the statement.
// Buffer form: wave-uniform base in a 128-bit descriptor (raw, stride 0),
// 32-bit per-lane byte offset (half the address payload of the global form).
typedef int knn_v4i __attribute__((ext_vector_type(4)));
__device__ __forceinline__ knn_v4i knn_rsrc(const void *base)
{
    const unsigned long long a = (unsigned long long)(uintptr_t)base;
    knn_v4i r;
    r.x = (int)(unsigned)a;
    r.y = (int)((unsigned)(a >> 32) & 0xffffu);
    r.z = -1;                 // num_records: no bounds check in practice
    r.w = 0x00020000;
    return r;
}
__device__ __forceinline__ void bglds16(knn_v4i rsrc, unsigned voff, unsigned lds_dst)
{
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
                 "buffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(voff), "s"(rsrc), "s"(__builtin_amdgcn_readfirstlane(lds_dst)) : "memory");
}
// 4-byte global form (corpus-norm slices: per-lane permuted gather)
__device__ __forceinline__ void glds4(const void *src, unsigned lds_dst)
{
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                 "global_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(src), "s"(__builtin_amdgcn_readfirstlane(lds_dst)) : "memory");
}

// ---------------------------------------------------------------------------
// Mode decision from the max-reduced meta (identical on every rank).
//   INT : every value an integer and every partial sum of the GEMM form
//         (norms, dot products, |q|^2+|c|^2, d^2) an integer below 2^p
//         (p = 53 / 24), so d^2 is exact, bit-identical to the reference's
//         S, and sqrt is injective on it.  fp64: (2 max|x|)^2 n
//         <= 2^51; fp32: n max|x|^2 <= 2^23 and n (max - min)^2 <= 2^24.
//   SCAN: non-finite values or norms near overflow -- no error bound.
//   GEMM: everything else.
// ---------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ int knn_mode_lim(const double *meta, int n, double lim)
{
    if constexpr (sizeof(T) == 8) {
        if (meta[KNN_META_NONFINITE] != 0.0 || !(meta[KNN_META_MAXNORM] < 1e290))
            return KNN_MODE_SCAN;
        double mx = meta[KNN_META_MAXABS];
        if (meta[KNN_META_NONINT] == 0.0 && mx * mx <= lim) return KNN_MODE_INT;
        return KNN_MODE_GEMM;
    } else {
        if (meta[KNN_META_NONFINITE] != 0.0 || !(meta[KNN_META_MAXNORM] < 1e37))
            return KNN_MODE_SCAN;
        const double mx = meta[KNN_META_MAXABS];
        const double rg = meta[KNN_META_MAXPOS] + meta[KNN_META_MAXNEG];
        if (meta[KNN_META_NONINT] == 0.0 && (double)n * mx * mx <= 8388608.0 &&
            (double)n * rg * rg <= 16777216.0)
            return KNN_MODE_INT;
        return KNN_MODE_GEMM;
    }
}
// lim = 2^51 / 4n (fp64 INT-mode limit on max|x|^2), the same correctly
// rounded quotient on the host or here; a caller with many waves passes the
// host's (k_merge_rank: no fp64 division a wave)
template <typename T>
__device__ __forceinline__ int knn_mode(const double *meta, int n)
{
    return knn_mode_lim<T>(meta, n, 2251799813685248.0 / (4.0 * (double)n));
}

// ---------------------------------------------------------------------------
// Register top-KP list: L ascending, insertion after equal keys (the lane's
// candidates arrive in increasing row order, so this is the reference's
// stable "lower index first" tie rule).  d >= L[KP-1] (incl. +inf,
// NaN, INT_MAX) is a no-op, so lanes without a candidate run it harmlessly.
// ---------------------------------------------------------------------------
template <int KP, typename T>
__device__ __forceinline__ void list_insert(T (&L)[KP], int (&I)[KP], T d, int id)
{
    bool c_hi = d < L[KP - 1];
#pragma unroll
    for (int e = KP - 1; e >= 0; e--) {
        bool c_lo = (e > 0) ? (d < L[e > 0 ? e - 1 : 0]) : false;
        T t = c_lo ? L[e > 0 ? e - 1 : 0] : d;
        int ti = c_lo ? I[e > 0 ? e - 1 : 0] : id;
        L[e] = c_hi ? t : L[e];
        I[e] = c_hi ? ti : I[e];
        c_hi = c_lo;
    }
}

__device__ __forceinline__ void wave_argmin(double &d, int &i)
{
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        double od = __shfl_xor(d, off);
        int oi = __shfl_xor(i, off);
        bool take = (od < d) || (od == d && oi < i);
        d = take ? od : d;
        i = take ? oi : i;
    }
}

// ---------------------------------------------------------------------------
// Byte blocks (the int8 contraction, knn_i8.hip; written by k_shadow8 from an
// element block or by k_pack8_* straight from the source, knn_kernels.hip)
// ---------------------------------------------------------------------------
// Row r of a byte block -> its slot in the norm array.  Tile t = r >> 7 owns
// 512 bytes; inside, [m-block b][lane half h][j][i] holds row 32b + 8j + 4h +
// i -- the row that accumulator register 4j + i of lane half h carries
// (32x32 C/D map: row = (reg & 3) + 8 (reg >> 2) + 4 (lane >> 5)), so a lane
// reads an m-block's 16 norms as 4 consecutive ds_read_b128.
__device__ __forceinline__ int i8_norm_pos(int r)
{
    const int rr = r & 127, b = rr >> 5, w = rr & 31;
    const int j = w >> 3, h = (w >> 2) & 1, i = w & 3;
    return (r & ~127) + (((b * 2 + h) * 4 + j) * 4 + i);
}

// A row's |x'|^2 is stored as two words (each array in i8_norm_pos order).
// The init word
//     IW(r) = -floor(|x'|^2 / 2)
// is where the row's MFMA accumulators start (the C operand of a tile's
// first K-step), so with A = q'.c' the accumulator ends at
//     acc = A + IW = (|q'|^2 - d^2 + p) / 2,   p = |x'|^2 & 1
// (A = (|q'|^2 + |x'|^2 - d^2) / 2, IW = -(|x'|^2 - p) / 2), and the epilogue
// filters on acc alone: 2 acc >= |q'|^2 - lim <=> d^2 <= lim + p admits every
// candidate with d^2 <= lim (and some with d^2 = lim + 1) without one VALU
// operation per candidate.  The slot word
//     K2(r) = 31 - slot(r) - 32 p,
// slot(r) = 16 (b & 1) + 4 j + i: the row's position among the 32
// accumulator registers of a pair of m-blocks (the lane's candidates in one
// epilogue group), increasing with the row, gives the survivors' exact key
//     v = 64 acc + K2 = 32 (|q'|^2 - d^2) + (31 - slot),
// which orders the lane's candidates by (d^2, row) in ONE signed integer:
// the lane's largest v is its nearest candidate, lowest row first on ties
// (SURVEY F1), and d^2 = |q'|^2 - (v >> 5), slot = 31 - (v & 31) come back
// out of it.  |x'|^2 = -2 IW - (K2 >> 5) (i8_norm_of).  Ranges (n <= 896
// bytes, |x'| <= 128, d^2 <= n 255^2): |acc| < 2^25, |v| < 2^31, and inside
// one lane (one query) the values span less than 32 (n 255^2 + 1) < 2^31
// (i8_next).
//
// Rows of more than 4 K-steps (rs > 128 bytes: MNIST) take the whole norm
// in the slot word and a zero init word:
//     K(r) = 31 - slot(r) - 32 |x'|^2,   IW(r) = 0,
// so acc = A, v = 64 A + K is the same key, i8_norm_of the same norm, and
// their kernels start the accumulators at zero instead of reading the init
// words (k_dist_topk_i8: SHORT) -- the accumulator filter that needs IW
// runs on short rows only, and on long rows the 8 init-word ds_read_b128 a
// tile were LDS traffic for nothing (|v| <= 64 n 128^2 + 32 n 128^2 < 2^31).
__device__ __forceinline__ bool i8_long_rows(int rs) { return rs > 128; }
__device__ __forceinline__ int i8_norm_word(int r, int nrm, int rs)
{
    const int rr = r & 127, b = rr >> 5, w = rr & 31;
    const int slot = 16 * (b & 1) + 4 * (w >> 3) + (w & 3);
    return 31 - slot - 32 * (i8_long_rows(rs) ? nrm : (nrm & 1));
}
__device__ __forceinline__ int i8_init_word(int nrm, int rs) { return i8_long_rows(rs) ? 0 : -(nrm >> 1); }
__device__ __forceinline__ int i8_norm_of(int k2, int iw) { return -2 * iw - (k2 >> 5); }
#endif
