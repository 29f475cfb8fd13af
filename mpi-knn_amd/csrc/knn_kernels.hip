// knn_kernels.hip -- CDNA4 (gfx950) kernels of the all-kNN engine.
//
// Hot path of yiapou13/mpi-knn: the distance loop + k-smallest insertion of
// knn-serial.c:72-93 (and its per-block copies mpi-knn-parallel_blocking.c:
// 155-181, 217-242).  Re-designed for MI355X:
//
//   k_pack_col / k_pack_row   column/row-major fp64/fp32 -> padded
//                row-major block + norms + meta in one pass (replaces
//                blk:100-109's packing).
//   k_dist_topk  fused fp64-MFMA contraction G = C.Q^T (v_mfma_f64_16x16x4)
//                with d^2 = |q|^2 + |c|^2 - 2G and a per-lane register top-k
//                (insertion network) behind a shared threshold.  One
//                workgroup = 128 queries x a corpus split; tiles of 128 rows
//                stream through a 4-stage LDS ring filled by global_load_lds.
//   k_merge      per query: tournament merge of the split/lane lists with
//                the running state (ring steps), exact re-rank of new
//                entries in reference order (GEMM mode).
//   k_finalize   order by (sqrt(S), idx), drop S == 0, certify that no
//                unseen candidate can enter the top-k, emit records.
//   k_rescan_*   exact reference-order scan for the (rare) queries the
//                certificate could not clear.
//
// Layout and roofline notes: DESIGN.md sec.4.
#include "knn_device.h"

// ---------------------------------------------------------------------------
// Element-type traits.  A staged chunk is 128 bytes of every row: 16 fp64
// or 32 fp32 features.  One 16-byte LDS fragment holds KSF k-steps of the
// 16x16x4 MFMA (2 fp64 / 4 fp32).  Result register r of lane group g holds
// tile row ROW(g, r) (probed: tools/probe/mfma_probe, mfma_f32_probe).
// ---------------------------------------------------------------------------
template <typename T> struct KT;
template <> struct KT<double> {
    typedef dbl4 acc_t;
    typedef dbl2 frag_t;
    static constexpr int KSF = 2;
    static constexpr double U = 1.1102230246251565e-16;   // 2^-53
    __device__ static __forceinline__ acc_t mfma(double a, double b, acc_t c)
    {
        return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
    }
    __device__ static constexpr int row(int g, int r) { return g + 4 * r; }
};
template <> struct KT<float> {
    typedef flt4 acc_t;
    typedef flt4 frag_t;
    static constexpr int KSF = 4;
    static constexpr double U = 5.9604644775390625e-08;   // 2^-24
    __device__ static __forceinline__ acc_t mfma(float a, float b, acc_t c)
    {
        return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
    }
    __device__ static constexpr int row(int g, int r) { return 4 * g + r; }
};
template <typename T> static constexpr int knn_bk() { return 128 / (int)sizeof(T); }

// fp16 contraction of fp32 blocks (H16): INT-mode data with |x| <= 2048 is
// exact in fp16, every product exact in fp32 and every partial sum an
// integer <= n max|x|^2 <= 2^23, so v_mfma_f32_16x16x32_f16 yields the same
// dot products as the fp32 MFMA chain, bit for bit, in any summation order.
// Lane (row, g) converts its two 16-byte fp32 slots of a chunk (features
// 4g..4g+3 of pieces 0 and 1) into one 8-half operand; the query side is
// converted identically, so each chunk's 32 features are summed once.
typedef _Float16 knn_h8 __attribute__((ext_vector_type(8)));
typedef _Float16 knn_h4 __attribute__((ext_vector_type(4)));
// fp64 blocks (H16 with ES 8): integer data with max|x| <= 256.  A chunk is
// 16 features; lane (row, g) converts its two 16-byte slots (features
// 2g, 2g+1 of pieces 0 and 1) into one 4-half operand of
// v_mfma_f32_16x16x16_f16.  Its fp32 sums are exact over 16 chunks (256
// features: |partial| <= 256 * 2^16 = 2^24), then flushed into the fp64
// accumulators, so the tile's dot products are the fp64 path's, bit for bit.
// Hardware conversions only: a plain (_Float16)(double) cast is folded
// into one f64->f16 rounding, which hipcc emulates in ~30 integer
// instructions (measured 2.5x slower than the fp64 kernel).  Here
// v_cvt_f32_f64 then v_cvt_pkrtz_f16_f32 -- exact for these integers.
typedef __fp16 knn_hp2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ knn_h4 knn_to_h4(dbl2 a, dbl2 b)
{
    const knn_hp2 lo = __builtin_amdgcn_cvt_pkrtz((float)a.x, (float)a.y);
    const knn_hp2 hi = __builtin_amdgcn_cvt_pkrtz((float)b.x, (float)b.y);
    typedef unsigned int u2 __attribute__((ext_vector_type(2)));
    u2 w;
    w.x = __builtin_bit_cast(unsigned int, lo);
    w.y = __builtin_bit_cast(unsigned int, hi);
    return __builtin_bit_cast(knn_h4, w);
}
__device__ __forceinline__ knn_h8 knn_to_h8(flt4 a, flt4 b)
{
    knn_h8 r;
    r[0] = (_Float16)a.x; r[1] = (_Float16)a.y; r[2] = (_Float16)a.z; r[3] = (_Float16)a.w;
    r[4] = (_Float16)b.x; r[5] = (_Float16)b.y; r[6] = (_Float16)b.z; r[7] = (_Float16)b.w;
    return r;
}

// (knn_mode: the search mode from the reduced meta, knn_device.h)

// Reference-order exact squared distance: S = S + (a-b)^2 over j = 0..n-1,
// two roundings per feature, no FMA (knn-serial.c:76-85; pow(x,2) -> x*x),
// in fp64 on the block's values (fp32 blocks: the fp32-rounded inputs).
// Rows are zero padded to n_pad (a multiple of 128 bytes) and S + (0-0)^2 =
// S, so the loop runs over whole 128-byte pieces, S bit-identical.  The sum
// is one dependent chain, and each lane's candidate row is its own gather:
// 8 pieces of 16 bytes of both rows are loaded before any is used (16 loads
// in flight a lane), so the chain waits on one memory latency every 128
// bytes instead of every 16 (k_merge's re-rank was latency-bound on those
// loads).
template <typename T>
__device__ __forceinline__ double knn_exact_sq_v(const T *__restrict__ a, const T *__restrict__ b,
                                                 int n_pad)
{
#pragma clang fp contract(off)
    typedef typename std::conditional<sizeof(T) == 8, dbl2, flt4>::type vec_t;
    constexpr int V = 16 / (int)sizeof(T), U = 8;
    const int nr = n_pad / V;   // a multiple of U (n_pad: 128-byte rows)
    double S = 0.0;
    for (int p = 0; p < nr; p += U) {
        vec_t va[U], vb[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            va[u] = ((const vec_t *)a)[p + u];
            vb[u] = ((const vec_t *)b)[p + u];
        }
#pragma unroll
        for (int u = 0; u < U; u++)
#pragma unroll
            for (int e = 0; e < V; e++) {
                const double t = (double)va[u][e] - (double)vb[u][e];
                const double t2 = t * t;
                S = S + t2;
            }
    }
    return S;
}

// Certificate margin: |GEMM-form d^2 - exact S| plus the reference's own
// rounding, for any candidate c of the search (|c|^2 <= maxnorm):
//   fp32 filter: fma-chain dot gamma_n (|q|^2+|c|^2), norm roundings and the
//   two final roundings 4u (|q|^2+|c|^2), times (1 + 2(n+4)u) for the
//   second-order terms; the reference's fp64 S: 4(n+2) 2^-53 (|q|^2+|c|^2).
//   fp64 filter: both at u = 2^-53, 8(n+4)u (|q|^2+|c|^2).
//   split fp16 filter (fp32 blocks, knn_shadow_split): each value scaled by
//   S = 2^e (maxabs S in [2^13, 2^14)) and split x S = hi + lo in fp16;
//   hi.hi + hi.lo + lo.hi on v_mfma_f32_16x16x32_f16.  Per element
//   |xS - hi - lo| <= 2^-22 |xS| + 2^-25 and the dropped lo.lo <=
//   2^-22 |q_j c_j| (+ subnormal terms): 3 2^-22 sum|q_j c_j|, 12u qc for d^2.
//   fp16 products are exact in fp32; each 32-feature chunk's 96 products
//   are summed apart in fp32 (any order: <= 95u sum|chunk terms|) and the
//   n/32 chunk sums added to the fp32 accumulator (<= (n/32) u sum|q_j
//   c_j|), so d^2 is off by (97 + n/32) 1.01 u qc; norms (fp64 blocks: their
//   fp64 norms rounded to fp32), qn + cn and the final fma 4u qc.  With a
//   20% margin (the MFMA's internal order is not specified; its precision
//   is at least fp32): ((136 + n/25) u + 4 (n+4) 2^-53) qc, fp32 and fp64
//   blocks alike.  Subnormal fp16 halves may be flushed by the MFMA:
//   then up to 2^-14 / S <= 2^-27 maxabs is lost per element, the absolute
//   part 2^-26 maxabs sqrt(n) (|q| + |c|).  The fp32 filter's is ~ (n + 4)
//   u qc.
template <typename TE>
__device__ __forceinline__ double knn_cert_E(int n, double qn, double maxnorm, int split = 0,
                                             double maxabs = 0.0)
{
    const double u = KT<TE>::U;
    const double nn = (double)n + 4.0, qc = qn + maxnorm;
    if (split) {
        const double ul = 5.9604644775390625e-08;   // 2^-24
        // the n/32 chunk sums are added in fp32 (k_dist_split, fp32 and fp64
        // blocks alike)
        const double acc = (double)n / 25.0;
        return ((136.0 + acc) * ul + 4.0 * nn * 1.1102230246251565e-16) * qc * (1.0 + 1e-6) +
               1.4901161193847656e-08 * maxabs * sqrt((double)n) * (sqrt(qn) + sqrt(maxnorm));
    }
    if constexpr (sizeof(TE) == 8) return 8.0 * nn * u * qc;
    else return nn * qc * (u * (1.0 + 2.0 * nn * u) + 4.0 * 1.1102230246251565e-16);
}

// ---------------------------------------------------------------------------
// Packing (blk:100-109): src (S = fp64 or fp32; col-major, ld >= rows |
// row-major, ld >= n) -> padded row-major block of T, the squared norms
// (fp64 accumulate, stored as T) and the meta (max|x|, max norm,
// non-integer, non-finite, max(x)+, max(-x)+), in ONE pass over the source
// (the norms are taken from the stored T values).  Per workgroup the meta
// is reduced, then one atomicMax per word (non-negative doubles order like
// their bits; the caller zeroes the meta).
// ---------------------------------------------------------------------------
struct knn_meta_acc {
    double mabs = 0.0, nonint = 0.0, nonfin = 0.0, mpos = 0.0, mneg = 0.0;
    __device__ __forceinline__ void add(double v, double &s)
    {
        s = fma(v, v, s);
        if (!__builtin_isfinite(v)) nonfin = 1.0;
        else {
            const double a = fabs(v);
            mabs = a > mabs ? a : mabs;
            mpos = v > mpos ? v : mpos;
            mneg = -v > mneg ? -v : mneg;
            if (v != rint(v)) nonint = 1.0;
        }
    }
};

// workgroup reduction of the 6 meta words (64 W threads) + atomicMax
template <int W>
__device__ __forceinline__ void knn_meta_flush_w(const knn_meta_acc &a, double mnorm, double *meta)
{
    __shared__ double red[W][6];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    double w[6] = {a.mabs, mnorm, a.nonint, a.nonfin, a.mpos, a.mneg};
#pragma unroll
    for (int q = 0; q < 6; q++)
        for (int off = 32; off > 0; off >>= 1) w[q] = fmax(w[q], __shfl_xor(w[q], off));
    if (lane == 0) {
#pragma unroll
        for (int q = 0; q < 6; q++) red[wave][q] = w[q];
    }
    __syncthreads();
    if (threadIdx.x < 6) {
        double v = red[0][threadIdx.x];
#pragma unroll
        for (int x = 1; x < W; x++) v = fmax(v, red[x][threadIdx.x]);
        if (!(v >= 0.0)) v = __builtin_inf();   // NaN norm -> treat as overflow
        atomicMax((unsigned long long *)&meta[threadIdx.x], (unsigned long long)__double_as_longlong(v));
    }
}
__device__ __forceinline__ void knn_meta_flush(const knn_meta_acc &a, double mnorm, double *meta)
{
    knn_meta_flush_w<4>(a, mnorm, meta);
}

// Column-major source (the .mat layout): a workgroup owns 64 rows and walks
// the columns in 64 x 64 tiles through LDS (reads: 64 consecutive rows of a
// column, 512 B; writes: 64 consecutive features of a row).  Thread (ty,
// tx) accumulates row tx's squared terms over columns = ty mod 4; the four
// partials are summed at the end (a fixed order).
template <typename T, typename S>
__global__ __launch_bounds__(256) void k_pack_col(T *__restrict__ blk, size_t rows, size_t rows_pad,
                                                  int n, int n_pad, const S *__restrict__ src, size_t ld)
{
    __shared__ T tile[64][65];
    __shared__ double part[4][64];
    T *norms = blk + rows_pad * (size_t)n_pad;
    double *meta = (double *)(norms + rows_pad);
    const size_t i0 = (size_t)blockIdx.x * 64;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    const size_t i = i0 + tx;
    knn_meta_acc ma;
    double s = 0.0;
    for (int j0 = 0; j0 < n_pad; j0 += 64) {
#pragma unroll 4
        for (int jj = ty; jj < 64; jj += 4) {
            const int j = j0 + jj;
            const T v = (i < rows && j < n) ? (T)src[i + (size_t)j * ld] : (T)0;
            tile[jj][tx] = v;
            ma.add((double)v, s);
        }
        __syncthreads();
        const int j = j0 + tx;
#pragma unroll 4
        for (int ii = ty; ii < 64; ii += 4)
            if (i0 + ii < rows_pad && j < n_pad) blk[(i0 + ii) * n_pad + j] = tile[tx][ii];
        __syncthreads();
    }
    part[ty][tx] = s;
    __syncthreads();
    double mnorm = 0.0;
    if (ty == 0 && i < rows_pad) {
        const double nr = (part[0][tx] + part[1][tx]) + (part[2][tx] + part[3][tx]);
        norms[i] = (T)nr;
        if (nr == nr) mnorm = nr;
        else ma.nonfin = 1.0;
    }
    knn_meta_flush(ma, mnorm, meta);
}

// ---------------------------------------------------------------------------
// Speculative byte block straight from the source (knn_block_pack_s8): the
// int8 contraction's rows x' = x - 128 (rows of rs = round_up(n, 32) bytes,
// zero past n and on padding rows), its norm words (i8_norm_word of the
// exact int32 |x'|^2) and the block meta of the element pack above (the same
// six words over the values as T).  The shift the int8 path uses is
// o = 128 - max(-x)+ of the reduced meta (knn_i8.hip), so the image is the
// one k_shadow8 would write exactly when every value is an integer in
// [0, 255] -- knn_s8_spec_ok on the reduced meta (MNIST pixels, SIFT
// descriptors); otherwise the caller packs the element block after all.  One
// read of the source and 1 byte written an element, instead of the element
// block (8 or 4 bytes written, read back by k_shadow8).
// ---------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ int knn_spec8(T v)
{
    // x - 128 of an in-window integer; anything else gives garbage the meta
    // rejects: NaN -> 0 and a clamp to [-32640, 32895], so the conversion is
    // defined and (x - 128)^2 < 2^31 (the squares are summed as unsigned)
    const T c = v == v ? (v < (T)-32640 ? (T)-32640 : (v > (T)32895 ? (T)32895 : v)) : (T)0;
    return (int)c - 128;
}

// col-major source (the .mat layout): a workgroup owns RW rows and walks
// the columns in 64-column tiles (RW = 64: each wave reads 64 consecutive
// rows of one column, 512-byte runs; RW = 32: two columns of 32 rows a
// wave), all of a thread's loads of a tile in flight before their
// conversion; bytes go through LDS into 16-byte row stores.  Thread (ty, tx)
// sums row tx's squares over columns = ty mod (256 / RW); the partials add
// exactly for the integer data the byte block holds (the meta decides
// that; rejected data is packed again from elements).
// (Issuing the next tile's loads before converting this one -- 32 in
// flight at RW = 64 -- measured slower: 106 -> 130 us for MNIST, rocprofv3.)
template <typename T, typename S, int RW>
__global__ __launch_bounds__(256) void k_pack8_col(signed char *__restrict__ dst, size_t rows, size_t rows_pad,
                                                   int n, int rs, const S *__restrict__ src, size_t ld)
{
    constexpr int CG = 256 / RW;      // column groups
    constexpr int NE = 64 / CG;       // loads a thread a tile
    __shared__ unsigned char tb[64][RW + 4];   // [column of the tile][row]
    __shared__ double part[CG][RW];
    __shared__ unsigned ipart[CG][RW];
    int *norms = (int *)(dst + rows_pad * (size_t)rs);
    double *meta = (double *)(norms + 2 * rows_pad);
    const size_t i0 = (size_t)blockIdx.x * RW;
    const int tx = threadIdx.x % RW, ty = threadIdx.x / RW;
    const size_t i = i0 + tx;
    const bool live = i < rows;
    const S *xp = src + (live ? i : 0);
    knn_meta_acc ma;
    double s = 0.0;
    unsigned si = 0u;
    for (int j0 = 0; j0 < rs; j0 += 64) {
        S v[NE];
#pragma unroll
        for (int e = 0; e < NE; e++) {
            const int j = j0 + ty + CG * e;
            v[e] = (live && j < n) ? __builtin_nontemporal_load(xp + (size_t)j * ld) : (S)0;
        }
#pragma unroll
        for (int e = 0; e < NE; e++) {
            const T x = (T)v[e];
            ma.add((double)x, s);
            const int xi = (live && j0 + ty + CG * e < n) ? knn_spec8(x) : 0;
            si += (unsigned)(xi * xi);
            tb[ty + CG * e][tx] = (unsigned char)xi;
        }
        __syncthreads();
        // row r = t / 4: 16 bytes at column 16 (t % 4) of the tile
        const int r = threadIdx.x >> 2, c0 = 16 * (threadIdx.x & 3);
        if (r < RW && i0 + r < rows_pad && j0 + c0 < rs) {
            unsigned w4[4];
#pragma unroll
            for (int q = 0; q < 4; q++)
                w4[q] = (unsigned)tb[c0 + 4 * q][r] | ((unsigned)tb[c0 + 4 * q + 1][r] << 8) |
                        ((unsigned)tb[c0 + 4 * q + 2][r] << 16) | ((unsigned)tb[c0 + 4 * q + 3][r] << 24);
            *(knn_v4i *)(dst + (i0 + r) * (size_t)rs + j0 + c0) = (knn_v4i){(int)w4[0], (int)w4[1], (int)w4[2], (int)w4[3]};
        }
        __syncthreads();
    }
    part[ty][tx] = s;
    ipart[ty][tx] = si;
    __syncthreads();
    double mnorm = 0.0;
    if (ty == 0 && i < rows_pad) {
        double nr = 0.0;
        unsigned ni = 0u;
        if constexpr (CG == 4) {
            nr = (part[0][tx] + part[1][tx]) + (part[2][tx] + part[3][tx]);
            ni = (ipart[0][tx] + ipart[1][tx]) + (ipart[2][tx] + ipart[3][tx]);
        } else {
#pragma unroll
            for (int q = 0; q < CG; q++) {
                nr += part[q][tx];
                ni += ipart[q][tx];
            }
        }
        norms[i8_norm_pos((int)i)] = i8_norm_word((int)i, (int)ni, rs);
        norms[rows_pad + i8_norm_pos((int)i)] = i8_init_word((int)ni, rs);
        if (nr == nr) mnorm = nr;
        else ma.nonfin = 1.0;
    }
    knn_meta_flush(ma, mnorm, meta);
    if (blockIdx.x == 0 && threadIdx.x == 0) meta[KNN_META_S8] = 1.0;
}

// row-major source: one wave per row, lane l converts the 8-element groups
// l, l + 64, ... (one 8-byte store each); VEC: 16-byte-aligned rows, whole
// groups read as 16-byte vectors (sift: 0.68 ms for 512 MB with scalar loads)
template <typename T, typename S, bool VEC>
__global__ __launch_bounds__(256) void k_pack8_row(signed char *__restrict__ dst, size_t rows, size_t rows_pad,
                                                   int n, int rs, const S *__restrict__ src, size_t ld)
{
    typedef typename std::conditional<sizeof(S) == 8, dbl2, flt4>::type svec_t;
    constexpr int SV = 16 / (int)sizeof(S);
    int *norms = (int *)(dst + rows_pad * (size_t)rs);
    double *meta = (double *)(norms + 2 * rows_pad);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int ng = rs / 8;
    knn_meta_acc ma;
    double mnorm = 0.0;
    for (size_t r = (size_t)blockIdx.x * 4 + wave; r < rows_pad; r += (size_t)gridDim.x * 4) {
        double s = 0.0;
        unsigned si = 0u;
        const S *x = src + r * ld;
        for (int g = lane; g < ng; g += 64) {
            unsigned lo = 0u, hi = 0u;
            S sv[8];
            if (VEC && r < rows && 8 * g + 8 <= n) {
#pragma unroll
                for (int q = 0; q < 8 / SV; q++) {
                    const svec_t w = *(const svec_t *)(x + 8 * g + SV * q);
#pragma unroll
                    for (int e = 0; e < SV; e++) sv[SV * q + e] = w[e];
                }
            } else {
#pragma unroll
                for (int e = 0; e < 8; e++) sv[e] = (r < rows && 8 * g + e < n) ? x[8 * g + e] : (S)0;
            }
#pragma unroll
            for (int e = 0; e < 8; e++) {
                const int j = 8 * g + e;
                const bool in = r < rows && j < n;
                const T v = in ? (T)sv[e] : (T)0;
                ma.add((double)v, s);
                const int xi = in ? knn_spec8(v) : 0;
                si += (unsigned)(xi * xi);
                if (e < 4) lo |= ((unsigned)xi & 0xffu) << (8 * e);
                else hi |= ((unsigned)xi & 0xffu) << (8 * (e - 4));
            }
            typedef unsigned u2 __attribute__((ext_vector_type(2)));
            *(u2 *)(dst + r * (size_t)rs + 8 * g) = (u2){lo, hi};
        }
        for (int off = 32; off > 0; off >>= 1) {
            s += __shfl_xor(s, off);
            si += (unsigned)__shfl_xor((int)si, off);
        }
        if (lane == 0) {
            norms[i8_norm_pos((int)r)] = i8_norm_word((int)r, (int)si, rs);
            norms[rows_pad + i8_norm_pos((int)r)] = i8_init_word((int)si, rs);
        }
        if (s == s) mnorm = s > mnorm ? s : mnorm;
        else ma.nonfin = 1.0;
    }
    knn_meta_flush(ma, mnorm, meta);
    if (blockIdx.x == 0 && threadIdx.x == 0) meta[KNN_META_S8] = 1.0;
}

// Row-major source: one wave per row (lane-strided features, butterfly sum).
template <typename T, typename S>
__global__ __launch_bounds__(256) void k_pack_row(T *__restrict__ blk, size_t rows, size_t rows_pad,
                                                  int n, int n_pad, const S *__restrict__ src, size_t ld)
{
    T *norms = blk + rows_pad * (size_t)n_pad;
    double *meta = (double *)(norms + rows_pad);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    knn_meta_acc ma;
    double mnorm = 0.0;
    for (size_t i = (size_t)blockIdx.x * 4 + wave; i < rows_pad; i += (size_t)gridDim.x * 4) {
        double s = 0.0;
        const S *x = src + i * ld;
        T *o = blk + i * (size_t)n_pad;
        for (int j = lane; j < n_pad; j += 64) {
            const T v = (i < rows && j < n) ? (T)x[j] : (T)0;
            o[j] = v;
            ma.add((double)v, s);
        }
        for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
        if (lane == 0) norms[i] = (T)s;
        if (s == s) mnorm = s > mnorm ? s : mnorm;
        else ma.nonfin = 1.0;
    }
    knn_meta_flush(ma, mnorm, meta);
}

// ---------------------------------------------------------------------------
// k_dist_topk
//
// Workgroup: 512 threads = 8 waves; 128 queries (wave w: queries 16w..16w+15)
// x corpus tiles of 128 rows (8 m-tiles of 16).  Per wave per 16-feature
// chunk: 8 m-tiles x 4 k-steps = 32 v_mfma_f64_16x16x4_f64.
//
// f64 MFMA operand map (probed, tools/probe): lane l supplies A[l&15][l>>4]
// and B[l>>4][l&15]; D reg r of lane l is D[(l>>4)+4r][l&15].  A = corpus
// rows, B = queries, so lane l ends with 32 d^2 of ONE query (l&15) against
// corpus rows 16mt + (l>>4) + 4r.  The 4 lanes sharing a query (g = l>>4)
// keep separate lists over disjoint row sets; they share a threshold.
//
// k-permutation: in a 16-feature chunk, k-step s = 2p+e of lane group g uses
// feature 8p + 2g + e, so each lane's two k-steps of piece p are one 16-byte
// slot (segment 4p+g of the row's 128 bytes): one ds_read_b128.
//
// Staging: a 4-deep ring of 32 KiB LDS stages filled by LDS-DMA
// (buffer_load_dwordx4 ... lds).  One load instruction moves 8 rows x 128
// contiguous bytes (full lines: lane 8r+s fetches 16-byte segment s^(r&7) of
// row r), so a 16-row block is two loads and its LDS image is
// [row][segment ^ (row&7)] -- the XOR keeps the fragment reads conflict-free.
// Each wave stages its own m-tile (loads 0,1) and its own 16 queries
// (loads 2,3): 4 instructions per chunk, scalar addressing.
//
// The schedule is branch-free: chunk x's load 0 issues in segment S3 of
// chunk x-4 (after the barrier that freed its stage) and loads 1..3 in
// S0..S2 of chunk x-3, one per segment.  Chunks past the end re-load the
// last valid chunk (clamped address) into their stage, so every chunk issues
// the same loads and "chunk c+1 landed" is always one static
// `s_waitcnt vmcnt(8)` (guide sec.5 'Pipelining across barriers'; LDS-DMA
// stays in flight across barriers).  A straight-line body keeps the
// accumulators in place: the previous loop (one flat loop with a conditional
// epilogue and a last-chunk branch) made the register allocator shuttle them
// with v_mov + s_nop after every S1/S3 MFMA.
//
// Corpus norms: one 1 KiB slice per tile, loaded two tiles ahead at the
// start of a tile into a ring [tile&7][g][32] (row 4k+g at [g][k]; waves
// 4..7 repeat the bytes of waves 0..3); the >= 8 loads that follow it before
// that tile's epilogue make the vmcnt(8) waits cover it.
//
// Segments per chunk, 8 MFMAs each (an m-tile's two k-steps back to back:
// measured 1.2% faster than splitting the dependent pair) with the LDS
// reads of the next segment's fragments between them:
//   S0 (p0, mt0-3) S1 (p0, mt4-7) S2 (p1, mt0-3) | lgkmcnt(0), vmcnt(8),
//   barrier | S3 (p1, mt4-7) reading chunk c+1's first fragments.
//
// LDS (one array, guide 'second __shared__ object' trap):
//   stage s at s*32K: C [mt][row 16][128 B] (16 KiB), Q [w][row 16][128 B]
//   4*32K:            corpus norms ring [tile&7][g][32]
// ---------------------------------------------------------------------------
#define KNN_NST 4
// STG = 1: waves 0..3 stage the chunk pieces of their SIMD partners w + 4 too
// (fp16 shadow rows of fp32 blocks: sift 607 vs 691 ms); STG = 0: every wave
// stages its own.  Round-1 ablations of this kernel (no staging, no barrier,
// no insertion, setprio, MFMA orders: DESIGN.md sec.4) were measured with the
// tuning harness at commit 1e35c3d; the product source carries no hooks.
template <typename T, int KL, int KS, int STG = 0, int H16 = 0>
__global__ __launch_bounds__(512, 2) void k_dist_topk(
    const T *__restrict__ qblk, const T *__restrict__ qnorm, size_t q_base, int nq,
    const T *__restrict__ cblk, const T *__restrict__ cnorm, size_t c_base, int nc,
    int n, int n_pad, int ntiles, int nsplit, int nqb, const double *__restrict__ meta,
    double *__restrict__ part_d, int *__restrict__ part_i, double *__restrict__ part_T,
    int nq_pad, unsigned long long *__restrict__ qthr, int uj, int xord)
{
    constexpr int NST = KNN_NST;
    // H16 2: qblk / cblk are fp16 shadow rows (k_shadow), n_pad their row
    // length; the norms stay in the element blocks.  (Split fp16 rows have a
    // kernel of their own, k_dist_split in knn_split.hip.)
    constexpr int RS = H16 == 2 ? 2 : (int)sizeof(T);   // bytes per staged element
    constexpr int BK = 128 / RS;                      // features per 128-B chunk
    // fp64 H16 (knn_to_h4): the fp32 MFMA output layout, row 4g + r of a
    // 16-row m-tile in lane group g, register r, instead of fp64's g + 4r
    constexpr bool H16D = H16 != 0 && sizeof(T) == 8;
    constexpr bool F32L = H16 != 0 && sizeof(T) == 8;   // fp64 accumulators, fp32 MFMA layout
    auto rowmap = [](int gg, int r) { return F32L ? 4 * gg + r : KT<T>::row(gg, r); };
    constexpr int ES = (int)sizeof(T);
    typedef typename KT<T>::acc_t acc_t;
    typedef typename KT<T>::frag_t frag_t;
    constexpr int KSF = KT<T>::KSF;
    __shared__ __attribute__((aligned(16))) char smem[NST * 32768 + 8192];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int g = lane >> 4, j16 = lane & 15;
    // xord 0, split-major: the first resident wave of workgroups shares one
    // corpus split, so its tiles are read from L2 by every XCD's workgroups.
    // xord 1, XCD-grouped: workgroups go to XCDs round-robin (blockIdx % 8),
    // so the nsplit workgroups of query block qb get ids 8(j nsplit + s) +
    // (qb % 8): one XCD, dispatched back to back -- they stream the same
    // query chunks in step (L2 hits), and co-resident blocks of one split
    // share corpus tiles.  The grid is padded to whole groups of 8 blocks.
    int qb, split;
    if (xord) {
        const int slot = blockIdx.x >> 3;
        split = slot % nsplit;
        qb = ((slot / nsplit) << 3) + (blockIdx.x & 7);
        if (qb >= nqb) return;
    } else {
        qb = blockIdx.x % nqb;
        split = blockIdx.x / nqb;
    }
    // long splits first: splits 0..tr-1 take tb+1 tiles, the rest tb, so in
    // split-major order the longest workgroups are dispatched first and the
    // short ones fill the tail (knn_engine.c: choose_splits models this)
    const int tb = ntiles / nsplit, tr = ntiles - tb * nsplit;
    const int t_lo = split * tb + (split < tr ? split : tr);
    const int t_hi = t_lo + tb + (split < tr ? 1 : 0);
    const int mode = knn_mode<T>(meta, n);
    const int qrow0 = qb * KNN_TQ;
    const int myq = qrow0 + 16 * wave + j16;          // block-local query row
    const long gq = (long)q_base + myq;
    const T qn = qnorm[myq];
    // consume qn here: its first real use (the epilogue) would otherwise get
    // a vmcnt(0) from hipcc that drains the staging ring once per tile
    asm volatile("" ::"v"(qn));
    const int nfc = n_pad / BK;
    // lane list slot behind the shared bound: INT mode k+1 candidates (exact
    // keys, tightest filter); GEMM mode the whole state (slack for the
    // certificate's error margin)
    const int ujm = (mode == KNN_MODE_INT) ? (uj & 255) : (uj >> 8);

    T L[KL];
    int I[KL];
#pragma unroll
    for (int e = 0; e < KL; e++) { L[e] = KNN_INF; I[e] = -1; }
    // Shared per-query bound across splits and ring steps (qthr, bits of a
    // non-negative double, atomicMin).  Any split's thr bounds the query's
    // (k+1)-th candidate over ALL rows (>= k+1 distinct candidates lie below
    // it), so a split may start filtering at the smallest bound published so
    // far.  Every value ever stored is a valid bound, so a stale read only
    // costs filter strength; the returning atomic reads it at the memory
    // side.  part_T still records the bound this split filtered with.
    // (fp32: every published value came from an fp32 bound, so the
    // conversion back is exact)
    T thr = (T)KNN_INF;
    if (qthr != nullptr && myq < nq)
        thr = (T)__longlong_as_double((long long)atomicMin(qthr + myq, 0x7ff0000000000000ull));
    if (myq >= nq) thr = -(T)KNN_INF;   // padding queries reject every candidate
    asm volatile("" ::"v"(thr));

    const int total = (mode == KNN_MODE_SCAN || t_hi <= t_lo) ? 0 : (t_hi - t_lo) * nfc;

    acc_t acc[8];
#pragma unroll
    for (int mt = 0; mt < 8; mt++) acc[mt] = (acc_t){0, 0, 0, 0};
    // fp64 H16: fp32 partial sums of up to 16 chunks (see knn_to_h4)
    flt4 acc32[H16D ? 8 : 1];
#pragma unroll
    for (int mt = 0; mt < (H16D ? 8 : 1); mt++) acc32[mt] = (flt4){0, 0, 0, 0};
    int grp = 0;
    auto flush32 = [&]() {
        if constexpr (H16D) {
#pragma unroll
            for (int mt = 0; mt < 8; mt++) {
#pragma unroll
                for (int r = 0; r < 4; r++) acc[mt][r] += (double)acc32[H16D ? mt : 0][r];
                acc32[H16D ? mt : 0] = (flt4){0, 0, 0, 0};
            }
            grp = 0;
        }
    };

    LDS_AS char *lds = (LDS_AS char *)smem;

    // ---- staging cursor (wave-uniform; clamps at the last chunk) ---------
    const int lr = lane >> 3, ls = lane & 7;
    const int seg_b = 16 * (ls ^ lr);                        // byte offset within the 128-B row
    // norms land permuted as [g][k] = norm of tile row 16(k>>2) + ROW(g, k&3)
    // (the rows lane group g holds, in register order), in 4-byte pieces:
    // 256 pieces a tile for fp64 (waves 0..3), 128 for fp32 (waves 0,1);
    // the other waves repeat the same bytes
    constexpr int NU = 128 * ES / 4;                         // 4-byte pieces per tile
    const int cn_unit = (__builtin_amdgcn_readfirstlane(wave) & (NU / 64 - 1)) * 64 + lane;
    const int cn_p = ES == 8 ? cn_unit >> 1 : cn_unit;       // norm index g*32 + k
    const int cn_k = cn_p & 31;
    const int cn_src_off = (16 * (cn_k >> 2) + rowmap(cn_p >> 5, cn_k & 3)) * ES +
                           (ES == 8 ? (cn_unit & 1) * 4 : 0);
    int s_c = 0, s_t = t_lo, s_fc = 0;                       // chunk being staged
    // Every wave stages its own m-tile and its own 16 queries.  All staging
    // addresses are scalar (wave_s, not the VGPR wave index): deriving the
    // LDS destination per load from a VGPR (v_readfirstlane into M0) cost
    // 2.9 ms.  STG = 1 moves all staging to waves 0..3 (they load for
    // their SIMD partner w+4 too): 0.6 ms slower on fp64 element rows once
    // addressing is scalar.
    const int wave_s = __builtin_amdgcn_readfirstlane(wave);
    constexpr bool SELF = STG == 0;
    const bool loader = SELF || wave_s < 4;
    auto glds1 = [&](int i) {
        if (!loader) return;
        const unsigned r8 = 8u * RS * (unsigned)n_pad;             // 8 rows, bytes
        const size_t fo = (size_t)128 * s_fc;                      // chunk offset, bytes
        const char *cb = (const char *)cblk +
                         (size_t)s_t * KNN_TC * n_pad * RS + fo;
        const char *qb0 = (const char *)qblk + (size_t)qrow0 * n_pad * RS + fo;
#pragma unroll
        for (int hw = 0; hw < (SELF ? 1 : 2); hw++) {
            const int ww = SELF ? wave_s : (wave_s & 3) + 4 * hw;
            const unsigned dst = (unsigned)(uintptr_t)lds + (unsigned)(s_c & (NST - 1)) * 32768u +
                                 (unsigned)ww * 2048u;
            const unsigned vo = (unsigned)((16 * ww + lr) * n_pad * RS + seg_b);
            if (i == 0) bglds16(knn_rsrc(cb), vo, dst);
            if (i == 1) bglds16(knn_rsrc(cb), vo + r8, dst + 1024);
            if (i == 2) bglds16(knn_rsrc(qb0), vo, dst + 16384);
            if (i == 3) bglds16(knn_rsrc(qb0), vo + r8, dst + 17408);
        }
    };
    auto advance = [&]() {
        s_c++;
        if (s_c < total) {
            if (++s_fc == nfc) {
                s_fc = 0;
                s_t++;
            }
        }
    };
    // norm slice of tile t (clamped to the split) into ring slot `slot`
    auto gnorm = [&](int t, int slot) {
        if (!loader) return;
        const int ts = t < t_hi ? t : t_hi - 1;
        const unsigned ndst = (unsigned)(uintptr_t)lds + NST * 32768u + (unsigned)(slot & 7) * 1024u +
                              (unsigned)(wave_s & (NU / 64 - 1)) * 256u;
        glds4((const char *)(cnorm + (size_t)ts * KNN_TC) + cn_src_off, ndst);
    };

    // ---- epilogue of tile t: d^2, threshold filter, insertion ------------
    // Common case (late in the scan): d^2, one masked-tile test on SGPRs,
    // the lane minimum against the bound, one ballot.  The per-candidate
    // pending mask is built only when some lane has a survivor.
    auto epilogue = [&](int t, acc_t (&A)[8]) {
        const LDS_AS T *cng = (const LDS_AS T *)(lds + NST * 32768 + (t & 7) * 1024) + 32 * g;
        const T lim = L[KL - 1] < thr ? L[KL - 1] : thr;
        // wave-uniform (scalar): only the block's last tile has rows >= nc,
        // and only tiles holding one of this wave's queries contain a self
        // pair.  Derived from wave_s, not the VGPR wave index, so it is a
        // scalar branch -- from the VGPR form hipcc predicated all 32
        // elements with exec masks (~9 issued instructions each).
        const int row0 = t * KNN_TC;
        const long gt0 = (long)c_base + row0, gw0 = (long)q_base + qrow0 + 16 * wave_s;
        const bool masked = (row0 + KNN_TC > nc) || (gw0 < gt0 + KNN_TC && gt0 < gw0 + 16);
        // d^2 overwrites the accumulators in place; the norms are read in
        // two halves of 4 m-tiles (one wait each, 16 temporaries)
#pragma unroll
        for (int hh = 0; hh < 2; hh++) {
            T cnr[4][4];
#pragma unroll
            for (int m4 = 0; m4 < 4; m4++) {
                const int mt = 4 * hh + m4;
                if constexpr (ES == 8) {
                    const dbl2 n01 = ((const LDS_AS dbl2 *)cng)[2 * mt];
                    const dbl2 n23 = ((const LDS_AS dbl2 *)cng)[2 * mt + 1];
                    cnr[m4][0] = n01.x; cnr[m4][1] = n01.y; cnr[m4][2] = n23.x; cnr[m4][3] = n23.y;
                } else {
                    const flt4 n4 = ((const LDS_AS flt4 *)cng)[mt];
                    cnr[m4][0] = n4.x; cnr[m4][1] = n4.y; cnr[m4][2] = n4.z; cnr[m4][3] = n4.w;
                }
            }
#pragma unroll
            for (int m4 = 0; m4 < 4; m4++)
#pragma unroll
                for (int r = 0; r < 4; r++)
                    A[4 * hh + m4][r] = fma((T)-2, A[4 * hh + m4][r], qn + cnr[m4][r]);
        }
        T lanemin = A[0][0];
#pragma unroll
        for (int mt = 0; mt < 8; mt++)
#pragma unroll
            for (int r = (mt == 0 ? 1 : 0); r < 4; r++) lanemin = fmin(lanemin, A[mt][r]);
        // zeros (INT-mode exact duplicates) and masked tiles only send the
        // wave down the slow path, where d^2 > 0 and the row mask are
        // applied (masking here made hipcc copy all 32 d^2 at the join)
        const bool any = masked || __ballot(lanemin <= lim) != 0ull;   // rare late in the scan
        if (any) {
            // INT mode: d^2 is exact and >= 0, so "S != 0" (serial:86) is d^2 > 0
            const T zfloor = (mode == KNN_MODE_INT) ? (T)0 : (T)-KNN_INF;
            unsigned pend_all = 0;
#pragma unroll
            for (int mt = 0; mt < 8; mt++)
#pragma unroll
                for (int r = 0; r < 4; r++)
                    pend_all |= (A[mt][r] <= lim) ? (1u << (4 * mt + r)) : 0u;
            if (masked) {
#pragma unroll
                for (int mt = 0; mt < 8; mt++)
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        const int row = row0 + 16 * mt + rowmap(g, r);
                        if (!(row < nc && (long)c_base + row != gq)) pend_all &= ~(1u << (4 * mt + r));
                    }
            }
            // one wave round per survivor of the busiest lane: each lane
            // takes its lowest pending candidate (= lowest row: the stable
            // tie order) through a 5-level select tree over the 32 d^2
            while (__ballot(pend_all != 0) != 0ull) {
                const int b = pend_all ? __builtin_ctz(pend_all) : 0;
                const bool b0 = b & 1, b1 = b & 2, b2 = b & 4, b3 = b & 8, b4 = b & 16;
                T v[8];
#pragma unroll
                for (int mt = 0; mt < 8; mt++) {
                    const T lo = b0 ? A[mt][1] : A[mt][0];
                    const T hi = b0 ? A[mt][3] : A[mt][2];
                    v[mt] = b1 ? hi : lo;
                }
                const T w0 = b2 ? v[1] : v[0], w1 = b2 ? v[3] : v[2];
                const T w2 = b2 ? v[5] : v[4], w3 = b2 ? v[7] : v[6];
                const T x0 = b3 ? w1 : w0, x1 = b3 ? w3 : w2;
                // d^2 <= zfloor (INT mode: an exact duplicate, S == 0) is
                // dropped here rather than in the survivor mask (rare)
                const T dsel = b4 ? x1 : x0;
                const T dd = (pend_all && dsel > zfloor) ? dsel : (T)KNN_INF;
                const int ii = (int)(c_base + row0 + 16 * (b >> 2) + rowmap(g, b & 3));
                pend_all &= pend_all - 1;
                list_insert<KL>(L, I, dd, ii);
            }
        }
#pragma unroll
        for (int mt = 0; mt < 8; mt++) A[mt] = (acc_t){0, 0, 0, 0};
        if (!any) return;
        // shared threshold of the query's 4 lanes: their union holds
        // >= 4(ujm+1) >= k+1 entries <= max_h L_h[ujm], and every lane
        // already rejects >= min_h L_h[KL-1]
        T lmin = L[KL - 1], u = L[0];
#pragma unroll
        for (int e = 1; e < KL; e++) u = (e == ujm) ? L[e] : u;
        lmin = fmin(lmin, __shfl_xor(lmin, 16));
        lmin = fmin(lmin, __shfl_xor(lmin, 32));
        u = fmax(u, __shfl_xor(u, 16));
        u = fmax(u, __shfl_xor(u, 32));
        thr = fmin(thr, fmin(lmin, u));   // monotone: rejections so far stay above it
    };

    // ---- fragments: quarter (p, h) = m-tiles 4h..4h+3 of piece p ---------
    auto cs_of = [&](int c) { return lds + (c & (NST - 1)) * 32768; };
    // 16-byte slot of (row, segment 4p+g) in a 16-row image
    const int fslot = j16 * 128 + 16 * ((4 * 0 + g) ^ (j16 & 7));
    const int fslot1 = j16 * 128 + 16 * ((4 * 1 + g) ^ (j16 & 7));
    frag_t f0[4], f1[4];
    frag_t b0, b1;
    auto rd = [&](LDS_AS char *st, int p, int h, frag_t (&f)[4], int j) {
        f[j] = *(const LDS_AS frag_t *)(st + (4 * h + j) * 2048 + (p ? fslot1 : fslot));
    };
    auto rdq = [&](LDS_AS char *st, int p) {
        return *(const LDS_AS frag_t *)(st + 16384 + wave * 2048 + (p ? fslot1 : fslot));
    };
    // one segment: 8 MFMAs on quarter h with fragments f and query piece b;
    // between them the reads `rdj(j)` of the next segment and one staging
    // load `stage()` (sched_barrier-pinned order)
    constexpr int SJ = 2;   // m-tile pair after which a segment's load issues
    // fp64: an m-tile's two k-steps back to back (measured 1.2% faster than
    // interleaving); fp32: v_mfma_f32_16x16x4 has a 40-cycle dependent
    // latency against a 32-cycle issue, so its 4 k-steps go round-robin
    // over the 4 m-tiles.
    constexpr bool PAIRS = ES == 8;
    auto segment = [&](const frag_t (&f)[4], const frag_t &b, int h, auto &&rdj, auto &&stage) {
        if constexpr (PAIRS) {
#pragma unroll
            for (int j = 0; j < 4; j++) {
                rdj(j);
                if (j == SJ) stage();
#pragma unroll
                for (int e = 0; e < KSF; e++) acc[4 * h + j] = KT<T>::mfma(f[j][e], b[e], acc[4 * h + j]);
                __builtin_amdgcn_sched_barrier(0);
            }
        } else {
#pragma unroll
            for (int j = 0; j < 4; j++) {
                acc[4 * h + j] = KT<T>::mfma(f[j][0], b[0], acc[4 * h + j]);
                rdj(j);
                if (j == SJ) stage();
                __builtin_amdgcn_sched_barrier(0);
            }
#pragma unroll
            for (int e = 1; e < KSF; e++)
#pragma unroll
                for (int j = 0; j < 4; j++) acc[4 * h + j] = KT<T>::mfma(f[j][e], b[e], acc[4 * h + j]);
            __builtin_amdgcn_sched_barrier(0);
        }
    };
    auto nothing = [&]() {};

    if (total > 0) {
        // prologue: norms of the first two tiles, chunks 0..2 whole and
        // chunk 3's load 0 (its loads 1..3 belong to S0..S2 of chunk 0)
        gnorm(t_lo, t_lo);
        gnorm(t_lo + 1, t_lo + 1);
#pragma unroll
        for (int x = 0; x < NST - 1; x++) {
#pragma unroll
            for (int i = 0; i < 4; i++) glds1(i);
            advance();
        }
        glds1(0);
        // norms + chunk 0 landed: younger are chunks 1, 2 and chunk 3's
        // load 0 -- 9 instructions per staged wave (18 for a loader of two)
        if constexpr (SELF) asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(18)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        b0 = rdq(cs_of(0), 0);
#pragma unroll
        for (int j = 0; j < 4; j++) rd(cs_of(0), 0, 0, f0, j);

        int c = 0;
        for (int t = t_lo; t < t_hi; t++) {
            gnorm(t + 2, t + 2);
            for (int fc = 0; fc < nfc; fc++, c++) {
                LDS_AS char *cs = cs_of(c);
                if constexpr (H16 == 2) {
                    // fp16 shadow rows: a 16-byte slot is a whole 8-half
                    // operand, two v_mfma_f32_16x16x32_f16 per m-tile per
                    // 64-feature chunk, no conversion.  fp64: fp32 partial
                    // sums flushed every 4 chunks (256 features, knn_to_h4)
                    glds1(1);
                    glds1(2);
                    glds1(3);
                    const knn_h8 q0 = *(const LDS_AS knn_h8 *)(cs + 16384 + wave * 2048 + fslot);
                    const knn_h8 q1 = *(const LDS_AS knn_h8 *)(cs + 16384 + wave * 2048 + fslot1);
#pragma unroll
                    for (int mt = 0; mt < 8; mt++) {
                        const knn_h8 a0 = *(const LDS_AS knn_h8 *)(cs + mt * 2048 + fslot);
                        const knn_h8 a1 = *(const LDS_AS knn_h8 *)(cs + mt * 2048 + fslot1);
                        if constexpr (H16D) {
                            acc32[mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0, q0, acc32[mt], 0, 0, 0);
                            acc32[mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1, q1, acc32[mt], 0, 0, 0);
                        } else {
                            acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0, q0, acc[mt], 0, 0, 0);
                            acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1, q1, acc[mt], 0, 0, 0);
                        }
                    }
                    if constexpr (H16D) {
                        if (++grp == 4) flush32();
                    }
                    advance();
                    __builtin_amdgcn_s_waitcnt(0xC07F);
                    if constexpr (SELF) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
                    else asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
                    __builtin_amdgcn_s_barrier();
                    glds1(0);
                    continue;
                }
                if constexpr (H16 == 1 && H16D) {
                    // fp16 MFMA on converted fp64 fragments (knn_to_h4); the
                    // output is in the fp32 layout (rowmap)
                    glds1(1);
                    glds1(2);
                    glds1(3);
                    const knn_h4 bh = knn_to_h4(rdq(cs, 0), rdq(cs, 1));
#pragma unroll
                    for (int mt = 0; mt < 8; mt++) {
                        const frag_t a0 = *(const LDS_AS frag_t *)(cs + mt * 2048 + fslot);
                        const frag_t a1 = *(const LDS_AS frag_t *)(cs + mt * 2048 + fslot1);
                        acc32[H16D ? mt : 0] = __builtin_amdgcn_mfma_f32_16x16x16f16(
                            knn_to_h4(a0, a1), bh, acc32[H16D ? mt : 0], 0, 0, 0);
                    }
                    if (++grp == 16) flush32();
                    advance();
                    __builtin_amdgcn_s_waitcnt(0xC07F);
                    if constexpr (SELF) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
                    else asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
                    __builtin_amdgcn_s_barrier();
                    glds1(0);
                    continue;
                }
                if constexpr (H16 == 1 && ES == 4) {
                    // fp16 MFMA on converted fp32 fragments (knn_to_h8): one
                    // 16x16x32 per m-tile per chunk.  Same staging sequence
                    // as below: loads 1..3 of chunk c+3, the chunk barrier,
                    // then load 0 of chunk c+4 into the freed stage.
                    glds1(1);
                    glds1(2);
                    glds1(3);
                    const knn_h8 bh = knn_to_h8(rdq(cs, 0), rdq(cs, 1));
#pragma unroll
                    for (int h = 0; h < 2; h++) {
#pragma unroll
                        for (int j = 0; j < 4; j++) {
                            rd(cs, 0, h, f0, j);
                            rd(cs, 1, h, f1, j);
                        }
#pragma unroll
                        for (int j = 0; j < 4; j++)
                            acc[4 * h + j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(
                                knn_to_h8(f0[j], f1[j]), bh, acc[4 * h + j], 0, 0, 0);
                    }
                    advance();
                    __builtin_amdgcn_s_waitcnt(0xC07F);
                    if constexpr (SELF) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
                    else asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
                    __builtin_amdgcn_s_barrier();
                    glds1(0);
                    continue;
                }
                // one staging load per segment, mid-segment: loads 1..3 of
                // chunk c+3 in S0..S2, load 0 of chunk c+4 in S3 (after the
                // barrier that freed its stage).  All 8 waves issuing right
                // after the barrier cost 4% (measured); spread, ~1%.
                // S0: (p0, mt0-3) on f0 || read (p0, mt4-7) into f1
                segment(f0, b0, 0, [&](int j) { rd(cs, 0, 1, f1, j); }, [&]() { glds1(1); });
                // S1: (p0, mt4-7) on f1 || read (p1, mt0-3) + B p1
                b1 = rdq(cs, 1);
                segment(f1, b0, 1, [&](int j) { rd(cs, 1, 0, f0, j); }, [&]() { glds1(2); });
                // S2: (p1, mt0-3) on f0 || read (p1, mt4-7) into f1
                segment(f0, b1, 0, [&](int j) { rd(cs, 1, 1, f1, j); }, [&]() { glds1(3); });
                advance();
                {
                    __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): this stage's reads done
                    // chunk c+1 landed: chunks c+2, c+3 may stay in flight
                    if constexpr (SELF) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
                    else asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
                    __builtin_amdgcn_s_barrier();         // chunk c+1 visible; stage c%4 free
                }
                LDS_AS char *cs1 = cs_of(c + 1);
                b0 = rdq(cs1, 0);
                // S3: (p1, mt4-7) on f1 || read (p0, mt0-3) of chunk c+1
                segment(f1, b1, 1, [&](int j) { rd(cs1, 0, 0, f0, j); }, [&]() { glds1(0); });
            }
            flush32();
            epilogue(t, acc);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");     // no LDS-DMA left in flight
    }

    // INT mode, exact d^2: if no lane's list ends at thr, nothing equal to
    // thr was ever turned away (the filter rejects only d^2 > thr, and a
    // full list only what ranks after its last entry), so every rejected
    // candidate has d^2 >= next(thr).  Publishing that lets the certificate
    // accept a k-th entry equal to thr -- on integer data with the top k
    // split evenly over the 4 lanes, thr IS the k-th value.
    T lastmin = L[KL - 1];
    lastmin = fmin(lastmin, __shfl_xor(lastmin, 16));
    lastmin = fmin(lastmin, __shfl_xor(lastmin, 32));
    T pub = thr;
    if (mode == KNN_MODE_INT && lastmin > thr && thr < (T)KNN_INF) pub = nextafter(thr, (T)KNN_INF);
    if (myq < nq) {
        const size_t base = (((size_t)split * nq_pad + myq) * 4 + g) * KL;
#pragma unroll
        for (int e = 0; e < KL; e++) {
            part_d[base + e] = (double)L[e];
            part_i[base + e] = I[e];
        }
        if (g == 0) {
            part_T[(size_t)split * nq_pad + myq] = (double)pub;
            if (qthr != nullptr && thr < (T)KNN_INF)
                atomicMin(qthr + myq, (unsigned long long)__double_as_longlong((double)thr));
        }
    }
}

// One step of a DPP argmin by (d, idx): lanes the row/bank masks leave out,
// and lanes whose source lies outside their row, see (+inf, INT_MAX)
template <int CTRL, int RM, int BM>
__device__ __forceinline__ void dpp_argmin_step(double &d, int &i)
{
    const int lo = __double2loint(d), hi = __double2hiint(d);
    const int olo = __builtin_amdgcn_update_dpp(0, lo, CTRL, RM, BM, false);
    const int ohi = __builtin_amdgcn_update_dpp(0x7ff00000, hi, CTRL, RM, BM, false);
    const int oi = __builtin_amdgcn_update_dpp(0x7fffffff, i, CTRL, RM, BM, false);
    const double od = __hiloint2double(ohi, olo);
    const bool take = (od < d) || (od == d && oi < i);
    d = take ? od : d;
    i = take ? oi : i;
}
// the same on packed (d^2 << 32 | idx) keys (INT mode with d^2 < 2^32)
template <int CTRL, int RM, int BM>
__device__ __forceinline__ void dpp_min_u64_step(unsigned long long &key)
{
    const unsigned lo = (unsigned)key, hi = (unsigned)(key >> 32);
    const unsigned olo = (unsigned)__builtin_amdgcn_update_dpp(-1, (int)lo, CTRL, RM, BM, false);
    const unsigned ohi = (unsigned)__builtin_amdgcn_update_dpp(-1, (int)hi, CTRL, RM, BM, false);
    const unsigned long long ok = ((unsigned long long)ohi << 32) | olo;
    key = ok < key ? ok : key;
}
__device__ __forceinline__ double readlane_f64(double v, int l)
{
    return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), l),
                            __builtin_amdgcn_readlane(__double2loint(v), l));
}

// ---------------------------------------------------------------------------
// k_merge: one wave per query.  Lane j < lpq*nsplit owns partial list j
// (lpq lists per query and split: 4 from k_dist_topk, 2 from k_dist_topk_i8),
// lane lpq*nsplit the running state; KP+1 rounds of a wave argmin over the
// heads select the new state (KP entries by (d^2, idx)) and the smallest
// dropped value, which lowers the rejection bound T.  GEMM mode: entries
// new in this step get their exact reference-order S from the resident
// block (the only step at which their rows are on this device).
// ---------------------------------------------------------------------------
// PF > 0: each lane's next PF entries are loaded up front, unconditionally
// (lanes without a list read a +inf list), and shifted as its head is taken;
// the running state is split over KP / PF lanes (sorted runs of PF), so a
// lane only goes back to memory after PF wins.  PF = 0: the head is loaded
// as it is consumed (one memory latency on every one of the KP + 1 rounds).
__device__ const double k_inf_d[8] = {KNN_INF, KNN_INF, KNN_INF, KNN_INF, KNN_INF, KNN_INF, KNN_INF, KNN_INF};
__device__ const int k_inf_i[8] = {0x7fffffff, 0x7fffffff, 0x7fffffff, 0x7fffffff,
                                   0x7fffffff, 0x7fffffff, 0x7fffffff, 0x7fffffff};
template <typename TE, int KP, int S, int PF = 0>
__global__ __launch_bounds__(256) void k_merge(
    const double *__restrict__ part_d, const int *__restrict__ part_i,
    const double *__restrict__ part_T, int nsplit, int lpq, int kl, int nq, int nq_pad, int first_step,
    double *__restrict__ st_d, double *__restrict__ st_x, int *__restrict__ st_i,
    double *__restrict__ st_T, const TE *__restrict__ qblk, size_t qnorm_off,
    const knn_merge_blocks_t mb, int n, int n_pad,
    const double *__restrict__ meta, int k, unsigned long long *__restrict__ qthr, int filt,
    const int *__restrict__ qperm)
{
    // S lanes a query (64, or 32 when nl + 1 <= 32: two queries a wave, so
    // twice the independent argmin chains a SIMD interleaves -- the merge is
    // bound by the latency of its KP + 1 dependent rounds, not by issue)
    constexpr int QPW = 64 / S;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int seg = lane / S, sl = lane - seg * S;
    const int q0 = (blockIdx.x * 4 + wave) * QPW;
    if (q0 >= nq) return;
    // qperm (knn_order.hip): the wave's queries in a cache-friendly order
    const int qi = q0 + seg;
    const bool qv = qi < nq;
    const int q = (qperm != nullptr && qv) ? qperm[qi] : qi;
    const unsigned long long segm = (S == 64) ? ~0ull : (0xffffffffull << (32 * seg));
    const int mode = knn_mode<TE>(meta, n);
    const int nl = lpq * nsplit;   // partial lists: [split][query][lpq][kl]

    static_assert(PF == 0 || (PF == 8 && KP % PF == 0), "prefetch depth");
    constexpr int NST = PF > 0 ? KP / PF : 1;   // state lanes
    const double *src_d = nullptr;
    const int *src_i = nullptr;
    int len = KP, opos0 = 0;   // opos0: the lane's first slot in the old state
    if (qv && sl < nl) {
        const int s = sl / lpq, gg = sl - s * lpq;
        const size_t base = (((size_t)s * nq_pad + q) * lpq + gg) * kl;
        src_d = part_d + base;
        src_i = part_i + base;
        len = kl;
    } else if (qv && !first_step && sl >= nl && sl < nl + NST) {
        opos0 = (sl - nl) * (KP / NST);
        src_d = st_d + (size_t)q * KP + opos0;
        src_i = st_i + (size_t)q * KP + opos0;
        len = KP / NST;
    }
    int pos = 0;
    constexpr int R = PF > 0 ? PF : 1;
    double Ld[R];
    int Li[R];
    double hd;
    int hi;
    if constexpr (PF > 0) {
        if (!src_d) {
            src_d = k_inf_d;
            src_i = k_inf_i;
            len = 0;
        }
#pragma unroll
        for (int j = 0; j < R; j++) {   // unconditional: one latency for all
            Ld[j] = src_d[j];
            Li[j] = src_i[j];
        }
#pragma unroll
        for (int j = 0; j < R; j++) Ld[j] = j < len ? Ld[j] : KNN_INF;
        hd = Ld[0];
        hi = hd == KNN_INF ? 0x7fffffff : Li[0];
    } else {
        hd = src_d ? src_d[0] : KNN_INF;
        hi = src_d ? src_i[0] : 0x7fffffff;
        if (hd == KNN_INF) hi = 0x7fffffff;
    }

    // T: rejection bound of the lane filters (every candidate a lane turned
    // away has d^2 >= T); Td: smallest d^2 dropped by a merge (those rank
    // after every kept entry by (d^2, idx), so only the GEMM certificate
    // needs them).
    double T = KNN_INF, Td = KNN_INF;
    if (qv && sl < nsplit) T = part_T[(size_t)sl * nq_pad + q];
    if (qv && sl == nl && !first_step) { T = st_T[2 * (size_t)q]; Td = st_T[2 * (size_t)q + 1]; }
    for (int off = S / 2; off > 0; off >>= 1) {
        T = fmin(T, __shfl_xor(T, off));
        Td = fmin(Td, __shfl_xor(Td, off));
    }

    // state slot r (0..KP-1) is kept by segment lane r % S in register r / S
    constexpr int NS = (KP + S - 1) / S;
    double sd[NS];
    int si[NS], ssrc[NS], spos[NS];
#pragma unroll
    for (int x = 0; x < NS; x++) { sd[x] = KNN_INF; si[x] = -1; ssrc[x] = 0; spos[x] = 0; }
    // INT mode: the state only needs the k + 1 smallest (exact keys, zeros
    // never admitted: k_finalize reads the k-th, the publication below the
    // (k+1)-th, and a later merge's top k + 1 comes from these and its new
    // lists); Td, the smallest dropped value, is a GEMM-certificate term
    const int rmax = (mode == KNN_MODE_INT && k + 1 < KP) ? k : KP;
    // INT mode with every d^2 below 2^32 ((|q| + |c|)^2 <= 4 max|x|^2 <
    // 2^32; list keys are exact integers, idx >= 0): argmin on packed keys
    const bool small_keys = mode == KNN_MODE_INT && 4.0 * meta[KNN_META_MAXNORM] < 4294967295.0;
    // GEMM mode: selection stops once the head passes the exact-S window of
    // the k-th kept entry (dk + 2E, below): such an entry can never reach
    // the top k, now or after a later merge (d^2_k only falls), so it is
    // dropped with everything behind it and the head becomes Td, the
    // smallest dropped value -- a query takes ~k + 1 rounds instead of
    // KP + 1, and only a query whose near ties crowd the window fills the
    // state.  dkc = the (k + z)-th selected entry, z = those <= E (d^2 <= E:
    // possibly S == 0, excluded results), as the window below.
    const bool gstop = mode == KNN_MODE_GEMM && qblk != nullptr;
    const double Eq = (gstop && qv) ? knn_cert_E<TE>(n, (double)qblk[qnorm_off + q], meta[KNN_META_MAXNORM],
                                                     filt, meta[KNN_META_MAXABS])
                                    : 0.0;
    int nsel = 0, nzs = 0;
    double dkc = KNN_INF;
    bool done = false;
    for (int r = 0; r <= rmax; r++) {
        // segment argmin of the heads by (d^2, idx): DPP row shifts (the
        // minimum of each 16-lane row in its lane 15), row broadcasts into
        // the segment's last lane, read back as scalars -- no LDS permutes
        double wd = hd;
        int wi = hi;
        if (small_keys) {
            // one 64-bit key per head: (d^2, idx) order is u64 order
            unsigned long long key = hd == KNN_INF ? ~0ull
                                                   : ((unsigned long long)(unsigned)hd << 32) | (unsigned)hi;
            dpp_min_u64_step<0x111, 0xf, 0xf>(key);
            dpp_min_u64_step<0x112, 0xf, 0xf>(key);
            dpp_min_u64_step<0x114, 0xf, 0xf>(key);
            dpp_min_u64_step<0x118, 0xf, 0xf>(key);
            dpp_min_u64_step<0x142, 0xa, 0xf>(key);
            if constexpr (S == 64) dpp_min_u64_step<0x143, 0xc, 0xf>(key);
            wd = key == ~0ull ? KNN_INF : (double)(unsigned)(key >> 32);
            wi = key == ~0ull ? 0x7fffffff : (int)(unsigned)key;
        } else {
            dpp_argmin_step<0x111, 0xf, 0xf>(wd, wi);   // row_shr:1
            dpp_argmin_step<0x112, 0xf, 0xf>(wd, wi);   // row_shr:2
            dpp_argmin_step<0x114, 0xf, 0xf>(wd, wi);   // row_shr:4
            dpp_argmin_step<0x118, 0xf, 0xf>(wd, wi);   // row_shr:8
            dpp_argmin_step<0x142, 0xa, 0xf>(wd, wi);   // row_bcast:15 -> rows 1, 3
            if constexpr (S == 64) dpp_argmin_step<0x143, 0xc, 0xf>(wd, wi);   // row_bcast:31 -> rows 2, 3
        }
        {
            const double d1 = readlane_f64(wd, 63);
            const int i1 = __builtin_amdgcn_readlane(wi, 63);
            if constexpr (S == 32) {
                const double d0 = readlane_f64(wd, 31);
                const int i0 = __builtin_amdgcn_readlane(wi, 31);
                wd = seg ? d1 : d0;
                wi = seg ? i1 : i0;
            } else {
                wd = d1;
                wi = i1;
            }
        }
        if (gstop && !done && dkc < KNN_INF && wd != KNN_INF &&
            wd > (dkc + 2.0 * Eq) * (1.0 + 1.0 / 524288.0)) {
            Td = fmin(Td, wd);   // every later head is >= wd
            done = true;
        }
        const bool live = wd != KNN_INF && !done;   // this query still has heads
        if (__ballot(live) == 0ull) break;
        const unsigned long long wall = __ballot(live && hd == wd && hi == wi);
        const unsigned long long who = wall & segm;
        const int wl = who ? __builtin_ctzll(who) : lane;   // wave lane of the winner
        int wpos;
        if constexpr (S == 32) {
            const unsigned w0 = (unsigned)wall, w1 = (unsigned)(wall >> 32);
            const int p0 = __builtin_amdgcn_readlane(pos, w0 ? __builtin_ctz(w0) : 0);
            const int p1 = __builtin_amdgcn_readlane(pos, w1 ? 32 + __builtin_ctz(w1) : 32);
            wpos = seg ? p1 : p0;
        } else {
            wpos = __builtin_amdgcn_readlane(pos, wall ? __builtin_ctzll(wall) : 0);
        }
        if constexpr (PF > 0) wpos += __shfl(opos0, wl);   // state runs: slot in the old state
        if (live) {
            if (r < KP) {
                nsel++;
                if (wd <= Eq) nzs++;
                else if (nsel - nzs == k) dkc = wd;
                if (sl == r % S) {
#pragma unroll
                    for (int x = 0; x < NS; x++) {
                        if (r / S == x) {
                            sd[x] = wd;
                            si[x] = wi;
                            ssrc[x] = (wl - seg * S >= nl && !first_step) ? 1 : 0;
                            spos[x] = wpos;
                        }
                    }
                }
            } else {
                Td = fmin(Td, wd);
            }
            if (lane == wl) {
                pos++;
                if constexpr (PF > 0) {
#pragma unroll
                    for (int j = 0; j + 1 < R; j++) {
                        Ld[j] = Ld[j + 1];
                        Li[j] = Li[j + 1];
                    }
                    Ld[R - 1] = KNN_INF;
                    if (pos % R == 0 && pos < len) {   // the prefetched run is used up (rare)
#pragma unroll
                        for (int j = 0; j < R; j++) {
                            const int pj = pos + j < len ? pos + j : len - 1;
                            Ld[j] = pos + j < len ? src_d[pj] : KNN_INF;
                            Li[j] = src_i[pj];
                        }
                    }
                    hd = Ld[0];
                    hi = hd == KNN_INF ? 0x7fffffff : Li[0];
                } else {
                    hd = (pos < len) ? src_d[pos] : KNN_INF;
                    hi = (pos < len) ? src_i[pos] : 0x7fffffff;
                    if (hd == KNN_INF) hi = 0x7fffffff;
                }
            }
        }
    }

    // INT mode (exact d^2): the new state's (k+1)-th nonzero entry bounds
    // the query's (k+1)-th candidate over all rows (k+1 distinct rows lie at
    // or below it) -- the distance kernels' qthr contract.  Published, it
    // lets every later ring step filter with the running answer instead of
    // the bound one split's lane lists reach (about the 32nd of that split's
    // rows).  fp32 blocks: rounded up to an fp32 value, as the kernels read
    // it back in fp32.
    if (qthr != nullptr && mode == KNN_MODE_INT) {
        int z = 0;
#pragma unroll
        for (int x = 0; x < NS; x++) z += __popcll(__ballot(sl + S * x < KP && sd[x] == 0.0) & segm);
        const int rk = k + z;
        if (rk < KP) {
            double u = KNN_INF;
#pragma unroll
            for (int x = 0; x < NS; x++) {
                const double v = __shfl(sd[x], seg * S + rk % S);
                if (rk / S == x) u = v;
            }
            if constexpr (sizeof(TE) == 4) u = (double)__double2float_ru(u);
            if (qv && sl == 0 && u < KNN_INF)
                atomicMin(qthr + q, (unsigned long long)__double_as_longlong(u));
        }
    }

    // GEMM mode: exact S of the new entries, from the resident block.  Let
    // z = the entries with d^2 <= E (possibly S == 0: excluded results) and
    // d^2_k the (k+z)-th d^2 of the new state.  An entry with d^2 > d^2_k +
    // 2E has S > d^2_k + E >= the k-th smallest nonzero S of the state, now
    // and after any later merge (d^2_k only falls), so it can never reach
    // the top k: its S is skipped and marked +inf (k_finalize ignores it).
    // A context begun from a byte block alone (knn_ctx_begin_s8) holds no
    // element rows: if the device meta says GEMM after all (a speculative
    // begin on data that did not qualify), no exact S is computed -- the new
    // entries get S = +inf and k_finalize fails every query (it sees no
    // query norms either) instead of reading through a null block
    const bool exact_ok = mode == KNN_MODE_GEMM && qblk != nullptr;
    double win = KNN_INF;
    if (exact_ok) {
        const double E = qv ? knn_cert_E<TE>(n, (double)qblk[qnorm_off + q], meta[KNN_META_MAXNORM], filt,
                                             meta[KNN_META_MAXABS])
                            : 0.0;
        int z = 0;
#pragma unroll
        for (int x = 0; x < NS; x++) z += __popcll(__ballot(sl + S * x < KP && sd[x] <= E) & segm);
        const int rk = k - 1 + z;
        double dk = KNN_INF;
        if (rk < KP) {
#pragma unroll
            for (int x = 0; x < NS; x++) {
                const double v = __shfl(sd[x], seg * S + rk % S);
                if (rk / S == x) dk = v;
            }
        }
        if (dk < KNN_INF) win = (dk + 2.0 * E) * (1.0 + 1.0 / 1048576.0);
    }
    double sx[NS];
#pragma unroll
    for (int x = 0; x < NS; x++) {
        sx[x] = sd[x];
        if (qv && sl + S * x < KP && mode == KNN_MODE_GEMM && si[x] >= 0) {
            if (ssrc[x]) {
                sx[x] = st_x[(size_t)q * KP + spos[x]];
            } else if (exact_ok && sd[x] <= win) {
                // the row's block (new entries come from this step's blocks)
                const TE *crow = (const TE *)mb.ptr[0];
                long row = 0;
#pragma unroll
                for (int j = 0; j < KNN_SPLIT_MAXBLK; j++)
                    if (j < mb.nblk && (long)si[x] >= mb.base[j] && (long)si[x] < mb.base[j] + mb.nc[j]) {
                        crow = (const TE *)mb.ptr[j];
                        row = (long)si[x] - mb.base[j];
                    }
                sx[x] = knn_exact_sq_v<TE>(qblk + (size_t)q * n_pad, crow + (size_t)row * n_pad, n_pad);
            } else {
                sx[x] = KNN_INF;
            }
        }
    }
    // every read of the old state (any lane, any slot) completes before the
    // first write (wave-private queries)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (qv) {
#pragma unroll
        for (int x = 0; x < NS; x++) {
            const int r = sl + S * x;
            if (r < KP) {
                st_d[(size_t)q * KP + r] = sd[x];
                st_x[(size_t)q * KP + r] = sx[x];
                st_i[(size_t)q * KP + r] = (sd[x] == KNN_INF) ? -1 : si[x];
            }
        }
        if (sl == 0) { st_T[2 * (size_t)q] = T; st_T[2 * (size_t)q + 1] = Td; }
    }
}

// ---------------------------------------------------------------------------
// k_merge_rank: the INT-mode merge of int8 lane lists (k_dist_topk_i8: exact
// integer d^2 < 2^31, zeros never admitted) by ranking instead of argmin
// rounds.  One wave per query.  The shared bound qthr[q] is an upper bound on
// the query's (k+1)-th smallest d^2 over all rows (k + 1 distinct rows lie at
// or below it), so no entry above it can be among the k + 1 smallest; the
// (k+1)-th smallest key among the lists' first entries and the state is a
// second such bound, usually far tighter.  Every list entry and state entry
// at or below both is compacted into LDS as a u64 key (d^2 << 32 | idx: u64
// order is the reference's (d, idx) order; keys are distinct),
// each candidate's rank is the number of smaller keys, and rank r < k + 1
// goes to state slot r.  The rank of a candidate costs C compares a lane
// (C candidates, ~31..60 at the end of a search);
// k_merge's k + 1 dependent wave-argmin rounds cost ~2k cycles each in
// latency (rocprofv3: 33 us for 7500 queries, 0.19 ms for 60000).
// State, T, Td and the publication as k_merge's INT mode (the (k+1)-th of
// the merged entries is published into qthr).
// ---------------------------------------------------------------------------
typedef unsigned long long knn_u64x2 __attribute__((ext_vector_type(2)));
// fin != 0 (the search's last merge, knn_ctx_end): k_finalize's INT-mode
// work in the same pass -- certify tau_k < T, emit the k records or put the
// query on the rescan list -- instead of writing the state.
struct knn_fin_args {
    knn_neighbour_t *out;
    int *fail_count, *fail_list, *mode_out;
    double *fbound;
    const double *meta;
    double lim;   // 2^51 / 4n, knn_mode_lim
    int n, force_fail;
};
template <typename TE, int KP, int KL>
__global__ __launch_bounds__(256) void k_merge_rank(
    const double *__restrict__ part_d, const int *__restrict__ part_i, const double *__restrict__ part_T,
    int nsplit, int lpq, int nq, int nq_pad, int first_step, double *__restrict__ st_d,
    double *__restrict__ st_x, int *__restrict__ st_i, double *__restrict__ st_T, int k,
    unsigned long long *__restrict__ qthr, int cap, int fin, knn_fin_args fa)
{
    extern __shared__ __attribute__((aligned(16))) unsigned long long mr_buf[];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int q = blockIdx.x * 4 + wave;
    if (q >= nq) return;   // wave-uniform, and no workgroup barrier below
    LDS_AS unsigned long long *buf = (LDS_AS unsigned long long *)mr_buf + (size_t)wave * cap;
    const int nl = lpq * nsplit;
    // any value read is a valid bound (it only falls); floor: d^2 are integers
    const double qb = __longlong_as_double((long long)qthr[q]);
    const double B = qb >= 4294967294.0 ? 4294967294.0 : floor(qb);
    const unsigned Bu = (unsigned)B;
    // T: the smallest rejection bound of the merged lanes (and the state);
    // read with the lists (one round of loads), reduced below
    double T = KNN_INF, Td = KNN_INF;
    if (lane < nsplit) T = part_T[(size_t)lane * nq_pad + q];
    if (!first_step && lane == 63) {
        T = fmin(T, st_T[2 * (size_t)q]);
        Td = st_T[2 * (size_t)q + 1];
    }
    const int mode = fin ? knn_mode_lim<TE>(fa.meta, fa.n, fa.lim) : KNN_MODE_INT;
    // list entries as 32-bit d^2 (exact integers < 2^31; +inf -> 0xffffffff,
    // above every bound): half the registers of doubles, 5 -> 6 waves a SIMD
    constexpr unsigned DINF = 0xffffffffu;
    unsigned d[KL];
    int id[KL];
#pragma unroll
    for (int e = 0; e < KL; e++) {
        d[e] = DINF;
        id[e] = 0;
    }
    int c = 0;
    if (lane < nl) {
        const int s = lpq == 2 ? lane >> 1 : lpq == 4 ? lane >> 2 : lane / lpq, g = lane - s * lpq;
        const size_t base = (((size_t)s * nq_pad + q) * lpq + g) * KL;
        // the list is sorted: its first 4 entries, then the rest in one
        // round if the 4th is still at or below the bound (two dependent
        // rounds at most: the merge is latency-bound, one wave a query)
#pragma unroll
        for (int e = 0; e < 4 && e < KL; e++) {
            const double v = part_d[base + e];
            d[e] = v < 4294967295.0 ? (unsigned)v : DINF;
            id[e] = part_i[base + e];
        }
        if (KL > 4 && d[3] <= Bu) {
#pragma unroll
            for (int e = 4; e < KL; e++) {
                const double v = part_d[base + e];
                d[e] = v < 4294967295.0 ? (unsigned)v : DINF;
                id[e] = part_i[base + e];
            }
        }
#pragma unroll
        for (int e = 0; e < KL; e++) c += d[e] <= Bu ? 1 : 0;   // a prefix (+inf past the end)
    }
    double sdv = KNN_INF;
    int siv = -1, cs = 0;
    if (!first_step && lane < KP) {
        sdv = st_d[(size_t)q * KP + lane];
        siv = st_i[(size_t)q * KP + lane];
        cs = (siv >= 0 && sdv <= B) ? 1 : 0;
    }
    // A tighter bound first: the (k+1)-th smallest key among the first HD
    // entries of every list and the state entries.  It is at or above the
    // (k+1)-th smallest key of all the entries (a subset's (k+1)-th is never
    // below the whole set's), so the entries at or below it still hold the
    // k + 1 smallest.  The shared bound B alone admitted ~100-170 entries a
    // query at P = 1 (7 splits x 2 lists x 12), and the rank loop's
    // broadcast LDS reads grow with C^2 / 64: 89 us a merge of 60000
    // queries, nearly all of it those reads (rocprofv3, round 6).
    unsigned long long lim = ~0ull;
#ifndef KNN_MR_NOTIGHT
    {
        constexpr int HD = KL < 4 ? KL : 4;
        const int hh = c < HD ? c : HD;    // lists are sorted: a prefix
        const int chh = hh + cs;
        int preh = 0, CH = 0;
#pragma unroll
        for (int b = 0; b < 5; b++) {
            const unsigned long long m = __ballot((chh >> b) & 1);
            preh += (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u)) << b;
            CH += __popcll(m) << b;
        }
        if (CH > k) {
#pragma unroll
            for (int e = 0; e < HD; e++)
                if (e < hh) buf[preh + e] = ((unsigned long long)d[e] << 32) | (unsigned)id[e];
            if (cs) buf[preh + hh] = ((unsigned long long)(unsigned)sdv << 32) | (unsigned)siv;
            __builtin_amdgcn_wave_barrier();
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            unsigned long long bk = ~0ull;
            for (int b0 = 0; b0 < CH; b0 += 64) {
                const int my = b0 + lane;
                const unsigned long long x = my < CH ? buf[my] : ~0ull;
                int r = 0, j = 0;
                for (; j + 4 <= CH; j += 4) {
                    const knn_u64x2 u = *(const LDS_AS knn_u64x2 *)(buf + j);
                    const knn_u64x2 w = *(const LDS_AS knn_u64x2 *)(buf + j + 2);
                    r += (u.x < x ? 1 : 0) + (u.y < x ? 1 : 0) + (w.x < x ? 1 : 0) + (w.y < x ? 1 : 0);
                }
                for (; j < CH; j++) r += buf[j] < x ? 1 : 0;
                const unsigned long long at = __ballot(my < CH && r == k);
                if (at) bk = __shfl(x, __builtin_ctzll(at));
            }
            // keep the entries at or below it (the lists are sorted by d, so
            // a prefix up to ties; counted and written entry by entry below)
            lim = bk;
            int c2 = 0;
#pragma unroll
            for (int e = 0; e < KL; e++)
                c2 += (e < c && (((unsigned long long)d[e] << 32) | (unsigned)id[e]) <= bk) ? 1 : 0;
            c = c2;
            if (cs && (((unsigned long long)(unsigned)sdv << 32) | (unsigned)siv) > bk) cs = 0;
            __builtin_amdgcn_wave_barrier();   // (the subset's slots are overwritten below)
        }
    }
#endif
    // exclusive prefix of the per-lane counts (<= KL + 1 < 32): bit-sliced
    // through mbcnt
    const int ct = c + cs;
    int pre = 0, C = 0;
#pragma unroll
    for (int b = 0; b < 5; b++) {
        const unsigned long long m = __ballot((ct >> b) & 1);
        pre += (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u)) << b;
        C += __popcll(m) << b;
    }
    {
        int w = pre;
#pragma unroll
        for (int e = 0; e < KL; e++) {
            const unsigned long long key = ((unsigned long long)d[e] << 32) | (unsigned)id[e];
            if (d[e] <= Bu && key <= lim) buf[w++] = key;
        }
    }
    if (cs) buf[pre + c] = ((unsigned long long)(unsigned)sdv << 32) | (unsigned)siv;
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");

    const int kk = k + 1 < KP ? k + 1 : KP;   // entries the state keeps
    for (int off = 32; off > 0; off >>= 1) {
        T = fmin(T, __shfl_xor(T, off));
        Td = fmin(Td, __shfl_xor(Td, off));
    }
    // fin: the records are written as the ranks come out; the query is
    // certified (or put on the rescan list, whose pass rewrites them) after
    const bool emit = fin != 0;
    if (fin) {
        if (blockIdx.x == 0 && threadIdx.x == 0) *fa.mode_out = mode;
        // slots past the candidates: {inf, 0, 0}
        if (lane < k && lane >= C) {
            knn_neighbour_t rec;
            rec.distance = KNN_INF;
            rec.idx = 0;
            rec.label = 0;
            fa.out[(size_t)q * k + lane] = rec;
        }
    }
    double tau = KNN_INF;   // fin: the k-th kept d^2
    double tk1 = KNN_INF;   // fin: the (k+1)-th, the seed of an uncertified query's re-search
    for (int b0 = 0; b0 < C; b0 += 64) {
        const int my = b0 + lane;
        const unsigned long long x = my < C ? buf[my] : ~0ull;
        int r = 0, j = 0;
        for (; j + 4 <= C; j += 4) {   // broadcast reads, 2 keys each
            const knn_u64x2 a = *(const LDS_AS knn_u64x2 *)(buf + j);
            const knn_u64x2 b = *(const LDS_AS knn_u64x2 *)(buf + j + 2);
            r += (a.x < x ? 1 : 0) + (a.y < x ? 1 : 0) + (b.x < x ? 1 : 0) + (b.y < x ? 1 : 0);
        }
        for (; j < C; j++) r += buf[j] < x ? 1 : 0;
        if (my < C) {
            const double dv = (double)(unsigned)(x >> 32);
            if (emit) {
                if (r < k) {
                    knn_neighbour_t rec;
                    rec.distance = sqrt(dv);
                    rec.idx = (int)(unsigned)x + 1;
                    rec.label = 0;
                    fa.out[(size_t)q * k + r] = rec;
                }
            } else if (r < kk) {
                st_d[(size_t)q * KP + r] = dv;
                st_x[(size_t)q * KP + r] = dv;
                st_i[(size_t)q * KP + r] = (int)(unsigned)x;
            }
            if (r == k && !emit) {   // the (k+1)-th: a bound on the query's (k+1)-th over all rows
                double u = dv;
                if constexpr (sizeof(TE) == 4) u = (double)__double2float_ru(u);
                atomicMin(qthr + q, (unsigned long long)__double_as_longlong(u));
            }
        }
        if (emit) {
            const unsigned long long at = __ballot(my < C && r == k - 1);
            if (at) tau = (double)(unsigned)(__shfl(x, __builtin_ctzll(at)) >> 32);
            const unsigned long long a1 = __ballot(my < C && r == k);
            if (a1) tk1 = (double)(unsigned)(__shfl(x, __builtin_ctzll(a1)) >> 32);
        }
    }
    if (emit) {
        // k_finalize, INT mode: zeros were never admitted, so the rank-(k-1)
        // candidate is tau; a candidate a lane turned away has d^2 >= T, and
        // with d^2 == T it may precede the k-th by index: certify tau < T
        const bool ok = mode == KNN_MODE_INT && !fa.force_fail && (T == KNN_INF || (C >= k && tau < T));
        if (!ok && C < k + 1 && mode == KNN_MODE_INT && !fa.force_fail) {
            // fewer than k + 1 entries under the shared bound: the k-th and
            // (k+1)-th over every entry of the lists and the state -- still
            // bounds on the query's k-th / (k+1)-th over all rows, which the
            // rescan (fbound) and the int8 re-search (qthr) start from; with
            // +inf instead they scanned cold (2.8 ms of k_rescan_step for two
            // MNIST queries)
            int c2 = 0;
            if (lane < nl) {
                const int s = lpq == 2 ? lane >> 1 : lpq == 4 ? lane >> 2 : lane / lpq, g = lane - s * lpq;
                const size_t base = (((size_t)s * nq_pad + q) * lpq + g) * KL;
#pragma unroll
                for (int e = 0; e < KL; e++) {
                    const double v = part_d[base + e];
                    d[e] = v < 4294967295.0 ? (unsigned)v : DINF;
                    id[e] = part_i[base + e];
                    c2 += d[e] != DINF ? 1 : 0;   // a prefix
                }
            }
            const int cs2 = (!first_step && lane < KP && siv >= 0 && sdv < KNN_INF) ? 1 : 0;
            const int ct2 = c2 + cs2;
            int pre2 = 0, C2 = 0;
#pragma unroll
            for (int b = 0; b < 5; b++) {
                const unsigned long long m = __ballot((ct2 >> b) & 1);
                pre2 += (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u)) << b;
                C2 += __popcll(m) << b;
            }
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int e = 0; e < KL; e++)
                if (e < c2) buf[pre2 + e] = ((unsigned long long)d[e] << 32) | (unsigned)id[e];
            if (cs2) buf[pre2 + c2] = ((unsigned long long)(unsigned)sdv << 32) | (unsigned)siv;
            __builtin_amdgcn_wave_barrier();
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            for (int b0 = 0; b0 < C2; b0 += 64) {
                const int my = b0 + lane;
                const unsigned long long x = my < C2 ? buf[my] : ~0ull;
                int r = 0;
                for (int j = 0; j < C2; j++) r += buf[j] < x ? 1 : 0;
                const unsigned long long a0 = __ballot(my < C2 && r == k - 1);
                if (a0) tau = (double)(unsigned)(__shfl(x, __builtin_ctzll(a0)) >> 32);
                const unsigned long long a1 = __ballot(my < C2 && r == k);
                if (a1) tk1 = (double)(unsigned)(__shfl(x, __builtin_ctzll(a1)) >> 32);
            }
        }
        if (!ok && lane == 0) {
            fa.fail_list[atomicAdd(fa.fail_count, 1)] = q;
            fa.fbound[q] = (fa.force_fail || mode != KNN_MODE_INT) ? KNN_INF : sqrt(tau);
            // k + 1 distinct rows lie at or below the (k+1)-th kept key: a
            // valid bound for the int8 re-search to start from (knn_engine.c
            // research8; INT mode only, the search is over)
            if (mode == KNN_MODE_INT && !fa.force_fail)
                qthr[q] = (unsigned long long)__double_as_longlong(sizeof(TE) == 4 ? (double)__double2float_ru(tk1) : tk1);
        }
        return;
    }
    if (lane < KP && lane >= (C < kk ? C : kk)) {
        st_d[(size_t)q * KP + lane] = KNN_INF;
        st_x[(size_t)q * KP + lane] = KNN_INF;
        st_i[(size_t)q * KP + lane] = -1;
    }
    if (lane == 0) {
        st_T[2 * (size_t)q] = T;
        st_T[2 * (size_t)q + 1] = Td;
    }
}

// ---------------------------------------------------------------------------
// k_merge_rank16: k_merge_rank's fin pass without a state (the search's only
// merge: a P = 1 search) when a query has at most 16 lists -- 16 lanes a
// query, 4 queries a wave.  Same bounds, keys, ranks, records, certificate
// and fallback as k_merge_rank (fin, first_step); a lane ranks the group's
// candidates gl, gl + 16, ... against all of them.  k_merge_rank ran one
// wave a query with 14 of 64 lanes holding lists: 651 VALU instructions a
// query, most of them per-query work (loads, conversions, compaction, the
// records' sqrt) done once a wave (SQ counters, round 6).
// ---------------------------------------------------------------------------
template <typename TE, int KL>
__global__ __launch_bounds__(256) void k_merge_rank16(
    const double *__restrict__ part_d, const int *__restrict__ part_i, const double *__restrict__ part_T,
    int nsplit, int lpq, int nq, int nq_pad, int k, unsigned long long *__restrict__ qthr, knn_fin_args fa)
{
    constexpr int CAPG = 16 * KL + 4;   // a group's keys (+ pad: groups 32 bytes apart mod 256)
    __shared__ __attribute__((aligned(16))) unsigned long long r16_buf[16 * CAPG];
    constexpr unsigned DINF = 0xffffffffu;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int grp = lane >> 4, gl = lane & 15;
    const int q = blockIdx.x * 16 + wave * 4 + grp;
    const bool qv = q < nq;
    if (__ballot(qv) == 0ull) return;   // wave-uniform; no workgroup barrier below
    LDS_AS unsigned long long *buf = (LDS_AS unsigned long long *)r16_buf + (size_t)(wave * 4 + grp) * CAPG;
    const unsigned long long gmask = 0xffffull << (16 * grp);
    const unsigned long long ltmask = (1ull << lane) - 1ull;
    const int nl = qv ? lpq * nsplit : 0;
    const int qq = qv ? q : 0;
    const double qb = __longlong_as_double((long long)qthr[qq]);
    const double B = qb >= 4294967294.0 ? 4294967294.0 : floor(qb);
    const unsigned Bu = (unsigned)B;
    double T = KNN_INF;
    if (qv && gl < nsplit) T = part_T[(size_t)gl * nq_pad + q];
    const int mode = knn_mode_lim<TE>(fa.meta, fa.n, fa.lim);

    unsigned d[KL];
    int id[KL];
#pragma unroll
    for (int e = 0; e < KL; e++) {
        d[e] = DINF;
        id[e] = 0;
    }
    int c = 0;
    if (gl < nl) {
        const int sp = lpq == 2 ? gl >> 1 : lpq == 4 ? gl >> 2 : gl / lpq, g = gl - sp * lpq;
        const size_t base = (((size_t)sp * nq_pad + q) * lpq + g) * KL;
#pragma unroll
        for (int e = 0; e < 4 && e < KL; e++) {
            const double v = part_d[base + e];
            d[e] = v < 4294967295.0 ? (unsigned)v : DINF;
            id[e] = part_i[base + e];
        }
        if (KL > 4 && d[3] <= Bu) {
#pragma unroll
            for (int e = 4; e < KL; e++) {
                const double v = part_d[base + e];
                d[e] = v < 4294967295.0 ? (unsigned)v : DINF;
                id[e] = part_i[base + e];
            }
        }
#pragma unroll
        for (int e = 0; e < KL; e++) c += d[e] <= Bu ? 1 : 0;   // a prefix
    }
    for (int off = 8; off > 0; off >>= 1) T = fmin(T, __shfl_xor(T, off));   // within the group

    // the tighter bound: the (k+1)-th smallest key among the lists' first
    // HD entries (k_merge_rank)
    unsigned long long lim = ~0ull;
    {
        constexpr int HD = KL < 4 ? KL : 4;
        const int hh = c < HD ? c : HD;
        int preh = 0, CH = 0;
#pragma unroll
        for (int b = 0; b < 3; b++) {
            const unsigned long long m = __ballot((hh >> b) & 1) & gmask;
            preh += __popcll(m & ltmask) << b;
            CH += __popcll(m) << b;
        }
#pragma unroll
        for (int e = 0; e < HD; e++)
            if (CH > k && e < hh) buf[preh + e] = ((unsigned long long)d[e] << 32) | (unsigned)id[e];
        __builtin_amdgcn_wave_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (CH > k) {   // (group-uniform)
            unsigned long long bk = ~0ull;
            for (int b0 = 0; b0 < CH; b0 += 64) {
                unsigned long long x[4];
                int r[4];
#pragma unroll
                for (int t = 0; t < 4; t++) {
                    const int my = b0 + gl + 16 * t;
                    x[t] = my < CH ? buf[my] : ~0ull;
                    r[t] = 0;
                }
                int j = 0;
                for (; j + 4 <= CH; j += 4) {
                    const knn_u64x2 u = *(const LDS_AS knn_u64x2 *)(buf + j);
                    const knn_u64x2 w = *(const LDS_AS knn_u64x2 *)(buf + j + 2);
#pragma unroll
                    for (int t = 0; t < 4; t++)
                        r[t] += (u.x < x[t] ? 1 : 0) + (u.y < x[t] ? 1 : 0) + (w.x < x[t] ? 1 : 0) + (w.y < x[t] ? 1 : 0);
                }
                for (; j < CH; j++) {
                    const unsigned long long u = buf[j];
#pragma unroll
                    for (int t = 0; t < 4; t++) r[t] += u < x[t] ? 1 : 0;
                }
#pragma unroll
                for (int t = 0; t < 4; t++) {
                    const unsigned long long at = __ballot(b0 + gl + 16 * t < CH && r[t] == k) & gmask;
                    if (at) bk = __shfl(x[t], __builtin_ctzll(at));
                }
            }
            lim = bk;
            int c2 = 0;
#pragma unroll
            for (int e = 0; e < KL; e++)
                c2 += (e < c && (((unsigned long long)d[e] << 32) | (unsigned)id[e]) <= bk) ? 1 : 0;
            c = c2;
        }
        __builtin_amdgcn_wave_barrier();   // (the subset's slots are overwritten below)
    }
    // compaction: the group's entries at or below both bounds
    int pre = 0, C = 0;
#pragma unroll
    for (int b = 0; b < 5; b++) {
        const unsigned long long m = __ballot((c >> b) & 1) & gmask;
        pre += __popcll(m & ltmask) << b;
        C += __popcll(m) << b;
    }
    {
        int w = pre;
#pragma unroll
        for (int e = 0; e < KL; e++) {
            const unsigned long long key = ((unsigned long long)d[e] << 32) | (unsigned)id[e];
            if (d[e] <= Bu && key <= lim) buf[w++] = key;
        }
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");

    if (blockIdx.x == 0 && threadIdx.x == 0) *fa.mode_out = mode;
    // slots past the candidates: {inf, 0, 0}
    for (int p = gl; p < k; p += 16)
        if (qv && p >= C) {
            knn_neighbour_t rec;
            rec.distance = KNN_INF;
            rec.idx = 0;
            rec.label = 0;
            fa.out[(size_t)q * k + p] = rec;
        }
    double tau = KNN_INF, tk1 = KNN_INF;
    for (int b0 = 0; b0 < C; b0 += 64) {   // (group-uniform trip count)
        unsigned long long x[4];
        int r[4];
#pragma unroll
        for (int t = 0; t < 4; t++) {
            const int my = b0 + gl + 16 * t;
            x[t] = my < C ? buf[my] : ~0ull;
            r[t] = 0;
        }
        const int nt = (C - b0 + 15) >> 4;   // live slots a lane this round (group-uniform)
        int j = 0;
        for (; j + 4 <= C; j += 4) {
            const knn_u64x2 u = *(const LDS_AS knn_u64x2 *)(buf + j);
            const knn_u64x2 w = *(const LDS_AS knn_u64x2 *)(buf + j + 2);
#pragma unroll
            for (int t = 0; t < 4; t++)
                if (t < nt)
                    r[t] += (u.x < x[t] ? 1 : 0) + (u.y < x[t] ? 1 : 0) + (w.x < x[t] ? 1 : 0) + (w.y < x[t] ? 1 : 0);
        }
        for (; j < C; j++) {
            const unsigned long long u = buf[j];
#pragma unroll
            for (int t = 0; t < 4; t++) r[t] += u < x[t] ? 1 : 0;
        }
#pragma unroll
        for (int t = 0; t < 4; t++) {
            const bool live = b0 + gl + 16 * t < C;
            if (live && r[t] < k) {
                knn_neighbour_t rec;
                rec.distance = sqrt((double)(unsigned)(x[t] >> 32));
                rec.idx = (int)(unsigned)x[t] + 1;
                rec.label = 0;
                fa.out[(size_t)q * k + r[t]] = rec;
            }
            const unsigned long long a0 = __ballot(live && r[t] == k - 1) & gmask;
            if (a0) tau = (double)(unsigned)(__shfl(x[t], __builtin_ctzll(a0)) >> 32);
            const unsigned long long a1 = __ballot(live && r[t] == k) & gmask;
            if (a1) tk1 = (double)(unsigned)(__shfl(x[t], __builtin_ctzll(a1)) >> 32);
        }
    }
    const bool ok = mode == KNN_MODE_INT && !fa.force_fail && (T == KNN_INF || (C >= k && tau < T));
    if (qv && !ok && C < k + 1 && mode == KNN_MODE_INT && !fa.force_fail) {
        // fewer than k + 1 entries under the bounds: the k-th and (k+1)-th
        // over every entry of the lists (k_merge_rank's fallback)
        int c2 = 0;
        if (gl < nl) {
            const int sp = lpq == 2 ? gl >> 1 : lpq == 4 ? gl >> 2 : gl / lpq, g = gl - sp * lpq;
            const size_t base = (((size_t)sp * nq_pad + q) * lpq + g) * KL;
#pragma unroll
            for (int e = 0; e < KL; e++) {
                const double v = part_d[base + e];
                d[e] = v < 4294967295.0 ? (unsigned)v : DINF;
                id[e] = part_i[base + e];
                c2 += d[e] != DINF ? 1 : 0;   // a prefix
            }
        }
        int pre2 = 0, C2 = 0;
#pragma unroll
        for (int b = 0; b < 5; b++) {
            const unsigned long long m = __ballot((c2 >> b) & 1) & gmask;
            pre2 += __popcll(m & ltmask) << b;
            C2 += __popcll(m) << b;
        }
#pragma unroll
        for (int e = 0; e < KL; e++)
            if (e < c2) buf[pre2 + e] = ((unsigned long long)d[e] << 32) | (unsigned)id[e];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        for (int my0 = 0; my0 < C2; my0 += 16) {
            const int my = my0 + gl;
            const unsigned long long x = my < C2 ? buf[my] : ~0ull;
            int r = 0;
            for (int j = 0; j < C2; j++) r += buf[j] < x ? 1 : 0;
            const unsigned long long a0 = __ballot(my < C2 && r == k - 1) & gmask;
            if (a0) tau = (double)(unsigned)(__shfl(x, __builtin_ctzll(a0)) >> 32);
            const unsigned long long a1 = __ballot(my < C2 && r == k) & gmask;
            if (a1) tk1 = (double)(unsigned)(__shfl(x, __builtin_ctzll(a1)) >> 32);
        }
    }
    if (qv && !ok && gl == 0) {
        fa.fail_list[atomicAdd(fa.fail_count, 1)] = q;
        fa.fbound[q] = (fa.force_fail || mode != KNN_MODE_INT) ? KNN_INF : sqrt(tau);
        if (mode == KNN_MODE_INT && !fa.force_fail)
            qthr[q] = (unsigned long long)__double_as_longlong(sizeof(TE) == 4 ? (double)__double2float_ru(tk1) : tk1);
    }
}

// ---------------------------------------------------------------------------
// k_finalize: one wave per query.  Order by (sqrt(S), idx) -- the key the
// reference keeps (knn-serial.c:86-90) -- drop S == 0, and certify: every
// candidate outside the state has approx d^2 >= T, hence exact S >= T - E
// (E bounds the GEMM-form plus the reference's own rounding); if
// T - E > tau (the k-th kept S, with a margin so sqrt cannot collapse
// them) nothing unseen can enter the list.  Uncertified queries go to the
// rescan list.
// ---------------------------------------------------------------------------
template <typename TE, int KP>
__global__ __launch_bounds__(256) void k_finalize(
    const double *__restrict__ st_d, const double *__restrict__ st_x,
    const int *__restrict__ st_i, const double *__restrict__ st_T,
    const TE *__restrict__ qnorm, int nq, int n, int k,
    const double *__restrict__ meta, knn_neighbour_t *__restrict__ out,
    int *__restrict__ fail_count, int *__restrict__ fail_list, int *__restrict__ mode_out,
    double *__restrict__ fbound, int force_fail, int filt)
{
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int q = blockIdx.x * 4 + wave;
    const int mode = knn_mode<TE>(meta, n);
    if (blockIdx.x == 0 && threadIdx.x == 0) *mode_out = mode;
    if (q >= nq) return;
    knn_neighbour_t *o = out + (size_t)q * k;

    // force_fail: tests of the rescan pass; no query norms (a context begun
    // from a byte block alone, knn_ctx_begin_s8) outside INT mode: nothing
    // exact to certify with -- every query takes the rescan
    if (mode == KNN_MODE_SCAN || force_fail || (mode != KNN_MODE_INT && qnorm == nullptr)) {
        if (lane == 0) {
            fail_list[atomicAdd(fail_count, 1)] = q;
            fbound[q] = KNN_INF;
        }
        return;
    }
    constexpr int NS = (KP + 63) / 64;   // state slot r on lane r & 63, register r >> 6
    double sd[NS], sx[NS];
    int si[NS];
#pragma unroll
    for (int x = 0; x < NS; x++) {
        const int r = lane + 64 * x;
        sd[x] = KNN_INF;
        sx[x] = KNN_INF;
        si[x] = -1;
        if (r < KP) {
            sd[x] = st_d[(size_t)q * KP + r];
            sx[x] = st_x[(size_t)q * KP + r];
            si[x] = st_i[(size_t)q * KP + r];
        }
    }
    const double T = st_T[2 * (size_t)q], Td = st_T[2 * (size_t)q + 1];
    const int kl = k - 1;
    if (mode == KNN_MODE_INT) {
        // state is sorted by exact (d^2, idx) and zeros were never admitted.
        // A candidate a lane filter turned away has d^2 >= T; with d^2 == T
        // it may precede the k-th by index, so certify only tau < T.
        bool valid[NS];
        int nnz = 0;
#pragma unroll
        for (int x = 0; x < NS; x++) {
            valid[x] = si[x] >= 0 && sd[x] < KNN_INF;
            nnz += __popcll(__ballot(valid[x]));
        }
        bool ok;
        double tau = KNN_INF;   // k-th exact d^2 kept: the rescan's bound
        if (nnz >= k) {
#pragma unroll
            for (int x = 0; x < NS; x++) {
                const double v = __shfl(sd[x], kl & 63);
                if ((kl >> 6) == x) tau = v;
            }
            ok = (T == KNN_INF) || (tau < T);
        } else {
            ok = (T == KNN_INF);
        }
        if (!ok) {
            if (lane == 0) {
                fail_list[atomicAdd(fail_count, 1)] = q;
                fbound[q] = sqrt(tau);
            }
            return;
        }
#pragma unroll
        for (int x = 0; x < NS; x++) {
            const int r = lane + 64 * x;
            if (r < k) {
                knn_neighbour_t rec;
                rec.distance = valid[x] ? sqrt(sd[x]) : KNN_INF;
                rec.idx = valid[x] ? si[x] + 1 : 0;
                rec.label = 0;
                o[r] = rec;
            }
        }
        return;
    }
    // GEMM mode
    bool valid[NS];
    double key[NS];
    int kid[NS], rank[NS];
#pragma unroll
    for (int x = 0; x < NS; x++) {
        valid[x] = (si[x] >= 0) && (sx[x] == sx[x]) && (sx[x] != 0.0) && (sx[x] < KNN_INF);
        key[x] = valid[x] ? sqrt(sx[x]) : KNN_INF;
        kid[x] = valid[x] ? si[x] : 0x7fffffff;
        rank[x] = 0;
    }
    // rank = number of entries before this one by (sqrt(S), idx); unused
    // slots (key inf, id max) precede nothing
    for (int j = 0; j < 64; j++) {
#pragma unroll
        for (int y = 0; y < NS; y++) {
            const double kj = __shfl(key[y], j);
            const int ij = __shfl(kid[y], j);
#pragma unroll
            for (int x = 0; x < NS; x++)
                rank[x] += (kj < key[x] || (kj == key[x] && ij < kid[x])) ? 1 : 0;
        }
    }
    int nnz = 0;
#pragma unroll
    for (int x = 0; x < NS; x++) nnz += __popcll(__ballot(valid[x]));
    const double Tb = fmin(T, Td);
    bool ok;
    double tau = KNN_INF;   // exact S of the k-th kept: the rescan's bound
    if (nnz >= k) {
#pragma unroll
        for (int x = 0; x < NS; x++) {
            const unsigned long long at = __ballot(valid[x] && rank[x] == kl);
            if (at) tau = __shfl(sx[x], __builtin_ctzll(at));
        }
        // E (knn_cert_E): |GEMM-form d^2 - exact S| plus the reference's
        // own rounding; T and Td are GEMM-form values
        const double E = knn_cert_E<TE>(n, (double)qnorm[q], meta[KNN_META_MAXNORM], filt, meta[KNN_META_MAXABS]);
        ok = (Tb == KNN_INF) || ((Tb - E) > tau * (1.0 + 1.7763568394002505e-15));
    } else {
        ok = (Tb == KNN_INF);
    }
    if (!ok) {
        if (lane == 0) {
            fail_list[atomicAdd(fail_count, 1)] = q;
            fbound[q] = sqrt(tau);
        }
        return;
    }
#pragma unroll
    for (int x = 0; x < NS; x++) {
        if (valid[x] && rank[x] < k) {
            knn_neighbour_t rec;
            rec.distance = key[x];
            rec.idx = si[x] + 1;
            rec.label = 0;
            o[rank[x]] = rec;
        }
        const int r = lane + 64 * x;
        if (r >= nnz && r < k) {
            knn_neighbour_t rec;
            rec.distance = KNN_INF;
            rec.idx = 0;
            rec.label = 0;
            o[r] = rec;
        }
    }
}

// ---------------------------------------------------------------------------
// Exact rescan (uncertified queries): the reference's arithmetic on every
// (query, row) pair -- S = S + (a-b)^2 in j order in fp64, key sqrt(S),
// 0 < key < inf as serial:86 admits -- merged into the query's running
// rescan list (its first k entries ordered by (key, idx)).
//
// A 256-thread workgroup takes 16 queries, 4 per wave.  The wave's 4 query
// rows are wave-uniform, so hipcc reads them with scalar loads into SGPRs;
// lane l streams rows l, l+64, ... with 16-byte loads and accumulates all 4
// S in registers, so each row is read once per 4 queries (and the 4 waves
// walk the rows in step, sharing L2/L1 lines).  Zero padding past n adds
// (0-0)^2 = 0, leaving S bit-identical, so the loop runs to a whole 16 B.
//
// Filter: only keys <= dcut can reach the top k, dcut = min(the bound
// k_finalize left in fbound (the k-th key of the uncertified state: k real
// candidates lie at or below it), the k-th key of the running list).  Each
// lane keeps its KT smallest admitted keys above a floor; the merge (wave
// argmin rounds, one query at a time) takes entries only up to B, the
// smallest KT-th key of any lane that dropped one, and if the list is not
// complete by then the wave scans again above the last key taken.
// ---------------------------------------------------------------------------
template <typename TE, int KP>
__global__ __launch_bounds__(256) void k_rescan_step(
    const int *__restrict__ fail_list, int nfail, const double *__restrict__ fbound,
    const TE *__restrict__ qblk, int n_pad_q, const TE *__restrict__ cblk, size_t c_base,
    int nc, int n, int n_pad, int k, const double *rs_bound, double *rs_d, int *rs_i,
    int rows_per_chunk, size_t chunk_stride)
{
#pragma clang fp contract(off)
    constexpr int KT = 4, QW = 4;
    constexpr int V = 16 / (int)sizeof(TE);          // elements per 16-byte load
    constexpr int NS = (KP + 63) / 64;                // list slot r: lane r & 63, reg r >> 6
    typedef typename std::conditional<sizeof(TE) == 8, dbl2, flt4>::type vec_t;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int slot0 = blockIdx.x * 16 + wave * QW;
    if (slot0 >= nfail) return;                       // wave-uniform
    // 16-byte pieces per row, whole 128-byte pieces: rows are zero padded to
    // n_pad (query and corpus blocks alike) and S + (0-0)^2 = S
    constexpr int U = 8;
    const int nr = n_pad / V;
    // corpus chunk blockIdx.y: rows [row0, row1) into its own list set
    const int row0 = blockIdx.y * rows_per_chunk;
    const int row1 = min(nc, row0 + rows_per_chunk);
    rs_d += blockIdx.y * chunk_stride;
    rs_i += blockIdx.y * chunk_stride;

    const TE *qp[QW];
    double dcut[QW];
    int slot[QW];
    bool done[QW];
#pragma unroll
    for (int x = 0; x < QW; x++) {
        slot[x] = slot0 + x;
        done[x] = slot[x] >= nfail;
        const int q = done[x] ? fail_list[slot0] : fail_list[slot[x]];
        qp[x] = qblk + (size_t)q * n_pad_q;
        const double kth = rs_bound[(size_t)(done[x] ? slot0 : slot[x]) * KP + (k - 1)];
        dcut[x] = fmin(fbound[q], kth);
    }
    // running list of each query: old (read) and new (written at the end)
    double nd[QW][NS];
    int ni[QW][NS];
    int produced[QW], pos_old[QW];
    double fd[QW];
    int fi[QW];
#pragma unroll
    for (int x = 0; x < QW; x++) {
#pragma unroll
        for (int s = 0; s < NS; s++) { nd[x][s] = KNN_INF; ni[x][s] = -1; }
        produced[x] = 0;
        pos_old[x] = 0;
        fd[x] = -1.0;
        fi[x] = -1;
    }

    for (;;) {
        double L[QW][KT];
        int I[QW][KT], cnt[QW];
#pragma unroll
        for (int x = 0; x < QW; x++) {
            cnt[x] = 0;
#pragma unroll
            for (int e = 0; e < KT; e++) { L[x][e] = KNN_INF; I[x][e] = 0x7fffffff; }
        }
        for (int row = row0 + lane; row < row1; row += 64) {
            const vec_t *cr = (const vec_t *)(cblk + (size_t)row * n_pad);
            double S[QW] = {0.0, 0.0, 0.0, 0.0};
            // 8 pieces of the row in flight before any is used (the sums are
            // dependent chains; one memory latency every 128 bytes, not 16)
            for (int p = 0; p < nr; p += U) {
                vec_t c[U];
#pragma unroll
                for (int u = 0; u < U; u++) c[u] = cr[p + u];
#pragma unroll
                for (int u = 0; u < U; u++)
#pragma unroll
                    for (int x = 0; x < QW; x++) {
                        const vec_t a = ((const vec_t *)qp[x])[p + u];
#pragma unroll
                        for (int e = 0; e < V; e++) {
                            const double t = (double)a[e] - (double)c[u][e];
                            const double t2 = t * t;
                            S[x] = S[x] + t2;
                        }
                    }
            }
            const int id = (int)(c_base + row);
#pragma unroll
            for (int x = 0; x < QW; x++) {
                const double d = sqrt(S[x]);
                if (!done[x] && d != 0.0 && d < KNN_INF && d <= dcut[x] &&
                    (d > fd[x] || (d == fd[x] && id > fi[x]))) {
                    cnt[x]++;
                    list_insert<KT>(L[x], I[x], d, id);   // rows ascend: ties stay in id order
                }
            }
        }
        bool again_any = false;
#pragma unroll
        for (int x = 0; x < QW; x++) {
            if (done[x]) continue;                        // wave-uniform
            double Bd = (cnt[x] > KT) ? L[x][KT - 1] : KNN_INF;
            int Bi = (cnt[x] > KT) ? I[x][KT - 1] : 0x7fffffff;
            wave_argmin(Bd, Bi);
            const double *od = rs_d + (size_t)slot[x] * KP;
            const int *oi = rs_i + (size_t)slot[x] * KP;
            int pos = 0;
            bool again = false;
            while (produced[x] < k) {
                double hd = (pos < KT) ? L[x][0] : KNN_INF;
                int hi = (pos < KT) ? I[x][0] : 0x7fffffff;
                if (hd == KNN_INF) hi = 0x7fffffff;
                bool mine = true;
                if (lane == 0 && pos_old[x] < k) {
                    const double v = od[pos_old[x]];
                    const int vi = (v == KNN_INF) ? 0x7fffffff : oi[pos_old[x]];
                    if (v < hd || (v == hd && vi < hi)) { hd = v; hi = vi; mine = false; }
                }
                double wd = hd;
                int wi = hi;
                wave_argmin(wd, wi);
                if (wd == KNN_INF) break;                                  // both sources empty
                if (Bd < wd || (Bd == wd && Bi < wi)) { again = true; break; }  // past B
                const int r = produced[x];
#pragma unroll
                for (int s = 0; s < NS; s++)
                    if (lane == (r & 63) && (r >> 6) == s) { nd[x][s] = wd; ni[x][s] = wi; }
                produced[x]++;
                fd[x] = wd;
                fi[x] = wi;
                const bool took = (hd == wd && hi == wi);
                const unsigned long long who = __ballot(took);
                const int wl = __builtin_ctzll(who);
                const bool from_old = __shfl((int)(!mine), wl) != 0;
                if (from_old) {
                    pos_old[x]++;
                } else if (lane == wl) {
                    // pop the lane's head (lists are shifted so L[0] is the head)
#pragma unroll
                    for (int e = 0; e < KT - 1; e++) { L[x][e] = L[x][e + 1]; I[x][e] = I[x][e + 1]; }
                    L[x][KT - 1] = KNN_INF;
                    I[x][KT - 1] = 0x7fffffff;
                    pos++;
                }
            }
            if (!again) done[x] = true;
            again_any |= again;
        }
        if (!again_any) break;
    }
    // all old-list reads precede the writes (the wave owns these slots)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int x = 0; x < QW; x++) {
        if (slot[x] >= nfail) continue;
#pragma unroll
        for (int s = 0; s < NS; s++) {
            const int r = lane + 64 * s;
            if (r < KP) {
                rs_d[(size_t)slot[x] * KP + r] = nd[x][s];
                rs_i[(size_t)slot[x] * KP + r] = (nd[x][s] == KNN_INF) ? -1 : ni[x][s];
            }
        }
    }
}

__global__ void k_fill_inf(double *p, int count)
{
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < count) p[i] = KNN_INF;
}

// begin(): the shared bounds (+inf), the int8 kernel's cross-split summaries
// (0x7f7f7f7f pairs: above every int8-mode d^2) and the two counters
// (unresolved queries, mode) in one launch instead of three
__global__ void k_begin_init(double *qthr, unsigned long long *qsum, int nq_pad, int *counts)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nq_pad) qthr[i] = KNN_INF;
    if (qsum != nullptr && i < nq_pad) {
#pragma unroll
        for (int j = 0; j < 4; j++) qsum[4 * (size_t)i + j] = 0x7f7f7f7f7f7f7f7full;
    }
    if (i < 2) counts[i] = 0;
}

// the search's (unresolved, mode) pair and the meta its kernels read into
// mapped host memory (knn_ctx_end reads them after synchronising with the
// stream; the meta is knn_ctx_search_meta's -- no separate read-back copy)
__global__ void k_count_out(const int *__restrict__ src, int *__restrict__ dst, const double *__restrict__ meta,
                            double *__restrict__ dst_meta)
{
    if (threadIdx.x < 2) dst[threadIdx.x] = src[threadIdx.x];
    if (meta != nullptr && threadIdx.x < KNN_META_DOUBLES) dst_meta[threadIdx.x] = meta[threadIdx.x];
}

extern "C" int knn_launch_count_out(const int *d_count, int *mapped, const double *meta, double *mapped_meta,
                                    void *stream)
{
    hipLaunchKernelGGL(k_count_out, dim3(1), dim3(64), 0, (hipStream_t)stream, d_count, mapped, meta, mapped_meta);
    return hipGetLastError() == hipSuccess ? KNN_OK : KNN_ERR_HIP;
}

extern "C" int knn_launch_begin_init(double *qthr, unsigned long long *qsum, int nq_pad, int *counts,
                                     void *stream)
{
    const int n = nq_pad > 2 ? nq_pad : 2;
    hipLaunchKernelGGL(k_begin_init, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       qthr, qsum, nq_pad, counts);
    return hipGetLastError() == hipSuccess ? KNN_OK : KNN_ERR_HIP;
}

extern "C" int knn_launch_fill_inf(double *p, int count, void *stream)
{
    if (count <= 0) return KNN_OK;
    hipLaunchKernelGGL(k_fill_inf, dim3((unsigned)((count + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, p, count);
    return hipGetLastError() == hipSuccess ? KNN_OK : KNN_ERR_HIP;
}

__global__ void k_rescan_init(double *rs_d, int *rs_i, int count)
{
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < count) { rs_d[i] = KNN_INF; rs_i[i] = -1; }
}

// Chunked rescan, second half: per query, the running list (list 0) and the
// C chunk lists (each already the exact top k of its rows, ordered by
// (key, idx)) merge into the running list.  One wave per query; lane j
// holds the head of list j; k argmin rounds.  Row ids are disjoint across
// lists, so no entry appears twice.
template <int KP>
__global__ __launch_bounds__(256) void k_rescan_merge(int nfail, int k, int nchunk,
                                                      double *__restrict__ rs_d,
                                                      int *__restrict__ rs_i)
{
    constexpr int NS = (KP + 63) / 64;
    const int lane = threadIdx.x & 63;
    const int slot = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (slot >= nfail) return;                        // wave-uniform
    const size_t stride = (size_t)nfail * KP;
    const bool live = lane <= nchunk;
    const double *ld = rs_d + (size_t)lane * stride + (size_t)slot * KP;
    const int *li = rs_i + (size_t)lane * stride + (size_t)slot * KP;
    double nd[NS];
    int ni[NS];
#pragma unroll
    for (int s = 0; s < NS; s++) { nd[s] = KNN_INF; ni[s] = -1; }
    int pos = 0;
    for (int r = 0; r < k; r++) {
        double hd = (live && pos < k) ? ld[pos] : KNN_INF;
        int hi = (hd == KNN_INF) ? 0x7fffffff : li[pos];
        const double md = hd;
        const int mi = hi;
        wave_argmin(hd, hi);
        if (hd == KNN_INF) break;                     // every list exhausted
#pragma unroll
        for (int s = 0; s < NS; s++)
            if (lane == (r & 63) && (r >> 6) == s) { nd[s] = hd; ni[s] = hi; }
        if (md == hd && mi == hi) pos++;             // ids are unique: one winner
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // reads of list 0 before its rewrite
#pragma unroll
    for (int s = 0; s < NS; s++) {
        const int r = lane + 64 * s;
        if (r < KP) {
            rs_d[(size_t)slot * KP + r] = nd[s];
            rs_i[(size_t)slot * KP + r] = (nd[s] == KNN_INF) ? -1 : ni[s];
        }
    }
}

__global__ void k_rescan_end(const int *__restrict__ fail_list, int nfail, int KP,
                             const double *__restrict__ rs_d, const int *__restrict__ rs_i,
                             int k, knn_neighbour_t *__restrict__ out)
{
    int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nfail * k) return;
    const int slot = t / k, r = t % k;
    const int q = fail_list[slot];
    knn_neighbour_t rec;
    const double d = rs_d[(size_t)slot * KP + r];
    const int id = rs_i[(size_t)slot * KP + r];
    const bool ok = d < KNN_INF && id >= 0;
    rec.distance = ok ? d : KNN_INF;
    rec.idx = ok ? id + 1 : 0;
    rec.label = 0;
    out[(size_t)q * k + r] = rec;
}

// ---------------------------------------------------------------------------
// C launchers
// ---------------------------------------------------------------------------
static int hip_status(void) { return hipGetLastError() == hipSuccess ? KNN_OK : KNN_ERR_HIP; }

template <typename T, typename S>
static int launch_pack(T *blk, size_t cap, size_t rows, size_t n, const S *src, size_t ld,
                       int layout, hipStream_t s)
{
    constexpr int dt = sizeof(T) == 8 ? KNN_F64 : KNN_F32;
    const size_t rp = knn_rows_pad(cap), np = knn_n_pad_dt(n, dt);
    double *meta = (double *)(blk + rp * np + rp);
    if (hipMemsetAsync(meta, 0, KNN_META_DOUBLES * sizeof(double), s) != hipSuccess)
        return KNN_ERR_HIP;
    if (layout == KNN_COLMAJOR) {
        hipLaunchKernelGGL(HIP_KERNEL_NAME(k_pack_col<T, S>), dim3((unsigned)((rp + 63) / 64)), dim3(256), 0, s,
                           blk, rows, rp, (int)n, (int)np, src, ld);
    } else {
        const unsigned nb = (unsigned)((rp + 3) / 4 < 8192 ? (rp + 3) / 4 : 8192);
        hipLaunchKernelGGL(HIP_KERNEL_NAME(k_pack_row<T, S>), dim3(nb), dim3(256), 0, s, blk, rows, rp,
                           (int)n, (int)np, src, ld);
    }
    return hip_status();
}

template <typename T, typename S>
static int launch_pack8(signed char *dst, size_t cap, size_t rows, size_t n, const S *src, size_t ld, int layout,
                        hipStream_t s)
{
    const size_t rp = knn_rows_pad(cap), rs = knn_s8_rs(n);
    double *meta = (double *)(dst + knn_s8_meta_offset(cap, n));
    if (hipMemsetAsync(meta, 0, KNN_META_DOUBLES * sizeof(double), s) != hipSuccess) return KNN_ERR_HIP;
    if (layout == KNN_COLMAJOR) {
        // (32-row workgroups, twice as many: 107.5 against 105.7 us for MNIST)
        hipLaunchKernelGGL(HIP_KERNEL_NAME(k_pack8_col<T, S, 64>), dim3((unsigned)((rp + 63) / 64)), dim3(256), 0,
                           s, dst, rows, rp, (int)n, (int)rs, src, ld);
    } else {
        const unsigned nb = (unsigned)((rp + 3) / 4 < 8192 ? (rp + 3) / 4 : 8192);
        const bool vec = ((uintptr_t)src % 16 == 0) && (ld * sizeof(S)) % 16 == 0;
        if (vec)
            hipLaunchKernelGGL(HIP_KERNEL_NAME(k_pack8_row<T, S, true>), dim3(nb), dim3(256), 0, s, dst, rows, rp,
                               (int)n, (int)rs, src, ld);
        else
            hipLaunchKernelGGL(HIP_KERNEL_NAME(k_pack8_row<T, S, false>), dim3(nb), dim3(256), 0, s, dst, rows, rp,
                               (int)n, (int)rs, src, ld);
    }
    return hip_status();
}

extern "C" int knn_launch_pack_s8(void *dst, int dtype, size_t cap, size_t rows, size_t n, const void *src,
                                  int src_dtype, size_t ld, int layout, void *stream)
{
    hipStream_t s = (hipStream_t)stream;
    signed char *d = (signed char *)dst;
    if (dtype == KNN_F64 && src_dtype == KNN_F64) return launch_pack8<double>(d, cap, rows, n, (const double *)src, ld, layout, s);
    if (dtype == KNN_F64 && src_dtype == KNN_F32) return launch_pack8<double>(d, cap, rows, n, (const float *)src, ld, layout, s);
    if (dtype == KNN_F32 && src_dtype == KNN_F64) return launch_pack8<float>(d, cap, rows, n, (const double *)src, ld, layout, s);
    if (dtype == KNN_F32 && src_dtype == KNN_F32) return launch_pack8<float>(d, cap, rows, n, (const float *)src, ld, layout, s);
    return KNN_ERR_INVALID;
}

// Ring wire form of a packed block (knn_wire_pack / knn_wire_unpack): the
// element array as int16 (exact for integer data with max|x| <= 32767),
// 8 elements a thread; norms and meta travel verbatim (hipMemcpyAsync).
typedef short knn_s8v __attribute__((ext_vector_type(8)));
template <typename T>
__global__ __launch_bounds__(256) void k_wire_pack(knn_s8v *__restrict__ w, const T *__restrict__ b,
                                                   size_t n8)
{
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += (size_t)gridDim.x * 256) {
        knn_s8v v;
#pragma unroll
        for (int e = 0; e < 8; e++) v[e] = (short)b[8 * i + e];
        w[i] = v;
    }
}
template <typename T>
__global__ __launch_bounds__(256) void k_wire_unpack(T *__restrict__ b, const knn_s8v *__restrict__ w,
                                                     size_t n8)
{
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += (size_t)gridDim.x * 256) {
        const knn_s8v v = w[i];
#pragma unroll
        for (int e = 0; e < 8; e++) b[8 * i + e] = (T)v[e];
    }
}

// fp16 shadow rows of a packed block for the H16 == 2 contraction: rows
// of round_up(n, 64) halves (zero padded), converted with v_cvt_pkrtz
// (exact: shadows are only made for integer data with max|x| <= 2048).
template <typename T>
__global__ __launch_bounds__(256) void k_shadow(knn_h8 *__restrict__ dst, const T *__restrict__ src,
                                                size_t rows, int n, int nps, int npd)
{
    const size_t per = (size_t)npd / 8, tot = rows * per;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < tot; i += (size_t)gridDim.x * 256) {
        const size_t r = i / per;
        const int c = (int)(i - r * per) * 8;
        const T *row = src + r * (size_t)nps;
        unsigned w[4];
#pragma unroll
        for (int e = 0; e < 4; e++) {
            const int j = c + 2 * e;
            const float x0 = j < n ? (float)row[j] : 0.f;
            const float x1 = j + 1 < n ? (float)row[j + 1] : 0.f;
            w[e] = __builtin_bit_cast(unsigned, __builtin_amdgcn_cvt_pkrtz(x0, x1));
        }
        typedef unsigned u4 __attribute__((ext_vector_type(4)));
        dst[i] = __builtin_bit_cast(knn_h8, (u4){w[0], w[1], w[2], w[3]});
    }
}

extern "C" int knn_launch_shadow(void *dst, const void *blk, int dtype, size_t rows_pad, size_t n,
                                 void *stream)
{
    const int npd = (int)knn_round_up(n, 64), nps = (int)knn_n_pad_dt(n, dtype);
    const size_t tot = rows_pad * (size_t)npd / 8;
    const unsigned grid = (unsigned)(tot / 256 + 1 < 8192 ? tot / 256 + 1 : 8192);
    hipStream_t s = (hipStream_t)stream;
    if (dtype == KNN_F64)
        hipLaunchKernelGGL(k_shadow<double>, dim3(grid), dim3(256), 0, s, (knn_h8 *)dst,
                           (const double *)blk, rows_pad, (int)n, nps, npd);
    else if (dtype == KNN_F32)
        hipLaunchKernelGGL(k_shadow<float>, dim3(grid), dim3(256), 0, s, (knn_h8 *)dst,
                           (const float *)blk, rows_pad, (int)n, nps, npd);
    else
        return KNN_ERR_INVALID;
    return hip_status();
}

// Split fp16 shadow rows (the split filter) of fp32 / fp64 blocks: per row
// and 32-feature group, the 32 halves hi = RN16(S x) then the 32 halves lo =
// RN16(S x - hi), each rounded once from the block's precision (S x - hi is
// exact there: Sterbenz); zero past n.  One thread per 16 bytes
// of source row (V = 2 fp64 / 4 fp32 features): a wave reads 1 KiB of a row
// contiguously and its 16-lane groups write whole 64-byte hi and lo runs.
// (Round 4's form, one thread per 8 features with 8-byte loads 64 bytes
// apart, moved a 7552 x 784 fp64 block in 35 us, 2 TB/s.)  Up to
// KNN_SPLIT_MAXBLK blocks per launch (a ring rank's received blocks).
struct knn_split_conv_t {
    char *dst[KNN_SPLIT_MAXBLK];
    const void *src[KNN_SPLIT_MAXBLK];
    long long i0[KNN_SPLIT_MAXBLK + 1];   // first flat work item of block b
    int nblk;
};

template <typename T>
__global__ __launch_bounds__(256) void k_shadow_split(const knn_split_conv_t cv, int n, int nps, int npd, float S)
{
    constexpr int V = 16 / (int)sizeof(T);
    typedef typename std::conditional<sizeof(T) == 8, dbl2, flt4>::type vec_t;
    typedef _Float16 hv_t __attribute__((ext_vector_type(V)));
    const int per = npd / V;   // work items a row
    const long long tot = cv.i0[cv.nblk];
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < tot; i += (long long)gridDim.x * 256) {
        int b = 0;
#pragma unroll
        for (int x = 1; x < KNN_SPLIT_MAXBLK; x++) b = (x < cv.nblk && i >= cv.i0[x]) ? x : b;
        const long long li = i - cv.i0[b];
        const long long r = li / per;
        const int j0 = (int)(li - r * per) * V;
        vec_t v{};
        if (j0 < n) v = *(const vec_t *)((const T *)cv.src[b] + r * (long long)nps + j0);
        hv_t hi, lo;
#pragma unroll
        for (int e = 0; e < V; e++) {
            // one rounding each, from the block's precision (x - hi is exact
            // in it: Sterbenz).  (Written as conversions through fp32, the
            // compiler folds them into these single roundings anyway.)
            const T x = (j0 + e < n) ? v[e] * (T)S : (T)0;
            const _Float16 h = (_Float16)x;
            hi[e] = h;
            lo[e] = (_Float16)(x - (T)h);
        }
        char *o = cv.dst[b] + r * (long long)npd * 4 + (long long)(j0 >> 5) * 128 + 2 * (j0 & 31);
        *(hv_t *)o = hi;
        *(hv_t *)(o + 64) = lo;
    }
}

// nblk blocks: dst[b] <- split rows of src[b] (rows_pad[b] rows each)
extern "C" int knn_launch_shadow_split_n(int nblk, void *const *dst, const void *const *src, const size_t *rows_pad,
                                         int dtype, size_t n, float S, void *stream)
{
    if (nblk < 1 || nblk > KNN_SPLIT_MAXBLK || n == 0) return KNN_ERR_INVALID;
    const int npd = (int)knn_round_up(n, 32), nps = (int)knn_n_pad_dt(n, dtype);
    const int V = dtype == KNN_F64 ? 2 : 4;
    knn_split_conv_t cv{};
    cv.nblk = nblk;
    cv.i0[0] = 0;
    for (int b = 0; b < nblk; b++) {
        if (!dst[b] || !src[b]) return KNN_ERR_INVALID;
        cv.dst[b] = (char *)dst[b];
        cv.src[b] = src[b];
        cv.i0[b + 1] = cv.i0[b] + (long long)rows_pad[b] * (npd / V);
    }
    for (int b = nblk + 1; b <= KNN_SPLIT_MAXBLK; b++) cv.i0[b] = cv.i0[nblk];
    const long long tot = cv.i0[nblk];
    const unsigned grid = (unsigned)(tot / 256 + 1 < 16384 ? tot / 256 + 1 : 16384);
    if (dtype == KNN_F32)
        hipLaunchKernelGGL(k_shadow_split<float>, dim3(grid), dim3(256), 0, (hipStream_t)stream, cv, (int)n, nps,
                           npd, S);
    else if (dtype == KNN_F64)
        hipLaunchKernelGGL(k_shadow_split<double>, dim3(grid), dim3(256), 0, (hipStream_t)stream, cv, (int)n, nps,
                           npd, S);
    else
        return KNN_ERR_INVALID;
    return hip_status();
}

extern "C" int knn_launch_shadow_split(void *dst, const void *blk, int dtype, size_t rows_pad, size_t n,
                                       float S, void *stream)
{
    return knn_launch_shadow_split_n(1, &dst, &blk, &rows_pad, dtype, n, S, stream);
}

extern "C" int knn_launch_wire(int unpack, void *dst, const void *src, int dtype, size_t cnt,
                               void *stream)
{
    if (cnt % 8) return KNN_ERR_INVALID;
    const size_t n8 = cnt / 8;
    const unsigned grid = (unsigned)(n8 / 256 + 1 < 4096 ? n8 / 256 + 1 : 4096);
    hipStream_t s = (hipStream_t)stream;
    if (dtype == KNN_F64 && !unpack)
        hipLaunchKernelGGL(k_wire_pack<double>, dim3(grid), dim3(256), 0, s, (knn_s8v *)dst,
                           (const double *)src, n8);
    else if (dtype == KNN_F64)
        hipLaunchKernelGGL(k_wire_unpack<double>, dim3(grid), dim3(256), 0, s, (double *)dst,
                           (const knn_s8v *)src, n8);
    else if (dtype == KNN_F32 && !unpack)
        hipLaunchKernelGGL(k_wire_pack<float>, dim3(grid), dim3(256), 0, s, (knn_s8v *)dst,
                           (const float *)src, n8);
    else if (dtype == KNN_F32)
        hipLaunchKernelGGL(k_wire_unpack<float>, dim3(grid), dim3(256), 0, s, (float *)dst,
                           (const knn_s8v *)src, n8);
    else
        return KNN_ERR_INVALID;
    return hip_status();
}

extern "C" int knn_launch_pack(void *blk, int dtype, size_t cap, size_t rows, size_t n,
                               const void *src, int src_dtype, size_t ld, int layout, void *stream)
{
    hipStream_t s = (hipStream_t)stream;
    if (dtype == KNN_F64 && src_dtype == KNN_F64)
        return launch_pack((double *)blk, cap, rows, n, (const double *)src, ld, layout, s);
    if (dtype == KNN_F64 && src_dtype == KNN_F32)
        return launch_pack((double *)blk, cap, rows, n, (const float *)src, ld, layout, s);
    if (dtype == KNN_F32 && src_dtype == KNN_F64)
        return launch_pack((float *)blk, cap, rows, n, (const double *)src, ld, layout, s);
    if (dtype == KNN_F32 && src_dtype == KNN_F32)
        return launch_pack((float *)blk, cap, rows, n, (const float *)src, ld, layout, s);
    return KNN_ERR_INVALID;
}

template <typename T, int KL, int KP>
static int launch_dist_topk(const T *qblk, size_t q_rows_pad, size_t q_base, int nq, const T *cblk,
                            size_t c_rows_pad, size_t c_base, int nc, int n, const double *meta,
                            int nsplit, double *part_d, int *part_i, double *part_T, int nq_pad,
                            double *qthr, int k, const void *qsh, const void *csh,
                            const void *cn_ptr, int flags, float m2s, hipStream_t s)
{
    const int xord = flags & 1;
    constexpr int dt = sizeof(T) == 8 ? KNN_F64 : KNN_F32;
    const int np = (int)knn_n_pad_dt(n, dt);
    const int nqb = (nq + KNN_TQ - 1) / KNN_TQ;
    const int ntiles = (nc + KNN_TC - 1) / KNN_TC;
    if (nqb <= 0 || nsplit <= 0 || k <= 0 || k > KP) return KNN_ERR_INVALID;
    // lane list slot of the shared bound (k_dist_topk): INT mode the max
    // over lanes covers >= k+1 candidates, GEMM mode >= max(KP, k+1)
    int uj_int = (k + 1 + 3) / 4 - 1;
    if (uj_int > KL - 1) uj_int = KL - 1;
    int uj_gemm = KP / 4 - 1 > uj_int ? KP / 4 - 1 : uj_int;
    // split fp16 filter: its error margin is ~2^-24 relative, not 2^-53, so
    // the published bound sits at the lanes' last entries (more distance
    // between the k-th and the bound for the certificate)
    if (flags & KNN_DIST_SPLIT) uj_gemm = KL - 1;
    if (uj_gemm > KL - 1) uj_gemm = KL - 1;
    const int uj = uj_int | (uj_gemm << 8);
    // geometry checks the kernel relies on (no out-of-bounds staging)
    if ((size_t)nqb * KNN_TQ > q_rows_pad || (size_t)ntiles * KNN_TC > c_rows_pad ||
        nq_pad < nqb * KNN_TQ)
        return KNN_ERR_INVALID;
    const T *qnorm = qblk + q_rows_pad * np;
    const T *cnorm = cn_ptr ? (const T *)cn_ptr : cblk + c_rows_pad * np;
    const int nqb_grid = xord ? (nqb + 7) / 8 * 8 : nqb;
    const dim3 grid((unsigned)(nqb_grid * nsplit));
    if (flags & KNN_DIST_SPLIT) {
        // split fp16 shadow rows (4 bytes a feature); m2s = -2 / S^2 undoes
        // the scaling in the epilogue's fma (a power of two: exact)
        if (!qsh || !csh) return KNN_ERR_INVALID;
        knn_split_blocks_t cb{};
        cb.nblk = 1;
        cb.sp[0] = csh;
        cb.nrm[0] = cnorm;
        cb.base[0] = (int64_t)c_base;
        cb.nc[0] = nc;
        cb.lim[0] = (int)c_rows_pad;
        return knn_launch_dist_split(dt, KL, qsh, qnorm, q_base, nq, &cb, n, meta, nsplit, part_d, part_i, part_T,
                                     nq_pad, qthr, uj, xord, m2s, s);
    }
    if ((flags & KNN_DIST_SHADOW) && (flags & KNN_DIST_H16)) {
        if (!qsh || !csh) return KNN_ERR_INVALID;
        const int nps = (int)knn_round_up((size_t)n, 64);   // shadow row length (halves)
        // shadow rows: waves 0..3 may stage for their SIMD partners too (STG
        // 1; partial lists byte-identical)
        // Every wave stages its own rows (STG 0) for fp64 blocks (mnist 10.0
        // vs 10.1 ms); fp32 (sift) 607 vs 691 ms with waves 0..3 staging.
        if constexpr (sizeof(T) == 8)
            hipLaunchKernelGGL(HIP_KERNEL_NAME(k_dist_topk<T, KL, KP, 0, 2>), grid, dim3(512), 0, s,
                               (const T *)qsh, qnorm, q_base, nq, (const T *)csh, cnorm, c_base, nc, n,
                               nps, ntiles, nsplit, nqb, meta, part_d, part_i, part_T, nq_pad,
                               (unsigned long long *)qthr, uj, xord);
        else
            hipLaunchKernelGGL(HIP_KERNEL_NAME(k_dist_topk<T, KL, KP, 1, 2>), grid, dim3(512), 0, s,
                               (const T *)qsh, qnorm, q_base, nq, (const T *)csh, cnorm, c_base, nc, n,
                               nps, ntiles, nsplit, nqb, meta, part_d, part_i, part_T, nq_pad,
                               (unsigned long long *)qthr, uj, xord);
        return hip_status();
    }
    {
        if (flags & KNN_DIST_H16) {   // host-checked: INT mode and max|x| <= 2048 (fp64: 256)
            hipLaunchKernelGGL(HIP_KERNEL_NAME(k_dist_topk<T, KL, KP, 0, 1>), grid, dim3(512), 0, s,
                               qblk, qnorm, q_base, nq, cblk, cnorm, c_base, nc, n, np, ntiles, nsplit,
                               nqb, meta, part_d, part_i, part_T, nq_pad, (unsigned long long *)qthr,
                               uj, xord);
            return hip_status();
        }
    }
    hipLaunchKernelGGL(HIP_KERNEL_NAME(k_dist_topk<T, KL, KP>), grid, dim3(512), 0, s, qblk, qnorm,
                       q_base, nq, cblk, cnorm, c_base, nc, n, np, ntiles, nsplit, nqb, meta, part_d,
                       part_i, part_T, nq_pad, (unsigned long long *)qthr, uj, xord);
    return hip_status();
}

// The served (element type, state capacity) pairs: fp64 k <= 16, 32 (16-deep
// lane lists); fp32 k <= 16, 32, 128.
#define KNN_DISPATCH(dtype, kp, CALL)                                          \
    do {                                                                       \
        if ((dtype) == KNN_F64 && (kp) == KNN_KP) { CALL(double, KNN_KL, KNN_KP); }       \
        else if ((dtype) == KNN_F64 && (kp) == KNN_KP_M) { CALL(double, KNN_KL, KNN_KP_M); } \
        else if ((dtype) == KNN_F32 && (kp) == KNN_KP) { CALL(float, KNN_KL, KNN_KP); }   \
        else if ((dtype) == KNN_F32 && (kp) == KNN_KP_M) { CALL(float, KNN_KL_M, KNN_KP_M); } \
        else if ((dtype) == KNN_F32 && (kp) == KNN_KP_L) { CALL(float, KNN_KL_L, KNN_KP_L); } \
        else return KNN_ERR_INVALID;                                           \
    } while (0)

extern "C" int knn_launch_dist_topk(int dtype, int kp, int k, const void *qblk, size_t q_rows_pad,
                                    size_t q_base, int nq, const void *cblk, size_t c_rows_pad,
                                    size_t c_base, int nc, int n, const double *meta, int nsplit,
                                    double *part_d, int *part_i, double *part_T, int nq_pad,
                                    double *qthr, const void *qsh, const void *csh,
                                    const void *cn_ptr, int flags, float m2s, void *stream)
{
#define CALL(T, KL, KP)                                                                        \
    return launch_dist_topk<T, KL, KP>((const T *)qblk, q_rows_pad, q_base, nq, (const T *)cblk, \
                                       c_rows_pad, c_base, nc, n, meta, nsplit, part_d, part_i,  \
                                       part_T, nq_pad, qthr, k, qsh, csh, cn_ptr, flags, m2s,     \
                                       (hipStream_t)stream)
    KNN_DISPATCH(dtype, kp, CALL);
#undef CALL
}

// the split filter over a table of element blocks (the engine's fused GEMM
// step): the same lane-list slot of the shared bound and query norms as
// launch_dist_topk's KNN_DIST_SPLIT branch
template <typename T, int KL, int KP>
static int launch_split_n(const T *qblk, size_t q_rows_pad, size_t q_base, int nq, const void *qsp,
                          const knn_split_blocks_t *cb, int n, const double *meta, int nsplit, double *part_d,
                          int *part_i, double *part_T, int nq_pad, double *qthr, int k, int xord, float m2s,
                          hipStream_t s)
{
    constexpr int dt = sizeof(T) == 8 ? KNN_F64 : KNN_F32;
    const int np = (int)knn_n_pad_dt(n, dt);
    const int nqb = (nq + KNN_TQ - 1) / KNN_TQ;
    if (nqb <= 0 || k <= 0 || k > KP || (size_t)nqb * KNN_TQ > q_rows_pad || nq_pad < nqb * KNN_TQ || !qsp)
        return KNN_ERR_INVALID;
    int uj_int = (k + 1 + 3) / 4 - 1;
    if (uj_int > KL - 1) uj_int = KL - 1;
    const int uj = uj_int | ((KL - 1) << 8);
    return knn_launch_dist_split(dt, KL, qsp, qblk + q_rows_pad * np, q_base, nq, cb, n, meta, nsplit, part_d, part_i,
                                 part_T, nq_pad, qthr, uj, xord, m2s, s);
}

extern "C" int knn_launch_dist_split_n(int dtype, int kp, int k, const void *qblk, size_t q_rows_pad, size_t q_base,
                                       int nq, const void *qsp, const knn_split_blocks_t *cb, int n,
                                       const double *meta, int nsplit, double *part_d, int *part_i, double *part_T,
                                       int nq_pad, double *qthr, int xord, float m2s, void *stream)
{
#define CALL(T, KL, KP)                                                                                    \
    return launch_split_n<T, KL, KP>((const T *)qblk, q_rows_pad, q_base, nq, qsp, cb, n, meta, nsplit, part_d, \
                                     part_i, part_T, nq_pad, qthr, k, xord, m2s, (hipStream_t)stream)
    KNN_DISPATCH(dtype, kp, CALL);
#undef CALL
}

extern "C" int knn_launch_merge(int dtype, int kp, int k, const double *part_d, const int *part_i,
                                const double *part_T, int nsplit, int lpq, int kl, int nq, int nq_pad,
                                int first_step, double *st_d, double *st_x, int *st_i,
                                double *st_T, const void *qblk, size_t q_rows_pad,
                                const void *cblk, size_t c_base, int nc, int n,
                                const double *meta, double *qthr, int filt, const int *qperm, void *stream)
{
    knn_merge_blocks_t mb{};
    mb.nblk = 1;
    mb.ptr[0] = cblk;
    mb.base[0] = (int64_t)c_base;
    mb.nc[0] = nc;
    return knn_launch_merge_n(dtype, kp, k, part_d, part_i, part_T, nsplit, lpq, kl, nq, nq_pad, first_step, st_d,
                              st_x, st_i, st_T, qblk, q_rows_pad, &mb, n, meta, qthr, filt, qperm, stream);
}

extern "C" int knn_launch_merge_n(int dtype, int kp, int k, const double *part_d, const int *part_i,
                                  const double *part_T, int nsplit, int lpq, int kl, int nq, int nq_pad,
                                  int first_step, double *st_d, double *st_x, int *st_i, double *st_T,
                                  const void *qblk, size_t q_rows_pad, const knn_merge_blocks_t *mbp, int n,
                                  const double *meta, double *qthr, int filt, const int *qperm, void *stream)
{
    if (!mbp || mbp->nblk < 1 || mbp->nblk > KNN_SPLIT_MAXBLK) return KNN_ERR_INVALID;
    const knn_merge_blocks_t mb = *mbp;
    if (lpq < 1 || kl < 1 || lpq * nsplit + 1 > 64 || k <= 0 || k > kp) return KNN_ERR_INVALID;
    const int np = (int)knn_n_pad_dt(n, dtype);
    const size_t qn_off = q_rows_pad * (size_t)np;
    // prefetched heads (KP = 32: the state as 4 runs of 8) when the lists
    // and state lanes fit; two queries a wave when they fit 32 lanes
    const int pf = kp == 32 && kl >= 8 && lpq * nsplit + 4 <= 64;
    const int two = lpq * nsplit + (pf ? 4 : 1) <= 32;
    const dim3 grid((unsigned)((nq + (two ? 7 : 3)) / (two ? 8 : 4)));
    hipStream_t s = (hipStream_t)stream;
#define CALL(T, KL, KP)                                                                          \
    if (pf && KP == 32 && two)                                                                   \
        hipLaunchKernelGGL(HIP_KERNEL_NAME(k_merge<T, 32, 32, 8>), grid, dim3(256), 0, s, part_d,  \
                           part_i, part_T, nsplit, lpq, kl, nq, nq_pad, first_step, st_d, st_x,    \
                           st_i, st_T, (const T *)qblk, qn_off, mb, n,                             \
                           np, meta, k, (unsigned long long *)qthr, filt, qperm);                         \
    else if (pf && KP == 32)                                                                     \
        hipLaunchKernelGGL(HIP_KERNEL_NAME(k_merge<T, 32, 64, 8>), grid, dim3(256), 0, s, part_d,  \
                           part_i, part_T, nsplit, lpq, kl, nq, nq_pad, first_step, st_d, st_x,    \
                           st_i, st_T, (const T *)qblk, qn_off, mb, n,                             \
                           np, meta, k, (unsigned long long *)qthr, filt, qperm);                         \
    else if (two)                                                                                \
        hipLaunchKernelGGL(HIP_KERNEL_NAME(k_merge<T, KP, 32>), grid, dim3(256), 0, s, part_d,     \
                           part_i, part_T, nsplit, lpq, kl, nq, nq_pad, first_step, st_d, st_x,    \
                           st_i, st_T, (const T *)qblk, qn_off, mb, n,                             \
                           np, meta, k, (unsigned long long *)qthr, filt, qperm);                         \
    else                                                                                         \
        hipLaunchKernelGGL(HIP_KERNEL_NAME(k_merge<T, KP, 64>), grid, dim3(256), 0, s, part_d,     \
                           part_i, part_T, nsplit, lpq, kl, nq, nq_pad, first_step, st_d, st_x,    \
                           st_i, st_T, (const T *)qblk, qn_off, mb, n,                             \
                           np, meta, k, (unsigned long long *)qthr, filt, qperm);                         \
    return hip_status()
    KNN_DISPATCH(dtype, kp, CALL);
#undef CALL
}

extern "C" int knn_launch_merge_rank(int dtype, int kp, int kl, int k, const double *part_d, const int *part_i,
                                     const double *part_T, int nsplit, int lpq, int nq, int nq_pad,
                                     int first_step, double *st_d, double *st_x, int *st_i, double *st_T,
                                     double *qthr, knn_neighbour_t *fin_out, int *fail_count, int *fail_list,
                                     int *mode_out, double *fbound, const double *meta, int n, int force_fail,
                                     void *stream)
{
    knn_fin_args fa;
    fa.out = fin_out;
    fa.fail_count = fail_count;
    fa.fail_list = fail_list;
    fa.mode_out = mode_out;
    fa.fbound = fbound;
    fa.meta = meta;
    fa.n = n;
    fa.lim = 2251799813685248.0 / (4.0 * (double)n);
    fa.force_fail = force_fail;
    const int fin = fin_out != nullptr;
    if (lpq < 1 || nsplit < 1 || lpq * nsplit > 64 || k <= 0 || k > kp || kp > 64 || nsplit > 64 ||
        (kl != KNN_I8_KL_S && kl != KNN_I8_KL))
        return KNN_ERR_INVALID;
#ifndef KNN_NO_RANK16
    if (fin && first_step && lpq * nsplit <= 16) {
        // the search's only merge (P = 1): 16 lanes a query
        const dim3 g16((unsigned)((nq + 15) / 16));
        hipStream_t s16 = (hipStream_t)stream;
#define RANK16(T, KL)                                                                              \
        hipLaunchKernelGGL(HIP_KERNEL_NAME(k_merge_rank16<T, KL>), g16, dim3(256), 0, s16, part_d, part_i, \
                           part_T, nsplit, lpq, nq, nq_pad, k, (unsigned long long *)qthr, fa)
        if (dtype == KNN_F64 && kl == KNN_I8_KL_S) RANK16(double, KNN_I8_KL_S);
        else if (dtype == KNN_F64) RANK16(double, KNN_I8_KL);
        else if (kl == KNN_I8_KL_S) RANK16(float, KNN_I8_KL_S);
        else RANK16(float, KNN_I8_KL);
#undef RANK16
        return hip_status();
    }
#endif
    const int cap = (lpq * nsplit * kl + kp + 1) & ~1;   // every candidate; 16-byte rows
    const size_t lds = 4 * (size_t)cap * sizeof(unsigned long long);
    const dim3 grid((unsigned)((nq + 3) / 4));
    hipStream_t s = (hipStream_t)stream;
#define RANK(T, KP, KL)                                                                            \
    hipLaunchKernelGGL(HIP_KERNEL_NAME(k_merge_rank<T, KP, KL>), grid, dim3(256), lds, s, part_d, part_i, \
                       part_T, nsplit, lpq, nq, nq_pad, first_step, st_d, st_x, st_i, st_T, k,       \
                       (unsigned long long *)qthr, cap, fin, fa)
    if (dtype == KNN_F64 && kp == KNN_KP && kl == KNN_I8_KL_S) RANK(double, KNN_KP, KNN_I8_KL_S);
    else if (dtype == KNN_F64 && kp == KNN_KP) RANK(double, KNN_KP, KNN_I8_KL);
    else if (dtype == KNN_F64 && kp == KNN_KP_M && kl == KNN_I8_KL_S) RANK(double, KNN_KP_M, KNN_I8_KL_S);
    else if (dtype == KNN_F64 && kp == KNN_KP_M) RANK(double, KNN_KP_M, KNN_I8_KL);
    else if (dtype == KNN_F32 && kp == KNN_KP && kl == KNN_I8_KL_S) RANK(float, KNN_KP, KNN_I8_KL_S);
    else if (dtype == KNN_F32 && kp == KNN_KP) RANK(float, KNN_KP, KNN_I8_KL);
    else if (dtype == KNN_F32 && kp == KNN_KP_M && kl == KNN_I8_KL_S) RANK(float, KNN_KP_M, KNN_I8_KL_S);
    else if (dtype == KNN_F32 && kp == KNN_KP_M) RANK(float, KNN_KP_M, KNN_I8_KL);
    else return KNN_ERR_INVALID;
#undef RANK
    return hip_status();
}

extern "C" int knn_launch_finalize(int dtype, int kp, const double *st_d, const double *st_x,
                                   const int *st_i, const double *st_T, const void *qblk,
                                   size_t q_rows_pad, int nq, int n, int k, const double *meta,
                                   knn_neighbour_t *out, int *fail_count, int *fail_list,
                                   int *mode_out, double *fbound, int force_fail, int filt, void *stream)
{
    if (k <= 0 || k > kp) return KNN_ERR_INVALID;
    const size_t off = q_rows_pad * knn_n_pad_dt(n, dtype);
    const dim3 grid((unsigned)((nq + 3) / 4));
    hipStream_t s = (hipStream_t)stream;
#define CALL(T, KL, KP)                                                                        \
    hipLaunchKernelGGL(HIP_KERNEL_NAME(k_finalize<T, KP>), grid, dim3(256), 0, s, st_d, st_x,   \
                       st_i, st_T, qblk ? (const T *)qblk + off : nullptr, nq, n, k, meta, out,  \
                       fail_count,                                                               \
                       fail_list, mode_out, fbound, force_fail, filt);                           \
    return hip_status()
    KNN_DISPATCH(dtype, kp, CALL);
#undef CALL
}

extern "C" int knn_launch_rescan_init(int kp, double *rs_d, int *rs_i, int nfail, void *stream)
{
    const int cnt = nfail * kp;
    if (cnt <= 0) return KNN_OK;
    hipLaunchKernelGGL(k_rescan_init, dim3((unsigned)((cnt + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, rs_d, rs_i, cnt);
    return hip_status();
}

extern "C" int knn_launch_rescan_step(int dtype, int kp, const int *fail_list, int nfail,
                                      const double *fbound, const void *qblk, const void *cblk,
                                      size_t c_base, int nc, int n, int k, double *rs_d,
                                      int *rs_i, void *stream)
{
    if (nfail <= 0) return KNN_OK;
    if (k <= 0 || k > kp || nc <= 0) return KNN_ERR_INVALID;
    const int np = (int)knn_n_pad_dt(n, dtype);
    hipStream_t s = (hipStream_t)stream;
    // Few uncertified queries give few workgroups (16 queries each): split
    // the block's rows over C chunks too (knn_rescan_chunks; the caller
    // sized rs_d/rs_i for 1 + C list sets), then merge the chunk lists.
    int C = knn_rescan_chunks(nfail);
    const int min_rows = 256;
    if (C > (nc + min_rows - 1) / min_rows) C = (nc + min_rows - 1) / min_rows;
    if (C < 1) C = 1;
    const int rpc = (nc + C - 1) / C;
    C = (nc + rpc - 1) / rpc;
    const size_t stride = (size_t)nfail * kp;
    if (C > 1) {
        hipLaunchKernelGGL(k_rescan_init, dim3((unsigned)((C * stride + 255) / 256)), dim3(256), 0, s,
                           rs_d + stride, rs_i + stride, (int)(C * stride));
    }
    double *ld = C > 1 ? rs_d + stride : rs_d;
    int *li = C > 1 ? rs_i + stride : rs_i;
#define CALL(T, KL, KP)                                                                          \
    hipLaunchKernelGGL(HIP_KERNEL_NAME(k_rescan_step<T, KP>),                                    \
                       dim3((unsigned)((nfail + 15) / 16), (unsigned)C), dim3(256), 0, s,         \
                       fail_list, nfail, fbound, (const T *)qblk, np, (const T *)cblk, c_base, nc, \
                       n, np, k, rs_d, ld, li, rpc, C > 1 ? stride : 0);                          \
    if (C > 1)                                                                                   \
        hipLaunchKernelGGL(HIP_KERNEL_NAME(k_rescan_merge<KP>), dim3((unsigned)((nfail + 3) / 4)), \
                           dim3(256), 0, s, nfail, k, C, rs_d, rs_i);                            \
    return hip_status()
    KNN_DISPATCH(dtype, kp, CALL);
#undef CALL
}

extern "C" int knn_launch_rescan_end(int kp, const int *fail_list, int nfail, const double *rs_d,
                                     const int *rs_i, int k, knn_neighbour_t *out, void *stream)
{
    const int cnt = nfail * k;
    if (cnt <= 0) return KNN_OK;
    hipLaunchKernelGGL(k_rescan_end, dim3((unsigned)((cnt + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, fail_list, nfail, kp, rs_d, rs_i, k, out);
    return hip_status();
}

// ---------------------------------------------------------------------------
// k_vote: the label vote + accuracy stage on the device (knn_classify_device;
// host twin knn_vote.c, same rules).  One wave per query: the k neighbour
// labels are counted into the wave's LDS histogram (nclasses <= 1024), lane
// 0 walks the classes in label order exactly like serial:121-124 /
// blk:263-266 (SERIAL / MPI, with their count-vs-label quirk) or
// takes a true majority (MAJORITY), then compares with the query's own
// label (serial:126-127).  The neighbour records get their .label filled
// (blk:176).  Empty slots and idx > nlabels are skipped.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_vote(knn_neighbour_t *__restrict__ nb, int m, int k,
                                              int nclasses, int rule,
                                              const double *__restrict__ labels,
                                              long long nlabels, long long q_base,
                                              int *__restrict__ pred,
                                              unsigned long long *__restrict__ matches)
{
    __shared__ int cls[4][KNN_VOTE_MAX_CLASSES];
    __shared__ unsigned hits[4];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int q = blockIdx.x * 4 + wave;
    int *c = cls[wave];
    for (int j = lane; j < nclasses; j += 64) c[j] = 0;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    unsigned hit = 0;
    if (q < m) {
        knn_neighbour_t *L = nb + (size_t)q * k;
        for (int i = lane; i < k; i += 64) {
            const int id = L[i].idx;
            int lab = 0;
            if (id > 0 && id <= nlabels) {
                lab = (int)labels[id - 1];
                L[i].label = lab;
                if (lab >= 1 && lab <= nclasses) atomicAdd(&c[lab - 1], 1);
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        if (lane == 0) {
            int most = 0;
            if (rule == KNN_VOTE_MAJORITY) {
                int best = 0;
                for (int j = 0; j < nclasses; j++) best = c[j] > best ? c[j] : best;
                for (int i = 0; i < k && best > 0; i++) {
                    const int id = L[i].idx;
                    if (id <= 0 || id > nlabels) continue;
                    const int lab = (int)labels[id - 1];
                    if (lab >= 1 && lab <= nclasses && c[lab - 1] == best) {
                        most = lab;
                        break;
                    }
                }
            } else {
                const int id0 = L[0].idx;
                const int nn0 = (id0 > 0 && id0 <= nlabels) ? (int)labels[id0 - 1] : 0;
                const int tie = rule == KNN_VOTE_MPI ? nn0 - 1 : nn0;
                for (int j = 0; j < nclasses; j++)
                    if (c[j] > most || (c[j] == most && (j + 1) == tie)) most = j + 1;
            }
            if (pred) pred[q] = most;
            const long long g = q_base + q;
            hit = (g < nlabels && (double)most == labels[g]) ? 1u : 0u;
        }
    }
    if (lane == 0) hits[wave] = hit;
    __syncthreads();
    if (threadIdx.x == 0 && matches) {
        const unsigned h = hits[0] + hits[1] + hits[2] + hits[3];
        if (h) atomicAdd(matches, (unsigned long long)h);
    }
}

extern "C" int knn_launch_vote(knn_neighbour_t *nb, size_t m, int k, int nclasses, int rule,
                               const double *labels, size_t nlabels, size_t q_base, int *pred,
                               unsigned long long *matches, void *stream)
{
    if (m == 0) return KNN_OK;
    if (nclasses > KNN_VOTE_MAX_CLASSES || m > 0x7fffffffULL) return KNN_ERR_UNSUPPORTED;
    hipStream_t s = (hipStream_t)stream;
    if (matches && hipMemsetAsync(matches, 0, sizeof(unsigned long long), s) != hipSuccess)
        return KNN_ERR_HIP;
    hipLaunchKernelGGL(k_vote, dim3((unsigned)((m + 3) / 4)), dim3(256), 0, s, nb, (int)m, k,
                       nclasses, rule, labels, (long long)nlabels, (long long)q_base, pred, matches);
    return hip_status();
}
