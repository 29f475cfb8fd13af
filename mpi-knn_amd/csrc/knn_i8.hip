// knn_i8.hip -- int8 MFMA contraction for 8-bit-window integer data.
//
// The distance stage of knn-serial.c:72-93 (and blk:155-181, 217-242) on
// data whose values are integers inside a window of 256 (MNIST pixels 0..255,
// SIFT descriptors): x' = x - o with o = lo + 128 (lo = the reduced meta's
// lower bound) is an exact int8, every product and every partial sum of
// q'.c' an exact int32 (|q'.c'| <= n 2^14), and
//     d^2 = |q'|^2 + |c'|^2 - 2 q'.c'
// is the reference's S bit for bit (S is an exact integer below 2^53 for such
// data; the shift cancels in every difference).  v_mfma_i32_32x32x32_i8
// runs at twice the fp16 rate and moves half its bytes.
//
//   k_shadow8          element block -> byte block: rows of x' (round_up(n,32)
//                      bytes) + |x'|^2 as int32 in the per-tile order the
//                      epilogue reads (i8_norm_pos) + the block's meta.
//   k_dist_topk_i8     fused contraction + per-lane top-KL (int32 keys).
//
// Layout and roofline notes: DESIGN.md sec.4.
#include "knn_device.h"

typedef int knn_v16i __attribute__((ext_vector_type(16)));

#define I8_NST 4                 // corpus stages in the LDS ring
#define I8_INF 0x7fffffff        // empty list slot / no bound

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

// a where the lane's bit of m is clear, b where it is set
__device__ __forceinline__ int i8_sel(unsigned long long m, int a, int b)
{
    int r;
    asm("v_cndmask_b32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(m));
    return r;
}

// One wave per row: x' = x - o (0 past n), 16 bytes a lane, |x'|^2 reduced
// in int32 (exact: n * 128^2 < 2^31).  o from the REDUCED meta, so every
// block of one search shifts alike.
template <typename T>
__global__ __launch_bounds__(256) void k_shadow8(signed char *__restrict__ dst, const T *__restrict__ src,
                                                 size_t rows_pad, int n, int nps, int rs,
                                                 const double *__restrict__ meta)
{
    int *norms = (int *)(dst + rows_pad * (size_t)rs);
    const int off = 128 - (int)meta[KNN_META_MAXNEG];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (size_t r = (size_t)blockIdx.x * 4 + wave; r < rows_pad; r += (size_t)gridDim.x * 4) {
        const T *x = src + r * (size_t)nps;
        int s = 0;
        for (int c0 = lane * 16; c0 < rs; c0 += 1024) {
            unsigned w[4];
#pragma unroll
            for (int e = 0; e < 4; e++) {
                unsigned word = 0;
#pragma unroll
                for (int y = 0; y < 4; y++) {
                    const int j = c0 + 4 * e + y;
                    const int v = j < n ? (int)x[j] - off : 0;
                    s += v * v;
                    word |= ((unsigned)v & 0xffu) << (8 * y);
                }
                w[e] = word;
            }
            *(knn_v4i *)(dst + r * (size_t)rs + c0) = (knn_v4i){(int)w[0], (int)w[1], (int)w[2], (int)w[3]};
        }
        for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
        if (lane == 0) norms[i8_norm_pos((int)r)] = s;
    }
}

// ---------------------------------------------------------------------------
// k_dist_topk_i8
//
// Workgroup: 256 threads = 4 waves, one per SIMD; 128 queries (wave w:
// queries 32w..32w+31) x a corpus split streamed in tiles of 128 rows and
// chunks of 128 bytes (128 features, 4 K-steps of 32).
//
// Operands (v_mfma_i32_32x32x32_i8, D = A.B): A = 32 corpus rows (m-block
// b of the tile), B = the wave's 32 queries; lane l (r = l & 31, h = l >> 5)
// supplies 16 bytes [32 s + 16 h, +16) of K-step s of row r / query r -- the
// same byte slots on both sides, so the sum runs over every feature once.
// D: lane l holds query r, rows 32b + 8(reg >> 2) + 4h + (reg & 3).  Each
// query's 128 candidates of a tile sit in 2 lanes (h = 0, 1), 64 each; the
// two lanes keep separate lists over disjoint rows and share a bound.
//
// Queries are resident in registers for the whole split (4 VGPRs per K-step,
// loaded once); the corpus streams through an I8_NST-stage LDS ring of 16 KiB
// images filled by LDS-DMA (buffer_load_dwordx4 ... lds): wave w stages rows
// 32w..32w+31 as 4 pieces of 8 rows x 128 B.  Image of a tile chunk: [row
// 128][128 B], 16-byte segment s of row r at slot s ^ ((r >> 1) & 7) -- the
// ds_read_b128 lane groups ({0-3,12-15,20-27}, ...) then hit 16 distinct
// bank quads.  One barrier per chunk: before it each wave waits for its own
// pieces of the chunk (counted vmcnt: the pieces of the next I8_NST - 2
// chunks stay in flight), after it the stage freed by the previous chunk is
// refilled.  Chunks past the split's end re-stage its last chunk, so every
// chunk issues the same corpus pieces and the count is static.  The tile's
// norms (512 B, permuted, i8_norm_pos) ride with its first chunk into a
// norm ring indexed by tile % I8_NST (norm pieces only make the count more
// conservative).
//
// Epilogue per tile: key = |c'|^2 - 2 q'.c' (int32), one masked-free test of
// the lane minimum against min(own KL-th, shared bound) - |q'|^2, then the
// survivors per m-block (lowest row first: the stable tie order) through a
// 4-level select tree into the KL-entry insertion network.  d^2 = key + |q'|^2
// is exact, so "S != 0" (serial:86) is d^2 > 0.
// ---------------------------------------------------------------------------
template <int KL, int NC, int WPS>
__global__ __launch_bounds__(256, WPS) void k_dist_topk_i8(
    const signed char *__restrict__ qsh, size_t q_rows_pad, size_t q_base, int nq,
    const signed char *__restrict__ csh, size_t c_rows_pad, size_t c_base, int nc, int rs,
    int nks, int ntiles, int nsplit, int nqb, double *__restrict__ part_d,
    int *__restrict__ part_i, double *__restrict__ part_T, int nq_pad,
    unsigned long long *__restrict__ qthr, int uj)
{
    constexpr int NST = I8_NST;
    __shared__ __attribute__((aligned(16))) char smem[NST * 16384 + NST * 512];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int wave_s = __builtin_amdgcn_readfirstlane(wave);
    const int r32 = lane & 31, h = lane >> 5;
    const int qb = blockIdx.x % nqb, split = blockIdx.x / nqb;
    // long splits first (split-major dispatch, knn_engine.c: choose_splits)
    const int tb = ntiles / nsplit, tr = ntiles - tb * nsplit;
    const int t_lo = split * tb + (split < tr ? split : tr);
    const int t_hi = t_lo + tb + (split < tr ? 1 : 0);
    const int qrow0 = qb * 128;
    const int myq = qrow0 + 32 * wave + r32;
    const long gq = (long)q_base + myq;
    const int nch = (nks + 3) >> 2;
    const int *qnorms = (const int *)(qsh + q_rows_pad * (size_t)rs);
    const int *cnorms = (const int *)(csh + c_rows_pad * (size_t)rs);

    // ---- resident query fragments (B), one per K-step --------------------
    // (address clamped to the last real K-step: never past the row's block)
    knn_v4i qf[4 * NC];
    {
        const signed char *qrow = qsh + (size_t)myq * rs + 16 * h;
#pragma unroll
        for (int s = 0; s < 4 * NC; s++) {
            const int sl = s < nks ? s : nks - 1;
            qf[s] = *(const knn_v4i *)(qrow + 32 * sl);
        }
    }
    const int qn = qnorms[i8_norm_pos(myq)];
    // shared per-query bound across splits and ring steps (qthr: bits of a
    // non-negative double, atomicMin).  INT-mode bounds are integers, or the
    // next double above one (strict publication), so floor() is the int bound.
    int thr = I8_INF;
    if (qthr != nullptr && myq < nq) {
        const double td = __longlong_as_double((long long)atomicMin(qthr + myq, 0x7ff0000000000000ull));
        thr = td >= 2147483647.0 ? I8_INF : (int)td;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

    int L[KL], I[KL];
#pragma unroll
    for (int e = 0; e < KL; e++) { L[e] = I8_INF; I[e] = -1; }
    const int ujm = uj < KL - 1 ? uj : KL - 1;

    // ---- staging cursor ----------------------------------------------------
    const int total = (t_hi > t_lo) ? (t_hi - t_lo) * nch : 0;
    unsigned voff[4];
#pragma unroll
    for (int p = 0; p < 4; p++) {
        const int rr = 32 * wave_s + 8 * p + (lane >> 3);
        voff[p] = (unsigned)(rr * rs + 16 * ((lane & 7) ^ ((rr >> 1) & 7)));
    }
    const unsigned lds0 = (unsigned)(uintptr_t)smem;
    int s_t = t_lo, s_c = 0, s_x = 0;
    auto stage = [&]() {
        const signed char *base = csh + (size_t)s_t * 128 * rs + 128 * s_c;
        const knn_v4i rsrc = knn_rsrc(base);
        const unsigned dst = lds0 + (unsigned)(s_x & (NST - 1)) * 16384u + (unsigned)wave_s * 4096u;
#pragma unroll
        for (int p = 0; p < 4; p++) bglds16(rsrc, voff[p], dst + 1024u * p);
        if (s_x < total && s_c == 0) {
            if (lane < 8)
                bglds16(knn_rsrc(cnorms + (size_t)s_t * 128 + 32 * wave_s), 16u * lane,
                        lds0 + NST * 16384u + (unsigned)(s_t & (NST - 1)) * 512u + 128u * wave_s);
        }
        s_x++;
        if (s_x < total) {
            if (++s_c == nch) {
                s_c = 0;
                s_t++;
            }
        }
    };

    // ---- epilogue of tile t -------------------------------------------------
    auto epilogue = [&](int t, knn_v16i (&A)[4]) {
        const LDS_AS knn_v4i *cn =
            (const LDS_AS knn_v4i *)((LDS_AS char *)smem + NST * 16384 + (t & (NST - 1)) * 512) + 4 * h;
        const int lim = L[KL - 1] < thr ? L[KL - 1] : thr;
        const int limq = lim == I8_INF ? I8_INF : lim - qn;
        int lmn = I8_INF;
#pragma unroll
        for (int b = 0; b < 4; b++) {
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const knn_v4i c4 = cn[8 * b + j];
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const int v = c4[i] - 2 * A[b][4 * j + i];
                    A[b][4 * j + i] = v;
                    lmn = v < lmn ? v : lmn;
                }
            }
        }
        const int row0 = t * 128;
        const long gt0 = (long)c_base + row0, gw0 = (long)q_base + qrow0 + 32 * wave_s;
        const bool masked = (row0 + 128 > nc) || (gw0 < gt0 + 128 && gt0 < gw0 + 32);
        if (!masked && __ballot(lmn <= limq) == 0ull) return;   // common late in the scan
#pragma unroll
        for (int b = 0; b < 4; b++) {
            unsigned pend = 0;
#pragma unroll
            for (int r = 0; r < 16; r++) pend |= (A[b][r] <= limq) ? (1u << r) : 0u;
            if (masked) {
#pragma unroll
                for (int r = 0; r < 16; r++) {
                    const int row = row0 + 32 * b + 8 * (r >> 2) + 4 * h + (r & 3);
                    if (!(row < nc && (long)c_base + row != gq)) pend &= ~(1u << r);
                }
            }
            while (__ballot(pend != 0) != 0ull) {
                const int r = pend ? __builtin_ctz(pend) : 0;
                // 4-level select tree on the bits of r, written as v_cndmask
                // on ballot masks: as plain selects LLVM folds the tree into a
                // dynamic index (a scratch round trip per round)
                const unsigned long long m0 = __ballot(r & 1), m1 = __ballot(r & 2),
                                         m2 = __ballot(r & 4), m3 = __ballot(r & 8);
                int v[8], w[4];
#pragma unroll
                for (int y = 0; y < 8; y++) v[y] = i8_sel(m0, A[b][2 * y], A[b][2 * y + 1]);
#pragma unroll
                for (int y = 0; y < 4; y++) w[y] = i8_sel(m1, v[2 * y], v[2 * y + 1]);
                const int x0 = i8_sel(m2, w[0], w[1]), x1 = i8_sel(m2, w[2], w[3]);
                const int d2 = i8_sel(m3, x0, x1) + qn;
                // d^2 == 0: an exact duplicate (S == 0, excluded by serial:86)
                const int dd = (pend && d2 > 0) ? d2 : I8_INF;
                const int id = (int)(c_base + row0 + 32 * b + 8 * (r >> 2) + 4 * h + (r & 3));
                pend &= pend - 1;
                list_insert<KL>(L, I, dd, id);
            }
        }
        // bound shared by the query's 2 lanes: their union holds >= 2(ujm+1)
        // >= k+1 entries <= max_h L_h[ujm]; each already rejects >= its L[KL-1]
        int lmin = L[KL - 1], u = L[0];
#pragma unroll
        for (int e = 1; e < KL; e++) u = (e == ujm) ? L[e] : u;
        const int lo = __shfl_xor(lmin, 32), uo = __shfl_xor(u, 32);
        lmin = lo < lmin ? lo : lmin;
        u = uo > u ? uo : u;
        const int nb = lmin < u ? lmin : u;
        thr = nb < thr ? nb : thr;
    };

    if (total > 0) {
#pragma unroll
        for (int x = 0; x < NST - 1; x++) stage();
        int x = 0;
        for (int t = t_lo; t < t_hi; t++) {
            knn_v16i acc[4];
#pragma unroll
            for (int b = 0; b < 4; b++)
#pragma unroll
                for (int i = 0; i < 16; i++) acc[b][i] = 0;
#pragma unroll
            for (int c = 0; c < NC; c++) {
                if (c < nch) {
                    // own pieces of chunk x landed (those of the next NST-2
                    // chunks may stay in flight); then every wave's
                    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
                    __builtin_amdgcn_s_barrier();
                    stage();   // chunk x + NST - 1 into the stage chunk x - 1 freed
                    const LDS_AS char *st = (const LDS_AS char *)smem + (x & (NST - 1)) * 16384 +
                                            r32 * 128;
#pragma unroll
                    for (int s = 0; s < 4; s++) {
                        if (4 * c + s < nks) {
                            const int slot = 16 * ((2 * s + h) ^ ((r32 >> 1) & 7));
                            knn_v4i a[4];
#pragma unroll
                            for (int b = 0; b < 4; b++)
                                a[b] = *(const LDS_AS knn_v4i *)(st + b * 4096 + slot);
#pragma unroll
                            for (int b = 0; b < 4; b++)
                                acc[b] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[b], qf[4 * c + s], acc[b], 0,
                                                                               0, 0);
                        }
                    }
                    x++;
                }
            }
            epilogue(t, acc);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no LDS-DMA left in flight
    }

    // strict publication (INT mode, exact keys): if neither lane's list ends
    // at thr, nothing equal to thr was turned away, so every rejected
    // candidate has d^2 >= next(thr) (k_finalize certifies tau < T)
    int lastmin = L[KL - 1];
    {
        const int o = __shfl_xor(lastmin, 32);
        lastmin = o < lastmin ? o : lastmin;
    }
    double pub = thr == I8_INF ? KNN_INF : (double)thr;
    if (lastmin > thr && thr < I8_INF) pub = nextafter((double)thr, KNN_INF);
    if (myq < nq) {
        const size_t base = (((size_t)split * nq_pad + myq) * 2 + h) * KL;
#pragma unroll
        for (int e = 0; e < KL; e++) {
            part_d[base + e] = L[e] == I8_INF ? KNN_INF : (double)L[e];
            part_i[base + e] = I[e];
        }
        if (h == 0) {
            part_T[(size_t)split * nq_pad + myq] = pub;
            if (qthr != nullptr && thr < I8_INF)
                atomicMin(qthr + myq, (unsigned long long)__double_as_longlong((double)thr));
        }
    }
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
extern "C" int knn_launch_shadow8(void *dst, const void *blk, int dtype, size_t rows_pad, size_t n,
                                  const double *meta, void *stream)
{
    const int rs = (int)knn_s8_rs(n), nps = (int)knn_n_pad_dt(n, dtype);
    const unsigned grid = (unsigned)(rows_pad / 4 + 1 < 8192 ? rows_pad / 4 + 1 : 8192);
    hipStream_t s = (hipStream_t)stream;
    if (dtype == KNN_F64)
        hipLaunchKernelGGL(k_shadow8<double>, dim3(grid), dim3(256), 0, s, (signed char *)dst,
                           (const double *)blk, rows_pad, (int)n, nps, rs, meta);
    else if (dtype == KNN_F32)
        hipLaunchKernelGGL(k_shadow8<float>, dim3(grid), dim3(256), 0, s, (signed char *)dst,
                           (const float *)blk, rows_pad, (int)n, nps, rs, meta);
    else
        return KNN_ERR_INVALID;
    return hipGetLastError() == hipSuccess ? KNN_OK : KNN_ERR_HIP;
}

template <int KL, int NC, int WPS>
static void launch_i8(dim3 grid, hipStream_t s, const void *qsh, size_t q_rows_pad, size_t q_base,
                      int nq, const void *csh, size_t c_rows_pad, size_t c_base, int nc, int rs,
                      int nks, int ntiles, int nsplit, int nqb, double *part_d, int *part_i,
                      double *part_T, int nq_pad, double *qthr, int uj)
{
    hipLaunchKernelGGL(HIP_KERNEL_NAME(k_dist_topk_i8<KL, NC, WPS>), grid, dim3(256), 0, s,
                       (const signed char *)qsh, q_rows_pad, q_base, nq, (const signed char *)csh,
                       c_rows_pad, c_base, nc, rs, nks, ntiles, nsplit, nqb, part_d, part_i, part_T,
                       nq_pad, (unsigned long long *)qthr, uj);
}

extern "C" int knn_launch_dist_i8(int kp, int k, const void *qsh, size_t q_rows_pad, size_t q_base,
                                  int nq, const void *csh, size_t c_rows_pad, size_t c_base, int nc,
                                  int n, int nsplit, double *part_d, int *part_i, double *part_T,
                                  int nq_pad, double *qthr, void *stream)
{
    const int rs = (int)knn_s8_rs((size_t)n), nks = rs / 32, nch = (nks + 3) / 4;
    const int nqb = (nq + 127) / 128, ntiles = (nc + 127) / 128;
    const int kl = knn_i8_kl(kp);
    if (nqb <= 0 || nsplit <= 0 || k <= 0 || k > kp || kl <= 0 || nch > 7) return KNN_ERR_INVALID;
    if ((size_t)nqb * 128 > q_rows_pad || (size_t)ntiles * 128 > c_rows_pad || nq_pad < nqb * 128)
        return KNN_ERR_INVALID;
    // lane-list slot of the shared bound: the 2 lanes of a query cover k + 1
    int uj = (k + 1 + 1) / 2 - 1;
    if (uj > kl - 1) uj = kl - 1;
    const dim3 grid((unsigned)(nqb * nsplit));
    hipStream_t s = (hipStream_t)stream;
#define I8_ARGS grid, s, qsh, q_rows_pad, q_base, nq, csh, c_rows_pad, c_base, nc, rs, nks, ntiles, nsplit, \
                nqb, part_d, part_i, part_T, nq_pad, qthr, uj
    if (nch == 1) {
        if (kl == KNN_I8_KL) launch_i8<KNN_I8_KL, 1, 2>(I8_ARGS);
        else launch_i8<KNN_I8_KL_L, 1, 1>(I8_ARGS);
    } else {
        if (kl == KNN_I8_KL) launch_i8<KNN_I8_KL, 7, 1>(I8_ARGS);
        else launch_i8<KNN_I8_KL_L, 7, 1>(I8_ARGS);
    }
#undef I8_ARGS
    return hipGetLastError() == hipSuccess ? KNN_OK : KNN_ERR_HIP;
}
