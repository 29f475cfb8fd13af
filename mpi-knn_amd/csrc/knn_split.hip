// knn_split.hip -- the split-fp16 filter kernel of real-valued searches
// (GEMM mode, fp32 and fp64 blocks): the distance loop of knn-serial.c:72-93
// as a tiled contraction, each value held as S x = hi + lo in fp16
// (k_shadow_split) and hi.hi + hi.lo + lo.hi contracted on
// v_mfma_f32_16x16x32_f16, followed by the per-lane top-KL lists of
// k_dist_topk (knn_kernels.hip).  The lists, the exact reference-order
// re-rank in k_merge and the certificate (knn_cert_E, split) are the GEMM
// mode's, so every reported distance is the reference's S, bit for bit.
//
// Why a kernel of its own (round 5): k_dist_topk's workgroup streams 128
// corpus rows against its 128 queries and re-stages the queries for every
// 128-row tile.  The queries of a workgroup are its own (no other workgroup
// reads them), so every re-stage misses L2: gist (500K x 960) fetched 10.8
// TB a launch against a 1.92 GB corpus and ran at the fabric's rate.  Here a
// tile is 256 rows, so each staged query chunk meets twice the rows:
//
//   workgroup 512 threads = 8 waves, 128 queries (wave w: queries 16w..+15);
//   tile = 256 corpus rows = 16 m-tiles of 16; a wave computes its 16
//   queries against all 16 m-tiles (64 fp32 accumulators a lane);
//   chunk = 128 bytes of every row (32 features: 32 hi then 32 lo halves);
//   LDS stage = 32 KiB of corpus rows, 4 stages filled by LDS-DMA (each
//   wave stages its own 2 m-tiles: 4 `buffer_load_dwordx4 ... lds` a
//   chunk), a ring of 4 norm slices (256 norms each) two tiles ahead; the
//   query B fragments go straight to registers (global_load_dwordx4, one
//   chunk ahead: a wave's queries are read by no other wave), 136 KiB.
//
// Accumulation (the error bound knn_cert_E(split) assumes exactly this):
// a chunk's 96 products are summed apart -- three MFMAs into a zeroed fp32
// temporary -- and the chunk sum is then added to the fp32 accumulator, so
// the accumulator's rounding runs over n/32 chunk sums, not 3n products.
// fp64 blocks take the same fp32 path (norms rounded to fp32 in the
// epilogue, lists in fp32): knn_cert_E charges them the fp32 accumulator's
// n/25 term like fp32 blocks.
//
// MFMA operand map (v_mfma_f32_16x16x32_f16, as in k_dist_topk's H16 paths):
// lane l = 16 g + j supplies A row j (corpus) and B column j (query) with the
// 8 halves of K-range [8g, 8g + 8) -- slot g of the chunk row (hi) or slot
// 4 + g (lo); D register r of lane l is row 4g + r of the m-tile, query j.
// A lane's 64 candidates of a tile are rows 16 mt + 4 g + r.
//
// LDS images: 8 rows x 128 B per DMA piece, segment s of row r at slot
// s ^ (r & 7), so the 16-byte fragment reads of a lane group hit distinct
// bank quads.
#include "knn_device.h"

typedef _Float16 knn_sh8 __attribute__((ext_vector_type(8)));

#define SP_TQ 128
#define SP_TC 256
#define SP_NST 4
#define SP_STAGE 32768                        /* 256 corpus rows x 128 B */
#define SP_NORM_OFF (SP_NST * SP_STAGE)       /* 131072 */
#define SP_NORM_SLOT 2048                     /* 256 norms x 8 B (fp32: first 1 KiB) */
#define SP_LDS (SP_NORM_OFF + 4 * SP_NORM_SLOT)
// Diagnostic builds only (tools/split_ablate.sh compiles copies with one of
// these set; the product library is built with none): SP_ABL_NOEPI skips the
// epilogue, SP_ABL_NOMFMA the contraction, SP_ABL_NOFRAG the fragment reads,
// SP_ABL_NODMA the staging loads.
#ifndef SP_ABL_NOEPI
#define SP_ABL_NOEPI 0
#endif
#ifndef SP_ABL_NOMFMA
#define SP_ABL_NOMFMA 0
#endif
#ifndef SP_ABL_NOFRAG
#define SP_ABL_NOFRAG 0
#endif
#ifndef SP_ABL_NODMA
#define SP_ABL_NODMA 0
#endif
#ifndef SP_D_SMALL   /* A-fragment prefetch depth (m-tiles) of the <= 24-entry kernels */
#define SP_D_SMALL 4
#endif
// (D must divide the 16 m-tiles: the next chunk's first D fragments are read
// into the slots mt % D of the current chunk's last D m-tiles, and the next
// chunk reads m-tile j from slot j % D -- a D = 3 build failed the parity
// tests, tools/r05_s37.sh)

#ifndef SP_NOPRE   /* (diagnostic: no next-chunk fragment prefetch) */
#define SP_NOPRE 0
#endif

// fp64 bound -> fp32 bound rounded up (still a bound: a candidate above it
// is above the fp64 one)
__device__ __forceinline__ float sp_bound_up(double d)
{
    float f = (float)d;
    if ((double)f < d) f = nextafterf(f, __builtin_inff());
    return f;
}

typedef int knn_si4 __attribute__((ext_vector_type(4)));

// D: A-fragment prefetch depth in m-tiles (the ds_reads of m-tile mt + D
// issue right after m-tile mt's MFMAs)
template <typename T, int KL, int D>
__global__ __launch_bounds__(512) void k_dist_split(
    const char *__restrict__ qsp, const T *__restrict__ qnorm, size_t q_base, int nq,
    const knn_split_blocks_t cb, int n, int rsb, int nsplit, int nqb, const double *__restrict__ meta,
    double *__restrict__ part_d, int *__restrict__ part_i, double *__restrict__ part_T, int nq_pad,
    unsigned long long *__restrict__ qthr, int uj, int xord, float m2s)
{
    constexpr int ES = (int)sizeof(T);
    static_assert(16 % D == 0, "fragment depth must divide the 16 m-tiles (next-chunk prefetch slots)");
    __shared__ __attribute__((aligned(16))) char smem[SP_LDS];
    LDS_AS char *lds = (LDS_AS char *)smem;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int g = lane >> 4, j16 = lane & 15;
    const int wave_s = __builtin_amdgcn_readfirstlane(wave);
    // workgroup order: split-major (xord 0) or XCD-grouped (xord 1), as
    // k_dist_topk
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
    const int ntiles = cb.t0[cb.nblk];
    // block of launch tile t (wave-uniform: the table is in the kernel
    // arguments, <= KNN_SPLIT_MAXBLK entries)
    auto blk_of = [&](int t) {
        int b = 0;
#pragma unroll
        for (int j = 1; j < KNN_SPLIT_MAXBLK; j++) b = (j < cb.nblk && t >= cb.t0[j]) ? j : b;
        return b;
    };
    const int tb = ntiles / nsplit, tr = ntiles - tb * nsplit;
    const int t_lo = split * tb + (split < tr ? split : tr);
    const int t_hi = t_lo + tb + (split < tr ? 1 : 0);
    const int mode = knn_mode<T>(meta, n);
    const int qrow0 = qb * SP_TQ;
    const int myq = qrow0 + 16 * wave + j16;
    const long gq = (long)q_base + myq;
    const float qn = (float)qnorm[myq];
    asm volatile("" ::"v"(qn));
    const int nfc = rsb / 128;
    const int ujm = (mode == KNN_MODE_INT) ? (uj & 255) : (uj >> 8);

    float L[KL];
    int I[KL];
#pragma unroll
    for (int e = 0; e < KL; e++) { L[e] = __builtin_inff(); I[e] = -1; }
    // the shared bound (k_dist_topk): any split's bound bounds the query's
    // (k+1)-th candidate over all rows
    float thr = __builtin_inff();
    if (qthr != nullptr && myq < nq)
        thr = sp_bound_up(__longlong_as_double((long long)atomicMin(qthr + myq, 0x7ff0000000000000ull)));
    if (myq >= nq) thr = -__builtin_inff();   // padding queries reject every candidate
    asm volatile("" ::"v"(thr));

    const int total = (mode == KNN_MODE_SCAN || t_hi <= t_lo) ? 0 : (t_hi - t_lo) * nfc;

    flt4 acc[16];
#pragma unroll
    for (int mt = 0; mt < 16; mt++) acc[mt] = (flt4){0, 0, 0, 0};

    // ---- staging cursor (wave-uniform; clamps at the last chunk) ---------
    const int lr = lane >> 3, ls = lane & 7;
    const int seg_b = 16 * (ls ^ lr);
    int s_c = 0, s_t = t_lo, s_fc = 0, s_st = 0;      // chunk being staged, its stage
    // the staged tile's block, row 0 and last allocated row (scalar; the
    // table is read only when the cursor crosses into the next block -- a
    // table load per piece put an lgkmcnt(0) behind every fragment read)
    int s_b = blk_of(t_lo);
    const char *s_row = (const char *)cb.sp[s_b] + (size_t)(t_lo - cb.t0[s_b]) * SP_TC * rsb;
    int s_lim = cb.lim[s_b] - 1 - (t_lo - cb.t0[s_b]) * SP_TC;
    int s_next = s_b + 1 < cb.nblk ? cb.t0[s_b + 1] : 0x7fffffff;
    // piece i (0..3) of a chunk: corpus rows 32 w + 8 i.. of the tile; rows
    // past the block's allocation are clamped to its last row (their
    // candidates are masked by index)
    auto glds1 = [&](int i) {
        if (SP_ABL_NODMA) return;
        const unsigned dst0 = (unsigned)(uintptr_t)lds + (unsigned)s_st * SP_STAGE;
        const char *cp = s_row + (size_t)128 * s_fc;
        int lrow = 32 * wave_s + 8 * i + lr;
        lrow = lrow < s_lim ? lrow : s_lim;
        bglds16(knn_rsrc(cp), (unsigned)(lrow * rsb + seg_b),
                dst0 + (unsigned)(2 * wave_s + (i >> 1)) * 2048u + (unsigned)(i & 1) * 1024u);
    };
    auto advance = [&]() {
        s_c++;
        s_st = s_st == SP_NST - 1 ? 0 : s_st + 1;
        if (s_c < total) {
            if (++s_fc == nfc) {
                s_fc = 0;
                if (++s_t == s_next) {   // the next block of the launch
                    s_b++;
                    s_row = (const char *)cb.sp[s_b];
                    s_lim = cb.lim[s_b] - 1;
                    s_next = s_b + 1 < cb.nblk ? cb.t0[s_b + 1] : 0x7fffffff;
                } else {
                    s_row += (size_t)SP_TC * rsb;
                    s_lim -= SP_TC;
                }
            }
        }
    };
    // The query fragments (B) of a chunk straight into registers: a lane's
    // two 16-byte slots (hi g, lo 4 + g) of its query row -- the only wave
    // that reads them, so no LDS round trip.  Issued from asm one chunk
    // ahead (counted by the ring's vmcnt waits, invisible to the compiler's
    // wait pass, which would otherwise drain the LDS-DMA ring before their
    // first use) and laundered after the wait that saw them land.
    const char *qrow = qsp + (size_t)myq * rsb + 16 * g;
    auto bload = [&](int fc, knn_si4 &h, knn_si4 &l) {
        const char *p = qrow + (size_t)128 * fc;
        asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(h) : "v"(p) : "memory");
        asm volatile("global_load_dwordx4 %0, %1, off offset:64" : "=v"(l) : "v"(p) : "memory");
    };
    // norm slice of tile t (clamped to the split) into ring slot t & 3:
    // [g][mt][r] = norm of tile row 16 mt + 4 g + r, in 4-byte pieces
    // (fp64: 512 pieces, one a lane of every wave; fp32: 256, waves 0..3)
    constexpr int NU = SP_TC * ES / 4;
    auto gnorm = [&](int t) {
        if (wave_s >= NU / 64) return;
        const int ts = t < t_hi ? t : t_hi - 1;
        const int b = blk_of(ts);
        const int u = 64 * wave_s + lane;
        const int p = ES == 8 ? u >> 1 : u;
        const int gg = p >> 6, k = p & 63;
        int row = (ts - cb.t0[b]) * SP_TC + 16 * (k >> 2) + 4 * gg + (k & 3);
        row = row < cb.lim[b] ? row : cb.lim[b] - 1;
        const char *src = (const char *)((const T *)cb.nrm[b] + row) + (ES == 8 ? (u & 1) * 4 : 0);
        glds4(src, (unsigned)(uintptr_t)lds + SP_NORM_OFF + (unsigned)(t & 3) * SP_NORM_SLOT +
                       (unsigned)wave_s * 256u);
    };

    // ---- epilogue of tile t: d^2, threshold filter, insertion ------------
    auto epilogue = [&](int t) {
        if (SP_ABL_NOEPI) {
#pragma unroll
            for (int mt = 0; mt < 16; mt++) asm volatile("" ::"v"(acc[mt]));
#pragma unroll
            for (int mt = 0; mt < 16; mt++) acc[mt] = (flt4){0, 0, 0, 0};
            return;
        }
        const LDS_AS T *cng = (const LDS_AS T *)(lds + SP_NORM_OFF + (t & 3) * SP_NORM_SLOT) + 64 * g;
        const float lim = L[KL - 1] < thr ? L[KL - 1] : thr;
        const int eb = blk_of(t);
        const long c_base = cb.base[eb];
        const int nc = cb.nc[eb];
        const int row0 = (t - cb.t0[eb]) * SP_TC;
        const long gt0 = (long)c_base + row0, gw0 = (long)q_base + qrow0 + 16 * wave_s;
        const bool masked = (row0 + SP_TC > nc) || (gw0 < gt0 + SP_TC && gt0 < gw0 + 16);
#pragma unroll
        for (int mt = 0; mt < 16; mt++) {
            float cn[4];
            if constexpr (ES == 8) {
                const dbl2 n01 = ((const LDS_AS dbl2 *)cng)[2 * mt];
                const dbl2 n23 = ((const LDS_AS dbl2 *)cng)[2 * mt + 1];
                cn[0] = (float)n01.x; cn[1] = (float)n01.y; cn[2] = (float)n23.x; cn[3] = (float)n23.y;
            } else {
                const flt4 n4 = ((const LDS_AS flt4 *)cng)[mt];
                cn[0] = n4.x; cn[1] = n4.y; cn[2] = n4.z; cn[3] = n4.w;
            }
#pragma unroll
            for (int r = 0; r < 4; r++) acc[mt][r] = __builtin_fmaf(m2s, acc[mt][r], qn + cn[r]);
        }
        float lanemin = acc[0][0];
#pragma unroll
        for (int mt = 0; mt < 16; mt++)
#pragma unroll
            for (int r = (mt == 0 ? 1 : 0); r < 4; r++) lanemin = fminf(lanemin, acc[mt][r]);
        const bool any = masked || __ballot(lanemin <= lim) != 0ull;
        if (any) {
            const float zfloor = (mode == KNN_MODE_INT) ? 0.f : -__builtin_inff();
            unsigned long long pend = 0;
#pragma unroll
            for (int mt = 0; mt < 16; mt++)
#pragma unroll
                for (int r = 0; r < 4; r++)
                    pend |= (acc[mt][r] <= lim) ? (1ull << (4 * mt + r)) : 0ull;
            if (masked) {
#pragma unroll
                for (int mt = 0; mt < 16; mt++)
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        const int row = row0 + 16 * mt + 4 * g + r;
                        if (!(row < nc && (long)c_base + row != gq)) pend &= ~(1ull << (4 * mt + r));
                    }
            }
            // one wave round per survivor of the busiest lane: the lowest
            // pending candidate (lowest row: the stable tie order) through a
            // 6-level select tree over the 64 d^2
            while (__ballot(pend != 0) != 0ull) {
                const int b = pend ? __builtin_ctzll(pend) : 0;
                const bool b0 = b & 1, b1 = b & 2, b2 = b & 4, b3 = b & 8, b4 = b & 16, b5 = b & 32;
                float v[16];
#pragma unroll
                for (int mt = 0; mt < 16; mt++) {
                    const float lo = b0 ? acc[mt][1] : acc[mt][0];
                    const float hi = b0 ? acc[mt][3] : acc[mt][2];
                    v[mt] = b1 ? hi : lo;
                }
                // (named temporaries: written as arrays, the tree was turned
                // into a private-memory table indexed by b)
                const float w0 = b2 ? v[1] : v[0], w1 = b2 ? v[3] : v[2], w2 = b2 ? v[5] : v[4];
                const float w3 = b2 ? v[7] : v[6], w4 = b2 ? v[9] : v[8], w5 = b2 ? v[11] : v[10];
                const float w6 = b2 ? v[13] : v[12], w7 = b2 ? v[15] : v[14];
                const float y0 = b3 ? w1 : w0, y1 = b3 ? w3 : w2, y2 = b3 ? w5 : w4, y3 = b3 ? w7 : w6;
                const float z0 = b4 ? y1 : y0, z1 = b4 ? y3 : y2;
                const float dsel = b5 ? z1 : z0;
                const float dd = (pend && dsel > zfloor) ? dsel : __builtin_inff();
                const int ii = (int)(c_base + row0 + 16 * (b >> 2) + 4 * g + (b & 3));
                pend &= pend - 1;
                list_insert<KL>(L, I, dd, ii);
            }
        }
#pragma unroll
        for (int mt = 0; mt < 16; mt++) acc[mt] = (flt4){0, 0, 0, 0};
        if (!any) return;
        // the query's 4 lanes' shared threshold (k_dist_topk)
        float lmin = L[KL - 1], u = L[0];
#pragma unroll
        for (int e = 1; e < KL; e++) u = (e == ujm) ? L[e] : u;
        lmin = fminf(lmin, __shfl_xor(lmin, 16));
        lmin = fminf(lmin, __shfl_xor(lmin, 32));
        u = fmaxf(u, __shfl_xor(u, 16));
        u = fmaxf(u, __shfl_xor(u, 32));
        thr = fminf(thr, fminf(lmin, u));
    };

    const int fs0 = j16 * 128 + 16 * (g ^ (j16 & 7));          // slot g: hi halves
    const int fs1 = j16 * 128 + 16 * ((4 + g) ^ (j16 & 7));    // slot 4 + g: lo halves

    if (total > 0) {
        // prologue: chunk 0's query fragments, the norm slices of the first
        // two tiles, chunks 0..2 (chunk 3 is staged during chunk 0)
        knn_si4 qh_c, ql_c, qh_n, ql_n;
        bload(0, qh_c, ql_c);
        gnorm(t_lo);
        gnorm(t_lo + 1);
#pragma unroll
        for (int x = 0; x < SP_NST - 1; x++) {
#pragma unroll
            for (int i = 0; i < 4; i++) glds1(i);
            advance();
        }
        // B(0), norms, chunk 0 landed: chunks 1, 2 (8 pieces) may stay in flight
        if (SP_ABL_NODMA) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        asm volatile("" : "+v"(qh_c), "+v"(ql_c));
        __builtin_amdgcn_s_barrier();

        int st = 0, fcq = 0;                          // stage / row chunk computed
        // A fragments of the first D m-tiles: read at the chunk's start, or
        // -- for every chunk but a tile's first -- during the previous
        // chunk's last D m-tiles.  The next chunk's stage is valid then: the
        // barrier that ended the chunk before saw every wave's pieces of it
        // land (vmcnt(4) leaves only the chunk three ahead in flight), and
        // it is overwritten only after the barrier that ends the next chunk.
        // Read at the start, the first fragments of all 8 waves queued behind
        // one another right after the barrier while the MFMA pipes idled.
        knn_sh8 ah[D], al[D];
        for (int t = t_lo; t < t_hi; t++) {
            gnorm(t + 2);
            for (int fc = 0; fc < nfc; fc++) {
                LDS_AS char *cs = lds + st * SP_STAGE;
                const bool pre = fc + 1 < nfc && !SP_ABL_NOFRAG && !SP_NOPRE;   // prefetch into the next chunk
                LDS_AS char *cn_ = lds + (st == SP_NST - 1 ? 0 : st + 1) * SP_STAGE;
                // next chunk's query fragments (the row's chunks cycle every tile)
                fcq = fcq + 1 == nfc ? 0 : fcq + 1;
                bload(fcq, qh_n, ql_n);
                knn_sh8 qh, ql;
                if (SP_ABL_NOFRAG) {
                    qh = ql = (knn_sh8){1, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
                    for (int d = 0; d < D; d++) ah[d] = al[d] = qh;
                } else {
                    qh = __builtin_bit_cast(knn_sh8, qh_c);
                    ql = __builtin_bit_cast(knn_sh8, ql_c);
                    if (fc == 0 || SP_NOPRE) {
#pragma unroll
                        for (int d = 0; d < D; d++) {
                            ah[d] = *(const LDS_AS knn_sh8 *)(cs + d * 2048 + fs0);
                            al[d] = *(const LDS_AS knn_sh8 *)(cs + d * 2048 + fs1);
                        }
                    }
                }
                flt4 tt[2];
#pragma unroll
                for (int mt = 0; mt < 16; mt++) {
                    const int sl = mt % D;
                    // the chunk's 96 products summed apart (cross terms
                    // first), then added to the accumulator (knn_cert_E)
                    if (SP_ABL_NOMFMA) {
                        asm volatile("" ::"v"(ah[sl]), "v"(al[sl]), "v"(qh), "v"(ql));
                        tt[mt & 1] = (flt4){0, 0, 0, 0};
                    } else {
                        flt4 x = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[sl], ql, (flt4){0, 0, 0, 0}, 0, 0, 0);
                        x = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[sl], qh, x, 0, 0, 0);
                        tt[mt & 1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[sl], qh, x, 0, 0, 0);
                    }
                    // m-tile mt + D's fragments into the slot just consumed
                    // (past the last m-tile: the next chunk's first ones)
                    if (mt + D < 16 && !SP_ABL_NOFRAG) {
                        ah[sl] = *(const LDS_AS knn_sh8 *)(cs + (mt + D) * 2048 + fs0);
                        al[sl] = *(const LDS_AS knn_sh8 *)(cs + (mt + D) * 2048 + fs1);
                    } else if (mt + D >= 16 && pre) {
                        ah[sl] = *(const LDS_AS knn_sh8 *)(cn_ + (mt + D - 16) * 2048 + fs0);
                        al[sl] = *(const LDS_AS knn_sh8 *)(cn_ + (mt + D - 16) * 2048 + fs1);
                    }
                    if (mt > 0) acc[mt - 1] += tt[(mt - 1) & 1];
                    // chunk c + 3 into the stage chunk c - 1 left (freed by the
                    // barrier that ended chunk c - 1), one piece every 4th m-tile
                    if ((mt & 3) == 2) {
                        glds1(mt >> 2);
                        if (mt == 14) advance();
                    }
                    __builtin_amdgcn_sched_barrier(0);
                }
                acc[15] += tt[1];
                __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): this stage's reads done
                // the next chunk's query fragments and pieces landed (and
                // chunk c + 2's): chunk c + 3's 4 pieces may stay in flight
                if (SP_ABL_NODMA) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // (no pieces to count)
                else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
                asm volatile("" : "+v"(qh_n), "+v"(ql_n));
                qh_c = qh_n;
                ql_c = ql_n;
                __builtin_amdgcn_s_barrier();
                st = st == SP_NST - 1 ? 0 : st + 1;
            }
            epilogue(t);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");     // no LDS-DMA left in flight
    }

    float lastmin = L[KL - 1];
    lastmin = fminf(lastmin, __shfl_xor(lastmin, 16));
    lastmin = fminf(lastmin, __shfl_xor(lastmin, 32));
    float pub = thr;
    if (mode == KNN_MODE_INT && lastmin > thr && thr < __builtin_inff()) pub = nextafterf(thr, __builtin_inff());
    if (myq < nq) {
        const size_t base = (((size_t)split * nq_pad + myq) * 4 + g) * KL;
#pragma unroll
        for (int e = 0; e < KL; e++) {
            part_d[base + e] = (double)L[e];
            part_i[base + e] = I[e];
        }
        if (g == 0) {
            part_T[(size_t)split * nq_pad + myq] = (double)pub;
            if (qthr != nullptr && thr < __builtin_inff())
                atomicMin(qthr + myq, (unsigned long long)__double_as_longlong((double)thr));
        }
    }
}

template <typename T, int KL, int D>
static int launch_split(const void *qsp, const T *qnorm, size_t q_base, int nq, const knn_split_blocks_t &cb, int n,
                        const double *meta, int nsplit, double *part_d, int *part_i, double *part_T, int nq_pad,
                        double *qthr, int uj, int xord, float m2s, hipStream_t s)
{
    const int rsb = (int)knn_split_rs((size_t)n);
    const int nqb = (nq + SP_TQ - 1) / SP_TQ;
    const int nqb_grid = xord ? (nqb + 7) / 8 * 8 : nqb;
    hipLaunchKernelGGL(HIP_KERNEL_NAME(k_dist_split<T, KL, D>), dim3((unsigned)(nqb_grid * nsplit)), dim3(512), 0, s,
                       (const char *)qsp, qnorm, q_base, nq, cb, n, rsb, nsplit, nqb, meta, part_d, part_i, part_T,
                       nq_pad, (unsigned long long *)qthr, uj, xord, m2s);
    return hipGetLastError() == hipSuccess ? KNN_OK : KNN_ERR_HIP;
}

// The launcher behind knn_launch_dist_topk's KNN_DIST_SPLIT (one block) and
// the engine's fused GEMM step (several): the table's tiles are 256-row
// tiles of each block in turn (t0 filled here), the last tile of a block
// clamped to its allocation in the kernel.
extern "C" int knn_launch_dist_split(int dtype, int kl, const void *qsp, const void *qnorm, size_t q_base,
                                     int nq, const knn_split_blocks_t *cbp, int n, const double *meta, int nsplit,
                                     double *part_d, int *part_i, double *part_T, int nq_pad, double *qthr, int uj,
                                     int xord, float m2s, void *stream)
{
    if (nq <= 0 || nsplit <= 0 || !qsp || !cbp || cbp->nblk < 1 || cbp->nblk > KNN_SPLIT_MAXBLK)
        return KNN_ERR_INVALID;
    knn_split_blocks_t cb = *cbp;
    cb.t0[0] = 0;
    for (int b = 0; b < cb.nblk; b++) {
        if (!cb.sp[b] || !cb.nrm[b] || cb.nc[b] <= 0 || cb.nc[b] > cb.lim[b] || cb.base[b] < 0) return KNN_ERR_INVALID;
        cb.t0[b + 1] = cb.t0[b] + (cb.nc[b] + SP_TC - 1) / SP_TC;
    }
    for (int b = cb.nblk + 1; b <= KNN_SPLIT_MAXBLK; b++) cb.t0[b] = cb.t0[cb.nblk];
    if (cb.t0[cb.nblk] < nsplit) return KNN_ERR_INVALID;
    hipStream_t s = (hipStream_t)stream;
#define SPL(T, KL)                                                                                          \
    return launch_split<T, KL, (KL > 24 ? 2 : SP_D_SMALL)>(qsp, (const T *)qnorm, q_base, nq, cb, n, meta, nsplit, part_d, \
                                                 part_i, part_T, nq_pad, qthr, uj, xord, m2s, s)
    if (dtype == KNN_F64 && kl == KNN_KL) SPL(double, KNN_KL);
    if (dtype == KNN_F32 && kl == KNN_KL) SPL(float, KNN_KL);
    if (dtype == KNN_F32 && kl == KNN_KL_M) SPL(float, KNN_KL_M);
    if (dtype == KNN_F32 && kl == KNN_KL_L) SPL(float, KNN_KL_L);
#undef SPL
    return KNN_ERR_INVALID;
}
