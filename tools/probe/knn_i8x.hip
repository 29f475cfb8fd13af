// ROUND-6 EXPERIMENT, NOT PART OF libknn (moved here from mpi-knn_amd/csrc
// after measurement).  Wired into the engine as the k <= 31
// long-row default (8-entry lists, 4 a query, k_merge_rank on them) it was
// bit-exact -- 108 int8 / golden / byte-block / P = 8 tests, all 60000 rows
// of the full-size fixture (tools/r06_s3.sh) -- but slower: mnist kernel
// 4.42 ms against the 32x32x32 half-tile kernel's 3.09 ms on the same box.
// Cause: two 16-query groups a lane need two lists and two epilogues' state
// beside 13 resident K-steps of query fragments (104 VGPRs); at two waves a
// SIMD (256 VGPRs) the 13- and 14-step instantiations spill 37-63 VGPRs
// (the 4- and 8-step ones fit).  The probe's clock gain (tools/probe/
// i8_shape_probe.hip) needs a layout that keeps the query fragments in
// fewer registers first.  Also tried: reloading the last NK - 8 steps' query
// fragments from L2 every tile (this file's NRES / reload()): 64-77 spilled
// VGPRs -- the pressure peak is the tile loop itself (query fragments,
// accumulators, the next tile's first A fragments and both groups' lists),
// not the epilogue.
// knn_i8x.hip -- the int8 contraction on v_mfma_i32_16x16x64_i8: the k <= 31
// default for rows of more than 4 K-steps (MNIST's n = 784).
//
// Same arithmetic, byte blocks, staging ring and survivor path as
// k_dist_topk_i8's half-tile kernel (knn_i8.hip: the distance stage of
// knn-serial.c:72-93 as an exact int8 contraction, d^2 = |q'|^2 + |c'|^2 -
// 2 q'.c', every partial sum an exact int32), on the 16x16 MFMA shape:
//
//   MI355X_MICROARCH.md DVFS item 7: the clock the chip holds under an MFMA
//   loop depends on the MFMA's shape.  Measured here (tools/probe/
//   i8_shape_probe.hip, profiles/r06_i8_shape_probe.log: the int8 loop
//   with its ds_read_b128 A fragments, two workgroups a CU, random bytes)
//   the 32x32x32 loop held 1.61 GHz and the 16x16x64 loop 1.93-1.96 GHz at
//   equal cycles per op: 3.36 against 3.01 POPS of useful work, the 16x16
//   loop paying 4% for 64-byte K-steps over 800-byte rows.
//
// Workgroup: 4 waves (one a SIMD, two workgroups a CU), 128 queries x a
// corpus split in 64-row tiles; wave w takes queries 32 w .. +31 as two
// 16-query groups s = 0, 1 against the tile's 4 m-tiles of 16 rows.  Per
// 64-byte K-step a wave reads 4 A fragments (ds_read_b128: lane l = 16 g + j
// holds row 16 mt + j, bytes [16 g, 16 g + 16) of the step) and issues 8
// MFMAs (each A fragment feeds both groups: the same LDS bytes per op as the
// 32x32 form).  Query B fragments stay in VGPRs (NK steps x 2 groups x 4);
// bytes past the row (the last step of an 800-byte row) are zero there, so
// the staged bytes they meet add nothing.
//
// C/D (dtype-independent on gfx950): lane l = 16 g + j, register r holds
// query j of its group against row 16 mt + 4 g + r.  So a lane carries two
// queries (one a group), 16 candidates each a tile; a query's candidates
// lie in its 4 lanes j, j + 16, j + 32, j + 48, one KL = 8 list each (lpq 4:
// 4 x 8 >= k + 1, so the max of their uj4-th entries bounds the query's
// (k+1)-th d^2 -- the 4-lane bound, by two shuffles).
//
// Keys: the byte block's slot words (knn_device.h, i8_norm_word) give the
// row at tile position R the slot 16 (R >> 5) + 4 ((R >> 3) & 3) + (R & 3);
// a lane's rows R = 16 mt + 4 g + r share bits 2 and 3 (from g), so their
// slots are distinct and increase with R: the exact key v = 64 acc + K =
// 32 (|q'|^2 - d^2) + 31 - slot orders the lane's candidates of one query by
// (d^2, row) as in the 32x32 kernel, and R comes back as
// 32 (slot >> 4) + 8 ((slot >> 2) & 3) + 4 (g & 1) + (slot & 3).
// The lane's 4 norm words of m-tile mt are consecutive (i8_norm_pos): one
// ds_read_b128 each, shared by both groups.
#include "knn_i8_dev.h"

// Diagnostic builds only (tools/i8x_variants.sh; the product library sets
// neither): I8X_PF = 1 reads the next K-step's four A fragments before this
// step's MFMAs (16 more VGPRs) instead of each right after its slot's last
// use; I8X_NOEPI = 1 replaces the epilogue with a sink (timing only)
#ifndef I8X_PF
#define I8X_PF 0
#endif
#ifndef I8X_NOEPI
#define I8X_NOEPI 0
#endif

// max of 16 values: 7 v_max3
__device__ __forceinline__ int i8x_max16(const int *v)
{
    const int m0 = i8_max3(v[0], v[1], v[2]), m1 = i8_max3(v[3], v[4], v[5]), m2 = i8_max3(v[6], v[7], v[8]);
    const int m3 = i8_max3(v[9], v[10], v[11]), m4 = i8_max3(v[12], v[13], v[14]);
    return i8_max3(i8_max3(m0, m1, m2), i8_max3(m3, m4, v[15]), m0);
}
// the largest of the 16 values below vm, or `none` (i8_next's unsigned
// minimum of vm - 1 - v; the lane's values of one query span < 2^31)
__device__ __forceinline__ int i8x_next16(const int *v, int vm, int none)
{
    const unsigned c = (unsigned)vm - 1u;
    unsigned m[6];
#pragma unroll
    for (int y = 0; y < 5; y++)
        m[y] = i8_min3u(c - (unsigned)v[3 * y], c - (unsigned)v[3 * y + 1], c - (unsigned)v[3 * y + 2]);
    m[5] = c - (unsigned)v[15];
    const unsigned u = i8_min3u(i8_min3u(m[0], m[1], m[2]), i8_min3u(m[3], m[4], m[5]), m[0]);
    return (int)u < 0 ? none : (int)(c - u);
}

// KL: lane-list entries (8); NK: 64-byte K-steps (bucket >= the rows'); NST:
// ring stages; NB: survivor-buffer entries a lane and group
template <int KL, int NK, int NST, int NB>
__global__ __launch_bounds__(256, 2) void k_dist_topk_i8x(
    const signed char *__restrict__ qsh, size_t q_rows_pad, size_t q_base, int nq,
    const knn_i8_blocks_t cb, size_t c_rows_pad, int rs,
    int ntiles, int nsplit, int nqb, double *__restrict__ part_d,
    int *__restrict__ part_i, double *__restrict__ part_T, int nq_pad,
    unsigned long long *__restrict__ qthr, int uj)
{
    constexpr int W = 4;                    // waves
    constexpr int TR = 64;                  // rows a tile (4 m-tiles of 16)
    constexpr int CHB = TR * 128;           // bytes a chunk (128 bytes of every row: 2 K-steps)
    constexpr int PW = CHB / 1024 / W;      // DMA pieces (1 KiB) per wave per chunk: 2
    constexpr int LPQ = 4;                  // lists per query (the query's 4 lanes)
    constexpr int NRB = TR * 8;             // norm ring bytes a stage: slot + init words
    constexpr int WPW = TR / W;             // norm words a wave stages of each array
    constexpr int NSEG = 8 * WPW;           // a wave's staged piece (both arrays)
    constexpr int NORM0 = NST * CHB;        // norm ring: [NST][W][slot words, init words]
    constexpr int BUF0 = NORM0 + NST * NRB; // [W][2][NB][64] survivor d^2, then ids
    constexpr int TB0 = BUF0 + 2 * W * 2 * NB * 256;   // block table
    constexpr int LDSB = TB0 + (int)((sizeof(i8_tab_lds) + 15) / 16 * 16);
    constexpr int NCH = (NK + 1) / 2;       // chunks a tile
    static_assert(PW == 2, "two DMA pieces a wave a chunk");
    __shared__ __attribute__((aligned(16))) char smem[LDSB];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int wave_s = __builtin_amdgcn_readfirstlane(wave);
    const int g4 = lane >> 4, j16 = lane & 15;
    // split-major order: long splits first (knn_engine.c: choose_splits)
    const int qb = blockIdx.x % nqb, split = blockIdx.x / nqb;
    ntiles *= 2;   // the host counts 128-row tiles
    const int tb = ntiles / nsplit, tr = ntiles - tb * nsplit;
    const int t_lo = split * tb + (split < tr ? split : tr);
    const int t_hi = t_lo + tb + (split < tr ? 1 : 0);
    const int qrow0 = qb * 128;
    int myq[2], lq[2];
#pragma unroll
    for (int s = 0; s < 2; s++) {
        myq[s] = qrow0 + 32 * wave + 16 * s + j16;
        lq[s] = myq[s] < nq ? myq[s] : nq - 1;
    }
    const int *qnorms = (const int *)(qsh + q_rows_pad * (size_t)rs);

    // ---- resident query fragments: step k, lane (g4, j16) = bytes
    // [64 k + 16 g4, +16) of its query row (zero past the row) ----------------
    // The first NRES steps stay resident; the last NRL are loaded again
    // every tile (from L2: each wave re-reads its own 32 rows), issued at
    // chunk CI's last step ahead of its stage and waited for at their first
    // use in chunk CU: resident, all NK steps took 104 of the 256 VGPRs a
    // wave has at two waves a SIMD, and the two groups' epilogue state
    // spilled 37-63 VGPRs (tools/r06_s3.sh)
    constexpr int NRES = NK < 8 ? NK : 8;
    constexpr int NRL = NK - NRES;
    constexpr int CU = NRES / 2, CI = CU - 3;
    static_assert(NRL == 0 || (CI >= 0 && NRES % 2 == 0), "reload schedule");
    knn_v4i qf[2][NRES];
    knn_v4i qr[2][NRL > 0 ? NRL : 1];
    int qn[2];
#pragma unroll
    for (int s = 0; s < 2; s++) {
        const signed char *qrow = qsh + (size_t)lq[s] * rs + 16 * g4;
#pragma unroll
        for (int k = 0; k < NRES; k++) {
            const bool in = 64 * k + 16 * g4 < rs;
            const knn_v4i v = *(const knn_v4i *)(qrow + (in ? 64 * k : 0));
            qf[s][k] = in ? v : (knn_v4i){0, 0, 0, 0};
        }
        qn[s] = i8_norm_of(qnorms[i8_norm_pos(lq[s])], qnorms[q_rows_pad + i8_norm_pos(lq[s])]);
    }
    int thr[2];
#pragma unroll
    for (int s = 0; s < 2; s++) {
        thr[s] = I8_INF;
        if (qthr != nullptr && myq[s] < nq) {
            const double td = __longlong_as_double((long long)atomicMin(qthr + myq[s], 0x7ff0000000000000ull));
            thr[s] = td >= 2147483647.0 ? I8_INF : (int)td;
        }
        if (myq[s] >= nq) thr[s] = -1;   // padding queries reject every candidate
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): the query loads (compiler-visible)

    int L[2][KL], I[2][KL];
#pragma unroll
    for (int s = 0; s < 2; s++)
#pragma unroll
        for (int e = 0; e < KL; e++) { L[s][e] = I8_INF; I[s][e] = -1; }
    const int uj4 = ((uj >> 8) & 255) < KL - 1 ? ((uj >> 8) & 255) : KL - 1;
    LDS_AS int *bk0 = (LDS_AS int *)(smem + BUF0) + wave_s * 2 * NB * 64 + lane;
    LDS_AS int *bi0 = bk0 + W * 2 * NB * 64;
    int cnt[2] = {0, 0};
    LDS_AS i8_tab_lds *tab = (LDS_AS i8_tab_lds *)(smem + TB0);
    if (threadIdx.x == 0) {
#pragma unroll
        for (int j = 0; j < KNN_I8_MAXBLK; j++) {
            tab->ptr[j] = (unsigned long long)(uintptr_t)cb.ptr[j];
            tab->nptr[j] = (unsigned long long)(uintptr_t)cb.nptr[j];
            tab->base[j] = cb.base[j];
            tab->nc[j] = cb.nc[j];
        }
#pragma unroll
        for (int j = 0; j <= KNN_I8_MAXBLK; j++) tab->t0[j] = cb.t0[j] * 2;
        tab->nblk = cb.nblk;
    }
    __syncthreads();

    // ---- staging (k_dist_topk_i8's ring: 2 pieces of 8 rows x 128 B a
    // wave a chunk, a tile's norm words with its first chunk) ---------------
    const int total = (t_hi > t_lo) ? (t_hi - t_lo) * NCH : 0;
    unsigned voff[PW];
#pragma unroll
    for (int p = 0; p < PW; p++) {
        const int rr = (TR / W) * wave_s + 8 * p + (lane >> 3);
        voff[p] = (unsigned)(rr * rs + 16 * ((lane & 7) ^ ((rr >> 1) & 7)));
    }
    const unsigned lds0 = (unsigned)(uintptr_t)smem;
    int s_t = t_lo, s_x = 0;
    // ring slots kept as counters (s_x % NST, s_t % NST: a modulo by the
    // 7-stage ring's non-power-of-two cost the kernel 49-63 spilled VGPRs)
    unsigned s_xs = 0, s_ts = (unsigned)t_lo % NST;
    unsigned s_coff = 0;
    int s_b = i8_blk_of(tab, t_lo);
    const int s_t0 = i8_rfl(tab->t0[s_b]);
    int s_t1 = i8_rfl(tab->t0[s_b + 1]);
    const signed char *s_row = (const signed char *)(uintptr_t)i8_rfl64((long long)tab->ptr[s_b]) +
                               (size_t)(t_lo - s_t0) * TR * rs;
    const int *s_nrow = (const int *)(uintptr_t)i8_rfl64((long long)tab->nptr[s_b]) + (size_t)(t_lo - s_t0) * TR;
    auto stage = [&]() {
        const unsigned dst = lds0 + s_xs * (unsigned)CHB + (unsigned)wave_s * (unsigned)(CHB / W);
        bglds16x2(i8_rsrc(s_row + s_coff), voff[0], voff[1], dst);
        if (s_x < total && s_coff == 0) {
            if (lane < WPW / 2)
                bglds16(i8_rsrc(s_nrow + WPW * wave_s),
                        lane < WPW / 4 ? 16u * lane : 4u * (unsigned)c_rows_pad + 16u * (lane - WPW / 4),
                        lds0 + NORM0 + s_ts * (unsigned)NRB + (unsigned)NSEG * wave_s);
        }
        s_x++;
        s_xs = s_xs + 1 == NST ? 0 : s_xs + 1;
        if (s_x < total) {
            s_coff += 128;
            if (s_coff == 128u * NCH) {
                s_coff = 0;
                s_ts = s_ts + 1 == NST ? 0 : s_ts + 1;
                if (++s_t == s_t1) {   // next block of the launch
                    s_b++;
                    s_row = (const signed char *)(uintptr_t)i8_rfl64((long long)tab->ptr[s_b]);
                    s_nrow = (const int *)(uintptr_t)i8_rfl64((long long)tab->nptr[s_b]);
                    s_t1 = i8_rfl(tab->t0[s_b + 1]);
                } else {
                    s_row += (size_t)TR * rs;
                    s_nrow += TR;
                }
            }
        }
    };
    // the next chunk's own pieces landed: the NST - 3 chunks staged after it
    // may stay in flight (the norm piece rides with a tile's first chunk,
    // which the count of older operations covers)
    auto wait_next = [&]() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PW * (NST - 3)) : "memory"); };
    auto nofs = [&](int v) -> int { return (v / (WPW / 4)) * NSEG + (v % (WPW / 4)) * 16; };
    // A fragment of m-tile mt, K-step ks2 (0, 1) of staged chunk xx: row
    // 16 mt + j16, segment 4 ks2 + g4 (image swizzle s ^ ((row >> 1) & 7);
    // (row >> 1) & 7 = (j16 >> 1) & 7 for every mt); conflict-free
    const int aswz = (j16 >> 1) & 7;
    // (xs: the chunk's ring slot)
    auto rdA1 = [&](unsigned xs, int ks2, int mt) -> knn_v4i {
        const LDS_AS char *p = (const LDS_AS char *)smem + xs * CHB + (16 * mt + j16) * 128 +
                               16 * ((4 * ks2 + g4) ^ aswz);
        return *(const LDS_AS knn_v4i *)p;
    };

    // reloaded query fragments: asm loads (invisible to the compiler's wait
    // pass, as the ring's), so the stage()s issued after them are younger:
    // 3 stages x 2 pieces by chunk CU, where vmcnt(6) sees them landed
    auto reload = [&]() {
#pragma unroll
        for (int s = 0; s < 2; s++)
#pragma unroll
            for (int j = 0; j < NRL; j++) {
                const int k = NRES + j;
                const signed char *p = qsh + (size_t)lq[s] * rs + 16 * g4 + (64 * k + 16 * g4 < rs ? 64 * k : 0);
                asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(qr[s][j]) : "v"(p) : "memory");
            }
    };
    auto reload_ready = [&]() {
        asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
#pragma unroll
        for (int s = 0; s < 2; s++)
#pragma unroll
            for (int j = 0; j < NRL; j++) {
                asm volatile("" : "+v"(qr[s][j]));
                if (64 * (NRES + j) + 16 * g4 >= rs) qr[s][j] = (knn_v4i){0, 0, 0, 0};   // past the row
            }
    };
    // the query fragment of K-step k (static after unrolling)
    auto qfrag = [&](int s, int k) -> knn_v4i { return k < NRES ? qf[s][k < NRES ? k : 0] : qr[s][k >= NRES ? k - NRES : 0]; };

    // ---- bounds (k_dist_topk_i8: every value bounds the query's (k+1)-th
    // d^2 over all rows, or is the lane's own KL-th) ------------------------
    auto refresh = [&](int s) {
        int lmin = L[s][KL - 1], u4 = L[s][0];
#pragma unroll
        for (int e = 1; e < KL; e++) u4 = (e == uj4) ? L[s][e] : u4;
        // the query's 4 lanes: 4 KL entries, >= k + 1 of them <= max(u4);
        // thr <= every lane's last entry keeps the published T a bound on
        // what a full list drops
        int o = __shfl_xor(lmin, 16);
        lmin = o < lmin ? o : lmin;
        o = __shfl_xor(lmin, 32);
        lmin = o < lmin ? o : lmin;
        o = __shfl_xor(u4, 16);
        u4 = o > u4 ? o : u4;
        o = __shfl_xor(u4, 32);
        u4 = o > u4 ? o : u4;
        const int nb = lmin < u4 ? lmin : u4;
        thr[s] = nb < thr[s] ? nb : thr[s];
    };
    auto merge = [&](int s) {
        const LDS_AS int *bk = bk0 + s * NB * 64, *bi = bi0 + s * NB * 64;
        for (int e = 0; __ballot(e < cnt[s]) != 0ull; e++) {
            int d = I8_INF, id = -1;
            if (e < cnt[s]) {
                d = bk[64 * e];
                id = bi[64 * e];
                d = d > 0 ? d : I8_INF;   // d^2 == 0: an exact duplicate (serial:86)
            }
            i8_insert<KL>(L[s], I[s], d, id);
        }
        cnt[s] = 0;
        refresh(s);
    };
    // the shared bound re-read every second tile (k_dist_topk_i8: an asm
    // load, laundered once the ring's waits have covered it)
    unsigned long long q_bits[2] = {0x7ff0000000000000ull, 0x7ff0000000000000ull};
    int q_ready = -1;
    auto qthr_issue = [&](int xnow) {
#pragma unroll
        for (int s = 0; s < 2; s++) {
            const unsigned long long *pq = qthr + lq[s];
            asm volatile("global_load_dwordx2 %0, %1, off sc1" : "=v"(q_bits[s]) : "v"(pq) : "memory");
        }
        q_ready = xnow;
    };
    auto qthr_apply = [&]() {
#pragma unroll
        for (int s = 0; s < 2; s++) {
            asm volatile("" : "+v"(q_bits[s]));
            const double td = __longlong_as_double((long long)q_bits[s]);
            const int tq = td >= 2147483647.0 ? I8_INF : (int)td;
            thr[s] = tq < thr[s] ? tq : thr[s];
        }
        q_ready = -1;
    };

    // ---- epilogue of tile t ------------------------------------------------------
    long c_base = 0;
    int nc = 0, e_t0 = 0, e_t1 = 0, e_b = 0;
    const int dmax = rs * 65025 + 1;
    int vnone[2];
#pragma unroll
    for (int s = 0; s < 2; s++) vnone[s] = 32 * (qn[s] - dmax) - 1;
    auto thr_v = [&](int s) -> int {
        const int lim = L[s][KL - 1] < thr[s] ? L[s][KL - 1] : thr[s];
        return lim >= dmax ? vnone[s] + 1 : 32 * (qn[s] - lim);
    };
    auto epilogue = [&](int t, unsigned ts, knn_v4i (&A)[2][4], int xdone) {
        const int lt = t - e_t0;
        const LDS_AS char *cn = (const LDS_AS char *)smem + NORM0 + ts * NRB;
        const int row0 = lt * TR;
        const long gt0 = (long)c_base + row0;
        const bool rmask = row0 + TR > nc;
        const int idb = (int)(c_base + row0) + 4 * (g4 & 1);
        if (qthr != nullptr) {
            if (q_ready >= 0 && xdone > q_ready) qthr_apply();
            if (q_ready < 0 && (t & 1) == 0) qthr_issue(s_x);
        }
#pragma unroll
        for (int s = 0; s < 2; s++) {
            // (one group at a time: its keys are the only ones live)
            __builtin_amdgcn_sched_barrier(0);
            const long gw0 = (long)q_base + qrow0 + 32 * wave + 16 * s;
            const bool masked = rmask || (gw0 < gt0 + TR && gt0 < gw0 + 16);
            LDS_AS int *bk = bk0 + s * NB * 64, *bi = bi0 + s * NB * 64;
            int v[16];
#pragma unroll
            for (int mt = 0; mt < 4; mt++) {
                // the lane's slot words of m-tile mt: rows 16 mt + 4 g4 + r
                const knn_v4i c4 =
                    *(const LDS_AS knn_v4i *)(cn + nofs(8 * (mt >> 1) + 4 * (g4 & 1) + 2 * (mt & 1) + (g4 >> 1)));
#pragma unroll
                for (int r = 0; r < 4; r++) v[4 * mt + r] = (int)((unsigned)A[s][mt][r] * 64u + (unsigned)c4[r]);
            }
            if (masked) {   // rows past the block, and the query itself
#pragma unroll
                for (int mt = 0; mt < 4; mt++)
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        const int rl = 16 * mt + 4 * g4 + r;
                        if (!(row0 + rl < nc && (long)c_base + row0 + rl != (long)q_base + myq[s])) v[4 * mt + r] = vnone[s];
                    }
            }
            int T = thr_v(s);
            int vm = i8x_max16(v);
            if (__ballot(vm >= T) == 0ull) continue;
            // survivors in (d^2, row) order, one a round per lane, into the
            // lane's LDS buffer; a full buffer anywhere merges the wave's
            do {
                if (vm >= T) {
                    const int slot = 31 - (vm & 31);
                    bk[64 * cnt[s]] = qn[s] - (vm >> 5);
                    bi[64 * cnt[s]] = idb + 32 * (slot >> 4) + 8 * ((slot >> 2) & 3) + (slot & 3);
                    cnt[s]++;
                }
                if (__ballot(cnt[s] == NB) != 0ull) {
                    merge(s);
                    T = thr_v(s);
                }
                vm = i8x_next16(v, vm, vnone[s]);
            } while (__ballot(vm >= T) != 0ull);
        }
    };

    // ---- main loop -------------------------------------------------------------
    if (total > 0) {
#pragma unroll
        for (int y = 0; y < NST - 2; y++) stage();
        wait_next();
        __builtin_amdgcn_s_barrier();
        knn_v4i a[4];
#pragma unroll
        for (int mt = 0; mt < 4; mt++) a[mt] = rdA1(0, 0, mt);
        stage();
        int x = 0;
        unsigned xs = 0, ts = (unsigned)t_lo % NST;   // ring slots of chunk x and tile t
        e_b = i8_blk_of(tab, t_lo);
        e_t0 = i8_rfl(tab->t0[e_b]);
        e_t1 = i8_rfl(tab->t0[e_b + 1]);
        c_base = (long)i8_rfl64(tab->base[e_b]);
        nc = i8_rfl(tab->nc[e_b]);
        for (int t = t_lo; t < t_hi; t++) {
            if (t == e_t1) {   // the epilogue's block moves on
                e_b++;
                e_t0 = e_t1;
                e_t1 = i8_rfl(tab->t0[e_b + 1]);
                c_base = (long)i8_rfl64(tab->base[e_b]);
                nc = i8_rfl(tab->nc[e_b]);
            }
            knn_v4i acc[2][4];
#pragma unroll
            for (int s = 0; s < 2; s++)
#pragma unroll
                for (int mt = 0; mt < 4; mt++) acc[s][mt] = (knn_v4i){0, 0, 0, 0};
#pragma unroll
            for (int c = 0; c < NCH; c++) {
                const int kt = NK - 2 * c < 2 ? NK - 2 * c : 2;   // static after unrolling
#pragma unroll
                for (int ks2 = 0; ks2 < 2; ks2++) {
                    if (ks2 < kt) {
                        // the chunk's last step: chunk x + 1 must be in LDS
                        // before its first fragments are read
                        const bool last = ks2 + 1 >= kt;
                        const bool more = !last || x + 1 < total;
                        if (NRL > 0 && c == CI && last) reload();
                        if (last && x + 1 < total) {
                            wait_next();
                            __builtin_amdgcn_s_barrier();   // B(x + 1)
                            stage();
                        }
                        if (NRL > 0 && 2 * c + ks2 == NRES) reload_ready();
#if I8X_PF
                        // the next step's 4 fragments first, then this step's MFMAs
                        knn_v4i an[4];
#pragma unroll
                        for (int mt = 0; mt < 4; mt++)
                            if (more) an[mt] = last ? rdA1(xs + 1 == NST ? 0 : xs + 1, 0, mt) : rdA1(xs, ks2 + 1, mt);
                        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                        for (int mt = 0; mt < 4; mt++) {
                            acc[0][mt] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[mt], qfrag(0, 2 * c + ks2), acc[0][mt], 0, 0, 0);
                            acc[1][mt] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[mt], qfrag(1, 2 * c + ks2), acc[1][mt], 0, 0, 0);
                        }
#pragma unroll
                        for (int mt = 0; mt < 4; mt++) a[mt] = an[mt];
#else
#pragma unroll
                        for (int mt = 0; mt < 4; mt++) {
                            acc[0][mt] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[mt], qfrag(0, 2 * c + ks2), acc[0][mt], 0, 0, 0);
                            acc[1][mt] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[mt], qfrag(1, 2 * c + ks2), acc[1][mt], 0, 0, 0);
                            // the next step's fragment of this m-tile into the slot
                            if (more) a[mt] = last ? rdA1(xs + 1 == NST ? 0 : xs + 1, 0, mt) : rdA1(xs, ks2 + 1, mt);
                            __builtin_amdgcn_sched_barrier(0);
                        }
#endif
                    }
                }
                x++;
                xs = xs + 1 == NST ? 0 : xs + 1;
            }
#if I8X_NOEPI
            {   // (diagnostic build: the epilogue replaced by a sink of the accumulators)
                int sk = 0;
#pragma unroll
                for (int s = 0; s < 2; s++)
#pragma unroll
                    for (int mt = 0; mt < 4; mt++)
#pragma unroll
                        for (int r = 0; r < 4; r++) sk ^= acc[s][mt][r];
                if (sk == 0x12345678) part_T[0] = 1.0;
            }
#else
            epilogue(t, ts, acc, x);
#endif
            ts = ts + 1 == NST ? 0 : ts + 1;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no LDS-DMA left in flight
        if (q_ready >= 0) qthr_apply();
    }
#pragma unroll
    for (int s = 0; s < 2; s++) merge(s);

    // strict publication (k_dist_topk_i8): if none of the query's lanes ends
    // its list at thr, every rejected candidate has d^2 >= next(thr)
#pragma unroll
    for (int s = 0; s < 2; s++) {
        int lastmin = L[s][KL - 1];
        int o = __shfl_xor(lastmin, 16);
        lastmin = o < lastmin ? o : lastmin;
        o = __shfl_xor(lastmin, 32);
        lastmin = o < lastmin ? o : lastmin;
        double pub = thr[s] == I8_INF ? KNN_INF : (double)thr[s];
        if (lastmin > thr[s] && thr[s] < I8_INF) pub = nextafter((double)thr[s], KNN_INF);
        if (myq[s] < nq) {
            const size_t base = (((size_t)split * nq_pad + myq[s]) * LPQ + g4) * KL;
#pragma unroll
            for (int e = 0; e < KL; e++) {
                part_d[base + e] = L[s][e] == I8_INF ? KNN_INF : (double)L[s][e];
                part_i[base + e] = I[s][e];
            }
            if (g4 == 0) part_T[(size_t)split * nq_pad + myq[s]] = pub;
            if (g4 == 0 && qthr != nullptr && thr[s] < I8_INF)
                atomicMin(qthr + myq[s], (unsigned long long)__double_as_longlong((double)thr[s]));
        }
    }
}

// a 7-stage ring: the second query group's survivor buffers take the 8th
// stage's LDS (two workgroups a CU: <= 80 KiB each)
template <int NK>
static void launch_i8x(dim3 grid, hipStream_t s, const void *qsh, size_t q_rows_pad, size_t q_base, int nq,
                       const knn_i8_blocks_t &cb, size_t c_rows_pad, int rs, int ntiles, int nsplit, int nqb,
                       double *part_d, int *part_i, double *part_T, int nq_pad, double *qthr, int uj)
{
    hipLaunchKernelGGL(HIP_KERNEL_NAME(k_dist_topk_i8x<KNN_I8_KL_X, NK, 7, 5>), grid, dim3(256), 0, s,
                       (const signed char *)qsh, q_rows_pad, q_base, nq, cb, c_rows_pad, rs, ntiles, nsplit, nqb,
                       part_d, part_i, part_T, nq_pad, (unsigned long long *)qthr, uj);
}

// called by knn_launch_dist_i8 (knn_i8.hip) for kl == KNN_I8_KL_X with the
// validated, padded block table
int knn_launch_dist_i8x(const void *qsh, size_t q_rows_pad, size_t q_base, int nq, const knn_i8_blocks_t *cb,
                        size_t c_rows_pad, int rs, int ntiles, int nsplit, int nqb, double *part_d, int *part_i,
                        double *part_T, int nq_pad, double *qthr, int uj, void *stream)
{
    const int nk = (rs + 63) / 64;
    if (rs <= 128 || nk > 14) return KNN_ERR_INVALID;   // long rows only (<= KNN_I8_MAX_N bytes)
    const dim3 grid((unsigned)(nqb * nsplit));
    hipStream_t s = (hipStream_t)stream;
#define I8X_ARGS grid, s, qsh, q_rows_pad, q_base, nq, *cb, c_rows_pad, rs, ntiles, nsplit, nqb, part_d, part_i, \
                 part_T, nq_pad, qthr, uj
    if (nk <= 4) launch_i8x<4>(I8X_ARGS);
    else if (nk <= 8) launch_i8x<8>(I8X_ARGS);
    else if (nk <= 13) launch_i8x<13>(I8X_ARGS);
    else launch_i8x<14>(I8X_ARGS);
#undef I8X_ARGS
    return hipGetLastError() == hipSuccess ? KNN_OK : KNN_ERR_HIP;
}
