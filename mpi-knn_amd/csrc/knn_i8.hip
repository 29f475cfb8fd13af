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
#include "knn_i8_dev.h"

// One wave per row: x' = x - o (0 past n), |x'|^2 reduced in int32 (exact:
// n 128^2 < 2^31) and stored as the epilogue's norm word (i8_norm_word).  Lane l converts the 8-element groups l, l + 64, ... of
// the row: 16-byte vector loads (a wave reads 64 contiguous groups), one
// 8-byte store.  o from the REDUCED meta, so every block of one search
// shifts alike.
template <typename T>
__global__ __launch_bounds__(256) void k_shadow8(signed char *__restrict__ dst, const T *__restrict__ src,
                                                 size_t rows_pad, int n, int nps, int rs,
                                                 const double *__restrict__ meta)
{
    typedef typename std::conditional<sizeof(T) == 8, dbl2, flt4>::type vec_t;
    constexpr int V = 16 / (int)sizeof(T);            // elements per 16-byte load
    int *norms = (int *)(dst + rows_pad * (size_t)rs);
    const int off = 128 - (int)meta[KNN_META_MAXNEG];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int ng = rs / 8;                             // 8-byte output groups a row
    for (size_t r = (size_t)blockIdx.x * 4 + wave; r < rows_pad; r += (size_t)gridDim.x * 4) {
        const T *x = src + r * (size_t)nps;
        int s = 0;
        for (int g = lane; g < ng; g += 64) {
            const int j0 = 8 * g;
            T v[8];
            if (j0 + 8 <= nps) {                        // whole group inside the padded row
#pragma unroll
                for (int q = 0; q < 8 / V; q++) {
                    const vec_t w = *(const vec_t *)(x + j0 + V * q);
#pragma unroll
                    for (int e = 0; e < V; e++) v[V * q + e] = w[e];
                }
            } else {
#pragma unroll
                for (int e = 0; e < 8; e++) v[e] = j0 + e < nps ? x[j0 + e] : (T)0;
            }
            unsigned lo = 0, hi = 0;
#pragma unroll
            for (int e = 0; e < 8; e++) {
                const int xi = j0 + e < n ? (int)v[e] - off : 0;
                s += xi * xi;
                if (e < 4) lo |= ((unsigned)xi & 0xffu) << (8 * e);
                else hi |= ((unsigned)xi & 0xffu) << (8 * (e - 4));
            }
            typedef unsigned u2 __attribute__((ext_vector_type(2)));
            *(u2 *)(dst + r * (size_t)rs + j0) = (u2){lo, hi};
        }
        for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
        if (lane == 0) {
            norms[i8_norm_pos((int)r)] = i8_norm_word((int)r, s, rs);
            norms[rows_pad + i8_norm_pos((int)r)] = i8_init_word(s, rs);
        }
    }
}

// ---------------------------------------------------------------------------
// k_dist_topk_i8
//
// Workgroup: W waves (4 or 8), 128 queries x a corpus split streamed in
// tiles of 128 rows and chunks of 128 bytes (128 features, 4 K-steps of 32).
// Wave w: queries 32 (w & 3) .. +31, m-blocks (32-row blocks of the tile)
// MB (w >> 2) .. +MB-1, MB = 16 / W.  With W = 8 two waves share each SIMD,
// so one wave's epilogue runs beside its partner's MFMAs.
//
// Operands (v_mfma_i32_32x32x32_i8, D = A.B): A = 32 corpus rows (one
// m-block), B = the wave's 32 queries; lane l (r = l & 31, h = l >> 5)
// supplies 16 bytes [32 s + 16 h, +16) of K-step s of row r / query r -- the
// same byte slots on both sides, so the sum runs over every feature once.
// D: lane l holds query r, rows 32b + 8(reg >> 2) + 4h + (reg & 3).  A
// query's candidates of a tile sit in 2 lanes of each wave covering it; each
// lane keeps its own list (lpq = 2 W / 4 lists per query), bounds are shared.
//
// Queries are resident in registers (4 VGPRs per K-step, loaded once); the
// corpus streams through an NST-stage LDS ring of 16 KiB chunk images filled
// by LDS-DMA (buffer_load_dwordx4 ... lds), 16 pieces of 8 rows x 128 B per
// chunk, 16 / W per wave.  Image: [row 128][128 B], 16-byte segment s of row
// r at slot s ^ ((r >> 1) & 7): the ds_read_b128 lane groups ({0-3,12-15,
// 20-27}, ...) hit 16 distinct bank quads.  The K-step count NKS is a
// template bucket (>= the data's; the extra K-steps multiply zero query
// fragments), so the chunk loop is static.  Barrier B(y) (chunk y visible) sits before the last K-step
// of chunk y-1, after the wave's counted vmcnt for its own pieces of chunk y;
// chunk y's first fragments then load under the last MFMAs of chunk y-1, and
// the stage of chunk y-2 takes chunk y + NST - 2.  Chunks past the split's
// end re-stage its last chunk (static count).  A tile's norms (512 B,
// permuted, i8_norm_pos) ride with its first chunk into a norm ring.
//
// Epilogue per tile: key = |c'|^2 - 2 q'.c' (int32) and the lane minimum
// against min(own KL-th, shared bound) - |q'|^2; survivors, lowest row first
// (the stable tie order), go through a select tree into a per-lane LDS
// buffer of NB entries (d^2 = key + |q'|^2).  When some lane's buffer is
// full the wave merges all buffers into the KL-entry register lists (one
// entry a round through the insertion network) and refreshes the bounds, so
// the network runs on dense rounds instead of once per survivor of the
// busiest lane per tile.  d^2 is exact, so "S != 0" (serial:86) is d^2 > 0,
// applied at the merge.
//
// Ablations of this kernel (no epilogue, keys only, no DMA, no barrier, no
// MFMA, survivor counters) were measured with the tuning
// harness at commit 8ea8e2a; the product source carries no hooks.
// ---------------------------------------------------------------------------
template <int KL, int NKS, int W, int WPS, int NST, int NB, int TM, int QG = 1>
__global__ __launch_bounds__(64 * W, WPS) void k_dist_topk_i8(
    const signed char *__restrict__ qsh, size_t q_rows_pad, size_t q_base, int nq,
    const knn_i8_blocks_t cb, size_t c_rows_pad, int rs,
    int nks, int ntiles, int nsplit, int nqb, double *__restrict__ part_d,
    int *__restrict__ part_i, double *__restrict__ part_T, int nq_pad,
    unsigned long long *__restrict__ qthr, int uj, unsigned long long *__restrict__ qsum)
{
    // TM m-blocks (32 rows each) a tile: 4 (128-row tiles) or 2 (64-row
    // half tiles: 4 waves, two workgroups a CU).  The 4 query groups of 32
    // take RHN = W / 4 waves each, MB = TM / RHN m-blocks a wave.  QG = 2
    // (short rows, 4 waves): each wave carries two groups of 32 queries
    // (workgroup queries 32 w.. and 128 + 32 w..) against the same A
    // fragments and accumulator init words -- every LDS byte read and every
    // corpus byte staged feeds twice the MFMAs (256 queries a workgroup).
    constexpr int TR = 32 * TM;             // rows a tile
    constexpr int RHN = W / 4;              // waves a query group (row halves)
    constexpr int MB = TM / RHN;            // m-blocks per wave
    constexpr int CHB = TR * 128;           // bytes a chunk (TR rows x 128 features)
    constexpr int PW = CHB / 1024 / W;      // DMA pieces (1 KiB) per wave per chunk
    constexpr int LPQ = 2 * RHN;            // lists per query
    constexpr int NRB = TR * 8;             // norm ring bytes a stage: slot + init words
    constexpr int WPW = TR / W;             // norm words a wave stages of each array
    constexpr int NSEG = 8 * WPW;           // a wave's staged piece (both arrays)
    constexpr int NORM0 = NST * CHB;        // norm ring: [NST][W][slot words, init words]
    // norm ring: NNR >= NST tile slots; a one-tile chunk ring (NST = chunks
    // a tile, e.g. 7) takes 8, a power of two, so that no epilogue or norm
    // stage computes a modulo-7
    constexpr int NNR = NST == (NKS + 3) / 4 ? 8 : NST;
    constexpr int BUF0 = NORM0 + NNR * NRB; // [W][QG][NB][64] survivor d^2, then ids
    constexpr int XB0 = BUF0 + 2 * W * QG * NB * 256;   // RHN = 2: [8][32] bound exchange (u4, v8, v16)
    constexpr int TB0 = XB0 + (RHN == 2 ? 3 * 8 * 32 * 4 : 0);   // block table
    static_assert(MB == 2 || MB == 4, "m-blocks a wave");
    static_assert(PW == 2 || PW == 4, "DMA pieces a wave");
    static_assert(QG == 1 || (QG == 2 && RHN == 1 && NKS <= 8), "two query groups: 4-wave short-row kernels");
    constexpr int QB = 128 * QG;            // queries a workgroup
    // rows of <= 4 K-steps carry init words (K2 / IW form); longer rows the
    // whole norm in the slot word and zero init words (knn_device.h): their
    // accumulators start at zero, no init-word reads
    constexpr bool SHORT = NKS <= 4;
    constexpr int LDSB = TB0 + (int)((sizeof(i8_tab_lds) + 15) / 16 * 16);
    __shared__ __attribute__((aligned(16))) char smem[LDSB];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int wave_s = __builtin_amdgcn_readfirstlane(wave);
    const int qg = wave_s & 3, rh = wave_s >> 2;
    const int r32 = lane & 31, h = lane >> 5;
    // split-major order: long splits first (knn_engine.c: choose_splits);
    // a query block's later splits start from the bounds its earlier ones
    // published (qthr)
    const int qb = blockIdx.x % nqb, split = blockIdx.x / nqb;
    // the host counts 128-row tiles; this kernel's tiles hold TR rows
    constexpr int TS = 4 / TM;
    ntiles *= TS;
    const int tb = ntiles / nsplit, tr = ntiles - tb * nsplit;
    const int t_lo = split * tb + (split < tr ? split : tr);
    const int t_hi = t_lo + tb + (split < tr ? 1 : 0);
    const int qrow0 = qb * QB;
    // query of group g; padding queries (>= nq) load row nq - 1 (with QG = 2
    // the last block may reach past the query block's rows) and reject all
    int myq[QG], lq[QG];
    long gq[QG];
#pragma unroll
    for (int g = 0; g < QG; g++) {
        myq[g] = qrow0 + 128 * g + 32 * qg + r32;
        lq[g] = myq[g] < nq ? myq[g] : nq - 1;
        gq[g] = (long)q_base + myq[g];
    }
    constexpr int NCH = (NKS + 3) / 4;      // chunks a tile
    const int nch = NCH;
    const int *qnorms = (const int *)(qsh + q_rows_pad * (size_t)rs);

    // ---- resident query fragments (B), one per K-step --------------------
    // NKS >= nks K-steps (the instantiation's bucket): those past nks get
    // zero fragments, so the (garbage) corpus bytes they meet add nothing.
    knn_v4i qf[QG][NKS];
    int qn[QG];   // |q'|^2
#pragma unroll
    for (int g = 0; g < QG; g++) {
        const signed char *qrow = qsh + (size_t)lq[g] * rs + 16 * h;
#pragma unroll
        for (int s = 0; s < NKS; s++) {
            const int sl = s < nks ? s : nks - 1;
            const knn_v4i v = *(const knn_v4i *)(qrow + 32 * sl);
            qf[g][s] = s < nks ? v : (knn_v4i){0, 0, 0, 0};
        }
        qn[g] = i8_norm_of(qnorms[i8_norm_pos(lq[g])], qnorms[q_rows_pad + i8_norm_pos(lq[g])]);
    }
    // shared per-query bound across splits and ring steps (qthr: bits of a
    // non-negative double, atomicMin).  INT-mode bounds are integers, or the
    // next double above one (strict publication), so floor() is the int bound.
    int thr[QG];
#pragma unroll
    for (int g = 0; g < QG; g++) {
        thr[g] = I8_INF;
        if (qthr != nullptr && myq[g] < nq) {
            const double td = __longlong_as_double((long long)atomicMin(qthr + myq[g], 0x7ff0000000000000ull));
            thr[g] = td >= 2147483647.0 ? I8_INF : (int)td;
        }
    }
    // padding queries of the last block (myq >= nq) reject every candidate:
    // with an open bound their lanes took the insertion path for every row,
    // and the one workgroup holding them set the launch's span (a 7500-row
    // ring step: 134 us against a 74 us average workgroup)
#pragma unroll
    for (int g = 0; g < QG; g++)
        if (myq[g] >= nq) thr[g] = -1;
    // vmcnt(0) through the builtin: hipcc's wait pass then knows the query
    // loads are complete (an asm wait would leave it inserting vmcnt(N)
    // before each later use of qf, draining the LDS-DMA ring)
    __builtin_amdgcn_s_waitcnt(0x0F70);

    int L[QG][KL], I[QG][KL];
#pragma unroll
    for (int g = 0; g < QG; g++)
#pragma unroll
        for (int e = 0; e < KL; e++) { L[g][e] = I8_INF; I[g][e] = -1; }
    // uj: list slot of the 2-lane bound (low byte) and of the 4-lane bound
    // (W = 8: the query's lanes in both waves; second byte)
    const int ujm = (uj & 255) < KL - 1 ? (uj & 255) : KL - 1;
    const int uj4 = ((uj >> 8) & 255) < KL - 1 ? ((uj >> 8) & 255) : KL - 1;
    LDS_AS int *xb = (LDS_AS int *)(smem + XB0);   // [3][8 waves][32]: u4, v8, v16
    // group g's entry e at bk0[64 (g NB + e)], its id W QG NB 64 words on
    LDS_AS int *bk0 = (LDS_AS int *)(smem + BUF0) + wave_s * QG * NB * 64 + lane;
    LDS_AS int *bi0 = bk0 + W * QG * NB * 64;
    int cnt[QG];   // buffered survivors of this lane
#pragma unroll
    for (int g = 0; g < QG; g++) cnt[g] = 0;
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
        for (int j = 0; j <= KNN_I8_MAXBLK; j++) tab->t0[j] = cb.t0[j] * TS;
        tab->nblk = cb.nblk;
    }
    if constexpr (RHN == 2) {
        if (h == 0) {
#pragma unroll
            for (int j = 0; j < 3; j++) xb[256 * j + wave_s * 32 + r32] = I8_INF;
        }
    }
    __syncthreads();

    // ---- staging ---------------------------------------------------------
    const int total = (t_hi > t_lo) ? (t_hi - t_lo) * nch : 0;
    unsigned voff[PW];
#pragma unroll
    for (int p = 0; p < PW; p++) {
        const int rr = (TR / W) * wave_s + 8 * p + (lane >> 3);
        voff[p] = (unsigned)(rr * rs + 16 * ((lane & 7) ^ ((rr >> 1) & 7)));
    }
    const unsigned lds0 = (unsigned)(uintptr_t)smem;
    // staging position: global tile s_t of block s_b, chunk byte offset
    // s_coff; s_row / s_nrow point at the tile's row 0 / first norm word and
    // advance by a tile at a time (wave-uniform: scalar registers)
    int s_t = t_lo, s_x = 0;
    unsigned s_coff = 0;
    int s_b = i8_blk_of(tab, t_lo);
    const int s_t0 = i8_rfl(tab->t0[s_b]);
    int s_t1 = i8_rfl(tab->t0[s_b + 1]);
    const signed char *s_row = (const signed char *)(uintptr_t)i8_rfl64((long long)tab->ptr[s_b]) +
                               (size_t)(t_lo - s_t0) * TR * rs;
    const int *s_nrow = (const int *)(uintptr_t)i8_rfl64((long long)tab->nptr[s_b]) + (size_t)(t_lo - s_t0) * TR;
    auto stage = [&]() {
        const unsigned dst = lds0 + ((unsigned)s_x % NST) * (unsigned)CHB + (unsigned)wave_s * (unsigned)(CHB / W);
        if constexpr (PW == 4) bglds16x4(i8_rsrc(s_row + s_coff), voff[0], voff[1], voff[2], voff[3], dst);
        else bglds16x2(i8_rsrc(s_row + s_coff), voff[0], voff[1], dst);
        // (one-chunk tiles: every stage carries its norm piece, the tail's
        // re-stages too -- the last tile's words again -- so that wait_next
        // can count it)
        if ((NCH == 1 || s_x < total) && s_coff == 0) {
            // the tile's two norm arrays in one piece a wave: lanes <
            // WPW / 4 the slot words, the next WPW / 4 lanes the init words
            // of the same rows (c_rows_pad words further on)
            if (lane < WPW / 2)
                bglds16(i8_rsrc(s_nrow + WPW * wave_s),
                        lane < WPW / 4 ? 16u * lane : 4u * (unsigned)c_rows_pad + 16u * (lane - WPW / 4),
                        lds0 + NORM0 + ((unsigned)s_t % NNR) * (unsigned)NRB + (unsigned)NSEG * wave_s);
        }
        s_x++;
        if (s_x < total) {
            s_coff += 128;
            if (s_coff == 128u * nch) {
                s_coff = 0;
                if (++s_t == s_t1) {   // next block of the launch
                    s_b++;
                    s_row = (const signed char *)(uintptr_t)i8_tab64(&tab->ptr[s_b]);
                    s_nrow = (const int *)(uintptr_t)i8_tab64(&tab->nptr[s_b]);
                    s_t1 = i8_tab32(&tab->t0[s_b + 1]);
                } else {
                    s_row += (size_t)TR * rs;
                    s_nrow += TR;
                }
            }
        }
    };
    // PF2's staging (the two-deep loop below): the chunk staged behind B(y)
    // is z = y + NST - 2, and y's position in its tile is static at every
    // call site, so z's position pz is too.  The chunk offset then rides in
    // soffset against one descriptor of the tile's rows (cached: rebuilt once
    // a tile), the norm piece goes out only at the site of a tile's first
    // chunk and the cursor advances only at the site of its last -- where
    // stage() spent ~40 scalar instructions a chunk on offsets, compares and
    // an exec-masked branch.  Past the split's end the last tile's rows are
    // re-staged (their slots are never read: the static count of pieces is
    // what the ring's waits assume).
    knn_v4i s_rs = i8_rsrc(s_row);
    // With a one-tile ring (NST == NCH) the slot of a chunk is its position
    // in its tile: static, like pz, so neither the stage's LDS address nor
    // the fragment reads' need slot arithmetic (rdA's base folds into the
    // ds_read offset)
    constexpr bool SSLOT = NST == NCH;
    auto stage_at = [&](int pz) {
        const unsigned dst = lds0 + (SSLOT ? (unsigned)pz : (unsigned)s_x % NST) * (unsigned)CHB +
                             (unsigned)wave_s * (unsigned)(CHB / W);
        bglds16x2s(s_rs, voff[0], voff[1], 128u * (unsigned)pz, dst);
        // (unconditional: past the split's end the cursor stays on the last
        // tile, so this re-stages that tile's words into its own slot --
        // identical bytes; a uniform branch here cost 242 VGPRs of spills)
        if (pz == 0)
            bglds16m(i8_rsrc(s_nrow + WPW * wave_s),
                     lane < WPW / 4 ? 16u * lane : 4u * (unsigned)c_rows_pad + 16u * (lane - WPW / 4),
                     lds0 + NORM0 + ((unsigned)s_t % NNR) * (unsigned)NRB + (unsigned)NSEG * wave_s,
                     (1ull << (WPW / 2)) - 1);
        s_x++;
        if (pz == NCH - 1 && s_x < total) {   // the next tile
            if (++s_t == s_t1) {   // next block of the launch
                s_b++;
                s_row = (const signed char *)(uintptr_t)i8_tab64(&tab->ptr[s_b]);
                s_nrow = (const int *)(uintptr_t)i8_tab64(&tab->nptr[s_b]);
                s_t1 = i8_tab32(&tab->t0[s_b + 1]);
            } else {
                s_row += (size_t)TR * rs;
                s_nrow += TR;
            }
            s_rs = i8_rsrc(s_row);
        }
    };
    // One-chunk tiles (SIFT's <= 4 K-steps; PW = 2): every stage opens a
    // tile, so stage1 keeps the ring slot and the norm-ring slot as counters
    // (NST = 7 there: no modulo-7 a stage), the chunk at soffset 0 of the
    // tile's cached descriptor, the norm piece under an asm exec mask (the
    // tail re-stages the last tile's words, as stage() does for these tiles)
    // and the cursor one tile on -- stage()'s offset arithmetic and branches
    // ran once a tile of 16 MFMAs here.  s_slot / s_nslot / s_rs are set
    // from the cursor after the prologue's stages.
    constexpr bool ONE = NCH == 1 && PW == 2;
    int s_slot = 0, s_nslot = 0;
    auto stage1 = [&]() {
        const unsigned dst = lds0 + (unsigned)s_slot * (unsigned)CHB + (unsigned)wave_s * (unsigned)(CHB / W);
        bglds16x2s(s_rs, voff[0], voff[1], 0u, dst);
        bglds16m(i8_rsrc(s_nrow + WPW * wave_s),
                 lane < WPW / 4 ? 16u * lane : 4u * (unsigned)c_rows_pad + 16u * (lane - WPW / 4),
                 lds0 + NORM0 + (unsigned)s_nslot * (unsigned)NRB + (unsigned)NSEG * wave_s, (1ull << (WPW / 2)) - 1);
        s_x++;
        s_slot = s_slot == NST - 1 ? 0 : s_slot + 1;
        if (s_x < total) {
            if (++s_t == s_t1) {   // next block of the launch
                s_b++;
                s_row = (const signed char *)(uintptr_t)i8_tab64(&tab->ptr[s_b]);
                s_nrow = (const int *)(uintptr_t)i8_tab64(&tab->nptr[s_b]);
                s_t1 = i8_tab32(&tab->t0[s_b + 1]);
            } else {
                s_row += (size_t)TR * rs;
                s_nrow += TR;
            }
            s_rs = i8_rsrc(s_row);
            s_nslot = s_nslot == NNR - 1 ? 0 : s_nslot + 1;
        }
    };
    // the next chunk's own pieces landed: the NST - 3 chunks staged after it
    // may stay in flight.  One-chunk tiles (SIFT) count each stage's norm
    // piece too: counted as PW a stage, the wait also drained a third of the
    // younger stages and the ring ran ~2 tiles ahead instead of NST - 3.
    // (The shared-bound loads issued between stages only make it stricter.)
    auto wait_next = [&]() {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NCH == 1 ? PW + 1 : PW) * (NST - 3)) : "memory");
    };
    // A fragments (MB m-blocks) of K-step ks of staged chunk xx
    // norm ring: byte offset of 16-byte group v (i8_norm_pos order, 4 words)
    // of a tile's slot words; its init words sit NSEG / 2 bytes further
    auto nofs = [&](int v) -> int { return (v / (WPW / 4)) * NSEG + (v % (WPW / 4)) * 16; };
    // accumulator init words of tile tt for the wave's MB m-blocks (the C
    // operand of the tile's first K-step): 4 ds_read_b128 an m-block
    auto rdI = [&](int tt, knn_v16i (&ini)[MB]) {
        const LDS_AS char *p = (const LDS_AS char *)smem + NORM0 + ((unsigned)tt % NNR) * NRB + NSEG / 2;
#pragma unroll
        for (int bb = 0; bb < MB; bb++) {
            knn_v4i r[4];
#pragma unroll
            for (int j = 0; j < 4; j++) r[j] = *(const LDS_AS knn_v4i *)(p + nofs(4 * h + 8 * (MB * rh + bb) + j));
            const knn_v8i lo = __builtin_shufflevector(r[0], r[1], 0, 1, 2, 3, 4, 5, 6, 7);
            const knn_v8i hi = __builtin_shufflevector(r[2], r[3], 0, 1, 2, 3, 4, 5, 6, 7);
            ini[bb] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
        }
    };
    auto rdA = [&](int xx, int ks, knn_v4i (&a)[MB]) {
        const LDS_AS char *p = (const LDS_AS char *)smem + ((unsigned)xx % NST) * CHB + (MB * rh * 32 + r32) * 128 +
                               16 * ((2 * ks + h) ^ ((r32 >> 1) & 7));
#pragma unroll
        for (int bb = 0; bb < MB; bb++) a[bb] = *(const LDS_AS knn_v4i *)(p + bb * 4096);
    };

    // ---- bounds ------------------------------------------------------------------
    // The bound a lane filters with: every value is an upper bound on the
    // query's (k+1)-th smallest d^2 over all rows (or the lane's own KL-th,
    // which it rejects anyway).  The wave's 2 lanes hold >= 2(ujm+1) >= k+1
    // entries <= max_h L_h[ujm].  W = 8: the 4 lanes of both waves hold >=
    // 4(uj4+1) >= k+1 entries <= the max of their L[uj4]; the partner wave's
    // half comes through LDS, lock-free -- a stale value is larger (lists
    // only shrink), so the max stays a valid bound, only a looser one.
    // Cross-split summaries (W = 8, k + 1 <= 32): splits of one launch cover
    // disjoint rows, so 4 splits' v8 (8 rows each) or 2 splits' v16 bound
    // the query's (k+1)-th d^2 -- over the union of their rows, 4x the rows
    // behind one split's own 4-lane bound.  Split s keeps (v8 << 32 | v16)
    // in slot s & 3 of qsum[query][4] (atomic min of the packed pair: a slot
    // holds one split's consistent pair, the smaller v8); every split reads
    // the 4 slots with the qthr re-read.  Publication is rate-limited: the
    // atomic stays counted in vmcnt (~2-3k cycles) and the ring's next
    // counted wait would sit it out.
    // (the 12-entry-list kernels only: the 17-entry ones have no registers
    // to spare at 28 K-steps)
    // (k <= 32 kernels: the shared-bound re-read, and the summaries for the
    // 12-entry lists; a query's LPQ lanes hold 8 / 16 rows at or below
    // their L[S8] / L[S16])
    constexpr bool REREAD = KL != KNN_I8_KL_L;
    // (QG = 2: no summaries -- their 8 VGPRs a group spill there)
    // (the two-deep-prefetch kernels below (PF2): none either -- they
    // measured as worth nothing at P = 1 and at the P = 8 fused shape
    // (DESIGN.md sec.8), and their pointer and 8 VGPRs spilled there, with a
    // vmcnt(0) reload draining the staging ring every second tile)
    constexpr bool PF2 = TM == 2 && QG == 1 && NKS >= 8 && NKS <= 25;
    constexpr bool SUM = REREAD && KL == KNN_I8_KL_S && QG == 1 && !PF2;
    constexpr int S8 = 8 / LPQ - 1, S16 = 16 / LPQ - 1;
    int q_pubx[QG];
#pragma unroll
    for (int g = 0; g < QG; g++) q_pubx[g] = -1000;
    auto qsum_publish = [&](int g, int v8, int v16) {
        if (!SUM || qsum == nullptr || rh != 0 || h != 0 || myq[g] >= nq) return;
        if (v8 >= I8_INF || s_x - q_pubx[g] < 4 * nch) return;
        q_pubx[g] = s_x;
        const unsigned long long val = ((unsigned long long)(unsigned)v8 << 32) | (unsigned)v16;
        unsigned long long *pq = qsum + (size_t)myq[g] * 4 + (split & 3);
        asm volatile("global_atomic_umin_x2 %0, %1, off" ::"v"(pq), "v"(val) : "memory");
    };
    auto refresh = [&](int g) {
        int lmin = L[g][KL - 1], u = L[g][0], u4 = L[g][0];
#pragma unroll
        for (int e = 1; e < KL; e++) {
            u = (e == ujm) ? L[g][e] : u;
            u4 = (e == uj4) ? L[g][e] : u4;
        }
        const int lo = __shfl_xor(lmin, 32), uo = __shfl_xor(u, 32), u4o = __shfl_xor(u4, 32);
        lmin = lo < lmin ? lo : lmin;
        u = uo > u ? uo : u;
        u4 = u4o > u4 ? u4o : u4;
        // short lane lists (2 KL < k + 1, uj bit 16): no 2-lane bound.  lmin
        // stays: thr <= every lane's last entry is what makes the published
        // T a bound on the candidates a full list drops
        int nb = lmin < u ? lmin : u;
        if (uj & (1 << 16)) nb = lmin;
        if constexpr (RHN == 2) {
            if (h == 0) xb[wave_s * 32 + r32] = u4;
            const int pu = xb[(wave_s ^ 4) * 32 + r32];
            u4 = pu > u4 ? pu : u4;
            nb = u4 < nb ? u4 : nb;
        }
        if constexpr (SUM) {
            // the split's summary for the other splits: v8 / v16 = the max
            // over the query's LPQ lanes of L[S8] / L[S16] -- 8 / 16 rows of
            // this split lie at or below them
            int v8 = L[g][S8], v16 = L[g][S16];
            const int v8o = __shfl_xor(v8, 32), v16o = __shfl_xor(v16, 32);
            v8 = v8o > v8 ? v8o : v8;
            v16 = v16o > v16 ? v16o : v16;
            if constexpr (RHN == 2) {
                if (h == 0) {
                    xb[256 + wave_s * 32 + r32] = v8;
                    xb[512 + wave_s * 32 + r32] = v16;
                }
                const int p8 = xb[256 + (wave_s ^ 4) * 32 + r32], p16 = xb[512 + (wave_s ^ 4) * 32 + r32];
                v8 = p8 > v8 ? p8 : v8;
                v16 = p16 > v16 ? p16 : v16;
            }
            qsum_publish(g, v8, v16);
        }
        thr[g] = nb < thr[g] ? nb : thr[g];
    };
    // buffered survivors -> lists, in buffer (= row) order, one entry a
    // round; the rounds are dense: a merge runs when some lane's buffer is
    // full, so most lanes insert a real entry every round
    auto merge = [&](int g) {
        const LDS_AS int *bk = bk0 + g * NB * 64, *bi = bi0 + g * NB * 64;
        for (int e = 0; __ballot(e < cnt[g]) != 0ull; e++) {
            int d = I8_INF, id = -1;
            if (e < cnt[g]) {
                d = bk[64 * e];
                id = bi[64 * e];
                d = d > 0 ? d : I8_INF;   // d^2 == 0: an exact duplicate (serial:86)
            }
            i8_insert<KL>(L[g], I[g], d, id);
        }
        cnt[g] = 0;
        refresh(g);
    };
    // The shared bound may fall while the workgroup runs (other splits end,
    // and the merge of an earlier ring step publishes the running answer
    // while a fused launch runs), so W = 8 workgroups re-read it every
    // second tile of several chunks (every tile: 1.3% slower at P = 1, no
    // better at P = 8), every tile when a tile is one chunk (sift).  The load is issued from asm, invisible to the compiler's wait
    // pass: a plain load made it drain every LDS-DMA piece in flight
    // (vmcnt(0)) before the value's first use.  It is complete once the ring
    // has waited past the pieces staged after it (wait_next: all but the
    // NST - 3 youngest chunks), i.e. after chunk q_ready; only then is the
    // value laundered (asm "+v", ordered after those waits) and used.  A
    // load issued with s_x = X0 stages out is older than stage X0's pieces;
    // at an epilogue with xdone > X0 the wait before barrier B(xdone) (or,
    // on the last tile, B(total - 1) >= X0) has seen stage X0 land.
    unsigned long long q_bits[QG];
    knn_v4i qs0[QG], qs1[QG];   // qsum slots 0-1, 2-3
#pragma unroll
    for (int g = 0; g < QG; g++) {
        q_bits[g] = 0x7ff0000000000000ull;
        qs0[g] = (knn_v4i){I8_INF, I8_INF, I8_INF, I8_INF};
        qs1[g] = qs0[g];
    }
    int q_ready = -1;   // -1: no load pending
    auto qthr_issue = [&](int xnow) {
#pragma unroll
        for (int g = 0; g < QG; g++) {
            const unsigned long long *pq = qthr + lq[g];
            asm volatile("global_load_dwordx2 %0, %1, off sc1" : "=v"(q_bits[g]) : "v"(pq) : "memory");
            if (SUM && qsum != nullptr) {
                const unsigned long long *ps = qsum + (size_t)lq[g] * 4;
                asm volatile("global_load_dwordx4 %0, %1, off sc1" : "=v"(qs0[g]) : "v"(ps) : "memory");
                asm volatile("global_load_dwordx4 %0, %1, off offset:16 sc1" : "=v"(qs1[g]) : "v"(ps) : "memory");
            }
        }
        q_ready = xnow;
    };
    auto qthr_apply = [&]() {
#pragma unroll
        for (int g = 0; g < QG; g++) {
            asm volatile("" : "+v"(q_bits[g]));
            if constexpr (SUM) asm volatile("" : "+v"(qs0[g]), "+v"(qs1[g]));
            const double td = __longlong_as_double((long long)q_bits[g]);
            int tq = td >= 2147483647.0 ? I8_INF : (int)td;
            if (SUM && qsum != nullptr) {
                // slot s = (v16, v8) as (lo, hi) dwords: qs0 = {v16_0, v8_0, v16_1, v8_1}
                const knn_v4i x0 = qs0[g], x1 = qs1[g];
                const int a8 = x0.y > x0.w ? x0.y : x0.w, b8 = x1.y > x1.w ? x1.y : x1.w;
                const int b4 = a8 > b8 ? a8 : b8;                        // 4 splits x 8 rows
                const int s1 = x0.x < x0.z ? x0.x : x0.z, l1 = x0.x < x0.z ? x0.z : x0.x;
                const int s2 = x1.x < x1.z ? x1.x : x1.z, l2 = x1.x < x1.z ? x1.z : x1.x;
                const int m1 = s1 > s2 ? s1 : s2, m2 = l1 < l2 ? l1 : l2;
                const int b2 = m1 < m2 ? m1 : m2;                        // 2nd smallest v16: 2 x 16 rows
                const int bs = b4 < b2 ? b4 : b2;
                tq = bs < tq ? bs : tq;
            }
            thr[g] = tq < thr[g] ? tq : thr[g];
        }
        q_ready = -1;
    };

    // ---- epilogue of tile t --------------------------------------------------
    // t: global tile of the launch; lt / c_base / nc: its block's tile,
    // first global id and rows (kept by the main loop)
    long c_base = 0;
    int nc = 0, e_t0 = 0, e_t1 = 0, e_b = 0;
    // Survivors are the candidates with d^2 <= lim = min(own KL-th, shared
    // bound).  The accumulators started at the rows' init words, so acc =
    // (|q'|^2 - d^2 + p) / 2 (i8_init_word): the filter 2 acc >= |q'|^2 -
    // lim <=> d^2 <= lim + p, i.e. acc >= Ta = ceil((|q'|^2 - lim) / 2), admits all of them
    // (and rows with d^2 = lim + 1, p = 1), straight off the MFMA output.
    // Lanes that pass build the exact keys v = 64 acc + K2 and select with
    // v >= T = 32 (|q'|^2 - lim).  An empty list (lim = INF) admits every
    // real candidate: Ta = INT_MIN + 1, T = 32 (|q'|^2 - DMAX) with DMAX
    // above every d^2 (n 255^2 < DMAX); masked slots take acc = INT_MIN /
    // v = vnone = T_open - 1, below every threshold.
    const int dmax = rs * 65025 + 1;
    int vnone[QG];
#pragma unroll
    for (int g = 0; g < QG; g++) vnone[g] = 32 * (qn[g] - dmax) - 1;
    constexpr int A_NONE = (int)0x80000000;
    auto thr_v = [&](int g) -> int {
        const int lim = L[g][KL - 1] < thr[g] ? L[g][KL - 1] : thr[g];
        return lim >= dmax ? vnone[g] + 1 : 32 * (qn[g] - lim);
    };
    auto thr_a = [&](int g) -> int {
        const int lim = L[g][KL - 1] < thr[g] ? L[g][KL - 1] : thr[g];
        return lim >= dmax ? A_NONE + 1 : (qn[g] - lim + 1) >> 1;
    };
    // short rows (<= 4 K-steps, SIFT; i8_long_rows): the accumulator
    // filter; their byte blocks carry the init words it needs
    constexpr bool ACCF = SHORT;
    auto epilogue = [&](int t, knn_v16i (&A)[QG][MB], int xdone) {
        const int lt = t - e_t0;
        const LDS_AS char *cn = (const LDS_AS char *)smem + NORM0 + ((unsigned)t % NNR) * NRB;
        const int row0 = lt * TR + 32 * MB * rh;
        const bool rmask = row0 + 32 * MB > nc;
        // (32-bit row ids: every id is an int, so the low words' difference
        // is the difference; the 64-bit compares ran as VALU ops a tile)
        const int gt0 = (int)c_base + row0;
        const int idb = gt0 + 4 * h;
        if constexpr (REREAD) {
            if (qthr != nullptr) {
                if (q_ready >= 0 && xdone > q_ready) qthr_apply();
                if (q_ready < 0 && (NCH == 1 || (t & 1) == 0)) qthr_issue(s_x);   // mnist: 3.89 -> 3.84 ms (kbench8)
            }
        }
#pragma unroll
        for (int g = 0; g < QG; g++) {
        const int gw0 = (int)q_base + qrow0 + 128 * g + 32 * qg;
        // the wave's 32 queries meet the wave's 32 MB rows: -32 < gw0 - gt0 < 32 MB
        const bool masked = rmask || (unsigned)(gw0 - gt0 + 31) < (unsigned)(32 * MB + 31);
        LDS_AS int *bk = bk0 + g * NB * 64, *bi = bi0 + g * NB * 64;
        // pairs of m-blocks = 32 candidates a lane, lower rows first (the
        // stable tie order across pairs; inside one, v orders by row)
#pragma unroll
        for (int pr = 0; pr < MB / 2; pr++) {
            int a[32];
#pragma unroll
            for (int bb = 0; bb < 2; bb++)
#pragma unroll
                for (int i = 0; i < 16; i++) a[16 * bb + i] = A[g][2 * pr + bb][i];
            if (masked) {   // rows past the block, and the query itself (acc > -2^25 otherwise)
#pragma unroll
                for (int x = 0; x < 32; x++) {
                    const int rloc = 32 * (2 * pr + (x >> 4)) + 8 * ((x >> 2) & 3) + (x & 3);
                    if (!(row0 + rloc + 4 * h < nc && idb + rloc != gq[g])) a[x] = A_NONE;
                }
            }
            // short rows (SHORT: SIFT) -- most groups end here, late in
            // the scan; long rows (MNIST) almost always hold a survivor in
            // some lane of the wave (kbench8 counters), so the exact keys
            // are built straight away
            if constexpr (ACCF) {
                if (__ballot(i8_max32(a) >= thr_a(g)) == 0ull) continue;
            }
            // exact keys of the group (slot words from the norm ring)
            int v[32];
#pragma unroll
            for (int bb = 0; bb < 2; bb++)
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const knn_v4i c4 = *(const LDS_AS knn_v4i *)(cn + nofs(4 * h + 8 * (MB * rh + 2 * pr + bb) + j));
#pragma unroll
                    for (int i = 0; i < 4; i++) v[16 * bb + 4 * j + i] = (int)((unsigned)a[16 * bb + 4 * j + i] * 64u + (unsigned)c4[i]);
                }
            if (masked) {
#pragma unroll
                for (int x = 0; x < 32; x++) v[x] = a[x] == A_NONE ? vnone[g] : v[x];
            }
            int T = thr_v(g);
            int vm = i8_max32(v);
            if (__ballot(vm >= T) == 0ull) continue;
            // survivors in (d^2, row) order, one a round per lane: into the
            // lane's LDS buffer (NB entries); a full buffer anywhere merges
            // the wave's buffers into the lists (dense insertion rounds)
            do {
                if (vm >= T) {
                    const int slot = 31 - (vm & 31);
                    bk[64 * cnt[g]] = qn[g] - (vm >> 5);   // d^2 (0 = a duplicate: dropped at the merge)
                    bi[64 * cnt[g]] = idb + 32 * (2 * pr + (slot >> 4)) + 8 * ((slot >> 2) & 3) + (slot & 3);
                    cnt[g]++;
                }
                if (__ballot(cnt[g] == NB) != 0ull) {
                    merge(g);
                    T = thr_v(g);
                }
                vm = i8_next(v, vm, vnone[g]);
            } while (__ballot(vm >= T) != 0ull);
        }
        }
    };

    // ---- main loop -------------------------------------------------------------
    // PF2 (half-tile kernel, long rows): A fragments are read two K-steps
    // ahead instead of one, so a read has four MFMAs (two of this wave's
    // K-steps) to land under instead of two.  Barrier B(y) then sits two
    // K-steps before chunk y's first one, and the stage issued after it
    // overwrites chunk y - 2's slot (z = y + NST - 2).  The reads still in
    // flight there are those of the two K-steps before chunk y: both in
    // chunk y - 1 unless it has a single K-step (a tile's last chunk at 25
    // K-steps), when the older one is chunk y - 2's last -- only that
    // barrier waits for them (lgkmcnt(0)) before the stage.
    // (PF2 is defined with the bounds above: 28 K-steps spill)
    if (total > 0) {
#pragma unroll
        for (int y = 0; y < NST - 2; y++) stage();
        wait_next();
        __builtin_amdgcn_s_barrier();
        knn_v4i acur[MB], anxt[MB], anx2[MB];
        rdA(0, 0, acur);
        if constexpr (PF2) rdA(0, 1, anxt);
        stage();
        if constexpr (PF2 || ONE) s_rs = i8_rsrc(s_row);   // the prologue's stages moved the cursor
        if constexpr (ONE) {
            s_slot = s_x % NST;
            s_nslot = s_t % NNR;
        }
        int x = 0, xs = 0;   // xs = x % NST (ONE)
        e_b = i8_blk_of(tab, t_lo);
        e_t0 = i8_rfl(tab->t0[e_b]);
        e_t1 = i8_rfl(tab->t0[e_b + 1]);
        c_base = (long)i8_rfl64(tab->base[e_b]);
        nc = i8_rfl(tab->nc[e_b]);
        for (int t = t_lo; t < t_hi; t++) {
            if (t == e_t1) {   // the epilogue's block moves on
                e_b++;
                e_t0 = e_t1;
                e_t1 = i8_tab32(&tab->t0[e_b + 1]);
                c_base = (long)i8_tab64(&tab->base[e_b]);
                nc = i8_tab32(&tab->nc[e_b]);
            }
            // the tile's accumulators start at its init words (read at the
            // tile's start, straight into the accumulator registers: held
            // from earlier they cost 32 more VGPRs, or 16 v_mov_b64 a tile
            // where the next tile's set is loaded beside the live one)
            knn_v16i acc[QG][MB];
            if constexpr (SHORT) {
                rdI(t, acc[0]);
            } else {
#pragma unroll
                for (int bb = 0; bb < MB; bb++)
#pragma unroll
                    for (int i = 0; i < 16; i++) acc[0][bb][i] = 0;
            }
            if constexpr (PF2) {
                // flat K-steps f of the tile; the fragments of f + 2 are read
                // at f (the next tile's first two K-steps at f = NKS - 2,
                // NKS - 1), behind B(y) when f + 2 opens chunk y.  The last
                // tile does the same (every wave of the workgroup runs the
                // same tiles, so the extra barrier matches; the chunk it
                // opens is a tail re-stage, read and never used): a runtime
                // "next tile?" branch here made the compiler copy the
                // fragment registers through waits at every tile's end
                const int x0 = x;
                constexpr bool more = true;
#pragma unroll
                for (int f = 0; f < NKS; f++) {
                    const int fn = f + 2;
                    if (fn < NKS) {
                        if ((fn & 3) == 0) {
                            // (chunk y - 1 is a whole chunk of 4 K-steps here)
                            wait_next();
                            __builtin_amdgcn_s_barrier();   // B(x0 + fn / 4)
                            rdA(SSLOT ? (fn >> 2) : x0 + (fn >> 2), 0, anx2);
                            stage_at(((fn >> 2) + NST - 2) % NCH);
                        } else {
                            rdA(SSLOT ? (fn >> 2) : x0 + (fn >> 2), fn & 3, anx2);
                            __builtin_amdgcn_sched_barrier(0);
                        }
                    } else if (more) {
                        if (fn == NKS) {
                            // a one-K-step last chunk: K-step NKS - 2's read
                            // (chunk y - 2's last) may still be in flight
                            if constexpr ((NKS & 3) == 1) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                            wait_next();
                            __builtin_amdgcn_s_barrier();   // B(x0 + NCH)
                            rdA(SSLOT ? 0 : x0 + NCH, 0, anx2);
                            stage_at((NST - 2) % NCH);
                        } else {
                            rdA(SSLOT ? 0 : x0 + NCH, 1, anx2);
                            __builtin_amdgcn_sched_barrier(0);
                        }
                    }
                    // one lgkmcnt wait for the K-step's fragments (the
                    // compiler waits before the asm that "defines" them)
                    // instead of one before each MFMA
                    asm volatile("" : "+v"(acur[0]), "+v"(acur[1]));
#pragma unroll
                    for (int bb = 0; bb < MB; bb++)
                        acc[0][bb] = __builtin_amdgcn_mfma_i32_32x32x32_i8(acur[bb], qf[0][f], acc[0][bb], 0, 0, 0);
#pragma unroll
                    for (int bb = 0; bb < MB; bb++) {
                        acur[bb] = anxt[bb];
                        anxt[bb] = anx2[bb];
                    }
                }
                x = x0 + NCH;
                epilogue(t, acc, x);
                continue;
            }
#pragma unroll
            for (int c = 0; c < NCH; c++) {
                const int kt = NKS - 4 * c < 4 ? NKS - 4 * c : 4;   // static after unrolling
#pragma unroll
                for (int ks = 0; ks < 4; ks++) {
                    if (ks < kt) {
                        if (ks + 1 < kt) {
                            rdA(ONE ? xs : x, ks + 1, anxt);
                            // keep the reads ahead of this K-step's MFMAs:
                            // left alone, the scheduler sinks them behind the
                            // MFMAs into the same registers, and each MFMA
                            // pair then waited out a ds_read's latency
                            __builtin_amdgcn_sched_barrier(0);
                        } else if (x + 1 < total) {
                            wait_next();
                            __builtin_amdgcn_s_barrier();   // B(x + 1)
                            rdA(ONE ? (xs == NST - 1 ? 0 : xs + 1) : x + 1, 0, anxt);
                            // the next tile's norms arrived with its first
                            // chunk: its init words load under this K-step's
                            // MFMAs and the epilogue
                            if constexpr (ONE) stage1();
                            else stage();
                        }
                        // (QG = 2: the first K-step of group 1 takes
                        // group 0's init words as its C operand)
#pragma unroll
                        for (int bb = 0; bb < MB; bb++) {
                            const knn_v16i c0 = acc[0][bb];
#pragma unroll
                            for (int g = 0; g < QG; g++)
                                acc[g][bb] = __builtin_amdgcn_mfma_i32_32x32x32_i8(
                                    acur[bb], qf[g][4 * c + ks], (c == 0 && ks == 0) ? c0 : acc[g][bb], 0, 0, 0);
                        }
#pragma unroll
                        for (int bb = 0; bb < MB; bb++) acur[bb] = anxt[bb];
                    }
                }
                x++;
                if constexpr (ONE) xs = xs == NST - 1 ? 0 : xs + 1;
            }
            epilogue(t, acc, x);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no LDS-DMA left in flight
        if constexpr (REREAD) {
            if (q_ready >= 0) qthr_apply();
        }
    }
#pragma unroll
    for (int g = 0; g < QG; g++) merge(g);

    // strict publication (INT mode, exact keys): if neither lane's list ends
    // at thr, nothing equal to thr was turned away, so every rejected
    // candidate has d^2 >= next(thr) (k_finalize certifies tau < T); W = 8:
    // T of the query = min over its two waves (LDS, after a barrier)
#pragma unroll
    for (int g = 0; g < QG; g++) {
    int lastmin = L[g][KL - 1];
    {
        const int o = __shfl_xor(lastmin, 32);
        lastmin = o < lastmin ? o : lastmin;
    }
    double pub = thr[g] == I8_INF ? KNN_INF : (double)thr[g];
    if (lastmin > thr[g] && thr[g] < I8_INF) pub = nextafter((double)thr[g], KNN_INF);
    if constexpr (RHN == 2) {
        double *xd = (double *)((char *)smem + NORM0);   // the norm ring is free now
        __syncthreads();
        if (h == 0 && rh == 1) xd[qg * 32 + r32] = pub;
        __syncthreads();
        if (rh == 0) {
            const double po = xd[qg * 32 + r32];
            pub = po < pub ? po : pub;
        }
    }
    if (myq[g] < nq) {
        const size_t base = (((size_t)split * nq_pad + myq[g]) * LPQ + 2 * rh + h) * KL;
#pragma unroll
        for (int e = 0; e < KL; e++) {
            part_d[base + e] = L[g][e] == I8_INF ? KNN_INF : (double)L[g][e];
            part_i[base + e] = I[g][e];
        }
        if (h == 0 && rh == 0) part_T[(size_t)split * nq_pad + myq[g]] = pub;
        if (h == 0 && qthr != nullptr && thr[g] < I8_INF)
            atomicMin(qthr + myq[g], (unsigned long long)__double_as_longlong((double)thr[g]));
    }
    }
}

// ---------------------------------------------------------------------------
// Re-search of uncertified queries on the int8 contraction (knn_ctx_end,
// single-block searches): their byte rows gathered into a query block of
// their own, searched again with 65-entry lane lists, and the certified
// results scattered back.
// ---------------------------------------------------------------------------
// dst row i = src row list[i] (bytes and norm words; rows >= cnt zero), and
// the row's shared bound: dst_qthr[i] = src_qthr[list[i]] (the re-search's
// seed, k_merge_rank)
__global__ __launch_bounds__(256) void k_gather8(signed char *__restrict__ dst, const signed char *__restrict__ src,
                                                 const int *__restrict__ list, int cnt, int rs, size_t src_rows_pad,
                                                 size_t dst_rows_pad, const unsigned long long *__restrict__ src_qthr,
                                                 unsigned long long *__restrict__ dst_qthr)
{
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    {
        const int i = blockIdx.x * 256 + threadIdx.x;
        if (i < cnt) dst_qthr[i] = src_qthr[list[i]];
    }
    const int *sn = (const int *)(src + src_rows_pad * (size_t)rs);
    int *dn = (int *)(dst + dst_rows_pad * (size_t)rs);
    for (size_t r = (size_t)blockIdx.x * 4 + wave; r < dst_rows_pad; r += (size_t)gridDim.x * 4) {
        const int q = r < (size_t)cnt ? list[r] : -1;
        for (int b = 4 * lane; b < rs; b += 256)
            *(int *)(dst + r * rs + b) = q >= 0 ? *(const int *)(src + (size_t)q * rs + b) : 0;
        if (lane == 0) {
            const int nrm = q >= 0 ? i8_norm_of(sn[i8_norm_pos(q)], sn[src_rows_pad + i8_norm_pos(q)]) : 0;
            dn[i8_norm_pos((int)r)] = i8_norm_word((int)r, nrm, rs);
            dn[dst_rows_pad + i8_norm_pos((int)r)] = i8_init_word(nrm, rs);
        }
    }
}

// flag[i] = 1 for the re-searched queries still uncertified (flag zeroed first)
__global__ void k_flag8_set(unsigned char *__restrict__ flag, const int *__restrict__ sub_fail,
                            const int *__restrict__ sub_cnt)
{
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j < *sub_cnt) flag[sub_fail[j]] = 1;
}
// certified re-searched queries: records into out; the rest onto a new list
__global__ void k_resolve8(const unsigned char *__restrict__ flag, const int *__restrict__ list, int cnt,
                           const knn_neighbour_t *__restrict__ sub_out, int k, knn_neighbour_t *__restrict__ out,
                           int *__restrict__ new_list, int *__restrict__ new_cnt)
{
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    const int i = t / k, r = t - i * k;
    if (i >= cnt) return;
    if (flag[i]) {
        if (r == 0) new_list[atomicAdd(new_cnt, 1)] = list[i];
        return;
    }
    out[(size_t)list[i] * k + r] = sub_out[(size_t)i * k + r];
}

extern "C" int knn_launch_gather8(void *dst, const void *src, const int *list, int cnt, size_t n,
                                  size_t src_rows_pad, size_t dst_rows_pad, const double *src_qthr,
                                  double *dst_qthr, void *stream)
{
    const int rs = (int)knn_s8_rs(n);
    unsigned grid = (unsigned)((dst_rows_pad + 3) / 4 < 1024 ? (dst_rows_pad + 3) / 4 : 1024);
    if (grid * 256u < (unsigned)cnt) grid = (unsigned)((cnt + 255) / 256);
    hipLaunchKernelGGL(k_gather8, dim3(grid), dim3(256), 0, (hipStream_t)stream, (signed char *)dst,
                       (const signed char *)src, list, cnt, rs, src_rows_pad, dst_rows_pad,
                       (const unsigned long long *)src_qthr, (unsigned long long *)dst_qthr);
    return hipGetLastError() == hipSuccess ? KNN_OK : KNN_ERR_HIP;
}

extern "C" int knn_launch_resolve8(unsigned char *flag, const int *list, int cnt, const int *sub_fail,
                                   const int *sub_cnt, const knn_neighbour_t *sub_out, int k,
                                   knn_neighbour_t *out, int *new_list, int *new_cnt, void *stream)
{
    hipStream_t s = (hipStream_t)stream;
    if (cnt <= 0) return KNN_OK;
    if (hipMemsetAsync(flag, 0, (size_t)cnt, s) != hipSuccess || hipMemsetAsync(new_cnt, 0, sizeof(int), s) != hipSuccess)
        return KNN_ERR_HIP;
    hipLaunchKernelGGL(k_flag8_set, dim3((unsigned)((cnt + 255) / 256)), dim3(256), 0, s, flag, sub_fail, sub_cnt);
    hipLaunchKernelGGL(k_resolve8, dim3((unsigned)(((size_t)cnt * k + 255) / 256)), dim3(256), 0, s, flag, list,
                       cnt, sub_out, k, out, new_list, new_cnt);
    return hipGetLastError() == hipSuccess ? KNN_OK : KNN_ERR_HIP;
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
extern "C" int knn_launch_shadow8(void *dst, const void *blk, int dtype, size_t rows_pad, size_t n,
                                  const double *meta, void *stream)
{
    const int rs = (int)knn_s8_rs(n), nps = (int)knn_n_pad_dt(n, dtype);
    const unsigned grid = (unsigned)((rows_pad + 3) / 4 < 4096 ? (rows_pad + 3) / 4 : 4096);
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

template <int KL, int NKS, int W, int WPS, int NST, int NB, int TM, int QG = 1>
static void launch_i8(dim3 grid, hipStream_t s, const void *qsh, size_t q_rows_pad, size_t q_base,
                      int nq, const knn_i8_blocks_t &cb, size_t c_rows_pad, int rs,
                      int nks, int ntiles, int nsplit, int nqb, double *part_d, int *part_i,
                      double *part_T, int nq_pad, double *qthr, int uj, unsigned long long *qsum)
{
    hipLaunchKernelGGL(HIP_KERNEL_NAME(k_dist_topk_i8<KL, NKS, W, WPS, NST, NB, TM, QG>), grid, dim3(64 * W), 0, s,
                       (const signed char *)qsh, q_rows_pad, q_base, nq, cb, c_rows_pad, rs, nks, ntiles,
                       nsplit, nqb, part_d, part_i, part_T, nq_pad, (unsigned long long *)qthr, uj,
                       KL != KNN_I8_KL_L ? qsum : nullptr);
}

extern "C" int knn_launch_dist_i8(int kp, int kl, int lpq, int k, const void *qsh, size_t q_rows_pad, size_t q_base,
                                  int nq, const knn_i8_blocks_t *cbp, size_t c_rows_pad, int n,
                                  int nsplit, double *part_d, int *part_i, double *part_T,
                                  int nq_pad, double *qthr, unsigned long long *qsum, void *stream)
{
    const int rs = (int)knn_s8_rs((size_t)n), nks = rs / 32;
    const int qg = knn_i8_qg(kl, lpq, (size_t)n);
    const int nqb = (nq + 128 * qg - 1) / (128 * qg);
    if (!cbp || cbp->nblk < 1 || cbp->nblk > KNN_I8_MAXBLK) return KNN_ERR_INVALID;
    // the table the kernel walks: block b = tiles [t0[b], t0[b+1]) of its
    // ceil(nc/128) tiles, ascending bases, rows inside the capacity
    knn_i8_blocks_t cb = *cbp;
    cb.t0[0] = 0;
    for (int b = 0; b < cb.nblk; b++) {
        if (!cb.nptr[b]) cb.nptr[b] = (const char *)cb.ptr[b] + c_rows_pad * (size_t)rs;
        if (!cb.ptr[b] || cb.nc[b] <= 0 || (size_t)cb.nc[b] > c_rows_pad || cb.base[b] < 0 ||
            (b > 0 && cb.base[b] < cb.base[b - 1] + cb.nc[b - 1]))
            return KNN_ERR_INVALID;
        cb.t0[b + 1] = cb.t0[b] + (cb.nc[b] + 127) / 128;
    }
    for (int b = cb.nblk; b < KNN_I8_MAXBLK; b++) {
        cb.ptr[b] = cb.ptr[cb.nblk - 1];
        cb.nptr[b] = cb.nptr[cb.nblk - 1];
        cb.base[b] = cb.base[cb.nblk - 1];
        cb.nc[b] = cb.nc[cb.nblk - 1];
        cb.t0[b + 1] = cb.t0[cb.nblk];
    }
    const int ntiles = cb.t0[cb.nblk];
    if (nqb <= 0 || nsplit <= 0 || k <= 0 || k > kp || kl <= 0 || nks > 28) return KNN_ERR_INVALID;
    // (QG = 2: the last block's padding queries load row nq - 1 and write nothing)
    if (qg == 1 && ((size_t)nqb * 128 > q_rows_pad || nq_pad < nqb * 128)) return KNN_ERR_INVALID;
    if ((size_t)nq > q_rows_pad || nq > nq_pad) return KNN_ERR_INVALID;
    // lane-list slot of the shared bound: the 2 lanes of a query cover k + 1
    int uj = (k + 1 + 1) / 2 - 1, uj4 = (k + 1 + 3) / 4 - 1;
    const int no2 = uj > kl - 1;   // 2 lists of kl cannot hold k + 1
    if (uj > kl - 1) uj = kl - 1;
    // the list shapes: 4 lists of kl a query (8 waves, 128-row tiles), or 2
    // (4-wave kernels: 65-entry lists, or 12-entry lists on 64-row tiles)
    const int half = kl == KNN_I8_KL_S && lpq == 2;
    if (!(lpq == 4 && (kl == KNN_I8_KL_S || kl == KNN_I8_KL)) && !(lpq == 2 && (half || kl == KNN_I8_KL_L)))
        return KNN_ERR_INVALID;
    if (lpq == 4 && 4 * kl < k + 1) return KNN_ERR_INVALID;   // the 4-lane bound needs 4 KL >= k + 1
    uj |= uj4 << 8;
    if (no2) uj |= 1 << 16;
    const dim3 grid((unsigned)(nqb * nsplit));
    hipStream_t s = (hipStream_t)stream;
    // cross-split summaries combine 4 x 8 or 2 x 16 rows: for k + 1 <= 32
    if (k + 1 > 32) qsum = nullptr;
#define I8_ARGS grid, s, qsh, q_rows_pad, q_base, nq, cb, c_rows_pad, rs, nks, ntiles, nsplit, \
                nqb, part_d, part_i, part_T, nq_pad, qthr, uj, qsum
    // One workgroup a CU (queries in up to 112 VGPRs), an 8-stage ring.
    // k <= 32: 8 waves (two a SIMD, 2 m-blocks each, 4 lists a query) and
    // 6-entry survivor buffers (merging sooner tightens the bounds sooner:
    // mnist 4.32 -> 3.93 ms against 8 entries, sift 320 -> 308 ms;
    // tools/probe/kbench8 variants);
    // k <= 128: 4 waves (one a SIMD, 4 m-blocks, 2 lists a query, 512 VGPRs).
    // K-step buckets: the smallest instantiated NKS >= nks
    if (half) {
        // 12-entry lists, 64-row half tiles: 4 waves (32 queries x 2
        // m-blocks each) and 80 KB of LDS a workgroup, so two workgroups
        // share a CU -- each SIMD runs one wave of each, whose barriers and
        // epilogues are independent: one's epilogue runs under the other's
        // MFMAs (the 8-wave form's two waves a SIMD sat at the same barriers)
        // Rows of <= 4 K-steps (SIFT): two query groups a wave, a 7-stage
        // ring (the second group's survivor buffers take the 8th stage's LDS)
        if (nks <= 4 && qg == 2) launch_i8<KNN_I8_KL_S, 4, 4, 2, 7, 5, 2, 2>(I8_ARGS);
        else if (nks <= 4) launch_i8<KNN_I8_KL_S, 4, 4, 2, 8, 5, 2>(I8_ARGS);
        else if (nks <= 8) launch_i8<KNN_I8_KL_S, 8, 4, 2, 8, 5, 2>(I8_ARGS);
        else if (nks <= 16) launch_i8<KNN_I8_KL_S, 16, 4, 2, 8, 5, 2>(I8_ARGS);
        else if (nks <= 25) launch_i8<KNN_I8_KL_S, 25, 4, 2, 7, 6, 2>(I8_ARGS);   // one-tile ring (SSLOT); 6-entry buffers (r06_s32)
        else launch_i8<KNN_I8_KL_S, 28, 4, 2, 8, 5, 2>(I8_ARGS);
    } else if (kl == KNN_I8_KL_S) {
        // 12-entry lists merge cheaply: 5-entry buffers (merging sooner)
        // against 6 -- kbench8, cold bounds: mnist 4.15 -> 3.91 ms, the P = 8
        // fused launch 0.69 -> 0.65 ms, sift 276 -> 277 ms; in bench.py and
        // the ring emulation within run-to-run noise
        if (nks <= 4) launch_i8<KNN_I8_KL_S, 4, 8, 2, 8, 5, 4>(I8_ARGS);
        else if (nks <= 8) launch_i8<KNN_I8_KL_S, 8, 8, 2, 8, 5, 4>(I8_ARGS);
        else if (nks <= 16) launch_i8<KNN_I8_KL_S, 16, 8, 2, 8, 5, 4>(I8_ARGS);
        else if (nks <= 25) launch_i8<KNN_I8_KL_S, 25, 8, 2, 8, 5, 4>(I8_ARGS);
        else launch_i8<KNN_I8_KL_S, 28, 8, 2, 8, 5, 4>(I8_ARGS);
    } else if (kl == KNN_I8_KL) {
        if (nks <= 4) launch_i8<KNN_I8_KL, 4, 8, 2, 8, 5, 4>(I8_ARGS);
        else if (nks <= 8) launch_i8<KNN_I8_KL, 8, 8, 2, 8, 5, 4>(I8_ARGS);
        else if (nks <= 16) launch_i8<KNN_I8_KL, 16, 8, 2, 8, 5, 4>(I8_ARGS);
        else if (nks <= 25) launch_i8<KNN_I8_KL, 25, 8, 2, 8, 5, 4>(I8_ARGS);
        else launch_i8<KNN_I8_KL, 28, 8, 2, 8, 5, 4>(I8_ARGS);
    } else if (kl == KNN_I8_KL_L) {
        if (nks <= 4) launch_i8<KNN_I8_KL_L, 4, 4, 1, 8, 8, 4>(I8_ARGS);
        else launch_i8<KNN_I8_KL_L, 28, 4, 1, 8, 8, 4>(I8_ARGS);
    } else {
        return KNN_ERR_INVALID;
    }
#undef I8_ARGS
    return hipGetLastError() == hipSuccess ? KNN_OK : KNN_ERR_HIP;
}
