/*
 * knn_internal.h -- launchers exported by knn_kernels.hip to the host C
 * engine (knn_engine.c).  Plain C ABI, device pointers, hipStream_t as void*.
 */
#ifndef KNN_INTERNAL_H
#define KNN_INTERNAL_H
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include "knn.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Tile geometry shared by host and device. */
#define KNN_TQ 128        /* queries per workgroup (8 waves x 16)      */
#define KNN_TC 128        /* corpus rows per tile                      */
#define KNN_BK 16         /* fp64 features per LDS chunk (128 B a row) */
#define KNN_KL 16         /* per-lane candidate list capacity, k <= 32 */
#define KNN_KP 32         /* per-query state / selection capacity      */
#define KNN_KL_M 24       /* fp32, 16 < k <= 32: a lane list overflows */
#define KNN_KP_M 64       /*   when > KL of the k fall in its quarter   */
#define KNN_KL_L 40       /* fp32, 32 < k <= 128:                        */
#define KNN_KP_L 128      /*   P(Bin(100, 1/4) > 40) ~ 3e-4 per lane   */
#define KNN_ROW_ALIGN 128 /* packed-block row padding                  */

/* meta doubles of a packed block */
#define KNN_META_MAXABS    0
#define KNN_META_MAXNORM   1
#define KNN_META_NONINT    2
#define KNN_META_NONFINITE 3
#define KNN_META_MAXPOS    4   /* max(x, 0)  */
#define KNN_META_MAXNEG    5   /* max(-x, 0) */
#define KNN_META_S8        7   /* 1: a speculative byte block (knn_block_pack_s8); MAX-reduced, so a
                                * ring knows whether any rank packed one */

/* engine modes (decided on device from the reduced meta) */
#define KNN_MODE_INT  0   /* integer data: GEMM-form d^2 is exact         */
#define KNN_MODE_GEMM 1   /* fp64 GEMM-form filter + exact re-rank        */
#define KNN_MODE_SCAN 2   /* non-finite / huge data: exact scan only      */

static inline size_t knn_round_up(size_t x, size_t a) { return (x + a - 1) / a * a; }
static inline size_t knn_rows_pad(size_t rows) { return knn_round_up(rows ? rows : 1, KNN_ROW_ALIGN); }
static inline size_t knn_n_pad(size_t n) { return knn_round_up(n ? n : 1, KNN_BK); }
/* element size and padded row length of a packed block of `dtype`
 * (KNN_F64 / KNN_F32): rows are padded to whole 128-byte chunks */
/* state capacity and per-lane list length serving k */
/* State capacity serving k.  With one corpus split, 16-deep lane lists
 * overflow for P(Bin(32, 1/4) >= 16) * 4 = 0.8% of queries at k = 32 (each
 * a rescan); fp32 has the registers for deeper lists, fp64 (k <= 32) not.
 * fp64 16 < k <= 32 keeps 16-deep lane lists but a 64-entry state: the
 * GEMM certificate's Td (the smallest value a merge drops) then sits past
 * the (k + 1)-th candidate's near ties -- with a 32-entry state at k = 30,
 * 228 of the 60000 real-valued MNIST-shape queries had their 33rd filter
 * value within 2E of the 30th and took the exact rescan. */
static inline int knn_kp_for(int k, int dtype)
{
    if (k <= 16) return KNN_KP;
    if (dtype != KNN_F32) return KNN_KP_M;
    return k <= 32 ? KNN_KP_M : KNN_KP_L;
}
static inline int knn_kl_for(int kp, int dtype)
{
    if (dtype != KNN_F32) return KNN_KL;
    return kp == KNN_KP ? KNN_KL : kp == KNN_KP_M ? KNN_KL_M : KNN_KL_L;
}
/* Corpus chunks of one exact rescan launch (k_rescan_step's grid.y): enough
 * that (nfail / 16) x C workgroups fill the chip, at most 32.  The rescan
 * list buffers hold 1 + C list sets (the running one, then one per chunk). */
static inline int knn_rescan_chunks(int nfail)
{
    const int wg = (nfail + 15) / 16;
    int c = wg > 0 ? (1024 + wg - 1) / wg : 1;
    return c > 32 ? 32 : (c < 1 ? 1 : c);
}
static inline size_t knn_esize(int dtype) { return dtype == KNN_F32 ? 4 : 8; }

/* Byte block (knn_i8.hip): the int8 form of a packed block for the int8
 * MFMA contraction of 8-bit-window integer data.  Rows of knn_s8_rs(n)
 * bytes (x - o, o = 128 - meta[MAXNEG]; 0 past n), then two int32 words per
 * row, each array in the per-tile order of i8_norm_pos: the slot/parity
 * words (i8_norm_word), then the accumulator init words (i8_init_word,
 * -floor(|x - o|^2 / 2)); then the block's 8 meta doubles. */
#define KNN_I8_MAX_N 896  /* 7 chunks of 128 features: queries stay in VGPRs */
#define KNN_I8_KL_S 12    /* per-lane list, k <= 32: 8-wave kernel, 4 lists a query  */
                          /* (4 KL >= k + 1: the 4-lane bound; no 2-lane bound)     */
#define KNN_I8_KL   17    /* the same with 17-entry lists (KNN_I8_KL=17)             */
#define KNN_I8_KL_L 65    /* k <= 128: 4-wave kernel, 2 lists a query (2 KL > k)    */
/* row bytes: whole K-steps of 32 */
static inline size_t knn_s8_rs(size_t n) { return knn_round_up(n ? n : 1, 32); }
static inline size_t knn_s8_norm_offset(size_t cap, size_t n) { return knn_rows_pad(cap) * knn_s8_rs(n); }
static inline size_t knn_s8_meta_offset(size_t cap, size_t n) { return knn_s8_norm_offset(cap, n) + knn_rows_pad(cap) * 8; }
static inline size_t knn_s8_bytes(size_t cap, size_t n)
{
    return knn_round_up(knn_s8_meta_offset(cap, n) + 8 * sizeof(double), 16);
}
/* Corpus blocks of one k_dist_topk_i8 launch (a fused ring step): byte
 * blocks of one capacity, ascending global base (so every lane meets its
 * candidates in increasing row order: the stable tie rule), block b holding
 * global tiles [t0[b], t0[b+1]) of the launch.  An entry may also be a
 * whole-tile range of a block: ptr / nptr / base advanced by its first tile. */
#define KNN_I8_MAXBLK 8
typedef struct {
    const void *ptr[KNN_I8_MAXBLK];   /* row 0 of the block (or of a tile range of it) */
    const void *nptr[KNN_I8_MAXBLK];  /* its norms; NULL: the block's, ptr + cap_pad * row bytes */
    int64_t base[KNN_I8_MAXBLK];
    int nc[KNN_I8_MAXBLK];
    int t0[KNN_I8_MAXBLK + 1];
    int nblk;
} knn_i8_blocks_t;
static inline int knn_i8_kl(int kp) { return kp <= KNN_KP_M ? KNN_I8_KL_S : KNN_I8_KL_L; }
/* lists per query: 2 for the 65-entry lists (k > 32) and for the 12-entry
 * lists on 64-row half tiles (the k <= 32 default); 4 for the 8-wave
 * kernel on 128-row tiles (17-entry lists) */
static inline int knn_i8_lpq(int kp, int kl) { return kp <= KNN_KP_M && kl != KNN_I8_KL_S ? 4 : 2; }
/* query groups a wave of the int8 kernel: 2 for the half-tile kernel on
 * rows of <= 4 K-steps (SIFT's n = 128: a workgroup of 256 queries, A
 * fragments and init words shared by both groups), else 1
 * (KNN_I8_QG1=1 forces 1).  A workgroup covers 128 qg queries. */
static inline int knn_i8_qg(int kl, int lpq, size_t n)
{
    const char *e = getenv("KNN_I8_QG1");
    return kl == KNN_I8_KL_S && lpq == 2 && knn_s8_rs(n) / 32 <= 4 && !(e && *e && *e != '0') ? 2 : 1;
}
static inline size_t knn_n_pad_dt(size_t n, int dtype)
{
    return knn_round_up(n ? n : 1, 128 / knn_esize(dtype));
}

/* Launchers.  dtype = element type of the packed blocks (KNN_F64 /
 * KNN_F32); block pointers are untyped device pointers. */
int knn_launch_pack(void *blk, int dtype, size_t cap, size_t rows, size_t n, const void *src,
                    int src_dtype, size_t ld, int layout, void *stream);
int knn_launch_dist_topk(int dtype, int kp, int k, const void *qblk, size_t q_rows_pad, size_t q_base, int nq,
                         const void *cblk, size_t c_rows_pad, size_t c_base, int nc,
                         int n, const double *meta, int nsplit,
                         double *part_d, int *part_i, double *part_T, int nq_pad,
                         double *qthr, const void *qsh, const void *csh, const void *cn_ptr,
                         int flags, float m2s, void *stream);
/* knn_launch_dist_topk flags */
#define KNN_DIST_XORD   1  /* XCD-grouped workgroup order                        */
#define KNN_DIST_H16    2  /* fp16 MFMA contraction (exact data only)             */
#define KNN_DIST_SHADOW 4  /* with H16: stage the fp16 shadow rows qsh / csh      */
#define KNN_DIST_SPLIT  8  /* fp32 blocks: split fp16 filter on the split shadow rows
                              qsh / csh (knn_launch_shadow_split); m2s = -2 / S^2   */
/* k_dist_split (knn_split.hip): the split fp16 filter on 256-row tiles,
 * over up to KNN_SPLIT_MAXBLK corpus blocks in one launch (block b: split
 * rows sp[b], norms nrm[b] of its element block, global ids base[b].., nc[b]
 * rows, lim[b] rows allocated; tiles [t0[b], t0[b+1]) of the launch -- the
 * launcher fills t0) */
#define KNN_SPLIT_TC 256
#define KNN_SPLIT_MAXBLK 8
typedef struct {
    const void *sp[KNN_SPLIT_MAXBLK];
    const void *nrm[KNN_SPLIT_MAXBLK];
    int64_t base[KNN_SPLIT_MAXBLK];
    int nc[KNN_SPLIT_MAXBLK];
    int lim[KNN_SPLIT_MAXBLK];
    int t0[KNN_SPLIT_MAXBLK + 1];
    int nblk;
} knn_split_blocks_t;
/* the element blocks a GEMM-mode merge re-ranks from (k_merge's exact S):
 * block j holds global ids base[j] .. base[j] + nc[j] - 1 */
typedef struct {
    const void *ptr[KNN_SPLIT_MAXBLK];
    int64_t base[KNN_SPLIT_MAXBLK];
    int nc[KNN_SPLIT_MAXBLK];
    int nblk;
} knn_merge_blocks_t;
int knn_launch_merge_n(int dtype, int kp, int k, const double *part_d, const int *part_i, const double *part_T,
                       int nsplit, int lpq, int kl, int nq, int nq_pad, int first_step, double *st_d, double *st_x,
                       int *st_i, double *st_T, const void *qblk, size_t q_rows_pad, const knn_merge_blocks_t *mb,
                       int n, const double *meta, double *qthr, int filt, const int *qperm, void *stream);
/* the split filter over several element blocks (their split rows in sp[],
 * their norms in nrm[]): knn_launch_dist_topk's KNN_DIST_SPLIT for a table */
int knn_launch_dist_split_n(int dtype, int kp, int k, const void *qblk, size_t q_rows_pad, size_t q_base, int nq,
                            const void *qsp, const knn_split_blocks_t *cb, int n, const double *meta, int nsplit,
                            double *part_d, int *part_i, double *part_T, int nq_pad, double *qthr, int xord,
                            float m2s, void *stream);
int knn_launch_dist_split(int dtype, int kl, const void *qsp, const void *qnorm, size_t q_base, int nq,
                          const knn_split_blocks_t *cb, int n, const double *meta, int nsplit, double *part_d,
                          int *part_i, double *part_T, int nq_pad, double *qthr, int uj, int xord, float m2s,
                          void *stream);
/* fp16 shadow rows (round_up(n, 64) halves a row) of a packed block */
int knn_launch_shadow(void *dst, const void *blk, int dtype, size_t rows_pad, size_t n, void *stream);
int knn_launch_fill_inf(double *p, int count, void *stream);
/* int8 re-search of uncertified queries (knn_i8.hip) */
int knn_launch_gather8(void *dst, const void *src, const int *list, int cnt, size_t n, size_t src_rows_pad,
                       size_t dst_rows_pad, const double *src_qthr, double *dst_qthr, void *stream);
int knn_launch_resolve8(unsigned char *flag, const int *list, int cnt, const int *sub_fail, const int *sub_cnt,
                        const knn_neighbour_t *sub_out, int k, knn_neighbour_t *out, int *new_list, int *new_cnt,
                        void *stream);
/* speculative byte block straight from the source (knn_block_pack_s8) */
int knn_launch_pack_s8(void *dst, int dtype, size_t cap, size_t rows, size_t n, const void *src, int src_dtype,
                       size_t ld, int layout, void *stream);
/* INT-mode merge of int8 lane lists (kl = KNN_I8_KL_S / KNN_I8_KL, kp <= 64)
 * by ranking the candidates at or below the shared bound (k_merge_rank) */
int knn_launch_merge_rank(int dtype, int kp, int kl, int k, const double *part_d, const int *part_i,
                          const double *part_T, int nsplit, int lpq, int nq, int nq_pad, int first_step,
                          double *st_d, double *st_x, int *st_i, double *st_T, double *qthr,
                          knn_neighbour_t *fin_out, int *fail_count, int *fail_list, int *mode_out, double *fbound,
                          const double *meta, int n, int force_fail, void *stream);
/* qthr = +inf, qsum (may be NULL) = empty summaries, counts[0..1] = 0 */
int knn_launch_begin_init(double *qthr, unsigned long long *qsum, int nq_pad, int *counts, void *stream);
/* counts[0..1] -> mapped host memory, and the meta (8 doubles; NULL: none)
 * -> mapped_meta (k_count_out) */
int knn_launch_count_out(const int *d_count, int *mapped, const double *meta, double *mapped_meta, void *stream);
/* split fp16 shadow rows of an fp32 / fp64 block: per 32 features 32 halves hi =
 * RN16(S x), then 32 halves lo = RN16(S x - hi); rows of round_up(n, 32) * 4
 * bytes; S a power of two (knn_engine.c: maxabs S in [2^13, 2^14)) */
static inline size_t knn_split_rs(size_t n) { return knn_round_up(n ? n : 1, 32) * 4; }
int knn_launch_shadow_split(void *dst, const void *blk, int dtype, size_t rows_pad, size_t n, float S,
                            void *stream);
/* the same for nblk <= KNN_SPLIT_MAXBLK blocks in one launch */
int knn_launch_shadow_split_n(int nblk, void *const *dst, const void *const *src, const size_t *rows_pad,
                              int dtype, size_t n, float S, void *stream);
/* knn_i8.hip: element block -> byte block (meta = the reduced meta) and the
 * int8 distance + top-k kernel (partial lists [split][query][2][kl]) */
int knn_launch_shadow8(void *dst, const void *blk, int dtype, size_t rows_pad, size_t n,
                       const double *meta, void *stream);
int knn_launch_dist_i8(int kp, int kl, int lpq, int k, const void *qsh, size_t q_rows_pad, size_t q_base, int nq,
                       const knn_i8_blocks_t *cb, size_t c_rows_pad, int n, int nsplit,
                       double *part_d, int *part_i, double *part_T, int nq_pad, double *qthr,
                       unsigned long long *qsum, void *stream);
int knn_launch_merge(int dtype, int kp, int k, const double *part_d, const int *part_i,
                     const double *part_T, int nsplit, int lpq, int kl, int nq, int nq_pad,
                     int first_step,
                     double *st_d, double *st_x, int *st_i, double *st_T, const void *qblk,
                     size_t q_rows_pad, const void *cblk, size_t c_base, int nc, int n,
                     const double *meta, double *qthr, int filt, const int *qperm, void *stream);
/* knn_order.hip: a query order for the GEMM-mode merge (queries grouped by
 * the clusters their list heads connect) */
size_t knn_order_tmp_bytes(int nq);
int knn_launch_order(const int *part_i, int nsplit, int lpq, int kl, int nq, int nq_pad, long long q_base,
                     int rounds, int *lab, int *keys, int *iota, int *perm, void *tmp, size_t tmp_bytes,
                     void *stream);
int knn_launch_finalize(int dtype, int kp, const double *st_d, const double *st_x, const int *st_i,
                        const double *st_T, const void *qblk, size_t q_rows_pad,
                        int nq, int n, int k, const double *meta,
                        knn_neighbour_t *out, int *fail_count, int *fail_list,
                        int *mode_out, double *fbound, int force_fail, int filt, void *stream);
int knn_launch_rescan_init(int kp, double *rs_d, int *rs_i, int nfail, void *stream);
int knn_launch_rescan_step(int dtype, int kp, const int *fail_list, int nfail,
                           const double *fbound, const void *qblk, const void *cblk,
                           size_t c_base, int nc, int n, int k, double *rs_d, int *rs_i,
                           void *stream);
int knn_launch_rescan_end(int kp, const int *fail_list, int nfail, const double *rs_d,
                          const int *rs_i, int k, knn_neighbour_t *out, void *stream);
int knn_launch_vote(knn_neighbour_t *nb, size_t m, int k, int nclasses, int rule,
                    const double *labels, size_t nlabels, size_t q_base, int *pred,
                    unsigned long long *matches, void *stream);
/* knn_kernels.hip: block elements <-> int16 wire elements (cnt % 8 == 0) */
int knn_launch_wire(int unpack, void *dst, const void *src, int dtype, size_t cnt, void *stream);
/* knn_engine.c: the value knn_last_search_seconds() returns (this thread) */
void knn_set_last_search_seconds(double s);

#ifdef __cplusplus
}
#endif

#endif
