/*
 * knn.h -- C ABI of libknn, the MI355X-native all-kNN engine.
 *
 * Drop-in boundary for the hot path of yiapou13/mpi-knn (snapshot
 * 2025-02-12).  The reference has no library API: its boundary is the
 * MATLAB MAT-API it consumes, the stage structure inside main() and the
 * CLI/stdout contract.  Each entry point below names the
 * reference lines it replaces.  Citations: serial:L = knn-serial.c,
 * blk:L = mpi-knn-parallel_blocking.c, nb:L = mpi-knn-parallel_non_blocking.c.
 *
 * Conventions
 *  - Every function returns an int status (KNN_OK == 0); nothing aborts and
 *    no C++ exception crosses the ABI.  knn_strerror() names a status.
 *  - Outputs are caller-owned.  The library owns device buffers it allocates.
 *  - "stream" arguments are hipStream_t passed as void* (NULL = default).
 *  - A context is used from one host thread at a time (not re-entrant).
 *  - Results follow the reference's SERIAL semantics (serial:72-93) for every
 *    device count: per query the k smallest distances sqrt(S), S = sum_j
 *    (x_qj - x_ij)^2 accumulated in j order in fp64 without FMA; exact
 *    zero distances (the point itself and exact duplicates) excluded; ties
 *    ordered by lower 1-based index; missing slots {INFINITY, 0, 0}.
 *
 * Environment switches read by the library (none changes a result; each
 * selects among exact code paths, for tests and diagnosis):
 *   KNN_NO_I8=1 / KNN_NO_H16=1 / KNN_NO_SHADOW=1 / KNN_NO_SPLIT=1
 *                         disable the int8 / fp16 contraction / fp16 shadow
 *                         rows / split fp16 filter (the next exact
 *                         contraction in line runs)
 *   KNN_I8_KL=17          17-entry int8 lane lists instead of 12
 *   KNN_SPLITS=s          corpus splits per launch instead of the model's
 *   KNN_ORDER=1 / KNN_NO_ORDER=1
 *                         GEMM-mode merge in the clustered query order
 *                         (default past 64 MB blocks) / always index order
 *   KNN_I8_QG1=1          one query group a wave on rows of <= 128 bytes
 *                         (the half-tile kernel otherwise carries two: 256
 *                         queries a workgroup sharing each staged row)
 *   KNN_FORCE_RESCAN=1    send every query through the exact rescan pass
 *   KNN_NO_RESEARCH8=1    no int8 re-search (65-entry lists) of uncertified
 *                         queries of a single-block search before the rescan
 *   KNN_FORCE_RING=1      knn_search runs the ring driver on one GPU
 *   KNN_RING_SCHEDULE=ring|direct
 *                         ring driver schedule: "ring" = the reference's
 *                         neighbour rotation (blk:187-244), "direct" = every
 *                         block to every rank at once (default; bit-identical
 *                         results, tested through the loopback transport and
 *                         gloo -- no multi-GPU node has run it yet)
 *   KNN_RING_FUSE=rest|all direct schedule: own block folded beside the
 *                         exchange (rest) or with the received blocks (all)
 *   KNN_RING_TIMEOUT_S=t  bound (seconds, default 300) on every wait for the
 *                         ring's transfers: RCCL asynchronous errors are
 *                         polled beside it, and a failed or stalled transfer
 *                         aborts the communicators and returns KNN_ERR_RCCL
 *                         (mpiknn/ring.py: RingError; bench.py: the process
 *                         group's timeout)
 *   KNN_RING_LOOPBACK=1   P virtual ranks on device 0 (tests)
 *   KNN_NO_SHADOW_RING=1  ring moves element blocks, not shadow/byte blocks
 *   KNN_XCD_ORDER=1 / 0   distance launches in the XCD-grouped / the
 *                         split-major workgroup order (unset: XCD-grouped
 *                         for split-filter launches of <= 2 splits)
 *   KNN_MAT / KNN_MPI_COMPAT  the CLIs: .mat path, bug-compatible mode
 *   (mpiknn/ring.py: KNN_NO_S8=1 packs element blocks, not the byte block
 *   of knn_block_pack_s8)
 */
#ifndef KNN_H
#define KNN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Only the entry points below are exported (libknn builds with
 * -fvisibility=hidden). */
#ifndef KNN_API
#define KNN_API __attribute__((visibility("default")))
#endif

/* blk:15-20 {double distance; int idx; int label;}.  serial:14-18 has the
 * same size and offsets for {distance, idx}. */
typedef struct {
    double  distance;
    int32_t idx;     /* 1-based global row (serial:89, blk:175), 0 = empty */
    int32_t label;   /* class label of that row (blk:176), 0 if unknown    */
} knn_neighbour_t;

enum knn_status {
    KNN_OK = 0,
    KNN_ERR_INVALID = 1,     /* bad argument / shape                      */
    KNN_ERR_NOMEM = 2,       /* host or device allocation failed          */
    KNN_ERR_HIP = 3,         /* HIP runtime error                         */
    KNN_ERR_IO = 4,          /* file could not be opened / read           */
    KNN_ERR_FORMAT = 5,      /* not a MAT-v5/v7 file, or variable missing */
    KNN_ERR_UNSUPPORTED = 6, /* valid request this build does not serve   */
    KNN_ERR_NODEVICE = 7,    /* no usable MI355X (gfx950) device          */
    KNN_ERR_RCCL = 8         /* RCCL ring error                           */
};

enum knn_layout { KNN_COLMAJOR = 0, KNN_ROWMAJOR = 1 };
enum knn_dtype  { KNN_F64 = 0, KNN_F32 = 1 };
enum knn_vote   { KNN_VOTE_SERIAL = 0, KNN_VOTE_MPI = 1, KNN_VOTE_MAJORITY = 2 };

/* Largest k served: KNN_F64 32 (the reference fixes NN = 30, serial:8 /
 * blk:9); KNN_F32 128 (BASELINE configs[4]: k = 100). */
#define KNN_MAX_K 32
#define KNN_MAX_K_F32 128

KNN_API const char *knn_strerror(int status);

/* ---------------------------------------------------------------------- *
 * Ingest -- replaces matOpen / matGetVariable / mxGetM / mxGetN / mxGetPr /
 * mxDestroyArray / matClose (serial:38-52, 100-109; blk:63-68, 72-79, 113-116;
 * nb:73-78, 82-89, 123-126).  Reads MAT-v5 (uncompressed) and v7 (zlib
 * miCOMPRESSED) files; any real numeric class is converted to double.
 * *X is column-major m x n (like mxGetPr of train_X), *labels has the
 * numel of lvar (m x 1).  lvar may be NULL.  Free both with knn_free().
 * ---------------------------------------------------------------------- */
KNN_API int  knn_load_mat(const char *path, const char *xvar, const char *lvar,
                  double **X, size_t *m, size_t *n, double **labels, size_t *nlabels);
KNN_API void knn_free(void *p);

/* ---------------------------------------------------------------------- *
 * Element type of the search (dtype):
 *   KNN_F64  the reference's arithmetic (results as described above).
 *   KNN_F32  the points are rounded to fp32 and filtered with fp32 MFMA
 *            (v_mfma_f32_16x16x4f32, 2x the fp64 rate).  Results are the
 *            exact k nearest neighbours OF THE fp32-ROUNDED POINTS under the
 *            reference's semantics: candidates are re-ranked by the
 *            reference-order fp64 sum S over the rounded values, certified,
 *            and rescanned when uncertified, exactly like the fp64 GEMM mode.
 *            Integer data with n*max|x|^2 <= 2^23 and n*(max-min)^2 <= 2^24
 *            (e.g. 8-bit pixels at n <= 128) is exact in fp32 arithmetic:
 *            identical to KNN_F64.  Otherwise the only deviation from the
 *            fp64 reference is the input rounding: |x - fp32(x)| <=
 *            2^-24 |x| per coordinate, so each reported distance is within
 *            2^-24 * (|q| + |c|) of the reference's (tests/test_gpu_f32.py).
 * ---------------------------------------------------------------------- */

/* ---------------------------------------------------------------------- *
 * One-call search on host arrays -- replaces the search section of
 * serial:54-93 and the whole ring of blk:81-244 / nb:91-259.
 * X: m x n fp64 in `layout`; labels (nullable, m doubles) fill .label;
 * ngpus >= 1 GPUs of this node (the corpus rotates over an RCCL ring when
 * ngpus > 1; results are byte-identical for every ngpus); dtype KNN_F64 or
 * KNN_F32 (above).  out: caller-owned m*k records.
 * ---------------------------------------------------------------------- */
KNN_API int knn_search(const double *X, size_t m, size_t n, int layout,
               const double *labels, int k, int ngpus, int dtype,
               knn_neighbour_t *out);

/* Bug-compatible mode (opt-in): the lists mpi-knn-parallel_
 * blocking.c / _non_blocking.c with `procs` ranks actually compute.  Rank
 * r keeps R = floor(m/procs) rows (the rest dropped, blk:81), folds its own
 * block, then the blocks of ranks r-2, r-3, ..., r-procs (= r again), each
 * truncated by the short first hop (blk:130-146: last ~2R/(n+2) rows zero)
 * and carrying idx 0 / label 0 (blk:169,231); block r-1 is never seen.
 * Ties keep scan order (blk:24-31).  fp64, k <= KNN_MAX_K, procs >= 2; the
 * ranks run one after another on device 0.  out: procs*R*k records, rank r
 * at out + r*R*k.  labels (nullable) fill .label of own-block records. */
KNN_API int knn_search_mpi_compat(const double *X, size_t m, size_t n, int layout,
                                  const double *labels, int k, int procs,
                                  knn_neighbour_t *out);

/* Search wall time of the last knn_search() on this thread, seconds: the
 * span the reference times (serial:70-98, blk:120-250) -- device compute
 * only, excluding load, H2D, D2H and vote. */
KNN_API double knn_last_search_seconds(void);

/* ---------------------------------------------------------------------- *
 * Vote + accuracy -- replaces serial:104-130 (rule SERIAL), blk:252-270 /
 * nb:269-288 (rule MPI); rule MAJORITY is a true majority (not in the
 * reference).  labels: per-row class labels (1..nclasses, as stored in the
 * .mat).  pred (nullable): m predicted labels.  *matches: rows whose
 * prediction equals their own label.  Empty slots (idx 0) are skipped where
 * the reference would read out of bounds.
 * ---------------------------------------------------------------------- */
KNN_API int knn_classify(const knn_neighbour_t *nb, size_t m, int k, int nclasses,
                 int vote_rule, const double *labels, int *pred, size_t *matches);

/* The same vote on the device, on the records knn_ctx_end / rescan_end
 * wrote (no host round trip).  d_nb: m*k records of queries with global ids
 * q_base..q_base+m-1, whose .label it fills (blk:176); d_labels: nlabels
 * row labels (global id i at d_labels[i-1]; ids > nlabels count as empty);
 * d_pred (nullable): m predictions; d_matches (nullable): one device
 * counter, set to the number of queries predicted as their own label.
 * nclasses <= KNN_VOTE_MAX_CLASSES (else KNN_ERR_UNSUPPORTED: use the host
 * knn_classify). */
#define KNN_VOTE_MAX_CLASSES 1024
KNN_API int knn_classify_device(knn_neighbour_t *d_nb, size_t m, int k, int nclasses,
                        int vote_rule, const double *d_labels, size_t nlabels, size_t q_base,
                        int *d_pred, unsigned long long *d_matches, void *stream);

/* ---------------------------------------------------------------------- *
 * Device-resident API (the engine underneath knn_search; used by the
 * per-rank RCCL ring driver and by bench.py).  All pointers named d_* are
 * device pointers on the context's device.
 *
 * A "packed block" holds up to `cap` points (its capacity) laid out for
 * the kernels:
 *   [cap_pad x n_pad fp64 row-major, zero padded][cap_pad fp64 squared
 *   norms][KNN_META_DOUBLES fp64 meta], cap_pad = cap rounded up to 128,
 *   n_pad = n rounded up to 16.  One contiguous buffer, so a ring hop moves
 *   a block with one send (blk:195-212 moved R*(n+2) doubles).  Every block
 *   of one ring has the same capacity, hence the same byte size.
 * ---------------------------------------------------------------------- */
#define KNN_META_DOUBLES 8

KNN_API size_t knn_block_bytes(size_t cap, size_t n);
/* Offset (bytes) of the meta doubles inside a packed block.  The meta of
 * all blocks of one search must be MAX-reduced into the d_meta passed to
 * knn_ctx_begin (a one-shot all-reduce of 8 doubles across ranks). */
KNN_API size_t knn_block_meta_offset(size_t cap, size_t n);
/* The same for blocks of element type dtype (KNN_F64 blocks above; KNN_F32
 * blocks hold fp32 rows padded to 32 features and fp32 norms, then the
 * same 8 fp64 meta words).  0 for an unknown dtype. */
KNN_API size_t knn_block_bytes_dt(size_t cap, size_t n, int dtype);
KNN_API size_t knn_block_meta_offset_dt(size_t cap, size_t n, int dtype);

/* Ring wire form of a packed block: the elements as int16, norms and meta
 * verbatim -- a quarter (fp64) or half (fp32) of the block bytes on the
 * link.  Exact only when knn_wire_ok(host copy of the reduced meta): every
 * value an integer with max|x| <= 32767.  knn_wire_unpack restores the
 * block bit for bit.  Used by mpiknn/ring.py between RCCL hops. */
KNN_API size_t knn_wire_bytes(size_t cap, size_t n, int dtype);
KNN_API int knn_wire_ok(const double *h_meta);
KNN_API int knn_wire_pack(void *d_wire, const void *d_block, size_t cap, size_t n, int dtype,
                          void *stream);
KNN_API int knn_wire_unpack(void *d_block, const void *d_wire, size_t cap, size_t n, int dtype,
                            void *stream);

/* Shadow block of a packed block: its rows as fp16 (round_up(n, 64) halves
 * a row), norms and meta verbatim.  When knn_ctx_shadow(ctx) is 1 after
 * knn_ctx_begin (the fp16 contraction is exact for this search and staged
 * from shadow rows), knn_ctx_step_shadow folds a shadow block instead of
 * the element block -- the ring then moves shadow blocks (2 bytes an
 * element).  The exact rescan (knn_ctx_rescan_step) still takes element
 * blocks. */
KNN_API size_t knn_shadow_bytes(size_t cap, size_t n, int dtype);
KNN_API size_t knn_shadow_norm_offset(size_t cap, size_t n);
KNN_API int knn_shadow_pack(void *d_sblock, const void *d_block, size_t cap, size_t n, int dtype,
                            void *stream);

/* Split fp16 rows of a packed block (the split-fp16 filter's form of
 * real-valued data): for rows_pad(cap) rows, per 32 features the 32 halves
 * hi = RN16(scale x) then the 32 halves lo = RN16(scale x - hi), each
 * rounded once from the block's precision, zero past n; rows of round_up(n, 32) * 4 bytes (knn_split_bytes).
 * scale: a power of two.  The engine converts the blocks of a split-filter
 * search itself; this entry point exposes the same conversion for tests
 * and tools. */
KNN_API size_t knn_split_bytes(size_t cap, size_t n);
KNN_API int knn_split_pack(void *d_dst, const void *d_block, size_t cap, size_t n, int dtype, double scale,
                           void *stream);

/* Pack rows (<= cap) points from a device source.  layout KNN_COLMAJOR:
 * element (i, j) at d_src[i + j*ld] (ld >= rows; the .mat layout,
 * serial:82); KNN_ROWMAJOR: d_src[i*ld + j] (ld >= n; blk:81-109).
 * Computes norms and meta.  Replaces blk:100-109 / nb:110-119. */
KNN_API int knn_block_pack(void *d_block, size_t cap, size_t rows, size_t n, const double *d_src,
                   size_t ld, int layout, void *stream);
/* Pack into a block of element type dtype from a source of src_dtype
 * (fp64 or fp32 device array, same layouts). */
KNN_API int knn_block_pack_dt(void *d_block, int dtype, size_t cap, size_t rows, size_t n,
                      const void *d_src, int src_dtype, size_t ld, int layout, void *stream);

typedef struct knn_ctx knn_ctx_t;

/* nq queries of dimension n; corpus blocks are packed with capacity
 * block_cap (knn_block_pack's cap) and hold at most block_cap rows. */
KNN_API int knn_ctx_create(knn_ctx_t **ctx, int device, size_t nq, size_t n,
                   size_t block_cap, int k);
/* A context over blocks of element type dtype (knn_ctx_create: KNN_F64). */
KNN_API int knn_ctx_create_dt(knn_ctx_t **ctx, int device, size_t nq, size_t n,
                      size_t block_cap, int k, int dtype);
KNN_API int knn_ctx_destroy(knn_ctx_t *ctx);

/* Start: the queries are the first nq rows of packed block d_qblock
 * (capacity q_cap) with global ids q_base..q_base+nq-1; d_meta = the
 * max-reduced meta of every corpus block. */
KNN_API int knn_ctx_begin(knn_ctx_t *ctx, const void *d_qblock, size_t q_cap, size_t q_base,
                  const double *d_meta, void *stream);
/* The same with the host copy of the reduced meta (h_meta, 8 doubles; the
 * ring drivers hold it after their all-reduce), so begin does not read it
 * back from the device (no stream synchronisation).  h_meta NULL = begin. */
KNN_API int knn_ctx_begin_meta(knn_ctx_t *ctx, const void *d_qblock, size_t q_cap, size_t q_base,
                               const double *d_meta, const double *h_meta, void *stream);

/* Speculative byte block (the int8 contraction's form) straight from the
 * source -- the fast path for 8-bit integer data (MNIST pixels, SIFT
 * descriptors).  Writes knn_s8_block_bytes(cap, n) bytes: rows of x - 128 as
 * int8, the int8 kernel's norm words, and at knn_s8_block_meta_offset the
 * block's 8 meta doubles (the same values knn_block_pack_dt computes, and
 * word 7 = 1: after the MAX-reduction it says some block was packed this
 * way; reduce them across blocks as usual).  The bytes are the int8 path's rows exactly
 * when knn_s8_spec_ok(reduced meta) -- every value an integer in [0, 255]
 * and the search int8-eligible; then knn_ctx_begin_s8 starts the search from
 * it (no element block, no conversion; a ring moves it as the shadow block),
 * otherwise pack the element block (knn_block_pack_dt) and knn_ctx_begin_meta.
 * One read of the source, 1 byte written an element (replaces the pack of
 * blk:100-109 plus the element -> byte conversion). */
KNN_API size_t knn_s8_block_bytes(size_t cap, size_t n);
KNN_API size_t knn_s8_block_meta_offset(size_t cap, size_t n);
KNN_API int knn_block_pack_s8(void *d_sblock, int dtype, size_t cap, size_t rows, size_t n, const void *d_src,
                              int src_dtype, size_t ld, int layout, void *stream);
KNN_API int knn_s8_spec_ok(const double *h_meta, size_t n, int dtype);
/* begin from the query block's speculative byte block (h_meta: the reduced
 * meta, host; KNN_ERR_INVALID unless knn_s8_spec_ok).  The element block is
 * needed only by the exact rescan: pack it and knn_ctx_attach_qblock before
 * knn_ctx_rescan_step when knn_ctx_end reports unresolved queries. */
KNN_API int knn_ctx_begin_s8(knn_ctx_t *ctx, const void *d_sblock, size_t q_cap, size_t q_base,
                             const double *d_meta, const double *h_meta, void *stream);
KNN_API int knn_ctx_attach_qblock(knn_ctx_t *ctx, const void *d_qblock, size_t q_cap);

/* Fold one packed corpus block (nc rows, global ids c_base..) into the
 * running neighbour lists.  Blocks may come in any order (ring order).
 * Asynchronous and overlapped: the step's distance kernel may start while
 * earlier steps still run (internal streams), and `stream` is made to wait
 * for step s - KNN_STEP_LAG only.  So work enqueued on `stream` after step
 * s returns may overwrite the blocks of steps <= s - KNN_STEP_LAG and no
 * later one: a ring rotates KNN_STEP_LAG + 2 receive buffers (knn_ring.c,
 * mpiknn/ring.py).  knn_ctx_end orders `stream` after every step. */
#define KNN_STEP_LAG 2
/* Shadow-block form of knn_ctx_step; valid while knn_ctx_shadow(ctx) is
 * nonzero after knn_ctx_begin: 1 = fp16 shadow blocks (knn_shadow_pack),
 * 2 = byte blocks of the int8 contraction (8-bit-window integer data, n <=
 * 896: rows as int8 x - o, o from the reduced meta, plus int32 norms).
 * knn_ctx_shadow_bytes / knn_ctx_shadow_pack size and pack a block of
 * capacity cap in the context's current form (the form a ring moves). */
KNN_API int knn_ctx_shadow(const knn_ctx_t *ctx);
KNN_API size_t knn_ctx_shadow_bytes(const knn_ctx_t *ctx, size_t cap);
KNN_API int knn_ctx_shadow_pack(knn_ctx_t *ctx, void *d_sblock, const void *d_block, size_t cap,
                                void *stream);
KNN_API int knn_ctx_step_shadow(knn_ctx_t *ctx, const void *d_sblock, size_t nc, size_t c_base,
                                void *stream);
KNN_API int knn_ctx_step(knn_ctx_t *ctx, const void *d_cblock, size_t nc,
                 size_t c_base, void *stream);
/* Fold nblk resident shadow-form blocks (d_sblocks[b]: nc[b] rows, global
 * ids c_base[b]..; any order) -- the direct-exchange ring's step over every
 * block received from the other ranks (blk:217-242 for all of them at
 * once).  Byte blocks (knn_ctx_shadow == 2) share one distance launch per 8
 * blocks, which counts as ONE step of the lag rule above: none of the
 * blocks may be overwritten before KNN_STEP_LAG further steps (or
 * knn_ctx_end).  fp16 shadow blocks fold one block a step. */
KNN_API int knn_ctx_step_shadow_n(knn_ctx_t *ctx, int nblk, const void *const *d_sblocks,
                                  const size_t *nc, const size_t *c_base, void *stream);
/* The same for nblk resident element blocks (d_cblocks[b]: packed blocks of
 * capacity block_cap): a search on the split-fp16 filter (real-valued data,
 * knn_ctx_split) folds up to 8 of them in one distance launch and one merge,
 * which count as ONE step of the lag rule; other searches fold one block a
 * step. */
KNN_API int knn_ctx_step_n(knn_ctx_t *ctx, int nblk, const void *const *d_cblocks, const size_t *nc,
                           const size_t *c_base, void *stream);

/* Finish: write nq*k records to d_out.  Returns in *unresolved (host; the
 * call synchronises the stream) the number of queries whose candidate set
 * could not be certified exact; if > 0 the caller runs one more pass over
 * every block with knn_ctx_rescan_step() then knn_ctx_rescan_end().  The
 * records are written behind the last merge on the context's own stream,
 * which first waits for `stream` as it stands at the call (so d_out may have
 * just been allocated, cleared or read on `stream`); `stream` is ordered
 * after the records on return.  A search begun with knn_ctx_begin_s8 whose
 * device meta turns out not to be INT-exact reports every query unresolved
 * (nothing is read through the missing element block). */
KNN_API int knn_ctx_end(knn_ctx_t *ctx, knn_neighbour_t *d_out, size_t *unresolved,
                void *stream);
KNN_API int knn_ctx_rescan_step(knn_ctx_t *ctx, const void *d_cblock, size_t nc,
                        size_t c_base, void *stream);
KNN_API int knn_ctx_rescan_end(knn_ctx_t *ctx, knn_neighbour_t *d_out, void *stream);
/* A ring rank's int8 re-search, between knn_ctx_end and the rescan pass:
 * the queries knn_ctx_end left uncertified are searched again on the int8
 * contraction with 65-entry lane lists (as a single-block search does inside
 * knn_ctx_end) against the nblk byte blocks the rank still holds (d_sblocks:
 * its own and the received ones, nc[b] rows from global id c_base[b] --
 * together every row of the corpus); certified queries get their records
 * in d_out.  *unresolved (host; the call synchronises the stream) is the
 * count the rescan pass still has to resolve -- 0 spares the rank the
 * element-block exchange of mpi-knn-parallel_blocking.c:187-214's repeat.
 * A no-op (returning the unchanged count) unless the search ran on the int8
 * contraction in INT mode (knn_ctx_shadow == 2) with k <= 32. */
KNN_API int knn_ctx_research_blocks(knn_ctx_t *ctx, int nblk, const void *const *d_sblocks, const size_t *nc,
                                    const size_t *c_base, knn_neighbour_t *d_out, size_t *unresolved,
                                    void *stream);

/* Convenience: the whole single-device pipeline on one packed block of
 * capacity m (queries == corpus == rows 0..m-1), including the rescan pass
 * when needed.  ctx must have nq == block_cap == m. */
KNN_API int knn_search_packed(knn_ctx_t *ctx, const void *d_block, size_t m,
                      knn_neighbour_t *d_out, void *stream);

/* Diagnostics of the last knn_ctx_end: engine mode (0 integer-exact,
 * 1 fp64 GEMM + exact re-rank, 2 exact scan) and the corpus split count. */
KNN_API int knn_ctx_info(const knn_ctx_t *ctx, int *mode, int *splits);

/* Input width in bits of the MFMA contraction of the current search: 64
 * (fp64 blocks), 32 (fp32 blocks), 16 when it runs on fp16 MFMA because
 * that is exact for the data (integers with max|x| <= 256 (fp64) / 2048
 * (fp32) in the exact-integer range; KNN_NO_H16=1 disables it), or 8 when
 * it runs on int8 MFMA (integers inside a window of 256 values, n <= 896:
 * exact int32 dot products; KNN_NO_I8=1 disables it).  Set by
 * knn_ctx_begin.  0 for a NULL context. */
KNN_API int knn_ctx_contraction_bits(const knn_ctx_t *ctx);
/* 1 when the current search filters with the split fp16 contraction: fp32
 * blocks in GEMM mode (non-integer data), each value scaled by a power of
 * two S and split as S x = hi + lo in fp16, hi.hi + hi.lo + lo.hi on fp16
 * MFMA (fp32 accumulate); the candidates are re-ranked by the exact fp64 S
 * and certified with that filter's error bound (knn_cert_E), so results are
 * those of the fp32 MFMA filter, bit for bit.  KNN_NO_SPLIT=1 disables it. */
KNN_API int knn_ctx_split(const knn_ctx_t *ctx);

/* Kernel timing with HIP events on the launch streams (the timers of
 * serial:70-98 at kernel granularity).  enable = 1 starts recording and
 * zeroes the totals, 0 stops (totals kept), -1 only reads.  Totals (ms) cover
 * every step since the last reset whose knn_ctx_end has returned: dist_ms is
 * the time during which some k_dist_topk runs (the union of their
 * intervals per search -- steps overlap, knn_ctx_step), merge_ms the time
 * k_merge work adds outside it; *launches counts k_dist_topk launches. */
KNN_API int knn_ctx_profile(knn_ctx_t *ctx, int enable, double *dist_ms, double *merge_ms,
                    int *launches);
/* The merge kernels' own time over the same steps (recorded while
 * knn_ctx_profile is on): *merge_kernel_ms sums the durations of every
 * k_merge / k_merge_rank launch (the exact fp64 re-rank of knn-serial.c:
 * 86-91 in GEMM mode; in INT mode the rank merge, which also finalizes at
 * the search's end), bracketed by events on the merge's stream; *merges
 * counts them and *bytes sums their algorithmic bytes (partial lists and
 * bounds read, state read and written or records written, and in GEMM mode
 * the query's and its k neighbours' rows for the exact S) -- bench.py
 * prices them against HBM. */
KNN_API int knn_ctx_profile_merge(knn_ctx_t *ctx, double *merge_kernel_ms, int *merges, double *bytes);

/* on != 0: the context's searches fold ONE block in one step (a P = 1
 * search, knn-serial.c:72-93 over the whole corpus): the step's distance
 * kernel and knn_ctx_end's merge run on the caller's stream, back to back,
 * with no event record or cross-stream wait between them, and end() does
 * not wait for the caller's stream on the host first.  A second step in such
 * a search falls back to the step schedule (exact either way).  Default 0. */
KNN_API int knn_ctx_set_solo(knn_ctx_t *ctx, int on);
/* The 8 meta doubles the last search's kernels read (copied to mapped host
 * memory by its last kernel; valid after knn_ctx_end returned KNN_OK): a
 * caller that began the search from a meta hint checks it with this,
 * without a read-back copy of its own on the stream. */
KNN_API int knn_ctx_search_meta(const knn_ctx_t *ctx, double *meta);

#ifdef __cplusplus
}
#endif
#endif /* KNN_H */
