/*
 * knn_engine.c -- host side of libknn (C, HIP runtime API).
 *
 * Owns device buffers and sequences the kernels of knn_kernels.hip:
 *   knn_block_pack  -> k_pack_col / k_pack_row (blk:100-109 packing)
 *   knn_ctx_step    -> k_dist_topk + k_merge (one ring step, blk:217-242)
 *   knn_ctx_end     -> k_finalize            (+ rescan pass when needed)
 * and implements the one-call knn_search() of include/knn.h on top.
 */
#include "knn_internal.h"

#include <hip/hip_runtime_api.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define HIPCHK(x)                                   \
    do {                                            \
        if ((x) != hipSuccess) return KNN_ERR_HIP;  \
    } while (0)
#define RCHK(x)                  \
    do {                         \
        int rc_ = (x);           \
        if (rc_) return rc_;     \
    } while (0)

#define KNN_MAX_LISTS 63  /* merge kernel: lpq*splits + 1 lists <= 64 lanes */
#define KNN_PSETS 4       /* partial-list sets: step s uses set s % 4   */
#define KNN_PROF_STEPS 64 /* steps timed between two knn_ctx_end calls */

struct knn_ctx {
    int device;
    int dtype;          /* element type of the packed blocks (KNN_F64 / KNN_F32) */
    size_t nq, nq_pad, n, block_cap;
    int k;
    int kp, kl;         /* state capacity / per-lane list length serving k */
    int xord;           /* workgroup order: 0 split-major, 1 XCD-grouped, -1 by the launch (xord_for) */
    int h16;            /* this search's contraction runs on fp16 MFMA (exact) */
    int i8;             /* ... on int8 MFMA over byte blocks (knn_i8.hip, exact) */
    int shadow;         /* step_shadow form: 0 none, 1 fp16 shadow rows, 2 byte blocks */
    void *qsh, *csh[KNN_PSETS];
    size_t qsh_bytes, csh_bytes;
    void *qs8, *cs8[KNN_PSETS];   /* byte blocks: the queries, converted corpus blocks */
    const void *q8;               /* the query byte block the kernels read: qs8 or the caller's (begin_s8) */
    size_t qs8_bytes;
    int split;          /* this search filters with the split fp16 contraction (fp32 GEMM mode) */
    float sscale;       /* its power-of-two pre-scale S */
    void *qsp, *csp[KNN_PSETS];   /* split shadow rows: the queries, converted corpus blocks */
    size_t qsp_bytes, csp_bytes;
    void *cspm[KNN_PSETS];        /* a fused GEMM step's blocks in split form, side by side */
    size_t cspm_bytes[KNN_PSETS];
    int lpq, klx;       /* partial lists of the active kernel: lpq per query and split, klx long */
    int i8_wgpc;        /* int8 distance workgroups a CU (2: the half-tile kernel) */
    int cus;
    /* per-step partial lists of k_dist_topk, KNN_PSETS sets used in turn
     * (step s+1's distance kernel runs while step s is merged), each
     * grown to the largest split count used so far with it (part_splits) */
    double *part_d[KNN_PSETS];        /* set pointers into the pair buffers */
    int *part_i[KNN_PSETS];
    double *part_T[KNN_PSETS];
    /* sets 2j and 2j+1 share one allocation, the odd set right behind the
     * even one, so a k_merge can read both steps' lists as one array */
    double *pp_d[KNN_PSETS / 2];
    int *pp_i[KNN_PSETS / 2];
    double *pp_T[KNN_PSETS / 2];
    int pp_cap[KNN_PSETS / 2];        /* splits per pair allocation */
    size_t pp_per[KNN_PSETS / 2];     /* list entries per split it was sized for */
    /* an even step whose merge waits for the next step (pairing) */
    int pend, pend_set, pend_nsplit, pend_nc, merged;
    /* a paired merge of a fused step, deferred to the next step or to
     * knn_ctx_end (which then merges and finalizes in one launch) */
    int pend2, pend2_set, pend2_nsplit;
    hipEvent_t *pend2_ev[2];
    int even_nsplit;                  /* splits of the last even step: the odd set's offset */
    const void *pend_cblk;
    size_t pend_cbase;
    hipEvent_t *pend_ev;
    /* overlapped step schedule (knn_ctx_step): distance kernels alternate
     * over two streams, merges run in order on a third */
    hipStream_t ds[2], ms;
    hipEvent_t ev_in, ev_m[KNN_PSETS], ev_ds[KNN_PSETS], ev_end;
    int nstep;
    /* per-query filter bound shared by all splits and ring steps */
    double *qthr;
    /* int8 kernel: per query 4 cross-split summary slots (k_dist_topk_i8) */
    unsigned long long *qsum;
    /* running state per query: KNN_KP x (approx d^2, exact S, idx), T pair */
    double *st_d, *st_x, *st_T;
    int *st_i;
    /* unresolved queries */
    int *fail_count, *fail_list, *mode_dev;
    /* the pair's host copy (pinned, mapped): k_count_out writes it behind
     * the last merge, so knn_ctx_end's read-back is no blit */
    int *h_count, *h_count_dev;
    double *fbound;     /* per query: rescan bound on the k-th key (k_finalize) */
    double *rs_d;
    int *rs_i;
    size_t rs_cap;
    /* current search */
    const void *qblk;
    size_t q_base, q_rows_pad;
    const double *meta;
    int first_step;
    int ended;          /* knn_ctx_end completed this search (no step since) */
    /* knn_ctx_set_solo: a search of one step runs its distance kernel and
     * merge on the caller's stream (solo_on: this search's first step did,
     * ms_keep holds the merge stream meanwhile) */
    int solo, solo_on;
    hipStream_t ms_keep;
    int nsplit_last;
    /* choose_splits cache: (corpus rows, list shape, kernel) -> split count;
     * a direct-exchange pass alternates two launch sizes, and one model
     * evaluation costs ~0.5 ms of host time at 15000 queries */
#define KNN_SPLIT_CACHE 8
    struct { size_t nc; int lpq, i8, split, solo, klx, best; } split_cache[KNN_SPLIT_CACHE];
    int split_next;
    int nfail;
    int mode;
    /* the int8 re-search of uncertified queries (knn_ctx_end, single-block
     * searches): host meta of the search, the step's block, a sub-context
     * with 65-entry lane lists and its buffers */
    double hmeta[KNN_META_DOUBLES];
    int have_hmeta;
    int split_solo;           /* choose_splits: this step folds the search's own query
                               * byte block first (a P = 1 search is only that) */
    int sub_research;         /* this context is such a sub-context: 65-entry lists
                               * over the most splits the merge takes */
    int one_block_q8;         /* the search's only step folded its own query byte block */
    size_t step0_nc, step0_cbase;
    struct knn_ctx *sub;
    size_t sub_cap;
    void *sub_q8;
    knn_neighbour_t *sub_out;
    unsigned char *sub_flag;
    int *fail_list2;
    /* the GEMM-mode merge's query order (knn_order.hip), found once a
     * search from its first merged lists */
    int *ord_lab, *ord_keys, *ord_iota, *ord_perm;
    void *ord_tmp;
    size_t ord_cap, ord_tmp_bytes;
    int ord_ready;
    /* kernel timing (knn_ctx_profile): 3 events per step bracket
     * k_dist_topk and k_merge */
    int prof_on, prof_pending, prof_launches;
    double prof_dist_ms, prof_merge_ms;
    hipEvent_t prof_ev[3 * KNN_PROF_STEPS];
    /* merge kernels (k_merge / k_merge_rank) alone: an event before and one
     * after each launch on its stream (knn_ctx_profile_merge) */
    int prof_mk_pending, prof_mk_launches;
    double prof_mk_ms, prof_mk_bytes;
    hipEvent_t prof_mk_ev[2 * KNN_PROF_STEPS];
};

static __thread double g_last_search_s = 0.0;

const char *knn_strerror(int status)
{
    switch (status) {
    case KNN_OK: return "ok";
    case KNN_ERR_INVALID: return "invalid argument";
    case KNN_ERR_NOMEM: return "out of memory";
    case KNN_ERR_HIP: return "HIP runtime error";
    case KNN_ERR_IO: return "I/O error";
    case KNN_ERR_FORMAT: return "unsupported or malformed MAT file";
    case KNN_ERR_UNSUPPORTED: return "unsupported request";
    case KNN_ERR_NODEVICE: return "no usable gfx950 device";
    case KNN_ERR_RCCL: return "RCCL error";
    default: return "unknown status";
    }
}

void knn_free(void *p) { free(p); }

double knn_last_search_seconds(void) { return g_last_search_s; }
void knn_set_last_search_seconds(double s) { g_last_search_s = s; }

static int dtype_ok(int dtype) { return dtype == KNN_F64 || dtype == KNN_F32; }

size_t knn_block_meta_offset_dt(size_t cap, size_t n, int dtype)
{
    if (!dtype_ok(dtype)) return 0;
    const size_t rp = knn_rows_pad(cap), np = knn_n_pad_dt(n, dtype);
    return (rp * np + rp) * knn_esize(dtype);
}

size_t knn_block_bytes_dt(size_t cap, size_t n, int dtype)
{
    if (!dtype_ok(dtype)) return 0;
    return knn_block_meta_offset_dt(cap, n, dtype) + KNN_META_DOUBLES * sizeof(double);
}

size_t knn_block_meta_offset(size_t cap, size_t n) { return knn_block_meta_offset_dt(cap, n, KNN_F64); }

/* Wire form: [rows_pad x n_pad int16][the block's norms and meta, verbatim] */
size_t knn_wire_bytes(size_t cap, size_t n, int dtype)
{
    if (!dtype_ok(dtype)) return 0;
    const size_t rp = knn_rows_pad(cap), np = knn_n_pad_dt(n, dtype);
    return knn_round_up(rp * np * sizeof(short) + rp * knn_esize(dtype) +
                        KNN_META_DOUBLES * sizeof(double), 16);
}

int knn_wire_ok(const double *h_meta)
{
    if (!h_meta) return 0;
    return h_meta[KNN_META_NONINT] == 0.0 && h_meta[KNN_META_NONFINITE] == 0.0 &&
           h_meta[KNN_META_MAXABS] <= 32767.0;
}

static int wire_copy(void *dst, const void *src, size_t cap, size_t n, int dtype, int unpack,
                     void *stream)
{
    if (!dst || !src || !dtype_ok(dtype)) return KNN_ERR_INVALID;
    const size_t rp = knn_rows_pad(cap), np = knn_n_pad_dt(n, dtype), es = knn_esize(dtype);
    const size_t cnt = rp * np;
    const size_t tail = rp * es + KNN_META_DOUBLES * sizeof(double);
    RCHK(knn_launch_wire(unpack, dst, src, dtype, cnt, stream));
    char *d = (char *)dst + cnt * (unpack ? es : sizeof(short));
    const char *s = (const char *)src + cnt * (unpack ? sizeof(short) : es);
    HIPCHK(hipMemcpyAsync(d, s, tail, hipMemcpyDeviceToDevice, (hipStream_t)stream));
    return KNN_OK;
}

int knn_wire_pack(void *d_wire, const void *d_block, size_t cap, size_t n, int dtype, void *stream)
{
    return wire_copy(d_wire, d_block, cap, n, dtype, 0, stream);
}

int knn_wire_unpack(void *d_block, const void *d_wire, size_t cap, size_t n, int dtype, void *stream)
{
    return wire_copy(d_block, d_wire, cap, n, dtype, 1, stream);
}

/* Shadow block: [rows_pad x round_up(n,64) fp16][the block's norms and
 * meta, verbatim] -- what the fp16 contraction stages (knn_ctx_step_shadow) */
size_t knn_shadow_norm_offset(size_t cap, size_t n)
{
    return knn_rows_pad(cap) * knn_round_up(n, 64) * 2;
}

size_t knn_shadow_bytes(size_t cap, size_t n, int dtype)
{
    if (!dtype_ok(dtype)) return 0;
    return knn_round_up(knn_shadow_norm_offset(cap, n) + knn_rows_pad(cap) * knn_esize(dtype) +
                        KNN_META_DOUBLES * sizeof(double), 16);
}

size_t knn_split_bytes(size_t cap, size_t n) { return knn_rows_pad(cap) * knn_split_rs(n); }

int knn_split_pack(void *d_dst, const void *d_block, size_t cap, size_t n, int dtype, double scale, void *stream)
{
    if (!d_dst || !d_block || !dtype_ok(dtype) || n == 0 || cap == 0 || !(scale > 0.0)) return KNN_ERR_INVALID;
    int e = 0;
    if (frexp(scale, &e) != 0.5) return KNN_ERR_INVALID;   /* a power of two */
    return knn_launch_shadow_split(d_dst, d_block, dtype, knn_rows_pad(cap), n, (float)scale, stream);
}

int knn_shadow_pack(void *d_sblock, const void *d_block, size_t cap, size_t n, int dtype, void *stream)
{
    if (!d_sblock || !d_block || !dtype_ok(dtype)) return KNN_ERR_INVALID;
    const size_t rp = knn_rows_pad(cap);
    RCHK(knn_launch_shadow(d_sblock, d_block, dtype, rp, n, stream));
    const size_t tail = rp * knn_esize(dtype) + KNN_META_DOUBLES * sizeof(double);
    HIPCHK(hipMemcpyAsync((char *)d_sblock + knn_shadow_norm_offset(cap, n),
                          (const char *)d_block + rp * knn_n_pad_dt(n, dtype) * knn_esize(dtype),
                          tail, hipMemcpyDeviceToDevice, (hipStream_t)stream));
    return KNN_OK;
}

size_t knn_block_bytes(size_t cap, size_t n) { return knn_block_bytes_dt(cap, n, KNN_F64); }

int knn_block_pack_dt(void *d_block, int dtype, size_t cap, size_t rows, size_t n,
                      const void *d_src, int src_dtype, size_t ld, int layout, void *stream)
{
    if (!d_block || !d_src || rows == 0 || n == 0 || rows > cap || cap > 0x7fffffffULL ||
        n > 0x7fffffffULL || !dtype_ok(dtype) || !dtype_ok(src_dtype))
        return KNN_ERR_INVALID;
    if (layout == KNN_COLMAJOR ? ld < rows : (layout == KNN_ROWMAJOR ? ld < n : 1))
        return KNN_ERR_INVALID;
    return knn_launch_pack(d_block, dtype, cap, rows, n, d_src, src_dtype, ld, layout, stream);
}

size_t knn_s8_block_bytes(size_t cap, size_t n) { return knn_s8_bytes(cap, n); }
size_t knn_s8_block_meta_offset(size_t cap, size_t n) { return knn_s8_meta_offset(cap, n); }

int knn_block_pack_s8(void *d_sblock, int dtype, size_t cap, size_t rows, size_t n, const void *d_src,
                      int src_dtype, size_t ld, int layout, void *stream)
{
    if (!d_sblock || !d_src || rows == 0 || n == 0 || rows > cap || cap > 0x7fffffffULL || n > KNN_I8_MAX_N ||
        !dtype_ok(dtype) || !dtype_ok(src_dtype))
        return KNN_ERR_INVALID;
    if (layout == KNN_COLMAJOR ? ld < rows : (layout == KNN_ROWMAJOR ? ld < n : 1)) return KNN_ERR_INVALID;
    return knn_launch_pack_s8(d_sblock, dtype, cap, rows, n, d_src, src_dtype, ld, layout, stream);
}

int knn_block_pack(void *d_block, size_t cap, size_t rows, size_t n, const double *d_src,
                   size_t ld, int layout, void *stream)
{
    return knn_block_pack_dt(d_block, KNN_F64, cap, rows, n, d_src, KNN_F64, ld, layout, stream);
}

static void ctx_free_buffers(knn_ctx_t *c)
{
    if (c->sub) knn_ctx_destroy(c->sub);
    hipFree(c->sub_q8);
    hipFree(c->sub_out);
    hipFree(c->sub_flag);
    hipFree(c->fail_list2);
    for (int b = 0; b < KNN_PSETS; b++) {
        if (c->ev_m[b]) hipEventDestroy(c->ev_m[b]);
        if (c->ev_ds[b]) hipEventDestroy(c->ev_ds[b]);
    }
    for (int b = 0; b < KNN_PSETS / 2; b++) {
        hipFree(c->pp_d[b]);
        hipFree(c->pp_i[b]);
        hipFree(c->pp_T[b]);
    }
    for (int b = 0; b < 2; b++) {
        if (c->ds[b]) hipStreamDestroy(c->ds[b]);
    }
    if (c->ms) hipStreamDestroy(c->ms);
    hipFree(c->qsh);
    for (int b = 0; b < KNN_PSETS; b++) hipFree(c->csh[b]);
    hipFree(c->qs8);
    for (int b = 0; b < KNN_PSETS; b++) hipFree(c->cs8[b]);
    hipFree(c->qsp);
    for (int b = 0; b < KNN_PSETS; b++) hipFree(c->csp[b]);
    for (int b = 0; b < KNN_PSETS; b++) hipFree(c->cspm[b]);
    if (c->ev_in) hipEventDestroy(c->ev_in);
    if (c->ev_end) hipEventDestroy(c->ev_end);
    hipFree(c->qthr);
    hipFree(c->qsum);
    hipFree(c->ord_lab);
    hipFree(c->ord_keys);
    hipFree(c->ord_iota);
    hipFree(c->ord_perm);
    hipFree(c->ord_tmp);
    hipFree(c->st_d);
    hipFree(c->st_x);
    hipFree(c->st_T);
    hipFree(c->st_i);
    hipFree(c->fail_count);
    if (c->h_count) hipHostFree(c->h_count);
    hipFree(c->fail_list);
    hipFree(c->fbound);
    hipFree(c->rs_d);
    hipFree(c->rs_i);
    for (int i = 0; i < 3 * KNN_PROF_STEPS; i++)
        if (c->prof_ev[i]) hipEventDestroy(c->prof_ev[i]);
    for (int i = 0; i < 2 * KNN_PROF_STEPS; i++)
        if (c->prof_mk_ev[i]) hipEventDestroy(c->prof_mk_ev[i]);
}

int knn_ctx_profile(knn_ctx_t *c, int enable, double *dist_ms, double *merge_ms, int *launches)
{
    if (!c) return KNN_ERR_INVALID;
    if (enable >= 0) {
        HIPCHK(hipSetDevice(c->device));
        if (enable && !c->prof_ev[0]) {
            for (int i = 0; i < 3 * KNN_PROF_STEPS; i++)
                HIPCHK(hipEventCreate(&c->prof_ev[i]));
            for (int i = 0; i < 2 * KNN_PROF_STEPS; i++)
                HIPCHK(hipEventCreate(&c->prof_mk_ev[i]));
        }
        c->prof_on = enable ? 1 : 0;
        if (enable) {
            c->prof_pending = 0;
            c->prof_launches = 0;
            c->prof_dist_ms = 0.0;
            c->prof_merge_ms = 0.0;
            c->prof_mk_pending = 0;
            c->prof_mk_launches = 0;
            c->prof_mk_ms = 0.0;
            c->prof_mk_bytes = 0.0;
        }
    }
    if (dist_ms) *dist_ms = c->prof_dist_ms;
    if (merge_ms) *merge_ms = c->prof_merge_ms;
    if (launches) *launches = c->prof_launches;
    return KNN_OK;
}

/* after the stream has been synchronised: fold the recorded steps of one
 * search.  Step i has events [3i] (distance kernel may start), [3i+1]
 * (distance kernel done), [3i+2] (merge done); overlapping steps are
 * counted once: dist = union of [3i, 3i+1], merge = union of [3i+1, 3i+2]
 * minus the distance union. */
static double interval_union(double *st, double *en, int n)
{
    for (int i = 1; i < n; i++)  /* insertion sort by start (n <= 64) */
        for (int j = i; j > 0 && st[j] < st[j - 1]; j--) {
            double t = st[j]; st[j] = st[j - 1]; st[j - 1] = t;
            t = en[j]; en[j] = en[j - 1]; en[j - 1] = t;
        }
    double total = 0.0, end = -1e30;
    for (int i = 0; i < n; i++) {
        const double s0 = st[i] > end ? st[i] : end;
        if (en[i] > s0) total += en[i] - s0;
        if (en[i] > end) end = en[i];
    }
    return total;
}

static int prof_collect(knn_ctx_t *c)
{
    const int n = c->prof_pending;
    double ds[KNN_PROF_STEPS], de[KNN_PROF_STEPS], as[KNN_PROF_STEPS], ae[KNN_PROF_STEPS];
    for (int i = 0; i < n; i++) {
        float s = 0.f, e = 0.f, me = 0.f;
        HIPCHK(hipEventElapsedTime(&s, c->prof_ev[0], c->prof_ev[3 * i]));
        HIPCHK(hipEventElapsedTime(&e, c->prof_ev[0], c->prof_ev[3 * i + 1]));
        HIPCHK(hipEventElapsedTime(&me, c->prof_ev[0], c->prof_ev[3 * i + 2]));
        ds[i] = as[i] = s;
        de[i] = e;
        ae[i] = me;
    }
    const double dist = interval_union(ds, de, n), all = interval_union(as, ae, n);
    c->prof_dist_ms += dist;
    c->prof_merge_ms += all > dist ? all - dist : 0.0;
    c->prof_launches += n;
    c->prof_pending = 0;
    for (int i = 0; i < c->prof_mk_pending; i++) {
        float ms = 0.f;
        HIPCHK(hipEventElapsedTime(&ms, c->prof_mk_ev[2 * i], c->prof_mk_ev[2 * i + 1]));
        c->prof_mk_ms += ms;
    }
    c->prof_mk_launches += c->prof_mk_pending;
    c->prof_mk_pending = 0;
    return KNN_OK;
}

int knn_ctx_set_solo(knn_ctx_t *c, int on)
{
    if (!c) return KNN_ERR_INVALID;
    c->solo = on ? 1 : 0;
    return KNN_OK;
}

int knn_ctx_search_meta(const knn_ctx_t *c, double *meta)
{
    if (!c || !meta || !c->ended) return KNN_ERR_INVALID;
    const volatile double *m = (const volatile double *)((const char *)c->h_count + 16);
    for (int i = 0; i < KNN_META_DOUBLES; i++) meta[i] = m[i];
    return KNN_OK;
}

int knn_ctx_profile_merge(knn_ctx_t *c, double *merge_kernel_ms, int *merges, double *bytes)
{
    if (!c) return KNN_ERR_INVALID;
    if (merge_kernel_ms) *merge_kernel_ms = c->prof_mk_ms;
    if (merges) *merges = c->prof_mk_launches;
    if (bytes) *bytes = c->prof_mk_bytes;
    return KNN_OK;
}

int knn_ctx_create_dt(knn_ctx_t **out, int device, size_t nq, size_t n, size_t block_cap, int k,
                      int dtype)
{
    if (!out || nq == 0 || n == 0 || block_cap == 0 || k <= 0 || !dtype_ok(dtype) ||
        k > (dtype == KNN_F32 ? KNN_MAX_K_F32 : KNN_MAX_K) || nq > 0x7fffffffULL ||
        block_cap > 0x7fffffffULL)
        return KNN_ERR_INVALID;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0 || device < 0 || device >= ndev)
        return KNN_ERR_NODEVICE;
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, device));
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return KNN_ERR_NODEVICE;
    HIPCHK(hipSetDevice(device));

    knn_ctx_t *c = (knn_ctx_t *)calloc(1, sizeof(*c));
    if (!c) return KNN_ERR_NOMEM;
    c->device = device;
    c->dtype = dtype;
    c->nq = nq;
    c->nq_pad = knn_round_up(nq, KNN_TQ);
    c->n = n;
    c->block_cap = block_cap;
    c->k = k;
    c->kp = knn_kp_for(k, dtype);
    c->kl = knn_kl_for(c->kp, dtype);
    c->lpq = 4;
    c->klx = c->kl;
    /* workgroup order: KNN_XCD_ORDER=1 / 0 forces the XCD-grouped / the
     * split-major order; unset (-1), split-filter launches of <= 2 splits
     * take the XCD-grouped one -- a query block's splits side by side on one
     * XCD share its query rows there (gist, 2 splits: 1419 -> 1399 ms a
     * launch), while at more splits it costs the corpus tiles' sharing
     * (mnist-real, 6 splits: 16.97 -> 19.99 ms) */
    {
        const char *xe = getenv("KNN_XCD_ORDER");
        c->xord = xe && xe[0] == '1' ? 1 : (xe && xe[0] == '0' ? 0 : -1);
    }
    c->cus = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;

    const size_t np = c->nq_pad;
    int ok = 1;
    ok &= hipMalloc((void **)&c->qthr, np * sizeof(double)) == hipSuccess;
    ok &= hipMalloc((void **)&c->qsum, np * 4 * sizeof(unsigned long long)) == hipSuccess;
    ok &= hipMalloc((void **)&c->st_d, np * c->kp * sizeof(double)) == hipSuccess;
    ok &= hipMalloc((void **)&c->st_x, np * c->kp * sizeof(double)) == hipSuccess;
    ok &= hipMalloc((void **)&c->st_i, np * c->kp * sizeof(int)) == hipSuccess;
    ok &= hipMalloc((void **)&c->st_T, np * 2 * sizeof(double)) == hipSuccess;
    /* [0] unresolved queries, [1] mode: one allocation, one read-back */
    ok &= hipMalloc((void **)&c->fail_count, 2 * sizeof(int)) == hipSuccess;
    ok &= hipMalloc((void **)&c->fail_list, np * sizeof(int)) == hipSuccess;
    ok &= hipMalloc((void **)&c->fbound, np * sizeof(double)) == hipSuccess;
    if (ok) c->mode_dev = c->fail_count + 1;
    /* mapped: [0] unresolved, [1] mode, then (at byte 16) the search's 8
     * meta doubles as its kernels read them (knn_ctx_search_meta) */
    ok &= hipHostMalloc((void **)&c->h_count, 16 + KNN_META_DOUBLES * sizeof(double), hipHostMallocMapped) ==
          hipSuccess;
    ok &= c->h_count && hipHostGetDevicePointer((void **)&c->h_count_dev, c->h_count, 0) == hipSuccess;
    for (int b = 0; b < 2; b++) {
        ok &= hipStreamCreateWithFlags(&c->ds[b], hipStreamNonBlocking) == hipSuccess;
    }
    for (int b = 0; b < KNN_PSETS; b++) {
        ok &= hipEventCreateWithFlags(&c->ev_m[b], hipEventDisableTiming) == hipSuccess;
        ok &= hipEventCreateWithFlags(&c->ev_ds[b], hipEventDisableTiming) == hipSuccess;
    }
    /* merges are short and gate the next steps: highest priority */
    int prio_lo = 0, prio_hi = 0;
    hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi);
    ok &= hipStreamCreateWithPriority(&c->ms, hipStreamNonBlocking, prio_hi) == hipSuccess;
    ok &= hipEventCreateWithFlags(&c->ev_in, hipEventDisableTiming) == hipSuccess;
    ok &= hipEventCreateWithFlags(&c->ev_end, hipEventDisableTiming) == hipSuccess;
    if (!ok) {
        ctx_free_buffers(c);
        free(c);
        return KNN_ERR_NOMEM;
    }
    *out = c;
    return KNN_OK;
}

int knn_ctx_create(knn_ctx_t **out, int device, size_t nq, size_t n, size_t block_cap, int k)
{
    return knn_ctx_create_dt(out, device, nq, n, block_cap, k, KNN_F64);
}

int knn_ctx_destroy(knn_ctx_t *c)
{
    if (!c) return KNN_OK;
    hipSetDevice(c->device);
    ctx_free_buffers(c);
    free(c);
    return KNN_OK;
}

int knn_ctx_contraction_bits(const knn_ctx_t *c)
{
    if (!c) return 0;
    if (c->i8) return 8;
    return (c->h16 || c->split) ? 16 : (c->dtype == KNN_F64 ? 64 : 32);
}

int knn_ctx_split(const knn_ctx_t *c) { return c ? c->split : 0; }

int knn_ctx_info(const knn_ctx_t *c, int *mode, int *splits)
{
    if (!c) return KNN_ERR_INVALID;
    if (mode) *mode = c->mode;
    if (splits) *splits = c->nsplit_last;
    return KNN_OK;
}

/* fp32 INT mode (knn_mode<float>: integers, n max|x|^2 <= 2^23,
 * n range^2 <= 2^24) with max|x| <= 2048, so every value is exact in fp16:
 * the fp16 MFMA contraction gives the fp32 path's dot products bit for bit
 * (knn_kernels.hip, knn_to_h8). */
static int knn_h16_exact(const double *meta, size_t n, int dtype)
{
    if (dtype == KNN_F64) {
        /* fp64 INT mode (knn_mode<double>) with max|x| <= 256: fp16 inputs
         * exact, fp32 sums exact over 256 features (knn_to_h4) */
        if (meta[KNN_META_NONFINITE] != 0.0 || !(meta[KNN_META_MAXNORM] < 1e290)) return 0;
        const double mx = meta[KNN_META_MAXABS];
        return meta[KNN_META_NONINT] == 0.0 && mx <= 256.0 &&
               mx * mx <= 2251799813685248.0 / (4.0 * (double)n);
    }
    if (meta[KNN_META_NONFINITE] != 0.0 || !(meta[KNN_META_MAXNORM] < 1e37)) return 0;
    const double mx = meta[KNN_META_MAXABS];
    const double rg = meta[KNN_META_MAXPOS] + meta[KNN_META_MAXNEG];
    return meta[KNN_META_NONINT] == 0.0 && mx <= 2048.0 && (double)n * mx * mx <= 8388608.0 &&
           (double)n * rg * rg <= 16777216.0;
}

/* INT mode for the element type (every key of the search exact) with every
 * value inside a window of 256 integers (hi - lo <= 255, lo = -meta[MAXNEG],
 * hi = meta[MAXPOS]) and n <= KNN_I8_MAX_N: x - (lo + 128) is an exact int8
 * and the int8 MFMA contraction gives d^2 exactly (knn_i8.hip). */
static int knn_i8_exact(const double *meta, size_t n, int dtype)
{
    if (n > KNN_I8_MAX_N || meta[KNN_META_NONFINITE] != 0.0 || meta[KNN_META_NONINT] != 0.0) return 0;
    if (!(meta[KNN_META_MAXNORM] < (dtype == KNN_F64 ? 1e290 : 1e37))) return 0;
    const double mx = meta[KNN_META_MAXABS];
    const double rg = meta[KNN_META_MAXPOS] + meta[KNN_META_MAXNEG];
    if (!(rg <= 255.0)) return 0;
    if (dtype == KNN_F64) return mx * mx <= 2251799813685248.0 / (4.0 * (double)n);
    return (double)n * mx * mx <= 8388608.0 && (double)n * rg * rg <= 16777216.0;
}

/* the speculative byte block (x - 128) is the one the int8 path would build:
 * int8-eligible data whose values all lie in [0, 255] (o = 128 - max(-x)+ =
 * 128) */
int knn_s8_spec_ok(const double *h_meta, size_t n, int dtype)
{
    const char *no_i8 = getenv("KNN_NO_I8");   /* the int8 path switched off (knn_ctx_begin_meta) */
    if (no_i8 && no_i8[0] == '1') return 0;
    return h_meta && dtype_ok(dtype) && knn_i8_exact(h_meta, n, dtype) && h_meta[KNN_META_MAXNEG] == 0.0 &&
           h_meta[KNN_META_MAXPOS] <= 255.0;
}

static int env_on(const char *name)
{
    const char *e = getenv(name);
    return e && e[0] == '1';
}

/* The split fp16 filter serves searches in GEMM mode (knn_mode: finite,
 * norms in range, not the exact-integer INT mode, whose filter must be
 * exact), fp32 and fp64 blocks.  Returns the pre-scale S = 2^(14 - e) with maxabs in
 * [2^(e-1), 2^e), so maxabs S in [2^13, 2^14) fits fp16 with room, or 0
 * when the filter does not apply (S^2 must stay well inside fp32, and the
 * epilogue's -2 / S^2 too). */
static float knn_split_scale(const double *meta, size_t n, int dtype)
{
    const double mx = meta[KNN_META_MAXABS];
    if (dtype == KNN_F32) {
        const double rg = meta[KNN_META_MAXPOS] + meta[KNN_META_MAXNEG];
        if (meta[KNN_META_NONFINITE] != 0.0 || !(meta[KNN_META_MAXNORM] < 1e37)) return 0.f;   /* SCAN */
        if (meta[KNN_META_NONINT] == 0.0 && (double)n * mx * mx <= 8388608.0 && (double)n * rg * rg <= 16777216.0)
            return 0.f;   /* INT mode */
    } else {
        if (meta[KNN_META_NONFINITE] != 0.0 || !(meta[KNN_META_MAXNORM] < 1e290)) return 0.f;   /* SCAN */
        if (meta[KNN_META_NONINT] == 0.0 && mx * mx <= 2251799813685248.0 / (4.0 * (double)n))
            return 0.f;   /* INT mode */
    }
    if (!(mx > 0.0)) return 0.f;
    int e = 0;
    (void)frexp(mx, &e);
    if (e < -40 || e > 40) return 0.f;
    return (float)ldexp(1.0, 14 - e);
}

/* d_s8: the query block as a byte block already (knn_block_pack_s8, valid by
 * knn_s8_spec_ok); d_qblock is then NULL until knn_ctx_attach_qblock */
static int ctx_begin(knn_ctx_t *c, const void *d_qblock, const void *d_s8, size_t q_cap, size_t q_base,
                     const double *d_meta, const double *h_meta, void *stream)
{
    HIPCHK(hipSetDevice(c->device));
    c->qblk = d_qblock;
    c->q8 = NULL;
    c->q_base = q_base;
    c->q_rows_pad = knn_rows_pad(q_cap);
    c->meta = d_meta;
    c->first_step = 1;
    c->ended = 0;
    if (c->solo_on) {   /* (a search abandoned before its end) */
        c->ms = c->ms_keep;
        c->solo_on = 0;
    }
    c->nstep = 0;
    c->pend = 0;
    c->pend_nsplit = 0;
    c->pend2 = 0;
    c->even_nsplit = 0;
    c->merged = 0;
    c->nfail = 0;
    c->h16 = 0;
    c->i8 = 0;
    /* the contraction for this search from the reduced meta: int8 MFMA on
     * byte blocks, else fp16 MFMA, when exact for the data (KNN_NO_I8=1 /
     * KNN_NO_H16=1 disable them).  A caller that holds the host copy of
     * the meta (the ring drivers, after their all-reduce) passes it; else
     * one 64-byte read. */
    const int no_i8 = env_on("KNN_NO_I8"), no_h16 = env_on("KNN_NO_H16"), no_split = env_on("KNN_NO_SPLIT");
    c->split = 0;
    c->sscale = 0.f;
    c->have_hmeta = 0;
    c->one_block_q8 = 0;
    c->ord_ready = 0;
    if (!(no_i8 && no_h16 && no_split)) {
        double hm[KNN_META_DOUBLES];
        if (!h_meta) {
            HIPCHK(hipMemcpyAsync(hm, d_meta, sizeof(hm), hipMemcpyDeviceToHost, (hipStream_t)stream));
            HIPCHK(hipStreamSynchronize((hipStream_t)stream));
            h_meta = hm;
        }
        memcpy(c->hmeta, h_meta, sizeof(c->hmeta));
        c->have_hmeta = 1;
        c->i8 = !no_i8 && knn_i8_exact(h_meta, c->n, c->dtype);
        if (d_s8 && !c->i8) return KNN_ERR_INVALID;
        c->h16 = !c->i8 && !no_h16 && knn_h16_exact(h_meta, c->n, c->dtype);
        if (!c->i8 && !c->h16 && !no_split) {
            c->sscale = knn_split_scale(h_meta, c->n, c->dtype);
            c->split = c->sscale > 0.f;
        }
    }
    /* int8 lane lists: 12 entries (k <= 32), 17 on request (KNN_I8_KL=17),
     * 65 in the re-search sub-context */
    c->klx = c->i8 ? (c->sub_research ? KNN_I8_KL_L : knn_i8_kl(c->kp)) : c->kl;
    if (c->i8 && !c->sub_research && c->klx == KNN_I8_KL_S && getenv("KNN_I8_KL") && atoi(getenv("KNN_I8_KL")) == KNN_I8_KL)
        c->klx = KNN_I8_KL;
    /* 12-entry lists run on 64-row half tiles, two workgroups a CU (2 lists a
     * query) */
    c->lpq = c->i8 ? (c->sub_research ? 2 : knn_i8_lpq(c->kp, c->klx)) : 4;
    c->i8_wgpc = c->i8 && c->klx == KNN_I8_KL_S && c->lpq == 2 ? 2 : 1;
    /* fp16 shadow rows of the query block (KNN_NO_SHADOW=1: convert the
     * element fragments in the kernel instead) */
    c->shadow = c->i8 ? 2 : (c->h16 && !env_on("KNN_NO_SHADOW"));
    if (c->i8 && d_s8) {
        c->q8 = d_s8;   /* the caller's byte block: no conversion */
    } else if (c->i8) {
        const size_t need = knn_s8_bytes(q_cap, c->n);
        if (need > c->qs8_bytes) {
            HIPCHK(hipStreamSynchronize((hipStream_t)stream));
            hipFree(c->qs8);
            c->qs8 = NULL;
            c->qs8_bytes = 0;
            if (hipMalloc(&c->qs8, need) != hipSuccess) return KNN_ERR_NOMEM;
            c->qs8_bytes = need;
        }
        RCHK(knn_launch_shadow8(c->qs8, d_qblock, c->dtype, c->q_rows_pad, c->n, d_meta, stream));
        c->q8 = c->qs8;
    } else if (c->split) {
        const size_t need = c->q_rows_pad * knn_split_rs(c->n);
        if (need > c->qsp_bytes) {
            HIPCHK(hipStreamSynchronize((hipStream_t)stream));
            hipFree(c->qsp);
            c->qsp = NULL;
            c->qsp_bytes = 0;
            if (hipMalloc(&c->qsp, need) != hipSuccess) return KNN_ERR_NOMEM;
            c->qsp_bytes = need;
        }
        RCHK(knn_launch_shadow_split(c->qsp, d_qblock, c->dtype, c->q_rows_pad, c->n, c->sscale, stream));
    } else if (c->shadow) {
        const size_t need = c->q_rows_pad * knn_round_up(c->n, 64) * 2;
        if (need > c->qsh_bytes) {
            HIPCHK(hipStreamSynchronize((hipStream_t)stream));
            hipFree(c->qsh);
            c->qsh = NULL;
            c->qsh_bytes = 0;
            if (hipMalloc(&c->qsh, need) != hipSuccess) return KNN_ERR_NOMEM;
            c->qsh_bytes = need;
        }
        RCHK(knn_launch_shadow(c->qsh, d_qblock, c->dtype, c->q_rows_pad, c->n, stream));
    }
    /* fail_count and mode_dev are one allocation: one launch resets both,
     * the bounds and (int8: 0x7f7f7f7f, above every int8-mode d^2 -- an
     * empty summary) the cross-split summaries */
    RCHK(knn_launch_begin_init(c->qthr, c->i8 ? c->qsum : NULL, (int)c->nq_pad, c->fail_count, stream));
    return KNN_OK;
}

int knn_ctx_begin_meta(knn_ctx_t *c, const void *d_qblock, size_t q_cap, size_t q_base,
                       const double *d_meta, const double *h_meta, void *stream)
{
    if (!c || !d_qblock || !d_meta || q_cap < c->nq) return KNN_ERR_INVALID;
    return ctx_begin(c, d_qblock, NULL, q_cap, q_base, d_meta, h_meta, stream);
}

int knn_ctx_begin_s8(knn_ctx_t *c, const void *d_sblock, size_t q_cap, size_t q_base, const double *d_meta,
                     const double *h_meta, void *stream)
{
    if (!c || !d_sblock || !d_meta || !h_meta || q_cap < c->nq) return KNN_ERR_INVALID;
    if (!knn_s8_spec_ok(h_meta, c->n, c->dtype) || env_on("KNN_NO_I8")) return KNN_ERR_INVALID;
    return ctx_begin(c, NULL, d_sblock, q_cap, q_base, d_meta, h_meta, stream);
}

int knn_ctx_attach_qblock(knn_ctx_t *c, const void *d_qblock, size_t q_cap)
{
    if (!c || !d_qblock || knn_rows_pad(q_cap) != c->q_rows_pad) return KNN_ERR_INVALID;
    c->qblk = d_qblock;
    return KNN_OK;
}

int knn_ctx_begin(knn_ctx_t *c, const void *d_qblock, size_t q_cap, size_t q_base,
                  const double *d_meta, void *stream)
{
    return knn_ctx_begin_meta(c, d_qblock, q_cap, q_base, d_meta, NULL, stream);
}

size_t knn_ctx_shadow_bytes(const knn_ctx_t *c, size_t cap)
{
    if (!c) return 0;
    if (c->shadow == 2) return knn_s8_bytes(cap, c->n);
    if (c->shadow == 1) return knn_shadow_bytes(cap, c->n, c->dtype);
    return 0;
}

int knn_ctx_shadow_pack(knn_ctx_t *c, void *d_sblock, const void *d_block, size_t cap, void *stream)
{
    if (!c || !d_sblock || !d_block || cap == 0) return KNN_ERR_INVALID;
    if (c->shadow == 1) return knn_shadow_pack(d_sblock, d_block, cap, c->n, c->dtype, stream);
    if (c->shadow != 2) return KNN_ERR_INVALID;
    HIPCHK(hipSetDevice(c->device));
    const size_t rp = knn_rows_pad(cap);
    if (d_block == c->qblk && rp == c->q_rows_pad && c->q8) {
        /* the query block (a ring's own block): begin converted it already */
        HIPCHK(hipMemcpyAsync(d_sblock, c->q8, knn_s8_meta_offset(cap, c->n), hipMemcpyDeviceToDevice,
                              (hipStream_t)stream));
    } else {
        RCHK(knn_launch_shadow8(d_sblock, d_block, c->dtype, rp, c->n, c->meta, stream));
    }
    HIPCHK(hipMemcpyAsync((char *)d_sblock + knn_s8_meta_offset(cap, c->n),
                          (const char *)d_block + knn_block_meta_offset_dt(cap, c->n, c->dtype),
                          KNN_META_DOUBLES * sizeof(double), hipMemcpyDeviceToDevice,
                          (hipStream_t)stream));
    return KNN_OK;
}

/* bytes of partial lists per corpus split (k_dist_topk -> k_merge) */
static size_t split_bytes(const knn_ctx_t *c)
{
    return c->nq_pad * ((size_t)c->lpq * c->klx * (sizeof(double) + sizeof(int)) + sizeof(double));
}

#define KNN_PART_BUDGET ((size_t)2 << 30) /* partial-list bytes above one split */

/* Makespan of one k_dist_topk launch, in tile times: nqb*nsplit workgroups
 * in split-major order (long splits first, knn_kernels.hip), each costing
 * its tiles plus KNN_WG_COST; workgroup i goes to XCD i % 8 and there to the
 * first free CU (one 512-thread workgroup per CU).  Large grids use the
 * list-scheduling bound instead of the simulation. */
#define KNN_XCDS 8
#define KNN_WG_COST 0.5        /* prologue + partial-list flush, in tiles   */
/* int8 kernel: a workgroup's fixed cost (query fragments into VGPRs, ring
 * fill, warming 512 empty lane lists, the flush) is ~60 K-step tiles'
 * worth: tile time scales with the K-steps, the fixed cost does not.
 * Calibrated on the emulated ring (tools/ring_emulate.py, KNN_SPLITS sweeps):
 * mnist P = 2 / 4 / 8 best at 1-3 / 1-2 / 4 splits, sift P = 4 / 8 at 1. */
#define KNN_WG_COST_I8_KSTEPS 60.0
/* k_merge per (query, split), in tile times: the GEMM merge re-ranks with
 * exact S, ~4.3 ns a (query, split) against a 27 us split-fp16 tile
 * (emulated mnist-real P = 2: 4 / 13 splits 1.03 / 2.19 ms of exposed
 * merge; 1e-6 here had the model pick 13 splits at P = 2 and 4, where 4-6
 * run 6-7% faster) */
#define KNN_MERGE_COST 1.6e-4
/* int8 kernel: k_merge's exposed time grows ~1.2e-4 tile times per (query,
 * split) (emulated P = 8 fused launch: 13 splits 0.10 ms against 4 splits
 * 0.06 ms of exposed merge at 7500 queries) */
#define KNN_MERGE_COST_I8 1.2e-4
static double launch_makespan(long nqb, long ntiles, int s, int cus, double wgc)
{
    const long tb = ntiles / s, tr = ntiles % s;
    const long w = nqb * s;
    const int per = cus / KNN_XCDS > 0 ? cus / KNN_XCDS : 1;
    if (w > 16L * cus || per > 64) {
        const double work = (double)nqb * ntiles + wgc * w;
        return work / cus + (tb + (tr ? 1 : 0)) + wgc;
    }
    double ms = 0.0;
    for (int x = 0; x < KNN_XCDS; x++) {
        double cu[64] = {0};
        for (long i = x; i < w; i += KNN_XCDS) {
            const long split = i / nqb;
            int best = 0;
            for (int u = 1; u < per; u++)
                if (cu[u] < cu[best]) best = u;
            cu[best] += (double)(tb + (split < tr ? 1 : 0)) + wgc;
        }
        for (int u = 0; u < per; u++)
            if (cu[u] > ms) ms = cu[u];
    }
    return ms;
}

/* remember a choose_splits result under every input it depends on */
static int split_cache_put(knn_ctx_t *c, size_t nc, int best)
{
    const int e = c->split_next++ % KNN_SPLIT_CACHE;
    c->split_cache[e].nc = nc;
    c->split_cache[e].lpq = c->lpq;
    c->split_cache[e].i8 = c->i8;
    c->split_cache[e].split = c->split;
    c->split_cache[e].solo = c->split_solo;
    c->split_cache[e].klx = c->klx;
    c->split_cache[e].best = best;
    return best;
}

/* the distance launch's workgroup order (c->xord, -1 = by the launch) */
static int xord_for(const knn_ctx_t *c, int nsplit)
{
    return c->xord >= 0 ? c->xord : (c->split && nsplit <= 2);
}

/* Corpus splits per query block: the count with the smallest modelled
 * launch makespan plus merge cost (each split adds a partial list per
 * query), keeping >= 4 tiles per split and the partial lists within
 * KNN_PART_BUDGET.  Cached per (corpus block size, lists a query, kernel
 * -- int8, split filter (256-row tiles) or other (128-row tiles) --,
 * own-block step, lane-list length): each of these changes the model. */
static int choose_splits(knn_ctx_t *c, size_t nc)
{
    const char *env = getenv("KNN_SPLITS");
    /* (workgroups of 128 qg queries: knn_i8_qg) */
    const long qpw = (long)KNN_TQ * (c->i8 ? knn_i8_qg(c->klx, c->lpq, c->n) : 1);
    const long nqb = (long)((c->nq + qpw - 1) / qpw);
    /* k_dist_split streams 256-row tiles: the model's tile unit is its tile */
    const long tc = c->split ? KNN_SPLIT_TC : KNN_TC;
    const long ntiles = (long)((nc + tc - 1) / tc);
    /* the re-search of a few uncertified queries: one query block, so the
     * launch's span is one workgroup's scan -- as many splits as the merge
     * takes (lpq * splits + 1 <= 64 lists) */
    if (c->sub_research) {
        const int sw = KNN_MAX_LISTS / c->lpq;
        return ntiles < sw ? (ntiles > 0 ? (int)ntiles : 1) : sw;
    }
    if (env && atoi(env) > 0) {   /* (the search's splits, not the re-search's) */
        int s = atoi(env);
        if (s > KNN_MAX_LISTS / c->lpq) s = KNN_MAX_LISTS / c->lpq;
        /* k_dist_split needs a tile a split (knn_launch_dist_split refuses
         * fewer): a small block takes fewer splits than asked */
        if (c->split && s > ntiles) s = ntiles > 0 ? (int)ntiles : 1;
        return s;
    }
    for (int e = 0; e < KNN_SPLIT_CACHE; e++)
        if (c->split_cache[e].best > 0 && c->split_cache[e].nc == nc && c->split_cache[e].lpq == c->lpq &&
            c->split_cache[e].i8 == c->i8 && c->split_cache[e].split == c->split &&
            c->split_cache[e].solo == c->split_solo && c->split_cache[e].klx == c->klx)
            return c->split_cache[e].best;
    int smax = KNN_MAX_LISTS / c->lpq;
    const size_t per = split_bytes(c);
    if (per > 0 && KNN_PART_BUDGET / per < (size_t)smax)
        smax = KNN_PART_BUDGET / per > 1 ? (int)(KNN_PART_BUDGET / per) : 1;
    const double wgc = c->i8 ? KNN_WG_COST_I8_KSTEPS / (double)(knn_s8_rs(c->n) / 32) : KNN_WG_COST * KNN_TC / tc;
    /* half-tile int8 kernel: two workgroups a CU, each at about half the
     * rate -- the model's slots double and its tile unit (a workgroup's
     * tile time) with them, so the merge term, priced in tile times, halves */
    const int slots = c->cus * (c->i8 ? c->i8_wgpc : 1);
    const double mc = (c->i8 ? KNN_MERGE_COST_I8 : KNN_MERGE_COST * KNN_TC / tc) / (c->i8 ? c->i8_wgpc : 1);
    /* int8 lists: at least s_min splits so that a lane list expects <= KL/3
     * of the query's k+1 nearest (lpq lists a split; the block may hold all
     * of them): one split of 17-entry lists over a whole corpus left
     * ~1e-3 of the queries uncertified (a lane list held 17 of the k) */
    int s_min = 1;
    if (c->i8) {
        /* the half-tile kernel's 2 lists a split see twice the rows a lane (long rows):
         * it takes 5(k+1)/KL lists a query (MNIST P = 1, uncertified
         * queries a pass: 58 at 4 splits, 2 at 6, 0 at 7; SIFT 334 at 5) */
        /* (in halves) short rows on the two-group kernel folding the own
         * query block: 2.5 (k+1)/KL -- a P = 1 search's uncertified
         * queries go to the int8 re-search (SIFT P = 1 emulated: 4 splits
         * 167.5 ms, 5 splits 170.3 ms, both 0 uncertified after it; a
         * ring's fused launch keeps 3: at P = 8 4 splits left 192 a pass
         * for the rescan, 5 splits 27) */
        const int kl = c->klx;
        const int f2 = (c->i8_wgpc == 2 && knn_s8_rs(c->n) / 32 > 8)
                           ? 10
                           : (c->split_solo && knn_i8_qg(c->klx, c->lpq, c->n) == 2 ? 5 : 6);
        s_min = (f2 * (c->k + 1) + 2 * c->lpq * kl - 1) / (2 * c->lpq * kl);
        if (s_min > smax) s_min = smax;
        if (s_min < 1) s_min = 1;
    }
    int best = s_min;
    double best_t = 0.0;
    /* short rows (<= 8 K-steps a tile: SIFT's n = 128) with a full grid at
     * s_min: s_min.  The per-tile epilogue outweighs the contraction there
     * and every extra split is another set of cold lane lists (emulated
     * sift P = 8 fused launch: 3 / 4 / 6 / 9 splits 38.2 / 38.9 / 40.2 /
     * 42.7 ms; the makespan model picked 9) */
    const int short_rows = c->i8 && knn_s8_rs(c->n) / 32 <= 8 && nqb * s_min >= slots;
    /* half-tile kernel, long rows, a grid of several rounds at s_min: s_min.
     * Measured (MNIST P = 1, kernel / step ms): 7 splits 3.17 / 3.47, 12
     * splits 3.18 / 3.55 -- the makespan model's tail estimate (12 ahead of
     * 7) does not hold with two workgroups a CU, and every split adds merge
     * work and a set of cold lists.  A single round (a ring rank's fused
     * launch) still takes the model: P = 8 6 / 7 / 8 splits 0.75 / 0.69 /
     * 0.67 ms a rank, the model's 8 */
    if (c->i8 && c->i8_wgpc == 2 && !short_rows && nqb * s_min >= slots) {
        best = s_min;
        /* between one and two rounds at s_min (a P = 4 rank's launches:
         * 118 query blocks x 7 splits on 512 slots), one full round wins
         * when its lane lists stay short enough (<= 6000 rows a list; MNIST
         * P = 1 left 2 queries uncertified at 5000, 58 at 7500): emulated
         * P = 4 rank 4 / 5 / 7 / 9 splits 1.121 / 1.233 / 1.187 / 1.193 ms */
        const long s1 = slots / nqb;
        if (nqb * s_min < 2L * slots && s1 >= 1 && s1 < s_min &&
            (double)nc / ((double)s1 * c->lpq) <= 6000.0)
            best = (int)s1;
        return split_cache_put(c, nc, best);
    }
    for (int s = s_min; s <= smax && !short_rows; s++) {
        if (s > s_min && ntiles / s < 4) break;
        const double t = launch_makespan(nqb, ntiles, s, slots, wgc) + mc * (double)c->nq * s;
        if (s == s_min || t < best_t * (1.0 - 2e-3)) {
            best = s;
            best_t = t;
        }
    }
    return split_cache_put(c, nc, best);
}

/* Partial lists of set `set` for nsplit splits.  Even set: the pair
 * allocation grows to 2*nsplit splits (room for an odd step of the same
 * size behind it).  Odd set: right behind the even set's `off` splits,
 * growing the allocation only when nothing in it is pending. */
static int ensure_part_buffers(knn_ctx_t *c, int nsplit, int set, int off)
{
    const int pr = set >> 1;
    const int need = (set & 1) ? off + nsplit : 2 * nsplit;
    const size_t per = c->nq_pad * (size_t)c->lpq * c->klx;
    if (per != c->pp_per[pr]) {
        /* list shape changed (another kernel): the old sets hold nothing pending */
        if (c->pend) return KNN_ERR_INVALID;
        if (c->pp_cap[pr]) HIPCHK(hipStreamSynchronize(c->ms));
        hipFree(c->pp_d[pr]);
        hipFree(c->pp_i[pr]);
        hipFree(c->pp_T[pr]);
        c->pp_d[pr] = NULL;
        c->pp_i[pr] = NULL;
        c->pp_T[pr] = NULL;
        c->pp_cap[pr] = 0;
        c->pp_per[pr] = per;
    }
    if (need > c->pp_cap[pr]) {
        if ((set & 1) && c->pend) return KNN_ERR_INVALID;   /* caller merges first */
        /* the pair may still be read by an earlier step's merge */
        HIPCHK(hipStreamSynchronize(c->ms));
        hipFree(c->pp_d[pr]);
        hipFree(c->pp_i[pr]);
        hipFree(c->pp_T[pr]);
        c->pp_d[pr] = NULL;
        c->pp_i[pr] = NULL;
        c->pp_T[pr] = NULL;
        c->pp_cap[pr] = 0;
        const int cap = need > 2 * nsplit ? need : 2 * nsplit;
        if (hipMalloc((void **)&c->pp_d[pr], (size_t)cap * per * sizeof(double)) != hipSuccess ||
            hipMalloc((void **)&c->pp_i[pr], (size_t)cap * per * sizeof(int)) != hipSuccess ||
            hipMalloc((void **)&c->pp_T[pr], (size_t)cap * c->nq_pad * sizeof(double)) != hipSuccess)
            return KNN_ERR_NOMEM;
        c->pp_cap[pr] = cap;
    }
    const int o = (set & 1) ? off : 0;
    c->part_d[set] = c->pp_d[pr] + (size_t)o * per;
    c->part_i[set] = c->pp_i[pr] + (size_t)o * per;
    c->part_T[set] = c->pp_T[pr] + (size_t)o * c->nq_pad;
    return KNN_OK;
}

/* k_merge of `nsets` consecutive steps' lists (1, or 2 = a pending even
 * step and the odd step behind it) starting at set `set`, on ms after
 * their distance kernels; records ev_m of every covered set. */
static int rank_merge_ok(const knn_ctx_t *c, int nsplit_total)
{
    return c->i8 && c->kp <= KNN_KP_M && (c->klx == KNN_I8_KL_S || c->klx == KNN_I8_KL) &&
           c->lpq * nsplit_total <= 64;
}

/* The GEMM-mode merge reads each window candidate's element row at random
 * (exact S); past the Infinity Cache (a block of more than 64 MB) it merges
 * the queries in the order of knn_order.hip, so that near queries -- which
 * share their candidates -- run together (KNN_ORDER=1 forces it,
 * KNN_NO_ORDER=1 disables it; results do not depend on it). */
static int want_order(const knn_ctx_t *c, size_t nc)
{
    if (c->i8 || c->h16 || env_on("KNN_NO_ORDER")) return 0;
    if (env_on("KNN_ORDER")) return 1;
    const size_t bytes = nc * knn_n_pad_dt(c->n, c->dtype) * knn_esize(c->dtype);
    return c->nq >= 8192 && bytes > ((size_t)64 << 20);
}

static int find_order(knn_ctx_t *c, int set, int nsplit)
{
    if (c->ord_cap < c->nq_pad) {
        hipFree(c->ord_lab);
        hipFree(c->ord_keys);
        hipFree(c->ord_iota);
        hipFree(c->ord_perm);
        hipFree(c->ord_tmp);
        c->ord_lab = c->ord_keys = c->ord_iota = c->ord_perm = NULL;
        c->ord_tmp = NULL;
        c->ord_cap = 0;
        const size_t b = c->nq_pad * sizeof(int);
        c->ord_tmp_bytes = knn_order_tmp_bytes((int)c->nq_pad);
        if (hipMalloc((void **)&c->ord_lab, b) != hipSuccess || hipMalloc((void **)&c->ord_keys, b) != hipSuccess ||
            hipMalloc((void **)&c->ord_iota, b) != hipSuccess || hipMalloc((void **)&c->ord_perm, b) != hipSuccess ||
            hipMalloc(&c->ord_tmp, c->ord_tmp_bytes ? c->ord_tmp_bytes : 16) != hipSuccess)
            return KNN_ERR_NOMEM;
        c->ord_cap = c->nq_pad;
    }
    /* 4 rounds: labels settle to cluster-sized pieces (pointer jumping
     * halves the distance to the piece's minimum each round) */
    RCHK(knn_launch_order(c->part_i[set], nsplit, c->lpq, c->klx, (int)c->nq, (int)c->nq_pad,
                          (long long)c->q_base, 4, c->ord_lab, c->ord_keys, c->ord_iota, c->ord_perm, c->ord_tmp,
                          c->ord_tmp_bytes, c->ms));
    c->ord_ready = 1;
    return KNN_OK;
}

/* fin_out: the search's last merge -- with the rank merge it finalizes
 * too (records into fin_out, *finalized = 1) */
static int launch_merge_sets_fin(knn_ctx_t *c, int set, int nsets, int nsplit_total, const void *cblk,
                                 size_t c_base, size_t nc, knn_neighbour_t *fin_out, int *finalized)
{
    if (finalized) *finalized = 0;
    hipEvent_t *mk = NULL;
    const int rank_merge = rank_merge_ok(c, nsplit_total);
    if (c->prof_on && c->prof_mk_pending < KNN_PROF_STEPS) {
        mk = &c->prof_mk_ev[2 * c->prof_mk_pending++];
        HIPCHK(hipEventRecord(mk[0], c->ms));
        /* the merge's algorithmic bytes: every partial list entry (d^2 as
         * fp64 + idx) and bound read, the old state read and the new one
         * written (KP x (d^2, S, idx) + 2 bounds), or with a finalizing rank
         * merge the k records; GEMM mode adds the exact re-rank's rows --
         * each query's row and its k neighbours' rows, the reads the
         * reference-order S of the reported neighbours cannot avoid */
        const double nq = (double)c->nq;
        const double es = c->dtype == KNN_F64 ? 8.0 : 4.0;
        double b = nq * (double)nsplit_total * ((double)c->lpq * c->klx * 12.0 + 8.0);
        if (c->merged) b += nq * ((double)c->kp * 20.0 + 16.0);
        b += (rank_merge && fin_out) ? nq * (double)c->k * 16.0 : nq * ((double)c->kp * 20.0 + 16.0);
        /* (GEMM mode: the split filter's searches always; otherwise the
         * previous search's mode, c->mode being set at knn_ctx_end) */
        if ((c->split || c->mode == KNN_MODE_GEMM) && !rank_merge)
            b += nq * (double)(c->k + 1) * (double)c->n * es;
        c->prof_mk_bytes += b;
    }
    /* int8 lists (exact INT-mode keys, k <= 32): the rank merge */
    if (rank_merge) {
        RCHK(knn_launch_merge_rank(c->dtype, c->kp, c->klx, c->k, c->part_d[set], c->part_i[set], c->part_T[set],
                                   nsplit_total, c->lpq, (int)c->nq, (int)c->nq_pad, !c->merged, c->st_d,
                                   c->st_x, c->st_i, c->st_T, c->qthr, fin_out, c->fail_count, c->fail_list,
                                   c->mode_dev, c->fbound, c->meta, (int)c->n, env_on("KNN_FORCE_RESCAN"), c->ms));
        if (fin_out && finalized) *finalized = 1;
    } else {
        const int *perm = NULL;
        if (want_order(c, nc)) {
            if (!c->ord_ready) RCHK(find_order(c, set, nsplit_total));
            perm = c->ord_perm;
        }
        RCHK(knn_launch_merge(c->dtype, c->kp, c->k, c->part_d[set], c->part_i[set], c->part_T[set],
                              nsplit_total, c->lpq, c->klx, (int)c->nq, (int)c->nq_pad, !c->merged, c->st_d, c->st_x,
                              c->st_i, c->st_T, c->qblk, c->q_rows_pad, cblk, c_base, (int)nc, (int)c->n,
                              c->meta, c->qthr, c->split, perm, c->ms));
    }
    if (mk) HIPCHK(hipEventRecord(mk[1], c->ms));
    c->merged = 1;
    /* (the search's last merge: nothing waits on its sets -- an event
     * record is one more packet on the queue before the read-back) */
    if (!(finalized && *finalized))
        for (int x = 0; x < nsets; x++) HIPCHK(hipEventRecord(c->ev_m[(set + x) % KNN_PSETS], c->ms));
    return KNN_OK;
}

static int launch_merge_sets(knn_ctx_t *c, int set, int nsets, int nsplit_total, const void *cblk,
                             size_t c_base, size_t nc)
{
    return launch_merge_sets_fin(c, set, nsets, nsplit_total, cblk, c_base, nc, NULL, NULL);
}

/* the deferred merge of a fused step and its pending partner */
static int flush_pend2(knn_ctx_t *c, knn_neighbour_t *fin_out, int *finalized)
{
    if (finalized) *finalized = 0;
    if (!c->pend2) return KNN_OK;
    c->pend2 = 0;
    RCHK(launch_merge_sets_fin(c, c->pend2_set, 2, c->pend2_nsplit, NULL, 0, 0, fin_out, finalized));
    for (int x = 0; x < 2; x++)
        if (c->pend2_ev[x]) HIPCHK(hipEventRecord(c->pend2_ev[x][2], c->ms));
    return KNN_OK;
}

/* merge the pending even step by itself */
static int merge_pending_fin(knn_ctx_t *c, knn_neighbour_t *fin_out, int *finalized)
{
    if (finalized) *finalized = 0;
    if (!c->pend) return KNN_OK;
    c->pend = 0;
    RCHK(launch_merge_sets_fin(c, c->pend_set, 1, c->pend_nsplit, c->pend_cblk, c->pend_cbase,
                               (size_t)c->pend_nc, fin_out, finalized));
    if (c->pend_ev) HIPCHK(hipEventRecord(c->pend_ev[2], c->ms));
    return KNN_OK;
}

static int merge_pending(knn_ctx_t *c) { return merge_pending_fin(c, NULL, NULL); }

/* Step schedule.  Step s runs k_dist_topk on stream ds[s % 2] into partial
 * set p = s % 4 and k_merge on stream ms (high priority), in step order:
 *   ds[s%2]: wait ev_in (the caller's stream at this call: the block has
 *            arrived, begin() is done) and ev_m[p] (merge s-4 has read the
 *            partial set), then k_dist_topk(s)              -> ev_ds[p]
 *   ms:      wait ev_ds[p] (implies ev_in), then k_merge(s) -> ev_m[p]
 *   caller:  wait ev_m[(s-2)%4] (step s-2 has finished reading its block);
 *            exact-integer contractions (int8 / fp16: k_merge never reads
 *            block rows) wait ev_ds[(s-2)%4], k_dist_topk(s-2) alone, so
 *            no merge sits on the chain that gates the next blocks
 * so k_dist_topk(s) starts while k_dist_topk(s-1) drains its last
 * workgroups -- a ring step no longer pays its launch tail -- and the
 * merges (which co-reside with the distance workgroups and so stretch
 * over the next contraction) have two steps of slack before anything waits
 * on them.  The caller's stream lags KNN_STEP_LAG = 2 steps: work it
 * enqueues after step s returns is ordered after step s-2 only, so a ring
 * rotates KNN_STEP_LAG + 2 receive buffers (knn.h).  knn_ctx_end joins
 * all. */
/* d_sblock: a shadow block (knn_shadow_pack) used in place of d_cblock.
 * xb (int8 contraction only, byte blocks): further byte blocks folded by the
 * same launch -- xb->ptr[0..nblk) with the rows / bases beside them, in any
 * order (sorted here); d_sblock / nc / c_base then unused. */
static int ctx_step_impl(knn_ctx_t *c, const void *d_cblock, const void *d_sblock, size_t nc,
                         size_t c_base, const knn_i8_blocks_t *xb, void *stream)
{
    knn_i8_blocks_t tab;
    memset(&tab, 0, sizeof(tab));
    if (xb) {
        if (!c || !c->i8 || xb->nblk < 1 || xb->nblk > KNN_I8_MAXBLK) return KNN_ERR_INVALID;
        /* ascending bases (insertion sort, <= 8 entries) */
        for (int b = 0; b < xb->nblk; b++) {
            if (!xb->ptr[b] || xb->nc[b] <= 0 || (size_t)xb->nc[b] > c->block_cap || xb->base[b] < 0)
                return KNN_ERR_INVALID;
            int j = tab.nblk++;
            while (j > 0 && tab.base[j - 1] > xb->base[b]) {
                tab.ptr[j] = tab.ptr[j - 1];
                tab.nptr[j] = tab.nptr[j - 1];
                tab.base[j] = tab.base[j - 1];
                tab.nc[j] = tab.nc[j - 1];
                j--;
            }
            tab.ptr[j] = xb->ptr[b];
            tab.nptr[j] = xb->nptr[b];
            tab.base[j] = xb->base[b];
            tab.nc[j] = xb->nc[b];
        }
        d_sblock = tab.ptr[0];
        c_base = (size_t)tab.base[0];
        nc = 0;   /* tile-rounded rows of the launch: the split model's input */
        for (int b = 0; b < tab.nblk; b++) nc += knn_round_up((size_t)tab.nc[b], KNN_TC);
        nc -= knn_round_up((size_t)tab.nc[tab.nblk - 1], KNN_TC) - (size_t)tab.nc[tab.nblk - 1];
    } else if (!c || !(d_cblock || d_sblock) || nc == 0 || nc > c->block_cap) {
        return KNN_ERR_INVALID;
    }
    if (d_sblock && !c->shadow) return KNN_ERR_INVALID;
    if (!d_cblock) d_cblock = d_sblock;   /* INT mode: k_merge never reads its rows */
    HIPCHK(hipSetDevice(c->device));
    RCHK(flush_pend2(c, NULL, NULL));   /* a deferred merge goes first, in step order */
    c->split_solo = c->i8 && c->nstep == 0 && !xb && d_sblock != NULL && d_sblock == c->q8 && nc == c->nq;
    int nsplit = choose_splits(c, nc);
    const int set = c->nstep % KNN_PSETS, ds_i = c->nstep & 1;
    c->nsplit_last = nsplit;
    /* pairing: in exact-integer (fp16) searches two consecutive steps share
     * one k_merge (8*nsplit + 1 <= 64 lists; INT mode never reads the
     * block rows in k_merge) -- half the merges, which at P = 8 cost about
     * as much as the contraction. */
    const int can_pair = (c->h16 || c->i8) && 2 * c->lpq * nsplit + 1 <= 64;
    /* a fused step behind a pending single-block step (the direct exchange:
     * own block, then the received ones) shares its merge when the lists fit
     * one merge wave: the own block's merge could not run beside the fused
     * launch anyway (every CU holds a distance workgroup; measured: the
     * merge ran on the ~20 CUs the fused launch left idle and ended after
     * it), so pairing drops a launch and its starved tail */
    const int pair_fused = xb && c->pend && (set & 1) && c->lpq * (c->pend_nsplit + nsplit) + 1 <= 64;
    /* a fused step (the direct exchange's received blocks) is never paired:
     * the previous step's merge runs beside it and publishes the (k+1)-th
     * d^2 of the blocks folded so far into qthr, which the fused launch's
     * workgroups re-read as they go (k_dist_topk_i8), so most of the rank's
     * work filters with the running answer instead of cold lane lists
     * (making the launch wait for that merge measured no faster, DESIGN.md
     * sec.5). */
    /* a split-filter (GEMM) search's first step on its own query block keeps
     * its merge pending: the direct exchange's fused step (knn_ctx_step_n)
     * merges both in one k_merge over a table of all their blocks -- the
     * own block's merge could not run beside the fused launch anyway (its
     * workgroups hold every register of every CU), so it ran alone after
     * it; any other next step merges it first, as a single merge */
    const int gemm_own = c->split && !xb && c->nstep == 0 && d_cblock == c->qblk;
    int pairing = 0;
    if ((set & 1) && c->pend) {
        pairing = (can_pair && nsplit == c->pend_nsplit && !xb) || pair_fused;
        if (!pairing) RCHK(merge_pending(c));
    }
    {
        if (!(set & 1)) c->even_nsplit = nsplit;
        const int rc0 = ensure_part_buffers(c, nsplit, set, c->even_nsplit);
        if (rc0 == KNN_ERR_INVALID && c->pend) {
            RCHK(merge_pending(c));
            pairing = 0;
            RCHK(ensure_part_buffers(c, nsplit, set, c->even_nsplit));
        } else if (rc0) {
            return rc0;
        }
    }
    const void *cblk = d_cblock;
    hipStream_t cs = (hipStream_t)stream, ds = c->ds[ds_i];
    if (c->solo_on) {
        /* a second step after a solo first one: back to the step schedule
         * (step 0's kernel ran on the caller's stream; its merge is pending
         * and will run on the merge stream) */
        HIPCHK(hipEventRecord(c->ev_ds[0], (hipStream_t)c->ms));
        HIPCHK(hipStreamWaitEvent(c->ms_keep, c->ev_ds[0], 0));
        c->ms = c->ms_keep;
        c->solo_on = 0;
    }
    /* a solo search (one block, one step: P = 1): the distance kernel on the
     * caller's stream, its merge behind it there -- no event record or
     * stream wait between pack, kernel and merge (each a queue packet of
     * 5-20 us, rocprofv3) */
    const int solo = c->solo && c->nstep == 0 && !xb;
    if (solo) {
        ds = cs;
        c->ms_keep = c->ms;
        c->ms = cs;
        c->solo_on = 1;
    } else {
        HIPCHK(hipEventRecord(c->ev_in, cs));
        HIPCHK(hipStreamWaitEvent(ds, c->ev_in, 0));
    }
    if (c->nstep >= KNN_PSETS) HIPCHK(hipStreamWaitEvent(ds, c->ev_m[set], 0));
    const void *csh = d_sblock, *cn_ptr = NULL;
    if (c->i8) {
        if (!d_sblock && d_cblock == c->qblk && knn_rows_pad(c->block_cap) == c->q_rows_pad) {
            csh = c->q8;   /* the query block itself (P = 1): its byte block exists */
        } else if (!d_sblock) {
            if (!c->cs8[set] && hipMalloc(&c->cs8[set], knn_s8_bytes(c->block_cap, c->n)) != hipSuccess)
                return KNN_ERR_NOMEM;
            RCHK(knn_launch_shadow8(c->cs8[set], d_cblock, c->dtype, knn_rows_pad(c->block_cap), c->n,
                                    c->meta, ds));
            csh = c->cs8[set];
        }
    } else if (c->split) {
        if (d_cblock == c->qblk && knn_rows_pad(c->block_cap) == c->q_rows_pad) {
            csh = c->qsp;   /* the query block itself (P = 1) */
        } else {
            const size_t need = knn_rows_pad(c->block_cap) * knn_split_rs(c->n);
            if (need > c->csp_bytes) {
                /* the sets may still be read by earlier steps' kernels */
                HIPCHK(hipDeviceSynchronize());
                for (int b = 0; b < KNN_PSETS; b++) {
                    hipFree(c->csp[b]);
                    c->csp[b] = NULL;
                }
                c->csp_bytes = need;
            }
            if (!c->csp[set] && hipMalloc(&c->csp[set], c->csp_bytes) != hipSuccess) return KNN_ERR_NOMEM;
            RCHK(knn_launch_shadow_split(c->csp[set], d_cblock, c->dtype, knn_rows_pad(nc), c->n, c->sscale, ds));
            csh = c->csp[set];
        }
    } else if (d_sblock) {
        cn_ptr = (const char *)d_sblock + knn_shadow_norm_offset(c->block_cap, c->n);
    } else if (c->shadow && d_cblock == c->qblk && knn_rows_pad(nc) <= c->q_rows_pad) {
        csh = c->qsh;   /* the query block itself (P = 1): its shadow exists */
    } else if (c->shadow) {
        const size_t need = knn_rows_pad(c->block_cap) * knn_round_up(c->n, 64) * 2;
        if (!c->csh[set]) {
            /* first use of this set (hipMalloc may synchronise the device) */
            if (hipMalloc(&c->csh[set], need) != hipSuccess) return KNN_ERR_NOMEM;
        }
        c->csh_bytes = need;
        RCHK(knn_launch_shadow(c->csh[set], d_cblock, c->dtype, knn_rows_pad(nc), c->n, ds));
        csh = c->csh[set];
    }
    hipEvent_t *ev = NULL;
    if (c->prof_on && c->prof_pending < KNN_PROF_STEPS) {
        ev = &c->prof_ev[3 * c->prof_pending++];
        HIPCHK(hipEventRecord(ev[0], ds));
    }
    if (c->i8) {
        c->one_block_q8 = c->nstep == 0 && !xb && csh == c->q8;
        c->step0_nc = nc;
        c->step0_cbase = c_base;
        if (!xb) {
            tab.nblk = 1;
            tab.ptr[0] = csh;
            tab.base[0] = (int64_t)c_base;
            tab.nc[0] = (int)nc;
        }
        RCHK(knn_launch_dist_i8(c->kp, c->klx, c->lpq, c->k, c->q8, c->q_rows_pad, c->q_base, (int)c->nq, &tab,
                                knn_rows_pad(c->block_cap), (int)c->n, nsplit, c->part_d[set],
                                c->part_i[set], c->part_T[set], (int)c->nq_pad, c->qthr,
                                c->qsum, ds));
    } else
        RCHK(knn_launch_dist_topk(c->dtype, c->kp, c->k, c->qblk, c->q_rows_pad, c->q_base, (int)c->nq,
                                  cblk, knn_rows_pad(c->block_cap), c_base, (int)nc, (int)c->n, c->meta,
                                  nsplit, c->part_d[set], c->part_i[set], c->part_T[set], (int)c->nq_pad,
                                  c->qthr, c->split ? c->qsp : c->qsh, csh, cn_ptr,
                                  (xord_for(c, nsplit) ? KNN_DIST_XORD : 0) | (c->h16 ? KNN_DIST_H16 : 0) |
                                      (c->shadow ? KNN_DIST_SHADOW : 0) | (c->split ? KNN_DIST_SPLIT : 0),
                                  c->split ? (float)(-2.0 / ((double)c->sscale * c->sscale)) : -2.f, ds));
    if (ev) HIPCHK(hipEventRecord(ev[1], ds));
    /* one event a step behind its distance kernel (each record is a marker
     * packet on the queue, ~5 us before whatever follows it there): the
     * merge stream, the caller's lag wait and knn_ctx_end all use ev_ds.
     * (The distance kernel waited for ev_in: ev_ds covers the block's
     * arrival too -- a second wait would add its own latency) */
    if (!solo) {
        HIPCHK(hipEventRecord(c->ev_ds[set], ds));
        HIPCHK(hipStreamWaitEvent(c->ms, c->ev_ds[set], 0));
    }
    if (pairing) {
        /* the pending even step (step s - 1, on the other distance stream) */
        HIPCHK(hipStreamWaitEvent(c->ms, c->ev_ds[(set + KNN_PSETS - 1) % KNN_PSETS], 0));
        c->pend = 0;
        if (xb && rank_merge_ok(c, c->pend_nsplit + nsplit)) {
            /* the fused step (the direct exchange's last): its merge waits
             * for the next call -- knn_ctx_end merges and finalizes in one
             * launch (a separate k_finalize cost its launch and ~20 us of
             * queue gap, rocprofv3) */
            c->pend2 = 1;
            c->pend2_set = c->pend_set;
            c->pend2_nsplit = c->pend_nsplit + nsplit;
            c->pend2_ev[0] = c->pend_ev;
            c->pend2_ev[1] = ev;
        } else {
            RCHK(launch_merge_sets(c, c->pend_set, 2, c->pend_nsplit + nsplit, cblk, c_base, nc));
            if (c->pend_ev) HIPCHK(hipEventRecord(c->pend_ev[2], c->ms));
            if (ev) HIPCHK(hipEventRecord(ev[2], c->ms));
        }
    } else if (!(set & 1) && (can_pair || gemm_own)) {
        c->pend = 1;
        c->pend_set = set;
        c->pend_nsplit = nsplit;
        c->pend_cblk = cblk;
        c->pend_cbase = c_base;
        c->pend_nc = (int)nc;
        c->pend_ev = ev;
    } else {
        RCHK(launch_merge_sets(c, set, 1, nsplit, cblk, c_base, nc));
        if (ev) HIPCHK(hipEventRecord(ev[2], c->ms));
    }
    /* step s - 2 is merged by now (a pending step is always s itself) */
    if (c->nstep >= KNN_STEP_LAG) {
        const int ps = (c->nstep - KNN_STEP_LAG) % KNN_PSETS;
        HIPCHK(hipStreamWaitEvent(cs, (c->i8 || c->h16) ? c->ev_ds[ps] : c->ev_m[ps], 0));
    }
    c->first_step = 0;
    c->ended = 0;
    c->nstep++;
    return KNN_OK;
}

int knn_ctx_step(knn_ctx_t *c, const void *d_cblock, size_t nc, size_t c_base, void *stream)
{
    return ctx_step_impl(c, d_cblock, NULL, nc, c_base, NULL, stream);
}

int knn_ctx_step_shadow(knn_ctx_t *c, const void *d_sblock, size_t nc, size_t c_base, void *stream)
{
    if (!d_sblock) return KNN_ERR_INVALID;
    return ctx_step_impl(c, NULL, d_sblock, nc, c_base, NULL, stream);
}

/* Several resident blocks in one step: byte blocks (knn_ctx_shadow == 2)
 * share one k_dist_topk_i8 launch per KNN_I8_MAXBLK blocks -- one launch's
 * fixed cost and one cold start instead of one per block, and splits long
 * enough to fill the CUs at P = 8; other forms fold one block a step. */
int knn_ctx_step_shadow_n(knn_ctx_t *c, int nblk, const void *const *d_sblocks, const size_t *nc,
                          const size_t *c_base, void *stream)
{
    if (!c || nblk < 1 || !d_sblocks || !nc || !c_base || !c->shadow) return KNN_ERR_INVALID;
    for (int b = 0; b < nblk; b++)
        if (!d_sblocks[b] || nc[b] == 0 || nc[b] > c->block_cap) return KNN_ERR_INVALID;
    if (c->shadow != 2) {
        for (int b = 0; b < nblk; b++) RCHK(ctx_step_impl(c, NULL, d_sblocks[b], nc[b], c_base[b], NULL, stream));
        return KNN_OK;
    }
    for (int b0 = 0; b0 < nblk; b0 += KNN_I8_MAXBLK) {
        knn_i8_blocks_t xb;
        memset(&xb, 0, sizeof(xb));
        xb.nblk = nblk - b0 < KNN_I8_MAXBLK ? nblk - b0 : KNN_I8_MAXBLK;
        for (int b = 0; b < xb.nblk; b++) {
            xb.ptr[b] = d_sblocks[b0 + b];
            xb.nc[b] = (int)nc[b0 + b];
            xb.base[b] = (int64_t)c_base[b0 + b];
        }
        RCHK(ctx_step_impl(c, NULL, NULL, 0, 0, &xb, stream));
    }
    return KNN_OK;
}

/* Several resident element blocks in one step of a split-filter (GEMM
 * mode) search: each block's split rows side by side, ONE k_dist_split
 * launch over all of them (block table) and ONE k_merge re-ranking from all
 * of them -- the direct exchange's received blocks at P = 8 were 7 launches
 * of ~8 tiles a workgroup and 7 merges. */
static int ctx_step_split_n(knn_ctx_t *c, int nblk, const void *const *d_cblocks, const size_t *nc,
                            const size_t *c_base, void *stream)
{
    HIPCHK(hipSetDevice(c->device));
    RCHK(flush_pend2(c, NULL, NULL));
    size_t nct = 0;   /* tile-rounded rows of the launch: the split model's input */
    for (int b = 0; b < nblk; b++) nct += knn_round_up(nc[b], KNN_SPLIT_TC);
    nct -= knn_round_up(nc[nblk - 1], KNN_SPLIT_TC) - nc[nblk - 1];
    c->split_solo = 0;
    const int nsplit = choose_splits(c, nct);
    const int set = c->nstep % KNN_PSETS, ds_i = c->nstep & 1;
    /* the pending own-block step (odd set right behind its lists) shares
     * this step's merge when the lists and the block table fit */
    int share = c->pend && (set & 1) && nblk + 1 <= KNN_SPLIT_MAXBLK &&
                c->lpq * (c->pend_nsplit + nsplit) + 1 <= 64;
    if (!share) RCHK(merge_pending(c));
    c->nsplit_last = nsplit;
    if (!(set & 1)) c->even_nsplit = nsplit;
    const int rc0 = ensure_part_buffers(c, nsplit, set, c->even_nsplit);
    if (rc0 == KNN_ERR_INVALID && c->pend) {
        /* the pair's lists cannot grow under the pending step's: merge it
         * alone first (as ctx_step_impl does) */
        RCHK(merge_pending(c));
        share = 0;
        RCHK(ensure_part_buffers(c, nsplit, set, c->even_nsplit));
    } else if (rc0) {
        return rc0;
    }
    hipStream_t cs = (hipStream_t)stream, ds = c->ds[ds_i];
    HIPCHK(hipEventRecord(c->ev_in, cs));
    HIPCHK(hipStreamWaitEvent(ds, c->ev_in, 0));
    if (c->nstep >= KNN_PSETS) HIPCHK(hipStreamWaitEvent(ds, c->ev_m[set], 0));
    const size_t per = knn_rows_pad(c->block_cap) * knn_split_rs(c->n);
    if (c->cspm_bytes[set] < per * (size_t)nblk) {
        /* (the set's last reader, merge s - 4, is ordered before ds above;
         * a free waits for the device) */
        HIPCHK(hipStreamSynchronize(ds));
        hipFree(c->cspm[set]);
        c->cspm[set] = NULL;
        c->cspm_bytes[set] = 0;
        if (hipMalloc(&c->cspm[set], per * (size_t)nblk) != hipSuccess) return KNN_ERR_NOMEM;
        c->cspm_bytes[set] = per * (size_t)nblk;
    }
    const size_t norm_off = knn_rows_pad(c->block_cap) * knn_n_pad_dt(c->n, c->dtype) * knn_esize(c->dtype);
    knn_split_blocks_t tab;
    knn_merge_blocks_t mb;
    memset(&tab, 0, sizeof(tab));
    memset(&mb, 0, sizeof(mb));
    tab.nblk = mb.nblk = nblk;
    /* the blocks' split rows in one conversion launch */
    void *cdst[KNN_SPLIT_MAXBLK];
    size_t crows[KNN_SPLIT_MAXBLK];
    for (int b = 0; b < nblk; b++) {
        cdst[b] = (char *)c->cspm[set] + per * (size_t)b;
        crows[b] = knn_rows_pad(nc[b]);
    }
    RCHK(knn_launch_shadow_split_n(nblk, cdst, d_cblocks, crows, c->dtype, c->n, c->sscale, ds));
    for (int b = 0; b < nblk; b++) {
        char *sp = (char *)cdst[b];
        tab.sp[b] = sp;
        tab.nrm[b] = (const char *)d_cblocks[b] + norm_off;
        tab.base[b] = mb.base[b] = (int64_t)c_base[b];
        tab.nc[b] = mb.nc[b] = (int)nc[b];
        tab.lim[b] = (int)knn_rows_pad(c->block_cap);
        mb.ptr[b] = d_cblocks[b];
    }
    hipEvent_t *ev = NULL;
    if (c->prof_on && c->prof_pending < KNN_PROF_STEPS) {
        ev = &c->prof_ev[3 * c->prof_pending++];
        HIPCHK(hipEventRecord(ev[0], ds));
    }
    RCHK(knn_launch_dist_split_n(c->dtype, c->kp, c->k, c->qblk, c->q_rows_pad, c->q_base, (int)c->nq, c->qsp, &tab,
                                 (int)c->n, c->meta, nsplit, c->part_d[set], c->part_i[set], c->part_T[set],
                                 (int)c->nq_pad, c->qthr, xord_for(c, nsplit), (float)(-2.0 / ((double)c->sscale * c->sscale)),
                                 ds));
    if (ev) HIPCHK(hipEventRecord(ev[1], ds));
    HIPCHK(hipEventRecord(c->ev_ds[set], ds));
    HIPCHK(hipStreamWaitEvent(c->ms, c->ev_ds[set], 0));
    int mset = set, mnsplit = nsplit;
    hipEvent_t *pev = NULL;
    if (share) {
        /* one merge of both steps: the pending set's lists, then this one's */
        HIPCHK(hipStreamWaitEvent(c->ms, c->ev_ds[(set + KNN_PSETS - 1) % KNN_PSETS], 0));
        c->pend = 0;
        mb.ptr[nblk] = c->pend_cblk;
        mb.base[nblk] = (int64_t)c->pend_cbase;
        mb.nc[nblk] = c->pend_nc;
        mb.nblk = nblk + 1;
        mset = c->pend_set;
        mnsplit = c->pend_nsplit + nsplit;
        nct += (size_t)c->pend_nc;
        pev = c->pend_ev;
    }
    const int *perm = NULL;
    if (want_order(c, nct)) {
        if (!c->ord_ready) RCHK(find_order(c, mset, mnsplit));
        perm = c->ord_perm;
    }
    RCHK(knn_launch_merge_n(c->dtype, c->kp, c->k, c->part_d[mset], c->part_i[mset], c->part_T[mset], mnsplit,
                            c->lpq, c->klx, (int)c->nq, (int)c->nq_pad, !c->merged, c->st_d, c->st_x, c->st_i,
                            c->st_T, c->qblk, c->q_rows_pad, &mb, (int)c->n, c->meta, c->qthr, c->split, perm, c->ms));
    c->merged = 1;
    HIPCHK(hipEventRecord(c->ev_m[set], c->ms));
    if (share) HIPCHK(hipEventRecord(c->ev_m[mset], c->ms));
    if (pev) HIPCHK(hipEventRecord(pev[2], c->ms));
    if (ev) HIPCHK(hipEventRecord(ev[2], c->ms));
    /* step s - 2 is merged by now (its merge read its blocks' rows) */
    if (c->nstep >= KNN_STEP_LAG) HIPCHK(hipStreamWaitEvent(cs, c->ev_m[(c->nstep - KNN_STEP_LAG) % KNN_PSETS], 0));
    c->first_step = 0;
    c->ended = 0;
    c->nstep++;
    return KNN_OK;
}

int knn_ctx_step_n(knn_ctx_t *c, int nblk, const void *const *d_cblocks, const size_t *nc, const size_t *c_base,
                   void *stream)
{
    if (!c || nblk < 1 || !d_cblocks || !nc || !c_base) return KNN_ERR_INVALID;
    for (int b = 0; b < nblk; b++)
        if (!d_cblocks[b] || nc[b] == 0 || nc[b] > c->block_cap) return KNN_ERR_INVALID;
    /* the split filter (real-valued data, GEMM mode): fused launches of up to
     * KNN_SPLIT_MAXBLK blocks; any other contraction folds one block a step */
    if (!c->split) {
        for (int b = 0; b < nblk; b++) RCHK(ctx_step_impl(c, d_cblocks[b], NULL, nc[b], c_base[b], NULL, stream));
        return KNN_OK;
    }
    for (int b0 = 0; b0 < nblk; b0 += KNN_SPLIT_MAXBLK) {
        const int nb = nblk - b0 < KNN_SPLIT_MAXBLK ? nblk - b0 : KNN_SPLIT_MAXBLK;
        RCHK(ctx_step_split_n(c, nb, d_cblocks + b0, nc + b0, c_base + b0, stream));
    }
    return KNN_OK;
}

int knn_ctx_shadow(const knn_ctx_t *c) { return c ? c->shadow : 0; }

/* Uncertified queries of a single-block int8 search (P = 1: the block is
 * the query block, resident as q8) are searched again on the int8
 * contraction with 65-entry lane lists -- a lane can then only overflow if
 * more than 64 rows tie at or below the query's (k+1)-th distance -- over
 * 31 corpus splits, each query starting from the (k+1)-th key the search
 * kept for it (k_merge_rank); the certified results replace the fp64
 * rescan for them, and what stays uncertified goes to the exact rescan as
 * before.  SIFT (1M x 128, k = 32): 186 queries, 8.4 ms of fp64 scan.
 * (12-entry lists over 31 splits certified none of MNIST's: those are
 * queries whose k-th and (k+1)-th distances tie, 35 of 60000.) */
static int ctx_end_device(knn_ctx_t *c, knn_neighbour_t *d_out, hipStream_t s);

static void research8_free(knn_ctx_t *c)
{
    if (c->sub) knn_ctx_destroy(c->sub);
    hipFree(c->sub_q8);
    hipFree(c->sub_out);
    hipFree(c->sub_flag);
    c->sub = NULL;
    c->sub_q8 = NULL;
    c->sub_out = NULL;
    c->sub_flag = NULL;
    c->sub_cap = 0;
}

/* The re-search proper: the c->nfail uncertified queries of fail_list
 * against the byte blocks of xb (NULL: the single-block search's own query
 * byte block, q8), the sub-search's q_base at q_base_sub (past every row id
 * of the blocks). */
static int research8_run(knn_ctx_t *c, int nblk, const void *const *blk, const size_t *bnc, const size_t *bbase,
                         size_t q_base_sub, knn_neighbour_t *d_out, hipStream_t s)
{
    const int nf = c->nfail;
    if (!c->sub || c->sub_cap < (size_t)nf) {
        research8_free(c);
        const size_t cap = knn_round_up((size_t)nf, KNN_TQ);
        RCHK(knn_ctx_create_dt(&c->sub, c->device, cap, c->n, c->block_cap, c->k, c->dtype));
        c->sub->sub_research = 1;
        if (hipMalloc(&c->sub_q8, knn_s8_bytes(cap, c->n)) != hipSuccess ||
            hipMalloc((void **)&c->sub_out, cap * (size_t)c->k * sizeof(knn_neighbour_t)) != hipSuccess ||
            hipMalloc((void **)&c->sub_flag, cap) != hipSuccess ||
            (!c->fail_list2 && hipMalloc((void **)&c->fail_list2, c->nq_pad * sizeof(int)) != hipSuccess)) {
            research8_free(c);   /* no half-built sub-context survives */
            return KNN_ERR_NOMEM;
        }
        c->sub_cap = cap;   /* only once every buffer exists */
    }
    knn_ctx_t *u = c->sub;
    u->nq = (size_t)nf;   /* within the capacity it was created with */
    u->nq_pad = knn_round_up((size_t)nf, KNN_TQ);
    /* q_base just past the block's last row id: no row is masked as "the
     * query itself" (its d^2 = 0 is dropped like every exact duplicate,
     * serial:86).  Begin first (it resets the bounds), then the gather: the
     * rows, and each query's bound -- k_merge_rank left the (k+1)-th kept
     * key of every uncertified query in qthr, so the re-search filters with
     * the running answer from its first tile (cold 65-entry lists admitted
     * every row of a lane's first tiles: 682 us for two MNIST queries) */
    RCHK(ctx_begin(u, NULL, c->sub_q8, c->sub_cap, q_base_sub, c->meta, c->hmeta, s));
    RCHK(knn_launch_gather8(c->sub_q8, c->q8, c->fail_list, nf, c->n, c->q_rows_pad, knn_rows_pad(c->sub_cap),
                            c->qthr, u->qthr, s));
    if (nblk > 0) {
        /* a ring rank: every block it holds, KNN_I8_MAXBLK to a launch */
        for (int b0 = 0; b0 < nblk; b0 += KNN_I8_MAXBLK) {
            knn_i8_blocks_t t;
            memset(&t, 0, sizeof(t));
            t.nblk = nblk - b0 < KNN_I8_MAXBLK ? nblk - b0 : KNN_I8_MAXBLK;
            for (int b = 0; b < t.nblk; b++) {
                t.ptr[b] = blk[b0 + b];
                t.nc[b] = (int)bnc[b0 + b];
                t.base[b] = (int64_t)bbase[b0 + b];
            }
            RCHK(ctx_step_impl(u, NULL, NULL, 0, 0, &t, s));
        }
    } else {
        RCHK(ctx_step_impl(u, NULL, c->q8, c->step0_nc, c->step0_cbase, NULL, s));
    }
    /* the sub-search's fail list and count stay on the device: resolve8
     * reads them there, so the only host read is the final count below */
    RCHK(ctx_end_device(u, c->sub_out, s));
    RCHK(knn_launch_resolve8(c->sub_flag, c->fail_list, nf, u->fail_list, u->fail_count, c->sub_out, c->k, d_out,
                             c->fail_list2, c->fail_count, s));
    /* (tests: a failure at this point, after resolve8 rewrote rows of d_out
     * and the device count -- knn_ctx_end's fallback must still be exact) */
    if (env_on("KNN_TEST_RESEARCH8_FAIL")) return KNN_ERR_HIP;
    int nn = 0;
    HIPCHK(hipMemcpyAsync(&nn, c->fail_count, sizeof(int), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    int *t = c->fail_list;
    c->fail_list = c->fail_list2;
    c->fail_list2 = t;
    c->nfail = nn;
    return KNN_OK;
}

static int research8(knn_ctx_t *c, knn_neighbour_t *d_out, hipStream_t s)
{
    /* INT mode only (c->mode: the device's verdict on the real meta): a
     * speculative begin (knn_ctx_begin_s8 on a stale host hint) whose data
     * turned out real-valued fails every query in GEMM mode, and the
     * sub-search would run GEMM work from a context with no element rows */
    if (c->mode != KNN_MODE_INT || !c->i8 || c->sub_research || !c->one_block_q8 || c->nstep != 1 || !c->have_hmeta ||
        c->step0_cbase != c->q_base || c->q_rows_pad != knn_rows_pad(c->block_cap) || c->kp > KNN_KP_M ||
        env_on("KNN_FORCE_RESCAN") || env_on("KNN_NO_RESEARCH8"))
        return KNN_OK;
    return research8_run(c, 0, NULL, NULL, NULL, c->step0_cbase + c->step0_nc, d_out, s);
}

/* rescan state for c->nfail uncertified queries (knn_ctx_end, and again
 * after a ring rank's re-search changed the count: the per-query chunk
 * layout depends on it) */
static int rescan_prep(knn_ctx_t *c, void *stream)
{
    if (c->nfail == 0) return KNN_OK;
    const size_t need = (size_t)c->nfail * (1 + (size_t)knn_rescan_chunks(c->nfail));
    if (need > c->rs_cap) {
        hipFree(c->rs_d);
        hipFree(c->rs_i);
        c->rs_d = NULL;
        c->rs_i = NULL;
        c->rs_cap = 0;
        size_t cap = need;
        if (hipMalloc((void **)&c->rs_d, cap * c->kp * sizeof(double)) != hipSuccess ||
            hipMalloc((void **)&c->rs_i, cap * c->kp * sizeof(int)) != hipSuccess)
            return KNN_ERR_NOMEM;
        c->rs_cap = cap;
    }
    return knn_launch_rescan_init(c->kp, c->rs_d, c->rs_i, c->nfail, stream);
}

/* A ring rank's int8 re-search (include/knn.h): after knn_ctx_end, its
 * uncertified queries against the byte blocks the rank holds. */
int knn_ctx_research_blocks(knn_ctx_t *c, int nblk, const void *const *d_sblocks, const size_t *nc,
                            const size_t *c_base, knn_neighbour_t *d_out, size_t *unresolved, void *stream)
{
    /* only right after knn_ctx_end: nfail and fail_list are this search's */
    if (!c || !d_out || nblk < 1 || !d_sblocks || !nc || !c_base || !c->ended) return KNN_ERR_INVALID;
    if (unresolved) *unresolved = (size_t)c->nfail;
    if (c->nfail == 0 || c->mode != KNN_MODE_INT || !c->i8 || c->shadow != 2 || c->sub_research || !c->q8 ||
        !c->have_hmeta || c->kp > KNN_KP_M || env_on("KNN_FORCE_RESCAN") || env_on("KNN_NO_RESEARCH8"))
        return KNN_OK;
    size_t q_end = 0;
    for (int b = 0; b < nblk; b++) {
        if (!d_sblocks[b] || nc[b] == 0 || nc[b] > c->block_cap) return KNN_ERR_INVALID;
        if (c_base[b] + nc[b] > q_end) q_end = c_base[b] + nc[b];
    }
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = (hipStream_t)stream;
    const int before = c->nfail;
    const int rc = research8_run(c, nblk, d_sblocks, nc, c_base, q_end, d_out, s);
    if (rc != KNN_OK) {
        /* as in knn_ctx_end: the exact rescan resolves the first pass's list */
        HIPCHK(hipStreamSynchronize(s));
        (void)hipGetLastError();
        c->nfail = before;
    }
    if (c->nfail != before) RCHK(rescan_prep(c, stream));
    if (unresolved) *unresolved = (size_t)c->nfail;
    return KNN_OK;
}

/* The device side of knn_ctx_end: the last merge / finalize on the merge
 * stream, `stream` ordered after them.  The records, the fail list and its
 * count are then on the device; no host read (research8's sub-context). */
static int ctx_end_device(knn_ctx_t *c, knn_neighbour_t *d_out, hipStream_t s)
{
    HIPCHK(hipEventRecord(c->ev_in, s));
    HIPCHK(hipStreamWaitEvent(c->ms, c->ev_in, 0));
    int fin = 0;
    RCHK(flush_pend2(c, d_out, &fin));
    if (!fin) RCHK(merge_pending_fin(c, d_out, &fin));
    if (!fin)
        RCHK(knn_launch_finalize(c->dtype, c->kp, c->st_d, c->st_x, c->st_i, c->st_T, c->qblk, c->q_rows_pad,
                                 (int)c->nq, (int)c->n, c->k, c->meta, d_out, c->fail_count,
                                 c->fail_list, c->mode_dev, c->fbound, env_on("KNN_FORCE_RESCAN"),
                                 c->split, c->ms));
    HIPCHK(hipEventRecord(c->ev_end, c->ms));
    HIPCHK(hipStreamWaitEvent(s, c->ev_end, 0));
    return KNN_OK;
}

/* knn_ctx_end's device part and count read-back, on stream c->ms (the
 * caller's stream has been waited for on the host) */
static int ctx_end_merge(knn_ctx_t *c, knn_neighbour_t *d_out)
{
    /* the last merge (deferred or pending) finalizes too when it is the
     * rank merge (INT-mode int8 lists) */
    int fin = 0;
    RCHK(flush_pend2(c, d_out, &fin));
    if (!fin) RCHK(merge_pending_fin(c, d_out, &fin));
    if (!fin)
        RCHK(knn_launch_finalize(c->dtype, c->kp, c->st_d, c->st_x, c->st_i, c->st_T, c->qblk, c->q_rows_pad,
                                 (int)c->nq, (int)c->n, c->k, c->meta, d_out, c->fail_count,
                                 c->fail_list, c->mode_dev, c->fbound, env_on("KNN_FORCE_RESCAN"),
                                 c->split, c->ms));
    c->h_count[0] = c->h_count[1] = -1;
    RCHK(knn_launch_count_out(c->fail_count, c->h_count_dev, c->meta,
                              (double *)((char *)c->h_count_dev + 16), c->ms));
    /* the host waits for the results, so the caller's stream needs no wait
     * packet on them (one would sit before that stream's next kernel) */
    HIPCHK(hipStreamSynchronize(c->ms));
    return KNN_OK;
}

int knn_ctx_end(knn_ctx_t *c, knn_neighbour_t *d_out, size_t *unresolved, void *stream)
{
    if (!c || !d_out || c->first_step) return KNN_ERR_INVALID;
    c->ended = 0;
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = (hipStream_t)stream;
    /* The last merge, finalize and the counter read-back run behind the
     * search's last distance launch: on the merge stream when earlier
     * merges ran there (they update the state in step order), otherwise on
     * that launch's own stream (after the other distance stream's last
     * launch) -- every cross-stream hop put 20-30 us on the pass's critical
     * path in the rocprofv3 traces (a P = 1 search: distance kernel ->
     * 25 us -> merge on the merge stream).  The records go to d_out, so
     * that stream first waits for the caller's stream as it stands now:
     * d_out may have just been allocated, cleared or read there (a caching
     * allocator hands out memory that pending work on the caller's stream
     * used last).  end() returns with the results complete (a host wait), so
     * whatever the caller enqueues afterwards follows them. */
    /* The orderings end() needs besides the last distance launch -- the
     * caller's stream as it stands now, and the other distance stream's last
     * launch -- are waited for on the HOST: end() blocks until the results
     * anyway, both are normally complete long before the last launch, and a
     * stream wait costs 20-25 us of GPU time on the queue even on an event
     * that completed long before (rocprofv3, P = 1: distance kernel -> 24 us
     * -> merge on the same queue, with only the caller-stream wait between).
     * Nothing on the caller's stream can wait on work end() enqueues. */
    /* A solo search's kernel and merge are on the caller's stream already
     * (knn_ctx_set_solo): nothing to wait for on the host, the merge follows
     * the kernel there. */
    hipStream_t ms = c->ms;
    if (c->solo_on) {
        if ((hipStream_t)stream != c->ms) {   /* end() on another stream than the step's */
            HIPCHK(hipEventRecord(c->ev_in, c->ms));
            HIPCHK(hipStreamWaitEvent(s, c->ev_in, 0));
            c->ms = s;
        }
    } else {
        HIPCHK(hipEventRecord(c->ev_in, s));
        HIPCHK(hipEventSynchronize(c->ev_in));
        if (!c->merged && c->nstep >= 1) {
            const int last = (c->nstep - 1) & 1;
            if (c->nstep >= 2) HIPCHK(hipEventSynchronize(c->ev_ds[(c->nstep - 2) % KNN_PSETS]));
            c->ms = c->ds[last];
        }
    }
    const int rc_end = ctx_end_merge(c, d_out);
    c->ms = c->solo_on ? c->ms_keep : ms;
    c->solo_on = 0;
    RCHK(rc_end);
    RCHK(prof_collect(c));
    c->nfail = ((volatile int *)c->h_count)[0];
    c->mode = ((volatile int *)c->h_count)[1];
    if (c->nfail < 0) return KNN_ERR_HIP;
    if (c->nfail > 0 && research8(c, d_out, s) != KNN_OK) {
        /* the re-search is an optimisation: on any failure of it the exact
         * rescan resolves the same queries.  The rescan reads only the host
         * count c->nfail and c->fail_list, both still the first pass's
         * (resolve8 writes the new list into fail_list2; they are swapped
         * only after the count's read-back succeeded).  What resolve8 may
         * already have changed is harmless: the d_out rows it rewrote are
         * rows of failed queries, which the rescan rewrites again, and the
         * device fail_count is read by nothing after this point and reset by
         * the next begin.  (test_gpu_s8.py injects this failure.) */
        HIPCHK(hipStreamSynchronize(s));
        (void)hipGetLastError();
    }
    if (unresolved) *unresolved = (size_t)c->nfail;
    RCHK(rescan_prep(c, stream));
    c->ended = 1;
    return KNN_OK;
}

int knn_ctx_rescan_step(knn_ctx_t *c, const void *d_cblock, size_t nc, size_t c_base,
                        void *stream)
{
    if (!c || !d_cblock || nc == 0) return KNN_ERR_INVALID;
    if (c->nfail == 0) return KNN_OK;
    if (!c->qblk) return KNN_ERR_INVALID;   /* begin_s8: knn_ctx_attach_qblock first */
    HIPCHK(hipSetDevice(c->device));
    return knn_launch_rescan_step(c->dtype, c->kp, c->fail_list, c->nfail, c->fbound, c->qblk,
                                  d_cblock, c_base, (int)nc, (int)c->n, c->k, c->rs_d, c->rs_i,
                                  stream);
}

int knn_ctx_rescan_end(knn_ctx_t *c, knn_neighbour_t *d_out, void *stream)
{
    if (!c || !d_out) return KNN_ERR_INVALID;
    if (c->nfail == 0) return KNN_OK;
    HIPCHK(hipSetDevice(c->device));
    return knn_launch_rescan_end(c->kp, c->fail_list, c->nfail, c->rs_d, c->rs_i, c->k, d_out,
                                 stream);
}

int knn_search_packed(knn_ctx_t *c, const void *d_block, size_t m, knn_neighbour_t *d_out,
                      void *stream)
{
    if (!c || !d_block || !d_out || m != c->nq || m != c->block_cap) return KNN_ERR_INVALID;
    const double *meta =
        (const double *)((const char *)d_block + knn_block_meta_offset_dt(m, c->n, c->dtype));
    size_t unresolved = 0;
    RCHK(knn_ctx_begin(c, d_block, m, 0, meta, stream));
    RCHK(knn_ctx_step(c, d_block, m, 0, stream));
    RCHK(knn_ctx_end(c, d_out, &unresolved, stream));
    if (unresolved) {
        RCHK(knn_ctx_rescan_step(c, d_block, m, 0, stream));
        RCHK(knn_ctx_rescan_end(c, d_out, stream));
    }
    return KNN_OK;
}

/* Multi-GPU one-call path lives in knn_ring.c. */
int knn_search_ring_host(const double *X, size_t m, size_t n, int layout, int k, int ngpus,
                         int dtype, knn_neighbour_t *out, double *seconds);

int knn_search(const double *X, size_t m, size_t n, int layout, const double *labels, int k,
               int ngpus, int dtype, knn_neighbour_t *out)
{
    if (!X || !out || m == 0 || n == 0 || k <= 0) return KNN_ERR_INVALID;
    if (!dtype_ok(dtype)) return KNN_ERR_UNSUPPORTED;
    if (k > (dtype == KNN_F32 ? KNN_MAX_K_F32 : KNN_MAX_K)) return KNN_ERR_UNSUPPORTED;
    if (layout != KNN_COLMAJOR && layout != KNN_ROWMAJOR) return KNN_ERR_INVALID;
    if (ngpus < 1) return KNN_ERR_INVALID;
    int rc = KNN_OK;
    /* KNN_FORCE_RING=1 runs the RCCL ring driver even on one GPU (tests) */
    const char *force = getenv("KNN_FORCE_RING");
    if (ngpus > 1 || (force && force[0] == '1')) {
        rc = knn_search_ring_host(X, m, n, layout, k, ngpus, dtype, out, &g_last_search_s);
    } else {
        knn_ctx_t *ctx = NULL;
        double *d_src = NULL;
        void *d_blk = NULL;
        knn_neighbour_t *d_out = NULL;
        hipEvent_t e0 = NULL, e1 = NULL;
        rc = knn_ctx_create_dt(&ctx, 0, m, n, m, k, dtype);
        if (rc) return rc;
        if (hipMalloc((void **)&d_src, m * n * sizeof(double)) != hipSuccess ||
            hipMalloc(&d_blk, knn_block_bytes_dt(m, n, dtype)) != hipSuccess ||
            hipMalloc((void **)&d_out, m * (size_t)k * sizeof(knn_neighbour_t)) != hipSuccess) {
            rc = KNN_ERR_NOMEM;
            goto done1;
        }
        if (hipMemcpy(d_src, X, m * n * sizeof(double), hipMemcpyHostToDevice) != hipSuccess ||
            hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) {
            rc = KNN_ERR_HIP;
            goto done1;
        }
        hipEventRecord(e0, NULL);
        rc = knn_block_pack_dt(d_blk, dtype, m, m, n, d_src, KNN_F64,
                               layout == KNN_COLMAJOR ? m : n, layout, NULL);
        if (!rc) rc = knn_search_packed(ctx, d_blk, m, d_out, NULL);
        hipEventRecord(e1, NULL);
        if (!rc) {
            float ms = 0.f;
            if (hipEventSynchronize(e1) != hipSuccess || hipEventElapsedTime(&ms, e0, e1) != hipSuccess)
                rc = KNN_ERR_HIP;
            g_last_search_s = ms * 1e-3;
        }
        if (!rc && hipMemcpy(out, d_out, m * (size_t)k * sizeof(knn_neighbour_t),
                             hipMemcpyDeviceToHost) != hipSuccess)
            rc = KNN_ERR_HIP;
    done1:
        if (e0) hipEventDestroy(e0);
        if (e1) hipEventDestroy(e1);
        hipFree(d_src);
        hipFree(d_blk);
        hipFree(d_out);
        knn_ctx_destroy(ctx);
    }
    if (!rc && labels) {
        for (size_t i = 0; i < m * (size_t)k; i++)
            out[i].label = out[i].idx > 0 ? (int32_t)labels[out[i].idx - 1] : 0;
    }
    return rc;
}
