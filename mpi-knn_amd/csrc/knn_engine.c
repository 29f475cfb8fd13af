/*
 * knn_engine.c -- host side of libknn (C, HIP runtime API).
 *
 * Owns device buffers and sequences the kernels of knn_kernels.hip:
 *   knn_block_pack  -> k_pack + k_norms      (blk:100-109 packing)
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

#define KNN_MAX_SPLITS 15 /* merge kernel: 4*splits + 1 lists <= 64 lanes */
#define KNN_PROF_STEPS 64 /* steps timed between two knn_ctx_end calls */

struct knn_ctx {
    int device;
    int dtype;          /* element type of the packed blocks (KNN_F64 / KNN_F32) */
    size_t nq, nq_pad, n, block_cap;
    int k;
    int kp, kl;         /* state capacity / per-lane list length serving k */
    int xord;           /* k_dist_topk workgroup order (0 split-major, 1 XCD-grouped) */
    int cus;
    /* per-step partial lists of k_dist_topk, grown to the largest split
     * count used so far (part_splits) */
    int part_splits;
    double *part_d;
    int *part_i;
    double *part_T;
    /* per-query filter bound shared by all splits and ring steps */
    double *qthr;
    /* running state per query: KNN_KP x (approx d^2, exact S, idx), T pair */
    double *st_d, *st_x, *st_T;
    int *st_i;
    /* unresolved queries */
    int *fail_count, *fail_list, *mode_dev;
    double *fbound;     /* per query: rescan bound on the k-th key (k_finalize) */
    double *rs_d;
    int *rs_i;
    size_t rs_cap;
    /* current search */
    const void *qblk;
    size_t q_base, q_rows_pad;
    const double *meta;
    int first_step;
    int nsplit_last;
    int nfail;
    int mode;
    /* kernel timing (knn_ctx_profile): 3 events per step bracket
     * k_dist_topk and k_merge */
    int prof_on, prof_pending, prof_launches;
    double prof_dist_ms, prof_merge_ms;
    hipEvent_t prof_ev[3 * KNN_PROF_STEPS];
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

int knn_block_pack(void *d_block, size_t cap, size_t rows, size_t n, const double *d_src,
                   size_t ld, int layout, void *stream)
{
    return knn_block_pack_dt(d_block, KNN_F64, cap, rows, n, d_src, KNN_F64, ld, layout, stream);
}

static void ctx_free_buffers(knn_ctx_t *c)
{
    hipFree(c->part_d);
    hipFree(c->part_i);
    hipFree(c->part_T);
    hipFree(c->qthr);
    hipFree(c->st_d);
    hipFree(c->st_x);
    hipFree(c->st_T);
    hipFree(c->st_i);
    hipFree(c->fail_count);
    hipFree(c->fail_list);
    hipFree(c->fbound);
    hipFree(c->mode_dev);
    hipFree(c->rs_d);
    hipFree(c->rs_i);
    for (int i = 0; i < 3 * KNN_PROF_STEPS; i++)
        if (c->prof_ev[i]) hipEventDestroy(c->prof_ev[i]);
}

int knn_ctx_profile(knn_ctx_t *c, int enable, double *dist_ms, double *merge_ms, int *launches)
{
    if (!c) return KNN_ERR_INVALID;
    if (enable >= 0) {
        HIPCHK(hipSetDevice(c->device));
        if (enable && !c->prof_ev[0]) {
            for (int i = 0; i < 3 * KNN_PROF_STEPS; i++)
                HIPCHK(hipEventCreate(&c->prof_ev[i]));
        }
        c->prof_on = enable ? 1 : 0;
        if (enable) {
            c->prof_pending = 0;
            c->prof_launches = 0;
            c->prof_dist_ms = 0.0;
            c->prof_merge_ms = 0.0;
        }
    }
    if (dist_ms) *dist_ms = c->prof_dist_ms;
    if (merge_ms) *merge_ms = c->prof_merge_ms;
    if (launches) *launches = c->prof_launches;
    return KNN_OK;
}

/* after the stream has been synchronised: fold the recorded steps */
static int prof_collect(knn_ctx_t *c)
{
    for (int i = 0; i < c->prof_pending; i++) {
        float a = 0.f, b = 0.f;
        HIPCHK(hipEventElapsedTime(&a, c->prof_ev[3 * i], c->prof_ev[3 * i + 1]));
        HIPCHK(hipEventElapsedTime(&b, c->prof_ev[3 * i + 1], c->prof_ev[3 * i + 2]));
        c->prof_dist_ms += a;
        c->prof_merge_ms += b;
        c->prof_launches++;
    }
    c->prof_pending = 0;
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
    /* tuning override: an fp32 context may take any variant holding k */
    if (dtype == KNN_F32 && getenv("KNN_FORCE_KP")) {
        const int f = atoi(getenv("KNN_FORCE_KP"));
        if ((f == KNN_KP || f == KNN_KP_M || f == KNN_KP_L) && k <= f) c->kp = f;
    }
    c->kl = knn_kl_for(c->kp);
    c->xord = getenv("KNN_XCD_ORDER") ? atoi(getenv("KNN_XCD_ORDER")) != 0 : 0;
    c->cus = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;

    const size_t np = c->nq_pad;
    int ok = 1;
    ok &= hipMalloc((void **)&c->qthr, np * sizeof(double)) == hipSuccess;
    ok &= hipMalloc((void **)&c->st_d, np * c->kp * sizeof(double)) == hipSuccess;
    ok &= hipMalloc((void **)&c->st_x, np * c->kp * sizeof(double)) == hipSuccess;
    ok &= hipMalloc((void **)&c->st_i, np * c->kp * sizeof(int)) == hipSuccess;
    ok &= hipMalloc((void **)&c->st_T, np * 2 * sizeof(double)) == hipSuccess;
    ok &= hipMalloc((void **)&c->fail_count, sizeof(int)) == hipSuccess;
    ok &= hipMalloc((void **)&c->fail_list, np * sizeof(int)) == hipSuccess;
    ok &= hipMalloc((void **)&c->fbound, np * sizeof(double)) == hipSuccess;
    ok &= hipMalloc((void **)&c->mode_dev, sizeof(int)) == hipSuccess;
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

int knn_ctx_info(const knn_ctx_t *c, int *mode, int *splits)
{
    if (!c) return KNN_ERR_INVALID;
    if (mode) *mode = c->mode;
    if (splits) *splits = c->nsplit_last;
    return KNN_OK;
}

int knn_ctx_begin(knn_ctx_t *c, const void *d_qblock, size_t q_cap, size_t q_base,
                  const double *d_meta, void *stream)
{
    if (!c || !d_qblock || !d_meta || q_cap < c->nq) return KNN_ERR_INVALID;
    HIPCHK(hipSetDevice(c->device));
    c->qblk = d_qblock;
    c->q_base = q_base;
    c->q_rows_pad = knn_rows_pad(q_cap);
    c->meta = d_meta;
    c->first_step = 1;
    c->nfail = 0;
    HIPCHK(hipMemsetAsync(c->fail_count, 0, sizeof(int), (hipStream_t)stream));
    RCHK(knn_launch_fill_inf(c->qthr, (int)c->nq_pad, stream));
    return KNN_OK;
}

/* bytes of partial lists per corpus split (k_dist_topk -> k_merge) */
static size_t split_bytes(const knn_ctx_t *c)
{
    return c->nq_pad * (4 * (size_t)c->kl * (sizeof(double) + sizeof(int)) + sizeof(double));
}

#define KNN_PART_BUDGET ((size_t)2 << 30) /* partial-list bytes above one split */

/* Corpus splits per query block: fill the CUs in whole waves of workgroups
 * (one 512-thread workgroup per CU), keep >= 4 tiles per split, and take
 * the fewest splits within 0.5% of the best fill (each split costs a
 * partial-list pass and its memory, capped at KNN_PART_BUDGET). */
static int choose_splits(const knn_ctx_t *c, size_t nc)
{
    const char *env = getenv("KNN_SPLITS");
    const long nqb = (long)((c->nq + KNN_TQ - 1) / KNN_TQ);
    const long ntiles = (long)((nc + KNN_TC - 1) / KNN_TC);
    if (env && atoi(env) > 0) {
        int s = atoi(env);
        return s > KNN_MAX_SPLITS ? KNN_MAX_SPLITS : s;
    }
    int smax = KNN_MAX_SPLITS;
    const size_t per = split_bytes(c);
    if (per > 0 && KNN_PART_BUDGET / per < (size_t)smax)
        smax = KNN_PART_BUDGET / per > 1 ? (int)(KNN_PART_BUDGET / per) : 1;
    double eff[KNN_MAX_SPLITS + 1] = {0};
    double best_eff = 0.0;
    for (int s = 1; s <= smax; s++) {
        if (s > 1 && ntiles / s < 4) break;
        const long w = nqb * s;
        const long rounds = (w + c->cus - 1) / c->cus;
        eff[s] = (double)w / (double)(rounds * c->cus);
        if (eff[s] > best_eff) best_eff = eff[s];
    }
    for (int s = 1; s <= smax; s++)
        if (eff[s] >= best_eff - 5e-3) return s;
    return 1;
}

static int ensure_part_buffers(knn_ctx_t *c, int nsplit)
{
    if (nsplit <= c->part_splits) return KNN_OK;
    hipFree(c->part_d);
    hipFree(c->part_i);
    hipFree(c->part_T);
    c->part_d = NULL;
    c->part_i = NULL;
    c->part_T = NULL;
    c->part_splits = 0;
    const size_t npart = (size_t)nsplit * c->nq_pad * 4 * (size_t)c->kl;
    if (hipMalloc((void **)&c->part_d, npart * sizeof(double)) != hipSuccess ||
        hipMalloc((void **)&c->part_i, npart * sizeof(int)) != hipSuccess ||
        hipMalloc((void **)&c->part_T, (size_t)nsplit * c->nq_pad * sizeof(double)) != hipSuccess)
        return KNN_ERR_NOMEM;
    c->part_splits = nsplit;
    return KNN_OK;
}

int knn_ctx_step(knn_ctx_t *c, const void *d_cblock, size_t nc, size_t c_base, void *stream)
{
    if (!c || !d_cblock || nc == 0 || nc > c->block_cap) return KNN_ERR_INVALID;
    HIPCHK(hipSetDevice(c->device));
    const int nsplit = choose_splits(c, nc);
    c->nsplit_last = nsplit;
    RCHK(ensure_part_buffers(c, nsplit));
    const void *cblk = d_cblock;
    hipEvent_t *ev = NULL;
    if (c->prof_on && c->prof_pending < KNN_PROF_STEPS) {
        ev = &c->prof_ev[3 * c->prof_pending++];
        HIPCHK(hipEventRecord(ev[0], (hipStream_t)stream));
    }
    RCHK(knn_launch_dist_topk(c->dtype, c->kp, c->k, c->qblk, c->q_rows_pad, c->q_base, (int)c->nq, cblk,
                              knn_rows_pad(c->block_cap), c_base, (int)nc, (int)c->n, c->meta, nsplit,
                              c->part_d, c->part_i, c->part_T, (int)c->nq_pad, c->qthr, c->xord,
                              stream));
    if (ev) HIPCHK(hipEventRecord(ev[1], (hipStream_t)stream));
    RCHK(knn_launch_merge(c->dtype, c->kp, c->k, c->part_d, c->part_i, c->part_T, nsplit, (int)c->nq,
                          (int)c->nq_pad, c->first_step, c->st_d, c->st_x, c->st_i, c->st_T, c->qblk,
                          c->q_rows_pad, cblk, c_base, (int)nc, (int)c->n, c->meta, stream));
    if (ev) HIPCHK(hipEventRecord(ev[2], (hipStream_t)stream));
    c->first_step = 0;
    return KNN_OK;
}

int knn_ctx_end(knn_ctx_t *c, knn_neighbour_t *d_out, size_t *unresolved, void *stream)
{
    if (!c || !d_out || c->first_step) return KNN_ERR_INVALID;
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = (hipStream_t)stream;
    RCHK(knn_launch_finalize(c->dtype, c->kp, c->st_d, c->st_x, c->st_i, c->st_T, c->qblk, c->q_rows_pad,
                             (int)c->nq, (int)c->n, c->k, c->meta, d_out, c->fail_count,
                             c->fail_list, c->mode_dev, c->fbound, stream));
    int host[2];
    HIPCHK(hipMemcpyAsync(&host[0], c->fail_count, sizeof(int), hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(&host[1], c->mode_dev, sizeof(int), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    RCHK(prof_collect(c));
    c->nfail = host[0];
    c->mode = host[1];
    if (unresolved) *unresolved = (size_t)c->nfail;
    if (c->nfail > 0) {
        if ((size_t)c->nfail > c->rs_cap) {
            hipFree(c->rs_d);
            hipFree(c->rs_i);
            c->rs_d = NULL;
            c->rs_i = NULL;
            c->rs_cap = 0;
            size_t cap = (size_t)c->nfail;
            if (hipMalloc((void **)&c->rs_d, cap * c->kp * sizeof(double)) != hipSuccess ||
                hipMalloc((void **)&c->rs_i, cap * c->kp * sizeof(int)) != hipSuccess)
                return KNN_ERR_NOMEM;
            c->rs_cap = cap;
        }
        RCHK(knn_launch_rescan_init(c->kp, c->rs_d, c->rs_i, c->nfail, stream));
    }
    return KNN_OK;
}

int knn_ctx_rescan_step(knn_ctx_t *c, const void *d_cblock, size_t nc, size_t c_base,
                        void *stream)
{
    if (!c || !d_cblock || nc == 0) return KNN_ERR_INVALID;
    if (c->nfail == 0) return KNN_OK;
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
