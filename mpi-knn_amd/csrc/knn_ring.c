/*
 * knn_ring.c -- knn_search() across the GPUs of one node: the corpus-block
 * ring of mpi-knn-parallel_{blocking,non_blocking}.c rebuilt on RCCL.
 *
 * Reference schedule (blk:122-244, nb:132-259): rank r owns rows
 * [r*R, (r+1)*R), R = m/P (remainder dropped), and passes blocks to r+1
 * each step with MPI_Send/Recv or Isend/Irecv+Wait, barrier-locked, with no
 * compute/comm overlap and a broken schedule.
 *
 * Here: device g owns queries [g*R, min(m,(g+1)*R)), R = ceil(m/P) (no row
 * dropped).  Step s computes on block (g - s) mod P while the same block is
 * sent to g+1 and block (g - s - 1) mod P is received from g-1, on a
 * separate comm stream per device (ncclSend/ncclRecv over xGMI, one group
 * per hop) -- double-buffered, so the next block lands while the current
 * one is being contracted.  Every device visits all P blocks exactly once;
 * results are byte-identical to the 1-GPU path (merge order is by (d, idx)).
 * The meta of all blocks is combined with one ncclAllReduce(max).
 *
 * Two schedules (KNN_RING_SCHEDULE, default "direct"):
 *   ring    the rotation above, one hop per step;
 *   direct  every device sends its block to every other device at once (one
 *           ncclGroup of P-1 sends and P-1 receives per device: on a fully
 *           connected xGMI node each transfer has a link of its own) while it
 *           folds its own block, then folds the P-1 received blocks -- int8
 *           byte blocks in one fused launch (knn_ctx_step_shadow_n).
 * Both move the search's shadow form when it has one (int8 byte blocks,
 * fp16 rows: knn_ctx_shadow) and element blocks otherwise; the exact rescan
 * always reads element blocks.
 *
 * The hop is a transport: RCCL over the node's GPUs; or (KNN_RING_LOOPBACK=1)
 * a loopback of P virtual ranks on device 0 whose transfers are device
 * copies on one "fabric" stream; or (KNN_RING_LOOPBACK=rccl) the same P
 * virtual ranks whose every transfer is an RCCL send to self and receive
 * from self on a one-device communicator (ncclCommInitAll with ndev = 1),
 * grouped exactly as the RCCL transport groups a hop or an exchange.  The
 * schedules, buffers, events and lag rule are the same for all three, so the
 * P >= 2 ring -- and its RCCL calls -- run on a one-GPU box
 * (tests/test_gpu_parity.py, tests/test_gpu_rccl_self.py).
 */
#include "knn_internal.h"

#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define KNN_RING_MAX 64
#define NRX (KNN_STEP_LAG + 2)  /* receive buffers per device */

enum { RING_RCCL = 0, RING_LOOPBACK = 1, RING_SELF = 2 };
typedef struct {
    int kind;
    hipStream_t fabric;         /* loopback / self: every hop's transfers, in hop order */
    ncclComm_t self;            /* RING_SELF: the one-device communicator */
    uint32_t *stall_h;          /* KNN_RING_TEST_STALL (loopback): the fabric stream */
    void *stall_d;              /*   waits on this word before its first transfer */
} ring_transport_t;

/* Progress marks: every fold and every transfer group records one (on the
 * stream it ran on); ring_drain's deadline restarts whenever one more of
 * them has completed, so KNN_RING_TIMEOUT_S bounds the time with no fold and
 * no transfer finishing -- a transfer that never lands -- not a pass. */
#define MK_MAX (2 * KNN_RING_MAX + 8)

typedef struct {
    int dev;
    size_t rows, base;          /* own block */
    void *qb;                   /* own packed block: the queries, never overwritten */
    void *qs;                   /* own block in the search's shadow form (or NULL) */
    void **rx;                  /* nrx receive buffers of rx_bytes each: ring NRX,
                                 * direct P - 1 (rx[j-1] <- block g - j) */
    size_t rx_bytes;            /* sized for the form the pass moves (shadow
                                 * or byte blocks); grown to element blocks
                                 * only when a rescan needs them */
    void *cur, *nxt;            /* block being folded / being received */
    int hop;                    /* hops made: hop h lands in rx[h % NRX] */
    double *src;                /* raw rows of the own block */
    double *meta;               /* reduced meta (8 doubles) */
    knn_neighbour_t *d_out;
    knn_ctx_t *ctx;
    hipStream_t cs, ms;         /* compute / comm streams */
    hipEvent_t ev_comp, ev_comm;
    hipEvent_t mk[MK_MAX];      /* progress marks (nmk recorded since the last drain) */
    int nmk, mkn;               /* recorded since the last drain / created */
    ncclComm_t comm;
} ring_dev_t;

static int ring_mark(ring_dev_t *e, hipStream_t s)
{
    if (e->nmk >= e->mkn) return KNN_OK;   /* (a pass records at most 2P) */
    return hipEventRecord(e->mk[e->nmk++], s) == hipSuccess ? KNN_OK : KNN_ERR_HIP;
}

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

/* KNN_RING_TEST_STALL=1 (loopback transport, tests): the fabric stream
 * waits on a host word nobody sets before its transfers, so they never
 * land; ring_drain's timeout sets it when it gives up.  No kernel spins: the
 * wait is the stream's own, and the queue drains once the word is set. */
static int ring_stall_hook(ring_transport_t *t)
{
    if (!t->stall_d) return KNN_OK;
    return hipStreamWaitValue32(t->fabric, t->stall_d, 1, hipStreamWaitValueGte, 0xffffffffu) == hipSuccess
               ? KNN_OK
               : KNN_ERR_HIP;
}

/* Loopback / self hop: virtual rank g's cur -> rank g+1's nxt, all on
 * device 0.  The fabric stream waits for every rank's compute-side event
 * (its nxt is free, its own block is packed) and runs the transfers in hop
 * order, so a block forwarded at hop h was received at hop h-1 on the same
 * stream.  The loopback copies; the self transport moves every block through
 * RCCL (send to self, receive from self). */
static int ring_hop_loopback(ring_dev_t *d, int P, size_t bytes, ring_transport_t *t)
{
    int rc;
    if (hipSetDevice(d[0].dev) != hipSuccess) return KNN_ERR_HIP;
    for (int g = 0; g < P; g++)
        if (hipStreamWaitEvent(t->fabric, d[g].ev_comp, 0) != hipSuccess) return KNN_ERR_HIP;
    if ((rc = ring_stall_hook(t))) return rc;
    if (t->kind == RING_SELF) {
        /* one group, as the RCCL transport's hop: P sends to self and P
         * receives from self on one communicator, matched in posting order
         * (send g pairs with the receive into rank g+1's nxt) */
        if (ncclGroupStart() != ncclSuccess) return KNN_ERR_RCCL;
        for (int g = 0; g < P; g++)
            if (ncclSend(d[g].cur, bytes, ncclUint8, 0, t->self, t->fabric) != ncclSuccess ||
                ncclRecv(d[(g + 1) % P].nxt, bytes, ncclUint8, 0, t->self, t->fabric) != ncclSuccess) {
                ncclGroupEnd();
                return KNN_ERR_RCCL;
            }
        if (ncclGroupEnd() != ncclSuccess) return KNN_ERR_RCCL;
    } else {
        for (int g = 0; g < P; g++)
            if (hipMemcpyAsync(d[(g + 1) % P].nxt, d[g].cur, bytes, hipMemcpyDeviceToDevice, t->fabric) !=
                hipSuccess)
                return KNN_ERR_HIP;
    }
    for (int g = 0; g < P; g++)
        if (hipEventRecord(d[g].ev_comm, t->fabric) != hipSuccess || ring_mark(&d[g], t->fabric))
            return KNN_ERR_HIP;
    return KNN_OK;
}

static int ring_hop(ring_dev_t *d, int P, size_t bytes, ring_transport_t *t)
{
    if (t->kind != RING_RCCL) return ring_hop_loopback(d, P, bytes, t);
    /* nxt[g] was read by step s-1's compute: the comm waits for it. */
    for (int g = 0; g < P; g++) {
        if (hipSetDevice(d[g].dev) != hipSuccess) return KNN_ERR_HIP;
        if (hipStreamWaitEvent(d[g].ms, d[g].ev_comp, 0) != hipSuccess) return KNN_ERR_HIP;
    }
    if (ncclGroupStart() != ncclSuccess) return KNN_ERR_RCCL;
    for (int g = 0; g < P; g++) {
        if (ncclSend(d[g].cur, bytes, ncclUint8, (g + 1) % P, d[g].comm, d[g].ms) != ncclSuccess ||
            ncclRecv(d[g].nxt, bytes, ncclUint8, (g - 1 + P) % P, d[g].comm, d[g].ms) != ncclSuccess) {
            ncclGroupEnd();
            return KNN_ERR_RCCL;
        }
    }
    if (ncclGroupEnd() != ncclSuccess) return KNN_ERR_RCCL;
    for (int g = 0; g < P; g++) {
        if (hipSetDevice(d[g].dev) != hipSuccess) return KNN_ERR_HIP;
        if (hipEventRecord(d[g].ev_comm, d[g].ms) != hipSuccess || ring_mark(&d[g], d[g].ms))
            return KNN_ERR_HIP;
    }
    return KNN_OK;
}

/* Bounded wait (KNN_RING_TIMEOUT_S, default 300 s) for one stream of every
 * device: `comm` = the transfers (the comm streams, or the fabric stream of
 * the loopback / self transports), else the compute streams (the meta
 * all-reduce runs there).  The bound is on progress, not on the pass: the
 * deadline restarts whenever another of the pass's progress marks (one per
 * fold and per transfer group, ring_mark) completes, so a long compute tail
 * of many folds never trips it, a transfer that never lands does.  RCCL and
 * self: polls each communicator's asynchronous error beside the streams, and
 * on an error or the deadline aborts every communicator (the caller then
 * skips ncclCommDestroy and every stream synchronisation) and returns
 * KNN_ERR_RCCL -- a dead peer or a stuck transfer ends the search with a
 * status instead of a hang in a later synchronisation.  Loopback: the same
 * status, with the stream synchronisations skipped likewise. */
static double ring_timeout_s(void)
{
    const char *e = getenv("KNN_RING_TIMEOUT_S");
    const double v = e ? atof(e) : 0.0;
    return v > 0.0 ? v : 300.0;
}

static int ring_marks_done(ring_dev_t *d, int P)
{
    int done = 0;
    for (int g = 0; g < P; g++) {
        if (hipSetDevice(d[g].dev) != hipSuccess) return -1;
        for (int x = 0; x < d[g].nmk; x++) done += hipEventQuery(d[g].mk[x]) == hipSuccess;
    }
    return done;
}

static int ring_drain(ring_dev_t *d, int P, ring_transport_t *t, int comm, int *aborted)
{
    const double tmo = ring_timeout_s();
    double deadline = now_s() + tmo;
    int marks = ring_marks_done(d, P);
    for (;;) {
        int pending = 0, bad = 0;
        if (t->kind != RING_RCCL && comm) {
            if (hipSetDevice(d[0].dev) != hipSuccess) return KNN_ERR_HIP;
            const hipError_t q = hipStreamQuery(t->fabric);
            if (q == hipErrorNotReady) pending = 1;
            else if (q != hipSuccess) return KNN_ERR_HIP;
        } else {
            for (int g = 0; g < P; g++) {
                if (hipSetDevice(d[g].dev) != hipSuccess) return KNN_ERR_HIP;
                const hipError_t q = hipStreamQuery(comm ? d[g].ms : d[g].cs);
                if (q == hipErrorNotReady) pending = 1;
                else if (q != hipSuccess) return KNN_ERR_HIP;
                if (t->kind == RING_RCCL && d[g].comm) {
                    ncclResult_t st = ncclSuccess;
                    if (ncclCommGetAsyncError(d[g].comm, &st) != ncclSuccess ||
                        (st != ncclSuccess && st != ncclInProgress))
                        bad = 1;
                }
            }
        }
        if (t->kind == RING_SELF && t->self) {
            ncclResult_t st = ncclSuccess;
            if (ncclCommGetAsyncError(t->self, &st) != ncclSuccess ||
                (st != ncclSuccess && st != ncclInProgress))
                bad = 1;
        }
        if (!pending && !bad) {
            /* the polled streams are idle; marks recorded on the other kind
             * of stream (compute or comm) may still be pending: keep those
             * (swapped to the front, so no event is lost) and drop only the
             * completed ones, so a later drain still counts their progress */
            for (int g = 0; g < P; g++) {
                if (hipSetDevice(d[g].dev) != hipSuccess) return KNN_ERR_HIP;
                int keep = 0;
                for (int x = 0; x < d[g].nmk; x++)
                    if (hipEventQuery(d[g].mk[x]) != hipSuccess) {
                        hipEvent_t e = d[g].mk[keep];
                        d[g].mk[keep++] = d[g].mk[x];
                        d[g].mk[x] = e;
                    }
                d[g].nmk = keep;
            }
            return KNN_OK;
        }
        const int now_marks = ring_marks_done(d, P);
        if (now_marks > marks) {
            marks = now_marks;
            deadline = now_s() + tmo;
        }
        if (bad || now_s() > deadline) {
            if (t->kind == RING_RCCL) {
                for (int g = 0; g < P; g++)
                    if (d[g].comm) ncclCommAbort(d[g].comm);
            } else if (t->kind == RING_SELF && t->self) {
                ncclCommAbort(t->self);
            }
            if (t->stall_h) {
                /* the test hook's stalled transfer: release it, so the
                 * process ends with its queues drained (tests only) */
                *(volatile uint32_t *)t->stall_h = 1;
                __sync_synchronize();
            }
            *aborted = 1;
            return KNN_ERR_RCCL;
        }
        const struct timespec ts = {0, 50000};   /* 50 us */
        nanosleep(&ts, NULL);
    }
}

static size_t rows_of(int b, size_t R, size_t m)
{
    const size_t base = (size_t)b * R;
    return (base + R <= m) ? R : m - base;
}

/* One step's fold of the block at `blk` (form: 0 element, else shadow) */
static int fold_one(ring_dev_t *e, const void *blk, size_t rows, size_t base, int rescan, int form)
{
    if (rescan) return knn_ctx_rescan_step(e->ctx, blk, rows, base, e->cs);
    return form ? knn_ctx_step_shadow(e->ctx, blk, rows, base, e->cs)
                : knn_ctx_step(e->ctx, blk, rows, base, e->cs);
}

/* Direct exchange: device g's `send` block to every other device, rx[j-1]
 * of device g receiving block g - j, all transfers of all devices in one
 * group (RCCL) or on the fabric stream (loopback); ev_comm marks arrival. */
static int direct_exchange(ring_dev_t *d, int P, size_t bytes, void *const *send, ring_transport_t *t)
{
    int rc;
    if (t->kind != RING_RCCL) {
        if (hipSetDevice(d[0].dev) != hipSuccess) return KNN_ERR_HIP;
        for (int g = 0; g < P; g++)
            if (hipStreamWaitEvent(t->fabric, d[g].ev_comp, 0) != hipSuccess) return KNN_ERR_HIP;
        if ((rc = ring_stall_hook(t))) return rc;
        if (t->kind == RING_SELF) {
            /* the RCCL transport's one group of the whole exchange: P(P-1)
             * sends to self, each followed by the receive it pairs with */
            if (ncclGroupStart() != ncclSuccess) return KNN_ERR_RCCL;
            for (int g = 0; g < P; g++)
                for (int j = 1; j < P; j++)
                    if (ncclSend(send[(g - j + P) % P], bytes, ncclUint8, 0, t->self, t->fabric) != ncclSuccess ||
                        ncclRecv(d[g].rx[j - 1], bytes, ncclUint8, 0, t->self, t->fabric) != ncclSuccess) {
                        ncclGroupEnd();
                        return KNN_ERR_RCCL;
                    }
            if (ncclGroupEnd() != ncclSuccess) return KNN_ERR_RCCL;
        } else {
            for (int g = 0; g < P; g++)
                for (int j = 1; j < P; j++)
                    if (hipMemcpyAsync(d[g].rx[j - 1], send[(g - j + P) % P], bytes, hipMemcpyDeviceToDevice,
                                       t->fabric) != hipSuccess)
                        return KNN_ERR_HIP;
        }
        for (int g = 0; g < P; g++)
            if (hipEventRecord(d[g].ev_comm, t->fabric) != hipSuccess || ring_mark(&d[g], t->fabric))
                return KNN_ERR_HIP;
        return KNN_OK;
    }
    for (int g = 0; g < P; g++) {
        if (hipSetDevice(d[g].dev) != hipSuccess) return KNN_ERR_HIP;
        if (hipStreamWaitEvent(d[g].ms, d[g].ev_comp, 0) != hipSuccess) return KNN_ERR_HIP;
    }
    if (ncclGroupStart() != ncclSuccess) return KNN_ERR_RCCL;
    for (int g = 0; g < P; g++)
        for (int j = 1; j < P; j++)
            if (ncclSend(send[g], bytes, ncclUint8, (g + j) % P, d[g].comm, d[g].ms) != ncclSuccess ||
                ncclRecv(d[g].rx[j - 1], bytes, ncclUint8, (g - j + P) % P, d[g].comm, d[g].ms) !=
                    ncclSuccess) {
                ncclGroupEnd();
                return KNN_ERR_RCCL;
            }
    if (ncclGroupEnd() != ncclSuccess) return KNN_ERR_RCCL;
    for (int g = 0; g < P; g++) {
        if (hipSetDevice(d[g].dev) != hipSuccess) return KNN_ERR_HIP;
        if (hipEventRecord(d[g].ev_comm, d[g].ms) != hipSuccess || ring_mark(&d[g], d[g].ms))
            return KNN_ERR_HIP;
    }
    return KNN_OK;
}

/* One direct pass: exchange (form: 0 element blocks, else the shadow form),
 * every device folds its own block, then the P-1 received ones. */
static int direct_pass(ring_dev_t *d, int P, size_t R, size_t m, size_t n, int dtype, int rescan,
                       int form, ring_transport_t *t, int *aborted)
{
    void *send[KNN_RING_MAX];
    const void *blk[KNN_RING_MAX];
    size_t nc[KNN_RING_MAX], base[KNN_RING_MAX];
    int rc;
    /* the own block is folded while the blocks travel, then the received
     * ones in one fused launch; KNN_RING_FUSE=all folds all P byte blocks in
     * one launch after the exchange */
    const char *fz = getenv("KNN_RING_FUSE");
    const int fuse_all = form && !rescan && P > 1 && knn_ctx_shadow(d[0].ctx) == 2 && fz &&
                         strcmp(fz, "all") == 0;
    const size_t bytes = form ? knn_ctx_shadow_bytes(d[0].ctx, R)
                              : knn_block_bytes_dt(R, n, dtype);
    for (int g = 0; g < P; g++) send[g] = form ? d[g].qs : d[g].qb;
    if (P > 1 && (rc = direct_exchange(d, P, bytes, send, t))) return rc;
    for (int g = 0; g < P && !fuse_all; g++) {
        if (hipSetDevice(d[g].dev) != hipSuccess) return KNN_ERR_HIP;
        if ((rc = fold_one(&d[g], send[g], d[g].rows, d[g].base, rescan, form))) return rc;
        if ((rc = ring_mark(&d[g], d[g].cs))) return rc;
    }
    /* the exchange has landed before the steps that read it are enqueued: a
     * step may synchronise a stream of its own (a growing buffer), which
     * would block on a transfer that never lands; this wait is bounded (the
     * own blocks' folds, enqueued above, run meanwhile) */
    if (P > 1 && (rc = ring_drain(d, P, t, 1, aborted))) return rc;
    for (int g = 0; g < P && P > 1; g++) {
        ring_dev_t *e = &d[g];
        if (hipSetDevice(e->dev) != hipSuccess) return KNN_ERR_HIP;
        if (hipStreamWaitEvent(e->cs, e->ev_comm, 0) != hipSuccess) return KNN_ERR_HIP;
        for (int j = 1; j < P; j++) {
            const int b = (g - j + P) % P;
            blk[j] = e->rx[j - 1];
            base[j] = (size_t)b * R;
            nc[j] = rows_of(b, R, m);
        }
        blk[0] = send[g];
        base[0] = e->base;
        nc[0] = e->rows;
        if (fuse_all) {
            rc = knn_ctx_step_shadow_n(e->ctx, P, blk, nc, base, e->cs);
        } else if (form && !rescan) {
            rc = knn_ctx_step_shadow_n(e->ctx, P - 1, blk + 1, nc + 1, base + 1, e->cs);
        } else if (!rescan) {
            rc = knn_ctx_step_n(e->ctx, P - 1, blk + 1, nc + 1, base + 1, e->cs);
        } else {
            rc = KNN_OK;
            for (int j = 1; j < P && !rc; j++) rc = fold_one(e, blk[j], nc[j], base[j], rescan, form);
        }
        if (rc) return rc;
        if (hipEventRecord(e->ev_comp, e->cs) != hipSuccess || ring_mark(e, e->cs)) return KNN_ERR_HIP;
    }
    return KNN_OK;
}

/* Rescan over the element blocks a direct pass left resident */
static int direct_pass_resident(ring_dev_t *d, int P, size_t R, size_t m)
{
    int rc;
    for (int g = 0; g < P; g++) {
        ring_dev_t *e = &d[g];
        if (hipSetDevice(e->dev) != hipSuccess) return KNN_ERR_HIP;
        if ((rc = knn_ctx_rescan_step(e->ctx, e->qb, e->rows, e->base, e->cs))) return rc;
        for (int j = 1; j < P; j++) {
            const int b = (g - j + P) % P;
            if ((rc = knn_ctx_rescan_step(e->ctx, e->rx[j - 1], rows_of(b, R, m), (size_t)b * R, e->cs)))
                return rc;
        }
    }
    return KNN_OK;
}

/* One full rotation: at step s device g folds block (g - off - s) mod P,
 * where off says how far the blocks have already moved. */
static int ring_pass(ring_dev_t *d, int P, size_t R, size_t m, size_t bytes, int off,
                     int rescan, int form, ring_transport_t *t, int *aborted)
{
    int rc;
    for (int s = 0; s < P; s++) {
        if (s < P - 1 && (rc = ring_hop(d, P, bytes, t))) return rc;
        for (int g = 0; g < P; g++) {
            const int b = ((g - off - s) % P + P) % P;
            const size_t base = (size_t)b * R;
            const size_t rows = rows_of(b, R, m);
            if (hipSetDevice(d[g].dev) != hipSuccess) return KNN_ERR_HIP;
            rc = fold_one(&d[g], d[g].cur, rows, base, rescan, form);
            if (rc) return rc;
            if (hipEventRecord(d[g].ev_comp, d[g].cs) != hipSuccess || ring_mark(&d[g], d[g].cs))
                return KNN_ERR_HIP;
        }
        if (s < P - 1) {
            /* hop s has landed before step s + 1 is enqueued (bounded; as in
             * direct_pass: a step's own stream synchronisation must never
             * wait on a transfer that does not land) */
            if ((rc = ring_drain(d, P, t, 1, aborted))) return rc;
            for (int g = 0; g < P; g++) {
                if (hipSetDevice(d[g].dev) != hipSuccess) return KNN_ERR_HIP;
                if (hipStreamWaitEvent(d[g].cs, d[g].ev_comm, 0) != hipSuccess) return KNN_ERR_HIP;
                /* the own block (queries) only ever leaves; receives
                 * rotate over KNN_STEP_LAG + 2 buffers because
                 * knn_ctx_step orders the compute stream after step
                 * s - KNN_STEP_LAG only (knn.h) */
                d[g].cur = d[g].nxt;
                d[g].hop++;
                d[g].nxt = d[g].rx[d[g].hop % NRX];
            }
        }
    }
    return KNN_OK;
}

/* Receive buffers of at least `bytes` on device e (all nrx of them).  A
 * shadow-form pass sizes them for its shadow blocks (a byte block is 1/8 of
 * an fp64 element block); the rare rescan grows them to element blocks
 * after the device has drained its streams. */
static int ensure_rx(ring_dev_t *e, int nrx, size_t bytes)
{
    if (e->rx_bytes >= bytes) return KNN_OK;
    if (hipSetDevice(e->dev) != hipSuccess) return KNN_ERR_HIP;
    if (e->rx_bytes && (hipStreamSynchronize(e->cs) != hipSuccess || hipStreamSynchronize(e->ms) != hipSuccess))
        return KNN_ERR_HIP;
    for (int b = 0; b < nrx; b++) {
        hipFree(e->rx[b]);
        e->rx[b] = NULL;
    }
    e->rx_bytes = 0;
    for (int b = 0; b < nrx; b++)
        if (hipMalloc(&e->rx[b], bytes) != hipSuccess) return KNN_ERR_NOMEM;
    e->rx_bytes = bytes;
    return KNN_OK;
}

/* Largest P' <= P whose ceil(m/P')-row blocks are all non-empty (results do
 * not depend on the block count; the reference CLIs accept any procs). */
static int ring_blocks_for(size_t m, int P)
{
    if ((size_t)P > m) P = (int)m;
    while (P > 1 && (size_t)(P - 1) * ((m + P - 1) / P) >= m) P--;
    return P < 1 ? 1 : P;
}

int knn_search_ring_host(const double *X, size_t m, size_t n, int layout, int k, int ngpus,
                         int dtype, knn_neighbour_t *out, double *seconds)
{
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return KNN_ERR_NODEVICE;
    if (ngpus < 1) return KNN_ERR_INVALID;
    ring_transport_t tr;
    memset(&tr, 0, sizeof(tr));
    const char *lb = getenv("KNN_RING_LOOPBACK");
    tr.kind = !lb ? RING_RCCL : lb[0] == '1' ? RING_LOOPBACK : strcmp(lb, "rccl") == 0 ? RING_SELF : RING_RCCL;
    /* RCCL: one block per GPU, at most the GPUs present (procs > GPUs runs on
     * every GPU); loopback and self: P virtual ranks on device 0 */
    int P = ngpus;
    if (tr.kind == RING_RCCL && P > ndev) P = ndev;
    if (P > KNN_RING_MAX) P = KNN_RING_MAX;
    P = ring_blocks_for(m, P);
    const size_t R = (m + P - 1) / P;
    const size_t bytes = knn_block_bytes_dt(R, n, dtype);
    if (bytes == 0) return KNN_ERR_INVALID;

    const char *sch = getenv("KNN_RING_SCHEDULE");
    const int direct = !(sch && strcmp(sch, "ring") == 0);
    const int nrx = (direct && P - 1 > NRX) ? P - 1 : NRX;
    ring_dev_t d[KNN_RING_MAX];
    memset(d, 0, sizeof(d));
    int devs[KNN_RING_MAX];
    ncclComm_t comms[KNN_RING_MAX];
    memset(comms, 0, sizeof(comms));
    int rc = KNN_OK, aborted = 0;
    for (int g = 0; g < P; g++) devs[g] = tr.kind == RING_RCCL ? g : 0;
    if (tr.kind == RING_RCCL) {
        if (ncclCommInitAll(comms, P, devs) != ncclSuccess) return KNN_ERR_RCCL;
    } else {
        if (hipSetDevice(0) != hipSuccess ||
            hipStreamCreateWithFlags(&tr.fabric, hipStreamNonBlocking) != hipSuccess)
            return KNN_ERR_HIP;
        if (tr.kind == RING_SELF && ncclCommInitAll(&tr.self, 1, devs) != ncclSuccess) {
            hipStreamDestroy(tr.fabric);
            return KNN_ERR_RCCL;
        }
        const char *st = getenv("KNN_RING_TEST_STALL");
        if (tr.kind == RING_LOOPBACK && st && st[0] == '1') {
            if (hipHostMalloc((void **)&tr.stall_h, 64, hipHostMallocMapped | hipHostMallocCoherent) !=
                    hipSuccess ||
                hipHostGetDevicePointer(&tr.stall_d, tr.stall_h, 0) != hipSuccess) {
                hipStreamDestroy(tr.fabric);
                return KNN_ERR_NOMEM;
            }
            tr.stall_h[0] = 0;
        }
    }

    for (int g = 0; g < P && !rc; g++) {
        ring_dev_t *e = &d[g];
        e->dev = devs[g];
        e->comm = comms[g];
        e->base = (size_t)g * R;
        e->rows = (e->base + R <= m) ? R : m - e->base;
        if (hipSetDevice(e->dev) != hipSuccess) { rc = KNN_ERR_HIP; break; }
        if (hipStreamCreateWithFlags(&e->cs, hipStreamNonBlocking) != hipSuccess ||
            hipStreamCreateWithFlags(&e->ms, hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&e->ev_comp, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&e->ev_comm, hipEventDisableTiming) != hipSuccess) {
            rc = KNN_ERR_HIP;
            break;
        }
        for (e->mkn = 0; e->mkn < 2 * P + 8 && e->mkn < MK_MAX; e->mkn++)
            if (hipEventCreateWithFlags(&e->mk[e->mkn], hipEventDisableTiming) != hipSuccess) {
                rc = KNN_ERR_HIP;
                break;
            }
        if (rc) break;
        const int rx_ok = (e->rx = (void **)calloc((size_t)nrx, sizeof(void *))) != NULL;
        if (!rx_ok || hipMalloc(&e->qb, bytes) != hipSuccess ||
            hipMalloc((void **)&e->src, e->rows * n * sizeof(double)) != hipSuccess ||
            hipMalloc((void **)&e->meta, KNN_META_DOUBLES * sizeof(double)) != hipSuccess ||
            hipMalloc((void **)&e->d_out, e->rows * (size_t)k * sizeof(knn_neighbour_t)) != hipSuccess) {
            rc = KNN_ERR_NOMEM;
            break;
        }
        /* own rows to the device: column-major rows are a 2-D sub-matrix */
        hipError_t he;
        if (layout == KNN_COLMAJOR)
            he = hipMemcpy2D(e->src, e->rows * sizeof(double), X + e->base, m * sizeof(double),
                             e->rows * sizeof(double), n, hipMemcpyHostToDevice);
        else
            he = hipMemcpy(e->src, X + e->base * n, e->rows * n * sizeof(double),
                           hipMemcpyHostToDevice);
        if (he != hipSuccess) { rc = KNN_ERR_HIP; break; }
        rc = knn_ctx_create_dt(&e->ctx, e->dev, e->rows, n, R, k, dtype);
    }
    for (int g = 0; g < P && !rc; g++)
        if (hipSetDevice(d[g].dev) != hipSuccess || hipDeviceSynchronize() != hipSuccess) rc = KNN_ERR_HIP;

    const double t0 = now_s();
    /* pack own block (blk:100-109) and reduce the meta over the ring */
    for (int g = 0; g < P && !rc; g++) {
        ring_dev_t *e = &d[g];
        hipSetDevice(e->dev);
        e->cur = e->qb;
        e->hop = 0;
        rc = knn_block_pack_dt(e->qb, dtype, R, e->rows, n, e->src, KNN_F64,
                               layout == KNN_COLMAJOR ? e->rows : n, layout, e->cs);
        if (!rc && hipMemcpyAsync(e->meta, (char *)e->qb + knn_block_meta_offset_dt(R, n, dtype),
                                  KNN_META_DOUBLES * sizeof(double), hipMemcpyDeviceToDevice,
                                  e->cs) != hipSuccess)
            rc = KNN_ERR_HIP;
    }
    /* the reduced meta, also on the host: it picks the contraction for every
     * rank (knn_ctx_begin_meta, no per-rank read-back) */
    double hm[KNN_META_DOUBLES];
    if (!rc && tr.kind == RING_RCCL) {
        if (ncclGroupStart() != ncclSuccess) rc = KNN_ERR_RCCL;
        for (int g = 0; g < P && !rc; g++)
            if (ncclAllReduce(d[g].meta, d[g].meta, KNN_META_DOUBLES, ncclFloat64, ncclMax,
                              d[g].comm, d[g].cs) != ncclSuccess)
                rc = KNN_ERR_RCCL;
        if (ncclGroupEnd() != ncclSuccess && !rc) rc = KNN_ERR_RCCL;
        if (!rc) rc = ring_drain(d, P, &tr, 0, &aborted);
        if (!rc && (hipSetDevice(d[0].dev) != hipSuccess ||
                    hipMemcpyAsync(hm, d[0].meta, sizeof(hm), hipMemcpyDeviceToHost, d[0].cs) != hipSuccess ||
                    hipStreamSynchronize(d[0].cs) != hipSuccess))
            rc = KNN_ERR_HIP;
    } else if (!rc) {
        /* loopback: max-reduce on the host (meta words are >= 0 or +inf) */
        for (int x = 0; x < KNN_META_DOUBLES; x++) hm[x] = 0.0;
        for (int g = 0; g < P && !rc; g++) {
            double gm[KNN_META_DOUBLES];
            if (hipMemcpyAsync(gm, d[g].meta, sizeof(gm), hipMemcpyDeviceToHost, d[g].cs) != hipSuccess ||
                hipStreamSynchronize(d[g].cs) != hipSuccess) {
                rc = KNN_ERR_HIP;
                break;
            }
            for (int x = 0; x < KNN_META_DOUBLES; x++) hm[x] = gm[x] > hm[x] ? gm[x] : hm[x];
        }
        for (int g = 0; g < P && !rc; g++)
            if (hipMemcpyAsync(d[g].meta, hm, sizeof(hm), hipMemcpyHostToDevice, d[g].cs) != hipSuccess)
                rc = KNN_ERR_HIP;
        /* self: each virtual rank's reduced meta once more through
         * ncclAllReduce(max) on the one-device communicator (the identity
         * over one rank: the call the RCCL transport makes, on its stream) */
        for (int g = 0; g < P && !rc && tr.kind == RING_SELF; g++)
            if (ncclAllReduce(d[g].meta, d[g].meta, KNN_META_DOUBLES, ncclFloat64, ncclMax, tr.self,
                              d[g].cs) != ncclSuccess)
                rc = KNN_ERR_RCCL;
        if (!rc && tr.kind == RING_SELF) rc = ring_drain(d, P, &tr, 0, &aborted);
    }
    /* the form blocks travel in: the search's shadow form when it has one
     * (P > 1; KNN_NO_SHADOW_RING=1 keeps element blocks) */
    const char *nsr = getenv("KNN_NO_SHADOW_RING");
    int form = 0;
    for (int g = 0; g < P && !rc; g++) {
        hipSetDevice(d[g].dev);
        rc = knn_ctx_begin_meta(d[g].ctx, d[g].qb, R, d[g].base, d[g].meta, hm, d[g].cs);
        if (!rc && g == 0) form = P > 1 && knn_ctx_shadow(d[g].ctx) != 0 && !(nsr && nsr[0] == '1');
        if (!rc && form) {
            if (!d[g].qs && hipMalloc(&d[g].qs, knn_ctx_shadow_bytes(d[g].ctx, R)) != hipSuccess)
                rc = KNN_ERR_NOMEM;
            if (!rc) rc = knn_ctx_shadow_pack(d[g].ctx, d[g].qs, d[g].qb, R, d[g].cs);
            d[g].cur = d[g].qs;
        }
        if (!rc) rc = ensure_rx(&d[g], nrx, form ? knn_ctx_shadow_bytes(d[g].ctx, R) : bytes);
        d[g].nxt = d[g].rx[0];
        if (!rc && hipEventRecord(d[g].ev_comp, d[g].cs) != hipSuccess) rc = KNN_ERR_HIP;
    }
    if (!rc && direct)
        rc = direct_pass(d, P, R, m, n, dtype, 0, form, &tr, &aborted);
    else if (!rc)
        rc = ring_pass(d, P, R, m, form ? knn_ctx_shadow_bytes(d[0].ctx, R) : bytes, 0, 0, form, &tr, &aborted);
    /* every transfer of the pass has landed (or the search fails here):
     * knn_ctx_end's synchronisation can then not wait on a stuck hop */
    if (!rc && P > 1) rc = ring_drain(d, P, &tr, 1, &aborted);
    size_t unresolved_total = 0;
    for (int g = 0; g < P && !rc; g++) {
        size_t u = 0;
        hipSetDevice(d[g].dev);
        rc = knn_ctx_end(d[g].ctx, d[g].d_out, &u, d[g].cs);
        if (!rc && u && direct && form && P > 1 && knn_ctx_shadow(d[g].ctx) == 2) {
            /* the byte blocks of the whole corpus are resident (own + P - 1
             * received): the int8 re-search of the uncertified queries runs
             * over them before any element-block exchange */
            const void *sb[KNN_RING_MAX];
            size_t snc[KNN_RING_MAX], sbase[KNN_RING_MAX];
            sb[0] = d[g].qs;
            snc[0] = d[g].rows;
            sbase[0] = d[g].base;
            for (int j = 1; j < P; j++) {
                const int b = (g - j + P) % P;
                sb[j] = d[g].rx[j - 1];
                snc[j] = rows_of(b, R, m);
                sbase[j] = (size_t)b * R;
            }
            rc = knn_ctx_research_blocks(d[g].ctx, P, sb, snc, sbase, d[g].d_out, &u, d[g].cs);
        }
        unresolved_total += u;
    }
    if (!rc && unresolved_total) {
        /* A pass makes P-1 hops, so device g now holds block g+1; rotate
         * once more for the exact rescan of uncertified queries
         * (KNN_FORCE_RESCAN=1: every query, for tests). */
        for (int g = 0; g < P && !rc; g++) {
            hipSetDevice(d[g].dev);
            if (hipEventRecord(d[g].ev_comp, d[g].cs) != hipSuccess) rc = KNN_ERR_HIP;
        }
        for (int g = 0; g < P && !rc; g++) rc = ensure_rx(&d[g], nrx, bytes);
        if (!rc && direct) {
            /* element blocks: exchanged again after a shadow-form pass (the
             * receive buffers held shadow blocks), else still resident */
            rc = form ? direct_pass(d, P, R, m, n, dtype, 1, 0, &tr, &aborted)
                      : direct_pass_resident(d, P, R, m);
        } else if (!rc && form) {
            /* the pass moved shadow blocks: a fresh rotation of element blocks */
            for (int g = 0; g < P; g++) {
                d[g].cur = d[g].qb;
                d[g].nxt = d[g].rx[++d[g].hop % NRX];
            }
            rc = ring_pass(d, P, R, m, bytes, 0, 1, 0, &tr, &aborted);
        } else if (!rc) {
            rc = ring_pass(d, P, R, m, bytes, P - 1, 1, 0, &tr, &aborted);
        }
        if (!rc && P > 1) rc = ring_drain(d, P, &tr, 1, &aborted);
        for (int g = 0; g < P && !rc; g++) {
            hipSetDevice(d[g].dev);
            rc = knn_ctx_rescan_end(d[g].ctx, d[g].d_out, d[g].cs);
        }
    }
    for (int g = 0; g < P && !rc; g++)
        if (hipSetDevice(d[g].dev) != hipSuccess || hipStreamSynchronize(d[g].cs) != hipSuccess) rc = KNN_ERR_HIP;
    if (seconds) *seconds = now_s() - t0;
    for (int g = 0; g < P && !rc; g++) {
        hipSetDevice(d[g].dev);
        if (hipMemcpy(out + d[g].base * (size_t)k, d[g].d_out,
                      d[g].rows * (size_t)k * sizeof(knn_neighbour_t), hipMemcpyDeviceToHost) != hipSuccess)
            rc = KNN_ERR_HIP;
    }

    for (int g = 0; g < P && (!aborted || tr.stall_h); g++) {
        hipSetDevice(d[g].dev);
        if (d[g].cs) hipStreamSynchronize(d[g].cs);
        if (d[g].ms) hipStreamSynchronize(d[g].ms);
    }
    /* (a stalled test transfer was released when the drain gave up) */
    if (tr.fabric && (!aborted || tr.stall_h)) hipStreamSynchronize(tr.fabric);
    for (int g = 0; g < P; g++) {
        hipSetDevice(d[g].dev);
        if (d[g].ctx) knn_ctx_destroy(d[g].ctx);
        hipFree(d[g].qb);
        hipFree(d[g].qs);
        for (int b = 0; b < nrx && d[g].rx; b++) hipFree(d[g].rx[b]);
        free(d[g].rx);
        hipFree(d[g].src);
        hipFree(d[g].meta);
        hipFree(d[g].d_out);
        if (d[g].ev_comp) hipEventDestroy(d[g].ev_comp);
        if (d[g].ev_comm) hipEventDestroy(d[g].ev_comm);
        for (int x = 0; x < MK_MAX; x++)
            if (d[g].mk[x]) hipEventDestroy(d[g].mk[x]);
        if (d[g].cs) hipStreamDestroy(d[g].cs);
        if (d[g].ms) hipStreamDestroy(d[g].ms);
        if (tr.kind == RING_RCCL && comms[g] && !aborted) ncclCommDestroy(comms[g]);
    }
    if (tr.self && !aborted) ncclCommDestroy(tr.self);
    if (tr.fabric) hipStreamDestroy(tr.fabric);
    if (tr.stall_h) hipHostFree(tr.stall_h);
    return rc;
}
