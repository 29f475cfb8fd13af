"""Per-rank corpus-block ring over torch.distributed (RCCL on ROCm).

The multi-process counterpart of knn_ring.c, used when one process drives
one GPU (bench.py under torch.distributed.run).  It replaces the MPI ring of
mpi-knn-parallel_blocking.c:122-244 / _non_blocking.c:132-259:

* rank g owns query rows [g*R, min(m, (g+1)*R)), R = ceil(m/P) (the
  reference uses floor(m/P) and drops the remainder, blk:81);
* step s folds block (g - s) mod P; the hop for step s+1 (isend to g+1,
  irecv from g-1) is posted BEFORE step s's kernels, so the transfer runs
  on RCCL's stream while the current block is contracted (the reference
  waits for every hop before computing);
* the own packed block stays resident as the query block; STEP_LAG + 2
  receive buffers rotate (every rank visits all P blocks exactly once --
  the reference visits r, r-2, ..., r-P and never r-1).  Not
  two: knn_ctx_step orders the caller's stream after step s - STEP_LAG only
  (its distance kernels overlap, include/knn.h), so the hop posted at step
  h may only land in the buffer step h - STEP_LAG - 1 read;
* the block meta is combined with one all_reduce(MAX) of 8 doubles;
* integer data (knn_wire_ok on the reduced meta: max|x| <= 32767) travels
  in the int16 wire form -- a quarter of an fp64 block, half of an fp32
  one -- and each rank unpacks what it receives (bit for bit) into an
  element block for its kernels.  Two wire receive buffers alternate: the
  one a hop lands in was last forwarded one hop earlier (r.wait()) and
  unpacked before that, both ordered on the caller's stream.  At P = 8 an
  fp64 MNIST block is 47 MB, about one contraction step on xGMI; its wire
  form is 12 MB.  KNN_NO_WIRE=1 sends element blocks;
* when the search contracts on fp16 shadow rows (knn_ctx_shadow after
  begin: exact-integer data), the ring moves shadow blocks instead --
  2 bytes an element, folded with knn_ctx_step_shadow, no per-rank unpack
  or conversion; the rare exact rescan then makes one more rotation of
  element blocks.

The engine object does the per-block work (GpuEngine: libknn kernels on the
current HIP stream).  Tests substitute a CPU engine to check the schedule
under gloo.

Failures: a peer that dies or stalls must not hang the survivors.  Every
exchange is waited for with a bound (KNN_RING_TIMEOUT_S, default 300 s; a
full-size P = 8 pass moves ~50 MB a rank and takes milliseconds).  Under
gloo each request's wait carries that timeout, and a failed or stalled peer
raises RingError on the survivors (tests/test_ring_cpu.py injects a stalled
peer).  Under nccl (RCCL) the wait stays a stream-ordered one -- a
host-blocking wait would stall the launch queue behind the transfers -- so
a stalled transfer does not raise here: the bound is the process group's
own timeout, which bench.py sets from the same variable at
init_process_group, and when it expires the RCCL watchdog aborts the
communicator and tears the process down with a non-zero exit (no hang,
but no RingError either).  Errors the nccl work reports at wait() time
still raise RingError.  The nccl branch runs on one GPU through a
world-size-1 RCCL group (tests/test_gpu_rccl_self.py).
"""
import datetime
import os

import numpy as np


class RingError(RuntimeError):
    """A block exchange of the ring failed or timed out on this rank."""


def ring_timeout_s():
    """The bound on one exchange (KNN_RING_TIMEOUT_S, seconds; default 300)."""
    return float(os.environ.get("KNN_RING_TIMEOUT_S", "300"))


def _wait_all(dist, reqs, rank, what, timeout_s):
    backend = None
    gb = getattr(dist, "get_backend", None)
    if gb is not None:
        try:
            backend = gb()
        except Exception:
            backend = None
    for r in reqs:
        try:
            if backend == "gloo":
                r.wait(timeout=datetime.timedelta(seconds=timeout_s))
            else:
                r.wait()
        except Exception as e:   # a dead or stalled peer: fail loudly, never hang
            raise RingError("rank %d: %s failed (%s)" % (rank, what, e)) from e


def partition(m, P):
    """Block b = rows [b*R, min(m, (b+1)*R)), R = ceil(m/P)."""
    R = -(-m // P)
    blocks = []
    for b in range(P):
        lo = min(b * R, m)
        hi = min((b + 1) * R, m)
        blocks.append((lo, hi - lo))
    return R, blocks


class GpuEngine:
    """libknn on one device; buffers are torch uint8 tensors on cuda."""

    def __init__(self, torch, device, n, R, nq, k, dtype="f64"):
        import mpiknn
        self.torch, self.mk = torch, mpiknn
        self.dev = torch.device("cuda", device)
        self.n, self.R, self.nq, self.k, self.dtype = n, R, nq, k, dtype
        nb = mpiknn.block_bytes(R, n, dtype)
        self.qb = torch.zeros(nb, dtype=torch.uint8, device=self.dev)
        self.rx = tuple(torch.empty(nb, dtype=torch.uint8, device=self.dev)
                        for _ in range(mpiknn.STEP_LAG + 2))
        self._wires = None
        self.meta_off = mpiknn.block_meta_offset(R, n, dtype)
        self.meta = self._meta_own = torch.zeros(mpiknn.META_DOUBLES, dtype=torch.float64, device=self.dev)
        self.out = torch.zeros(max(nq, 1) * k * 16, dtype=torch.uint8, device=self.dev)
        self.ctx = mpiknn.Context(device, max(nq, 1), n, R, k, dtype)
        # the speculative byte block (knn_block_pack_s8): tried while the
        # data keeps qualifying (n within the int8 kernel's reach)
        import os
        self.try_s8 = n <= 896 and os.environ.get("KNN_NO_S8", "0") != "1"
        self.spec = False
        self.spec_hint = None      # the host meta of the last search begun from the byte block
        self._meta_pinned = None
        self._src = None
        self.sq = None

    def stream(self):
        return self.torch.cuda.current_stream(self.dev).cuda_stream

    def pack(self, src, layout_col, elements=False):
        """src: this rank's rows on the device, (rows, n) float64 or float32
        (any strides matching the layout: col-major -> src.t() contiguous).
        8-bit integer data: the speculative byte block straight from src
        (self.spec; meta word 7 = 1), else / elements=True the element block."""
        rows = src.shape[0]
        self._src = (src, layout_col)
        self.spec = False
        if rows > 0 and self.try_s8 and not elements:
            if self.sq is None:
                self.sq = self.torch.empty(self.mk.s8_block_bytes(self.R, self.n), dtype=self.torch.uint8,
                                           device=self.dev)
            ld, lay, sdt = self._layout(src, layout_col)
            self.mk.block_pack_s8(self.sq.data_ptr(), self.R, rows, self.n, src.data_ptr(), ld, lay, self.stream(),
                                  dtype=self.dtype, src_dtype=sdt)
            # the meta the search and the ring reduce: the byte block's own
            # words (a view: no copy)
            mo = self.mk.s8_block_meta_offset(self.R, self.n)
            self.meta = self.sq[mo:mo + 8 * self.mk.META_DOUBLES].view(self.torch.float64)
            self.spec = True
            return
        self.meta = self._meta_own
        if rows == 0:
            # a rank past the last row (m < P * ceil(m/P) - R): no queries,
            # an empty block; meta 0 is neutral for the MAX all-reduce
            self.qb.zero_()
            self.meta.zero_()
            return
        ld, lay, sdt = self._layout(src, layout_col)
        self.mk.block_pack(self.qb.data_ptr(), self.R, rows, self.n, src.data_ptr(), ld, lay,
                           self.stream(), dtype=self.dtype, src_dtype=sdt)
        self.meta.copy_(self.qb[self.meta_off:self.meta_off + 8 * self.mk.META_DOUBLES]
                        .view(self.torch.float64))

    def _layout(self, src, layout_col):
        if layout_col:
            assert src.stride(0) == 1
            return src.stride(1), self.mk.COLMAJOR, ("f32" if src.dtype == self.torch.float32 else "f64")
        assert src.stride(1) == 1
        return src.stride(0), self.mk.ROWMAJOR, ("f32" if src.dtype == self.torch.float32 else "f64")

    def meta_host(self, meta):
        """an asynchronous read-back of meta into pinned host memory (valid
        once the current stream has passed this point)"""
        if self._meta_pinned is None:
            self._meta_pinned = self.torch.empty(self.mk.META_DOUBLES, dtype=self.torch.float64, pin_memory=True)
        self._meta_pinned.copy_(meta, non_blocking=True)
        return self._meta_pinned

    def pack_elements(self):
        """the element block of the last pack's source into qb (the exact
        rescan reads it; the reduced meta in self.meta is left as it is)"""
        src, layout_col = self._src
        if src.shape[0] == 0:
            self.qb.zero_()
            return
        ld, lay, sdt = self._layout(src, layout_col)
        self.mk.block_pack(self.qb.data_ptr(), self.R, src.shape[0], self.n, src.data_ptr(), ld, lay,
                           self.stream(), dtype=self.dtype, src_dtype=sdt)

    def wires(self, count=3):
        """own wire block + wire receive buffers (at least `count` in all,
        allocated on first use)"""
        if self._wires is None or len(self._wires) < count:
            wb = self.mk.wire_bytes(self.R, self.n, self.dtype)
            self._wires = tuple(self.torch.empty(wb, dtype=self.torch.uint8, device=self.dev)
                                for _ in range(max(3, count)))
        return self._wires

    def recv_buffers(self, count):
        """`count` element-block receive buffers (the direct exchange keeps
        every other rank's block resident: P - 1 of them)"""
        if len(self.rx) < count:
            nb = self.mk.block_bytes(self.R, self.n, self.dtype)
            self.rx = self.rx + tuple(self.torch.empty(nb, dtype=self.torch.uint8, device=self.dev)
                                      for _ in range(count - len(self.rx)))
        return self.rx[:count]

    def wire_pack(self, wire):
        self.mk.wire_pack(wire.data_ptr(), self.qb.data_ptr(), self.R, self.n, self.dtype,
                          self.stream())

    def wire_unpack(self, buf, wire):
        self.mk.wire_unpack(buf.data_ptr(), wire.data_ptr(), self.R, self.n, self.dtype,
                            self.stream())

    def begin(self, q_base, h_meta=None):
        if self.spec:
            self.ctx.begin_s8(self.sq.data_ptr(), self.R, q_base, self.meta.data_ptr(), h_meta, self.stream())
            return
        self.ctx.begin(self.qb.data_ptr(), self.R, q_base, self.meta.data_ptr(), self.stream(),
                       h_meta=h_meta)

    def attach_elements(self):
        """before an exact rescan of a search begun from the byte block"""
        if self.spec:
            self.pack_elements()
            self.ctx.attach_qblock(self.qb.data_ptr(), self.R)

    def shadow_bytes(self):
        return self.ctx.shadow_bytes(self.R)

    def shadow_block(self):
        """own shadow block in the search's form (knn_ctx_shadow_pack of the
        packed own block: fp16 rows or the int8 byte block; the speculative
        byte block itself when the search began from it)"""
        if self.spec:
            return self.sq
        sb = self.ctx.shadow_bytes(self.R)
        if getattr(self, "_sqb", None) is None or self._sqb.numel() != sb:
            self._sqb = self.torch.empty(sb, dtype=self.torch.uint8, device=self.dev)
        self.ctx.shadow_pack(self._sqb.data_ptr(), self.qb.data_ptr(), self.R, self.stream())
        return self._sqb

    def step_shadow(self, sbuf, rows, base):
        self.ctx.step_shadow(sbuf.data_ptr(), rows, base, self.stream())

    def step_shadow_n(self, sbufs, rows, bases):
        self.ctx.step_shadow_n([b.data_ptr() for b in sbufs], rows, bases, self.stream())

    def step_n(self, bufs, rows, bases):
        self.ctx.step_n([b.data_ptr() for b in bufs], rows, bases, self.stream())

    def step(self, buf, rows, base, rescan=False):
        if rescan:
            self.ctx.rescan_step(buf.data_ptr(), rows, base, self.stream())
        else:
            self.ctx.step(buf.data_ptr(), rows, base, self.stream())

    def end(self):
        return self.ctx.end(self.out.data_ptr(), self.stream())

    def research(self, sbufs, rows, bases):
        """int8 re-search of the queries end() left uncertified against the
        byte blocks this rank holds (knn_ctx_research_blocks); returns the
        count still unresolved"""
        return self.ctx.research_blocks([b.data_ptr() for b in sbufs], rows, bases, self.out.data_ptr(),
                                        self.stream())

    def rescan_end(self):
        self.ctx.rescan_end(self.out.data_ptr(), self.stream())

    def result(self):
        host = self.out.cpu().numpy()
        return host.view(self.mk.NB_DTYPE).reshape(-1, self.k)[: self.nq]


def ring_search(dist, torch, engine, rank, P, m, q_base, schedule=None, timeout_s=None):
    """Run the ring on this rank.  `engine` holds the packed own block
    (engine.pack done).  Collective calls: all_reduce(meta), the block
    exchange of each pass, all_reduce(unresolved).  Returns the number of
    queries that took the exact rescan pass on this rank.

    schedule (default: KNN_RING_SCHEDULE, else "direct"):
      "ring"    P-1 hops to the right neighbour, one block folded per hop
                (the reference's rotation, blk:187-244 / nb:196-259);
      "direct"  every rank sends its block to every other rank at once --
                P-1 point-to-point transfers, each on the xGMI link joining
                the two GPUs of a fully connected node -- while the own block
                is folded; the P-1 received blocks are then folded together
                (one fused int8 launch for byte blocks, knn_ctx_step_shadow_n).
                A ring hop carries one block over one link per step; the
                direct exchange spreads the same bytes over all seven links of
                an 8-GPU node in the time of one hop.

    The default is "direct": both schedules are bit-identical and run the
    same P2P primitive (batch_isend_irecv = one RCCL group), the direct one
    in one group of 2(P-1) operations a rank, which needs no ordering across
    groups (tested under gloo at P = 2..8 and through the one-GPU loopback
    at P = 2..12).  Neither has run over RCCL with P > 1 yet: set
    KNN_RING_SCHEDULE=ring to fall back to the reference's rotation.

    timeout_s bounds every exchange wait (default ring_timeout_s()); a
    failed or stalled peer raises RingError (module docstring)."""
    if timeout_s is None:
        timeout_s = ring_timeout_s()
    if schedule is None:
        schedule = os.environ.get("KNN_RING_SCHEDULE", "direct")
    if schedule not in ("ring", "direct"):
        raise ValueError("unknown ring schedule %r" % (schedule,))
    R, blocks = partition(m, P)
    ctx = getattr(engine, "ctx", None)
    if ctx is not None and hasattr(ctx, "set_solo"):
        # P = 1 folds one block in one step: kernel and merge on the caller's
        # stream, no cross-stream events (knn_ctx_set_solo)
        ctx.set_solo(P == 1)
    wire = False
    h_meta = None
    verify = None
    ring_hint = None
    if P > 1:
        dist.all_reduce(engine.meta, op=dist.ReduceOp.MAX)
        ring_hint = getattr(engine, "ring_hint", None)
        if ring_hint is not None and hasattr(engine, "meta_host"):
            # the reduced meta of this engine's last search as the hint (the
            # same data, search after search): the contraction is chosen from
            # it at once, the device-side reduction orders the kernels (under
            # nccl the all-reduce is stream-ordered, no host wait), and its
            # result is read back behind the search and checked after end()
            # -- a mismatch (new data) runs the search again, on every rank
            # alike: the reduced meta and the hint are the same everywhere
            h_meta = ring_hint
            verify = True   # (read back behind the pass's steps, below)
        else:
            h_meta = engine.meta.cpu().numpy()   # the ring needs it on the host anyway
    spec = getattr(engine, "spec", False)
    if h_meta is None and spec:
        hint = getattr(engine, "spec_hint", None)
        if hint is not None:
            # P = 1 and the last search's meta accepted the byte block: start
            # without waiting for this one's read-back (the host would sit in
            # a stream sync while the GPU idles); the meta is read back
            # behind the search and checked after it -- on a mismatch the
            # search runs again from the element block
            h_meta = hint
            verify = True   # (read back behind the pass's steps, below)
        else:
            h_meta = engine.meta.cpu().numpy()   # (P = 1: begin would read it back anyway)
    if h_meta is not None and h_meta[7] != 0.0 and not engine.mk.s8_spec_ok(h_meta, engine.n, engine.dtype):
        # some rank packed the speculative byte block (meta word 7) and the
        # reduced meta rejects it: every rank packs its element block and
        # the meta is reduced again (the decision is the same on every rank)
        if spec:
            engine.pack(engine._src[0], engine._src[1], elements=True)
            engine.try_s8 = False   # this data does not qualify: straight to elements next time
        spec = False
        if P > 1:
            dist.all_reduce(engine.meta, op=dist.ReduceOp.MAX)
            h_meta = engine.meta.cpu().numpy()
        else:
            h_meta = None
    if P > 1:
        wire = (os.environ.get("KNN_NO_WIRE", "0") != "1" and hasattr(engine, "wires") and
                engine.mk.wire_ok(h_meta))
    engine.begin(q_base, h_meta=h_meta)
    if spec and P == 1 and verify is None:
        engine.spec_hint = h_meta
    # byte / fp16 shadow blocks are what the steps fold (and the ring moves);
    # at P = 1 only a search begun from the byte block folds it explicitly
    shadow = ((P > 1 or spec) and hasattr(engine, "step_shadow") and engine.ctx.shadow() != 0 and
              os.environ.get("KNN_NO_SHADOW_RING", "0") != "1")

    rx = engine.rx
    # cur: the block folded next; send: what goes on the link
    state = {"cur": engine.qb, "send": engine.qb, "hop": 0}
    if shadow:
        sb = engine.shadow_bytes()
        own_s = engine.shadow_block()
        srx = tuple(b[:sb] for b in rx)      # shadow blocks fit the element buffers
        state["cur"] = state["send"] = own_s
    if wire:
        ws = engine.wires(P if schedule == "direct" else 3)
        own_w, wa, wb = ws[0], ws[1], ws[2]
    if wire and not shadow:
        engine.wire_pack(own_w)
        state["send"] = own_w

    def one_pass(off, rescan):
        use_shadow = shadow and not rescan
        use_wire = wire and not use_shadow
        for s in range(P):
            reqs = []
            if s < P - 1:
                h = state["hop"]
                nxt = (srx if use_shadow else rx)[h % len(rx)]
                land = ((wa, wb)[h % 2]) if use_wire else nxt
                ops = [dist.P2POp(dist.isend, state["send"], (rank + 1) % P),
                       dist.P2POp(dist.irecv, land, (rank - 1) % P)]
                reqs = dist.batch_isend_irecv(ops)
            b = (rank - off - s) % P
            base, rows = blocks[b]
            if rows == 0:
                pass   # an empty block (partition: m < P * R) is not folded
            elif use_shadow:
                engine.step_shadow(state["cur"], rows, base)
            else:
                engine.step(state["cur"], rows, base, rescan)
            _wait_all(dist, reqs, rank, "ring hop %d" % s, timeout_s)
            if s < P - 1:
                if use_wire:
                    engine.wire_unpack(nxt, land)
                state["cur"] = nxt
                state["send"] = land
                state["hop"] += 1

    def recv_bufs(count):
        if hasattr(engine, "recv_buffers"):
            return engine.recv_buffers(count)
        return tuple(torch.empty_like(engine.rx[0]) for _ in range(count))

    def direct_pass(rescan, resident):
        """own block first, then the P-1 others, received all at once.
        resident: element blocks already held from the first pass (rescan)"""
        use_shadow = shadow and not rescan
        use_wire = wire and not use_shadow
        own = own_s if use_shadow else engine.qb
        peers = [(rank - j) % P for j in range(1, P)]   # buffer j-1 holds block rank - j
        reqs, land, ebufs = [], [], []
        if resident is None and P > 1:
            ebufs = recv_bufs(P - 1)
            if use_shadow:
                land = [b[:sb] for b in ebufs]
            elif use_wire:
                land = list(engine.wires(P)[1:P])
            else:
                land = list(ebufs)
            send = own_w if use_wire else own
            if use_wire and rescan:   # the first pass moved shadow blocks
                engine.wire_pack(own_w)
            ops = []
            for j in range(1, P):
                ops.append(dist.P2POp(dist.isend, send, (rank + j) % P))
                ops.append(dist.P2POp(dist.irecv, land[j - 1], (rank - j) % P))
            reqs = dist.batch_isend_irecv(ops)
        base, rows = blocks[rank]
        # the own block is folded while the other blocks travel, then the
        # received ones in one fused launch ("rest"); KNN_RING_FUSE=all waits
        # for the exchange and folds all P blocks in one launch (the same
        # compute time in the P = 4 / 8 emulation, the exchange exposed)
        fuse = os.environ.get("KNN_RING_FUSE", "rest")
        fuse_all = (use_shadow and fuse == "all" and P > 1 and resident is None and
                    engine.ctx.shadow() == 2)
        if fuse_all or rows == 0:
            pass   # (an empty own block is not folded)
        elif use_shadow:
            engine.step_shadow(own, rows, base)
        else:
            engine.step(own, rows, base, rescan)
        _wait_all(dist, reqs, rank, "direct exchange", timeout_s)
        if resident is not None:
            fold = resident
        elif use_wire:
            fold = list(ebufs)
            for j in range(P - 1):
                engine.wire_unpack(fold[j], land[j])
        else:
            fold = land
        bs = [blocks[b] for b in peers]
        # empty blocks (m < P * R leaves the last ranks without rows) are
        # exchanged like the others but never folded
        nz = [(buf, b, r) for buf, (b, r) in zip(fold, bs) if r > 0]
        if fuse_all:
            if rows > 0:
                nz = [(own, base, rows)] + nz
            engine.step_shadow_n([x for x, _, _ in nz], [r for _, _, r in nz], [b for _, b, _ in nz])
        elif use_shadow and len(nz) > 0:
            engine.step_shadow_n([x for x, _, _ in nz], [r for _, _, r in nz], [b for _, b, _ in nz])
        elif not rescan and len(nz) > 1 and hasattr(engine, "step_n"):
            # element blocks (real-valued data: one fused split-filter step)
            engine.step_n([x for x, _, _ in nz], [r for _, _, r in nz], [b for _, b, _ in nz])
        else:
            for buf, b, r in nz:
                engine.step(buf, r, b, rescan)
        if use_shadow:
            # every block of the corpus stays resident in the search's form:
            # the int8 re-search of uncertified queries runs over them
            held_s[:] = ([(own, base, rows)] if rows > 0 else []) + [x for x in nz if x[0] is not own]
            return None
        return fold

    held_s = []
    if schedule == "direct":
        held = direct_pass(False, None)
    else:
        one_pass(0, False)
    if verify is True:
        if P == 1 and hasattr(ctx, "search_meta"):
            # the search's last kernel copies the meta it read into mapped
            # memory (knn_ctx_search_meta): no read-back copy on the stream
            verify = "search_meta"
        else:
            # the meta's read-back, enqueued behind the steps: on the
            # caller's stream it would sit between the pack and the search's
            # first kernel (a 6 us copy on the critical path); end() waits
            verify = engine.meta_host(engine.meta)
    unresolved = engine.end()
    if isinstance(verify, str):
        verify = ctx.search_meta()
    if (unresolved > 0 and held_s and P > 1 and hasattr(engine, "research") and engine.ctx.shadow() == 2):
        # a ring rank's uncertified queries: searched again on the int8
        # contraction (65-entry lists) over the byte blocks it holds, before
        # any element-block exchange for the exact rescan
        unresolved = engine.research([x for x, _, _ in held_s], [r for _, _, r in held_s],
                                     [b for _, b, _ in held_s])
    if verify is not None and P == 1:
        # (the read-back was enqueued on the caller's stream before end(),
        # which waits for that stream: it has landed)
        if not engine.mk.s8_spec_ok(verify.numpy() if hasattr(verify, "numpy") else np.asarray(verify),
                                    engine.n, engine.dtype):
            engine.spec_hint = None   # not this data: the checked path, from the start
            return ring_search(dist, torch, engine, rank, P, m, q_base, schedule, timeout_s)
    if verify is not None and P > 1:
        if not np.array_equal(np.asarray(verify.numpy() if hasattr(verify, "numpy") else verify), ring_hint):
            engine.ring_hint = None   # new data: again, from the reduced meta itself
            return ring_search(dist, torch, engine, rank, P, m, q_base, schedule, timeout_s)
    if P > 1 and h_meta is not None and hasattr(engine, "meta_host"):
        engine.ring_hint = np.array(h_meta, dtype=np.float64, copy=True)
    total = unresolved
    if P > 1:
        # (a buffer kept on the engine: filled in place, no host-to-device
        # copy a pass)
        t = getattr(engine, "_unres_buf", None)
        if t is None or t.device != engine.meta.device:
            t = engine._unres_buf = torch.zeros(1, dtype=torch.float64, device=engine.meta.device)
        t.fill_(float(unresolved))
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        total = int(t.item())
    if total > 0 and spec:
        engine.attach_elements()   # the exact rescan reads element blocks
    if total > 0 and schedule == "direct":
        # element blocks still resident unless the pass moved shadow blocks
        direct_pass(True, held)
        engine.rescan_end()
    elif total > 0:
        if shadow:
            # the rescan needs element rows: a fresh rotation from the own block
            state.update(cur=engine.qb, send=engine.qb)
            if wire:
                engine.wire_pack(own_w)
                state["send"] = own_w
            one_pass(0, True)
        else:
            one_pass(P - 1, True)
        engine.rescan_end()
    return unresolved
