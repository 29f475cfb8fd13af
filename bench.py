#!/usr/bin/env python3
"""bench.py -- all-kNN queries/sec on MI355X (BASELINE.json metric).

Workload (default, BASELINE.json configs[1]/[2]): all-kNN, k = 30, fp64,
over an MNIST-784-shaped corpus of m = 60000 rows (synthetic integer pixels
0..255 -- no dataset can be fetched; see mpiknn/synth.py), leave-one-out
(exact zero distances excluded) like knn-serial.c:72-93.  One "step" = one
full all-kNN pass with the corpus already resident in HBM (column-major, the
.mat layout): pack -> ring of P corpus blocks (k_dist_topk + k_merge per
block) -> finalize (+ exact rescan if any query needs it).
value = m / step time (whole job).

--workload mnist-real: the same shape real-valued (mnist_like / 255 + N(0,
1e-3)), so the GEMM mode runs: the split-fp16 filter (S x = hi + lo, three
fp16 MFMAs a product, fp64 accumulation) + the exact fp64 re-rank and
certificate (KNN_NO_SPLIT=1: the fp64 MFMA filter instead).
--workload sift: configs[3], 1M x 128 fp32 k = 32 (SIFT-like integers,
row-major fvecs layout).  --workload gist: configs[4]'s shape, n = 960 fp32
k = 100, with m = 500000 by default (configs[4] is 4M rows on 8 GPUs; pass
--m 4000000 for the full size).  Both run the fp32 path (include/knn.h).

  python bench.py [--gpus N --steps K --warmup W] [--workload mnist|mnist-real|sift|gist]
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

N > 1: one process per GPU, RCCL (torch.distributed "nccl") ring of corpus
blocks, strong scaling (total work fixed).  Rank 0 prints one JSON line.
Under a launcher (WORLD_SIZE set) --gpus must equal WORLD_SIZE; without one,
--gpus N starts the N rank processes itself (launch_ranks) and exits
non-zero when fewer than N GPUs are visible.
"""
import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "mpi-knn_amd"))

FP64_MFMA_PEAK_TFLOPS = 78.6   # MI355X dense fp64 matrix (spec; 78.2 measured, tools/probe)
FP32_MFMA_PEAK_TFLOPS = 157.3  # dense fp32 matrix (spec, MI355X_MICROARCH.md; 155 measured)
FP16_MFMA_PEAK_TFLOPS = 2500.0  # dense fp16 matrix (spec ~2.5 PF, MI355X_MICROARCH.md)
I8_MFMA_PEAK_TOPS = 5000.0      # dense int8 matrix: 2x the fp16 rate per clock (MI355X_MICROARCH.md)
HBM_PEAK_GBS = 8000.0           # HBM3E, ~8 TB/s (MI355X_MICROARCH.md)

METRIC = "all-kNN queries/sec (MNIST-784, k=30) at 1/2/4/8 GPUs + % MFMA peak"   # BASELINE.json

WORKLOADS = {
    # name: (m, n, k, dtype, layout_col, description)
    "mnist": (60000, 784, 30, "f64", True,
              "all-kNN MNIST-784 k=%d (configs[1]: %dx%d fp64, leave-one-out)"),
    # configs[1] on real-valued rows (mnist_train_svd.mat is
    # real-valued): GEMM mode, split-fp16 filter (k_dist_split) + exact fp64
    # re-rank in k_merge
    "mnist-real": (60000, 784, 30, "f64", True,
                   "all-kNN MNIST-784 real-valued k=%d (configs[1] shape: %dx%d fp64, GEMM mode)"),
    "sift": (1_000_000, 128, 32, "f32", False,
             "all-kNN SIFT-like k=%d (configs[3]: %dx%d fp32, integer-valued)"),
    "gist": (500_000, 960, 100, "f32", False,
             "all-kNN GIST-like k=%d (configs[4] shape: %dx%d fp32, real-valued)"),
}


def cpu_baseline(X, k, budget_s):
    """The oracle (oracle/knn_oracle.c, a C port of serial:72-93 with OpenMP
    over queries) on a bounded sample of the same workload: the first q
    queries against the full corpus, q sized to ~budget_s of CPU time."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or os.cpu_count()
    q = 4 * threads
    while True:
        t0 = time.perf_counter()
        oracle.knn(X, k, rows=(0, q), nthreads=threads)
        dt = time.perf_counter() - t0
        if dt >= 0.5 * budget_s or q >= X.shape[0]:
            break
        q = int(min(X.shape[0], max(2 * q, q * budget_s / max(dt, 1e-3))))
    return {"value": q / dt, "unit": "queries/s", "cores": threads, "kind": "port",
            "sample": "%d of %d queries against the full %dx%d corpus (oracle/knn_oracle.c, "
                      "OpenMP over queries, %.1f s)" % (q, X.shape[0], X.shape[0], X.shape[1], dt)}


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n_ranks):
    """`--gpus N` (N > 1) with no launcher around us (WORLD_SIZE unset): start
    N rank processes of this script, torch.distributed.run-style env (RANK,
    LOCAL_RANK, WORLD_SIZE, MASTER_ADDR=127.0.0.1, MASTER_PORT), one per GPU,
    and return the first failing rank's exit code (0 when all succeed).  The
    reference takes its rank count from the launch the same way
    (mpi-knn-parallel_blocking.c:53-61: MPI_Comm_size of mpiexec -n P).

    This parent touches no GPU: it only counts the devices (which does not
    initialise HIP on this image) and refuses, with a non-zero exit, to start
    more ranks than there are GPUs -- a P = 1 line under an n_gpus = N request
    is never printed.  The ranks are children (no exec)."""
    import subprocess
    if not os.environ.get("KNN_BENCH_TEST_ENGINE"):
        import torch
        visible = torch.cuda.device_count()
        if visible < n_ranks:
            print("bench.py: --gpus %d needs %d visible GPUs, %d found; not running" % (n_ranks, n_ranks, visible),
                  file=sys.stderr, flush=True)
            return 2
    port = _free_port()
    procs = []
    for r in range(n_ranks):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n_ranks),
                   LOCAL_WORLD_SIZE=str(n_ranks), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   KNN_BENCH_LAUNCHER="bench.py")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc, live = 0, list(procs)
    while live:
        for p in list(live):
            c = p.poll()
            if c is None:
                continue
            live.remove(p)
            if c != 0 and rc == 0:
                # a failed rank ends the job: its peers would block in the
                # next collective until the group's timeout
                rc = c if c > 0 else 128 - c
                print("bench.py: rank %d exited with %d; stopping the others" % (procs.index(p), c),
                      file=sys.stderr, flush=True)
                for q in live:
                    q.terminate()
        time.sleep(0.1)
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); default: WORLD_SIZE under a launcher, else 1")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="mnist")
    ap.add_argument("--m", type=int, default=None)
    ap.add_argument("--n", type=int, default=None)
    ap.add_argument("--k", type=int, default=None)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--check", type=int, default=8, help="queries re-checked against the oracle")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    ap.add_argument("--secondary-steps", type=int, default=3,
                    help="mnist: also time the real-valued GEMM path this many steps (0: off)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ:
        if args.gpus is not None and args.gpus > 1:
            sys.exit(launch_ranks(args.gpus))
        if args.gpus is not None and args.gpus < 1:
            sys.exit("bench.py: --gpus must be >= 1")
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus is None:
        args.gpus = world
    if world != args.gpus:
        # the line's n_gpus is the ranks that ran: never a P = 1 line for an
        # N-GPU request, nor the reverse
        sys.exit("bench.py: --gpus %d but the launcher started %d ranks (WORLD_SIZE)" % (args.gpus, world))
    # KNN_BENCH_TEST_ENGINE=module:factory (tests/bench_standin.py only): a CPU
    # stand-in engine under gloo, so the multi-rank bench path runs in the
    # CPU test suite; the product bench always runs libknn on the GPU
    test_engine = os.environ.get("KNN_BENCH_TEST_ENGINE")
    import torch
    if test_engine:
        import importlib
        mod, attr = test_engine.split(":")
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        args.engine_factory = getattr(importlib.import_module(mod), attr)
        backend = "gloo"
    else:
        args.engine_factory = None
        backend = "nccl"
        visible = torch.cuda.device_count()
        if local >= visible:
            sys.exit("bench.py: rank %d needs GPU %d, %d visible" % (rank, local, visible))
        torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import datetime
        import torch.distributed as dist
        from mpiknn.ring import ring_timeout_s
        # a stalled or dead peer ends the run (RCCL watchdog) instead of
        # hanging it: the bound of every ring exchange (mpiknn/ring.py)
        kw = {} if test_engine else {"device_id": torch.device("cuda", local)}
        dist.init_process_group(backend, timeout=datetime.timedelta(seconds=ring_timeout_s()), **kw)
    P = world
    args.backend = backend if dist is not None else None

    res = run_workload(args.workload, args.steps, args.warmup, args, torch, dist, rank, P, local,
                       args.check, args.m, args.n, args.k)
    # configs[1]'s real-valued form (mnist_train_svd.mat): the
    # GEMM-mode contraction (split-fp16 filter + exact fp64 re-rank), timed by
    # the same clock a few steps, reported beside the int8 headline
    secondary = None
    if args.workload == "mnist" and args.secondary_steps > 0:
        secondary = run_workload("mnist-real", args.secondary_steps, 1, args, torch, dist, rank, P, local,
                                 min(args.check, 4), None, None, None)
    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return
    out = res["line"]
    if secondary is not None:
        sl = secondary["line"]
        out["secondary"] = {"label": "secondary: real-valued rows, GEMM mode -- split-fp16 filter + exact fp64 "
                                     "re-rank (not the headline)",
                            "workload": sl["config"]["workload"], "value": sl["value"], "unit": sl["unit"],
                            "ms_per_step": sl["ms_per_step"], "steps": sl["steps"], "warmup": sl["warmup"],
                            "engine": sl["engine"], "check": sl["check"],
                            "check_all_rows": sl["check_all_rows"], "roofline": sl["roofline"]}
    if P == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(res["X"].astype(np.float64, copy=False), res["k"], args.cpu_seconds)
    print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def run_workload(workload, steps, warmup, args, torch, dist, rank, P, local, ncheck, m_arg, n_arg, k_arg):
    """Time `steps` all-kNN passes of one workload on this rank (after
    `warmup` untimed ones), barrier + synchronize on both sides, the max
    over ranks; returns the JSON line (rank 0) and the corpus."""
    import mpiknn
    import mpiknn.ring as ring
    from mpiknn import synth

    m0, n0, k0, dtype, layout_col, wdesc = WORKLOADS[workload]
    m = m_arg or m0
    n = n_arg or n0
    k = k_arg or k0
    if workload == "mnist":
        X, _ = synth.mnist_like(m, n)
        data = "synthetic (MNIST-784 shape, integer pixels 0..255, seed 1234)"
    elif workload == "mnist-real":
        X, _ = synth.mnist_real(m, n)
        data = "synthetic (MNIST-784 shape / 255 + N(0, 1e-3): real-valued fp64)"
    elif workload == "sift":
        X = synth.sift_like(m, n)
        data = "synthetic (SIFT-like: 1024-centre mixture, integers 0..255, fp32)"
    else:
        X = synth.gist_like(m, n)
        data = "synthetic (GIST-like: 256-centre mixture in [0,1), fp32)"
    R, blocks = ring.partition(m, P)
    base, rows = blocks[rank]
    standin = args.engine_factory is not None
    dev = torch.device("cpu") if standin else torch.device("cuda", local)
    if layout_col:
        # own rows, column-major on the device (the .mat layout, serial:82)
        raw = torch.from_numpy(np.ascontiguousarray(X[base:base + rows].T)).to(dev).t()
    else:
        raw = torch.from_numpy(np.ascontiguousarray(X[base:base + rows])).to(dev)
    if standin:
        engine = args.engine_factory(torch, n, R, rows, k, dtype)
    else:
        engine = ring.GpuEngine(torch, local, n, R, rows, k, dtype=dtype)

    def step():
        engine.pack(raw, layout_col=layout_col)
        return ring.ring_search(dist, torch, engine, rank, P, m, base)

    def sync():
        if not standin:
            torch.cuda.synchronize()

    def barrier():
        sync()
        if dist is not None:
            if standin:
                dist.barrier()
            else:
                dist.barrier(device_ids=[local])
        sync()

    last = [time.perf_counter()]

    def progress(what):
        # keeps long runs visibly alive (stderr, rank 0, at most every 20 s)
        now = time.perf_counter()
        if rank == 0 and now - last[0] > 20.0:
            print("[bench] %s %s" % (workload, what), file=sys.stderr, flush=True)
            last[0] = now

    for i in range(warmup):
        step()
        progress("warmup %d/%d" % (i + 1, warmup))
    unresolved = 0
    barrier()
    t0 = time.perf_counter()
    for i in range(steps):
        unresolved += step()
        progress("step %d/%d" % (i + 1, steps))
    barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    # the roofline's kernel time: the same step again with the HIP timing
    # events on (knn_ctx_profile), outside the timed region -- each event
    # record sits on the launch queues, so they stay out of ms_per_step
    prof_steps = min(steps, 5)
    engine.ctx.profile(1)
    pack_evs = []
    for i in range(prof_steps):
        if standin:
            step()
        else:
            # the pack runs on the caller's (torch's current) stream: timed
            # there with torch events
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            engine.pack(raw, layout_col=layout_col)
            e1.record()
            pack_evs.append((e0, e1))
            ring.ring_search(dist, torch, engine, rank, P, m, base)
        progress("profiled step %d/%d" % (i + 1, prof_steps))
    barrier()
    dist_ms, merge_ms, launches = engine.ctx.profile(0)
    mk_ms, mk_n, mk_bytes = engine.ctx.profile_merge() if not standin else (0.0, 0, 0.0)
    pack_ms = sum(e0.elapsed_time(e1) for e0, e1 in pack_evs) / max(len(pack_evs), 1)
    # the pack's algorithmic bytes: the rank's rows read once in the source
    # precision, written once as the byte block (8-bit data: round_up(n, 32)
    # bytes + two norm words a row) or the element block (n elements + the
    # norm)
    es_src = raw.element_size()
    if getattr(engine, "spec", False):
        pack_bytes = rows * n * es_src + rows * (-(-n // 32) * 32 + 8)
        pack_form = "byte block (k_pack8_col / k_pack8_row)"
    else:
        es_blk = 8 if dtype == "f64" else 4
        pack_bytes = rows * n * es_src + rows * (n + 1) * es_blk
        pack_form = "element block (k_pack_col / k_pack_row)"
    mode, splits = engine.ctx.info()
    cbits = engine.ctx.contraction_bits()

    # parity spot-check of this rank's first queries against the oracle
    # (after the timed region: the checker is never on the measured path)
    check = None
    if ncheck > 0 and rank == 0:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        got = engine.result()[:ncheck]
        # the fp32 path is exact on the fp32 points (X is already fp32 there)
        ref = oracle.knn(X.astype(np.float64, copy=False), k, rows=(base, min(ncheck, rows)))
        mism = int((got["idx"] != ref["idx"]).sum() +
                   (got["distance"].view(np.uint64) != ref["distance"].view(np.uint64)).sum())
        check = {"queries": int(len(ref)), "mismatches": mism}
    # every row of configs[1]/[2] (60000x784, k = 30) against the oracle's
    # committed per-row hashes (tests/golden/*_rowhash.npz, made by
    # tests/golden/make_golden.py): each rank hashes its own rows, the
    # mismatch count is summed over the ranks -- at P = 8 this is the
    # multi-GPU run's parity, every row (after the timed region)
    all_rows = None
    fx = {"mnist": "mnist_like", "mnist-real": "mnist_real"}.get(workload)
    fpath = os.path.join(ROOT, "tests", "golden", "%s_rowhash.npz" % fx) if fx else None
    if fpath and (m, n, k) == (60000, 784, 30) and os.path.exists(fpath):
        sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
        from rowhash import row_hashes
        with np.load(fpath, allow_pickle=False) as z:
            want = z["hash"][base:base + rows]
        bad = int((row_hashes(engine.result()) != want).sum()) if rows > 0 else 0
        if dist is not None:
            t = torch.tensor([float(bad)], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.SUM)
            bad = int(t.item())
        all_rows = {"rows": m, "mismatches": bad,
                    "fixture": "tests/golden/%s_rowhash.npz (oracle, every row)" % fx}
    if rank != 0:
        return {"line": None, "X": X, "k": k}

    ms_per_step = elapsed / steps * 1e3
    # dominant kernel k_dist_topk: algorithmic FLOP = 2 * queries * corpus * n
    # per rank per step, over its measured event time
    flops_rank = 2.0 * rows * m * n * prof_steps
    achieved = flops_rank / (dist_ms * 1e-3) / 1e12 if dist_ms > 0 else None
    # the MFMA the contraction ran on: fp32 searches on exactly representable
    # 8-bit-style integer data contract on fp16 MFMA (include/knn.h)
    split = engine.ctx.split()
    kernel = "k_dist_topk_i8" if cbits == 8 else ("k_dist_split" if split else "k_dist_topk")
    traffic, traffic_src, traffic_stale = None, None, None
    try:
        with open(args.traffic_json) as f:
            tj = json.load(f)
        key = "m%d_n%d_p%d" % (m, n, P) + ("" if dtype == "f64" else "_" + dtype) + \
            ("_real" if workload == "mnist-real" else "")
        rec = tj.get(key)
        if rec:
            # the PMC figure counts only while it was taken on the kernel that
            # runs here, built from the source as it is now
            src = rec.get("source")
            same = (str(rec.get("kernel", "")).split("<")[0] == kernel and src is not None and
                    os.path.exists(os.path.join(ROOT, src)) and
                    hashlib.sha1(open(os.path.join(ROOT, src), "rb").read()).hexdigest() == rec.get("source_sha1"))
            if same:
                traffic = rec.get("hbm_bytes_per_launch")
                traffic_src = ("rocprofv3 PMC FETCH_SIZE x2 + WRITE_SIZE of %s on the same workload at P = 1 "
                               "(%s; kernel source sha1 %s = this build's; not measured inside this run)"
                               % (rec["kernel"], rec.get("profile", "profiles/pmc_traffic.json"),
                                  rec["source_sha1"][:12]))
            else:
                traffic_stale = ("profiles/pmc_traffic.json[%s] was measured on %s built from an older source "
                                 "(%s); not reported" % (key, rec.get("kernel"), rec.get("profile", "?")))
    except (OSError, ValueError, KeyError, TypeError):
        pass
    peak = {64: FP64_MFMA_PEAK_TFLOPS, 32: FP32_MFMA_PEAK_TFLOPS,
            16: FP16_MFMA_PEAK_TFLOPS, 8: I8_MFMA_PEAK_TOPS}[cbits]
    if split:
        # split fp16 filter: 3 fp16 MFMAs (hi.hi, hi.lo, lo.hi) per
        # algorithmic multiply-add, so its roofline is a third of fp16's
        peak = FP16_MFMA_PEAK_TFLOPS / 3.0
    dtype_peak = FP64_MFMA_PEAK_TFLOPS if dtype == "f64" else FP32_MFMA_PEAK_TFLOPS
    roofline = {
        "kernel": kernel,
        "bound": "mfma",
        "achieved": achieved,
        "peak": peak,
        "unit": "TFLOP/s",
        "mfma_input": "f16 split x S = hi + lo (3 MFMAs a product; exact after the fp64 re-rank and "
                      "certificate)" if split else
                      {64: "f64", 32: "f32", 16: "f16 (exact on this data)",
                       8: "i8 (exact on this data: int32 dot products)"}[cbits],
        "frac": (achieved / peak) if achieved else None,
        "frac_basis": "achieved = algorithmic FLOP / distance-kernel busy time from HIP events on the "
                      "launch streams (knn_ctx_profile) over profiled_steps extra steps run after the "
                      "timed region; the rocprofv3 --kernel-trace average of the same kernel is "
                      "committed in profiles/ (DESIGN.md sec.6)",
        # an exact reduced-precision contraction (i8 / f16) has no "fraction
        # of the fp64 peak": its rate against the element type's MFMA peak
        # (BASELINE's "% of fp64 MFMA peak" wording) is an equivalent, > 1 here
        "frac_of_dtype_peak": (achieved / dtype_peak) if (achieved and cbits >= 32) else None,
        "dtype_peak_equiv": (achieved / dtype_peak) if (achieved and cbits < 32) else None,
        "filter": "split-f16" if split else None,
        "traffic": traffic,
        "traffic_source": traffic_src,
        "traffic_stale": traffic_stale,
        # distance-stage busy time (union of the overlapped k_dist_topk
        # launches, knn_ctx_profile) per launch; at P = 1 one launch a step
        "avg_launch_ms": dist_ms / max(launches, 1),
        "launches": launches,
        "exposed_merge_ms_per_step": merge_ms / max(prof_steps, 1),
        "profiled_steps": prof_steps,
        # the HBM-side passes around the contraction (north_star: "achieved
        # HBM GB/s for the top-k and norm passes"): the merge kernels (the
        # exact fp64 re-rank / the int8 rank merge, knn_ctx_profile_merge:
        # HIP events on the merge's stream, the engine's algorithmic byte
        # count) and the pack / norm pass (torch events on its stream)
        "merge": {
            # (a P = 1 int8 search's only merge runs as k_merge_rank16)
            "kernel": ("k_merge_rank16" if P == 1 else "k_merge_rank") if cbits == 8 else "k_merge",
            "bound": "hbm",
            "ms_per_step": mk_ms / max(prof_steps, 1),
            "launches_per_step": mk_n / max(prof_steps, 1),
            "bytes_per_step": mk_bytes / max(prof_steps, 1),
            "achieved": (mk_bytes / (mk_ms * 1e-3) / 1e9) if mk_ms > 0 else None,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": (mk_bytes / (mk_ms * 1e-3) / 1e9 / HBM_PEAK_GBS) if mk_ms > 0 else None,
        },
        "pack": {
            "kernel": pack_form,
            "bound": "hbm",
            "ms_per_step": pack_ms,
            "bytes_per_step": pack_bytes,
            "achieved": (pack_bytes / (pack_ms * 1e-3) / 1e9) if pack_ms > 0 else None,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": (pack_bytes / (pack_ms * 1e-3) / 1e9 / HBM_PEAK_GBS) if pack_ms > 0 else None,
        },
    }
    line = {
        "metric": METRIC if workload == "mnist" else
                  "all-kNN queries/sec (%s, k=%d) at %d GPUs + %% MFMA peak" % (
                      wdesc.split(" k=")[0].replace("all-kNN ", ""), k, P),
        "value": m / (ms_per_step * 1e-3),
        "unit": "queries/s",
        "n_gpus": P,
        "steps": steps,
        "warmup": warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "strong",
        # BASELINE.md publishes no number for this metric ("published": {}),
        # so there is nothing to divide by
        "vs_baseline": None,
        "dtype": dtype,
        "data": data,
        "config": {"workload": wdesc % (k, m, n), "m": m, "n": n, "k": k,
                   "parallelism": "ring%d" % P},
        # the ranks' process group: RCCL ("nccl") across P GPUs, one process
        # each; null at P = 1 (no collective)
        "rccl_world": P if args.backend == "nccl" else None,
        "launcher": os.environ.get("KNN_BENCH_LAUNCHER") or ("torch.distributed.run" if P > 1 else None),
        "engine": {"mode": ("cpu stand-in (test only)" if standin else mpiknn.MODE_NAMES.get(mode, str(mode))),
                   "splits": splits,
                   "unresolved_queries": unresolved},
        "check": check,
        "check_all_rows": all_rows,
        "roofline": roofline,
        "cpu_baseline": None,
    }
    return {"line": line, "X": X, "k": k}


if __name__ == "__main__":
    main()
