#!/usr/bin/env python3
"""bench.py -- all-kNN queries/sec on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1]/[2]): all-kNN, k = 30, fp64, over an
MNIST-784-shaped corpus of m = 60000 rows (synthetic integer pixels 0..255 --
no dataset can be fetched; see mpiknn/synth.py), leave-one-out (exact zero
distances excluded) like knn-serial.c:72-93.  One "step" = one full all-kNN
pass with the corpus already resident in HBM (column-major, the .mat layout):
pack -> ring of P corpus blocks (k_dist_topk + k_merge per block) -> finalize
(+ exact rescan if any query needs it).  value = m / step time (whole job).

  python bench.py [--gpus N --steps K --warmup W]
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

N > 1: one process per GPU, RCCL (torch.distributed "nccl") ring of corpus
blocks, strong scaling (total work fixed).  Rank 0 prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "mpi-knn_amd"))

FP64_MFMA_PEAK_TFLOPS = 78.6   # MI355X dense fp64 matrix (spec; 78.2 measured, tools/probe)


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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--m", type=int, default=60000)
    ap.add_argument("--n", type=int, default=784)
    ap.add_argument("--k", type=int, default=30)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--check", type=int, default=8, help="queries re-checked against the oracle")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    P = world

    import mpiknn
    import mpiknn.ring as ring
    from mpiknn.synth import mnist_like

    m, n, k = args.m, args.n, args.k
    X, y = mnist_like(m, n)
    R, blocks = ring.partition(m, P)
    base, rows = blocks[rank]
    dev = torch.device("cuda", local)
    # own rows, column-major on the device (the .mat layout, serial:82)
    raw_t = torch.from_numpy(np.ascontiguousarray(X[base:base + rows].T)).to(dev)
    raw = raw_t.t()
    engine = ring.GpuEngine(torch, local, n, R, rows, k)

    def step():
        engine.pack(raw, layout_col=True)
        return ring.ring_search(dist, torch, engine, rank, P, m, base)

    def barrier():
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier(device_ids=[local])
        torch.cuda.synchronize()

    for _ in range(args.warmup):
        step()
    engine.ctx.profile(1)
    unresolved = 0
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        unresolved += step()
    barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    dist_ms, merge_ms, launches = engine.ctx.profile(0)
    mode, splits = engine.ctx.info()

    # parity spot-check of this rank's first queries against the oracle
    check = None
    if args.check > 0 and rank == 0:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        got = engine.result()[: args.check]
        ref = oracle.knn(X, k, rows=(base, min(args.check, rows)))
        mism = int((got["idx"] != ref["idx"]).sum() +
                   (got["distance"].view(np.uint64) != ref["distance"].view(np.uint64)).sum())
        check = {"queries": int(len(ref)), "mismatches": mism}

    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return

    ms_per_step = elapsed / args.steps * 1e3
    # dominant kernel k_dist_topk: algorithmic FLOP = 2 * queries * corpus * n
    # per rank per step, over its measured event time
    flops_rank = 2.0 * rows * m * n * args.steps
    achieved = flops_rank / (dist_ms * 1e-3) / 1e12 if dist_ms > 0 else None
    traffic = None
    try:
        with open(args.traffic_json) as f:
            tj = json.load(f)
        key = "m%d_n%d_p%d" % (m, n, P)
        traffic = tj.get(key, {}).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        pass
    roofline = {
        "kernel": "k_dist_topk",
        "bound": "mfma",
        "achieved": achieved,
        "peak": FP64_MFMA_PEAK_TFLOPS,
        "unit": "TFLOP/s",
        "frac": (achieved / FP64_MFMA_PEAK_TFLOPS) if achieved else None,
        "traffic": traffic,
        "avg_launch_ms": dist_ms / max(launches, 1),
        "launches": launches,
        "merge_ms_per_step": merge_ms / max(args.steps, 1),
    }
    out = {
        "metric": "all-kNN queries/sec (MNIST-784, k=30) at 1/2/4/8 GPUs + % MFMA peak",
        "value": m / (ms_per_step * 1e-3),
        "unit": "queries/s",
        "n_gpus": P,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (MNIST-784 shape, integer pixels 0..255, seed 1234)",
        "config": {"workload": "all-kNN MNIST-784 k=%d (configs[1]: %dx%d fp64, leave-one-out)" % (k, m, n),
                   "m": m, "n": n, "k": k, "parallelism": "ring%d" % P},
        "engine": {"mode": mpiknn.MODE_NAMES.get(mode, str(mode)), "splits": splits,
                   "unresolved_queries": unresolved},
        "check": check,
        "roofline": roofline,
        "cpu_baseline": None,
    }
    if P == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(X, k, args.cpu_seconds)
    print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
