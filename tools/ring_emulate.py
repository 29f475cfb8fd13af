#!/usr/bin/env python3
"""One rank's share of a P-GPU ring, emulated on one GPU (diagnostic only).

The scaling bench (N = 2/4/8 GPUs) is run by the driver; this tool measures
what each rank computes there -- rank 0's R = ceil(m/P) query rows against
the P corpus blocks, k_dist_topk + k_merge per block, then finalize -- with
the blocks already resident in the form the ring moves (byte / fp16 shadow
blocks when the search stages them, element blocks otherwise; no RCCL hop),
so the compute-side strong-scaling efficiency t(1) / (P * t_rank(P)) can be
read before an 8-GPU node runs it.

  python tools/ring_emulate.py [--workload mnist|mnist-real|sift|gist]
                               [--ranks 1,2,4,8] [--steps 3] [--m M]

configs[3] (sift, 1M x 128 fp32, k = 32) and configs[4] (gist, 4M x 960 fp32,
k = 100) are 8-GPU configurations: --ranks 8 gives their per-rank work
(125K x 8 blocks of 125K rows; 500K x 8 blocks of 500K rows).  The gist-shaped
corpus is generated on the device (a 256-centre mixture in [0, 1), like
mpiknn.synth.gist_like) to keep 15 GB off the host.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-knn_amd"))

WORKLOADS = {   # m, n, k, dtype
    "mnist": (60000, 784, 30, "f64"),
    "mnist-real": (60000, 784, 30, "f64"),
    "sift": (1_000_000, 128, 32, "f32"),
    "gist": (4_000_000, 960, 100, "f32"),
}


def corpus(torch, workload, m, n, dev):
    from mpiknn import synth
    if workload == "mnist":
        return torch.from_numpy(synth.mnist_like(m, n)[0]).to(dev)
    if workload == "mnist-real":
        return torch.from_numpy(synth.mnist_real(m, n)[0]).to(dev)
    if workload == "sift":
        return torch.from_numpy(synth.sift_like(m, n)).to(dev)
    g = torch.Generator(device=dev)
    g.manual_seed(0x6157)
    centres = torch.rand((256, n), generator=g, device=dev) * 0.5 + 0.1
    X = torch.empty((m, n), dtype=torch.float32, device=dev)
    step = 1 << 18
    for lo in range(0, m, step):
        hi = min(m, lo + step)
        lab = torch.randint(0, 256, (hi - lo,), generator=g, device=dev)
        X[lo:hi] = (centres[lab] + 0.08 * torch.randn((hi - lo, n), generator=g, device=dev)
                    ).clamp_(0.0, float(np.nextafter(np.float32(1), np.float32(0))))
    return X


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="mnist")
    ap.add_argument("--ranks", default="1,2,4,8")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warm", type=int, default=3, help="untimed passes before the timed ones")
    ap.add_argument("--m", type=int, default=None)
    ap.add_argument("--splits", default=None,
                    help="comma list: repeat each P with KNN_SPLITS forced to each value (a sweep)")
    ap.add_argument("--fuse", choices=("none", "rest", "all"), default="rest",
                    help="byte-block steps: one launch per block (the neighbour ring), the own "
                         "block then every other block in one launch (the direct-exchange "
                         "ring's default), or all blocks in one launch (KNN_RING_FUSE=all)")
    ap.add_argument("--no-research", action="store_true",
                    help="skip the ring rank's int8 re-search of uncertified queries")
    args = ap.parse_args()

    import torch
    import mpiknn
    import mpiknn.ring as ring

    dev = torch.device("cuda", 0)
    m0, n, k, dt = WORKLOADS[args.workload]
    m = args.m or m0
    Xd = corpus(torch, args.workload, m, n, dev)
    res = {}
    runs = [(int(p), None) for p in args.ranks.split(",")]
    if args.splits:
        runs = [(P, int(sp)) for P, _ in runs for sp in args.splits.split(",")]
    for P, sp in runs:
        if sp is not None:
            os.environ["KNN_SPLITS"] = str(sp)
        R, blocks = ring.partition(m, P)
        eng = ring.GpuEngine(torch, 0, n, R, blocks[0][1], k, dtype=dt)
        sdt = "f32" if Xd.dtype == torch.float32 else "f64"
        eng.pack(Xd[0:blocks[0][1]], layout_col=False)
        nb = mpiknn.block_bytes(R, n, dt)
        bufs = []
        for b, (base, rows) in enumerate(blocks):
            t = torch.zeros(nb, dtype=torch.uint8, device=dev)
            mpiknn.block_pack(t.data_ptr(), R, rows, n, Xd[base:base + rows].data_ptr(), n,
                              mpiknn.ROWMAJOR, eng.stream(), dtype=dt, src_dtype=sdt)
            bufs.append(t)
            mb = t[eng.meta_off:eng.meta_off + 8 * mpiknn.META_DOUBLES].view(torch.float64)
            eng.meta.copy_(torch.maximum(eng.meta, mb))   # the ring's all_reduce(MAX)
        h_meta = eng.meta.cpu().numpy()
        # the own block as bench.py's ring has it: the speculative byte block
        # straight from the rows when the reduced meta accepts it (8-bit
        # integer data), else the element block
        spec = eng.spec and mpiknn.s8_spec_ok(h_meta, n, dt)
        if eng.spec and not spec:
            eng.pack(Xd[0:blocks[0][1]], layout_col=False, elements=True)
            eng.meta.copy_(torch.stack([t[eng.meta_off:eng.meta_off + 8 * mpiknn.META_DOUBLES].view(torch.float64)
                                        for t in bufs]).max(dim=0).values)
            h_meta = eng.meta.cpu().numpy()

        # what the ring moves: the search's shadow form when it has one
        eng.begin(0, h_meta=h_meta)
        shadow = (P > 1 or spec) and eng.ctx.shadow() != 0
        sbufs = []
        if shadow:
            for b, t in enumerate(bufs):
                if b == 0 and spec:
                    sbufs.append(eng.sq)
                    continue
                sb = torch.empty(eng.ctx.shadow_bytes(R), dtype=torch.uint8, device=dev)
                eng.ctx.shadow_pack(sb.data_ptr(), t.data_ptr(), R, eng.stream())
                sbufs.append(sb)
        for b, (base, rows) in enumerate(blocks):
            if shadow:
                eng.step_shadow(sbufs[b], rows, base)
            else:
                eng.step(bufs[b], rows, base)
        eng.end()

        fuse = args.fuse if shadow and P > 1 and eng.ctx.shadow() == 2 else "none"
        # element blocks of a split-filter search: the direct schedule's fused step
        efuse = args.fuse if not shadow and P > 1 and eng.ctx.split() else "none"

        def one():
            eng.begin(0, h_meta=h_meta)
            if fuse == "all":
                eng.ctx.step_shadow_n([b.data_ptr() for b in sbufs], [r for _, r in blocks],
                                      [bs for bs, _ in blocks], eng.stream())
            elif fuse == "rest":
                eng.step_shadow(sbufs[0], blocks[0][1], blocks[0][0])
                eng.ctx.step_shadow_n([b.data_ptr() for b in sbufs[1:]], [r for _, r in blocks[1:]],
                                      [bs for bs, _ in blocks[1:]], eng.stream())
            elif efuse == "rest":
                # the own block as ring.py folds it: the engine's own query
                # block (the fused step then shares the own step's merge)
                eng.step(eng.qb, blocks[0][1], blocks[0][0])
                eng.step_n(bufs[1:], [r for _, r in blocks[1:]], [bs for bs, _ in blocks[1:]])
            elif efuse == "all":
                eng.step_n([eng.qb] + bufs[1:], [r for _, r in blocks], [bs for bs, _ in blocks])
            else:
                for b, (base, rows) in enumerate(blocks):
                    if shadow:
                        eng.step_shadow(sbufs[b], rows, base)
                    else:
                        eng.step(bufs[b], rows, base)
            u = eng.end()
            u2 = u
            if u and fuse in ("rest", "all") and not args.no_research:
                # ring.py's direct schedule: the int8 re-search over the
                # resident byte blocks before any element-block exchange
                u2 = eng.research(sbufs, [r for _, r in blocks], [bs for bs, _ in blocks])
            return u, u2

        for _ in range(args.warm):
            one()
        torch.cuda.synchronize()
        # timed without the profiling events (each event record sits on the
        # launch queues), then the same passes profiled for the breakdown
        t0 = time.perf_counter()
        unres = unres2 = 0
        for _ in range(args.steps):
            u, u2 = one()
            unres += u
            unres2 += u2
        torch.cuda.synchronize()
        dt_s = (time.perf_counter() - t0) / args.steps
        eng.ctx.profile(1)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            one()
        torch.cuda.synchronize()
        dtp_s = (time.perf_counter() - t0) / args.steps
        dist_ms, merge_ms, launches = eng.ctx.profile(0)
        flops = 2.0 * blocks[0][1] * m * n * args.steps
        res[P] = {"rank_ms": dt_s * 1e3, "rank_ms_profiled": dtp_s * 1e3,
                  "dist_busy_ms_per_pass": dist_ms / args.steps,
                  "dist_tflops": flops / (dist_ms * 1e-3) / 1e12 if dist_ms > 0 else None,
                  "exposed_merge_ms_per_pass": merge_ms / args.steps,
                  "splits": eng.ctx.info()[1], "shadow_ring": shadow, "fuse": fuse if shadow else efuse,
                  "contraction_bits": eng.ctx.contraction_bits(), "unresolved": unres,
                  "unresolved_after_research": unres2}
        print(json.dumps({"P": P, **res[P]}), file=sys.stderr, flush=True)
        if sp is not None:
            res["%d/s%d" % (P, sp)] = res.pop(P)
        del bufs, sbufs, eng
        torch.cuda.empty_cache()
    if args.splits:
        print(json.dumps({"workload": args.workload, "sweep": res}, indent=1))
        return
    t1 = res[min(res)]["rank_ms"] * min(res)
    for P, r in res.items():
        r["projected_qps"] = m / (r["rank_ms"] * 1e-3)
        r["compute_efficiency"] = t1 / (P * r["rank_ms"])
    print(json.dumps({"workload": args.workload, "m": m, "n": n, "k": k, "dtype": dt,
                      "ranks": res}, indent=1))


if __name__ == "__main__":
    main()
