#!/usr/bin/env python3
"""One rank's share of a P-GPU ring, emulated on one GPU (diagnostic only).

The scaling bench (N = 2/4/8 GPUs) is run by the driver; this tool measures
what each rank computes there -- its R = ceil(m/P) query rows against the P
corpus blocks, k_dist_topk + k_merge per block, then finalize -- with the
blocks already resident (no RCCL hop), so that the compute-side strong-scaling
efficiency t(1) / (P * t_rank(P)) can be read before an 8-GPU node runs it.

  python tools/ring_emulate.py [--workload mnist] [--ranks 1,2,4,8] [--steps 3]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-knn_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", default="1,2,4,8")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--m", type=int, default=60000)
    ap.add_argument("--n", type=int, default=784)
    ap.add_argument("--k", type=int, default=30)
    args = ap.parse_args()

    import torch
    import mpiknn
    import mpiknn.ring as ring
    from mpiknn import synth

    dev = torch.device("cuda", 0)
    m, n, k = args.m, args.n, args.k
    X, _ = synth.mnist_like(m, n)
    Xd = torch.from_numpy(X).to(dev)
    res = {}
    for P in [int(p) for p in args.ranks.split(",")]:
        R, blocks = ring.partition(m, P)
        eng = ring.GpuEngine(torch, 0, n, R, blocks[0][1], k)
        eng.pack(Xd[0:blocks[0][1]], layout_col=False)
        nb = mpiknn.block_bytes(R, n)
        bufs = []
        for b, (base, rows) in enumerate(blocks):
            t = torch.zeros(nb, dtype=torch.uint8, device=dev)
            mpiknn.block_pack(t.data_ptr(), R, rows, n, Xd[base:base + rows].data_ptr(), n,
                              mpiknn.ROWMAJOR, eng.stream())
            bufs.append(t)
            mb = t[eng.meta_off:eng.meta_off + 8 * mpiknn.META_DOUBLES].view(torch.float64)
            eng.meta.copy_(torch.maximum(eng.meta, mb))   # the ring's all_reduce(MAX)

        # what the ring moves: shadow blocks when the search stages fp16
        # shadow rows (mpiknn/ring.py), element blocks otherwise
        eng.begin(0)
        shadow = P > 1 and eng.ctx.shadow() == 1
        for b, (base, rows) in enumerate(blocks):
            eng.step(bufs[b], rows, base)
        eng.end()
        sbufs = []
        if shadow:
            for t in bufs:
                sb = torch.empty(mpiknn.shadow_bytes(R, n), dtype=torch.uint8, device=dev)
                mpiknn.shadow_pack(sb.data_ptr(), t.data_ptr(), R, n, "f64", eng.stream())
                sbufs.append(sb)

        def one():
            eng.begin(0)
            for b, (base, rows) in enumerate(blocks):
                if shadow:
                    eng.step_shadow(sbufs[b], rows, base)
                else:
                    eng.step(bufs[b], rows, base)
            return eng.end()

        one()
        torch.cuda.synchronize()
        eng.ctx.profile(1)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            one()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / args.steps
        dist_ms, merge_ms, launches = eng.ctx.profile(0)
        flops = 2.0 * blocks[0][1] * m * n * args.steps
        res[P] = {"rank_ms": dt * 1e3, "dist_busy_ms_per_pass": dist_ms / args.steps,
                  "dist_tflops": flops / (dist_ms * 1e-3) / 1e12 if dist_ms > 0 else None,
                  "exposed_merge_ms_per_pass": merge_ms / args.steps,
                  "splits": eng.ctx.info()[1], "shadow_ring": shadow}
        del bufs, sbufs, eng
        torch.cuda.empty_cache()
    t1 = res[min(res)]["rank_ms"]
    for P, r in res.items():
        r["projected_qps"] = m / (r["rank_ms"] * 1e-3)
        r["compute_efficiency"] = t1 / (P * r["rank_ms"])
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
