"""Drive tools/probe/kbench8 (k_dist_topk_i8 timings) on real engine data.

  python tools/probe/kbench8.py [--workload mnist|sift] [--iters 5]
         [--variant 0,1] [--splits 4,6] [--m M] [--keep-qthr | --ideal-qthr]

Variant v selects (NST staging stages, NB survivor-buffer entries): 0 (7, 8),
1 (8, 3), 2 (8, 4), 3 (7, 6), 4 (7, 4), 5 (8, 5) the 8-wave kernel, 6 the half-tile kernel (4 waves, 64-row
tiles, two workgroups a CU; the product) (12-entry lists).  Prints one JSON line per (variant,
splits)."""
import argparse
import ctypes
import json
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "mpi-knn_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="mnist")
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--splits", default="", help="comma list")
    ap.add_argument("--variant", default="0")
    ap.add_argument("--keep-qthr", action="store_true",
                    help="timed launches start from the previous launch's bounds (converged)")
    ap.add_argument("--m", type=int, default=0, help="use the first M rows (queries = corpus)")
    ap.add_argument("--nq", type=int, default=0,
                    help="queries = the first NQ rows (a P-way ring rank's fused launch: NQ = M / P)")
    ap.add_argument("--ideal-qthr", action="store_true",
                    help="bounds preset to each query's (k+1)-th d^2 over the FULL set (a late ring step)")
    a = ap.parse_args()
    so = os.environ.get("KB8_SO") or os.path.join(HERE, "libkbench8.so")
    if not os.path.exists(so):
        raise SystemExit("build first: make -C tools/probe kbench8")
    import torch
    import mpiknn
    import mpiknn.ring as ring
    from mpiknn import synth
    if a.workload == "mnist":
        X, _ = synth.mnist_like(60000, 784)
        k, dt, splits = 30, "f64", 6
    else:
        X = synth.sift_like(1000000, 128)
        k, dt, splits = 32, "f32", 3
    Xfull = X
    if a.m:
        X = np.ascontiguousarray(X[:a.m])
    m, n = X.shape
    eng = ring.GpuEngine(torch, 0, n, m, m, k, dtype=dt)
    eng.pack(torch.from_numpy(np.ascontiguousarray(X)).to("cuda:0"), layout_col=False, elements=True)
    eng.begin(0)
    assert eng.ctx.shadow() == 2, "data not int8-eligible"
    sb = torch.empty(eng.ctx.shadow_bytes(m), dtype=torch.uint8, device="cuda:0")
    eng.ctx.shadow_pack(sb.data_ptr(), eng.qb.data_ptr(), m, eng.stream())
    torch.cuda.synchronize()
    nq = a.nq or m
    nq_pad = (nq + 127) // 128 * 128
    rp = (m + 127) // 128 * 128
    kl = 12   # KNN_I8_KL_S (the product lists), 4 lists a query
    smax = max(int(x) for x in (a.splits or str(splits)).split(","))
    pd = torch.empty(smax * nq_pad * 4 * kl, dtype=torch.float64, device="cuda:0")
    pi = torch.empty(smax * nq_pad * 4 * kl, dtype=torch.int32, device="cuda:0")
    pT = torch.empty(smax * nq_pad, dtype=torch.float64, device="cuda:0")
    qthr = torch.empty(nq_pad, dtype=torch.float64, device="cuda:0")
    if a.ideal_qthr:
        # (k+1)-th nonzero d^2 of each query over all rows (exact: integer
        # data, fp64 sums far below 2^53)
        F = torch.from_numpy(np.ascontiguousarray(Xfull)).to("cuda:0").double()
        Q = F[:nq]
        nrm = (F * F).sum(1)
        b = torch.full((nq_pad,), float("inf"), dtype=torch.float64, device="cuda:0")
        for lo in range(0, nq, 1024):
            hi = min(nq, lo + 1024)
            d2 = nrm[lo:hi, None] + nrm[None, :] - 2.0 * Q[lo:hi] @ F.t()
            d2[d2 <= 0] = float("inf")
            b[lo:hi] = torch.topk(d2, k + 1, dim=1, largest=False).values[:, k]
        qthr.copy_(b)
    L = ctypes.CDLL(so)
    p, sz, i = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
    L.kbench8.argtypes = [i, p, sz, i, p, sz, i, i, i, i, p, p, p, i, p, i, i]
    L.kbench8.restype = ctypes.c_float
    flop = 2.0 * nq * m * n
    counts = getattr(L, "kb8_counts", None)   # the "count" ablation only
    if counts is not None:
        counts.argtypes = [p]
        cbuf = (ctypes.c_ulonglong * 8)()
        counts(cbuf)
    for var, splits in [(int(x), int(s)) for x in a.variant.split(",")
                        for s in (str(a.splits) if a.splits else str(splits)).split(",")]:
        ms = L.kbench8(var, sb.data_ptr(), rp, nq, sb.data_ptr(), rp, m, n, k, splits,
                       pd.data_ptr(), pi.data_ptr(), pT.data_ptr(), nq_pad, qthr.data_ptr(), a.iters,
                       2 if a.ideal_qthr else (0 if a.keep_qthr else 1))
        rec = {"workload": a.workload, "m": m, "nq": nq, "keep_qthr": a.keep_qthr, "ideal": a.ideal_qthr,
               "variant": var, "splits": splits, "ms": ms,
               "tops": flop / (ms * 1e-3) / 1e12 if ms > 0 else None}
        stamps = getattr(L, "kb8_stamps", None)   # the "stamp" ablation only
        if stamps is not None:
            nwg = min(((nq + 127) // 128) * splits, 16384)
            buf = (ctypes.c_ulonglong * (4 * nwg))()
            stamps.argtypes = [p, i]
            stamps(buf, nwg)
            st = np.frombuffer(buf, dtype=np.uint64).reshape(nwg, 4).astype(np.int64)
            t0 = st[:, 0].min()
            us = lambda v: v * 0.01   # 100 MHz ticks
            q = lambda v: [round(float(np.percentile(v, x)), 1) for x in (0, 10, 50, 90, 100)]
            rec["stamps_us"] = {
                "start_after_launch_p0_10_50_90_100": q(us(st[:, 0] - t0)),
                "prologue": q(us(st[:, 1] - st[:, 0])),
                "loop": q(us(st[:, 2] - st[:, 1])),
                "end": q(us(st[:, 3] - st[:, 2])),
                "wg_total": q(us(st[:, 3] - st[:, 0])),
                "launch_span": round(float(us(st[:, 3].max() - t0)), 1)}
        if counts is not None:
            counts(cbuf)
            names = ("past_acc_filter", "keys_built", "exact_survivors", "extract_rounds", "merges")
            rec["per_launch"] = {nm: cbuf[j] / (a.iters + 1) for j, nm in enumerate(names)}
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
