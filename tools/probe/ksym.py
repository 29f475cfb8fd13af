"""Drive tools/probe/ksym (the self-join's symmetric launch)
on real engine data: times S + prep + T + scatter and checks coverage -- for
a sample of queries, the exact k nearest (by (d^2, id)) must all be among
the union of S's lists, T's lists and the query's column bucket.

  python tools/probe/ksym.py [--m 60000] [--qa 59] [--splits-t 7] [--iters 5]
                             [--wcap 4096] [--cap 512] [--check 2000]

Needs tools/probe/abl/libkbench8_sym.so (python tools/probe/ablate.py sym),
or KSYM_SO."""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "mpi-knn_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=60000)
    ap.add_argument("--qa", type=int, default=59, help="seed query blocks (rows [0, 128 qa))")
    ap.add_argument("--splits-s", type=int, default=1)
    ap.add_argument("--splits-t", default="7")
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--wcap", type=int, default=4096)
    ap.add_argument("--cap", type=int, default=512)
    ap.add_argument("--check", type=int, default=2000, help="queries checked (0: none)")
    a = ap.parse_args()
    so = os.environ.get("KSYM_SO") or os.path.join(HERE, "abl", "libkbench8_sym.so")
    import torch
    import mpiknn.ring as ring
    from mpiknn import synth
    X, _ = synth.mnist_like(60000, 784)
    X = np.ascontiguousarray(X[:a.m])
    m, n = X.shape
    k = 30
    eng = ring.GpuEngine(torch, 0, n, m, m, k, dtype="f64")
    eng.pack(torch.from_numpy(X).to("cuda:0"), layout_col=False, elements=True)
    eng.begin(0)
    assert eng.ctx.shadow() == 2, "data not int8-eligible"
    sb = torch.empty(eng.ctx.shadow_bytes(m), dtype=torch.uint8, device="cuda:0")
    eng.ctx.shadow_pack(sb.data_ptr(), eng.qb.data_ptr(), m, eng.stream())
    torch.cuda.synchronize()
    dev = "cuda:0"
    nq_pad = (m + 127) // 128 * 128
    rp = nq_pad
    kl, lpq = 12, 2
    nqb = nq_pad // 128
    st_max = max(int(s) for s in a.splits_t.split(","))
    pd_s = torch.empty(a.splits_s * nq_pad * lpq * kl, dtype=torch.float64, device=dev)
    pi_s = torch.empty(a.splits_s * nq_pad * lpq * kl, dtype=torch.int32, device=dev)
    pT_s = torch.empty(a.splits_s * nq_pad, dtype=torch.float64, device=dev)
    pd_t = torch.empty(st_max * nq_pad * lpq * kl, dtype=torch.float64, device=dev)
    pi_t = torch.empty(st_max * nq_pad * lpq * kl, dtype=torch.int32, device=dev)
    pT_t = torch.empty(st_max * nq_pad, dtype=torch.float64, device=dev)
    qthr = torch.empty(nq_pad, dtype=torch.float64, device=dev)
    wcnt = torch.zeros(nqb * st_max, dtype=torch.int32, device=dev)
    wbuf = torch.empty(nqb * st_max * a.wcap * 4, dtype=torch.int32, device=dev)
    ccnt = torch.zeros(m, dtype=torch.int32, device=dev)
    cbuf = torch.empty(m * a.cap, dtype=torch.int64, device=dev)
    L = ctypes.CDLL(so)
    p, i = ctypes.c_void_p, ctypes.c_int
    L.ksym.argtypes = [p, ctypes.c_size_t, i, i, i, i, i, i, p, p, p, p, p, p, i, p, p, p, i, p, p, i, i, p]
    L.ksym.restype = i
    exact = None
    for sp in [int(s) for s in a.splits_t.split(",")]:
        ms = (ctypes.c_float * 5)()
        rc = L.ksym(sb.data_ptr(), rp, m, n, k, a.qa, a.splits_s, sp, pd_s.data_ptr(), pi_s.data_ptr(),
                    pT_s.data_ptr(), pd_t.data_ptr(), pi_t.data_ptr(), pT_t.data_ptr(), nq_pad, qthr.data_ptr(),
                    wcnt.data_ptr(), wbuf.data_ptr(), a.wcap, ccnt.data_ptr(), cbuf.data_ptr(), a.cap, a.iters, ms)
        if rc != 0:
            raise SystemExit("ksym rc %d" % rc)
        wc = wcnt[:nqb * sp].cpu().numpy().astype(np.int64)
        cc = ccnt.cpu().numpy().astype(np.int64)
        rec = {"m": m, "qa": a.qa, "splits_s": a.splits_s, "splits_t": sp,
               "ms": {"S": ms[0], "prep": ms[1], "T": ms[2], "scatter": ms[3], "total": ms[4]},
               "column_survivors": int(wc.sum()), "wg_max": int(wc.max()), "wg_over_cap": int((wc > a.wcap).sum()),
               "row_max": int(cc.max()), "row_mean": float(cc.mean()), "rows_over_cap": int((cc > a.cap).sum())}
        if a.check:
            rng = np.random.default_rng(5)
            qs = np.sort(rng.choice(m, size=min(a.check, m), replace=False))
            if exact is None:
                F = torch.from_numpy(X).to(dev).double()
                nrm = (F * F).sum(1)
                ex = []
                for lo in range(0, len(qs), 256):
                    qq = torch.from_numpy(qs[lo:lo + 256]).to(dev)
                    d2 = nrm[qq, None] + nrm[None, :] - 2.0 * F[qq] @ F.t()
                    d2 = torch.round(d2)
                    d2[d2 <= 0] = float("inf")
                    # (d^2, id) order: d^2 * 2^17 + id is exact in fp64 (d^2 < 2^31)
                    key = d2 * 131072.0 + torch.arange(m, device=dev, dtype=torch.float64)[None, :]
                    ex.append(torch.topk(key, k, dim=1, largest=False).values.cpu().numpy())
                exact = np.concatenate(ex)
            pdS = pd_s.view(a.splits_s, nq_pad, lpq * kl).cpu().numpy()
            piS = pi_s.view(a.splits_s, nq_pad, lpq * kl).cpu().numpy()
            pdT = pd_t[:sp * nq_pad * lpq * kl].view(sp, nq_pad, lpq * kl).cpu().numpy()
            piT = pi_t[:sp * nq_pad * lpq * kl].view(sp, nq_pad, lpq * kl).cpu().numpy()
            cb = cbuf.view(m, a.cap).cpu().numpy()
            miss = 0
            miss_q = []
            for j, q in enumerate(qs):
                d = np.concatenate([pdS[:, q].ravel(), pdT[:, q].ravel()])
                ids = np.concatenate([piS[:, q].ravel(), piT[:, q].ravel()])
                c = int(min(cc[q], a.cap))
                col = cb[q, :c].view(np.uint64)
                d = np.concatenate([d, (col >> np.uint64(32)).astype(np.float64)])
                ids = np.concatenate([ids, (col & np.uint64(0xffffffff)).astype(np.int64)])
                ok = (d < np.inf) & (d > 0) & (ids >= 0)
                have = set((d[ok] * 131072.0 + ids[ok]).tolist())
                want = set(exact[j].tolist())
                lost = len(want - have)
                if lost:
                    miss += 1
                    if len(miss_q) < 10:
                        miss_q.append(int(q))
            rec["checked"] = len(qs)
            rec["queries_missing_neighbours"] = miss
            rec["missing_sample"] = miss_q
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
