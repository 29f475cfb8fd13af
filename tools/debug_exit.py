import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mpi-knn_amd"))
import faulthandler; faulthandler.enable()
case = sys.argv[1]
import numpy as np
if case in ("b", "c", "d"):
    import torch; torch.cuda.init(); x = torch.zeros(10, device="cuda")
import mpiknn
X = np.random.default_rng(0).integers(0, 9, (300, 20)).astype(np.float64)
r, _ = mpiknn.search(X, 5)
if case in ("c",):
    c = mpiknn.Context(0, 300, 20, 300, 5); c.close()
if case in ("d",):
    import mpiknn.ring as ring
    e = ring.GpuEngine(torch, 0, 20, 300, 300, 5)
    Xd = torch.from_numpy(X).cuda()
    e.pack(Xd, False); e.begin(0); e.step(e.qb, 300, 0); e.end()
print("case", case, "done", flush=True)
