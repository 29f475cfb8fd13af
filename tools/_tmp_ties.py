import sys, os, json
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "mpi-knn_amd"))
import numpy as np, torch
from mpiknn import synth
X, _ = synth.mnist_like(60000, 784)
F = torch.from_numpy(X).cuda().double()
nrm = (F * F).sum(1)
res = []
for lo in range(0, 60000, 2048):
    hi = min(60000, lo + 2048)
    d2 = nrm[lo:hi, None] + nrm[None, :] - 2.0 * F[lo:hi] @ F.t()
    d2 = torch.round(d2)
    d2[d2 <= 0] = float("inf")
    v, i = torch.topk(d2, 33, dim=1, largest=False)
    res.append(v.cpu())
V = torch.cat(res).numpy()
tie30 = np.nonzero(V[:, 29] == V[:, 30])[0]
tie_any = np.nonzero((V[:, 28] == V[:, 29]) | (V[:, 29] == V[:, 30]) | (V[:, 30] == V[:, 31]))[0]
print(json.dumps({"tie_30_31": len(tie30), "rows": tie30[:20].tolist(), "tie_near_boundary": len(tie_any)}))
