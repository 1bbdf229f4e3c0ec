"""Serial build census: repeated Engine.prepare of one cloud (900K uniform by default), printing the
engine's event-timed ms_build per call. Run under `rocprofv3 --kernel-trace` and summarise with
`scripts/prof_db.py <db> --timeline N` to split the build into kernel time and inter-kernel gaps.
usage: python scripts/prof_build.py [n] [k] [reps]"""
import sys

import torch

from cuda_knearests_amd._ext import load
from cuda_knearests_amd.utils import uniform_cloud

n = int(sys.argv[1]) if len(sys.argv) > 1 else 900000
k = int(sys.argv[2]) if len(sys.argv) > 2 else 16
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
C = load()
dev = torch.device("cuda", 0)
pts = uniform_cloud(n, seed=0, device=dev)
e = C.Engine(k)
ms = []
for _ in range(reps):
    e.prepare(pts)
    ms.append(e.info()["ms_build"])
torch.cuda.synchronize()
s = sorted(ms)
print("ms_build", " ".join(f"{v:.4f}" for v in ms), "median", f"{s[len(s) // 2]:.4f}", flush=True)
