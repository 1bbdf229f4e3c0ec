"""In-process interleaved A/B of the grid build: _C vs _C_<variant> (same points, same dims).
usage: python scripts/ab_build.py <variant> [n,n,...] [k] [rounds]  -> one JSON line per n
Both modules' layouts are compared (cell_start equal; with in-cell order the rows too)."""
import importlib, json, sys, torch
from cuda_knearests_amd.ops import knn_ops as ops
from cuda_knearests_amd.utils import uniform_cloud

var = sys.argv[1]
ns = [int(v) for v in (sys.argv[2] if len(sys.argv) > 2 else "20000,900000,12500000").split(",")]
k = int(sys.argv[3]) if len(sys.argv) > 3 else 16
rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 10
A = importlib.import_module("cuda_knearests_amd._C")
B = importlib.import_module(f"cuda_knearests_amd._C_{var}")
dev = torch.device("cuda", 0)
for n in ns:
    pts = uniform_cloud(n, seed=0, device=dev)
    plan = ops.Plan.auto(n, k)
    ra, rb = A.build(pts, plan.dims, True, None), B.build(pts, plan.dims, True, None)
    torch.cuda.synchronize()
    same = all(torch.equal(x, y) for x, y in zip(ra[:3], rb[:3]))
    res = {}
    for name, M in (("C", A), (var, B)):
        res[name] = []
    reps = 50 if n < 2_000_000 else 10
    for r in range(rounds):
        for name, M in (("C", A), (var, B)):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                M.build(pts, plan.dims, False, None)
            e1.record()
            e1.synchronize()
            res[name].append(e0.elapsed_time(e1) / reps)
    out = {"n": n, "k": k, "dims": plan.dims, "identical_deterministic": same}
    for name, v in res.items():
        v.sort()
        out[name + "_ms"] = [round(v[len(v) // 2], 4), round(v[0], 4)]
    print(json.dumps(out), flush=True)
