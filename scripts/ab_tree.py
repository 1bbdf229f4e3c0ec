"""Interleaved A/B of tree-path kernel variants on the native engine (900K clustered / surface,
K=16; AB_K=k for another K). Every configuration runs in its OWN process (one extension module per
process: KN_C_VARIANT=<suffix>): round 6 saw two engines from two different extension modules in one
process end in an illegal memory access twice (profiles/ab_r6_global_out.txt), while each module
alone is clean. Rows are compared through a saved reference file.
usage: python scripts/ab_tree.py suffix[,suffix...] [rounds] [steps]"""
import json
import os
import subprocess
import sys
import tempfile

CHILD = r'''
import json, os, sys, time, torch
from cuda_knearests_amd._ext import load
from cuda_knearests_amd.utils import clustered_cloud, surface_cloud
gen, k, steps, ref = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
C = load()
dev = torch.device("cuda", 0)
pts = {"clustered": clustered_cloud, "surface": surface_cloud}[gen](900000, seed=0, device=dev)
e = C.Engine(k)
e.prepare(pts)
e.solve()
i, d = e.results(dev)
same = None
if os.path.exists(ref):
    r = torch.load(ref, weights_only=True)
    same = bool(torch.equal(i.cpu(), r["i"]) and torch.equal(d.cpu(), r["d"]))
else:
    torch.save({"i": i.cpu(), "d": d.cpu()}, ref)
e.launch_pipelined(20, -1)
e.sync()
t0 = time.perf_counter()
e.launch_pipelined(steps, -1)
e.sync()
print(json.dumps({"ms": (time.perf_counter() - t0) * 1e3 / steps, "same": same, "counters": e.counters()}))
'''

sufs = [""] + [s for s in (sys.argv[1].split(",") if len(sys.argv) > 1 else []) if s]
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 4
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 30
k = int(os.environ.get("AB_K", "16"))
tmp = tempfile.mkdtemp()
for gen in ("clustered", "surface"):
    ref = os.path.join(tmp, f"ref_{gen}.pt")
    res = {s or "base": [] for s in sufs}
    flags = {}
    for r in range(rounds):
        order = sufs if r % 2 == 0 else list(reversed(sufs))
        for suf in order:
            env = dict(os.environ)
            env.pop("KN_C_VARIANT", None)
            if suf:
                env["KN_C_VARIANT"] = suf.lstrip("_")
            out = subprocess.run([sys.executable, "-c", CHILD, gen, str(k), str(steps), ref], env=env,
                                 capture_output=True, text=True, timeout=300)
            if out.returncode != 0:
                sys.stderr.write(out.stderr[-2000:])
                raise SystemExit(f"{suf or 'base'} failed ({out.returncode})")
            d = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1])
            res[suf or "base"].append(d["ms"])
            flags[suf or "base"] = (d["same"], d["counters"])
    for name, acc in res.items():
        acc.sort()
        print(f"{gen} {name}: median {acc[len(acc) // 2]:.4f} min {acc[0]:.4f} ms/step identical "
              f"{flags[name][0]} counters {flags[name][1]}", flush=True)
