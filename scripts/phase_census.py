"""Per-phase wave-cycle census of the query kernel (KN_PHASES build, _C_phases).
usage: python scripts/phase_census.py [variant] [n] [k ...]   -> one JSON line per K

Phases (query.hip, KN_PH_MARK): stage = cell bounds + row prefix + LDS staging (+ the kernel
tail), setup = per-chunk query lookup, scan = the lane walk (row setup + hot loop), rerank =
exact window re-rank (+ cooperative paths), certify = certification + fallback append. Shares
are of the summed wave cycles (s_memtime, shader clock) -- what each phase occupies of a wave's
lifetime, including the cycles other waves on its SIMD issue in the meantime."""
import importlib, json, sys, torch
from cuda_knearests_amd.ops import knn_ops as ops
from cuda_knearests_amd.utils import uniform_cloud

var = "phases"
if len(sys.argv) > 1 and not sys.argv[1].isdigit():
    var = sys.argv.pop(1)  # optional first argument: the KN_PHASES variant (_C_<var>)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 900000
ks = [int(v) for v in sys.argv[2:]] or [16, 50]
B = importlib.import_module("cuda_knearests_amd._C_" + var)
dev = torch.device("cuda", 0)
pts = uniform_cloud(n, seed=0, device=dev)
inf = float("inf")
names = ["stage", "setup", "scan", "rerank", "certify"]
for k in ks:
    plan = ops.Plan.auto(n, k)
    s, cs, perm, geom = B.build(pts, plan.dims, True, None)
    args = (s, cs, geom, plan.dims, k, n, None, [-inf, -inf, -inf, inf, inf, inf], plan.tile, plan.halo,
            plan.lds_capacity, True, True, 0)
    for _ in range(3):
        B.query(*args, xsub=plan.xsub)
    torch.cuda.synchronize()
    B.debug_phase_cycles(True)
    reps = 10
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(reps):
        B.query(*args, xsub=plan.xsub)
    ev1.record()
    ev1.synchronize()
    v = B.debug_phase_cycles(True)
    tot = sum(v[:5])
    out = {"variant": var, "n": n, "k": k, "ms_query_instrumented": ev0.elapsed_time(ev1) / reps,
           "waves": v[6] // reps, "chunks": v[5] // reps,
           "cycles_per_wave": tot / max(1, v[6]),
           "share": {nm: round(v[i] / tot, 4) for i, nm in enumerate(names)},
           "cycles_per_chunk": {nm: round(v[i] / max(1, v[5]), 1) for i, nm in enumerate(names)}}
    print(json.dumps(out), flush=True)
