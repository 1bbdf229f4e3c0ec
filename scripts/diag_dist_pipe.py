"""Native pipelined distributed steps (kn::DistPipeline, csrc/runtime/dist.hpp) at world 1 over a
real RCCL communicator, with and without forced collectives (the rank's own rows through an RCCL
self send / recv + unpack): per-call asynchronous steps, batched run_steps (unrolled graphs,
resident priming), in-place refills of the input between calls (caller-stream ordering), a moved
share (flag fails, the synchronous call recovers), per-phase profile. Rows are compared bit for
bit with the torch-path reference (DistributedKNearests(native_pipeline=False)).
Every combination runs in three pipeline modes: captured hipGraphs (KN_DIST_CAPTURE=1), eager
stages (=0, the default) and an injected capture failure (KN_DIST_CAPTURE_FAIL=1),
which must fall back to the eager mode and stay exact.
usage: python scripts/diag_dist_pipe.py [steps] [n] [force modes, e.g. 0,1] [capture modes, e.g. 1,0,fail]"""
import os
import sys

import torch
import torch.distributed as dist

from cuda_knearests_amd.parallel import DistributedKNearests
from cuda_knearests_amd.utils import uniform_cloud

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
n = int(sys.argv[2]) if len(sys.argv) > 2 else 900000
modes = [m == "1" for m in sys.argv[3].split(",")] if len(sys.argv) > 3 else [False, True]
caps = sys.argv[4].split(",") if len(sys.argv) > 4 else ["1", "0", "fail"]
verbose = os.environ.get("KN_DIAG_VERBOSE") == "1"


def say(*a):
    if verbose:
        print(*a, flush=True)

for k_, v in (("MASTER_ADDR", "127.0.0.1"), ("MASTER_PORT", "29543"), ("RANK", "0"), ("WORLD_SIZE", "1")):
    os.environ.setdefault(k_, v)
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", device_id=dev)


def reference(p):
    r = DistributedKNearests(k=16, native_pipeline=False)
    r.graph_steady = False
    r.solve(p)
    x = r.solve(p)  # eager steady step
    assert x.valid() and x.stats.get("steady")
    return x.ids.clone(), x.neighbors.clone(), x.d2.clone()


def same(res, ref):
    return (torch.equal(res.ids, ref[0]) and torch.equal(res.neighbors, ref[1]) and torch.equal(res.d2, ref[2]))


pts = uniform_cloud(n, seed=3, device=dev)
perm = torch.randperm(n, device=dev)
pts_perm = pts[perm].contiguous()
ref = reference(pts)
ref_perm = reference(pts_perm)
ok_all = True
for cap, force in [(c, f) for c in caps for f in modes]:
    os.environ["KN_DIST_CAPTURE"] = "0" if cap == "0" else "1"
    os.environ["KN_DIST_CAPTURE_FAIL"] = "1" if cap == "fail" else "0"
    want_mode = "graph" if cap == "1" else "eager"
    dk = DistributedKNearests(k=16, force_collectives=force)
    full = dk.solve(pts)
    r_full = same(full, ref)
    say("full step done")
    r0 = dk.solve(pts, async_=True)
    say("first pipelined step enqueued")
    ok0 = r0.valid()
    say("first pipelined step valid", ok0, same(r0, ref))
    res = [dk.solve(pts, async_=True) for _ in range(steps)]
    say("async steps enqueued")
    piped = bool(res[-1].stats.get("pipelined"))
    valid = all(r.valid() for r in res)
    rows = same(res[-1], ref)
    say("async steps checked")
    batch = dk.run_steps(pts, 20, resident=True)
    say("batch done")
    b_ok = batch.valid() and same(batch, ref)
    batch2 = dk.run_steps(pts, 7)  # after a primed call, an odd count without priming
    b2_ok = batch2.valid() and same(batch2, ref)
    # in-place refills between calls: each step must see its own contents (the permuted cloud has
    # the same bbox and counts, so the flag cannot tell -- only stream ordering can)
    buf = pts.clone()
    dk2 = DistributedKNearests(k=16, force_collectives=force)
    dk2.solve(buf)
    outs = []
    for i in range(6):
        buf.copy_(pts_perm if i % 2 else pts)
        r = dk2.solve(buf, async_=True)
        outs.append((r, i % 2))
        if len(outs) == 2:  # check before the set is reused by the step after next
            for rr, which in outs:
                if not rr.valid():
                    p = dk2._pipe["pipe"]
                    st = dk2._steady
                    msg = (f"refill step invalid (force {force}, step {i}, which {which}): planned tot "
                           f"{st['tot'].tolist()} set0 {p.debug_words(0)} set1 {p.debug_words(1)} "
                           f"last_set {p.last_set()} flags {[x.valid() for x, _ in outs]}")
                    print(msg, flush=True)
                    os.makedirs("gpurun_out", exist_ok=True)
                    with open("gpurun_out/diag_refill.txt", "a") as f:
                        f.write(msg + "\n")
                    dist.destroy_process_group()
                    sys.exit(1)
            refill = all(same(rr, ref_perm if w else ref) for rr, w in outs)
            outs = []
            if not refill:
                break
    # a fresh tensor every step (same shape): the pipeline is rebound, not rebuilt
    dk3 = DistributedKNearests(k=16, force_collectives=force)
    dk3.solve(pts)
    fresh = True
    first_pipe = None
    for i in range(4):
        r = dk3.solve(pts.clone(), async_=True)
        fresh = fresh and r.valid() and same(r, ref)
        if i == 0:
            first_pipe = dk3._pipe["pipe"] if dk3._pipe else None
    fresh = fresh and dk3._pipe is not None and dk3._pipe["pipe"] is first_pipe
    prof = dk.profile_step(pts)
    prof_ok = all(v >= 0.0 for v in prof.values()) and len(prof) == 5
    moved = pts * 0.5
    bad = dk.solve(moved, async_=True)
    inval = not bad.valid()
    rec = same(dk.solve(moved), reference(moved))
    # a share of another size under the steady plan: rebound (no rebuild), the step's flag fails,
    # the synchronous call recovers through the full step
    dk.solve(moved)
    small = moved[: moved.size(0) - 1000].contiguous()
    bad2 = dk.solve(small, async_=True)
    inval = inval and not bad2.valid()
    rec = rec and same(dk.solve(small), reference(small))
    mode_ok = dk2.pipe_mode == want_mode and batch.stats.get("pipe_mode") == want_mode
    print(f"capture {cap} force {force} mode {batch.stats.get('pipe_mode')} full {r_full} pipelined {piped} "
          f"valid {valid} rows {rows} batch {b_ok} {b2_ok} refill {refill} fresh {fresh} moved share invalid {inval} "
          f"recovered {rec} profile {prof}", flush=True)
    ok_all = (ok_all and r_full and piped and valid and rows and b_ok and b2_ok and refill and inval and rec and prof_ok
              and mode_ok and fresh)
print("ALL OK" if ok_all else "FAILED", flush=True)
dist.destroy_process_group()
sys.exit(0 if ok_all else 1)
