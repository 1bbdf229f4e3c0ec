"""GPU tests of the multi-GPU path on ONE device:
* the native router (route.hip) against the torch reference router, bit for bit;
* the full distributed solve on 2/4/8 virtual ranks (LoopbackTransport threads) with the native
  router + HIP kernels, against the kd-tree oracle;
* the RCCL path itself (torch.distributed "nccl", world 1) end to end.
"""
import os
import socket

import pytest
import torch

from cuda_knearests_amd.parallel import SpatialDecomposition, halo_send_width, route_rows_torch
from cuda_knearests_amd.utils import uniform_cloud
from cuda_knearests_amd.utils.check import assert_knn_exact

from test_distributed import _loopback_check

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("world,h", [(1, 30.0), (2, 25.0), (8, 40.0), (12, 15.0)])
def test_native_router_matches_torch(cuda, ext, world, h):
    n = 50_000
    p = uniform_cloud(n, seed=world, device=cuda)
    ids = torch.arange(n, dtype=torch.int32, device=cuda) * 3 + 7
    lo, hi = (0.0, 0.0, 0.0), (1000.0, 1000.0, 1000.0)
    dec = SpatialDecomposition(world, lo, hi)
    hs = halo_send_width(h, lo, hi)
    ref, cnt = route_rows_torch(dec, p, ids, hs)
    bc, totals = ext.route_count(p, list(lo), list(hi), list(dec.grid), dec.boxes(), hs)
    assert torch.equal(totals, cnt)
    send = ext.route_scatter(p, ids, list(lo), list(hi), list(dec.grid), dec.boxes(), hs, bc, totals, ref.size(0))
    assert torch.equal(send.view(torch.int32), ref.view(torch.int32))
    # unpack as if every source sent this buffer: owned rows of all sources first, then halo
    c = cnt.tolist()
    own = [a for a, _ in c]
    halo = [b for _, b in c]
    pts, gids = ext.route_unpack(send, own, halo)
    segs, o = [], 0
    for a, b in c:
        segs.append((send[o:o + a], send[o + a:o + a + b]))
        o += a + b
    exp = torch.cat([s[0] for s in segs] + [s[1] for s in segs])
    assert torch.equal(pts, exp[:, :3].contiguous())
    assert torch.equal(gids, exp[:, 3].contiguous().view(torch.int32))


@pytest.mark.parametrize("world", [2, 8, 12])
def test_native_router_balanced_matches_torch(cuda, ext, world):
    # count-balanced kd boxes: the native router's owner / halo decisions == the torch reference
    from cuda_knearests_amd.parallel.decomposition import balanced_splits
    from cuda_knearests_amd.utils import clustered_cloud

    n = 50_000
    p = clustered_cloud(n, seed=world).to(cuda)
    ids = torch.arange(n, dtype=torch.int32, device=cuda)
    lo_t, hi_t = p.min(0).values.double(), p.max(0).values.double()
    lo, hi = tuple(lo_t.tolist()), tuple(hi_t.tolist())
    grid = SpatialDecomposition(world, lo, hi).grid
    sp = balanced_splits(p, lo_t, hi_t, grid, lambda t: t)
    dec = SpatialDecomposition(world, lo, hi, grid, sp.tolist())
    hs = halo_send_width(12.0, lo, hi)
    ref, cnt = route_rows_torch(dec, p, ids, hs)
    own = cnt[:, 0].double()
    assert float(own.max() / own.mean()) < 1.05
    bc, totals = ext.route_count(p, list(lo), list(hi), list(grid), dec.boxes(), hs, dec.splits)
    assert torch.equal(totals, cnt)
    send = ext.route_scatter(p, ids, list(lo), list(hi), list(grid), dec.boxes(), hs, bc, totals, ref.size(0),
                             dec.splits)
    assert torch.equal(send.view(torch.int32), ref.view(torch.int32))
    # device plan with the same splits: same boxes (and this rank's box in the header)
    metas = ext.local_meta(p).repeat(world).contiguous()
    plan, hdr = ext.route_plan(metas, world - 1, list(grid), 16, 2.5, sp)
    blo, bhi = dec.rank_box(world - 1)
    assert hdr[12:18].cpu().tolist() == list(blo) + list(bhi)
    bc2, totals2 = ext.route_count_dev(p, plan, world)
    assert torch.equal(totals2[:, 0], cnt[:, 0])


def test_loopback_gpu_clustered_balanced(cuda):
    # 8 virtual ranks, clustered cloud: exact, and the count-balanced boxes hold max/mean <= 1.3
    out = _loopback_check(8, 16, "clustered", cuda, native=True, n=40000, scatter="random")
    own = torch.tensor([s["n_owned"] for *_, s in out], dtype=torch.float64)
    assert float(own.max() / own.mean()) <= 1.3, own.tolist()


@pytest.mark.parametrize("world,k,gen", [(2, 16, "uniform"), (4, 8, "clustered"), (8, 16, "uniform"), (8, 50, "uniform")])
def test_loopback_gpu_matches_single(cuda, world, k, gen):
    _loopback_check(world, k, gen, cuda, native=True, n=30000, scatter="random")


def test_loopback_gpu_growth_round(cuda):
    out = _loopback_check(8, 16, "uniform", cuda, native=True, n=20000, halo_factor=0.05)
    assert max(s["rounds"] for *_, s in out) > 1


def test_rccl_world1_end_to_end(cuda):
    import torch.distributed as dist

    import cuda_knearests_amd as kn
    from cuda_knearests_amd.parallel import DistributedKNearests

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    store = dist.TCPStore("127.0.0.1", port, 1, True)
    dist.init_process_group("nccl", store=store, rank=0, world_size=1, device_id=cuda)
    try:
        p = uniform_cloud(40000, seed=77, device=cuda)
        dk = DistributedKNearests(k=16)
        r = dk.solve(p)
        i, d = kn.knn(p, 16)
        assert torch.equal(r.ids.long().cpu(), torch.arange(p.size(0)))
        assert torch.equal(r.d2, d)
        assert torch.equal(r.neighbors, i)
        # steady state: sync-free steps, same rows bit for bit; new points of the same size run
        # through the same step and fail its on-device check
        for _ in range(3):
            r2 = dk.solve(p, async_=True)
        assert r2.valid() and r2.stats["steady"]
        assert torch.equal(r2.d2, d) and torch.equal(r2.neighbors, i)
        q = uniform_cloud(40000, seed=78, device=cuda) * 0.5
        r3 = dk.solve(q, async_=True)
        assert not r3.valid()
        r4 = dk.solve(q)  # synchronous: re-plans
        i4, d4 = kn.knn(q, 16)
        assert torch.equal(r4.d2, d4) and torch.equal(r4.neighbors, i4)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n,offset", [(0, 0), (1, 0), (777, 0), (300_000, 0), (300_001, 1), (5, 3)])
def test_local_meta_matches_torch(cuda, ext, n, offset):
    """offset > 0: a row slice whose base is not 16-B aligned (scalar-load path)."""
    p = uniform_cloud(n + offset, seed=n, device=cuda, lo=-250.0, hi=640.0)[offset:]
    assert p.is_contiguous()
    v = ext.local_meta(p).cpu()
    assert v.dtype == torch.float64 and v.numel() == 8
    assert v[6].item() == n and v[7].item() == 0.0
    if n == 0:
        assert torch.isinf(v[:3]).all() and (v[:3] > 0).all() and (v[3:6] < 0).all()
        return
    mn, mx = torch.aminmax(p, dim=0)
    assert torch.equal(v[:3], mn.double().cpu())
    assert torch.equal(v[3:6], mx.double().cpu())


@pytest.mark.parametrize("world", [2, 8])
def test_device_plan_matches_host_plan(cuda, world):
    """Device-planned routing (one host sync) == host-planned routing, bit for bit."""
    from cuda_knearests_amd.parallel import DistributedKNearests, run_loopback

    n = 40000
    cloud = uniform_cloud(n, seed=90 + world)
    owner = torch.randint(0, world, (n,), generator=torch.Generator().manual_seed(world))

    def fn(device_plan):
        def body(t):
            m = owner == t.rank
            dk = DistributedKNearests(k=16, transport=t, device_plan=device_plan)
            ids = torch.nonzero(m).flatten().to(torch.int32)
            r = dk.solve(cloud[m].contiguous().to(cuda), ids.to(cuda))
            return r.ids.cpu(), r.neighbors.cpu(), r.d2.cpu(), r.stats
        return run_loopback(world, body)

    a, b = fn(True), fn(False)
    for (ia, na, da, sa), (ib, nb, db, sb) in zip(a, b):
        assert torch.equal(ia, ib) and torch.equal(na, nb) and torch.equal(da, db)
        assert sa["halo_width"] == pytest.approx(sb["halo_width"], rel=1e-12)


def test_device_plan_default_ids(cuda):
    """ids=None: global id = rank offset + local index, generated inside route_scatter."""
    import cuda_knearests_amd as kn
    from cuda_knearests_amd.parallel import DistributedKNearests, run_loopback

    world, n, k = 4, 30000, 8
    cloud = uniform_cloud(n, seed=123)
    owner = torch.randint(0, world, (n,), generator=torch.Generator().manual_seed(1))
    parts = [cloud[owner == r].contiguous() for r in range(world)]
    cat = torch.cat(parts)

    def body(t):
        r = DistributedKNearests(k=k, transport=t).solve(parts[t.rank].to(cuda))
        return r.ids.cpu(), r.neighbors.cpu(), r.d2.cpu()

    out = run_loopback(world, body)
    oi, od = kn.knn_cpu(cat, k, "kdtree")
    seen = torch.zeros(n, dtype=torch.bool)
    for ids_r, nb, d2 in out:
        ids_r = ids_r.long()
        seen[ids_r] = True
        assert torch.equal(d2, od[ids_r])
        assert_knn_exact(cat, ids_r, nb.cpu(), d2.cpu(), od[ids_r])
    assert bool(seen.all())


def _staged_worker(rank, world, port, q):
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from cuda_knearests_amd.parallel import DistributedKNearests, HostStagedTransport
    from cuda_knearests_amd.utils import uniform_cloud as uc

    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    n = 40000
    cloud = uc(n, seed=31)
    owner = torch.arange(n) % world
    m = owner == rank
    ids = torch.nonzero(m).flatten().to(torch.int32)
    dk = DistributedKNearests(k=16, transport=HostStagedTransport())
    r = dk.solve(cloud[m].contiguous().to(dev), ids.to(dev))
    q.put((rank, r.ids.cpu().numpy().copy(), r.neighbors.cpu().numpy().copy(), r.d2.cpu().numpy().copy(),
           dict(r.stats)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_multiprocess_native_path_host_staged(cuda, world):
    """Multi-PROCESS rehearsal of the native (device-planned) distributed path: separate
    processes on one GPU, collectives through gloo (RCCL refuses several ranks per GPU)."""
    import torch.multiprocessing as mp

    import cuda_knearests_amd as kn

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = [ctx.Process(target=_staged_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    n = 40000
    cloud = uniform_cloud(n, seed=31)
    oi, od = kn.knn_cpu(cloud, 16, "kdtree")
    seen = torch.zeros(n, dtype=torch.bool)
    for rank, ids, nb, d2, stats in out:
        ids, nb, d2 = torch.from_numpy(ids).long(), torch.from_numpy(nb), torch.from_numpy(d2)
        assert not bool(seen[ids].any())
        seen[ids] = True
        assert torch.equal(d2, od[ids])
        assert_knn_exact(cloud.cpu(), ids, nb.cpu(), d2.cpu(), od[ids])
    assert bool(seen.all())


@pytest.mark.parametrize("world,rank", [(1, 0), (4, 0), (4, 2), (8, 7)])
def test_route_begin_self_last(cuda, ext, world, rank):
    """route_begin (plan + counts + scatter, one call) == the separate launches, with the rank's
    own segment moved to the end; route_unpack_split == route_unpack of the full buffer."""
    from cuda_knearests_amd.parallel import factor3

    n = 30000
    p = uniform_cloud(n, seed=5 + world, device=cuda)
    ids = torch.arange(n, dtype=torch.int32, device=cuda) * 5 + 1
    metas = ext.local_meta(p).repeat(world).contiguous()  # every rank "has" the same box
    grid = list(factor3(world, (1.0, 1.0, 1.0)))
    plan, sync, bc, send = ext.route_begin(p, ids, metas, rank, grid, 16, 2.5, world * n + 1024)
    hdr, totals = sync[:48].view(torch.float64), sync[48:48 + 2 * world].view(world, 2)
    plan2, hdr2 = ext.route_plan(metas, rank, grid, 16, 2.5)
    assert torch.equal(plan, plan2) and torch.equal(hdr, hdr2)
    bc2, totals2 = ext.route_count_dev(p, plan2, world)
    assert torch.equal(totals, totals2) and torch.equal(bc, bc2)
    c = totals.cpu().tolist()
    need = sum(a + b for a, b in c)
    assert need <= send.size(0)
    if world > 1:
        assert sum(b for _, b in c) > 0  # some halo rows
    ref = ext.route_scatter_dev(p, ids, plan2, world, bc2, totals2, need)
    segs, o = [], 0
    for a, b in c:
        segs.append(ref[o:o + a + b])
        o += a + b
    exp = torch.cat([segs[d] for d in range(world) if d != rank] + [segs[rank]])
    assert torch.equal(send[:need].view(torch.int32), exp.view(torch.int32))
    # unpack: the full buffer as if every source sent it vs the split form
    own = [a for a, _ in c]
    halo = [b for _, b in c]
    full_pts, full_gids = ext.route_unpack(ref, own, halo)
    x = need - (own[rank] + halo[rank])
    sp, sg = ext.route_unpack_split(send[:x].contiguous(), send[x:need].contiguous(), own, halo, rank)
    assert torch.equal(sp, full_pts) and torch.equal(sg, full_gids)


def test_distributed_send_buffer_regrow(cuda):
    """First step with a send buffer far too small (headroom -1): the re-scatter path gives the
    same results as the default sizing."""
    from cuda_knearests_amd.parallel import DistributedKNearests, run_loopback

    world, n = 4, 30000
    cloud = uniform_cloud(n, seed=11)
    owner = torch.randint(0, world, (n,), generator=torch.Generator().manual_seed(2))

    def fn(headroom):
        def body(t):
            m = owner == t.rank
            dk = DistributedKNearests(k=16, transport=t)
            dk.send_headroom = headroom
            ids = torch.nonzero(m).flatten().to(torch.int32)
            r = dk.solve(cloud[m].contiguous().to(cuda), ids.to(cuda))
            return r.ids.cpu(), r.neighbors.cpu(), r.d2.cpu()
        return run_loopback(world, body)

    for (ia, na, da), (ib, nb, db) in zip(fn(0.25), fn(-1.0)):
        assert torch.equal(ia, ib) and torch.equal(na, nb) and torch.equal(da, db)


def test_speculative_routing_repeat_and_change(cuda):
    """Repeated solves take the speculative exchange (plan from the previous step's metas, one
    all-gather of {meta, counts}); a changed cloud falls back to re-planning. Every result must
    equal a non-speculative solve of the same data."""
    from cuda_knearests_amd.parallel import DistributedKNearests, run_loopback

    world, n, k = 4, 24000, 12
    cloud = uniform_cloud(n, seed=31)
    owner = torch.randint(0, world, (n,), generator=torch.Generator().manual_seed(4))

    def body(t):
        m = owner == t.rank
        ids = torch.nonzero(m).flatten().to(torch.int32).to(cuda)
        pts = cloud[m].contiguous().to(cuda)
        spec = DistributedKNearests(k=k, transport=t)
        ref = DistributedKNearests(k=k, transport=t)
        ref.speculative = False
        outs = []
        # step 1 (normal), step 2 (speculative hit), step 3: rank 0 drops half its points (miss),
        # step 4: hit again on the changed cloud
        for step in range(4):
            if step >= 2 and t.rank == 0:
                keep = torch.arange(pts.size(0), device=cuda) % 2 == 0
                p, i = pts[keep].contiguous(), ids[keep].contiguous()
            else:
                p, i = pts, ids
            a = spec.solve(p, i)
            b = ref.solve(p, i)
            outs.append((torch.equal(a.ids, b.ids) and torch.equal(a.neighbors, b.neighbors)
                         and torch.equal(a.d2, b.d2), spec._spec is not None))
        return outs

    for outs in run_loopback(world, body):
        assert all(eq for eq, _ in outs)
        assert all(cached for _, cached in outs)


@pytest.mark.parametrize("world", [1, 4])
def test_steady_state_async_steps(cuda, world):
    """After one validated step the solve runs with no host synchronisation (steady state): the
    rows equal the validated step's bit for bit and the device flag says valid. A step whose
    points changed (same sizes) fails the on-device check: valid() is False, and a synchronous
    solve of the same points re-plans and is exact."""
    import cuda_knearests_amd as kn
    from cuda_knearests_amd.parallel import DistributedKNearests, run_loopback

    n, k = 24000, 12
    cloud = uniform_cloud(n, seed=77)
    moved = cloud.clone()
    moved[:, 0] = (moved[:, 0] * 0.9 + 37.0)  # same sizes, different geometry (metas change)
    owner = torch.arange(n) % world

    def body(t):
        m = owner == t.rank
        ids = torch.nonzero(m).flatten().to(torch.int32).to(cuda)
        dk = DistributedKNearests(k=k, transport=t, halo_field=0)  # steady after ONE full step
        r0 = dk.solve(cloud[m].contiguous().to(cuda), ids)
        r1 = dk.solve(cloud[m].contiguous().to(cuda), ids, async_=True)
        ok1 = r1.valid()
        r2 = dk.solve(moved[m].contiguous().to(cuda), ids, async_=True)
        ok2 = r2.valid()
        r3 = dk.solve(moved[m].contiguous().to(cuda), ids)
        return (r0.ids.cpu(), r0.neighbors.cpu(), r0.d2.cpu(), r1.ids.cpu(), r1.neighbors.cpu(), r1.d2.cpu(),
                bool(r1.stats.get("steady")), ok1, ok2, r3.ids.cpu(), r3.neighbors.cpu(), r3.d2.cpu())

    out = run_loopback(world, body)
    _, od = kn.knn_cpu(moved, k, "kdtree")
    for (i0, n0, d0, i1, n1, d1, steady, ok1, ok2, i3, n3, d3) in out:
        assert steady and ok1 and not ok2
        assert torch.equal(i0, i1) and torch.equal(n0, n1) and torch.equal(d0, d1)
        ids = i3.long()
        assert torch.equal(d3, od[ids])
        assert_knn_exact(moved, ids, n3, d3, od[ids])


def test_adaptive_local_grid_clustered(cuda):
    """Clustered shares: the occupancy-adaptive local grid (as the 1-GPU engine's) re-bins the
    dense ranks finer, sends fewer queries to the exact path than the fixed grid, stays exact,
    and the steady (sync-free) step reuses the validated step's grid bit for bit."""
    import cuda_knearests_amd as kn
    from cuda_knearests_amd.parallel import DistributedKNearests, run_loopback
    from cuda_knearests_amd.utils import clustered_cloud

    n, k, world = 60000, 16, 4
    cloud = clustered_cloud(n, seed=5)
    owner = torch.arange(n) % world
    _, od = kn.knn_cpu(cloud, k, "kdtree")

    def run(adaptive):
        def body(t):
            m = owner == t.rank
            ids = torch.nonzero(m).flatten().to(torch.int32).to(cuda)
            dk = DistributedKNearests(k=k, transport=t, adaptive=adaptive, halo_field=0)
            r0 = dk.solve(cloud[m].contiguous().to(cuda), ids)
            r1 = dk.solve(cloud[m].contiguous().to(cuda), ids, async_=True)
            ok = r1.valid()
            return (r0.ids.cpu(), r0.neighbors.cpu(), r0.d2.cpu(), r1.neighbors.cpu(), r1.d2.cpu(), ok,
                    r0.stats)
        return run_loopback(world, body)

    fixed, adapt = run(False), run(True)
    for out in (fixed, adapt):
        for i0, n0, d0, n1, d1, ok, _ in out:
            ids = i0.long()
            assert torch.equal(d0, od[ids])
            assert_knn_exact(cloud, ids, n0, d0, od[ids])
            assert ok and torch.equal(n0, n1) and torch.equal(d0, d1)
    ex_fixed = sum(o[-1]["exact_path"] for o in fixed)
    ex_adapt = sum(o[-1]["exact_path"] for o in adapt)
    refined = [o[-1]["local_dims"] != f[-1]["local_dims"] for o, f in zip(adapt, fixed)]
    assert any(refined), [o[-1]["local_dims"] for o in adapt]
    assert ex_adapt <= ex_fixed, (ex_adapt, ex_fixed)


def test_rccl_world1_graph_replay(cuda):
    """Steady distributed steps replayed from a hipGraph (torch.cuda.CUDAGraph, the default at
    world 1): back-to-back replays without host synchronisation are all valid and give the eager
    steady step's rows (and the routed full step's) bit for bit; a call with other input storage
    recaptures on graph-owned buffers with the same rows; a moved share reports invalid through
    the in-graph flag and the synchronous call recovers the full step's rows."""
    import subprocess
    import sys

    from cuda_knearests_amd.utils import REPO

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, PYTHONPATH=str(REPO), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
               RANK="0", WORLD_SIZE="1")
    r = subprocess.run([sys.executable, str(REPO / "scripts" / "diag_dist_graph.py"), "60", "200000"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    assert "graph True valid True same rows as eager True" in r.stdout
    assert "staged True True moved share invalid True recovered True" in r.stdout


@pytest.mark.parametrize("world,gen,hf", [(4, "uniform", 0.6), (8, "clustered", 1.0)])
def test_steady_forwarding_on_device(cuda, world, gen, hf):
    """A halo too narrow for every query (uncertified queries each step): the validated step
    forwards them on the host, and the following asynchronous steady steps forward them ON THE
    DEVICE (fixed slots, equal-split all-to-alls): every steady step is valid and its rows equal
    the kd-tree oracle's (route.hip launch_fwd_pack / launch_fwd_merge)."""
    import cuda_knearests_amd as kn
    from cuda_knearests_amd.parallel import DistributedKNearests, run_loopback
    from cuda_knearests_amd.utils import clustered_cloud

    n, k = 30000, 16
    cloud = uniform_cloud(n, seed=91) if gen == "uniform" else clustered_cloud(n, seed=92)
    owner = torch.arange(n) % world

    def body(t):
        m = owner == t.rank
        ids = torch.nonzero(m).flatten().to(torch.int32).to(cuda)
        pts = cloud[m].contiguous().to(cuda)
        dk = DistributedKNearests(k=k, transport=t, halo_factor=hf, halo_field=0)
        dk.halo_boost_max = 1.0  # no adaptive halo: the steady steps forward on the device
        r0 = dk.solve(pts, ids)
        outs = []
        for _ in range(3):
            r = dk.solve(pts, ids, async_=True)
            outs.append((r.valid(), bool(r.stats.get("steady")), r.ids.cpu(), r.neighbors.cpu(), r.d2.cpu()))
        return r0.stats, outs

    out = run_loopback(world, body)
    _, od = kn.knn_cpu(cloud, k, "kdtree")
    assert any(st["forwarded"] > 0 for st, _ in out), "the halo was wide enough: nothing was forwarded"
    for st, outs in out:
        for ok, steady, ids, nb, d2 in outs:
            assert steady and ok, (st, steady, ok)
            ids = ids.long()
            assert torch.equal(d2, od[ids])
            assert_knn_exact(cloud, ids, nb, d2, od[ids])


def test_adaptive_halo_boost(cuda):
    """A validated step that needed forwarding widens the halo (x1.6 per full step, kept across
    steps) instead of entering the steady state with device forwarding; once a step needs none,
    the asynchronous steady steps follow, every row exact (distributed.py halo_boost)."""
    import cuda_knearests_amd as kn
    from cuda_knearests_amd.parallel import DistributedKNearests, run_loopback

    world, n, k = 4, 30000, 16
    cloud = uniform_cloud(n, seed=93)
    owner = torch.arange(n) % world

    def body(t):
        m = owner == t.rank
        ids = torch.nonzero(m).flatten().to(torch.int32).to(cuda)
        pts = cloud[m].contiguous().to(cuda)
        dk = DistributedKNearests(k=k, transport=t, halo_factor=0.6, halo_field=0)
        hist = []
        for _ in range(6):
            r = dk.solve(pts, ids, async_=True)
            hist.append((bool(r.stats.get("steady")), r.valid(), int(r.stats["forwarded"]), dk.halo_boost,
                         r.ids.cpu(), r.d2.cpu()))
        return hist

    out = run_loopback(world, body)
    _, od = kn.knn_cpu(cloud, k, "kdtree")
    for hist in out:
        assert hist[0][2] > 0 and hist[-1][3] > 1.0, [h[:4] for h in hist]  # forwarded, then widened
        assert hist[-1][0], [h[:4] for h in hist]  # steady by the last step
        for steady, ok, _, _, ids, d2 in hist:
            assert ok
            assert torch.equal(d2, od[ids.long()])


def test_rccl_world1_native_pipeline(cuda):
    """kn::DistPipeline at world 1 over a real RCCL communicator, plain and with forced
    collectives (the own rows through an RCCL self send / recv + unpack): asynchronous per-call
    steps, batched unrolled run_steps (with and without resident priming), in-place refills
    between calls, a moved share and the per-phase profile; rows bit-identical to the torch
    path's (scripts/diag_dist_pipe.py)."""
    import subprocess
    import sys

    from cuda_knearests_amd.utils import REPO

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, PYTHONPATH=str(REPO), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
               RANK="0", WORLD_SIZE="1")
    r = subprocess.run([sys.executable, str(REPO / "scripts" / "diag_dist_pipe.py"), "30", "200000"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    assert "ALL OK" in r.stdout


@pytest.mark.parametrize("world,gen", [(2, "uniform"), (4, "uniform"), (8, "uniform"), (8, "clustered")])
def test_native_pipeline_loopback_layouts(cuda, world, gen):
    """kn::DistPipeline at world > 1 without RCCL (loopback mode, one GPU): every virtual rank's
    pipeline routes its share, the test moves the rows between the ranks' send / receive buffers
    exactly as the grouped ncclSend / ncclRecv would, then unpack + build + query + flag; the rows
    are bit-identical to the torch path's steady step and every local flag is clear. This checks
    the send / receive offsets, the unpack table and the local plan the RCCL pipeline uses."""
    from cuda_knearests_amd._ext import load
    from cuda_knearests_amd.parallel import DistributedKNearests, SpatialDecomposition, run_loopback
    from cuda_knearests_amd.utils import clustered_cloud

    C = load()
    n = 60000
    if gen == "uniform":
        shares = []
        for r in range(world):
            blo, bhi = SpatialDecomposition(world, (0.0,) * 3, (1000.0,) * 3).rank_box(r)
            u = uniform_cloud(n, seed=400 + r, device=cuda, lo=0.0, hi=1.0)
            shares.append((u * torch.tensor([bhi[a] - blo[a] for a in range(3)], device=cuda)
                           + torch.tensor(blo, device=cuda)).contiguous())
    else:
        shares = [c.contiguous() for c in clustered_cloud(n * world, seed=77).to(cuda).chunk(world)]

    def body(t):
        dk = DistributedKNearests(k=16, transport=t)
        r1 = dk.solve(shares[t.rank])
        for _ in range(6):  # clustered: full steps widen the halo until nothing is forwarded
            r1 = dk.solve(shares[t.rank])  # steady step, torch path (loopback transport)
            if r1.stats.get("steady"):
                break
        assert r1.valid() and r1.stats.get("steady")
        return dk._steady, r1.ids.clone(), r1.neighbors.clone(), r1.d2.clone()

    out = run_loopback(world, body)
    pipes = []
    for r, (st, _, _, _) in enumerate(out):
        pipes.append(C.DistPipe(None, shares[r], None, st["plan"], st["metas"], [int(v) for v in st["tot"].tolist()],
                                [float(v) for v in st["hdr"]], list(st["grid"]), list(st["dims"]), list(st["recv_own"]),
                                list(st["recv_halo"]), list(st["cross_send"]), list(st["cross_recv"]), list(st["place"]),
                                int(st["cap"]), 16, 0.0, True, int(st["exact_grid"]), int(st["use_tree"]), False,
                                [world, r], st.get("field"), st.get("field_cert")))
    for p in pipes:
        p.loopback_stage(0)
    for r in range(world):
        for d in range(world):
            m = out[r][0]["cross_send"][d]
            if d != r and m:
                assert out[d][0]["cross_recv"][r] == m
                pipes[d].recv_view(r, m).copy_(pipes[r].send_view(d, m))
    torch.cuda.synchronize()
    for p in pipes:
        p.loopback_stage(1)
    for r, (st, ids, nb, d2) in enumerate(out):
        g, i, d = pipes[r].outputs(0)
        assert pipes[r].flag_local() == 0, r
        assert torch.equal(g, ids) and torch.equal(i, nb) and torch.equal(d, d2), r
    # send / recv views own their pipeline: drop every pipe, allocate and
    # free other device memory, then read the views -- still the pipelines' rows
    held = []
    for r in range(world):
        for d in range(world):
            m = out[r][0]["cross_send"][d]
            if d != r and m:
                held.append((pipes[r].send_view(d, m), pipes[d].recv_view(r, m)))
    snap = [(a.clone(), b.clone()) for a, b in held]
    outs = [pp.outputs(0) for pp in pipes]
    del pipes, p
    junk = [C.DistPipe.__name__, torch.full((1 << 22,), 7.0, device=cuda)]
    torch.cuda.synchronize()
    for (a, b), (a0, b0) in zip(held, snap):
        assert torch.equal(a, a0) and torch.equal(b, b0) and torch.equal(a, b)
    for r, (st, ids, nb, d2) in enumerate(out):
        assert torch.equal(outs[r][1], nb), r
    del junk


@pytest.mark.parametrize("world,gen", [(4, "uniform"), (8, "clustered")])
def test_halo_field(cuda, world, gen):
    """Density-adaptive halo field (route.hip field_splat / field_cert): the first full step routes
    with the global widths and splats the measured K-th distances; the second routes each point
    with its field cell's width and certifies every query. Uniform: fewer halo rows, the field step
    becomes the steady plan. Small clustered cloud: sparse outliers force coarse cells, the field
    ships MORE rows than the global widths, and the solver falls back to them for good. Either
    way the steady steps are valid and exact, and a moved cloud fails the steady check and the
    synchronous solve recovers the exact rows."""
    import cuda_knearests_amd as kn
    from cuda_knearests_amd.parallel import DistributedKNearests, run_loopback
    from cuda_knearests_amd.utils import clustered_cloud

    n, k = 40000 * world, 16
    cloud = uniform_cloud(n, seed=61) if gen == "uniform" else clustered_cloud(n, seed=62)
    moved = cloud.clone()
    moved[:, 1] = moved[:, 1] * 0.8 + 11.0
    owner = torch.arange(n) % world

    def body(t):
        m = owner == t.rank
        ids = torch.nonzero(m).flatten().to(torch.int32).to(cuda)
        pts = cloud[m].contiguous().to(cuda)
        dk = DistributedKNearests(k=k, transport=t)
        r0 = dk.solve(pts, ids)
        r1 = dk.solve(pts, ids)
        rs = r1
        for _ in range(3):  # until steady (the fallback adds one more full step)
            rs = dk.solve(pts, ids, async_=True)
            if rs.stats.get("steady"):
                break
        ok2 = rs.valid()
        r3 = dk.solve(moved[m].contiguous().to(cuda), ids, async_=True)
        ok3 = r3.valid()
        r4 = dk.solve(moved[m].contiguous().to(cuda), ids)
        return (dict(r0.stats), dict(r1.stats), ok2, bool(rs.stats.get("steady")), ok3, dict(rs.stats),
                rs.ids.cpu(), rs.neighbors.cpu(), rs.d2.cpu(), r4.ids.cpu(), r4.d2.cpu(), dk.halo_field_g)

    out = run_loopback(world, body)
    _, od = kn.knn_cpu(cloud, k, "kdtree")
    _, odm = kn.knn_cpu(moved, k, "kdtree")
    halo0 = sum(o[0]["n_halo"] for o in out)
    halo1 = sum(o[1]["n_halo"] for o in out)
    for s0, s1, ok2, steady2, ok3, ss, i2, n2, d2, i4, d4, g in out:
        assert not s0["halo_field"] and s1["halo_field"] and s1["forwarded"] == 0, (s0, s1)
        assert ok2 and steady2 and not ok3
        assert torch.equal(d2, od[i2.long()])
        assert_knn_exact(cloud, i2.long(), n2, d2, od[i2.long()])
        assert torch.equal(d4, odm[i4.long()])
        if gen == "uniform":
            assert ss["halo_field"] and g > 0  # the field is the steady plan
        else:
            assert not ss["halo_field"] and g == 0  # fell back to the global widths
    if gen == "uniform":
        assert halo1 < halo0, (halo1, halo0)
    else:
        assert halo1 >= halo0, (halo1, halo0)


@pytest.mark.parametrize("inject", [None, "1"])
def test_bench_two_ranks_supervised_fallback(cuda, inject):
    """the N-GPU bench must not lose its number. `bench.py --gpus 2` on this one
    GPU (KN_SAME_DEVICE=1, gloo process group). With KN_DIST_INJECT_FAIL=1 rank 1 raises in its first
    pipelined launch: the supervisors kill the first attempt's children on BOTH ranks (rank 0's is
    blocked in a collective) and the fallback attempt (KN_DIST_PIPE=0) prints the one JSON line,
    naming its path and the failure, with 0 bad rows on every rank."""
    import json
    import subprocess
    import sys

    from cuda_knearests_amd.utils import REPO
    from cuda_knearests_amd.utils.supervise import free_port

    env = dict(os.environ, KN_SAME_DEVICE="1", KN_DIST_BACKEND="gloo", MASTER_PORT=str(free_port()))
    env.pop("KN_DIST_INJECT_FAIL", None)
    if inject:
        env["KN_DIST_INJECT_FAIL"] = inject
    r = subprocess.run([sys.executable, str(REPO / "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "2",
                        "--points", "60000"], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["value"] > 0
    assert d["check"]["bad_rows_all_ranks"] == 0
    if inject:
        assert d["dist_path"] == "torch_steady"
        fa = d["failed_attempts"][0]
        assert fa["path"] == "native_pipeline" and fa["rc"] != 0
        # the injected rank is among the failed ones (its blocked peer may die first) and its
        # stderr names the failure
        by_rank = {x["rank"]: x for x in fa["failed_ranks"]}
        assert 1 in by_rank and by_rank[1]["rc"] != 0, fa
        assert any("injected failure" in s for s in by_rank[1]["stderr_tail"]), fa
    else:
        assert d["dist_path"] == "native_pipeline" and d["first_attempt_rc"] == 0
