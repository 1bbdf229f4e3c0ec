"""Multi-process distributed path on CPU ranks (gloo) -- SURVEY §4.2 item 3.

Each rank gets an arbitrary share of a global cloud; DistributedKNearests redistributes,
exchanges halos and solves locally. The union of the per-rank results must equal the
single-process oracle for every point (global ids, distance-aware).
"""
import os
import socket
import sys

import pytest
import torch
import torch.multiprocessing as mp

from cuda_knearests_amd.utils.check import assert_knn_exact

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, k, gen, partitioned, halo_factor, q):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from cuda_knearests_amd.parallel import DistributedKNearests, SpatialDecomposition
    from cuda_knearests_amd.utils import clustered_cloud, uniform_cloud

    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n = 6000
    cloud = uniform_cloud(n, 42) if gen == "uniform" else clustered_cloud(n, 43)
    ids = torch.arange(n, dtype=torch.int32)
    if partitioned:
        lo, hi = tuple(cloud.min(0).values.tolist()), tuple(cloud.max(0).values.tolist())
        dec = SpatialDecomposition(world, lo, hi)
        mine = dec.owner(cloud) == rank
    else:
        mine = (torch.arange(n) % world) == rank  # scattered, not spatial
    dk = DistributedKNearests(k=k, halo_factor=halo_factor)
    res = dk.solve(cloud[mine].contiguous(), ids[mine].contiguous(), partitioned=partitioned)
    # numpy copies travel by value (tensors would go through fds that die with the worker)
    q.put((rank, res.ids.numpy().copy(), res.neighbors.numpy().copy(), res.d2.numpy().copy(), res.stats))
    dist.barrier()
    dist.destroy_process_group()


def _run(world, k, gen="uniform", partitioned=False, halo_factor=1.6):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, k, gen, partitioned, halo_factor, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    return [(r, torch.from_numpy(i), torch.from_numpy(nb), torch.from_numpy(d), s) for r, i, nb, d, s in out]


@pytest.mark.parametrize("world,k,gen,partitioned", [
    (2, 8, "uniform", False),
    (2, 16, "uniform", True),
    (4, 16, "clustered", False),
])
def test_distributed_matches_single(world, k, gen, partitioned):
    import cuda_knearests_amd as kn
    from cuda_knearests_amd.utils import clustered_cloud, uniform_cloud

    out = _run(world, k, gen, partitioned)
    n = 6000
    cloud = uniform_cloud(n, 42) if gen == "uniform" else clustered_cloud(n, 43)
    oi, od = kn.knn_cpu(cloud, k, "kdtree")
    seen = torch.zeros(n, dtype=torch.bool)
    for rank, ids, nb, d2, stats in out:
        ids = ids.long()
        assert not bool(seen[ids].any()), "a point is owned by two ranks"
        seen[ids] = True
        assert torch.equal(d2, od[ids]), f"rank {rank}: distances differ"
        assert_knn_exact(cloud.cpu(), ids, nb.cpu(), d2.cpu(), od[ids])
    assert bool(seen.all()), "some points were lost in redistribution"


def test_halo_growth_round():
    # a deliberately tiny halo forces uncertified queries -> the halo doubles until certified
    out = _run(2, 16, "uniform", False, halo_factor=0.05)
    assert max(s["rounds"] for *_, s in out) > 1


def test_decomposition_factors():
    from cuda_knearests_amd.parallel import SpatialDecomposition, factor3

    assert sorted(factor3(2)) == [1, 1, 2]
    assert sorted(factor3(4)) == [1, 2, 2]
    assert factor3(8) == (2, 2, 2)
    assert sorted(factor3(6)) == [1, 2, 3]
    d = SpatialDecomposition(8, (0, 0, 0), (1000, 1000, 1000))
    pts = torch.rand(10000, 3) * 1000
    o = d.owner(pts)
    for r in range(8):
        lo, hi = d.rank_box(r)
        m = o == r
        assert bool(((pts[m] >= torch.tensor(lo)) & (pts[m] <= torch.tensor(hi))).all())
    cb = d.complete_box(0, 10.0)
    assert cb[0] == float("-inf") and cb[3] == 510.0


def test_balanced_splits_kd_layout():
    # count-balanced kd splits: every point lies in its owner's box, every box holds ~N/world
    from cuda_knearests_amd.parallel import SpatialDecomposition
    from cuda_knearests_amd.parallel.decomposition import balanced_splits, split_count
    from cuda_knearests_amd.utils import clustered_cloud

    pts = clustered_cloud(40000, seed=3)
    lo, hi = pts.min(0).values.double(), pts.max(0).values.double()
    for grid in [(2, 2, 2), (2, 1, 1), (3, 2, 1), (1, 1, 4)]:
        world = grid[0] * grid[1] * grid[2]
        sp = balanced_splits(pts, lo, hi, grid, lambda t: t)
        assert sp.dtype == torch.float32 and sp.numel() == split_count(grid)
        d = SpatialDecomposition(world, tuple(lo.tolist()), tuple(hi.tolist()), grid, sp.tolist())
        o = d.owner(pts)
        cnt = torch.bincount(o, minlength=world).double()
        assert float(cnt.max() / cnt.mean()) < 1.05, (grid, cnt.tolist())
        for r in range(world):
            blo, bhi = d.rank_box(r)
            m = o == r
            assert bool(((pts[m] >= torch.tensor(blo)) & (pts[m] <= torch.tensor(bhi))).all())
    # equal-volume boxes of the same clustered cloud are far from balanced
    dv = SpatialDecomposition(8, tuple(lo.tolist()), tuple(hi.tolist()), (2, 2, 2))
    cv = torch.bincount(dv.owner(pts), minlength=8).double()
    assert float(cv.max() / cv.mean()) > 1.3


def _loopback_check(world, k, gen, device, native, n=6000, halo_factor=1.6, scatter="mod", balance="count"):
    """Run the distributed solve on `world` virtual ranks (threads, LoopbackTransport) and
    compare the union of the per-rank results with the single-process kd-tree oracle."""
    import cuda_knearests_amd as kn
    from cuda_knearests_amd.parallel import DistributedKNearests, run_loopback
    from cuda_knearests_amd.utils import clustered_cloud, uniform_cloud

    cloud = uniform_cloud(n, 42) if gen == "uniform" else clustered_cloud(n, 43)
    ids = torch.arange(n, dtype=torch.int32)
    owner = torch.arange(n) % world if scatter == "mod" else torch.randint(0, world, (n,), generator=torch.Generator().manual_seed(5))

    def fn(t):
        m = owner == t.rank
        dk = DistributedKNearests(k=k, halo_factor=halo_factor, transport=t, native_route=native, balance=balance)
        r = dk.solve(cloud[m].contiguous().to(device), ids[m].contiguous().to(device))
        return r.ids.cpu(), r.neighbors.cpu(), r.d2.cpu(), r.stats

    out = run_loopback(world, fn)
    oi, od = kn.knn_cpu(cloud, k, "kdtree")
    seen = torch.zeros(n, dtype=torch.bool)
    for ids_r, nb, d2, stats in out:
        ids_r = ids_r.long()
        assert not bool(seen[ids_r].any()), "a point is owned by two ranks"
        seen[ids_r] = True
        assert torch.equal(d2, od[ids_r]), "distances differ from the oracle"
        assert_knn_exact(cloud.cpu(), ids_r, nb.cpu(), d2.cpu(), od[ids_r])
    assert bool(seen.all()), "some points were lost in routing"
    return out


@pytest.mark.parametrize("world,gen", [(3, "uniform"), (8, "clustered")])
def test_loopback_cpu_matches_single(world, gen):
    _loopback_check(world, 8, gen, "cpu", native=False)


def test_loopback_cpu_clustered_balanced_owners():
    # clustered cloud over 8 ranks: exact, and count-balanced boxes keep max/mean owned <= 1.3
    out = _loopback_check(8, 16, "clustered", "cpu", native=False, n=16000)
    own = torch.tensor([s["n_owned"] for *_, s in out], dtype=torch.float64)
    assert float(own.max() / own.mean()) <= 1.3, own.tolist()
    outv = _loopback_check(8, 16, "clustered", "cpu", native=False, n=16000, balance="volume")
    ownv = torch.tensor([s["n_owned"] for *_, s in outv], dtype=torch.float64)
    assert float(ownv.max() / ownv.mean()) > float(own.max() / own.mean())


def test_loopback_cpu_growth_round():
    out = _loopback_check(4, 16, "uniform", "cpu", native=False, halo_factor=0.05)
    assert max(s["rounds"] for *_, s in out) > 1


def _transport_worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from cuda_knearests_amd.parallel import TorchDistTransport

    dist.init_process_group("gloo", rank=rank, world_size=world)
    t = TorchDistTransport()
    cat = t.all_gather_cat(torch.arange(8, dtype=torch.float64) + 100 * rank)
    # uneven all-to-all: rank r sends (d + 1) rows of value 10 r + d to rank d
    send = torch.cat([torch.full((d + 1, 4), float(10 * rank + d)) for d in range(world)])
    out = torch.empty(sum(rank + 1 for _ in range(world)), 4)
    t.all_to_all_single(out, send, [rank + 1] * world, [d + 1 for d in range(world)])
    m = torch.tensor([float(rank * 3 % 5)])
    t.all_reduce_max(m)
    q.put((rank, cat.numpy().copy(), out.numpy().copy(), float(m.item())))
    dist.barrier()
    dist.destroy_process_group()


def test_torch_transport_collectives():
    """TorchDistTransport (the RCCL path's collectives) on gloo CPU ranks."""
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_transport_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted([q.get(timeout=300) for _ in range(world)], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    exp_cat = torch.cat([torch.arange(8, dtype=torch.float64) + 100 * r for r in range(world)])
    for rank, cat, recv, m in out:
        assert torch.equal(torch.from_numpy(cat), exp_cat)
        exp = torch.cat([torch.full((rank + 1, 4), float(10 * s + rank)) for s in range(world)])
        assert torch.equal(torch.from_numpy(recv), exp)
        assert m == max(float(r * 3 % 5) for r in range(world))


def _failing_worker(rank, world, port, mode):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import time

    import torch.distributed as dist

    from cuda_knearests_amd.parallel import CollectiveError, DistributedKNearests
    from cuda_knearests_amd.utils import uniform_cloud

    dist.init_process_group("gloo", rank=rank, world_size=world)
    if rank == 1:
        if mode == "raise":
            raise RuntimeError("simulated rank failure before the exchange")
        time.sleep(120)  # "hang": never joins the collective
        os._exit(0)
    dk = DistributedKNearests(k=8, timeout_s=8.0)
    try:
        dk.solve(uniform_cloud(2000, 5 + rank))
    except CollectiveError as e:
        print(f"rank {rank}: {e}", flush=True)
        os._exit(3)  # the group is unusable: exit non-zero, no teardown collectives
    os._exit(0)


@pytest.mark.parametrize("mode", ["raise", "hang"])
def test_dead_peer_fails_fast(mode):
    """SURVEY §5 failure detection: when a peer rank raises (its process exits) or hangs, the
    surviving rank's collective fails with CollectiveError within the library timeout and the
    process exits non-zero instead of blocking forever."""
    import time

    world = 2
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_failing_worker, args=(r, world, port, mode)) for r in range(world)]
    t0 = time.time()
    for p in procs:
        p.start()
    procs[0].join(timeout=90)
    elapsed = time.time() - t0
    for p in procs[1:]:
        if p.is_alive():
            p.kill()
        p.join(timeout=30)
    assert procs[0].exitcode == 3, f"rank 0 exit code {procs[0].exitcode}"
    assert elapsed < 80, f"rank 0 took {elapsed:.0f} s to fail"
