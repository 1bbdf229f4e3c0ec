"""GPU tests of the Morton-leaf tree path (csrc/kernels/tree.hip, kn/tree.h) against the kd-tree
oracle: bitwise-equal distances, ids distinct / not self / reproducing their distance
(cuda_knearests_amd/utils/check.py), on the clouds the grid cannot adapt to and on the
reference's uniform ones."""
import pytest
import torch

import cuda_knearests_amd as kn
from cuda_knearests_amd.utils import clustered_cloud, surface_cloud, uniform_cloud
from cuda_knearests_amd.utils.check import assert_knn_exact

pytestmark = pytest.mark.gpu


def _check(p, idx, d2, k, n_queries=None):
    nq = p.size(0) if n_queries is None else n_queries
    pc = p.cpu()
    oi, od = kn.knn_cpu(pc, k, "kdtree")
    idx, d2 = idx.cpu(), d2.cpu()
    assert idx.shape == (nq, k)
    mism = (d2 != od[:nq]).any(1)
    assert int(mism.sum()) == 0, f"{int(mism.sum())} rows differ; first {int(mism.nonzero()[0, 0])}"
    assert_knn_exact(pc, torch.arange(nq), idx, d2, od[:nq])


@pytest.mark.parametrize("k,gen", [(1, "uniform"), (8, "clustered"), (16, "uniform"), (16, "clustered"),
                                   (16, "surface"), (32, "clustered"), (50, "clustered"), (64, "surface"),
                                   (100, "clustered")])
def test_tree_vs_oracle(cuda, k, gen):
    mk = {"uniform": uniform_cloud, "clustered": clustered_cloud, "surface": surface_cloud}[gen]
    p = mk(40000, seed=600 + k).to(cuda)
    g = kn.build_grid(p, k, adaptive=True)
    idx, d2, info = kn.query(g, k, algo="tree", return_info=True)
    _check(p, idx, d2, k)
    if k <= 64:
        # near-ties and visit-cap overflows only: the exact finish is a small minority
        assert int(info["counters"][0]) < p.size(0) // 20


@pytest.mark.parametrize("k", [1, 16, 50])
def test_tree_forced_exact_finish(cuda, k):
    # flags bit 0 sends every query through the exact traversal (the rare branch, covered)
    p = clustered_cloud(20000, seed=700 + k).to(cuda)
    g = kn.build_grid(p, k, adaptive=True)
    idx, d2, info = kn.query(g, k, algo="tree", return_info=True, flags=1)
    assert int(info["counters"][0]) == p.size(0)
    _check(p, idx, d2, k)
    i2, e2 = kn.query(g, k, algo="tree")
    assert torch.equal(idx, i2) and torch.equal(d2, e2)


def test_tree_matches_grid_bitwise(cuda):
    # same arithmetic, same tie rule (d2, id): identical output to the grid path
    p = uniform_cloud(50000, seed=801, device=cuda)
    g = kn.build_grid(p, 16)
    i1, e1 = kn.query(g, 16)
    i2, e2 = kn.query(g, 16, algo="tree")
    assert torch.equal(i1, i2) and torch.equal(e1, e2)


def test_tree_duplicates_tiny_and_subsets(cuda):
    p = uniform_cloud(3000, seed=9)
    p = torch.cat([p, p, p[:100]]).to(cuda)  # exact duplicates: d2 = 0 ties
    g = kn.build_grid(p, 8)
    idx, d2 = kn.query(g, 8, algo="tree")
    _check(p, idx, d2, 8)
    for n in (1, 2, 3, 9, 17, 63, 64, 65, 129):
        q = uniform_cloud(n, seed=n, device=cuda)
        g = kn.build_grid(q, 8)
        idx, d2 = kn.query(g, 8, algo="tree")
        _check(q, idx, d2, 8)
    # queries = a prefix of the original indices, ids through an id map
    p = clustered_cloud(30000, seed=11).to(cuda)
    g = kn.build_grid(p, 16, adaptive=True)
    idx, d2 = kn.query(g, 16, n_queries=12345, algo="tree")
    _check(p, idx, d2, 16, n_queries=12345)
    id_map = torch.arange(p.size(0), device=cuda, dtype=torch.int32) * 3
    i2, e2 = kn.query(g, 16, n_queries=12345, id_map=id_map, algo="tree")
    assert torch.equal(i2, idx * 3) and torch.equal(e2, d2)


def test_tree_single_point_cluster(cuda):
    # 20K points on one spot plus a sparse background: every Morton code of the cluster collides
    g0 = torch.Generator().manual_seed(5)
    core = 500 + 1e-3 * torch.randn((20000, 3), generator=g0)
    bg = 1000 * torch.rand((2000, 3), generator=g0)
    p = torch.cat([core, bg]).to(cuda)
    g = kn.build_grid(p, 16, adaptive=True)
    idx, d2 = kn.query(g, 16, algo="tree")
    _check(p, idx, d2, 16)


@pytest.mark.parametrize("gen,expect", [("clustered", "tree"), ("uniform", "grid")])
def test_engine_auto_algo(cuda, gen, expect):
    # kn::Engine (C API runtime): the tree when the adaptive grid was refined; steps through
    # launch_graph (eager for the tree: the leaf count sizes its node buffer) stay exact
    from cuda_knearests_amd._ext import load

    C = load()
    p = (clustered_cloud if gen == "clustered" else uniform_cloud)(40000, seed=31).to(cuda)
    e = C.Engine(16)
    e.prepare(p)
    e.solve()
    assert e.info()["algo"] == expect
    idx, d2 = e.results(cuda)
    _check(p, idx, d2, 16)
    e.prepare_async(p)
    e.launch_graph(2)
    e.sync()
    i2, e2 = e.results(cuda)
    assert torch.equal(i2, idx) and torch.equal(e2, d2)
    # forced structures agree bit for bit
    for algo in (1, 2):
        f = C.Engine(16, algo=algo)
        f.prepare(p)
        f.solve()
        i3, e3 = f.results(cuda)
        assert torch.equal(e3, d2)


def test_knearests_model_tree(cuda):
    p = clustered_cloud(30000, seed=41).to(cuda)
    m = kn.KNearests(k=16, device=cuda).prepare(p).solve()
    assert m.info["algo"] == "tree"
    _check(p, m.neighbors, m.distances, 16)
    m.step(p, capture=True)
    _check(p, m.neighbors, m.distances, 16)


@pytest.mark.parametrize("k,gen", [(16, "uniform"), (50, "uniform"), (16, "clustered")])
def test_engine_pipelined_steps(cuda, k, gen):
    """kn::Engine::launch_pipelined: step i+1's binning on a second stream over the other grid set
    while step i queries. Results of any step count equal the graph replay's bit for bit, the
    engine's grid afterwards is the last step's (stored-space getters stay consistent), and the
    tree path falls back to launch_graph."""
    from cuda_knearests_amd._ext import load

    C = load()
    p = (clustered_cloud if gen == "clustered" else uniform_cloud)(60000, seed=53).to(cuda)
    e = C.Engine(k)
    e.prepare(p)
    e.solve()
    idx, d2 = e.results(cuda)
    _check(p, idx, d2, k)
    perm0 = e.get_permutation()
    for steps in (1, 2, 3, 4, 7):
        e.launch_pipelined(steps)
        e.sync()
        i2, e2 = e.results(cuda)
        assert torch.equal(i2, idx) and torch.equal(e2, d2), steps
        assert torch.equal(e.get_permutation(), perm0), steps
    e.launch_graph(2)
    e.sync()
    i3, e3 = e.results(cuda)
    assert torch.equal(i3, idx) and torch.equal(e3, d2)


@pytest.mark.parametrize("k", [16])
def test_engine_pipeline_relabel_then_new_points(cuda, k):
    """A serial graph captured before an even number of pipelined steps must not survive the
    grid-set relabel: launch_graph -> launch_pipelined(2) -> new points -> launch_graph
    rebuilds into the LIVE set, so the permutation and the rows match a fresh engine on the new
    points; set_k after an even pipelined run keeps the live grid (no use of freed memory)."""
    from cuda_knearests_amd._ext import load

    C = load()
    p = uniform_cloud(50000, seed=71).to(cuda)
    q = (p + 0.37).contiguous()  # moved cloud, same size
    e = C.Engine(k)
    e.prepare(p)
    e.launch_graph(1)
    e.launch_pipelined(2)
    e.sync()
    e.prepare_async(q)
    e.launch_graph(1)
    e.sync()
    ref = C.Engine(k)
    ref.prepare(q)
    ref.solve()
    i1, d1 = e.results(cuda)
    i0, d0 = ref.results(cuda)
    assert torch.equal(i1, i0) and torch.equal(d1, d0)
    assert torch.equal(e.get_permutation(), ref.get_permutation())
    # even pipelined run, then a K change: the grid stays valid for the next solve
    e.launch_pipelined(2)
    e.sync()
    e.set_k(8)
    e.solve()
    ref.set_k(8)
    ref.solve()
    i1, d1 = e.results(cuda)
    i0, d0 = ref.results(cuda)
    assert torch.equal(i1, i0) and torch.equal(d1, d0)


@pytest.mark.parametrize("unroll", [0, 4])
def test_engine_stream_of_clouds(cuda, unroll):
    """kn::Engine::stream_step: 7 DIFFERENT clouds through pipelined steps (the next cloud is
    binned while the current one queries); every step's rows equal the kd-tree oracle's on its
    own cloud, and a resident pipelined run afterwards solves the last cloud."""
    from cuda_knearests_amd._ext import load

    C = load()
    k = 16
    n = 30000
    clouds = [uniform_cloud(n, seed=900 + j).to(cuda) for j in range(7)]
    clouds[3] = (clouds[3] * 0.5 + 100.0).contiguous()  # another domain: the bbox is per build
    e = C.Engine(k)
    e.prepare(clouds[0])
    e.launch_pipelined(2, unroll)  # a primed resident pipeline first: the stream must not use it
    for j, c in enumerate(clouds):
        e.stream_step(c, clouds[j + 1] if j + 1 < len(clouds) else None)
        e.sync()
        idx, d2 = e.results(cuda)
        _check(c, idx, d2, k)
        perm = e.get_permutation()
        assert torch.equal(perm.sort().values, torch.arange(n, dtype=perm.dtype)), j
    e.launch_pipelined(6, unroll)
    e.sync()
    idx, d2 = e.results(cuda)
    _check(clouds[-1], idx, d2, k)


@pytest.mark.parametrize("mode", ["eager", "graph"])
@pytest.mark.parametrize("k,gen", [(16, "uniform"), (50, "uniform"), (32, "uniform"), (16, "clustered")])
def test_engine_stream_batch(cuda, k, gen, mode):
    """kn::Engine::stream_batch: a batch of DISTINCT clouds, every step's rows written straight
    into the caller's buffers and equal to the kd-tree oracle's on its own cloud. mode "eager"
    (default): a second pipeline over the same grid sets, one step_with() per cloud, queries
    alternating between the two query streams; "graph": one captured graph per power-of-two chunk
    (pointer table written per launch; 11 steps = chunks of 8, 2 and 1). K=32 runs the exact finish
    as the build-stream epilogue, K=50 on the query stream, clustered clouds the tree path; a
    resident pipelined launch and a stream step afterwards still solve their clouds."""
    from cuda_knearests_amd._ext import load
    from cuda_knearests_amd.utils import clustered_cloud

    C = load()
    n = 30000
    mk = uniform_cloud if gen == "uniform" else clustered_cloud
    clouds = [mk(n, seed=700 + j).to(cuda) for j in range(11)]
    clouds[4] = (clouds[4] * 0.25 + 300.0).contiguous()  # another domain: the bbox is per build
    e = C.Engine(k)
    e.prepare(clouds[0])
    e.launch_pipelined(4, 2)  # a primed resident pipeline first
    idx = [torch.empty(n, k, dtype=torch.int32, device=cuda) for _ in clouds]
    d2 = [torch.empty(n, k, dtype=torch.float32, device=cuda) for _ in clouds]
    e.stream_batch(clouds, idx, d2, mode=mode)
    e.sync()
    for j, c in enumerate(clouds):
        _check(c, idx[j], d2[j], k)
    # a second batch reuses the pipeline / captured graphs (and the same output buffers)
    e.stream_batch(clouds[::-1][:3], idx[:3], d2[:3], mode=mode)
    e.sync()
    for j, c in enumerate(clouds[::-1][:3]):
        _check(c, idx[j], d2[j], k)
    e.launch_pipelined(2, 0)  # the resident cloud after a batch: the last batch cloud
    e.sync()
    i2, e2 = e.results(cuda)
    _check(clouds[::-1][2], i2, e2, k)
    e.stream_step(clouds[5], None)
    e.sync()
    i3, e3 = e.results(cuda)
    _check(clouds[5], i3, e3, k)


def test_tree_long_axis(cuda):
    """Tree path on a grid with more than 1,024 cells along one axis (the cells'
    Morton codes were u32 and overflowed past 128 bricks per axis). Multi-GPU ranks build such
    grids from their box extents (slab-shaped shares); here a uniform 1000 x 8 x 8 slab is binned
    into a 2048 x 8 x 8 grid and queried through the tree: rows equal the oracle's."""
    from cuda_knearests_amd._ext import load

    C = load()
    k = 16
    n = 120000
    g = torch.Generator().manual_seed(17)
    p = (torch.rand(n, 3, generator=g) * torch.tensor([1000.0, 8.0, 8.0])).contiguous()
    dims = [2048, 8, 8]
    s, cs, perm, geom = C.build(p.to(cuda), dims, True, None)
    ws, nodes, leaves = C.tree_build(s, cs, geom, dims, True)
    assert leaves > 0
    idx, d2, counters = C.tree_query(ws, nodes, dims, n, k, n)
    torch.cuda.synchronize()
    _check(p, idx, d2, k)


@pytest.mark.parametrize("qstreams", [1, 2])
@pytest.mark.parametrize("k", [16, 50])
def test_engine_stream_after_unrolled(cuda, k, qstreams):
    """A stream step issued right after an UNROLLED resident launch, with no sync in between
    (the unrolled graph's last queries and its primed build use both grid sets, so the
    stream step's copy into a set must wait for the whole graph, not for a pre-graph event).
    K=16 has no epilogue (nothing on the side stream follows the graph), K=50 has one. Every
    stream step's rows equal the oracle's on its own cloud. One query stream and two sets
    (set_pipeline_shape) is the shape that really runs unrolled graphs; with the default
    two query streams the same calls run per-step graphs."""
    from cuda_knearests_amd._ext import load

    C = load()
    unroll = 4
    n = 40000
    base = uniform_cloud(n, seed=41).to(cuda)
    clouds = [uniform_cloud(n, seed=950 + j).to(cuda) for j in range(3)]
    e = C.Engine(k)
    if qstreams == 1:
        e.set_pipeline_shape(1, 2)
    e.prepare(base)
    for rep in range(2):
        e.launch_pipelined(2 * unroll, unroll)  # unrolled graphs, primed at the end
        for j, c in enumerate(clouds):
            e.stream_step(c, clouds[j + 1] if j + 1 < len(clouds) else None)
            if j == 0:
                continue  # first result checked after the next step was enqueued as well
            e.sync()
            idx, d2 = e.results(cuda)
            _check(c, idx, d2, k)
        e.prepare(base)


@pytest.mark.parametrize("qstreams", [1, 2])
@pytest.mark.parametrize("unroll", [2, 4, 8])
def test_engine_unrolled_pipeline(cuda, unroll, qstreams):
    """Unrolled pipelined graphs (U steps per graph launch, pipeline.hpp) give the serial step's
    rows bit for bit, for step counts that are not multiples of U, and mix with per-step launches
    and serial graph replays. qstreams 1 (two sets) runs the unrolled graphs themselves; 2 the
    default per-step graphs of two query streams."""
    from cuda_knearests_amd._ext import load

    C = load()
    p = uniform_cloud(60000, seed=57).to(cuda)
    e = C.Engine(16)
    if qstreams == 1:
        e.set_pipeline_shape(1, 2)
    e.prepare(p)
    e.solve()
    idx, d2 = e.results(cuda)
    for steps in (unroll, unroll + 1, 3 * unroll + 3, 1):
        e.launch_pipelined(steps, unroll)
        e.sync()
        i2, e2 = e.results(cuda)
        assert torch.equal(i2, idx) and torch.equal(e2, d2), steps
    e.launch_graph(1)
    e.launch_pipelined(2 * unroll, unroll)
    e.sync()
    i3, e3 = e.results(cuda)
    assert torch.equal(i3, idx) and torch.equal(e3, d2)
