"""Data-parallel layer on CPU (gloo, world_size 2): GradArena all-reduce, sharding, and the
"G shards == one big batch" gradient equivalence of the training loss (with the sum-type sparsity
term scaled by G), computed with the CPU oracle as the stand-in for the per-rank kernels."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _loss(orc, raw, z, d, target, sparsity_scale):
    rgb, _, _, _, _, ent = orc.composite(raw, z, d, None, True)
    return torch.mean((rgb - target) ** 2) + 1e-3 * sparsity_scale * ent.sum()


def _worker(rank, world, port, out_dir):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from indoor_nerf_amd.dist import GradArena, init_process_group, shard
    from oracle import nerf_oracle as orc
    r, w, _ = init_process_group(backend="gloo")
    assert (r, w) == (rank, world)
    g = torch.Generator().manual_seed(0)
    R, S = 64, 32
    raw_full = torch.randn(R, S, 4, generator=g)
    z = torch.sort(2 + 4 * torch.rand(R, S, generator=g), -1)[0]
    d = torch.randn(R, 3, generator=g)
    target = torch.rand(R, 3, generator=g)
    # "parameters": the raw field values of this rank's rays are produced from a shared leaf
    param = torch.nn.Parameter(raw_full.clone())
    other = torch.nn.Parameter(torch.ones(5))
    arena = GradArena([param, other])
    arena.zero_()
    mine = shard(param, rank, world)
    loss = _loss(orc, mine, shard(z, rank, world), shard(d, rank, world), shard(target, rank, world), float(world))
    loss = loss + (other * (rank + 1)).sum()
    loss.backward()
    assert param.grad.data_ptr() == arena.flat.data_ptr()
    arena.allreduce_mean()
    np.save(os.path.join(out_dir, f"grad_{rank}.npy"), param.grad.numpy())
    np.save(os.path.join(out_dir, f"other_{rank}.npy"), other.grad.numpy())
    dist.destroy_process_group()


def test_dp_allreduce_matches_single_batch(tmp_path, oracle):
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    g0, g1 = np.load(tmp_path / "grad_0.npy"), np.load(tmp_path / "grad_1.npy")
    np.testing.assert_array_equal(g0, g1)                         # replicas agree after the all-reduce
    np.testing.assert_allclose(np.load(tmp_path / "other_0.npy"), np.full(5, 1.5, np.float32))
    # single-process reference: the same loss on the whole batch
    g = torch.Generator().manual_seed(0)
    R, S = 64, 32
    raw = torch.randn(R, S, 4, generator=g).requires_grad_(True)
    z = torch.sort(2 + 4 * torch.rand(R, S, generator=g), -1)[0]
    d = torch.randn(R, 3, generator=g)
    target = torch.rand(R, 3, generator=g)
    _loss(oracle, raw, z, d, target, 1.0).backward()
    np.testing.assert_allclose(g0, raw.grad.numpy(), rtol=1e-5, atol=1e-8)


def test_shard_layout():
    from indoor_nerf_amd.dist import shard
    t = torch.arange(12).reshape(6, 2)
    assert shard(t, 1, 3).tolist() == [[4, 5], [6, 7]]
    try:
        shard(t, 0, 4)
    except ValueError:
        pass
    else:
        raise AssertionError("uneven shard must raise")


def test_shard_ranges_tile_every_parameter():
    from indoor_nerf_amd.dist import shard_ranges
    sizes = [2048, 1024, 1984, 4096, 192, 1 << 12, 1 << 12, 5]
    offsets = list(np.cumsum([0] + sizes[:-1]))
    total = sum(sizes)
    for world in (1, 2, 3, 8):
        count = -(-total // world)
        covered = [np.zeros(n, np.int32) for n in sizes]
        for r in range(world):
            for i, rg in enumerate(shard_ranges(offsets, sizes, r * count, (r + 1) * count)):
                if rg is not None:
                    covered[i][rg[0]:rg[1]] += 1
        assert all((c == 1).all() for c in covered), world


class _SgdShard:
    """Stand-in for RAdam.set_shard/step on CPU: p[a:b] -= 0.5 * (grad shard x grad_scale) (RAdam's
    kernel reads the reduce-scatter's sum x 1/G the same way)."""

    def __init__(self, params):
        self.params, self.shard, self.grad_scale = params, None, 1.0

    def set_shard(self, shard, grad_scale=1.0):
        self.shard, self.grad_scale = shard, grad_scale

    def step(self):
        with torch.no_grad():
            for p in self.params:
                if self.shard is None:
                    p.view(-1).sub_(0.5 * p.grad.view(-1))
                elif p in self.shard:
                    a, b, g = self.shard[p]
                    p.view(-1)[a:b].sub_(0.5 * (g * self.grad_scale))


def _zero_worker(rank, world, port, out_dir, buckets=False):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from indoor_nerf_amd.dist import (GradArena, ShardedOptimizer, allreduce_calibration_stats, allreduce_mean_,
                                      init_process_group)
    init_process_group(backend="gloo", force=world == 1)   # world 1: the forced one-rank group (bench.py NERF_DIST_FORCE)
    assert dist.is_initialized() and dist.get_world_size() == world
    calls = {"rs": 0, "ag": 0}
    rs, ag = dist.reduce_scatter_tensor, dist.all_gather_into_tensor

    def rs_count(*a, **k):
        calls["rs"] += 1
        return rs(*a, **k)

    def ag_count(*a, **k):
        calls["ag"] += 1
        return ag(*a, **k)
    dist.reduce_scatter_tensor, dist.all_gather_into_tensor = rs_count, ag_count
    g = torch.Generator().manual_seed(0)
    params = [torch.nn.Parameter(torch.randn(n, generator=g)) for n in (300, 77, 1024, 5)]
    opt = _SgdShard(params)
    # buckets: the arena split before the third parameter (dist.ShardedOptimizer's per-bucket shards)
    arena = GradArena(params, pad_to=world * 64, bucket_starts=[params[2]] if buckets else ())
    assert len(arena.buckets) == (2 if buckets else 1)
    sh = ShardedOptimizer(opt, arena)
    for step in range(3):
        arena.zero_()
        gr = torch.Generator().manual_seed(10 * step + rank)
        for p in params:
            p.grad.copy_(torch.randn(p.shape, generator=gr))
        sh.reduce_grads()
        opt.step()
        sh.gather_params()
    np.save(os.path.join(out_dir, f"p_{rank}.npy"), torch.cat([p.detach().view(-1) for p in params]).numpy())
    np.save(os.path.join(out_dir, f"calls_{rank}.npy"), np.array([calls["rs"], calls["ag"]]))
    # A-CAQ calibration statistics: order-preserving uint32 images of (min, max) in int32
    vals = torch.tensor([[-3.0 + rank, 2.0 * rank], [0.5 * rank, -1.0 - rank]])

    def f2ord(x):
        u = x.view(torch.int32).to(torch.int64) & 0xFFFFFFFF
        u = torch.where(u >= 1 << 31, (~u) & 0xFFFFFFFF, u | (1 << 31))
        return torch.where(u >= 1 << 31, u - (1 << 32), u).to(torch.int32)
    st = torch.stack([f2ord(vals[:, 0]), f2ord(vals[:, 1])], 1)
    allreduce_calibration_stats(st)
    np.save(os.path.join(out_dir, f"st_{rank}.npy"), st.numpy())
    m = torch.tensor([1.0 + rank])
    allreduce_mean_(m)
    np.save(os.path.join(out_dir, f"m_{rank}.npy"), m.numpy())
    dist.destroy_process_group()


def test_sharded_optimizer_one_rank_group(tmp_path):
    """The forced one-rank process group (dist.init_process_group(force=True), bench.py
    NERF_DIST_FORCE=1): the ZeRO-1 collectives of one rank leave one process's own update."""
    mp.start_processes(_zero_worker, args=(1, _free_port(), str(tmp_path), True), nprocs=1, join=True,
                       start_method="spawn")
    g = torch.Generator().manual_seed(0)
    params = [torch.randn(n, generator=g) for n in (300, 77, 1024, 5)]
    for step in range(3):
        gr = torch.Generator().manual_seed(10 * step)
        grads = [torch.randn(p.shape, generator=gr) for p in params]
        for p, gp in zip(params, grads):
            p.sub_(0.5 * gp)
    np.testing.assert_array_equal(np.load(tmp_path / "p_0.npy"), torch.cat(params).numpy())
    # the collectives ran (3 steps x 2 buckets each), not a local shortcut
    assert np.load(tmp_path / "calls_0.npy").tolist() == [6, 6]


@pytest.mark.parametrize("buckets", [False, True], ids=["one_bucket", "two_buckets"])
def test_sharded_optimizer_gloo(tmp_path, buckets):
    """reduce_scatter_tensor / all_gather_into_tensor (the production collectives, every backend) over
    one bucket or two: the replicas agree and equal one process's update with the mean gradient."""
    world = 2
    mp.start_processes(_zero_worker, args=(world, _free_port(), str(tmp_path), buckets), nprocs=world, join=True,
                       start_method="spawn")
    p0, p1 = np.load(tmp_path / "p_0.npy"), np.load(tmp_path / "p_1.npy")
    np.testing.assert_array_equal(p0, p1)
    # single-process reference: full update with the mean gradient
    g = torch.Generator().manual_seed(0)
    params = [torch.randn(n, generator=g) for n in (300, 77, 1024, 5)]
    for step in range(3):
        grads = []
        for r in range(world):
            gr = torch.Generator().manual_seed(10 * step + r)
            grads.append([torch.randn(p.shape, generator=gr) for p in params])
        for i, p in enumerate(params):
            p.sub_(0.5 * ((grads[0][i] + grads[1][i]) * 0.5))
    np.testing.assert_array_equal(p0, torch.cat(params).numpy())
    # calibration statistics: elementwise min of mins, max of maxes over the ranks
    for r in range(world):
        st = np.load(tmp_path / f"st_{r}.npy").astype(np.int64) & 0xFFFFFFFF
        u = np.where(st >= 1 << 31, st & 0x7FFFFFFF, (~st) & 0xFFFFFFFF).astype(np.uint32).view(np.float32)
        np.testing.assert_array_equal(u, np.array([[-3.0, 2.0], [0.0, -1.0]], np.float32))
        np.testing.assert_allclose(np.load(tmp_path / f"m_{r}.npy"), [1.5])


class _MomentShard(_SgdShard):
    """_SgdShard with RAdam-like moments: on each rank only the rank's shard of exp_avg / exp_avg_sq
    holds the true values (k * (index + 1)); the rest holds rank-specific garbage."""

    def __init__(self, params, rank):
        super().__init__(params)
        self.rank = rank
        self.state = {p: {"exp_avg": torch.full(p.shape, -100.0 - rank), "exp_avg_sq": torch.full(p.shape, 7.0 + rank)}
                      for p in params}

    def fill_shard(self):
        for p in self.params:
            if p in self.shard:
                a, b, _ = self.shard[p]
                idx = torch.arange(a, b, dtype=torch.float32) + 1
                self.state[p]["exp_avg"].view(-1)[a:b] = idx
                self.state[p]["exp_avg_sq"].view(-1)[a:b] = 2 * idx

    def state_dict(self):
        return {"state": {i: {k: v.clone() for k, v in self.state[p].items()} for i, p in enumerate(self.params)}}


def _ckpt_worker(rank, world, port, out_dir, buckets=True):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from indoor_nerf_amd.dist import GradArena, ShardedOptimizer, init_process_group
    from indoor_nerf_amd.model import save_checkpoint
    init_process_group(backend="gloo")
    g = torch.Generator().manual_seed(0)
    params = [torch.nn.Parameter(torch.randn(n, generator=g)) for n in (300, 77, 1024, 5)]
    opt = _MomentShard(params, rank)
    sh = ShardedOptimizer(opt, GradArena(params, pad_to=world * 64, bucket_starts=[params[2]] if buckets else ()))
    opt.fill_shard()
    kw = {"network_fn": torch.nn.Linear(2, 2), "network_fine": None, "embed_fn": torch.nn.Linear(3, 1)}
    wrote = save_checkpoint(os.path.join(out_dir, "ckpt.tar"), 42, kw, opt, sharded=sh)
    np.save(os.path.join(out_dir, f"wrote_{rank}.npy"), np.array([int(wrote)]))
    dist.destroy_process_group()


def test_sharded_checkpoint_collective_save(tmp_path):
    """save_checkpoint(sharded=...) is collective: every rank calls it, the moment shards are
    assembled with one all-reduce, and exactly one rank (0) writes the reference's dict."""
    world = 2
    mp.start_processes(_ckpt_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    assert [int(np.load(tmp_path / f"wrote_{r}.npy")[0]) for r in range(world)] == [1, 0]
    ck = torch.load(tmp_path / "ckpt.tar", weights_only=True)
    assert ck["global_step"] == 42
    for i, n in enumerate((300, 77, 1024, 5)):
        idx = torch.arange(n, dtype=torch.float32) + 1
        st = ck["optimizer_state_dict"]["state"][i]
        torch.testing.assert_close(st["exp_avg"], idx, rtol=0, atol=0)
        torch.testing.assert_close(st["exp_avg_sq"], 2 * idx, rtol=0, atol=0)


def test_gather_gate_levels_from_buckets():
    """ShardedOptimizer's gated all-gather plan: the buckets after the first that hold only
    hash-table levels (._nerf_level, set by HashEmbedder), in ascending level order, each gated at its
    first level; a bucket with any other parameter ends the plan. No gates without overlap / on CPU."""
    from indoor_nerf_amd.dist import GradArena, ShardedOptimizer

    def make(starts):
        mlp = [torch.nn.Parameter(torch.zeros(n)) for n in (300, 77)]
        tabs = [torch.nn.Parameter(torch.zeros(1 << 10, 2)) for _ in range(4)]
        for i, t in enumerate(tabs):
            t._nerf_level = i
        params = mlp + tabs
        sh = ShardedOptimizer(_SgdShard(params), GradArena(params, pad_to=64, bucket_starts=starts(mlp, tabs)))
        return sh

    sh = make(lambda m, t: [t[2]])
    assert sh.gate_levels() == [] and sh._gates == {}       # overlap needs CUDA buckets
    assert sh._gate_levels() == {1: 2}
    assert make(lambda m, t: [t[1], t[3]])._gate_levels() == {1: 1, 2: 3}
    assert make(lambda m, t: [m[1]])._gate_levels() == {}     # bucket 1 holds an MLP tensor
    assert make(lambda m, t: [])._gate_levels() == {}


def test_table_gate_join_order():
    """hashgrid's gate registry: join() runs the host finish once, then the stream wait; gate_tables
    joins an older set first; take_gates hands the set over."""
    from indoor_nerf_amd import hashgrid

    class _Stream:
        def __init__(self):
            self.waited = []

        def wait_event(self, ev):
            self.waited.append(ev)

    calls = []
    s = _Stream()
    g = hashgrid.TableGate(8, "ev8", finish=lambda: calls.append("finish"))
    g.join(s)
    g.join(s)
    assert calls == ["finish"] and s.waited == ["ev8", "ev8"]
    hashgrid.gate_tables("cpu:test", [hashgrid.TableGate(12, "b"), hashgrid.TableGate(4, "a")])
    got = hashgrid.take_gates("cpu:test")
    assert [x.level for x in got] == [4, 12] and hashgrid.take_gates("cpu:test") == []
