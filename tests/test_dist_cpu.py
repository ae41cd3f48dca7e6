"""Data-parallel layer on CPU (gloo, world_size 2): GradArena all-reduce, sharding, and the
"G shards == one big batch" gradient equivalence of the training loss (with the sum-type sparsity
term scaled by G), computed with the CPU oracle as the stand-in for the per-rank kernels."""
import os
import socket

import numpy as np
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
