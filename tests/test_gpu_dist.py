"""Data parallelism on the HIP path, rehearsed with two ranks on one GPU (gloo: both processes
share cuda:0; on a node each rank owns a GPU and the collectives run on RCCL).

* ShardedOptimizer (dist.py; reduce-scatter -> RAdam on 1/G of the elements -> all-gather) against
  the replicated path (all-reduce mean -> RAdam on every element), both driving the HIP RAdam
  kernel (csrc/optim.hip) on the same per-rank gradients for 9 steps (RAdam's rectified mode
  starts at step 6, radam.py:61-79): parameters bit-identical, replicas bit-identical.
* A full graphed training iteration (GraphedTrainStep) with the sharded optimizer: replicas stay
  bit-identical and the loss is finite.
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _init(rank, world, port):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "tests", "golden")):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0")
    from indoor_nerf_amd.dist import init_process_group
    init_process_group(backend="gloo")
    torch.cuda.set_device(0)


def _params(dev, seed):
    g = torch.Generator().manual_seed(seed)
    shapes_mlp = [(64, 32), (16, 64), (64, 31), (64, 64), (3, 64)]
    mlp = [torch.nn.Parameter((torch.rand(s, generator=g) - 0.5).to(dev)) for s in shapes_mlp]
    tabs = [torch.nn.Parameter(((torch.rand(1 << 15, 2, generator=g) * 2 - 1) * 1e-4).to(dev)) for _ in range(3)]
    return mlp, tabs


def _radam_worker(rank, world, port, out):
    _init(rank, world, port)
    import indoor_nerf_amd as nerf
    dev = torch.device("cuda:0")
    runs = {}
    for sharded in (False, True):
        mlp, tabs = _params(dev, 0)
        opt = nerf.RAdam([{"params": mlp, "weight_decay": 1e-6}, {"params": tabs, "eps": 1e-15}], lr=5e-4,
                         betas=(0.9, 0.99))
        arena = nerf.GradArena(mlp + tabs, pad_to=world * 64 if sharded else 1)
        sh = nerf.ShardedOptimizer(opt, arena) if sharded else None
        for step in range(1, 10):
            g = torch.Generator().manual_seed(1000 * step + rank)
            arena.zero_()
            with torch.no_grad():
                for p in mlp + tabs:
                    p.grad.copy_((torch.randn(p.shape, generator=g) * 1e-2).to(dev))
            if sharded:
                sh.reduce_grads()
                opt.step()
                sh.gather_params()
            else:
                arena.allreduce_mean()
                opt.step()
        torch.cuda.synchronize()
        runs[sharded] = [p.detach().cpu() for p in mlp + tabs]
    torch.save({"repl": runs[False], "shard": runs[True]}, os.path.join(out, f"radam_{rank}.pt"))
    torch.distributed.destroy_process_group()


def test_sharded_radam_bit_identical(tmp_path):
    world = 2
    mp.start_processes(_radam_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    r0 = torch.load(tmp_path / "radam_0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "radam_1.pt", weights_only=True)
    for a, b, c, d in zip(r0["repl"], r0["shard"], r1["repl"], r1["shard"]):
        assert torch.equal(a, b)          # sharded == replicated, bit for bit
        assert torch.equal(a, c) and torch.equal(b, d)   # replicas agree
    # the update did something
    mlp0, tabs0 = _params("cpu", 0)
    assert not torch.equal(r0["shard"][0], mlp0[0].detach())


def _train_worker(rank, world, port, out):
    _init(rank, world, port)
    import indoor_nerf_amd as nerf
    from indoor_nerf_amd.graphs import GraphedTrainStep
    from tables import blender_bbox, synthetic_rays
    dev = torch.device("cuda:0")
    lo, hi = blender_bbox()
    args = nerf.make_args(bounding_box=(torch.from_numpy(lo), torch.from_numpy(hi)), finest_res=1024, N_samples=64,
                          N_importance=128, white_bkgd=True, perturb=1.0, tv_loss_weight=1e-6)
    torch.manual_seed(rank)         # different initial replicas: broadcast_params must align them
    nerf.manual_seed(77 + rank)
    kw, _, _, grad_vars, opt = nerf.create_nerf(args, device=dev)
    kw.update(near=2.0, far=6.0)
    params = grad_vars + list(kw["embed_fn"].parameters())
    nerf.broadcast_params(params)
    arena = nerf.GradArena(params, pad_to=world * 64)
    sh = nerf.ShardedOptimizer(opt, arena)
    ro, rd = synthetic_rays(512, seed=50 + rank)
    rays = (torch.from_numpy(ro).to(dev), torch.from_numpy(rd).to(dev))
    target = torch.rand(512, 3, device=dev, generator=torch.Generator(device=dev).manual_seed(rank))
    st = GraphedTrainStep(rays, target, kw, opt, args, grad_hook=sh.reduce_grads, post_hook=sh.gather_params,
                          loss_scale_sparsity=float(world), tv_generator=torch.Generator().manual_seed(7),
                          zero_grad=arena.zero_)
    losses = []
    for it in range(1, 7):
        loss, _ = st(it)
        losses.append(float(loss))
    torch.cuda.synchronize()
    torch.save({"params": [p.detach().cpu() for p in params], "losses": losses, "captures": st.captures},
               os.path.join(out, f"train_{rank}.pt"))
    torch.distributed.destroy_process_group()


def test_sharded_graphed_training_replicas_agree(tmp_path):
    world = 2
    mp.start_processes(_train_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    r0 = torch.load(tmp_path / "train_0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "train_1.pt", weights_only=True)
    assert r0["captures"] == 1
    assert all(torch.isfinite(torch.tensor(l)) for l in r0["losses"] + r1["losses"])
    for a, b in zip(r0["params"], r1["params"]):
        assert torch.equal(a, b)
