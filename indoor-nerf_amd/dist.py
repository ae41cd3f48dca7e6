"""Data parallelism for the training step: one process per GPU, rays sharded, parameters replicated,
gradients reduced with ONE all-reduce per step (RCCL over xGMI via torch.distributed 'nccl';
'gloo' on CPU for tests).

The reference has no distributed code; this is the build's DP layer (§8(e)).
All parameter gradients live in one flat GradArena buffer (p.grad are views into it), so the
fused backward kernels accumulate straight into the buffer that is all-reduced, zeroing is one
memset, and the collective is a single 67 MB bucket (16 x 2^19 x 2 table entries + 2 x 9,344
MLP weights) — large enough to run at per-link xGMI bandwidth with RCCL's multi-channel rings.
"""
import os

import torch
import torch.distributed as dist


def env_rank_world():
    return int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)), int(os.environ.get("LOCAL_RANK", 0))


def init_process_group(backend=None):
    """Init from torchrun's env (RANK/WORLD_SIZE/MASTER_*); no-op for a single process."""
    rank, world, local = env_rank_world()
    if world == 1 or (dist.is_available() and dist.is_initialized()):
        return rank, world, local
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29517")
    if backend is None:
        # NERF_DIST_BACKEND=gloo: rehearse the multi-rank path on one GPU (ranks share cuda:0)
        backend = os.environ.get("NERF_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
    if backend == "nccl":
        torch.cuda.set_device(local)
    dist.init_process_group(backend=backend, rank=rank, world_size=world)
    return rank, world, local


def shard(t, rank, world, dim=0):
    """Contiguous equal shard `rank` of `world` along dim (strong scaling of one global batch)."""
    n = t.shape[dim]
    if n % world:
        raise ValueError(f"shard: size {n} is not divisible by world size {world}")
    step = n // world
    return t.narrow(dim, rank * step, step)


class GradArena:
    """One flat fp32 buffer holding the .grad of every parameter (views), in parameter order."""

    def __init__(self, params):
        # quantizer scalars (soft_bits, range_scale, v_max) never receive a gradient in the
        # reference (their uses are detached): they keep grad None, so the optimizer skips them
        self.params = [p for p in params if p.requires_grad and not getattr(p, "_nerf_no_grad", False)]
        total = sum(p.numel() for p in self.params)
        dev = self.params[0].device
        self.flat = torch.zeros(total, device=dev, dtype=torch.float32)
        self.views = []
        off = 0
        for p in self.params:
            v = self.flat[off:off + p.numel()].view_as(p)
            self.views.append(v)
            off += p.numel()
        self.attach()

    def attach(self):
        for p, v in zip(self.params, self.views):
            p.grad = v

    def zero_(self):
        self.flat.zero_()
        self.attach()

    def allreduce_mean(self, group=None):
        world = dist.get_world_size(group) if dist.is_initialized() else 1
        if world == 1:
            return
        dist.all_reduce(self.flat, op=dist.ReduceOp.SUM, group=group)
        self.flat.mul_(1.0 / world)


def broadcast_params(params, src=0):
    """Make every rank start from rank `src`'s parameters."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return
    for p in params:
        dist.broadcast(p.data, src=src)
