"""Batch sharding across the GPUs of one node.

The eval forward is per-image independent, so a batch of B images is split
into contiguous shards, one per rank (one process per GPU), with no data-path
collective.  The only exchange is the optional final collect of the outputs
on rank 0 / all ranks: one all_gather over RCCL (xGMI) in fp16 or fp32.
"""
import torch
import torch.distributed as dist


def shard_bounds(total, world, rank):
    """Contiguous [start, stop) of rank's shard; shards differ by at most one image."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} for world size {world}")
    base, extra = divmod(total, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def local_shard(x, world=None, rank=None):
    world = dist.get_world_size() if world is None else world
    rank = dist.get_rank() if rank is None else rank
    a, b = shard_bounds(x.shape[0], world, rank)
    return x[a:b]


def gather_shards(local, total, group=None):
    """Collect every rank's shard into a [total, ...] tensor on every rank.

    Shards are padded to the largest shard size so one all_gather (RCCL
    all_gather_into_tensor on ROCm devices, list all_gather on gloo/CPU) moves
    them; the padding is dropped afterwards."""
    world = dist.get_world_size(group)
    per = -(-total // world)
    pad = per - local.shape[0]
    buf = local if pad == 0 else torch.cat([local, local.new_zeros((pad,) + tuple(local.shape[1:]))])
    buf = buf.contiguous()
    if buf.is_cuda:
        out = buf.new_empty((per * world,) + tuple(buf.shape[1:]))
        dist.all_gather_into_tensor(out, buf, group=group)
        parts = list(out.split(per))
    else:
        parts = [torch.empty_like(buf) for _ in range(world)]
        dist.all_gather(parts, buf, group=group)
    keep = []
    for r, p in enumerate(parts):
        a, b = shard_bounds(total, world, r)
        keep.append(p[: b - a])
    return torch.cat(keep)


def gather_to_rank0(local, total, group=None, dst=0):
    """Collect every rank's shard on rank `dst` only ("gather to
    rank 0 if only rank 0 writes"): one gather, so the fabric carries each
    shard once instead of to every rank as the all-gather does.  Returns the
    [total, ...] tensor on `dst`, None elsewhere.  Shards are padded to the
    largest size (dist.gather needs equal shapes); padding is dropped.

    `dst` and the shard order are GROUP ranks (shard r is group rank r's);
    dist.gather takes a global rank, so `dst` is translated for it."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if not 0 <= dst < world:
        raise ValueError(f"dst {dst} is not a rank of the group (size {world})")
    dst_global = dst if group is None else dist.get_global_rank(group, dst)
    per = -(-total // world)
    pad = per - local.shape[0]
    buf = local if pad == 0 else torch.cat([local, local.new_zeros((pad,) + tuple(local.shape[1:]))])
    buf = buf.contiguous()
    parts = [torch.empty_like(buf) for _ in range(world)] if rank == dst else None
    dist.gather(buf, parts, dst=dst_global, group=group)
    if rank != dst:
        return None
    keep = []
    for r, p in enumerate(parts):
        a, b = shard_bounds(total, world, r)
        keep.append(p[: b - a])
    return torch.cat(keep)


def sharded_forward(model, x_local, total, collect=False, collect_dtype=None):
    """Run this rank's shard; optionally all-gather the enhanced images."""
    with torch.no_grad():
        enh, refl, illu = model(x_local)
    if not collect:
        return enh, refl, illu
    src = enh if collect_dtype is None else enh.to(collect_dtype)
    return gather_shards(src, total), refl, illu


def allreduce_grads(optimizer, group=None):
    """Data-parallel training: average the gradients over the
    ranks with ONE all-reduce of the optimiser's flat gradient buffer (RCCL
    over xGMI on ROCm devices; gloo on CPU).  BatchNorm statistics stay per
    rank, as the reference has no SyncBN.  Call between the backward and the
    unscale / clip (trainers.train.train_step's grad_hook)."""
    world = dist.get_world_size(group)
    g = optimizer.flat.grad
    dist.all_reduce(g, op=dist.ReduceOp.SUM, group=group)
    g.div_(world)
