"""Data-parallel attack over the GPUs of one node.

Images are independent, so the batch is split into contiguous shards, one per rank (one process
per GPU, ``torch.distributed`` with the ``nccl`` backend = RCCL over xGMI). Every rank runs the
whole PGD loop on its shard with no collective in the data path; the only exchange is ONE
``all_gather_into_tensor`` of the final adversarial images (shards padded to equal size).
The reference itself is single-GPU (``device = "cuda:0"``, attack_main2.py:843).
"""
import torch
import torch.distributed as dist


def shard_bounds(n, world, rank):
    """Contiguous, balanced split of n items: the first n % world ranks take one extra."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    q, r = divmod(n, world)
    lo = rank * q + min(rank, r)
    hi = lo + q + (1 if rank < r else 0)
    return lo, hi


def gather_shards(local, n_total, group=None):
    """All-gather equal-padded shards and trim back to the first n_total rows (rank order)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    per = -(-n_total // world)
    lo, hi = shard_bounds(n_total, world, rank)
    if local.shape[0] != hi - lo:
        raise ValueError("local shard size does not match shard_bounds")
    send = local.new_zeros((per,) + tuple(local.shape[1:]))
    send[: hi - lo] = local
    out = local.new_empty((per * world,) + tuple(local.shape[1:]))
    dist.all_gather_into_tensor(out, send.contiguous(), group=group)
    pieces = []
    for r in range(world):
        a, b = shard_bounds(n_total, world, r)
        pieces.append(out[r * per: r * per + (b - a)])
    return torch.cat(pieces, 0)


def attack_distributed(net, imgs, eps, steps, *, target, group=None, **kw):
    """Every rank passes the full batch (or at least its shape-compatible copy); each attacks its
    contiguous shard on its own GPU and all ranks return the full adversarial batch."""
    from .pgd import attack
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    n = imgs.shape[0]
    lo, hi = shard_bounds(n, world, rank)
    tgt = target if target.shape[0] == 1 else target[lo:hi]
    dev = net.decoder.device
    local = attack(net, imgs[lo:hi], eps, steps, target=tgt, **kw).to(dev)
    if dist.get_backend(group) == "gloo":
        local = local.cpu()
    return gather_shards(local, n, group).to(imgs.device)
