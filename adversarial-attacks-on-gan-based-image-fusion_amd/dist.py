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


def attack_distributed(net, imgs, eps, steps, *, target, group=None, random_start=False, seed=0,
                       **kw):
    """Every rank passes the full batch (or at least its shape-compatible copy); each attacks its
    contiguous shard on its own GPU and all ranks return the full adversarial batch.

    * A rank whose shard is empty (world > n) runs no attack and contributes only the zero padding
      of the all-gather (every rank must still enter the collective).
    * The random-start noise is drawn ONCE for the full batch from ``seed`` (the same host draw as
      a single-GPU ``attack(..., random_start=True, seed=seed)``) and sliced per shard, so the
      output does not depend on the world size.
    * fp16 loss-scale overflows are decided job-wide (``pgd.rescale_consensus``, one int32 MAX
      all-reduce per attack run): every shard re-runs at the same λ, and a fatal overflow raises
      FloatingPointError on EVERY rank (an empty-shard rank included) before the all-gather, so
      no rank is left blocked in the collective."""
    from . import pgd
    group = group if group is not None else dist.group.WORLD
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    n = imgs.shape[0]
    lo, hi = shard_bounds(n, world, rank)
    gather_dev = torch.device("cpu") if dist.get_backend(group) == "gloo" else net.decoder.device
    if hi == lo:
        pgd.idle_rank_consensus(group)
        local = torch.zeros((0,) + tuple(imgs.shape[1:]), dtype=torch.float32, device=gather_dev)
        return gather_shards(local, n, group).to(imgs.device)
    tgt = target if target.shape[0] == 1 else target[lo:hi]
    noise = None
    if random_start:
        noise = pgd.make_start_noise(tuple(imgs.shape), seed)[lo:hi]
    local = pgd.attack(net, imgs[lo:hi], eps, steps, target=tgt, random_start=random_start,
                       seed=seed, start_noise=noise, group=group, **kw)
    return gather_shards(local.to(gather_dev, torch.float32), n, group).to(imgs.device)
