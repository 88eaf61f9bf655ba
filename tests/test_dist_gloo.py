"""Multi-process (world_size 2, gloo, CPU) coverage of the data-parallel shard + all-gather path
used by bench.py and gfa_amd.dist.attack_distributed on RCCL."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import gfa_import  # noqa: F401
    from gfa_amd.dist import gather_shards, shard_bounds
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        full = torch.arange(n * 6, dtype=torch.float32).view(n, 2, 3)
        lo, hi = shard_bounds(n, world, rank)
        local = full[lo:hi] * 2 + rank * 0  # stand-in for the per-shard attack (elementwise)
        got = gather_shards(local, n)
        out_q.put((rank, torch.equal(got, full * 2)))
    finally:
        dist.destroy_process_group()


def test_gather_shards_world2_uneven():
    ctx = mp.get_context("spawn")
    for n in (5, 8):
        q = ctx.Queue()
        port = _free_port()
        procs = [ctx.Process(target=_worker, args=(r, 2, port, n, q)) for r in range(2)]
        for p in procs:
            p.start()
        res = [q.get(timeout=120) for _ in procs]
        for p in procs:
            p.join(timeout=120)
            assert p.exitcode == 0
        assert all(ok for _, ok in res), res
