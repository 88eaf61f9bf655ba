"""Multi-process (world_size 2, gloo, CPU) coverage of the data-parallel shard + all-gather path
used by bench.py and gfa_amd.dist.attack_distributed on RCCL."""
import os
import socket

import torch
import torch.distributed as dist
import pytest
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


def _fake_attack(net, imgs, eps, steps, *, target, random_start=False, seed=0, start_noise=None,
                 **kw):
    """CPU elementwise stand-in for pgd.attack: depends on the image, its own target row and the
    random-start noise, so shard order, target slicing and noise slicing are all visible."""
    assert imgs.shape[0] >= 1, "attack() must not run on an empty shard"
    from gfa_amd import pgd
    pgd.rescale_consensus(pgd.RUN_OK, kw.get("group"))  # the engine's one status round per run
    out = imgs * 0.5 + target.expand_as(imgs) * 0.25
    if random_start:
        assert start_noise is not None and start_noise.shape == imgs.shape
        out = out + 1e-3 * start_noise
    return out + steps * eps


class _FakeEngine:
    """The loss-scale state of AttackEngine around its real _with_rescale: overflows on the
    listed ranks for the first `runs` attack runs (dtype picks rescalable fp16 vs fatal fp32)."""

    def __init__(self, rank, bad_ranks, runs, dtype):
        from gfa_amd import pgd
        self.rank, self.bad, self.runs, self.dtype = rank, bad_ranks, runs, dtype
        self.loss_scale = pgd.DEFAULT_LOSS_SCALE[dtype]
        self.rescales, self.n_runs = 0, 0

    def set_loss_scale(self, lam):
        self.loss_scale = lam

    def overflowed(self):
        return [0] if self.rank in self.bad and self.n_runs <= self.runs else []


def _overflow_worker(rank, world, port, n, bad_ranks, runs, dtype, out_q):
    """attack_distributed with a stand-in attack that runs AttackEngine._with_rescale on a fake
    engine: reports (rank, outcome, λ, rescales, re-runs)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import types

    import gfa_import  # noqa: F401
    from gfa_amd import dist as gdist
    from gfa_amd import pgd
    state = {}

    def fake(net, imgs, eps, steps, *, target, group=None, **kw):
        eng = _FakeEngine(rank, bad_ranks, runs, dtype)
        state["eng"] = eng

        def once():
            eng.n_runs += 1
            return imgs * 0.5
        return pgd.AttackEngine._with_rescale(eng, once, group)

    pgd.attack = fake
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        imgs = torch.rand(n, 3, 4, 4, generator=torch.Generator().manual_seed(3))
        net = types.SimpleNamespace(decoder=types.SimpleNamespace(device=torch.device("cpu")))
        try:
            got = gdist.attack_distributed(net, imgs, 8 / 255, 3, target=imgs)
            outcome = "ok" if torch.equal(got, imgs * 0.5) else "wrong"
        except FloatingPointError:
            outcome = "raised"
        eng = state.get("eng")
        out_q.put((rank, outcome, eng.loss_scale if eng else None,
                   eng.rescales if eng else None, eng.n_runs if eng else 0))
    finally:
        dist.destroy_process_group()


def _run_overflow(world, n, bad_ranks, runs, dtype):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_overflow_worker,
                         args=(r, world, port, n, bad_ranks, runs, dtype, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    return res


def test_fp16_rescale_is_decided_job_wide():
    """An fp16 overflow on ONE rank's shard re-runs EVERY shard at the lowered λ (world 3, the
    third rank with an empty shard takes part in the status rounds): all ranks finish with the
    same λ = 2^8 / 16 and two runs; the gathered output is complete."""
    from gfa_amd import pgd
    res = _run_overflow(3, 2, bad_ranks=(1,), runs=1, dtype=torch.float16)
    lam = pgd.DEFAULT_LOSS_SCALE[torch.float16] / pgd.RESCALE
    for rank, outcome, scale, rescales, n_runs in res:
        assert outcome == "ok", res
        if rank < 2:  # ranks 0, 1 attack; rank 2's shard is empty
            assert (scale, rescales, n_runs) == (lam, 1, 2), res


def test_fatal_overflow_raises_on_every_rank():
    """A non-finite fp32 gradient on one rank raises FloatingPointError on EVERY rank (the
    empty-shard rank too) instead of leaving the others blocked in the all-gather."""
    res = _run_overflow(3, 2, bad_ranks=(0,), runs=99, dtype=torch.float32)
    assert [o for _, o, *_ in res] == ["raised"] * 3, res


def _attack_worker(rank, world, port, n, tgt1, rs, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import types

    import gfa_import  # noqa: F401
    from gfa_amd import dist as gdist
    from gfa_amd import pgd
    pgd.attack = _fake_attack  # the distributed wrapper looks it up at call time
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = torch.Generator().manual_seed(3)
        imgs = torch.rand(n, 3, 4, 4, generator=g) * 2 - 1
        target = torch.rand(1 if tgt1 else n, 3, 4, 4, generator=g) * 2 - 1
        net = types.SimpleNamespace(decoder=types.SimpleNamespace(device=torch.device("cpu")))
        got = gdist.attack_distributed(net, imgs, 8 / 255, 3, target=target, random_start=rs,
                                       seed=11)
        noise = pgd.make_start_noise(tuple(imgs.shape), 11) if rs else None
        want = _fake_attack(net, imgs, 8 / 255, 3, target=target, random_start=rs,
                            start_noise=noise)
        out_q.put((rank, torch.equal(got, want)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n,tgt1,rs", [(2, 5, False, True), (3, 7, True, False),
                                             (3, 8, False, True), (3, 2, False, True)])
def test_attack_distributed_matches_single_process(world, n, tgt1, rs):
    """attack_distributed over gloo (world 2 and 3, uneven n, world > n with an empty shard,
    per-image or broadcast target, random start) returns on every rank exactly the single-process
    result: shard order, target slicing, the world-size-independent noise draw and the trimmed
    all-gather."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_attack_worker, args=(r, world, port, n, tgt1, rs, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert all(ok for _, ok in res), res
