"""The data-parallel layer on RCCL: a world-1 ``nccl`` process group on the box's
GPU, so ``init_process_group("nccl", device_id=…)``, the job-wide loss-scale status round
(``pgd.rescale_consensus``: an int32 MAX all-reduce on the device) and the outputs'
``all_gather_into_tensor`` (``dist.gather_shards``) run through RCCL on ROCm. The shard split
itself (world 2/3, uneven, empty shards) is covered over gloo in test_dist_gloo.py; the 8-GPU
run is the driver's. Reference: single device, ``code/attack/attack_main2.py:843``."""
import socket

import pytest
import torch
import torch.distributed as dist

from gpu_helpers import seeded

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture
def nccl_world1(cuda):
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_port()}", rank=0,
                            world_size=1, device_id=cuda)
    try:
        assert dist.get_backend() == "nccl"
        yield dist.group.WORLD
    finally:
        dist.destroy_process_group()


def test_gather_shards_nccl_world1(cuda, nccl_world1):
    from gfa_amd.dist import gather_shards
    x = seeded(4, (5, 3, 8, 8)).to(cuda)
    got = gather_shards(x, 5)
    torch.cuda.synchronize()
    assert got.device == x.device and torch.equal(got, x)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
def test_attack_distributed_nccl_world1_equals_attack(cuda, nccl_world1, dtype):
    """attack_distributed over RCCL (one rank) returns exactly the single-process attack(): the
    same shard, the same random-start draw, the status round on the device, the all-gather."""
    from gfa_amd import attack, networks
    from gfa_amd.dist import attack_distributed
    net = networks.build_net(32, seed=0, dtype=dtype, device=cuda)
    x0 = seeded(1, (3, 3, 32, 32)).to(cuda)
    t = seeded(2, (3, 3, 32, 32)).to(cuda)
    got = attack_distributed(net, x0, 8 / 255, 3, target=t, random_start=True, seed=5,
                             alpha=2 / 255)
    want = attack(net, x0, 8 / 255, 3, target=t, random_start=True, seed=5, alpha=2 / 255)
    torch.cuda.synchronize()
    assert got.shape == x0.shape and torch.equal(got, want)
    assert ((got - x0).abs() <= 16 / 255 + 1e-6).all()  # ε in [0,1] units on [-1,1] images


@pytest.mark.parametrize("world,n,dtype", [(2, 5, "fp32"), (3, 2, "fp16")])
def test_attack_distributed_multirank_real_engine(cuda, tmp_path, world, n, dtype):
    """`world` ranks (processes started by torch.distributed.run, a child of this test) share the
    box's one GPU over gloo and run the REAL HIP engine: attack_distributed's contiguous shards
    (uneven; at world 3 with n = 2 one rank has an empty shard and only joins the status rounds
    and the all-gather), and bench.py's timed leg with the product networks. Every rank's
    gathered output equals the single-process attack() bit for bit (each image's arithmetic is
    independent of the other images of its launch: ordered reductions), and the bench leg's
    all-gather puts every shard in place."""
    import os
    import subprocess
    import sys
    from gfa_amd import attack, networks
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT", "MASTER_ADDR"):
        env.pop(k, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={world}", "--rdzv-backend=c10d", "--rdzv-endpoint=127.0.0.1:0",
           "--local-addr=127.0.0.1", os.path.join(root, "tests", "dist_rank_worker.py"),
           str(tmp_path), str(n), dtype]
    p = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                       timeout=240, cwd=root)
    assert p.returncode == 0, p.stderr[-4000:]
    T = {"fp32": torch.float32, "fp16": torch.float16}[dtype]
    net = networks.build_net(32, seed=0, dtype=T, device=cuda)
    x0 = seeded(1, (n, 3, 32, 32)).to(cuda)
    t = seeded(2, (n, 3, 32, 32)).to(cuda)
    want = attack(net, x0, 8 / 255, 3, target=t, random_start=True, seed=5, alpha=2 / 255).cpu()
    for r in range(world):
        res = torch.load(os.path.join(tmp_path, f"rank{r}.pt"), weights_only=True)
        nd = int((res["attack"] != want).sum())
        b = res["bench"]
        print(f"world {world} rank {r}: {nd} of {want.numel()} values differ from attack(); "
              f"bench leg gathered_ok {b['gathered_ok']} output_ok {b['output_ok']} "
              f"n_total {b['n_total']} ({b['elapsed']:.2f} s)")
        assert torch.equal(res["attack"], want)
        assert b["gathered_ok"] and b["output_ok"] and b["n_total"] == world
