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
