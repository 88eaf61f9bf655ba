"""One rank of tests/test_gpu_dist.py's multi-process runs (launched by torch.distributed.run as
a child process of the test): the REAL HIP attack engine on the box's one GPU, several ranks
sharing it over a gloo process group (RCCL needs one GPU per rank; the collectives' semantics —
shard split, status rounds, all-gather — are the backend's, the data path is the product's).
Writes this rank's results to $OUT/rank<r>.pt. Not a test module."""
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import gfa_import  # noqa: E402,F401


def main():
    out_dir, n, dtype_name = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    dtype = {"fp32": torch.float32, "fp16": torch.float16}[dtype_name]
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    try:
        torch.cuda.set_device(0)
        cuda = torch.device("cuda", 0)
        from gfa_amd import networks
        from gfa_amd.dist import attack_distributed
        from gpu_helpers import seeded
        net = networks.build_net(32, seed=0, dtype=dtype, device=cuda)
        x0 = seeded(1, (n, 3, 32, 32)).to(cuda)
        t = seeded(2, (n, 3, 32, 32)).to(cuda)
        got = attack_distributed(net, x0, 8 / 255, 3, target=t, random_start=True, seed=5,
                                 alpha=2 / 255)
        res = {"attack": got.cpu()}
        # bench.py's timed leg with the product engine (e4e + StyleGAN2 + VGG16) on this rank
        import bench
        args = bench.parse(["--steps", "1", "--warmup", "1", "--batch", "1", "--size", "256",
                            "--pgd-steps", "2", "--no-roofline", "--no-cpu-baseline",
                            "--dtype", dtype_name])
        r = bench.run_leg(args, dtype_name, 1, 1, cuda, world, rank, False)
        res["bench"] = {k: r[k] for k in ("gathered_ok", "output_ok", "n_total", "elapsed")}
        torch.save(res, os.path.join(out_dir, f"rank{rank}.pt"))
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
