"""Benchmark: attacked images/sec, PGD-20 L∞ ε=8/255 at 256², 1/2/4/8 MI355X (BASELINE.json).

One "step" = one complete PGD-20 attack (target precompute + 20 iterations + the final RCCL
all-gather when N>1) over this rank's batch of 128 synthetic 256² image pairs (BASELINE config #4:
batch 1024 over 8 GPUs = 128 per GPU; weak scaling) through the reference's networks: the e4e
encoder (IR-SE50 Encoder4Editing), the StyleGAN2 synthesis and the VGG16 trunk, random-init.
Inputs are resident in HBM before the timed region. Rank 0 prints ONE JSON line.

    python bench.py [--gpus N --steps K --warmup W --batch B --dtype fp16|bf16|fp32
                     --encoder e4e|linear]
    torchrun --nproc-per-node N bench.py --gpus N ...
"""
import argparse
import glob
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
import gfa_import  # noqa: E402,F401
from gfa_amd import ops, pgd  # noqa: E402
from gfa_amd.dist import gather_shards  # noqa: E402
from gfa_amd.e4e import E4EEncoder  # noqa: E402
from gfa_amd.encoder import SyntheticEncoder  # noqa: E402
from gfa_amd.stylegan2 import SynthesisNet  # noqa: E402
from gfa_amd.vgg import VGGNet  # noqa: E402
from gfa_amd.weights import (make_e4e_weights, make_encoder_weights,  # noqa: E402
                             make_generator_weights, make_vgg_weights)

METRIC = "attacked images/sec, PGD-20 L∞ ε=8/255 at 256², 1/2/4/8 MI355X"  # BASELINE.json
DT = {"fp32": torch.float32, "fp16": torch.float16, "bf16": torch.bfloat16}
DT_NAME = {"fp32": "f32", "fp16": "f16", "bf16": "bf16"}
# MI355X_MICROARCH.md chip table: dense MFMA peaks (TFLOP/s)
PEAK_TFLOPS = {"fp32": 157.3, "fp16": 2500.0, "bf16": 2500.0}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=128, help="images per GPU")
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--pgd-steps", type=int, default=20)
    ap.add_argument("--dtype", default="fp16", choices=list(DT))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-steps", type=int, default=10)
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--norm", default="linf", choices=["linf", "l2_cw"],
                    help="linf = PGD L∞ (the headline); l2_cw = C&W-L2 with the VGG perceptual "
                         "objective (BASELINE config #5 at --size 1024 --dtype fp16), c = 1e-4, "
                         "lr = 0.01, --pgd-steps iterations with the reference's early stop")
    ap.add_argument("--encoder", default="e4e", choices=["e4e", "linear"],
                    help="e4e = Encoder4Editing(50,'ir_se'), the reference's net.encoder "
                         "(code/utils/model_utils.py:24; default); linear = the SURVEY.md §7 "
                         "stand-in (rounds before the e4e encoder existed)")
    return ap.parse_args()


def encoder_weights(kind, size):
    return make_e4e_weights(size, seed=1) if kind == "e4e" else make_encoder_weights(size, seed=1)


def cpu_baseline(size, pgd_steps, sample_steps, encoder):
    """The oracle (CPU restatement, fp32, all host cores) on a bounded sample: one 256² image,
    `sample_steps` PGD iterations, extrapolated to a PGD-`pgd_steps` attack."""
    from oracle import attack_ref, vgg_ref
    # the box's CPU share (OMP_NUM_THREADS is set to it there); affinity shows the whole machine
    cores = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    cores = max(1, min(cores, len(os.sched_getaffinity(0))))
    torch.set_num_threads(cores)
    gp = make_generator_weights(size, seed=0)
    ep = encoder_weights(encoder, size)
    vp = vgg_ref.load_positional(make_vgg_weights(1234))
    g = torch.Generator().manual_seed(123)
    x0 = torch.rand(1, 3, size, size, generator=g) * 2 - 1
    t = torch.rand(1, 3, size, size, generator=g) * 2 - 1
    refs = attack_ref.Refs(gp, vp, ep, x0, t, size)
    attack_ref.loss_grad(gp, vp, ep, x0, refs, size)  # warm-up
    t0 = time.perf_counter()
    adv = x0.clone()
    for _ in range(sample_steps):
        _, gr = attack_ref.loss_grad(gp, vp, ep, adv, refs, size)
        adv = attack_ref.project_step(adv, x0, gr, 2 * 8 / 255, 2 * 2 / 255)
    dt = (time.perf_counter() - t0) / sample_steps
    return {"value": 1.0 / (dt * pgd_steps), "unit": "attacked images/s", "cores": cores,
            "kind": "port",
            "sample": f"oracle fp32 CPU, 1 image @{size}², {sample_steps} PGD step(s) timed "
                      f"({dt:.2f} s/step) extrapolated to PGD-{pgd_steps}; "
                      f"torch.set_num_threads({cores})"}


def pmc_traffic(dtype, batch, size, pgd_steps, encoder="linear"):
    """HBM bytes per conv_kernel launch from the newest committed PMC profile of this exact
    workload (profiles/rNN_bench_<dtype>_b<batch>.json, written by profiles/summarize_rocprof.py
    from separate FETCH_SIZE / WRITE_SIZE rocprofv3 passes of this bench; FETCH_SIZE ×2 per the
    gfx950 correction). PMC counters cannot be read from inside the timed process, hence a file."""
    if size != 256 or pgd_steps != 20:
        return None, None
    suffix = "_e4e" if encoder == "e4e" else ""
    files = sorted(glob.glob(os.path.join(ROOT, "profiles",
                                          f"r*_bench_{dtype}_b{batch}{suffix}.json")))
    for f in reversed(files):
        with open(f) as fh:
            d = json.load(fh)
        v = d.get("conv_kernel", {}).get("hbm_bytes_per_launch")
        if v:
            return v, os.path.relpath(f, ROOT)
    return None, None


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("launch N>1 with torch.distributed.run (one process per GPU)")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    T = DT[args.dtype]
    S, B = args.size, args.batch
    gp = make_generator_weights(S, seed=0)
    ep = encoder_weights(args.encoder, S)
    vs = make_vgg_weights(1234)
    enc = (E4EEncoder(ep, S, dtype=T, device=dev) if args.encoder == "e4e"
           else SyntheticEncoder(ep, S, device=dev))
    eng = pgd.AttackEngine(enc,
                           SynthesisNet(gp, S, dtype=T, device=dev),
                           VGGNet(vs, dtype=T, device=dev))
    g = torch.Generator().manual_seed(1000 + rank)
    x0 = (torch.rand(B, 3, S, S, generator=g) * 2 - 1).to(dev)
    tgt = (torch.rand(B, 3, S, S, generator=g) * 2 - 1).to(dev)
    eps, alpha = 8 / 255, 2 / 255
    n_total = B * world

    cw_runs = []

    def one_step():
        if args.norm == "l2_cw":
            adv = eng.run_cw(x0, tgt, args.pgd_steps, c=1e-4, lr=0.01)
            cw_runs.append(eng.cw_steps_run)
        else:
            adv = eng.run(x0, tgt, args.pgd_steps, eps, alpha)
        if world > 1:
            gather_shards(adv, n_total)
        return adv

    for _ in range(args.warmup):
        one_step()
    torch.cuda.synchronize()
    prof = []
    if not args.no_roofline:
        ops.PROFILE = prof
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_ref = torch.cuda.Event(enable_timing=True)  # origin of the conv launches' event intervals
    t_ref.record()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        one_step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ops.PROFILE = None
    if world > 1:
        tt = torch.tensor([elapsed], device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = tt.item()
    ms = elapsed / args.steps * 1e3
    timed_cw = cw_runs[args.warmup:]
    iters = sum(timed_cw) / len(timed_cw) if timed_cw else args.pgd_steps
    value = n_total * args.steps / elapsed
    flops_img_step = pgd.algorithmic_flops_per_image_step(eng.G, eng.V, eng.E)
    out = {
        "metric": METRIC if (S, args.pgd_steps, args.norm) == (256, 20, "linf") else
                  (f"attacked images/sec, PGD-{args.pgd_steps} L∞ ε=8/255 at {S}², "
                   if args.norm == "linf" else
                   f"attacked images/sec, C&W-L2 (c=1e-4, lr=0.01, ≤{args.pgd_steps} iterations, "
                   f"early stop) with the VGG perceptual objective at {S}², ")
                  + f"{world} MI355X (non-headline config)",
        "value": value, "unit": "attacked images/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": ms, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": DT_NAME[args.dtype],
        "data": f"synthetic: seeded U(-1,1) image/target pairs, seeded random-init StyleGAN2 "
                f"({S}², cm=2), VGG16 trunk and "
                + ("e4e Encoder4Editing(50,'ir_se')" if args.encoder == "e4e"
                   else "linear stand-in encoder") + " (no checkpoints offline)",
        "config": {"workload": (f"PGD-{args.pgd_steps} L∞ eps=8/255 alpha=2/255" if args.norm ==
                                "linf" else f"C&W-L2 ≤{args.pgd_steps} iterations") + f" at {S}², "
                               f"{B} images/GPU"
                               + (" (BASELINE config #4 per-GPU share)" if (S, B) == (256, 128)
                                  else "") + ", "
                               f"RCCL all-gather of outputs when N>1",
                   "encoder": args.encoder, "norm": args.norm, "images_per_gpu": B, "global_batch": n_total, "size": S,
                   "pgd_steps": args.pgd_steps, "parallelism": f"dp{world}",
                   **({"cw_iterations_run": timed_cw} if timed_cw else {}),
                   "algorithmic_gflop_per_image_step": flops_img_step / 1e9,
                   "effective_tflops": flops_img_step * B * iters * world
                   / (elapsed / args.steps) / 1e12,
                   "peak_hbm_gb_per_gpu": torch.cuda.max_memory_allocated(dev) / 1e9},
    }
    if prof:
        # the e4e style heads run on side streams, so launches overlap: a launch's own duration
        # includes the time it shares the chip. The conv-busy time is the union of the launches'
        # [start, end] event intervals (all on the device clock, origin t_ref); achieved =
        # algorithmic FLOPs ÷ conv-busy time, avg_launch_us = conv-busy time per launch.
        iv = sorted((t_ref.elapsed_time(a), t_ref.elapsed_time(b)) for a, b, _ in prof)
        sum_ms = sum(e - s0 for s0, e in iv)
        tot_ms, (cs, ce) = 0.0, iv[0]
        for s0, e in iv[1:]:
            if s0 > ce:
                tot_ms += ce - cs
                cs, ce = s0, e
            else:
                ce = max(ce, e)
        tot_ms += ce - cs
        tot_fl = sum(f for _, _, f in prof)
        n = len(prof)
        ach = tot_fl / (tot_ms * 1e-3) / 1e12
        peak = PEAK_TFLOPS[args.dtype]
        traffic, src = pmc_traffic(args.dtype, B, S, args.pgd_steps, args.encoder)
        out["roofline"] = {
            "kernel": "3x3 conv: every conv API call of the step (mia::conv_halo_kernel, "
                      "mia::upconv_halo_kernel + its edge launch, mia::conv_kernel, "
                      "mia::conv_wres_kernel, mia::conv_thin_*: StyledConv fwd, up-conv, dgrads, VGG fwd/dgrad"
                      + (", e4e convs and their input gradients)" if args.encoder == "e4e"
                         else ")"),
            "bound": "mfma", "achieved": ach, "peak": peak, "unit": "TFLOP/s", "frac": ach / peak,
            "traffic": traffic, "traffic_unit": "bytes/launch", "traffic_source": src,
            "launches": n, "avg_launch_us": tot_ms / n * 1e3,
            "avg_launch_us_overlapped": sum_ms / n * 1e3,
            "algorithmic_gflop_per_launch": tot_fl / n / 1e9,
            "share_of_step_time": tot_ms / (elapsed * 1e3)}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(S, args.pgd_steps, args.cpu_sample_steps,
                                           args.encoder)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
