"""Benchmark: attacked images/sec, PGD-20 L∞ ε=8/255 at 256², 1/2/4/8 MI355X (BASELINE.json).

One "step" = one complete PGD-20 attack (target precompute + 20 iterations + the final RCCL
all-gather when N>1) over this rank's batch of 128 synthetic 256² image pairs (BASELINE config #4:
batch 1024 over 8 GPUs = 128 per GPU; weak scaling) through the reference's networks: the e4e
encoder (IR-SE50 Encoder4Editing), the StyleGAN2 synthesis and the VGG16 trunk, random-init.
Inputs are resident in HBM before the timed region. Rank 0 prints ONE JSON line.

    python bench.py [--gpus N --steps K --warmup W --batch B --dtype fp32|fp16|bf16
                     --encoder e4e|linear --lowp fp16|bf16|none]
    torchrun --nproc-per-node N bench.py --gpus N ...

`value` is measured at fp32, the reference's arithmetic (the reference runs its networks in
torch's default float32 on cuda:0, code/attack/interpolation.py:1095). A reduced-precision run of
the same workload (fp16 by default) is reported beside it as the labelled sub-record
`low_precision` (N=1 only); it is never `value`.
"""
import argparse
import gc
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
# MI355X_MICROARCH.md chip table: dense MFMA peaks (TFLOP/s). fp32 runs on the bf16 matrix pipe
# as exact three-way bf16 splits with six bf16 products per fp32 product (conv_common.h,
# mfma_chunk<float>): its peak is 2500 / 6 = 416.7 fp32 TFLOP/s. MIA_F32_ARITH=native (the A/B
# build on v_mfma_f32_16x16x4_f32): 157.3.
PEAK_TFLOPS = {"fp32": 2500.0 / 6, "fp32native": 157.3, "fp16": 2500.0, "bf16": 2500.0}
F32_ARITH_NOTE = {
    "bf16x6": "fp32 storage and accumulation; each fp32 operand split exactly into three bf16 "
              "terms (hi+mid+lo), six bf16 products per fp32 product on v_mfma_f32_16x16x32_bf16 "
              "(dropped terms < 2^-23|ab|; error vs fp64 = the native fp32 MFMA's, "
              "tests/test_gpu_kernels.py::test_fp32_arithmetic_is_fp32_accurate)",
    "native": "fp32 on v_mfma_f32_16x16x4_f32"}


def arith_key(dtype):
    """Profile / peak key of a compute dtype: fp32 is split by its arithmetic."""
    from gfa_amd import _lib
    return "fp32native" if dtype == "fp32" and _lib.F32_ARITH == "native" else dtype


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks, one per GPU (default: WORLD_SIZE under a launcher, else 1)")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=128, help="images per GPU")
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--pgd-steps", type=int, default=20)
    ap.add_argument("--dtype", default="fp32", choices=list(DT),
                    help="compute dtype of `value` (default fp32 = the reference's precision)")
    ap.add_argument("--lowp", default="fp16", choices=["fp16", "bf16", "none"],
                    help="dtype of the labelled reduced-precision sub-record (N=1 only)")
    ap.add_argument("--lowp-steps", type=int, default=2)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-pgd-steps", type=int, default=None,
                    help="PGD iterations of the wall-clocked CPU attack (default: --pgd-steps)")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--norm", default="linf", choices=["linf", "l2_cw"],
                    help="linf = PGD L∞ (the headline); l2_cw = C&W-L2 with the VGG perceptual "
                         "objective (BASELINE config #5 at --size 1024 --dtype fp16), c = 1e-4, "
                         "lr = 0.01, --pgd-steps iterations with the reference's early stop")
    ap.add_argument("--cw-fixed", action="store_true",
                    help="l2_cw: run all --pgd-steps iterations (no early stop) — a labelled "
                         "fixed-work timing beside the reference-semantics line")
    ap.add_argument("--encoder", default="e4e", choices=["e4e", "linear"],
                    help="e4e = Encoder4Editing(50,'ir_se'), the reference's net.encoder "
                         "(code/utils/model_utils.py:24; default); linear = the SURVEY.md §7 "
                         "stand-in (rounds before the e4e encoder existed)")
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                    help="cpu: gloo process group on host tensors — only with --engine-factory "
                         "(tests of the multi-rank leg); the product bench runs on cuda")
    ap.add_argument("--engine-factory", default=None, help=argparse.SUPPRESS)
    return ap.parse_args(argv)


def _die_with_parent():
    """preexec_fn of the launcher child: PR_SET_PDEATHSIG(SIGTERM), so a SIGKILL of this process
    (a `timeout -k` escalation skips the signal forwarding below) still ends the launcher, which
    then terminates its ranks. Runs between fork and exec in the child; no GPU is involved."""
    import ctypes
    import signal
    libc = ctypes.CDLL(None, use_errno=True)
    PR_SET_PDEATHSIG = 1
    libc.prctl(PR_SET_PDEATHSIG, int(signal.SIGTERM), 0, 0, 0)


def spawn_workers(n, argv):
    """`--gpus N` without a launcher: start the N one-process-per-GPU ranks as ONE child
    (`python -m torch.distributed.run --nproc-per-node N … bench.py <same args>`) and return its
    exit code. This process touches no GPU (no HIP call before or after), so nothing is exec'd
    from an initialised process; the ranks' rank 0 prints the JSON line on the shared stdout.
    The rendezvous store binds its own free port (c10d endpoint 127.0.0.1:0: no probe-then-bind
    race), and SIGTERM / SIGINT to this process are forwarded to the child's process group, so a
    `timeout` around the bench also ends the launcher and its ranks; a SIGKILL of this process
    reaches the launcher as SIGTERM through its parent-death signal (_die_with_parent)."""
    import signal
    import subprocess
    import uuid
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={n}", "--rdzv-backend=c10d", "--rdzv-endpoint=127.0.0.1:0",
           f"--rdzv-id={uuid.uuid4().hex}", "--local-addr=127.0.0.1",
           os.path.abspath(__file__), *argv]
    log(f"spawning {n} ranks: {' '.join(cmd[1:5])} …")
    child = subprocess.Popen(cmd, env=dict(os.environ, MASTER_ADDR="127.0.0.1"),
                             start_new_session=True, preexec_fn=_die_with_parent)

    def forward(signum, _frame):
        try:
            os.killpg(child.pid, signum)
        except ProcessLookupError:
            pass

    old = {sig: signal.signal(sig, forward) for sig in (signal.SIGTERM, signal.SIGINT)}
    try:
        return child.wait()
    finally:
        for sig, h in old.items():
            signal.signal(sig, h)
        if child.poll() is None:  # the parent is leaving early (an exception): end the ranks
            forward(signal.SIGTERM, None)
            try:
                child.wait(timeout=30)
            except subprocess.TimeoutExpired:
                forward(signal.SIGKILL, None)


def encoder_weights(kind, size):
    return make_e4e_weights(size, seed=1) if kind == "e4e" else make_encoder_weights(size, seed=1)


def log(msg):
    """Liveness / progress line on stderr (stdout carries only the JSON line)."""
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def _progress(tag):
    t0 = time.perf_counter()
    n = [0]

    def cb(_):
        n[0] += 1
        log(f"{tag}: iteration {n[0]} done, {time.perf_counter() - t0:.1f} s")
    return cb


def cpu_baseline(size, pgd_steps, encoder, batch8=True):
    """The oracle (CPU restatement, fp32, all host cores) on a bounded sample of the same
    workload, wall-clocked end to end (target precompute + every iteration; SURVEY.md §8(d): B=1
    and B=min(N,8)): ONE complete PGD-`pgd_steps` attack of one 256² image, and — `batch8` — one
    of a batch of 8 (≈ 1–2 min on the box's 16 cores)."""
    from oracle import attack_ref, vgg_ref
    # the box's CPU share (OMP_NUM_THREADS is set to it there); affinity shows the whole machine
    cores = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    cores = max(1, min(cores, len(os.sched_getaffinity(0))))
    torch.set_num_threads(cores)
    gp = make_generator_weights(size, seed=0)
    ep = encoder_weights(encoder, size)
    vp = vgg_ref.load_positional(make_vgg_weights(1234))
    g = torch.Generator().manual_seed(123)
    x0 = torch.rand(8, 3, size, size, generator=g) * 2 - 1
    t = torch.rand(8, 3, size, size, generator=g) * 2 - 1
    eps, alpha = 8 / 255, 2 / 255
    attack_ref.pgd(gp, vp, ep, x0[:1], t[:1], size, eps, alpha, 1)  # warm-up (allocator, threads)
    t0 = time.perf_counter()
    adv = attack_ref.pgd(gp, vp, ep, x0[:1], t[:1], size, eps, alpha, pgd_steps,
                         progress=_progress("cpu baseline B=1"))
    dt = time.perf_counter() - t0
    assert adv.shape == x0[:1].shape
    out = {"value": 1.0 / dt, "unit": "attacked images/s", "cores": cores, "kind": "port",
           "sample": f"oracle fp32 CPU: one complete PGD-{pgd_steps} attack of 1 image @{size}² "
                     f"({encoder} encoder), wall clock {dt:.1f} s incl. the target precompute; "
                     f"torch.set_num_threads({cores})"}
    if batch8:
        t0 = time.perf_counter()
        adv = attack_ref.pgd(gp, vp, ep, x0, t, size, eps, alpha, pgd_steps,
                             progress=_progress("cpu baseline B=8"))
        dt8 = time.perf_counter() - t0
        assert adv.shape == x0.shape
        out["batch8"] = {"value": 8.0 / dt8, "unit": "attacked images/s", "cores": cores,
                         "sample": f"the same, one complete PGD-{pgd_steps} attack of a batch of "
                                   f"8 images (B = min(N, 8), SURVEY.md §8(d)), wall clock "
                                   f"{dt8:.1f} s"}
    return out


def pmc_profile(dtype, batch, size, pgd_steps, encoder="linear"):
    """The newest committed PMC profile of this exact workload
    (profiles/rNN_bench_<dtype>_b<batch>[_e4e].json, written by profiles/summarize_rocprof.py from
    separate FETCH_SIZE / WRITE_SIZE / MFMA-busy rocprofv3 passes of this bench; FETCH_SIZE ×2 per
    the gfx950 correction). PMC counters cannot be read from inside the timed process."""
    if size != 256 or pgd_steps != 20:
        return None, None
    suffix = "_e4e" if encoder == "e4e" else ""
    files = sorted(glob.glob(os.path.join(ROOT, "profiles",
                                          f"r*_bench_{dtype}_b{batch}{suffix}.json")))
    for f in reversed(files):
        with open(f) as fh:
            d = json.load(fh)
        if d.get("conv_kernel", {}).get("hbm_bytes_per_launch"):
            return d["conv_kernel"], os.path.relpath(f, ROOT)
    return None, None


def union_ms(iv):
    """Total length of the union of [start, end] intervals (ms)."""
    iv = sorted(iv)
    tot, (cs, ce) = 0.0, iv[0]
    for s0, e in iv[1:]:
        if s0 > ce:
            tot += ce - cs
            cs, ce = s0, e
        else:
            ce = max(ce, e)
    return tot + ce - cs


EPS, ALPHA = 8 / 255, 2 / 255  # α = 2/255 (recorded in config)


def build_engine(args, dtype, dev):
    """The bench's networks at `dtype` (seeded random init)."""
    T = DT[dtype]
    S = args.size
    gp = make_generator_weights(S, seed=0)
    ep = encoder_weights(args.encoder, S)
    vs = make_vgg_weights(1234)
    enc = (E4EEncoder(ep, S, dtype=T, device=dev) if args.encoder == "e4e"
           else SyntheticEncoder(ep, S, device=dev))
    return pgd.AttackEngine(enc, SynthesisNet(gp, S, dtype=T, device=dev),
                            VGGNet(vs, dtype=T, device=dev))


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def run_leg(args, dtype, steps, warmup, dev, world, rank, roofline, make_engine=build_engine):
    """Build the networks at `dtype`, run `warmup` untimed and `steps` timed complete attacks
    (barrier + synchronize on both sides, max over ranks), each ending in the all-gather of the
    shards when world > 1. Returns the measurements. `make_engine` (tests: a CPU stub under
    gloo) builds the engine."""
    S, B = args.size, args.batch
    eng = make_engine(args, dtype, dev)
    g = torch.Generator().manual_seed(1000 + rank)
    x0 = (torch.rand(B, 3, S, S, generator=g) * 2 - 1).to(dev)
    tgt = (torch.rand(B, 3, S, S, generator=g) * 2 - 1).to(dev)
    eps, alpha = EPS, ALPHA
    n_total = B * world
    cw_runs = []
    gathered = []

    def one_step():
        # world > 1: the fp16 loss-scale decision is taken job-wide (pgd.rescale_consensus), as
        # in dist.attack_distributed, so no rank is left alone in the all-gather
        grp = dist.group.WORLD if world > 1 else None
        if args.norm == "l2_cw":
            adv = eng.run_cw(x0, tgt, args.pgd_steps, c=1e-4, lr=0.01,
                             early_stop=not args.cw_fixed, group=grp)
            cw_runs.append(eng.cw_steps_run)
        else:
            adv = eng.run(x0, tgt, args.pgd_steps, eps, alpha, group=grp)
        if world > 1:
            # gloo (the CPU tests, and several ranks sharing one GPU) gathers host tensors
            gloo = dist.get_backend() == "gloo"
            gathered[:] = [gather_shards(adv.cpu() if gloo else adv, n_total)]
        return adv

    cuda = dev.type == "cuda"
    if cuda:
        torch.cuda.reset_peak_memory_stats(dev)
    for _ in range(warmup):
        one_step()
    _sync(dev)
    log(f"{dtype}: {warmup} warm-up step(s) done")
    prof = []
    if roofline and cuda:
        ops.PROFILE = prof
    if world > 1:
        dist.barrier()
    _sync(dev)
    if cuda:
        t_ref = torch.cuda.Event(enable_timing=True)  # origin of the conv launches' intervals
        t_ref.record()
    t0 = time.perf_counter()
    for _ in range(steps):
        adv = one_step()
    _sync(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    log(f"{dtype}: {steps} timed step(s), {elapsed:.2f} s")
    ops.PROFILE = None
    if world > 1:
        tt = torch.tensor([elapsed], device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = tt.item()
    # sanity of the output the timed region produced: finite, inside the ε-ball and [-1, 1]
    ok = bool(torch.isfinite(adv).all()) and float(adv.abs().max()) <= 1.0
    if args.norm == "linf":
        ok = ok and float((adv - x0).abs().max()) <= 2 * eps + 1e-6
    timed_cw = cw_runs[warmup:]
    r = {"elapsed": elapsed, "n_total": n_total, "timed_cw": timed_cw,
         "iters": sum(timed_cw) / len(timed_cw) if timed_cw else args.pgd_steps,
         "flops_img_step": pgd.algorithmic_flops_per_image_step(eng.G, eng.V, eng.E),
         "peak_hbm_gb": torch.cuda.max_memory_allocated(dev) / 1e9 if cuda else 0.0,
         "output_ok": ok}
    if gathered:  # the all-gathered job output: n_total images, this rank's shard in place
        ga = gathered[0]
        r["gathered_ok"] = (tuple(ga.shape) == (n_total,) + tuple(adv.shape[1:])
                            and torch.equal(ga[rank * B:(rank + 1) * B], adv.to(ga.device)))
    if prof:
        # The conv-busy time is the union of the conv API calls' [start, end] event intervals
        # (device clock, origin t_ref; one stream, so no overlap); achieved = algorithmic FLOPs ÷
        # conv-busy time, avg_launch_us = conv-busy time per call. profiles/summarize_rocprof.py
        # --bench-line reproduces it from the rocprofv3 trace of the same command.
        iv = [(t_ref.elapsed_time(a), t_ref.elapsed_time(b)) for a, b, _ in prof]
        r["conv_busy_ms"] = union_ms(iv)
        r["conv_sum_ms"] = sum(e - s0 for s0, e in iv)
        r["conv_flops"] = sum(f for _, _, f in prof)
        r["conv_launches"] = len(prof)
    del eng, x0, tgt
    return r


def roofline_record(args, dtype, r):
    tot_ms, n = r["conv_busy_ms"], r["conv_launches"]
    ach = r["conv_flops"] / (tot_ms * 1e-3) / 1e12
    key = arith_key(dtype)
    peak = PEAK_TFLOPS[key]
    pmc, src = pmc_profile(key, args.batch, args.size, args.pgd_steps, args.encoder)
    rec = {"kernel": "3x3 conv: every conv API call of the step (mia::conv_halo_kernel, "
                     "mia::upconv_halo_kernel + its edge launch, mia::conv_kernel, "
                     "mia::conv_wres_kernel, mia::conv_wres128_kernel, mia::conv_thin_*: StyledConv fwd, up-conv, dgrads, "
                     "VGG fwd/dgrad" + (", e4e convs and their input gradients)"
                                        if args.encoder == "e4e" else ")"),
           "bound": "mfma", "achieved": ach, "peak": peak, "unit": "TFLOP/s", "frac": ach / peak,
           "traffic": pmc.get("hbm_bytes_per_launch") if pmc else None,
           "traffic_unit": "bytes/launch", "traffic_source": src,
           "launches": n, "avg_launch_us": tot_ms / n * 1e3,
           "avg_launch_us_overlapped": r["conv_sum_ms"] / n * 1e3,
           "algorithmic_gflop_per_launch": r["conv_flops"] / n / 1e9,
           "share_of_step_time": tot_ms / (r["elapsed"] * 1e3)}
    if pmc and pmc.get("mfma_busy_frac") is not None:
        rec["mfma_busy_frac_pmc"] = pmc["mfma_busy_frac"]
    if dtype == "fp32":
        from gfa_amd import _lib
        rec["arithmetic"] = F32_ARITH_NOTE[_lib.F32_ARITH]
        rec["peak_note"] = ("2500 TFLOP/s dense bf16 / 6 products" if key == "fp32"
                            else "v_mfma_f32_16x16x4_f32")
    return rec


def headline_record(args, r, world, dist_world):
    """The JSON line's headline fields from run_leg's measurements (`value` = every rank's images
    ÷ the max-over-ranks time)."""
    S, B = args.size, args.batch
    elapsed, n_total = r["elapsed"], r["n_total"]
    ms = elapsed / args.steps * 1e3
    value = n_total * args.steps / elapsed
    flops_img_step = r["flops_img_step"]
    timed_cw = r["timed_cw"]
    out = {
        "metric": METRIC if (S, args.pgd_steps, args.norm) == (256, 20, "linf") else
                  (f"attacked images/sec, PGD-{args.pgd_steps} L∞ ε=8/255 at {S}², "
                   if args.norm == "linf" else
                   f"attacked images/sec, C&W-L2 (c=1e-4, lr=0.01, "
                   + ("" if args.cw_fixed else "≤") + f"{args.pgd_steps} iterations"
                   + (", no early stop" if args.cw_fixed else ", early stop")
                   + f") with the VGG perceptual objective at {S}², ")
                  + f"{world} MI355X (non-headline config)",
        "value": value, "unit": "attacked images/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": ms, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": DT_NAME[args.dtype],
        "data": f"synthetic: seeded U(-1,1) image/target pairs, seeded random-init StyleGAN2 "
                f"({S}², cm=2), VGG16 trunk and "
                + ("e4e Encoder4Editing(50,'ir_se')" if args.encoder == "e4e"
                   else "linear stand-in encoder") + " (no checkpoints offline)",
        "config": {"workload": (f"PGD-{args.pgd_steps} L∞ eps=8/255 alpha=2/255" if args.norm ==
                                "linf" else f"C&W-L2 "
                                + ("" if args.cw_fixed else "≤") + f"{args.pgd_steps} iterations")
                               + f" at {S}², {B} images/GPU"
                               + (" (BASELINE config #4 per-GPU share)" if (S, B) == (256, 128)
                                  else "") + ", "
                               f"RCCL all-gather of outputs when N>1",
                   "encoder": args.encoder, "norm": args.norm, "images_per_gpu": B,
                   "global_batch": n_total, "size": S,
                   "pgd_steps": args.pgd_steps, "eps": EPS,
                   **({"alpha": ALPHA} if args.norm == "linf" else {}),
                   "parallelism": f"dp{world}",
                   "dist_world_size": dist_world,
                   **({"cw_iterations_run": timed_cw} if timed_cw else {}),
                   "algorithmic_gflop_per_image_step": flops_img_step / 1e9,
                   "effective_tflops": flops_img_step * B * r["iters"] * world
                   / (elapsed / args.steps) / 1e12,
                   "peak_hbm_gb_per_gpu": r["peak_hbm_gb"],
                   "output_in_eps_ball_and_finite": r["output_ok"],
                   **({"gathered_output_ok": r["gathered_ok"]} if "gathered_ok" in r else {}),
                   **({"fp32_arithmetic": arith_key("fp32")} if args.dtype == "fp32" else {})},
    }
    return out


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and (args.gpus or 1) > 1:
        # `python bench.py --gpus N` (no launcher): this process becomes the launcher
        sys.exit(spawn_workers(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus is None:  # under an external launcher without --gpus: one rank per GPU
        args.gpus = world
    elif world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world} (one process per GPU)")
    make_engine = build_engine
    if args.engine_factory:
        import importlib
        mod, fn = args.engine_factory.split(":")
        make_engine = getattr(importlib.import_module(mod), fn)
    elif args.device != "cuda":
        raise SystemExit("--device cpu needs --engine-factory: the attack engine is HIP-only")
    if args.device == "cuda":
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    else:
        dev = torch.device("cpu")
    dist_world = 1
    if world > 1:
        if dev.type == "cuda":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
        dist_world = dist.get_world_size()
    S = args.size
    r = run_leg(args, args.dtype, args.steps, args.warmup, dev, world, rank,
                not args.no_roofline, make_engine=make_engine)
    out = headline_record(args, r, world, dist_world)
    if "conv_busy_ms" in r:
        out["roofline"] = roofline_record(args, args.dtype, r)
    if world == 1 and args.lowp != "none" and args.lowp != args.dtype:
        gc.collect()
        if dev.type == "cuda":
            torch.cuda.empty_cache()
        lw = max(1, min(args.warmup, 1))
        rl = run_leg(args, args.lowp, args.lowp_steps, lw, dev, world, rank,
                     not args.no_roofline, make_engine=make_engine)
        sub = {"note": "reduced-precision run of the same workload; NOT the headline value",
               "dtype": DT_NAME[args.lowp], "value": rl["n_total"] * args.lowp_steps
               / rl["elapsed"], "unit": "attacked images/s", "steps": args.lowp_steps,
               "warmup": lw, "ms_per_step": rl["elapsed"] / args.lowp_steps * 1e3,
               "output_in_eps_ball_and_finite": rl["output_ok"]}
        if "conv_busy_ms" in rl:
            sub["roofline"] = roofline_record(args, args.lowp, rl)
        out["low_precision"] = sub
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(S, args.cpu_pgd_steps or args.pgd_steps, args.encoder)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
