"""Per-layer conv time table of one bench step (GPU, tuning aid; not part of the product path).

Usage: MIA_HEAD_STREAMS=1 python tools/layer_table.py [--batch 128] [--pgd-steps 20]
Runs the bench workload (e4e + StyleGAN2 + VGG, fp16) once untimed, then once with every conv
API call bracketed by HIP events (ops.PROFILE) and labelled (ops.PROFILE_TAGS); prints the
labels sorted by total time with calls, µs per call and algorithmic TFLOP/s."""
import argparse
import collections
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import gfa_import  # noqa: E402,F401
from gfa_amd import ops, pgd  # noqa: E402
from gfa_amd.e4e import E4EEncoder  # noqa: E402
from gfa_amd.stylegan2 import SynthesisNet  # noqa: E402
from gfa_amd.vgg import VGGNet  # noqa: E402
from gfa_amd.weights import make_generator_weights, make_vgg_weights  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--pgd-steps", type=int, default=20)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--dtype", default="fp16", choices=["fp16", "bf16", "fp32"])
    a = ap.parse_args()
    if os.environ.get("E4E_MERGE_BELOW_TILES"):  # A/B of the merged first head convs (e4e.py)
        # the threshold of the dtype being run (fp32 reads MERGE_BELOW_TILES, 2-byte types
        # MERGE_BELOW_TILES_2B); "1e9" (merge every head) parses as well as an integer
        import gfa_amd.e4e as e4e_mod
        lim = int(float(os.environ["E4E_MERGE_BELOW_TILES"]))
        setattr(e4e_mod, "MERGE_BELOW_TILES" if a.dtype == "fp32" else "MERGE_BELOW_TILES_2B",
                lim)
    dev = torch.device("cuda:0")
    T, S, B = bench.DT[a.dtype], a.size, a.batch
    enc = E4EEncoder(bench.encoder_weights("e4e", S), S, dtype=T, device=dev)
    eng = pgd.AttackEngine(enc, SynthesisNet(make_generator_weights(S, seed=0), S, dtype=T,
                                             device=dev), VGGNet(make_vgg_weights(1234), dtype=T,
                                                                 device=dev))
    g = torch.Generator().manual_seed(1000)
    x0 = (torch.rand(B, 3, S, S, generator=g) * 2 - 1).to(dev)
    tgt = (torch.rand(B, 3, S, S, generator=g) * 2 - 1).to(dev)
    eng.run(x0, tgt, a.pgd_steps, 8 / 255, 2 / 255)
    torch.cuda.synchronize()
    prof, tags = [], []
    ops.PROFILE, ops.PROFILE_TAGS = prof, tags
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    eng.run(x0, tgt, a.pgd_steps, 8 / 255, 2 / 255)
    e1.record()
    torch.cuda.synchronize()
    ops.PROFILE = ops.PROFILE_TAGS = None
    assert len(prof) == len(tags)
    agg = collections.defaultdict(lambda: [0, 0.0, 0.0])
    for (b, e, fl), t in zip(prof, tags):
        r = agg[t]
        r[0] += 1
        r[1] += b.elapsed_time(e)
        r[2] += fl
    tot = sum(r[1] for r in agg.values())
    step = e0.elapsed_time(e1)
    print(f"step {step:.1f} ms, conv calls {len(prof)}, conv time {tot:.1f} ms "
          f"({sum(r[2] for r in agg.values()) / tot / 1e9:.0f} TFLOP/s)")
    peak = 416.7 if a.dtype == "fp32" else 2500.0
    # the StyleGAN2 modulated convs' forward, FLOP-weighted: the stride-1 StyledConvs ("mod"
    # labels, the per-image weight pass included), then with the up-sampling convs' forwards
    for name, sel in (("stride-1 StyledConv", lambda t: " mod" in t),
                      ("+ up-conv forwards", lambda t: " mod" in t or "upconv_fwd" in t)):
        rows = [r for t, r in agg.items() if sel(t)]
        if rows:
            n, ms, fl = (sum(r[i] for r in rows) for i in range(3))
            print(f"modulated forward ({name}): {n} calls, {fl / 1e12:.1f} TFLOP in {ms:.1f} ms "
                  f"= {fl / (ms * 1e-3) / 1e12:.1f} TF/s = {fl / (ms * 1e-3) / 1e12 / peak:.3f} "
                  f"of {peak:.0f}")
    for t, (n, ms, fl) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"{t:48s} {n:5d} calls {ms:8.2f} ms {ms / n * 1e3:8.1f} us/call "
              f"{fl / (ms * 1e-3) / 1e12:7.1f} TF/s {100 * ms / step:5.1f}%")


if __name__ == "__main__":
    main()
