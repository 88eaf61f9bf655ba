"""Phase breakdown of the fp32 x6 halo kernel inside the bench workload (diagnostic; GPU).

Loads the diagnostic build libmiattack_stamps.so (csrc/Makefile `stamps`: wave 0 of every block
of conv_halo_x6_kernel adds s_memtime deltas of its prologue, in-loop splits and epilogue to a
device array), runs one warm-up PGD attack and one measured attack of the bench workload (fp32,
e4e + StyleGAN2 + VGG16) and prints, per kernel variant, the cycles per block split into phases,
the MFMA-only lower bound of the main loop (16 cycles per v_mfma_f32_16x16x32_bf16, two waves per
SIMD) and the in-kernel clock (s_memtime / s_memrealtime × 100 MHz).

Usage: python tools/probe/x6_stamps.py [--batch 128] [--pgd-steps 20]
"""
import argparse
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import gfa_import  # noqa: E402,F401
from gfa_amd import _lib, pgd  # noqa: E402

_lib.LIB_PATH = os.path.join(os.path.dirname(_lib.LIB_PATH), "libmiattack_stamps.so")
from gfa_amd.e4e import E4EEncoder  # noqa: E402
from gfa_amd.stylegan2 import SynthesisNet  # noqa: E402
from gfa_amd.vgg import VGGNet  # noqa: E402
from gfa_amd.weights import make_generator_weights, make_vgg_weights  # noqa: E402

# MFMA cycles per K-step per SIMD: 2 halves × FM·FN fragments × 3 MFMAs × 16 cycles × 2 waves
MFMA_CYC = {0: 2 * 8 * 3 * 16 * 2, 1: 2 * 16 * 3 * 16 * 2}
NAMES = {0: "BN=64", 1: "BN=128", 2: "BN=64 PRO", 3: "BN=128 PRO"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--pgd-steps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    T, S, B = torch.float32, 256, a.batch
    enc = E4EEncoder(bench.encoder_weights("e4e", S), S, dtype=T, device=dev)
    eng = pgd.AttackEngine(enc, SynthesisNet(make_generator_weights(S, seed=0), S, dtype=T,
                                             device=dev), VGGNet(make_vgg_weights(1234), dtype=T,
                                                                 device=dev))
    g = torch.Generator().manual_seed(1000)
    x0 = (torch.rand(B, 3, S, S, generator=g) * 2 - 1).to(dev)
    tgt = (torch.rand(B, 3, S, S, generator=g) * 2 - 1).to(dev)
    lib = _lib.load()
    assert os.path.basename(_lib.LIB_PATH) == "libmiattack_stamps.so"
    fn = lib.mia_debug_x6_stamps
    fn.restype, fn.argtypes = ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]
    buf = (ctypes.c_ulonglong * 64)()
    eng.run(x0, tgt, a.pgd_steps, 8 / 255, 2 / 255)
    torch.cuda.synchronize()
    assert fn(buf, 1) == 0
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    eng.run(x0, tgt, a.pgd_steps, 8 / 255, 2 / 255)
    e1.record()
    torch.cuda.synchronize()
    assert fn(buf, 0) == 0
    print(f"attack {e0.elapsed_time(e1):.1f} ms")
    for v in range(4):
        r = [buf[v * 16 + i] for i in range(16)]
        nb = r[0]
        if not nb:
            continue
        tot, pro, cv, epi, rt, steps = r[1], r[2], r[3], r[4], r[5], r[6]
        loop = tot - pro - epi - cv
        ideal = steps * MFMA_CYC[v & 1]
        print(f"{NAMES[v]:11s} blocks {nb:9d}  cycles/block {tot / nb:9.0f}  "
              f"prologue {pro / tot:6.1%}  splits {cv / tot:6.1%}  epilogue {epi / tot:6.1%}  "
              f"loop {loop / tot:6.1%}  loop vs MFMA-only {ideal / loop:6.1%}  "
              f"clock {tot / rt * 0.1:5.2f} GHz  step-end wait+barrier: weights wave "
              f"{r[7] / loop:6.1%} halo wave {r[8] / loop:6.1%} of the loop")


if __name__ == "__main__":
    main()
