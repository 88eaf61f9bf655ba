"""Small / streaming kernels at the bench's shapes: timing and bit-identity across two libraries
(tuning aid; GPU only).

    MIA_LIB_VARIANT=<lib> python tools/probe/small_ab.py [--dtype fp32] [--save /tmp/ew_x.pt]
    python tools/probe/small_ab.py --compare /tmp/ew_a.pt /tmp/ew_b.pt

Times (HIP events, 20 calls each) mia_torgb_fwd at the 256² generator's seven ToRGB layers, the
StyledConv style gradient through the demodulation (mia_demod_bwd) and the e4e SE module's two
small FC kernels (mia_se_fwd_parts / mia_se_bwd_parts) at their IR-SE50 shapes; prints µs per call
and, for ToRGB, the algorithmic HBM rate (input read once). --save keeps every output (seeded
inputs) so that two libraries' outputs can be compared bitwise with --compare."""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def timeit(call, reps=20):
    for _ in range(3):
        call()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        call()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def run(a):
    import gfa_import  # noqa: F401
    from gfa_amd import ops
    T = {"fp16": torch.float16, "bf16": torch.bfloat16, "fp32": torch.float32}[a.dtype]
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(7)
    N = a.batch
    out = {}
    tot = tot_b = 0.0
    for R, C in ((4, 512), (8, 512), (16, 512), (32, 512), (64, 512), (128, 256), (256, 128)):
        pre = torch.randn(N, R, R, C, device=dev, generator=g).to(T)
        st = torch.randn(N, C, device=dev, generator=g)
        wr = torch.randn(3, C, device=dev, generator=g) / C ** 0.5
        b = torch.randn(3, device=dev, generator=g)
        skip = torch.randn(N, 3, R // 2, R // 2, device=dev, generator=g) if R > 4 else None
        rgb = torch.empty(N, 3, R, R, device=dev)
        us = timeit(lambda: ops.torgb_fwd(pre, st, wr, b, skip, rgb))
        tot += us
        out[f"torgb_{R}"] = rgb.clone()
        grgb = torch.randn(N, 3, R, R, device=dev, generator=g)
        ga = torch.empty_like(pre)
        gs = torch.empty(N, C, device=dev)
        ub = timeit(lambda: ops.torgb_bwd(grgb, pre, st, wr, ga, gs, accumulate=False))
        gs.zero_()
        ops.torgb_bwd(grgb, pre, st, wr, ga, gs, accumulate=False)
        out[f"torgb_bwd_{R}"] = torch.cat([ga.float().flatten(), gs.flatten()])
        tot_b += ub
        print(f"torgb R={R:3d} C={C:3d}: fwd {us:8.1f} us {pre.numel() * pre.element_size() / us / 1e6:5.2f} TB/s"
              f" | bwd {ub:8.1f} us {2 * pre.numel() * pre.element_size() / ub / 1e6:5.2f} TB/s", flush=True)
    print(f"torgb per generator forward: fwd {tot:.1f} us, bwd {tot_b:.1f} us "
          f"(x20 per PGD-20 step: {tot * 20 / 1e3:.2f} + {tot_b * 20 / 1e3:.2f} ms)")
    for R, C in ((256, 128), (64, 512)):
        act = torch.randn(N, R, R, C, device=dev, generator=g).to(T)
        st = torch.randn(N, C, device=dev, generator=g)
        wr = torch.randn(3, C, device=dev, generator=g) / C ** 0.5
        grgb = torch.randn(N, 3, R, R, device=dev, generator=g)
        gy = torch.empty_like(act)
        gs = torch.empty(N, C, device=dev)
        q = torch.empty(N, C, device=dev)
        dm = torch.rand(N, C, device=dev, generator=g) + 0.5
        nz = torch.randn(R * R, device=dev, generator=g)
        bz = torch.randn(C, device=dev, generator=g)
        uf = timeit(lambda: ops.torgb_bwd_front(grgb, act, st, wr, gy, gs, dm, nz, 0.3, bz, q))
        gs.zero_()
        q.zero_()
        ops.torgb_bwd_front(grgb, act, st, wr, gy, gs, dm, nz, 0.3, bz, q)
        out[f"torgb_front_{R}"] = torch.cat([gy.float().flatten(), gs.flatten(), q.flatten()])
        print(f"torgb_bwd_front R={R:3d} C={C:3d}: {uf:8.1f} us {2 * act.numel() * act.element_size() / uf / 1e6:5.2f} TB/s",
              flush=True)
    tot = 0.0
    for Cin, Cout, calls in ((512, 512, 10), (256, 512, 1), (128, 256, 1), (512, 256, 1)):
        q = torch.randn(N, Cout, device=dev, generator=g)
        dm = torch.rand(N, Cout, device=dev, generator=g) + 0.5
        wsq = torch.rand(Cout, Cin, device=dev, generator=g)
        s = torch.randn(N, Cin, device=dev, generator=g)
        gs = torch.zeros(N, Cin, device=dev)
        us = timeit(lambda: ops.demod_bwd(q, dm, wsq, s, gs))
        gs.zero_()
        ops.demod_bwd(q, dm, wsq, s, gs)
        out[f"demod_{Cin}_{Cout}"] = gs.clone()
        tot += us * calls
        print(f"demod_bwd Cin={Cin} Cout={Cout}: {us:7.1f} us", flush=True)
    for S, pf in ((256, 1), (256, 2)):
        img = torch.rand(N, 3, S, S, device=dev, generator=g) * 2 - 1
        y = torch.empty(N, S // pf, S // pf, 8, dtype=T, device=dev)
        us = timeit(lambda: ops.image_to_nhwc(img, y, pf, 8))
        out[f"image_to_nhwc_{S}_{pf}"] = y.float().clone()
        print(f"image_to_nhwc S={S} pf={pf}: {us:7.1f} us "
              f"{(img.numel() * 4 + y.numel() * y.element_size()) / us / 1e6:5.2f} TB/s", flush=True)
    for Cin, Cout in ((512, 512), (256, 128)):
        s = torch.randn(N, Cin, device=dev, generator=g)
        wsq = torch.rand(Cout, Cin, device=dev, generator=g)
        dm = torch.empty(N, Cout, device=dev)
        us = timeit(lambda: ops.style_demod(s, wsq, dm))
        out[f"style_demod_{Cin}_{Cout}"] = dm.clone()
        print(f"style_demod Cin={Cin} Cout={Cout}: {us:7.1f} us", flush=True)
    for C, hw in ((64, 128 * 128), (128, 64 * 64), (256, 32 * 32), (512, 16 * 16)):
        Cr = C // 16
        nch = ops.chan_sum_parts(N, hw)
        part = torch.randn(N * nch * C, device=dev, generator=g)
        w1 = torch.randn(Cr, C, device=dev, generator=g) / C ** 0.5
        w2 = torch.randn(C, Cr, device=dev, generator=g) / Cr ** 0.5
        u = torch.empty(N, Cr, device=dev)
        s = torch.empty(N, C, device=dev)
        gavg = torch.empty(N, C, device=dev)
        uf = timeit(lambda: ops.se_fwd_parts(part, hw, w1, w2, u, s))
        ub = timeit(lambda: ops.se_bwd_parts(part, hw, s, u, w1, w2, gavg))
        out[f"se_{C}"] = torch.cat([u.flatten(), s.flatten(), gavg.flatten()])
        print(f"se C={C:3d} hw={hw:5d} nch={nch:3d}: fwd {uf:6.1f} us  bwd {ub:6.1f} us", flush=True)
    if a.save:
        torch.save({k: v.cpu() for k, v in out.items()}, a.save)


def compare(pa, pb):
    A = torch.load(pa, weights_only=True)
    B = torch.load(pb, weights_only=True)
    bad = 0
    for k in A:
        same = torch.equal(A[k], B[k])
        bad += not same
        print(f"{k:16s} {'bit-identical' if same else 'DIFFERS (max abs %.3g)' % (A[k] - B[k]).abs().max()}")
    return bad


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="fp32", choices=["fp16", "bf16", "fp32"])
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--save", default=None)
    ap.add_argument("--compare", nargs=2, default=None)
    a = ap.parse_args()
    if a.compare:
        sys.exit(1 if compare(*a.compare) else 0)
    run(a)


if __name__ == "__main__":
    main()
