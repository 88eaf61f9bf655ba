"""Per-layer table of the VGG cascade (tools/vgg_cascade.py) from rocprofv3 runs: duration,
algorithmic TFLOP/s, HBM bytes from PMC (FETCH_SIZE ×2 per the gfx950 correction + WRITE_SIZE,
separate passes) and the achieved HBM GB/s (north_star: "rocprof reports achieved HBM GB/s on the
VGG conv cascade").

    python tools/vgg_layers_summary.py --trace kernel_trace.csv --fetch fetch.csv --write write.csv
        [--mfma mfma.csv] --batch 128 --dtype fp32 --out profiles/r02_vgg_cascade_fp32_b128

The cascade's last rep is the last 25 dispatches that are not runtime fills / copies; they are
labelled in launch order (tools/vgg_cascade.LABELS; every process launches the same sequence, so
the passes align by position)."""
import argparse
import csv
import json
import os
import re
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from vgg_cascade import LABELS  # noqa: E402

SKIP = re.compile(r"rocclr|fillBuffer|copyBuffer|Copy")
# (Cin, Cout, output side) per conv label at 256² input (code/vgg.py:12-39)
CONVS = {"conv1_1": (3, 64, 256), "conv1_2": (64, 64, 256), "conv2_1": (64, 128, 128),
         "conv2_2": (128, 128, 128), "conv3_1": (128, 256, 64), "conv3_2": (256, 256, 64),
         "conv3_3": (256, 256, 64), "conv4_1": (256, 512, 32), "conv4_2": (512, 512, 32)}


def dispatches(path, kind):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            if SKIP.search(r["Kernel_Name"]):
                continue
            rows.append(r)
    if kind == "trace":
        return [(r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
                for r in rows][-len(LABELS):]
    per = defaultdict(dict)
    order = []
    for r in rows:
        d = int(r["Dispatch_Id"])
        if d not in per:
            order.append(d)
        per[d][r["Counter_Name"]] = per[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return [per[d] for d in order][-len(LABELS):]


# input-gradient epilogue operands read besides g, in units of the layer's Cin planes: the ReLU
# mask of the layer below (mask_a) and the tap-MSE term (tap_a = the mask tensor at conv1_2, +
# its target) — vgg.VGGNet.backward
AUX = {"dconv4_2": 1, "dconv3_3": 1, "dconv3_2": 1, "dconv3_1": 2, "dconv2_2": 1, "dconv1_2": 2}


# pools: (input channels, input side); the 2×2 window's input gradient at pool1 carries the fused
# conv1_2 tap-MSE term (maxpool2_bwd<…, true>: reads the tap and its target)
POOLS = {"pool1": (64, 256, True), "pool2": (128, 128, False), "pool3": (256, 64, False)}


def work(label, N, esize):
    """(algorithmic FLOP, algorithmic HBM bytes: inputs read once + outputs written once)."""
    base = label.lstrip("d")
    if base in POOLS:
        c, r, tap = POOLS[base]
        ro = -(-r // 2)
        big, small = N * r * r * c * esize, N * ro * ro * c * esize
        if label.startswith("d"):  # read x (+ tap target) and g_out, write g_in
            return 0, big * (3 if tap else 2) + small
        return 0, big + small
    if label == "tap4_2":  # read the tap and its target, write the gradient (32², 512 ch)
        return 0, 3 * N * 32 * 32 * 512 * esize
    if base not in CONVS:
        return 0, None
    cin, cout, r = CONVS[base]
    cin_p = 8 if cin == 3 else cin
    fl = 2 * N * r * r * 9 * cin * cout
    if label.startswith("d"):  # read g (Cout planes) + aux (Cin planes), write Cin planes
        return fl, N * r * r * (cout + cin_p * (1 + AUX.get(label, 0))) * esize
    return fl, N * r * r * (cin_p + cout) * esize


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace", required=True)
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--mfma")
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--dtype", default="fp32")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    es = 4 if a.dtype == "fp32" else 2
    tr = dispatches(a.trace, "trace")
    fe = dispatches(a.fetch, "pmc")
    wr = dispatches(a.write, "pmc")
    mf = dispatches(a.mfma, "pmc") if a.mfma else [{}] * len(LABELS)
    assert len(tr) == len(fe) == len(wr) == len(LABELS), (len(tr), len(fe), len(wr))
    rows, tot_ns, tot_b, tot_alg = [], 0, 0.0, 0.0
    lines = [f"# VGG16 cascade per layer ({a.dtype}, {a.batch} images at 256²: code/vgg.py:44-64 "
             f"forward + the tap-MSE input gradient)", "",
             "rocprofv3 kernel trace + separate FETCH_SIZE / WRITE_SIZE passes (FETCH_SIZE ×2, "
             "gfx950 correction); last rep of tools/vgg_cascade.py. GB/s = PMC HBM bytes ÷ "
             "dispatch duration; alg. MB = inputs read once + outputs written once; PMC/alg = "
             "the wasted-traffic ratio (re-reads of halos / weights beyond one pass).", "",
             "| layer | kernel | µs | TFLOP/s | HBM MB (PMC) | alg. MB | PMC/alg | HBM GB/s | "
             "MFMA busy |",
             "|---|---|---|---|---|---|---|---|---|"]
    for lab, (name, ns), f, w, m in zip(LABELS, tr, fe, wr, mf):
        hb = 2.0 * f.get("FETCH_SIZE", 0.0) * 1024 + w.get("WRITE_SIZE", 0.0) * 1024
        fl, alg = work(lab, a.batch, es)
        busy = None
        if m.get("SQ_VALU_MFMA_BUSY_CYCLES") and m.get("GRBM_GUI_ACTIVE"):
            busy = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (m["GRBM_GUI_ACTIVE"] / 8 * 1024)
        kn = re.sub(r"^_ZN3mia\d+", "", name).split("I")[0][:28]
        r = dict(layer=lab, kernel=kn, us=ns / 1e3, tflops=fl / ns / 1e3 if fl else None,
                 hbm_mb=hb / 1e6, alg_mb=alg / 1e6 if alg else None, gbs=hb / ns,
                 mfma_busy=busy)
        rows.append(r)
        tot_ns += ns
        tot_b += hb
        tot_alg += alg or 0.0
        lines.append(f"| {lab} | `{kn}` | {ns / 1e3:.1f} | "
                     f"{'' if not fl else f'{fl / ns / 1e3:.1f}'} | {hb / 1e6:.1f} | "
                     f"{'' if not alg else f'{alg / 1e6:.1f}'} | "
                     f"{'' if not alg else f'{hb / alg:.2f}'} | {hb / ns:.0f} | "
                     f"{'' if busy is None else f'{busy:.2f}'} |")
    lines += ["", f"cascade: {tot_ns / 1e3:.0f} µs, {tot_b / 1e6:.0f} MB HBM (PMC) vs "
              f"{tot_alg / 1e6:.0f} MB algorithmic = {tot_b / tot_alg:.2f}× wasted-traffic ratio; "
              f"{tot_b / tot_ns:.0f} GB/s average (PMC bytes), "
              f"{tot_alg / tot_ns:.0f} GB/s algorithmic"]
    open(a.out + ".md", "w").write("\n".join(lines) + "\n")
    json.dump({"layers": rows, "total_us": tot_ns / 1e3, "total_hbm_mb": tot_b / 1e6,
               "total_alg_mb": tot_alg / 1e6},
              open(a.out + ".json", "w"), indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main()
