"""Summarize a rocprofv3 run of bench.py into the committed per-round profile files.

    python profiles/summarize_rocprof.py <kernel_stats.csv> [--fetch counter_collection.csv]
        [--write counter_collection.csv] [--steps S] --out profiles/rNN_<name>

Writes <out>.md (per-kernel table, time per bench step) and <out>.json (the dominant kernel's
aggregate: every conv_kernel<...> instantiation is the same implicit-GEMM conv, so the launch
average is Σ duration / Σ calls over them — the figure bench.py's live HIP-event roofline must
agree with). HBM traffic per launch follows /opt/skills/guides/MI355X_MICROARCH.md §HBM:
FETCH_SIZE and WRITE_SIZE come from separate --pmc passes, are in KiB, and FETCH_SIZE is doubled
on gfx950 (it tallies 128-B requests at 64 B).
"""
import argparse
import csv
import gzip
import json
import os
import re
from collections import defaultdict

# every kernel a conv API call of the attack launches (ops.conv3x3 / conv2d / upconv_fwd /
# upconv_dgrad / s2_dgrad_halo — the calls bench.py brackets with HIP events): the implicit-GEMM
# tiles, the halo tiles (fp32 x6 and fp16 / bf16), the halo up-convs (fp32 upconv_x6_kernel and
# fp16 / bf16 upconv_halo_kernel, both also in DG mode for the stride-2 input gradients), the
# weights-resident and thin-channel kernels (the fp32 VALU VGG / e4e input layers included)
CONV = re.compile(r"conv_(halo_|wres_|wres32_|wres128_|halo_x6_|halo_x6s_|halo_x6h_)?kernel|upconv_(halo|x6|x6s)_kernel|"
                  r"conv_thin(_in|_out|_out_strip|32)(_f32)?_kernel|modulate_weights_kernel")
# the up-conv FORWARD through the halo kernel (mia_upconv_fwd_halo[_split]) is ONE API call that
# launches TWO kernels (the halo up-conv for the interior + a generic conv_kernel for the last row
# / column), so the per-call count that bench.py's HIP events see is launches − these launches
# (the DG = 1 input-gradient mode is one launch: fp16 upconv_halo_kernel<T, PRO, DG>,
# fp32 upconv_x6_kernel<DG, PRO, …>)
# fp32 upconv_x6_kernel<DG, PRO, …>; (rocprofv3 writes demangled names; mangled forms too)
PAIRED = re.compile(r"upconv_halo_kernel<[^<>]*(<[^<>]*>)?[^<>]*, (true|false), false>|"
                    r"upconv_x6_kernel<false,|upconv_halo_kernelI\w+?Lb[01]ELb0E|"
                    r"upconv_x6_kernelILb0E|modulate_weights_kernel")
# template parameter names per kernel (csrc/*.hip), so that every instantiation prints in full —
# tile, epilogue feature mask and flags — and each PMC row maps to one launch class (verdict r05
# item 7: the round-5 fp16 tables collapsed the EPI argument)
TPARAMS = {
    "conv_kernel": ("T", "tile", "pro", "smallc", "epi", "x6b"),
    "conv_halo_kernel": ("T", "tile", "pro", "epi"),
    "conv_halo_x6_kernel": ("bn", "pro", "epi", "early", "prio", "unr", "tps"),
    "conv_halo_x6s_kernel": ("pro", "epi"),
    "upconv_halo_kernel": ("T", "pro", "dgrad", "bn"),
    "upconv_x6_kernel": ("dgrad", "pro", "early", "prio"),
    "upconv_x6s_kernel": ("dgrad", "pro"),
    "conv_wres_kernel": ("T", "tile", "epi"),
    "conv_wres128_kernel": ("T", "cin", "epi", "cout"),
    "conv_wres32_kernel": ("T", "pro", "epi"),
    "blur4_strip_kernel": ("T", "fwd", "noise"),
    "torgb_bwd_kernel": ("T", "front"),
    "maxpool2_bwd_kernel": ("T", "tap"),
}
# halo_epilogue.h namespace epi: the feature bits of an EPI mask (bits 8-9: the activation)
EPI_BITS = ((1, "osc"), (2, "noise"), (4, "bias"), (8, "tap"), (16, "mask"), (32, "acc"),
            (64, "sdot"), (128, "bab"), (1024, "msl"), (2048, "csum"))
EPI_ACT = {1: "relu", 2: "lrelu", 3: "prelu"}
_TYPES = {"f": "f32", "DF16_": "f16", "DF16b": "bf16", "i": "int", "b": "bool"}


def _epi(v):
    if v < 0:
        return str(v)
    parts = [n for bit, n in EPI_BITS if v & bit]
    if (v >> 8) & 3:
        parts.append(EPI_ACT.get((v >> 8) & 3, "act?"))
    return "|".join(parts) or "0"


def _args(m, i):
    """Parse an Itanium template-argument list starting after 'I' at m[i]; returns (list, i)."""
    out = []
    while i < len(m) and m[i] != "E":
        if m.startswith("Lb", i):
            out.append(m[i + 2] == "1")
            i += 4
        elif m.startswith("Li", i) or m.startswith("Lj", i):
            j = m.index("E", i)
            t = m[i + 2:j]
            out.append(-int(t[1:]) if t.startswith("n") else int(t))
            i = j + 1
        elif m.startswith("NS_", i) or m.startswith("N3mia", i):
            i += 3 if m.startswith("NS_", i) else 5
            k = i
            while m[k].isdigit():
                k += 1
            ln = int(m[i:k])
            name = m[k:k + ln]
            i = k + ln
            sub = []
            if m[i] == "I":
                sub, i = _args(m, i + 1)
                i += 1  # the template list's E
            i += 1      # the nested name's E
            out.append((name, sub))
        else:
            for tok, nm in _TYPES.items():
                if m.startswith(tok, i):
                    out.append(nm)
                    i += len(tok)
                    break
            else:
                raise ValueError(m[i:])
    return out, i


def _fmt(v, pname):
    if isinstance(v, str):  # a type argument
        return v
    if isinstance(v, bool):
        return f"{pname}={int(v)}"
    if isinstance(v, tuple):
        name, sub = v
        if name == "Tile" and len(sub) == 5:  # Tile<WM, WN, FM, FN, STAGES>
            wm, wn, fm, fn, st = sub
            return f"{wm * fm * 16}x{wn * fn * 16},{st}st"
        if name == "HaloTile" and len(sub) >= 2:  # HaloTile<BN, PH, …>
            return f"{sub[1]}x16px x {sub[0]}ch," + ",".join(map(str, sub[2:]))
        return f"{name}<{','.join(map(str, sub))}>"
    if pname == "epi" and isinstance(v, int):
        return f"epi={_epi(v)}"
    return f"{pname}={v}" if pname not in ("T", "tile") else str(v)


def short(name):
    """Kernel name with every template argument (mangled rocprofv3 names are demangled here)."""
    m = re.match(r"_ZN3mia(\d+)", name)
    if m:
        ln = int(m.group(1))
        base = name[m.end():m.end() + ln]
        i = m.end() + ln
        if i < len(name) and name[i] == "I":
            try:
                args, _ = _args(name, i + 1)
            except (ValueError, IndexError):
                return base + "<?>"
            pn = TPARAMS.get(base, ())
            return base + "<" + ",".join(_fmt(v, pn[j] if j < len(pn) else f"a{j}")
                                        for j, v in enumerate(args)) + ">"
        return base
    return name.split("(")[0]


def read_stats(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((r["Name"], int(r["Calls"]), int(r["TotalDurationNs"])))
    return rows


def read_pmc(path, counter):
    per = defaultdict(lambda: [0, 0.0])
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] != counter:
                continue
            k = r["Kernel_Name"]
            per[k][0] += 1
            per[k][1] += float(r["Counter_Value"]) * 1024.0  # KiB → bytes
    return per


def busy_union_ns(trace_path, pattern=None):
    """GPU-busy time of a kernel trace: the union of the dispatch intervals (the e4e style heads
    run on side streams, so kernel durations overlap and their sum exceeds the busy time).
    pattern: only the kernels whose name it matches (the conv kernels: conv-busy time)."""
    iv = []
    opener = gzip.open if trace_path.endswith(".gz") else open
    with opener(trace_path, "rt") as f:
        for r in csv.DictReader(f):
            if pattern is None or pattern.search(r["Kernel_Name"]):
                iv.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    iv.sort()
    busy, (cs, ce) = 0, iv[0]
    for s0, e0 in iv[1:]:
        if s0 > ce:
            busy += ce - cs
            cs, ce = s0, e0
        else:
            ce = max(ce, e0)
    return busy + ce - cs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("stats")
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--mfma", help="counter_collection.csv of the SQ_VALU_MFMA_BUSY_CYCLES / "
                    "GRBM_GUI_ACTIVE / SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE pass")
    ap.add_argument("--steps", type=int, default=3, help="bench steps in the trace (warmup+timed)")
    ap.add_argument("--out", required=True)
    ap.add_argument("--title", default="")
    ap.add_argument("--bench-line", help="the bench JSON line of the same command: its conv FLOPs "
                    "per step ÷ this trace's conv-busy time per step is the roofline `achieved` "
                    "reproduced from the profile")
    a = ap.parse_args()
    rows = read_stats(a.stats)
    tot = sum(r[2] for r in rows)
    conv_calls = sum(c for n, c, t in rows if CONV.search(n)) - sum(
        c for n, c, t in rows if PAIRED.search(n))
    conv_ns = sum(t for n, c, t in rows if CONV.search(n))
    out = {"source": a.stats, "bench_steps_in_trace": a.steps,
           "kernel_ms_per_step": tot / 1e6 / a.steps,
           "conv_kernel": {"launches": conv_calls, "total_ms": conv_ns / 1e6,
                           "avg_launch_us": conv_ns / conv_calls / 1e3 if conv_calls else None,
                           "share_of_kernel_time": conv_ns / tot}}
    lines = [f"# {a.title}", "", f"rocprofv3 --kernel-trace --stats; {a.steps} bench steps in the "
             f"trace; kernel time per step {tot / 1e6 / a.steps:.1f} ms", ""]
    trace = a.stats.replace("kernel_stats.csv", "kernel_trace.csv")
    if trace != a.stats and not os.path.exists(trace) and os.path.exists(trace + ".gz"):
        trace += ".gz"  # the committed traces are gzipped
    if trace != a.stats and os.path.exists(trace):
        busy = busy_union_ns(trace)
        cbusy = busy_union_ns(trace, CONV)
        out["gpu_busy_ms_per_step_incl_setup"] = busy / 1e6 / a.steps
        out["conv_kernel"]["busy_ms"] = cbusy / 1e6
        out["conv_kernel"]["avg_busy_us_per_call"] = cbusy / conv_calls / 1e3
        lines += [f"GPU busy (union of dispatch intervals, incl. the one-off setup before the first "
                  f"step) {busy / 1e6 / a.steps:.1f} ms per step (one stream: the kernels do not "
                  f"overlap). "
                  f"Conv-busy time (union of the conv dispatches) {cbusy / 1e6 / a.steps:.1f} ms "
                  f"per step = {cbusy / conv_calls / 1e3:.1f} µs per conv API call (bench.py's "
                  f"avg_launch_us is the union of its HIP-event intervals around the same calls, "
                  f"which also hold each call's launch gap and reduction finish).", ""]
        if a.bench_line:
            bl = json.loads(open(a.bench_line).read().strip().splitlines()[-1])
            rf = bl["roofline"]
            flops_step = rf["algorithmic_gflop_per_launch"] * 1e9 * rf["launches"] / bl["steps"]
            calls_step = rf["launches"] / bl["steps"]
            ach = flops_step / (cbusy / a.steps * 1e-9) / 1e12
            out["conv_kernel"]["bench_calls_per_step"] = calls_step
            out["conv_kernel"]["trace_calls_per_step"] = conv_calls / a.steps
            out["conv_kernel"]["achieved_tflops_from_trace"] = ach
            out["conv_kernel"]["achieved_tflops_bench"] = rf["achieved"]
            lines += [f"Roofline reproduced from this trace: the bench line's conv work "
                      f"{flops_step / 1e12:.1f} TFLOP per step ({calls_step:.0f} conv API calls; "
                      f"this trace: {conv_calls / a.steps:.0f} per step) ÷ the trace's conv-busy "
                      f"time = {ach:.1f} TFLOP/s; the bench line's live HIP-event figure "
                      f"{rf['achieved']:.1f} TFLOP/s ({100 * (rf['achieved'] / ach - 1):+.1f} %).",
                      ""]
    lines += [
             "| kernel | calls/step | ms/step | avg µs | share |", "|---|---|---|---|---|"]
    for n, c, t in sorted(rows, key=lambda r: -r[2]):
        lines.append(f"| `{short(n)}` | {c / a.steps:.0f} | {t / 1e6 / a.steps:.2f} | "
                     f"{t / c / 1e3:.1f} | {100 * t / tot:.2f}% |")
    lines += ["", f"conv API calls (all conv kernels; a halo up-conv call = its 2 launches): "
              f"{conv_calls} calls, average "
              f"{out['conv_kernel']['avg_launch_us']:.1f} µs, {100 * conv_ns / tot:.1f}% of kernel time"]
    if a.fetch and a.write:
        fe, wr = read_pmc(a.fetch, "FETCH_SIZE"), read_pmc(a.write, "WRITE_SIZE")
        fb = sum(v[1] for k, v in fe.items() if CONV.search(k))
        fl = sum(v[0] for k, v in fe.items() if CONV.search(k)) - sum(
            v[0] for k, v in fe.items() if PAIRED.search(k))
        wb = sum(v[1] for k, v in wr.items() if CONV.search(k))
        wl = sum(v[0] for k, v in wr.items() if CONV.search(k)) - sum(
            v[0] for k, v in wr.items() if PAIRED.search(k))
        per = 2.0 * fb / fl + wb / wl
        out["conv_kernel"]["hbm_bytes_per_launch"] = per
        out["conv_kernel"]["fetch_bytes_per_launch_x2"] = 2.0 * fb / fl
        out["conv_kernel"]["write_bytes_per_launch"] = wb / wl
        out["conv_kernel"]["pmc_launches"] = [fl, wl]
        lines += ["", "PMC (separate passes, FETCH_SIZE×2 per the gfx950 correction):",
                  f"conv HBM bytes per API call = {per / 1e6:.1f} MB "
                  f"(fetch {2 * fb / fl / 1e6:.1f} MB, write {wb / wl / 1e6:.1f} MB, "
                  f"{fl} calls)", "", "| kernel | fetch MB/launch (×2) | write MB/launch |",
                  "|---|---|---|"]
        for k in sorted(fe, key=lambda k: -fe[k][1]):
            w = wr.get(k, [1, 0.0])
            lines.append(f"| `{short(k)}` | {2 * fe[k][1] / fe[k][0] / 1e6:.2f} | "
                         f"{w[1] / max(w[0], 1) / 1e6:.2f} |")
    if a.mfma:
        c = {k: read_pmc(a.mfma, k) for k in ("SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE",
                                              "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE")}
        busy, gui = c["SQ_VALU_MFMA_BUSY_CYCLES"], c["GRBM_GUI_ACTIVE"]

        def agg(d, pat=CONV):
            return sum(v[1] for k, v in d.items() if pat.search(k)) / 1024.0  # undo KiB scaling

        # GRBM_GUI_ACTIVE is summed over the 8 XCDs → ÷8 = the dispatch's cycles; the MFMA busy
        # cycles are summed over every SIMD (256 CUs × 4) → busy fraction of the matrix pipes
        frac = agg(busy) / (agg(gui) / 8.0 * 1024.0)
        ldsc = agg(c["SQ_LDS_BANK_CONFLICT"]) / max(agg(c["SQ_LDS_IDX_ACTIVE"]), 1.0)
        out["conv_kernel"]["mfma_busy_frac"] = frac
        out["conv_kernel"]["lds_bank_conflict_frac"] = ldsc
        lines += ["", "PMC pass SQ_VALU_MFMA_BUSY_CYCLES / GRBM_GUI_ACTIVE / SQ_LDS_BANK_CONFLICT / "
                  "SQ_LDS_IDX_ACTIVE (MFMA busy = busy cycles ÷ (GRBM_GUI_ACTIVE/8 × 1024 SIMDs); "
                  "LDS conflict = conflict cycles ÷ LDS-active cycles):",
                  f"conv kernels: MFMA busy {frac:.3f}, LDS bank-conflict cycles {ldsc:.4f} of "
                  f"LDS-active", "", "| kernel | launches | MFMA busy | LDS conflict |",
                  "|---|---|---|---|"]
        for k in sorted(busy, key=lambda k: -busy[k][1])[:40]:
            g = gui.get(k, [1, 0.0])[1] / 1024.0
            ia = c["SQ_LDS_IDX_ACTIVE"].get(k, [1, 0.0])[1]
            bc = c["SQ_LDS_BANK_CONFLICT"].get(k, [1, 0.0])[1]
            lines.append(f"| `{short(k)}` | {busy[k][0]} | "
                         f"{busy[k][1] / 1024.0 / max(g / 8.0 * 1024.0, 1.0):.3f} | "
                         f"{bc / ia if ia else 0.0:.4f} |")
    open(a.out + ".md", "w").write("\n".join(lines) + "\n")
    json.dump(out, open(a.out + ".json", "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
