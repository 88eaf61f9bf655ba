"""CPU tests of the host side: weight re-layouts, the C ABI surface, API validation, sharding."""
import ctypes
import math
import os
import re
import subprocess
import sys

import pytest
import torch
import torch.nn.functional as F

from conftest import ROOT
from gfa_amd import layouts
from gfa_amd.dist import shard_bounds
from oracle import stylegan2_ref

HEADER = os.path.join(ROOT, "include", "miattack.h")


def _conv_via_matrix(x, m, cout, cin):
    """Apply a [Cout][Kpad] kernel matrix the way the HIP kernel does (tap-major K)."""
    N, _, H, W = x.shape
    cols = F.unfold(x, 3, padding=1)  # (N, cin*9, HW) with ci-major, tap-minor
    cols = cols.view(N, cin, 9, H * W).transpose(1, 2).reshape(N, 9 * cin, H * W)
    y = m[:, :9 * cin] @ cols
    return y.view(N, cout, H, W)


def test_fwd_and_dgrad_matrices():
    g = torch.Generator().manual_seed(0)
    w = torch.randn(6, 5, 3, 3, generator=g, dtype=torch.float64)
    x = torch.randn(2, 5, 7, 7, generator=g, dtype=torch.float64)
    m = layouts.fwd_matrix(w, torch.float64)
    assert torch.allclose(_conv_via_matrix(x, m, 6, 5), F.conv2d(x, w, padding=1))
    gy = torch.randn(2, 6, 7, 7, generator=g, dtype=torch.float64)
    xx = x.clone().requires_grad_(True)
    (gx,) = torch.autograd.grad((F.conv2d(xx, w, padding=1) * gy).sum(), xx)
    md = layouts.dgrad_matrix(w, torch.float64)
    assert torch.allclose(_conv_via_matrix(gy, md, 5, 6), gx)


def test_kpad():
    assert layouts.kpad_for(8, torch.float16) == 128 and layouts.kpad_for(8, torch.float32) == 96
    assert layouts.kpad_for(512, torch.float16) == 4608


def test_upconv_phases_equal_convtranspose_plus_blur():
    """conv_transpose2d(stride 2) + Blur(pad (1,1)) == 4 phase 3×3 convs, pixel-shuffled."""
    g = torch.Generator().manual_seed(1)
    cout, cin, R = 4, 3, 5
    W = torch.randn(cout, cin, 3, 3, generator=g, dtype=torch.float64)
    x = torch.randn(2, cin, R, R, generator=g, dtype=torch.float64)
    t = F.conv_transpose2d(x, W.transpose(0, 1), stride=2)
    ref = stylegan2_ref.upfirdn2d(t, stylegan2_ref.make_kernel([1, 3, 3, 1], torch.float64) * 4,
                                  pad=(1, 1))
    V = layouts.upconv_phases(W)
    y = F.conv2d(x, V, padding=1)
    out = torch.empty_like(ref)
    for p in range(4):
        out[:, :, p // 2::2, p % 2::2] = y[:, p * cout:(p + 1) * cout]
    assert torch.allclose(out, ref, atol=1e-12)


def _header_functions():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\**\s+\**(mia_\w+)\(", txt, re.M)))


def test_library_exports_every_header_symbol():
    from gfa_amd import _lib
    names = _header_functions()
    assert len(names) >= 30
    assert set(names) == set(_lib.SIGNATURES), set(names) ^ set(_lib.SIGNATURES)
    assert os.path.exists(_lib.LIB_PATH), "run __graft_entry__.build() first"
    lib = _lib.load()  # loads without a GPU; no compute call is made
    for n in names:
        assert hasattr(lib, n), n
    assert lib.mia_version() == 1
    assert lib.mia_conv_kpad(8, 1) == 128  # host-only helper


def test_kernel_variant_switch_table():
    """mia_set_tuning / mia_get_tuning (host-only, no GPU): the measured-best defaults, a set value
    read back, and an unknown name rejected with the library's error (include/miattack.h)."""
    from gfa_amd import _lib
    defaults = {"MIA_CONV_HALO": 1, "MIA_CONV_X6": 1, "MIA_HALO_EPI": 1, "MIA_CONV_WRES32": 1,
                "MIA_HALO_C64": 1, "MIA_CONV_WRES128": 1}
    for name, v in defaults.items():
        if os.environ.get(name) is None:
            assert _lib.get_tuning(name) == v, name
    old = _lib.set_tuning("MIA_CONV_WRES32", 0)
    try:
        assert _lib.get_tuning("MIA_CONV_WRES32") == 0
    finally:
        _lib.set_tuning("MIA_CONV_WRES32", old)
    assert _lib.get_tuning("MIA_CONV_WRES32") == old
    with pytest.raises(_lib.MiaError, match="unknown tuning switch"):
        _lib.set_tuning("MIA_NO_SUCH_SWITCH", 1)
    # round 6: switches whose alternative was measured dead are gone from the table
    for gone in ("MIA_THIN_F32", "MIA_EPI_PRERED"):
        with pytest.raises(_lib.MiaError, match="unknown tuning switch"):
            _lib.get_tuning(gone)


# ds_read_b128 serves a wave in 4 lane groups of 16 (MI355X_MICROARCH.md §LDS)
_B128_GROUPS = [[0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27],
                [4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31]]
_B128_GROUPS += [[ln + 32 for ln in g] for g in _B128_GROUPS]


@pytest.mark.parametrize("cin", [64, 128])
def test_wres128_halo_image_is_bank_conflict_free(cin):
    """conv_wres128.hip's halo LDS image: pixel hr (rows padded to 20), 32-channel sub-plane s,
    stored chunk c ^ sw(hr % 20) at (hr/4)·GB + s·256 + (hr%4)·64 + 16·chunk, sw(v) = (v>>1)&3.
    Every A-fragment read (lane: pixel column frow + dx of halo row q, chunk fq) puts the 16 lanes
    of each ds_read_b128 group on 16 distinct 16-byte bank slots, for every q, dx and s; and the
    DMA's lane → (pixel, sub-plane, chunk) decode writes every logical chunk exactly once."""
    PB = 2 * cin
    GB = 4 * PB
    sw = lambda v: (v >> 1) & 3  # noqa: E731

    def addr(hr, s, chunk):
        return (hr // 4) * GB + s * 256 + (hr % 4) * 64 + ((chunk ^ sw(hr % 20)) << 4)

    for q in range(10):
        for dx in range(3):
            for s in range(cin // 32):
                for grp in _B128_GROUPS:
                    slots = {(addr(q * 20 + (ln & 15) + dx, s, ln >> 4) // 16) % 16 for ln in grp}
                    assert len(slots) == 16, (q, dx, s)
    seen = set()
    hbuf = 200 * PB
    for b in range(0, hbuf, 16):  # the kernel's DMA decode of LDS byte b
        g, rem = divmod(b, GB)
        s, pp, cs = rem >> 8, (rem >> 6) & 3, (rem >> 4) & 3
        hr = 4 * g + pp
        chunk = cs ^ sw(hr % 20)
        assert addr(hr, s, chunk) == b
        seen.add((hr, s, chunk))
    assert len(seen) == 200 * (cin // 32) * 4


@pytest.mark.parametrize("cname,pyname", [("mia_conv_args", "ConvArgs"),
                                          ("mia_conv_group", "ConvGroup"),
                                          ("mia_conv_batch", "ConvBatch"),
                                          ("mia_gemm_seg", "GemmSeg"),
                                          ("mia_gemm_group", "GemmGroup")])
def test_abi_struct_layout_matches_c(tmp_path, cname, pyname):
    """ctypes mirrors of the ABI structs have the C compiler's offsets and sizes."""
    from gfa_amd import _lib
    S = getattr(_lib, pyname)
    fields = [f for f, _ in S._fields_]
    src = tmp_path / "off.c"
    body = "\n".join(f'printf("%s %zu\\n", "{f}", offsetof({cname}, {f}));' for f in fields)
    src.write_text(f'#include <stdio.h>\n#include <stddef.h>\n#include "miattack.h"\n'
                   f'int main(void){{ {body} printf("size %zu\\n", sizeof({cname})); '
                   f'return 0; }}\n')
    exe = tmp_path / "off"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)],
                   check=True)
    out = dict(line.split() for line in subprocess.run([str(exe)], capture_output=True,
                                                         text=True, check=True).stdout.split("\n")
               if line)
    for f in fields:
        assert int(out[f]) == getattr(S, f).offset, f
    assert int(out["size"]) == ctypes.sizeof(S)


def test_shard_bounds_cover_and_balance():
    for n in (1, 7, 128, 1024, 1023):
        for world in (1, 2, 3, 8):
            spans = [shard_bounds(n, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1


class _StubDecoder:
    size = 32
    device = torch.device("cpu")


class _StubNet:
    decoder = _StubDecoder()
    vgg = object()


def test_attack_argument_validation_before_any_device_work():
    from gfa_amd import attack
    x = torch.zeros(2, 3, 32, 32)
    t = torch.zeros(1, 3, 32, 32)
    net = _StubNet()
    with pytest.raises(ValueError):
        attack(net, torch.zeros(2, 3, 16, 16), 8 / 255, 2, target=t)   # wrong size
    with pytest.raises(ValueError):
        attack(net, x + 2.0, 8 / 255, 2, target=t)                     # out of [-1,1]
    with pytest.raises(ValueError):
        attack(net, x, 8 / 255, 2)                                     # no target
    with pytest.raises(ValueError):
        attack(net, x, -1.0, 2, target=t)                              # eps <= 0
    with pytest.raises(ValueError):
        attack(net, x, 8 / 255, 2, target=t, norm="l2")                # unsupported norm
    with pytest.raises(ValueError):
        attack(net, x, None, 2, target=t, norm="adam", lr=0.0)         # Adam needs lr > 0
    with pytest.raises(ValueError):
        attack(net, x, None, 2, target=t, norm="linf")                 # PGD needs eps
    with pytest.raises(ValueError):
        attack(net, x, 8 / 255, 1.5, target=t)                         # integer steps


def test_no_cpu_fallback_in_product():
    """The product package never imports the oracle and every op goes through the C ABI."""
    pkg = os.path.join(ROOT, "adversarial-attacks-on-gan-based-image-fusion_amd")
    for fn in os.listdir(pkg):
        if fn.endswith(".py"):
            src = open(os.path.join(pkg, fn)).read()
            assert not re.search(r"^\s*(from|import)\s+oracle", src, re.M), fn
            assert "torch.nn.functional" not in src, fn  # no torch compute fallback
    assert math.isfinite(1.0) and sys.version_info >= (3, 8)


def test_upconv_subpixel_matrices_equal_conv_transpose():
    """The four sub-pixel phase GEMMs reproduce conv_transpose2d(stride 2, pad 0) exactly."""
    g = torch.Generator().manual_seed(2)
    cout, cin, R = 3, 4, 5
    W = torch.randn(cout, cin, 3, 3, generator=g, dtype=torch.float64)
    x = torch.randn(2, cin, R, R, generator=g, dtype=torch.float64)
    T = F.conv_transpose2d(x, W.transpose(0, 1), stride=2)  # (2, cout, 2R+1, 2R+1)
    mats = layouts.upconv_subpixel_matrices(W, torch.float64)
    for ph, m in enumerate(mats):
        py, px = ph >> 1, ph & 1
        kh, kw = 2 - py, 2 - px
        ho, wo = R + 1 - py, R + 1 - px
        xp = F.pad(x, [kw - 1, 1, kh - 1, 1])  # input m + t − (k−1), zero outside
        out = torch.zeros(2, cout, ho, wo, dtype=torch.float64)
        for ty in range(kh):
            for tx in range(kw):
                blk = m[:, (ty * kw + tx) * cin:(ty * kw + tx + 1) * cin]  # (cout, cin)
                out += torch.einsum("oc,nchw->nohw", blk, xp[:, :, ty:ty + ho, tx:tx + wo])
        assert torch.allclose(out, T[:, :, py::2, px::2], atol=1e-12), ph
    # the adjoint (stride-2 conv with the un-flipped kernel) is the input gradient
    xx = x.clone().requires_grad_(True)
    gT = torch.randn(T.shape, generator=g, dtype=torch.float64)
    (gx,) = torch.autograd.grad((F.conv_transpose2d(xx, W.transpose(0, 1), stride=2) * gT).sum(), xx)
    md = layouts.upconv_dgrad_matrix(W, torch.float64)
    cols = F.unfold(gT, 3, stride=2).view(2, cout, 9, R * R).transpose(1, 2).reshape(2, 9 * cout, -1)
    assert torch.allclose((md[:, :9 * cout] @ cols).view(2, cin, R, R), gx, atol=1e-12)


def _emulate_conv2d(x, groups, out_hw, cout, stride=1):
    """CPU restatement of mia_conv2d's group semantics (include/miattack.h) on NHWC fp64."""
    N, H, W, Cin = x.shape
    y = torch.zeros(N, out_hw[0], out_hw[1], cout, dtype=torch.float64)
    for g in groups:
        kh, kw = g["kh"], g["kw"]
        py, px = g.get("pad", (0, 0))
        ay, ax = g.get("a", (1, 1))
        by, bx = g.get("b", (0, 0))
        wm = g["w"].double()[:, :kh * kw * Cin].reshape(cout, kh, kw, Cin)
        for i in range(g["ho"]):
            for j in range(g["wo"]):
                acc = torch.zeros(N, cout, dtype=torch.float64)
                for ty in range(kh):
                    for tx in range(kw):
                        yy, xx = stride * i + ty - py, stride * j + tx - px
                        if 0 <= yy < H and 0 <= xx < W:
                            acc += x[:, yy, xx, :] @ wm[:, ty, tx, :].t()
                y[:, ay * i + by, ax * j + bx, :] = acc
    return y


@pytest.mark.parametrize("H", [8, 7, 2, 1])
def test_stride2_dgrad_phase_layout_is_the_adjoint(H):
    """layouts.s2_dgrad_phases + e4e._phase_groups (the 4-phase sub-pixel input gradient of a
    stride-2, pad-1 3×3 conv) equal autograd of F.conv2d, by a CPU emulation of the kernel's
    group semantics — including odd sizes and the 2→1 / 1→1 tail of a GradualStyleBlock."""
    import torch.nn.functional as F
    from gfa_amd import e4e, layouts
    g = torch.Generator().manual_seed(0)
    cin, cout = 3, 5
    w = torch.randn(cout, cin, 3, 3, generator=g, dtype=torch.float64)
    x = torch.randn(2, cin, H, H, generator=g, dtype=torch.float64, requires_grad=True)
    y = F.conv2d(x, w, stride=2, padding=1)
    gy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    (gx,) = torch.autograd.grad(y, x, gy)
    groups = e4e._phase_groups(layouts.s2_dgrad_phases(w, torch.float32), H)
    got = _emulate_conv2d(gy.permute(0, 2, 3, 1), groups, (H, H), cin)
    assert torch.allclose(got.permute(0, 3, 1, 2), gx, atol=1e-5)
    # the forward through the same emulation (fwd_matrix layout, stride 2)
    ho = (H - 1) // 2 + 1
    fwd = _emulate_conv2d(x.detach().permute(0, 2, 3, 1),
                          [dict(w=layouts.fwd_matrix(w, torch.float64), kh=3, kw=3, pad=(1, 1),
                                ho=ho, wo=ho)], (ho, ho), cout, stride=2)
    assert torch.allclose(fwd.permute(0, 3, 1, 2), y.detach(), atol=1e-10)


@pytest.mark.parametrize("R", [2, 3])
def test_s2_dgrad_halo_packing_is_the_adjoint(R):
    """layouts.s2_dgrad_halo_matrix under the DG-mode semantics of the halo up-conv kernel
    (offsets +j over the UPCONV_HALO_STEPS table, output phase 1 − p) equals autograd of a
    stride-2 pad-1 conv — a CPU emulation of csrc/conv_upconv.hip's K-step loop."""
    import torch.nn.functional as F
    from gfa_amd import layouts
    g0 = torch.Generator().manual_seed(1)
    cin, cout, N = 64, 128, 2  # forward conv: cin → cout; the gradient runs cout (Cg) → cin (Cx)
    w = torch.randn(cout, cin, 3, 3, generator=g0, dtype=torch.float64)
    x = torch.randn(N, cin, 2 * R, 2 * R, generator=g0, dtype=torch.float64, requires_grad=True)
    y = F.conv2d(x, w, stride=2, padding=1)
    gy = torch.randn(y.shape, generator=g0, dtype=torch.float64)
    (gx,) = torch.autograd.grad(y, x, gy)
    pk = layouts.s2_dgrad_halo_matrix(w, torch.float64)  # (Cg/64, 5, 2, Cx, 64)
    g = torch.zeros(N, R + 1, R + 1, cout, dtype=torch.float64)
    g[:, :R, :R] = gy.permute(0, 2, 3, 1)
    acc = torch.zeros(4, N, R, R, cin, dtype=torch.float64)
    for st, ((jy, jx), phases) in enumerate(layouts.UPCONV_HALO_STEPS):
        gs = g[:, jy:jy + R, jx:jx + R]
        for slot, ph in enumerate(phases):
            if ph is None:
                continue
            wm = pk[:, st, slot].permute(1, 0, 2).reshape(cin, cout)  # [Cx][Cg]
            acc[ph] += gs @ wm.t()
    out = torch.zeros(N, 2 * R, 2 * R, cin, dtype=torch.float64)
    for ph in range(4):
        py, px = ph >> 1, ph & 1
        out[:, 1 - py::2, 1 - px::2] = acc[ph]
    assert torch.allclose(out.permute(0, 3, 1, 2), gx, atol=1e-9)


def test_upconv_halo_packing_fp32_rows():
    """fp32 operand rows hold 32 channels (128 B): the packed halo up-conv weights are
    (Cin/32, 5, 2, Cout, 32) and carry the same entries as the 64-channel packing."""
    from gfa_amd import layouts
    w = torch.randn(64, 128, 3, 3, generator=torch.Generator().manual_seed(2), dtype=torch.float64)
    p32 = layouts.upconv_halo_matrix(w, torch.float32)
    p64 = layouts.upconv_halo_matrix(w, torch.float64)
    assert tuple(p32.shape) == (4, 5, 2, 64, 32) and tuple(p64.shape) == (2, 5, 2, 64, 64)
    a = p32.double().permute(2, 1, 3, 0, 4).reshape(2, 5, 64, 128)
    b = p64.permute(2, 1, 3, 0, 4).reshape(2, 5, 64, 128)
    assert torch.allclose(a, b.float().double())


def test_psp_checkpoint_split(tmp_path):
    """A pSp/e4e checkpoint (state_dict with encoder.* / decoder.* keys, latent_avg, opts) saved
    by torch.save loads with weights_only=True and splits into the generator and e4e dicts."""
    from gfa_amd import networks
    from gfa_amd.weights import make_e4e_weights, make_generator_weights
    gp = make_generator_weights(32, seed=0)
    ep = make_e4e_weights(32, seed=1)
    sd = {f"decoder.{k}": v for k, v in gp.items()}
    sd.update({f"encoder.{k}": v for k, v in ep.items() if torch.is_tensor(v) and k != "latent_avg"})
    sd["encoder.input_layer.1.num_batches_tracked"] = torch.tensor(5)
    path = tmp_path / "e4e_test.pt"
    torch.save({"state_dict": sd, "latent_avg": ep["latent_avg"],
                "opts": {"stylegan_size": 32, "start_from_latent_avg": True}}, path)
    dec, enc, opts = networks.psp_params_from_checkpoint(str(path))
    assert set(dec) == set(gp) and opts["stylegan_size"] == 32
    assert enc["kind"] == "e4e" and torch.equal(enc["latent_avg"], ep["latent_avg"])
    assert torch.equal(enc["body.3.shortcut_layer.0.weight"], ep["body.3.shortcut_layer.0.weight"])
    with pytest.raises(ValueError):
        networks.psp_params_from_checkpoint({"state_dict": {}, "latent_avg": ep["latent_avg"]})


def test_records_round_trip_and_grid_formats(tmp_path):
    """§8(f)-4 on-disk formats (gfa_amd.records): the attack_main2.py:1097-1111 torch.save dumps
    round-trip through weights_only loads; make_grid / save_image follow torchvision's layout and
    quantisation; the grid reload cuts the reference's tiles (interpolation.py:1386-1394)."""
    import torch
    from gfa_amd import records
    g = torch.Generator().manual_seed(0)
    adv = [torch.rand(2, 3, 8, 8, generator=g) * 2 - 1 for _ in range(3)]
    ben = [torch.rand(2, 3, 8, 8, generator=g) * 2 - 1 for _ in range(3)]
    loss = [torch.rand(2, generator=g) for _ in range(3)]
    paths = records.save_records(tmp_path / "adv", tmp_path / "benign", all_adv_inputs=adv,
                                 all_inputs=ben, all_adv_rec_loss=loss, all_rec_loss=loss)
    assert sorted(os.path.basename(p) for p in paths.values()) == sorted(
        ["all_adv_inputs.npz", "all_inputs.npz", "all_adv_rec_loss.npz", "all_rec_loss.npz"])
    r = records.load_records(tmp_path / "adv")
    assert torch.equal(r["all_adv_inputs"], torch.cat(adv)) and r["all_adv_rec_loss"].shape == (6,)
    # make_grid geometry: 10 tiles of 8², nrow 8 → 2 rows; 2-pixel separators, zero padding
    x = torch.rand(10, 3, 8, 8, generator=g)
    grid = records.make_grid(x)
    assert grid.shape == (3, 2 * 10 + 2, 8 * 10 + 2)
    assert torch.equal(grid[:, 2:10, 12:20], x[1]) and torch.equal(grid[:, 12:20, 2:10], x[8])
    assert grid[:, :2].abs().sum() == 0 and grid[:, 10:12].abs().sum() == 0
    tiles = records.grid_tiles(grid, 10, 8)
    assert all(torch.equal(t[0], x[k]) for k, t in enumerate(tiles))
    assert torch.equal(records.make_grid(x[:1]), x[0])
    # save_image → PNG (lossless) → reload: the quantised grid, mapped to [-1, 1]
    p = records.save_image(x[:5], str(tmp_path / "grid.png"))
    back = records.load_image_tensor(p)
    q = torch.from_numpy(records.to_uint8_hwc(records.make_grid(x[:5]))).permute(2, 0, 1)
    assert torch.equal(back, (q.float() / 255 - 0.5) / 0.5)
    ref_t = records.reference_tiles(back, 5, 8)
    assert torch.equal(ref_t[0], records.grid_tiles(back, 5, 8)[0])  # offset quirk: tile 0 exact
    assert torch.equal(ref_t[1][0], back[:, 2:10, 10:18])
    # per-image JPEG names (attack_main2.py:164-171)
    assert os.path.basename(records.save_image_idx(x[0] * 2 - 1, str(tmp_path), 7)) == "00007.jpg"


def test_split_f32_is_exact():
    """layouts.split_f32 (the pre-split weights of the split-once fp32 halo kernel): unpacking the
    [hi×4 | mid×4] quads and the lo plane gives hi + mid + lo == w exactly, each term a bf16
    value, for normal, tiny, negative and zero weights."""
    import torch
    from gfa_amd import layouts
    g = torch.Generator().manual_seed(0)
    w = torch.randn(8, 64, generator=g) * torch.logspace(-30, 3, 64)[None, :]
    w[0, :4] = torch.tensor([0.0, -0.0, 1.0, -3.1415927])
    sp = layouts.split_f32(w)
    cout, kpad = w.shape
    words = sp.view(torch.int32).to(torch.int64) & 0xFFFFFFFF
    hm = words[:cout * kpad].reshape(cout, kpad // 4, 4)
    lw = words[cout * kpad:].reshape(cout, kpad // 4, 2)

    def halves(x):  # int64 words → (low16, high16) as fp32 values of bf16 fields
        lo16, hi16 = x & 0xFFFF, x >> 16
        f = lambda h: (h << 16).to(torch.int32).view(torch.float32).double()  # noqa: E731
        return f(lo16), f(hi16)

    parts = []
    for src in (hm[..., 0:2], hm[..., 2:4], lw):
        a0, a1 = halves(src[..., 0])
        a2, a3 = halves(src[..., 1])
        parts.append(torch.stack([a0, a1, a2, a3], -1).reshape(cout, kpad))
    h, m, l = parts
    assert torch.equal(h + m + l, w.double())
    assert (h.abs() >= m.abs()).all() and (m.abs() >= l.abs()).all()


def test_make_grid_geometry_matches_reference_files():
    """records.make_grid lays tiles out as the reference's own saved grids
    (/root/reference/images/*.jpg, recorded by oracle/gen_golden_grids.py as size + per-column /
    per-row mean brightness): 5 tiles of 1024² at padding 2 → 5132 × 1028, the 6-image partial
    fusion sweep → 6158 × 1028, single images unpadded; every padding column / row of make_grid is
    a black stripe in the reference's file and every tile column / row is not."""
    import numpy as np
    from gfa_amd import records
    d = np.load(os.path.join(os.path.dirname(__file__), "golden", "reference_grids.npz"))
    files = sorted({k.rsplit("/", 1)[0] for k in d.files})
    assert len(files) >= 10
    for f in files:
        w, h = (int(v) for v in d[f"{f}/size"])
        n = 1 if (w, h) == (1024, 1024) else (w - 2) // 1026
        assert n in (1, 5, 6), (f, w, h)
        # a small stand-in tile of the same layout: make_grid's geometry scales with the tile
        grid = records.make_grid(torch.ones(n, 3, 1024, 1024), padding=2)
        assert tuple(grid.shape) == (3, h, w), (f, tuple(grid.shape))
        if n == 1:
            continue
        col_is_pad = (grid[0].sum(0) == 0).numpy()
        row_is_pad = (grid[0].sum(1) == 0).numpy()
        col, row = d[f"{f}/col"], d[f"{f}/row"]
        assert col[col_is_pad].max() < 12 and col[~col_is_pad].min() > 20, f
        assert row[row_is_pad].max() < 12 and row[~row_is_pad].min() > 20, f


def test_host_code_under_address_and_ub_sanitizers():
    """the library's host code (C ABI validation, error-string state, tuning table,
    scratch bookkeeping) compiled with -Xarch_host -fsanitize=address,undefined and driven by
    tools/asan/host_abi_check.cpp through the public entry points, valid and invalid arguments
    (no kernel launch). First run builds it (make asan, ≈ 1.5 min on 8 cores)."""
    import shutil
    import subprocess
    if shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"):
        pytest.skip("no hipcc")
    csrc = os.path.join(ROOT, "adversarial-attacks-on-gan-based-image-fusion_amd", "csrc")
    jobs = str(min(8, os.cpu_count() or 1))
    b = subprocess.run(["make", "-C", csrc, "-j", jobs, "asan"], stdout=subprocess.PIPE,
                       stderr=subprocess.STDOUT, text=True, timeout=900)
    assert b.returncode == 0, b.stdout[-3000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([os.path.join(csrc, "build", "asan_host_abi_check")], env=env,
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=300)
    assert r.returncode == 0 and "host ABI checks: ok" in r.stdout, r.stdout[-3000:]
