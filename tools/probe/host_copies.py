"""Counts, during one warm fp32 attack step (default bench workload at a small batch), the calls
that move data through the host or re-split fp32 weights: layouts.split_f32 (a cache miss of
split_for) and torch Tensor.to / copy_ / clone issued from Python (GPU, diagnostic)."""
import collections
import os
import sys
import traceback

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import gfa_import  # noqa: E402,F401
from gfa_amd import layouts, pgd  # noqa: E402
from gfa_amd.e4e import E4EEncoder  # noqa: E402
from gfa_amd.stylegan2 import SynthesisNet  # noqa: E402
from gfa_amd.vgg import VGGNet  # noqa: E402
from gfa_amd.weights import make_generator_weights, make_vgg_weights  # noqa: E402

dev = torch.device("cuda:0")
T, S, B = torch.float32, 256, int(os.environ.get("B", "4"))
enc = E4EEncoder(bench.encoder_weights("e4e", S), S, dtype=T, device=dev)
eng = pgd.AttackEngine(enc, SynthesisNet(make_generator_weights(S, seed=0), S, dtype=T, device=dev),
                       VGGNet(make_vgg_weights(1234), dtype=T, device=dev))
g = torch.Generator().manual_seed(1000)
x0 = (torch.rand(B, 3, S, S, generator=g) * 2 - 1).to(dev)
tgt = (torch.rand(B, 3, S, S, generator=g) * 2 - 1).to(dev)
eng.run(x0, tgt, 2, 8 / 255, 2 / 255)
torch.cuda.synchronize()

sites = collections.Counter()
orig_split = layouts.split_f32


def split_spy(w):
    st = traceback.extract_stack(limit=6)[:-1]
    sites[("split_f32", tuple(f"{os.path.basename(f.filename)}:{f.lineno}" for f in st[-3:]),
           tuple(w.shape))] += 1
    return orig_split(w)


layouts.split_f32 = split_spy
for name in ("to", "copy_", "clone"):
    orig = getattr(torch.Tensor, name)

    def spy(self, *a, _orig=orig, _name=name, **k):
        st = traceback.extract_stack(limit=5)[:-1]
        if any("gfa_amd" in f.filename or "adversarial" in f.filename for f in st):
            sites[(_name, tuple(f"{os.path.basename(f.filename)}:{f.lineno}" for f in st[-2:]),
                   tuple(self.shape))] += 1
        return _orig(self, *a, **k)
    setattr(torch.Tensor, name, spy)

eng.run(x0, tgt, 2, 8 / 255, 2 / 255)
torch.cuda.synchronize()
print(f"batch {B}, 2 PGD iterations; call sites:")
for k, v in sites.most_common(40):
    print(f"{v:6d}  {k}")
