import sys, os, collections, traceback
sys.path.insert(0, os.getcwd())
import torch
import gfa_import  # noqa
from gfa_amd import layouts, pgd
import bench
from gfa_amd.e4e import E4EEncoder
from gfa_amd.stylegan2 import SynthesisNet
from gfa_amd.vgg import VGGNet
from gfa_amd.weights import make_generator_weights, make_vgg_weights
calls = collections.Counter()
orig = layouts.split_f32
def counting(w):
    st = traceback.extract_stack(limit=4)
    calls[(tuple(w.shape), st[-3].filename.split('/')[-1] + ':' + str(st[-3].lineno))] += 1
    return orig(w)
layouts.split_f32 = counting
dev = torch.device("cuda:0")
S, B = 256, 4
T = torch.float32
enc = E4EEncoder(bench.encoder_weights("e4e", S), S, dtype=T, device=dev)
eng = pgd.AttackEngine(enc, SynthesisNet(make_generator_weights(S, seed=0), S, dtype=T, device=dev),
                       VGGNet(make_vgg_weights(1234), dtype=T, device=dev))
x0 = torch.rand(B, 3, S, S, device=dev) * 2 - 1
t = torch.rand(B, 3, S, S, device=dev) * 2 - 1
eng.run(x0, t, 2, 8 / 255, 2 / 255)
torch.cuda.synchronize()
print("after run 1:", sum(calls.values()))
calls.clear()
eng.run(x0, t, 3, 8 / 255, 2 / 255)
torch.cuda.synchronize()
print("after run 2 (3 iters):", sum(calls.values()))
for k, v in calls.most_common(20):
    print(v, k)
