import sys, os, torch
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import gfa_import  # noqa
from gpu_helpers import engine, seeded, grad_stats
cuda = torch.device("cuda:0")
for size, N, enc in ((256, 8, "e4e"), (256, 8, "linear"), (1024, 2, "e4e")):
    x0 = seeded(400, (N, 3, size, size)); t = seeded(401, (N, 3, size, size))
    x = (x0 + 0.02 * seeded(405, x0.shape)).clamp(-1, 1)
    e32, _ = engine(size, torch.float32, cuda, encoder=enc)
    e32.prepare(x0.to(cuda), t.to(cuda))
    g32 = e32.full_gradient(x.to(cuda)).cpu().double()
    gl = e32.ws.get("g.lat", (N, e32.G.n_latent, 512), torch.float32)
    print(size, N, enc, "fp32 |g| max", g32.abs().max().item(), "g_lat absmax", gl.abs().max().item(), flush=True)
    del e32; torch.cuda.empty_cache()
    for ls in (2.0**16, 2.0**12, 2.0**8, 2.0**4, 1.0):
        eng, _ = engine(size, torch.float16, cuda, encoder=enc)
        eng.loss_scale = ls
        eng.__init__(eng.E, eng.G, eng.V, loss_scale=ls)
        eng.prepare(x0.to(cuda), t.to(cuda))
        g = eng.full_gradient(x.to(cuda)).cpu().double()
        nan = (~torch.isfinite(g)).double().mean().item()
        gg = torch.nan_to_num(g)
        nrm, mx, agree = grad_stats(gg, g32)
        print(f"  fp16 ls=2^{int(torch.log2(torch.tensor(ls)))} nonfinite {nan:.4f} norm {nrm:.3f} agree {agree:.4f} zero {(g==0).double().mean().item():.4f}", flush=True)
        del eng; torch.cuda.empty_cache()
