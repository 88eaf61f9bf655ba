"""HBM write / read / copy bandwidth of plain torch kernels at the thin layers' tensor sizes (GPU,
tuning aid): the yardstick for the write-bound VGG conv1_1 / e4e input-layer forwards."""
import torch

dev = torch.device("cuda:0")
for nbytes in (1 << 30, 2 << 30):
    y = torch.empty(nbytes // 2, dtype=torch.float16, device=dev)
    x = torch.empty_like(y).normal_()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for name, fn, traffic in (("fill (write)", lambda: y.fill_(1.0), nbytes),
                              ("sum (read)", lambda: x.sum(), nbytes),
                              ("copy", lambda: y.copy_(x), 2 * nbytes)):
        fn()
        torch.cuda.synchronize()
        e0.record()
        for _ in range(10):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 10
        print(f"{nbytes / 2**30:.0f} GiB {name:14s} {ms * 1e3:8.1f} us  {traffic / ms / 1e9:6.2f} TB/s",
              flush=True)
    del x, y
