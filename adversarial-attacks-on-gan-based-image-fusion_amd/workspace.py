"""Named, shape-stable device buffers reused across attack steps (no per-step allocation, so a
step can later be captured into a HIP graph)."""
import torch


class Workspace:
    def __init__(self, device):
        self.device = torch.device(device)
        self._bufs = {}
        # objects derived from this workspace's buffers (e.g. the e4e GemmPlans, which hold
        # pointers into them): they live and die with the workspace, never with the network
        self.cache = {}

    def get(self, name, shape, dtype):
        shape = tuple(int(s) for s in shape)
        t = self._bufs.get(name)
        if t is None or tuple(t.shape) != shape or t.dtype != dtype:
            t = torch.empty(shape, dtype=dtype, device=self.device)
            self._bufs[name] = t
        return t

    def nbytes(self):
        return sum(t.numel() * t.element_size() for t in self._bufs.values())

    def clear(self):
        self._bufs.clear()
        self.cache.clear()
