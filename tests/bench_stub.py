"""CPU stand-in for pgd.AttackEngine, used by the gloo tests of bench.py's multi-rank leg (in
process via ``bench.run_leg(make_engine=…)`` and through ``bench.py --device cpu
--engine-factory bench_stub:make_engine``). Test infrastructure only."""
import time
import types

import torch


class StubEngine:
    """An elementwise 'attack' with a rank-dependent delay (so the max over ranks is visible), the
    engine's one loss-scale status round per run when given a group, and the flop attributes
    bench.py reports."""

    def __init__(self, rank):
        import os
        self.rank = rank
        pid_dir = os.environ.get("STUB_PID_DIR")
        if pid_dir:  # test_bench_parent_sigkill_ends_ranks: which processes must not outlive it
            with open(os.path.join(pid_dir, f"rank{rank}.pid"), "w") as f:
                f.write(f"{os.getpid()} {os.getppid()}\n")
        self.sleep = float(os.environ.get("STUB_SLEEP_S", "0"))
        self.status_rounds = 0
        self.G = types.SimpleNamespace(flops_fwd_per_image=10.0)
        self.V = types.SimpleNamespace(flops_fwd_per_image=1.0)
        self.E = types.SimpleNamespace(flops_fwd_per_image=3.0)

    def run(self, x0, t, steps, eps, alpha, group=None):
        time.sleep(self.sleep or 0.05 * (1 + self.rank))
        if group is not None:
            import gfa_import  # noqa: F401
            from gfa_amd import pgd
            assert pgd.rescale_consensus(pgd.RUN_OK, group) == pgd.RUN_OK
            self.status_rounds += 1
        return torch.clamp(x0 + 2 * eps * torch.sign(t - x0), -1.0, 1.0)


def make_engine(args, dtype, dev):
    import os
    return StubEngine(int(os.environ.get("RANK", "0")))
