# round 4: the RCCL world-1 tests (nccl process group on the box's GPU) and smoke
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/dist.log 2>&1; tail -12 gpurun_out/dist.log; tail -1 gpurun_out/dist.log | grep -q " passed" && ! grep -q FAILED gpurun_out/dist.log &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo smoke-ok && tail -12 gpurun_out/smoke.log
