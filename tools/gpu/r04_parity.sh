# round 4: RCCL world-1 tests, the bounded mask-forced parity tests (prints the flip audits),
# the VGG golden gradient, then smoke
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/dist.log 2>&1; tail -5 gpurun_out/dist.log; tail -1 gpurun_out/dist.log | grep -q " passed" && ! grep -q FAILED gpurun_out/dist.log &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_networks.py::test_vgg_taps_and_grad_vs_reference_golden tests/test_gpu_configs.py::test_cfg2_pgd10_batch32_fp32 -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/parity.log 2>&1; grep -E "forced flips|VGG golden|passed|failed|FAILED|Error" gpurun_out/parity.log | head -40;
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo smoke-ok; tail -12 gpurun_out/smoke.log
