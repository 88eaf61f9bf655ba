# round 3: parity tests with printed residuals, the cfg2 determinism / batch-invariance test,
# VGG golden residuals
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py "tests/test_gpu_configs.py::test_cfg2_pgd10_batch32_fp32" "tests/test_gpu_networks.py::test_vgg_taps_and_grad_vs_reference_golden" -v -s --timeout 300 --timeout-method thread > gpurun_out/r03_det.log 2>&1; grep -E "PASS|FAIL|^E |rel |norm|differ|L0|stable|passed|failed" gpurun_out/r03_det.log | tail -40
