# 32-channel halo up-conv tile: parity, then the 1024² bf16 layer table
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "upconv_halo_fwd" --timeout 200 --timeout-method thread > gpurun_out/up32_tests.log 2>&1; echo tests-rc=$?; tail -2 gpurun_out/up32_tests.log
bash tools/gpu/layers1024.sh && head -12 gpurun_out/layers1024.log | cut -c1-110
