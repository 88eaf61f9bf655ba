# fp32 kernel-level parity under the bf16-split arithmetic (no -x: the failure pattern matters)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_e4e.py -m gpu -q -k "float32" --timeout 300 --timeout-method thread > gpurun_out/emu_ktests.log 2>&1; echo tests-rc=$? ; tail -40 gpurun_out/emu_ktests.log | grep -E "FAILED|passed|failed"
