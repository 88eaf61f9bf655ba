# X6B generic-kernel tiles: fp32 parity (kernels, e4e, networks), then isolated timings X6 on/off
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_e4e.py tests/test_gpu_networks.py tests/test_gpu_parity.py -m gpu -q -rA -k "float32 or fp32 or vs_oracle or parity or mask_for_mask or teacher" --timeout 300 --timeout-method thread > gpurun_out/x6b_tests.log 2>&1; echo tests-rc=$?; grep -E "FAILED|passed|failed|max-abs err|mask-for-mask" gpurun_out/x6b_tests.log | tail -20
timeout -k 10 300 python -u tools/conv_ab.py --dtype fp32 --batch 64 --iters 3 --only "${ONLY:-head s2|vgg 256² 64|dgrad+tap 256²|e4e prelu 256²|e4e acc 128²|e4e mask+slope 128²|dgrad 128²}" MIA_CONV_X6=1,0 > gpurun_out/x6b_ab.log 2>&1 && cat gpurun_out/x6b_ab.log
