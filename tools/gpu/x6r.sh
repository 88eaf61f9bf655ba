# x6 halo variants: fp32 parity, then timings variant 2 (weights in VGPRs) vs 1 (LDS ring)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -rA -k "float32 and (halo or bias_relu or modconv or sdot or tap or fp32_arith)" --timeout 300 --timeout-method thread > gpurun_out/x6r_tests.log 2>&1; echo tests-rc=$?; grep -E "FAILED|passed|failed|max-abs err" gpurun_out/x6r_tests.log | tail -12
timeout -k 10 300 python -u tools/conv_ab.py --dtype fp32 --batch 64 --iters 3 --only "${ONLY:-mod 256²|mod 128²|mod 64²|vgg 128² 128|vgg 64² 256|vgg 32²|dgrad+sdot 256²|dgrad+tap 64²|e4e prelu 64²|e4e acc 32²}" MIA_X6_VARIANT=2,1 > gpurun_out/x6r_ab.log 2>&1 && cat gpurun_out/x6r_ab.log
