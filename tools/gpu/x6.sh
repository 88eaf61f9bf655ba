# split-once fp32 halo kernel: fp32 kernel parity, then isolated timings x6 vs on-the-fly split
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_e4e.py -m gpu -q -rA -k "float32" --timeout 300 --timeout-method thread > gpurun_out/x6_tests.log 2>&1; echo tests-rc=$?; grep -E "FAILED|passed|failed|max-abs err" gpurun_out/x6_tests.log | tail -20
timeout -k 10 300 python -u tools/conv_ab.py --dtype fp32 --batch 64 --iters 3 --only "${ONLY:-mod 256²|mod 128²|mod 64²|vgg 128² 128|vgg 64² 256|vgg 32²|dgrad+sdot 256²|dgrad+tap 64²|e4e prelu 64²|e4e acc 32²|e4e mask+slope 32²}" MIA_CONV_X6=1,0 > gpurun_out/x6_ab.log 2>&1 && cat gpurun_out/x6_ab.log
