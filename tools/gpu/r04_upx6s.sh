# round 4: the two-blocks-per-CU up-conv form — bitwise / fp64 tests, then the fp32 per-layer
# table A/B (MIA_UPCONV_X6S=0,1)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_e4e.py -k "upconv or s2_dgrad or fp32_arithmetic" -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/upx6s_test.log 2>&1; tail -3 gpurun_out/upx6s_test.log; grep -E "^E  |FAILED" gpurun_out/upx6s_test.log | head; tail -1 gpurun_out/upx6s_test.log | grep -q " passed" && ! grep -q FAILED gpurun_out/upx6s_test.log &&
DT=fp32 bash tools/gpu/layers_ab.sh MIA_UPCONV_X6S=0,1 && grep -E "step|upconv|s2_dgrad" gpurun_out/layers_a.log | head -16 && echo ---- && grep -E "step|upconv|s2_dgrad" gpurun_out/layers_b.log | head -16
