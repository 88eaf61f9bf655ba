# round 4: the two-blocks-per-CU 64-channel x6 tile — bitwise tests, smoke's split arithmetic,
# then the fp32 per-layer table A/B (MIA_X6_64S=0,1)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "x6_halo_variants_bitwise or fp32_arithmetic" -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/x6s_test.log 2>&1; tail -3 gpurun_out/x6s_test.log; grep -E "^E  |FAILED" gpurun_out/x6s_test.log | head; tail -1 gpurun_out/x6s_test.log | grep -q " passed" && ! grep -q FAILED gpurun_out/x6s_test.log &&
DT=fp32 bash tools/gpu/layers_ab.sh MIA_X6_64S=0,1 && grep -E "step|64->64|64->128|128->64|tap" gpurun_out/layers_a.log | head -14 && echo ---- && grep -E "step|64->64|64->128|128->64|tap" gpurun_out/layers_b.log | head -14
