# round 4: tests of the 64-column two-taps-per-step x6 tile and the merged style-head convs, then
# the fp32 per-layer table with both off (a) and both on (b, the defaults)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_e4e.py -k "x6_halo_variants_bitwise or merged_per_source or fp32_arithmetic or thin32" -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/ab2_test.log 2>&1; tail -3 gpurun_out/ab2_test.log; tail -1 gpurun_out/ab2_test.log | grep -q " passed" && ! grep -q FAILED gpurun_out/ab2_test.log &&
env MIA_X6_UNR=1 MIA_E4E_MERGE_HEADS=0 timeout -k 10 400 python -u tools/layer_table.py --dtype fp32 --top 80 > gpurun_out/layers_a.log 2>&1 &&
timeout -k 10 400 python -u tools/layer_table.py --dtype fp32 --top 80 > gpurun_out/layers_b.log 2>&1 && head -36 gpurun_out/layers_a.log && echo ---- && head -36 gpurun_out/layers_b.log
