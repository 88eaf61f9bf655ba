# round 4: the fp32 64-column x6 tile with two taps per K-step — bitwise tests, then the fp32
# per-layer table A/B (MIA_X6_UNR=1: one tap per step; 2: two)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "x6_halo_variants_bitwise or fp32_arithmetic" -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/tps_test.log 2>&1; tail -3 gpurun_out/tps_test.log; tail -1 gpurun_out/tps_test.log | grep -q " passed" && ! grep -q FAILED gpurun_out/tps_test.log &&
DT=fp32 bash tools/gpu/layers_ab.sh MIA_X6_UNR=1,2 && head -30 gpurun_out/layers_a.log && echo ---- && head -30 gpurun_out/layers_b.log
