# round 4: the two-blocks-per-CU 128-column x6 tile (half-K weight stages) — bitwise tests, then
# the fp32 per-layer table A/B (MIA_X6_128S=0 vs every Cin)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -k "x6_128_two_block or x6_halo_variants_bitwise" -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/x6h_test.log 2>&1; tail -3 gpurun_out/x6h_test.log; grep -E "^E  |FAILED" gpurun_out/x6h_test.log | head -20; tail -1 gpurun_out/x6h_test.log | grep -q " passed" && ! grep -q FAILED gpurun_out/x6h_test.log &&
DT=fp32 bash tools/gpu/layers_ab.sh MIA_X6_128S=0,4096 && head -45 gpurun_out/layers_a.log && echo ---- && head -45 gpurun_out/layers_b.log
