# Reproduce at commit 245ea98 (the MIA_X6_M32 variant was removed from the source after this A/B).
# round 6 A/B (verdict r05 item 2): the fp32 x6 halo kernel's 128-channel unrolled loop on
# v_mfma_f32_32x32x16_bf16 (libmiattack_m32.so: make variant VARIANT=m32 VARIANT_FLAGS=-DMIA_X6_M32=1)
# against the product library (16x16x32). First the variant's numerics (the x6 kernel tests and the
# fp32 split-arithmetic check under MIA_LIB_VARIANT=m32), then fp32 layer tables, alternating.
set -o pipefail
mkdir -p gpurun_out
MIA_LIB_VARIANT=m32 timeout -k 10 400 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "fp32_arith" > gpurun_out/r06_m32_tests.log 2>&1 || { tail -30 gpurun_out/r06_m32_tests.log; exit 1; }
MIA_LIB_VARIANT=m32 timeout -k 10 400 python -u -c "import __graft_entry__ as g; g.smoke()" >> gpurun_out/r06_m32_tests.log 2>&1 || { tail -30 gpurun_out/r06_m32_tests.log; exit 1; }
grep -E "halo:|passed|smoke|norm" gpurun_out/r06_m32_tests.log | head -20
for v in "" m32 "" m32; do env MIA_HEAD_STREAMS=1 MIA_LIB_VARIANT=$v timeout -k 10 400 python -u tools/layer_table.py --dtype fp32 --top 60 > gpurun_out/layers_fp32_m32_${v:-def}.log 2>&1 || exit 1; echo "== ${v:-def}"; head -4 gpurun_out/layers_fp32_m32_${v:-def}.log; grep "x6\|halo" gpurun_out/layers_fp32_m32_${v:-def}.log | head -12; done && echo ok
