# round 6: fp32 modulated-input generic launches of < 2048 128×128 tiles (the generator's 4² / 8²
# StyledConvs, the 4→8 / 8→16 up-convs and the up-conv edges) on 64×64 tiles
# (libmiattack_st2k.so, -DMIA_F32_PRO_SMALLTILE=2048) against 128×128: fp32 layer tables
# (tools/layer_table.py) alternating, the up-conv / generator tests on the variant
set -o pipefail
mkdir -p gpurun_out
MIA_LIB_VARIANT=st2k timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_networks.py -k "upconv or synthesis or upsampling or styled" > gpurun_out/r06_st2k_tests.log 2>&1 || { tail -30 gpurun_out/r06_st2k_tests.log; exit 1; }
echo "== tests st2k: $(tail -1 gpurun_out/r06_st2k_tests.log)"
for v in "" st2k "" st2k; do echo "== ${v:-prod}"; MIA_LIB_VARIANT=$v timeout -k 10 400 python -u tools/layer_table.py --dtype fp32 --top 400 > gpurun_out/r06_st2k_layers_${v:-prod}.log 2>&1 || exit 1; grep "^step\|^conv3x3 4x4\|^conv3x3 8x8\|upconv_fwd.* (128, 4,\|upconv_fwd.* (128, 8,\|mia_upconv_fwd " gpurun_out/r06_st2k_layers_${v:-prod}.log; done && echo ok
