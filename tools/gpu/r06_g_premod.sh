# round 6: fp32 4² / 8² StyledConvs with the input modulated once (MIA_G_PREMOD_RES=16, product)
# against the per-fragment modulated-input conv (MIA_G_PREMOD_RES=0): synthesis / attack-gradient
# tests, fp32 layer tables alternating
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_networks.py tests/test_gpu_parity.py -k "synthesis or upsampling or attack_gradient or pgd or objective" > gpurun_out/r06_gpm_tests.log 2>&1 || { tail -30 gpurun_out/r06_gpm_tests.log; exit 1; }
echo "== tests: $(tail -1 gpurun_out/r06_gpm_tests.log)"
for v in 0 16 0 16; do echo "== MIA_G_PREMOD_RES=$v"; MIA_G_PREMOD_RES=$v timeout -k 10 400 python -u tools/layer_table.py --dtype fp32 --top 400 > gpurun_out/r06_gpm_layers_$v.log 2>&1 || exit 1; grep "^step\|^conv3x3 4x4\|^conv3x3 8x8" gpurun_out/r06_gpm_layers_$v.log; done && echo ok
