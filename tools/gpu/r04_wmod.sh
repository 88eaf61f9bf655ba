# round 4: per-image modulated weights for the fp16 / bf16 StyledConv forward — kernel tests, then
# the fp16 per-layer table A/B (MIA_G_WMOD_RES=0: LDS-modulated halo; 128: per-image weights)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "per_image_weights or modconv_fwd" -m gpu -v -s --timeout 200 --timeout-method thread > gpurun_out/wmod_test.log 2>&1; grep -E "per-image|passed|failed|Error" gpurun_out/wmod_test.log | head -20; tail -1 gpurun_out/wmod_test.log | grep -q " passed" && ! grep -q FAILED gpurun_out/wmod_test.log &&
DT=fp16 bash tools/gpu/layers_ab.sh MIA_G_WMOD_RES=0,128 && grep -E "mod|step" gpurun_out/layers_a.log | head -12 && echo ---- && grep -E "mod|step" gpurun_out/layers_b.log | head -12
