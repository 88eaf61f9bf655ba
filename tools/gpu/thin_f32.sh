# fp32 VALU thin kernels: parity, then the fp32 per-layer table
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "thin_vgg" --timeout 120 --timeout-method thread > gpurun_out/thin_f32_tests.log 2>&1; echo tests-rc=$?; tail -3 gpurun_out/thin_f32_tests.log
env MIA_HEAD_STREAMS=1 timeout -k 10 400 python -u tools/layer_table.py --dtype fp32 --top 100 > gpurun_out/layers_f32b.log 2>&1 && echo layers-ok && grep -E "step|256x256 (8->64|64->8)" gpurun_out/layers_f32b.log
