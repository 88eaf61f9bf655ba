# split-once up-conv forward + stride-2 dgrad: parity, then the fp32 layer table
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_e4e.py -m gpu -x -q -k "upconv or s2_dgrad" --timeout 200 --timeout-method thread > gpurun_out/upx6_tests.log 2>&1; echo tests-rc=$?; tail -3 gpurun_out/upx6_tests.log
env MIA_HEAD_STREAMS=1 timeout -k 10 400 python -u tools/layer_table.py --dtype fp32 --top 100 > gpurun_out/layers_f32d.log 2>&1 && echo layers-ok && grep -E "step|s2_dgrad|upconv_fwd" gpurun_out/layers_f32d.log
