# round 5: the per-image weight pass (mia_modulate_weights, 2-D grid + styles in LDS): its tests,
# then the fp16 layer table
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -s --timeout 120 --timeout-method thread -k "per_image_weights or wres128_modconv" > gpurun_out/wmod_test.log 2>&1 && echo tests-ok &&
env MIA_HEAD_STREAMS=1 timeout -k 10 400 python -u tools/layer_table.py --dtype fp16 --top 60 > gpurun_out/layers_fp16_wmod2.log 2>&1 && echo layers-ok
