# round 5: wres128 dgrad variant — kernel tests, the fp16 layer table on/off, the fp16 oracle test
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -v -s --timeout 120 --timeout-method thread -k "wres128 or per_image_weights or modconv_bwd" > gpurun_out/wres128_test.log 2>&1 && echo tests-ok &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_lowp_oracle.py -x -v -s --timeout 300 --timeout-method thread -k "float16-256" > gpurun_out/lowp_fp16.log 2>&1 && echo lowp-ok &&
env MIA_HEAD_STREAMS=1 MIA_CONV_WRES128=1 timeout -k 10 400 python -u tools/layer_table.py --dtype fp16 --top 60 > gpurun_out/layers_fp16_w128_on.log 2>&1 &&
env MIA_HEAD_STREAMS=1 MIA_CONV_WRES128=0 timeout -k 10 400 python -u tools/layer_table.py --dtype fp16 --top 60 > gpurun_out/layers_fp16_w128_off.log 2>&1 && echo layers-ok
# the VGG cascade per layer on the product routing (verdict r04 item 6): trace + PMC passes
bash tools/profile_vgg.sh > gpurun_out/profile_vgg.log 2>&1 && echo vgg-ok
