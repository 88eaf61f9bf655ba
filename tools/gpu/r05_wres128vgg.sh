# round 5: conv_wres128 on the VGG conv2_2 launches (BIAS|RELU forward, MASK input gradient):
# kernel tests, the VGG golden / network tests, then fp16 layer tables with the kernel on / off
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q -s --timeout 120 --timeout-method thread -k "wres128" > gpurun_out/wres128vgg_test.log 2>&1 && echo tests-ok && tail -1 gpurun_out/wres128vgg_test.log &&
timeout -k 10 500 python -u -m pytest tests/test_gpu_networks.py tests/test_gpu_e4e.py -x -q --timeout 200 --timeout-method thread > gpurun_out/wres128vgg_net.log 2>&1 && echo net-ok && tail -1 gpurun_out/wres128vgg_net.log &&
for t in 1 0; do env MIA_HEAD_STREAMS=1 MIA_CONV_WRES128=$t timeout -k 10 400 python -u tools/layer_table.py --dtype fp16 --top 60 > gpurun_out/layers_fp16_w128vgg$t.log 2>&1 || exit 1; grep -E "^step|128x128 128->128|256x256 128->128|64x64 128->128" gpurun_out/layers_fp16_w128vgg$t.log; done && echo layers-ok
