# X6B tile with the register epilogues (fp32 up-conv adjoints + head convs): parity, layer table
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_e4e.py tests/test_gpu_networks.py -m gpu -x -q -k "front or bab or style_head or upconv or dgrad or stylegan or generator" --timeout 200 --timeout-method thread > gpurun_out/x6epi_tests.log 2>&1; echo tests-rc=$?; tail -3 gpurun_out/x6epi_tests.log
env MIA_HEAD_STREAMS=1 timeout -k 10 400 python -u tools/layer_table.py --dtype fp32 --top 100 > gpurun_out/layers_f32e.log 2>&1 && echo layers-ok && grep -E "step|upconv_dgrad|s2 g1 k3|conv2d 32x32 512->512" gpurun_out/layers_f32e.log
