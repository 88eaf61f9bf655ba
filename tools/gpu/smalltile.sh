set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "style_head_shapes or large_m or bias_relu" > gpurun_out/t_small.log 2>&1 && echo tests-ok &&
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_e4e.py > gpurun_out/t_e4e.log 2>&1 && echo e4e-ok &&
timeout -k 10 300 python -u tools/conv_ab.py --iters 20 --only "head" MIA_CONV_SMALLTILE=512,1024 > gpurun_out/ab_small.log 2>&1 && echo ab-ok &&
bash tools/gpu/layers_ab.sh MIA_CONV_SMALLTILE=512,1024
