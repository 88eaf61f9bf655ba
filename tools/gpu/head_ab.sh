# deep-ring parity + A/B on the e4e style-head shapes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "style_head_shapes" > gpurun_out/t_deep.log 2>&1 && echo tests-ok &&
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_e4e.py > gpurun_out/t_e4e.log 2>&1 && echo e4e-ok &&
timeout -k 10 300 python -u tools/conv_ab.py --iters 20 --only "head" MIA_CONV_TILE=0,2 > gpurun_out/ab_deep.log 2>&1 && echo ab-ok
