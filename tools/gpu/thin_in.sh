# VGG / e4e input-layer thin kernels: parity and timing
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "thin" > gpurun_out/t_thin.log 2>&1 && echo tests-ok &&
timeout -k 10 300 python -u tools/conv_ab.py --iters 10 --only "thin" MIA_CONV_THIN=0,1 > gpurun_out/ab_thin.log 2>&1 && echo ab-ok
