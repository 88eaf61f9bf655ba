set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "register_epilogue or halo_and_generic or style_head" > gpurun_out/t_wres2.log 2>&1 && echo tests-ok &&
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_e4e.py > gpurun_out/t_e4e.log 2>&1 && echo e4e-ok &&
timeout -k 10 300 python -u tools/conv_ab.py --iters 10 --only "64→64" MIA_CONV_WRES=1 > gpurun_out/ab_wres2.log 2>&1 && echo ab-ok
