set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "thin" > gpurun_out/t_thin.log 2>&1 && echo thin-ok &&
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_e4e.py > gpurun_out/t_e4e.log 2>&1 && echo e4e-ok &&
MIA_HEAD_STREAMS=1 timeout -k 10 300 python -u tools/layer_table.py --top 70 > gpurun_out/layers.log 2>&1 && echo layers-ok
