set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_e4e.py tests/test_gpu_networks.py > gpurun_out/t_regepi.log 2>&1 && echo tests-ok &&
bash tools/gpu/layers_ab.sh MIA_EPI_PRERED=0,1
