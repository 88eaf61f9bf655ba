# x6 halo kernel, taps unrolled with lane-constant fragment offsets (MIA_X6_UNR)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_e4e.py tests/test_gpu_networks.py tests/test_gpu_parity.py > gpurun_out/x6unr_tests.log 2>&1 &&
bash tools/gpu/layers_ab.sh MIA_X6_UNR=0,1 &&
timeout -k 10 300 python -u tools/probe/x6_stamps.py > gpurun_out/x6_stamps.log 2>&1
