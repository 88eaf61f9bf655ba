# round-2 parity tests (objective pin, mask-for-mask e4e, teacher-forced PGD, configs)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_networks.py -m gpu -v -s --timeout 300 --timeout-method thread ${K:+-k "$K"} > gpurun_out/t_parity.log 2>&1; echo "pytest rc=$?"
