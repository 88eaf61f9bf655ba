# fusion-evaluation metrics + StyleFusionSimple parity
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_metrics.py tests/test_gpu_networks.py -k "metrics or ssim or cal_ or style_fusion" > gpurun_out/t_metrics.log 2>&1 && echo metrics-ok
