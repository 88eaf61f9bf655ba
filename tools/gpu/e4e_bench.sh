# e4e encoder parity, then the default bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_e4e.py > gpurun_out/t_e4e.log 2>&1 && echo e4e-ok &&
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1 && echo bench-ok && tail -1 gpurun_out/bench.log | cut -c1-400
