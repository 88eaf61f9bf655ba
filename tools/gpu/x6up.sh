# split-once fp32 up-conv / stride-2 adjoint halo kernels: parity + timings + bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_e4e.py -m gpu -q -rA -k "float32" --timeout 300 --timeout-method thread > gpurun_out/x6up_tests.log 2>&1; echo tests-rc=$?; grep -E "FAILED|passed|failed|max-abs err" gpurun_out/x6up_tests.log | tail -12
timeout -k 10 300 python -u tools/conv_ab.py --dtype fp32 --batch 64 --iters 3 --only "up " MIA_CONV_X6=1,0 > gpurun_out/x6up_ab.log 2>&1 && cat gpurun_out/x6up_ab.log &&
bash tools/gpu/bench1.sh > gpurun_out/x6up_bench.log 2>&1; head -3 gpurun_out/x6up_bench.log; grep -E "s2_dgrad|upconv" gpurun_out/b1_layers.log | head -8
