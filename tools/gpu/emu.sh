# fp32 arithmetic A/B: parity of every fp32 test, one fp32 bench step per arithmetic
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -k "float32 or fp32 or f32 or networks or parity or e4e or configs or smoke" --timeout 300 --timeout-method thread > gpurun_out/emu_tests.log 2>&1; echo tests-rc=$? ; grep -E "FAILED|passed|failed" gpurun_out/emu_tests.log | tail -15; grep -E "max-abs err" gpurun_out/emu_tests.log
timeout -k 10 400 python -u bench.py --steps 1 --warmup 1 --lowp none --no-cpu-baseline > gpurun_out/emu_bench.log 2>&1 && echo bench-ok && tail -1 gpurun_out/emu_bench.log | cut -c1-300 &&
MIA_F32_ARITH=native timeout -k 10 400 python -u bench.py --steps 1 --warmup 1 --lowp none --no-cpu-baseline > gpurun_out/emu_bench_native.log 2>&1 && echo bench-native-ok && tail -1 gpurun_out/emu_bench_native.log | cut -c1-300
