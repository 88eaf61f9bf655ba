# level-batched e4e style heads: batched-conv parity, the e4e + network suites, layer table, bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_e4e.py tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/heads_tests.log 2>&1; echo tests-rc=$?; tail -3 gpurun_out/heads_tests.log
timeout -k 10 400 python -u tools/layer_table.py --dtype fp32 --top 100 > gpurun_out/layers_f32f.log 2>&1 && echo layers-ok && grep -E "step|batched|s2 g1 k3|g4 k1" gpurun_out/layers_f32f.log
timeout -k 10 500 python -u bench.py --lowp none --no-cpu-baseline > gpurun_out/bench_heads.log 2>&1 && tail -1 gpurun_out/bench_heads.log | cut -c1-250
