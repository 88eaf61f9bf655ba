# fp32 (reference precision) probe: one bench step and the per-layer conv table
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --dtype fp32 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bench_fp32.log 2>&1 && echo bench-ok && tail -1 gpurun_out/bench_fp32.log | cut -c1-400 &&
MIA_HEAD_STREAMS=1 timeout -k 10 400 python -u tools/layer_table.py --dtype fp32 --pgd-steps 4 --top 80 > gpurun_out/layers_fp32.log 2>&1 && echo layers-ok
