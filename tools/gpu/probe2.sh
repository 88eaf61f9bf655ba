# fp32 halo up-conv: targeted parity tests, then the fp32 bench step and layer table
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "upconv_halo or s2_dgrad_halo or e4e or attack_gradient or synthesis" > gpurun_out/t_probe2.log 2>&1 && echo tests-ok &&
timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --lowp none > gpurun_out/bench_fp32.log 2>&1 && echo bench-ok && tail -1 gpurun_out/bench_fp32.log | cut -c1-300 &&
MIA_HEAD_STREAMS=1 timeout -k 10 300 python -u tools/layer_table.py --dtype fp32 --pgd-steps 4 --top 80 > gpurun_out/layers_fp32.log 2>&1 && echo layers-ok
