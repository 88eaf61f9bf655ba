# round 3: cfg3 (PGD-40, 1024², bf16) and cfg5 (C&W-L2, 1024², fp16; reference early stop and the
# labelled fixed-20-iteration timing) bench lines + the 1024² bf16 per-layer table
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u bench.py --size 1024 --pgd-steps 40 --dtype bf16 --batch 32 --no-cpu-baseline > gpurun_out/bench_cfg3.log 2> gpurun_out/bench_cfg3.err && echo cfg3-ok && tail -1 gpurun_out/bench_cfg3.log | cut -c1-300 &&
timeout -k 10 500 python -u bench.py --size 1024 --pgd-steps 20 --dtype fp16 --batch 32 --norm l2_cw --no-cpu-baseline > gpurun_out/bench_cfg5.log 2> gpurun_out/bench_cfg5.err && echo cfg5-ok && tail -1 gpurun_out/bench_cfg5.log | cut -c1-300 &&
timeout -k 10 500 python -u bench.py --size 1024 --pgd-steps 20 --dtype fp16 --batch 32 --norm l2_cw --cw-fixed --no-cpu-baseline > gpurun_out/bench_cfg5_fixed.log 2> gpurun_out/bench_cfg5_fixed.err && echo cfg5-fixed-ok && tail -1 gpurun_out/bench_cfg5_fixed.log | cut -c1-300 &&
timeout -k 10 300 python -u tools/layer_table.py --size 1024 --dtype bf16 --batch 32 --pgd-steps 4 --top 40 > gpurun_out/layers1024.log 2>&1 && echo layers-ok
