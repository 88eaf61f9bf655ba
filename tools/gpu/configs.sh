# supplementary bench lines: BASELINE config #3 (PGD-40 1024² bf16) and #5 (C&W-L2 1024² fp16, 20 fixed iterations)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u bench.py --size 1024 --pgd-steps 40 --dtype bf16 --batch 32 --no-cpu-baseline > gpurun_out/bench_cfg3.log 2>&1 && echo cfg3-ok && tail -1 gpurun_out/bench_cfg3.log | cut -c1-200 &&
timeout -k 10 500 python -u bench.py --size 1024 --pgd-steps 20 --dtype fp16 --batch 32 --norm l2_cw --cw-fixed --no-cpu-baseline > gpurun_out/bench_cfg5.log 2>&1 && echo cfg5-ok && tail -1 gpurun_out/bench_cfg5.log | cut -c1-300
