# round 4: the cfg3 (PGD-40, 1024², bf16, 32 images) and cfg5 (C&W-L2, 1024², fp16, 32 images,
# reference early stop and fixed 20 iterations) bench lines of the final tree
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u bench.py --size 1024 --pgd-steps 40 --dtype bf16 --batch 32 --lowp none --no-cpu-baseline > gpurun_out/bench_cfg3.log 2>&1 && echo cfg3-ok && tail -1 gpurun_out/bench_cfg3.log | cut -c1-160 &&
timeout -k 10 500 python -u bench.py --size 1024 --pgd-steps 20 --dtype fp16 --batch 32 --norm l2_cw --lowp none --no-cpu-baseline --cw-fixed > gpurun_out/bench_cfg5f.log 2>&1 && echo cfg5-fixed-ok && tail -1 gpurun_out/bench_cfg5f.log | cut -c1-160
