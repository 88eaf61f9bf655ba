# 32-channel thin kernel: parity, A/B, cfg3 bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "thin32 or fused_backward_front or modconv" > gpurun_out/t_thin32.log 2>&1 && echo tests-ok &&
timeout -k 10 300 python -u tools/conv_ab.py --batch 32 --iters 5 --only "1024²" MIA_CONV_THIN32=0,1 > gpurun_out/ab_thin32.log 2>&1 && echo ab-ok &&
timeout -k 10 500 python -u bench.py --size 1024 --pgd-steps 40 --dtype bf16 --batch 32 --no-cpu-baseline > gpurun_out/bench_cfg3.log 2>&1 && echo cfg3-ok
