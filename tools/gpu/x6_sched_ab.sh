# fp32 x6 halo kernel: step hand-off by LDS stage counters (libmiattack_sched1.so, MIA_X6_SCHED=1)
# vs one block barrier per K-step (the default build): bitwise parity of the unrolled schedule
# with the rolled loop, then the per-layer fp32 tables of both builds
set -o pipefail
mkdir -p gpurun_out
MIA_LIB_VARIANT=sched1 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "x6_halo_variants_bitwise or fp32_arithmetic" > gpurun_out/sched1_tests.log 2>&1 && echo sched1-tests-ok && tail -1 gpurun_out/sched1_tests.log &&
timeout -k 10 300 python -u tools/layer_table.py --dtype fp32 --top 30 > gpurun_out/layers_base.log 2>&1 && echo base-ok &&
MIA_LIB_VARIANT=sched1 timeout -k 10 300 python -u tools/layer_table.py --dtype fp32 --top 30 > gpurun_out/layers_sched1.log 2>&1 && echo sched1-ok &&
head -14 gpurun_out/layers_base.log && head -14 gpurun_out/layers_sched1.log
