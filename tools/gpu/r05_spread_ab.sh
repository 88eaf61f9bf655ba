# round 5: weights-resident kernels with the next halo's DMA spread over the MFMA loop (default
# build) vs issued at the patch start (libmiattack_nospread.so), fp16 layer tables; correctness
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q -s --timeout 120 --timeout-method thread -k "wres128 and not 256" > gpurun_out/wres128_test.log 2>&1 && echo tests-ok &&
env MIA_HEAD_STREAMS=1 timeout -k 10 400 python -u tools/layer_table.py --dtype fp16 --top 60 > gpurun_out/layers_fp16_spread.log 2>&1 &&
env MIA_HEAD_STREAMS=1 MIA_LIB_VARIANT=nospread timeout -k 10 400 python -u tools/layer_table.py --dtype fp16 --top 60 > gpurun_out/layers_fp16_nospread.log 2>&1 &&
env MIA_HEAD_STREAMS=1 timeout -k 10 400 python -u tools/layer_table.py --dtype fp16 --top 60 > gpurun_out/layers_fp16_spread2.log 2>&1 && echo layers-ok
