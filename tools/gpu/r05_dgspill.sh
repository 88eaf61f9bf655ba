# round 5: conv_wres128 input gradient with its epilogue lane terms recomputed per patch (no
# VGPR spills): kernel tests, then fp16 layer tables (default build twice around the probe)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "wres128" > gpurun_out/dgspill_test.log 2>&1 && echo tests-ok && tail -1 gpurun_out/dgspill_test.log &&
for v in "" noepi ""; do env MIA_HEAD_STREAMS=1 MIA_LIB_VARIANT=$v timeout -k 10 400 python -u tools/layer_table.py --dtype fp16 --top 60 > gpurun_out/layers_fp16_dgspill_${v:-base}.log 2>&1 || exit 1; grep -E "^step|256x256 128->128" gpurun_out/layers_fp16_dgspill_${v:-base}.log; done && echo ok
