set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/layer_table.py --dtype fp32 --top 60 > gpurun_out/layers_a.log 2>&1 &&
MIA_LIB_VARIANT=nosplit timeout -k 10 400 python -u tools/layer_table.py --dtype fp32 --top 60 > gpurun_out/layers_b.log 2>&1; grep -E "step| s2 |upconv_dgrad|conv2d_batched" gpurun_out/layers_a.log; echo ----; grep -E "step| s2 |upconv_dgrad|conv2d_batched" gpurun_out/layers_b.log
