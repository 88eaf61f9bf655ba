# round 5 A/B on one box: inline-asm fragment reads with counted waits in the weights-resident
# kernels. default = both (conv_wres 4 ahead, conv_wres128 3 ahead); w64 = conv_wres compiler-
# scheduled; w0 = both compiler-scheduled (conv_wres128 1 ahead). fp16 layer tables, alternating.
set -o pipefail
mkdir -p gpurun_out
for v in "" w0 w64 "" w0; do env MIA_HEAD_STREAMS=1 MIA_LIB_VARIANT=$v timeout -k 10 400 python -u tools/layer_table.py --dtype fp16 --top 60 > gpurun_out/layers_fp16_ar_${v:-def}.log 2>&1 || exit 1; echo "== ${v:-def}"; grep -E "^step|64->64|128->128" gpurun_out/layers_fp16_ar_${v:-def}.log; done && echo ok
