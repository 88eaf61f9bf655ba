#!/bin/bash
# A/B of non-temporal conv epilogue stores (variant build MIA_EPI_NT) over the whole bench step:
# layer tables at fp16 and fp32, default library then the variant, then default again.
set -o pipefail
mkdir -p gpurun_out
for d in fp16 fp32; do
  for v in "" epint ""; do
    MIA_HEAD_STREAMS=1 MIA_LIB_VARIANT=$v timeout -k 10 400 python -u tools/layer_table.py --dtype $d --top 40 > gpurun_out/layers_${d}_epint_${v:-def}.log 2>&1 || exit 1
    echo "== $d ${v:-def}"; grep -E "^step|^modulated" gpurun_out/layers_${d}_epint_${v:-def}.log
  done
done
