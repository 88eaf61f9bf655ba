#!/bin/bash
# per-layer rocprofv3 evidence of the VGG cascade (tools/vgg_cascade.py): trace, FETCH_SIZE,
# WRITE_SIZE and MFMA-busy passes; tools/vgg_layers_summary.py joins them.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
A="--reps 2 ${VARGS:-}"
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/vgg_trace -o run -- python3 tools/vgg_cascade.py $A > gpurun_out/vgg_trace.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/vgg_fetch -o run -- python3 tools/vgg_cascade.py $A > gpurun_out/vgg_fetch.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/vgg_write -o run -- python3 tools/vgg_cascade.py $A > gpurun_out/vgg_write.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d gpurun_out/vgg_mfma -o run -- python3 tools/vgg_cascade.py $A > gpurun_out/vgg_mfma.log 2>&1
python3 tools/vgg_layers_summary.py --trace "$(find gpurun_out/vgg_trace -name '*kernel_trace.csv' | head -1)" \
  --fetch "$(find gpurun_out/vgg_fetch -name '*counter_collection.csv' | head -1)" \
  --write "$(find gpurun_out/vgg_write -name '*counter_collection.csv' | head -1)" \
  --mfma "$(find gpurun_out/vgg_mfma -name '*counter_collection.csv' | head -1)" \
  --out gpurun_out/vgg_layers ${SARGS:-}
