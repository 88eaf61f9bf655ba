#!/bin/bash
# rocprofv3 evidence for bench.py (run on the GPU box from the repo root):
#   1. kernel trace + stats of the bench (warmup 1 + 2 timed steps = 3 steps in the trace)
#   2. FETCH_SIZE and 3. WRITE_SIZE in separate --pmc passes (MI355X_MICROARCH.md §HBM)
#   4. MFMA busy cycles + GRBM_GUI_ACTIVE + LDS bank conflicts in a fourth pass
# Outputs land in gpurun_out/prof_*; profiles/summarize_rocprof.py turns them into profiles/.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
ARGS="--steps 2 --warmup 1 --no-cpu-baseline --lowp none ${EXTRA:-}"  # EXTRA="--dtype fp16"
T=${TAG:-}
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_trace$T \
  -o run -- python3 bench.py $ARGS > gpurun_out/prof_trace$T.log 2>&1
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_fetch$T \
  -o run -- python3 bench.py $ARGS > gpurun_out/prof_fetch$T.log 2>&1
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_write$T \
  -o run -- python3 bench.py $ARGS > gpurun_out/prof_write$T.log 2>&1
timeout -s KILL 400 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT \
  SQ_LDS_IDX_ACTIVE --output-format csv -d gpurun_out/prof_mfma$T \
  -o run -- python3 bench.py $ARGS > gpurun_out/prof_mfma$T.log 2>&1
find gpurun_out/prof_trace$T gpurun_out/prof_fetch$T gpurun_out/prof_write$T gpurun_out/prof_mfma$T -name "*.csv" | head -20
