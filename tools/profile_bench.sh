#!/bin/bash
# rocprofv3 evidence for bench.py (run on the GPU box from the repo root):
#   1. kernel trace + stats of the default bench (warmup 1 + 2 timed steps = 3 steps in the trace)
#   2. FETCH_SIZE and 3. WRITE_SIZE in separate --pmc passes (MI355X_MICROARCH.md §HBM)
# Outputs land in gpurun_out/prof_*; profiles/summarize_rocprof.py turns them into profiles/.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
ARGS="--steps 2 --warmup 1 --no-cpu-baseline ${EXTRA:-}"  # EXTRA="--encoder e4e", TAG=_e4e
T=${TAG:-}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_trace$T \
  -o run -- python3 bench.py $ARGS > gpurun_out/prof_trace$T.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_fetch$T \
  -o run -- python3 bench.py $ARGS > gpurun_out/prof_fetch$T.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_write$T \
  -o run -- python3 bench.py $ARGS > gpurun_out/prof_write$T.log 2>&1
find gpurun_out/prof_trace$T gpurun_out/prof_fetch$T gpurun_out/prof_write$T -name "*.csv" | head -20
