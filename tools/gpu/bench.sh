# default bench line only
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2>&1 && echo bench-ok && tail -1 gpurun_out/bench.log | cut -c1-200
