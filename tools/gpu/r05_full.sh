# round 5: GPU suite (incl. the multi-rank real-engine tests), then the default bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1 && echo tests-ok && tail -1 gpurun_out/gputest.log &&
timeout -k 10 600 python -u bench.py > gpurun_out/bench.log 2>gpurun_out/bench.err && echo bench-ok && tail -1 gpurun_out/bench.log | cut -c1-400
