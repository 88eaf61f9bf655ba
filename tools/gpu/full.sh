# full GPU check: parity suite, then the default bench line (round-end driver order)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest.log 2>&1 && echo tests-ok &&
timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2>&1 && echo bench-ok && tail -1 gpurun_out/bench.log
