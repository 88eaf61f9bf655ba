# round-3 evidence part A: GPU suite, smoke, default bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1 && echo tests-ok && tail -1 gpurun_out/gputest.log &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo smoke-ok &&
timeout -k 10 600 python -u bench.py > gpurun_out/bench.log 2> gpurun_out/bench.err && echo bench-ok && tail -1 gpurun_out/bench.log | cut -c1-200
