# round-end evidence: GPU parity suite, the default bench line, rocprofv3 trace + PMC passes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest.log 2>&1 && echo tests-ok &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")" > gpurun_out/smoke.log 2>&1 && echo smoke-ok &&
timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2>&1 && echo bench-ok && tail -1 gpurun_out/bench.log | cut -c1-300 &&
TAG=_e4e bash tools/profile_bench.sh > gpurun_out/profile.log 2>&1 && echo profile-ok
