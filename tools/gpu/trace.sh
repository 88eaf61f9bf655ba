# head-shape parity, then a kernel trace of the default bench (time split only)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "style_head_shapes" > gpurun_out/t_head.log 2>&1 && echo tests-ok &&
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_trace_now -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_trace_now.log 2>&1 && echo trace-ok
