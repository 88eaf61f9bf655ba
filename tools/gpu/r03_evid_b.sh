# round-3 evidence part B: the default bench line, then rocprofv3 trace + PMC passes of the fp32
# headline (summarise with profiles/summarize_rocprof.py --bench-line)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py > gpurun_out/bench.log 2> gpurun_out/bench.err && echo bench-ok && tail -1 gpurun_out/bench.log | cut -c1-200 &&
TAG=_f32 bash tools/profile_bench.sh > gpurun_out/profile_f32.log 2>&1 && echo profile-f32-ok
