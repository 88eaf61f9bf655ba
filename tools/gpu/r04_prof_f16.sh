# round 4: rocprofv3 trace + FETCH/WRITE/MFMA-busy passes of the fp16 sub-record (tools/profile_bench.sh)
set -o pipefail
mkdir -p gpurun_out
TAG=_f16 EXTRA="--dtype fp16" bash tools/profile_bench.sh > gpurun_out/profile_f16.log 2>&1 && echo profile-f16-ok && grep '^{' gpurun_out/prof_trace_f16.log | tail -1 | cut -c1-200
