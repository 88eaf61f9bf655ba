# round 4: rocprofv3 trace + FETCH/WRITE/MFMA-busy passes of the fp32 headline (tools/profile_bench.sh)
set -o pipefail
mkdir -p gpurun_out
TAG=_f32 bash tools/profile_bench.sh > gpurun_out/profile_f32.log 2>&1 && echo profile-f32-ok && grep '^{' gpurun_out/prof_trace_f32.log | tail -1 | cut -c1-200
