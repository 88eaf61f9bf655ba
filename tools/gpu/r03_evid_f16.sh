# round-3 final evidence: rocprofv3 trace + PMC passes of the fp16 sub-record workload
set -o pipefail
mkdir -p gpurun_out
TAG=_f16 EXTRA="--dtype fp16" bash tools/profile_bench.sh > gpurun_out/profile_f16.log 2>&1 && echo profile-f16-ok
