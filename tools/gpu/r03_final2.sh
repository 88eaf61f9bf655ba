# round-3 final evidence part 2: rocprofv3 trace + PMC passes of the fp32 headline or of the fp16
# sub-record workload (tools/profile_bench.sh); CSVs gzipped on the box (gpurun returns ≤ 64 MiB)
set -o pipefail
mkdir -p gpurun_out
T=${1:-f32}
if [ $T = f32 ]; then TAG=_f32 bash tools/profile_bench.sh > gpurun_out/profile_f32.log 2>&1 && echo profile-f32-ok;
else TAG=_f16 EXTRA="--dtype fp16" bash tools/profile_bench.sh > gpurun_out/profile_f16.log 2>&1 && echo profile-f16-ok; fi &&
find gpurun_out -name "*.csv" -size +1M -exec gzip -f {} \; && du -sh gpurun_out
