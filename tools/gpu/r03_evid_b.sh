# round-3 evidence part B: rocprofv3 trace + PMC passes of the fp32 headline and of the fp16
# sub-record's workload, fp32 per-layer table
set -o pipefail
mkdir -p gpurun_out
TAG=_f32 bash tools/profile_bench.sh > gpurun_out/profile_f32.log 2>&1 && echo profile-f32-ok &&
TAG=_f16 EXTRA="--dtype fp16" bash tools/profile_bench.sh > gpurun_out/profile_f16.log 2>&1 && echo profile-f16-ok &&
timeout -k 10 400 python -u tools/layer_table.py --dtype fp32 --top 100 > gpurun_out/layers_f32.log 2>&1 && echo layers-ok
