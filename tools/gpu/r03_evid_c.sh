# round-3 evidence part C: rocprofv3 trace + PMC passes of the fp16 sub-record's workload, the
# fp32 and fp16 per-layer tables
set -o pipefail
mkdir -p gpurun_out
TAG=_f16 EXTRA="--dtype fp16" bash tools/profile_bench.sh > gpurun_out/profile_f16.log 2>&1 && echo profile-f16-ok &&
timeout -k 10 400 python -u tools/layer_table.py --dtype fp32 --top 100 > gpurun_out/layers_f32.log 2>&1 && echo layers-f32-ok &&
timeout -k 10 400 python -u tools/layer_table.py --dtype fp16 --top 100 > gpurun_out/layers_f16.log 2>&1 && echo layers-f16-ok
