# r02 evidence for the fp32 (bf16x6) headline: rocprofv3 trace + PMC passes of the default bench,
# then the fp32 per-layer conv table (heads serialised)
set -o pipefail
mkdir -p gpurun_out
TAG=_f32 bash tools/profile_bench.sh > gpurun_out/profile.log 2>&1 && echo profile-ok &&
env MIA_HEAD_STREAMS=1 timeout -k 10 400 python -u tools/layer_table.py --dtype fp32 --top 100 > gpurun_out/layers_f32.log 2>&1 && echo layers-ok
