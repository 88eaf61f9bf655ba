# A/B of the split-once stride-2 dgrad threshold (MIA_S2DG_X6_MINCIN)
set -o pipefail
mkdir -p gpurun_out
env MIA_HEAD_STREAMS=1 MIA_S2DG_X6_MINCIN=${MINC:-64} timeout -k 10 400 python -u tools/layer_table.py --dtype fp32 --top 100 > gpurun_out/layers_s2ab.log 2>&1 && echo layers-ok && grep -E "step|s2_dgrad" gpurun_out/layers_s2ab.log
