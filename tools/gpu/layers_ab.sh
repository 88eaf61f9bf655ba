# per-layer conv table under two settings of one tuning switch: VAR=a,b
set -o pipefail
mkdir -p gpurun_out
V=${1%%=*}; A=${1#*=}; A1=${A%%,*}; A2=${A#*,}
env MIA_HEAD_STREAMS=1 $V=$A1 timeout -k 10 400 python -u tools/layer_table.py --dtype ${DT:-fp32} --top 80 > gpurun_out/layers_a.log 2>&1 &&
env MIA_HEAD_STREAMS=1 $V=$A2 timeout -k 10 400 python -u tools/layer_table.py --dtype ${DT:-fp32} --top 80 > gpurun_out/layers_b.log 2>&1 && echo ok
