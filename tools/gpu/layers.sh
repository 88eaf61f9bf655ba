# per-layer conv table of one bench step (heads serial so per-call times are not overlapped)
set -o pipefail
mkdir -p gpurun_out
MIA_HEAD_STREAMS=1 timeout -k 10 300 python -u tools/layer_table.py --top 70 > gpurun_out/layers.log 2>&1 && echo ok
