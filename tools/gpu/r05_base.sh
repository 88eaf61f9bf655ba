# round 5 baseline on this round's boxes: GPU suite, then the fp16 per-layer table (default routing)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1 && echo tests-ok && tail -1 gpurun_out/gputest.log &&
env MIA_HEAD_STREAMS=1 timeout -k 10 400 python -u tools/layer_table.py --dtype fp16 --top 60 > gpurun_out/layers_fp16_base.log 2>&1 && echo layers-ok
