# per-layer conv table of the 1024² bf16 workload (cfg3 shape, 4 PGD steps)
set -o pipefail
mkdir -p gpurun_out
MIA_HEAD_STREAMS=1 timeout -k 10 300 python -u tools/layer_table.py --size 1024 --dtype bf16 --batch 32 --pgd-steps 4 --top 40 > gpurun_out/layers1024.log 2>&1 && echo ok
