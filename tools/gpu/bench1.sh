# one fp32 bench step + fp32 per-layer table (tuning loop)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --steps 1 --warmup 1 --lowp none --no-cpu-baseline > gpurun_out/b1.log 2>&1 && echo bench-ok && tail -1 gpurun_out/b1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['achieved'], d['roofline']['frac'])" &&
MIA_HEAD_STREAMS=1 timeout -k 10 400 python -u tools/layer_table.py --dtype fp32 --pgd-steps 2 --top 45 > gpurun_out/b1_layers.log 2>&1 && echo layers-ok && head -45 gpurun_out/b1_layers.log
