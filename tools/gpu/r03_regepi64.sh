# round 3: specialised register epilogues on the 64-column generic tile — full GPU suite, the
# 512² A/B (MIA_CONV_REGEPI), the fp32 bench and the 1024² bf16 layer table
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest.log 2>&1; tail -2 gpurun_out/gputest.log; grep -E "^E  |FAILED" gpurun_out/gputest.log | head -20; tail -1 gpurun_out/gputest.log | grep -q " passed" && ! grep -q FAILED gpurun_out/gputest.log &&
timeout -k 10 200 python -u tools/conv_ab.py --batch 32 --dtype bf16 --only "512²" MIA_CONV_REGEPI=0,1 > gpurun_out/regepi_ab.log 2>&1 && grep -v amdgpu.ids gpurun_out/regepi_ab.log &&
timeout -k 10 300 python -u tools/layer_table.py --size 1024 --dtype bf16 --batch 32 --pgd-steps 4 --top 40 > gpurun_out/layers1024.log 2>&1 && head -12 gpurun_out/layers1024.log | grep -v amdgpu &&
timeout -k 10 600 python -u bench.py --no-cpu-baseline > gpurun_out/bench.log 2> gpurun_out/bench.err && python3 -c "import json;d=json.loads(open('gpurun_out/bench.log').read().strip().splitlines()[-1]);print('fp32',d['value'],d['roofline']['achieved'],d['roofline']['frac'],'fp16',d.get('low_precision',{}).get('value'))"
