# round 3: BIAS / ACC / BIAS|ACC register epilogues on the generic tile — new stride-2 tests, the full
# GPU suite, then the fp32 bench (MIA_CONV_REGEPI=0 run for the A/B) and the fp16 layer table
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest.log 2>&1; tail -2 gpurun_out/gputest.log; grep -E "^E  |FAILED" gpurun_out/gputest.log | head -20; tail -1 gpurun_out/gputest.log | grep -q " passed" && ! grep -q FAILED gpurun_out/gputest.log &&
timeout -k 10 600 python -u bench.py --no-cpu-baseline --lowp none > gpurun_out/bench_new.log 2> gpurun_out/bench_new.err && python3 -c "import json;d=json.loads(open('gpurun_out/bench_new.log').read().strip().splitlines()[-1]);print('new fp32',d['value'],d['roofline']['achieved'])" &&
timeout -k 10 400 python -u tools/layer_table.py --dtype fp32 --top 60 > gpurun_out/layers_f32.log 2>&1 && echo layers-ok
