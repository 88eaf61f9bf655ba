# round-3 final evidence part 1: GPU suite, smoke, default bench line (with the CPU baseline)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest.log 2>&1; tail -2 gpurun_out/gputest.log; grep -E "^E  |FAILED" gpurun_out/gputest.log | head -20; tail -1 gpurun_out/gputest.log | grep -q " passed" && ! grep -q FAILED gpurun_out/gputest.log &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo smoke-ok &&
timeout -k 10 600 python -u bench.py > gpurun_out/bench.log 2> gpurun_out/bench.err && echo bench-ok && python3 -c "import json;d=json.loads(open('gpurun_out/bench.log').read().strip().splitlines()[-1]);print('fp32',d['value'],d['roofline']['achieved'],d['roofline']['frac'],'fp16',d.get('low_precision',{}).get('value'),'cpu',d['cpu_baseline']['value'])"
