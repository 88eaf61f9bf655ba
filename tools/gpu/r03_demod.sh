# round 3: coalesced style_demod / chunked demod_bwd — full GPU suite, then the cfg3 line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest.log 2>&1; tail -2 gpurun_out/gputest.log; grep -E "^E  |FAILED" gpurun_out/gputest.log | head -20; tail -1 gpurun_out/gputest.log | grep -q " passed" && ! grep -q FAILED gpurun_out/gputest.log &&
timeout -k 10 500 python -u bench.py --size 1024 --pgd-steps 40 --dtype bf16 --batch 32 --no-cpu-baseline > gpurun_out/bench_cfg3.log 2> gpurun_out/bench_cfg3.err && echo cfg3-ok && python3 -c "import json;d=json.loads(open('gpurun_out/bench_cfg3.log').read().strip().splitlines()[-1]);print('cfg3',d['value'],d['ms_per_step'],d['roofline']['frac'])"
