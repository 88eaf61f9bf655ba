# round 4: the VGG golden test (prints the tie accounting), the GPU suite, smoke, the default bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_networks.py::test_vgg_taps_and_grad_vs_reference_golden tests/test_gpu_metrics.py -m gpu -v -s --timeout 200 --timeout-method thread > gpurun_out/golden.log 2>&1; grep -E "VGG golden|passed|failed|Error" gpurun_out/golden.log | head;
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1; tail -2 gpurun_out/gputest.log; grep -E "^E  |FAILED" gpurun_out/gputest.log | head -20; tail -1 gpurun_out/gputest.log | grep -q " passed" && ! grep -q FAILED gpurun_out/gputest.log &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo smoke-ok &&
timeout -k 10 900 python -u bench.py > gpurun_out/bench.log 2> gpurun_out/bench.err && echo bench-ok && python3 -c "import json;d=json.loads(open('gpurun_out/bench.log').read().strip().splitlines()[-1]);print('fp32',d['value'],d['roofline']['achieved'],d['roofline']['frac'],'fp16',d.get('low_precision',{}).get('value'),'cpu',d['cpu_baseline']['value'])"
