# round 3: fp16 / bf16 modulated forward with the epilogue operands prefetched into the free halo
# buffer + the style row after the DMA issue — bitwise halo tests, then the modulated-forward timing
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_networks.py -x -q --timeout 120 --timeout-method thread -k "halo or modconv or styled or generator" > gpurun_out/halo_tests.log 2>&1; tail -2 gpurun_out/halo_tests.log; grep -E "^E  |FAILED" gpurun_out/halo_tests.log | head; tail -1 gpurun_out/halo_tests.log | grep -q " passed" && ! grep -q FAILED gpurun_out/halo_tests.log &&
timeout -k 10 200 python -u tools/probe/premod_ab.py --out gpurun_out/auxp.pt > gpurun_out/auxp.log 2>&1; grep -v amdgpu.ids gpurun_out/auxp.log; rm -f gpurun_out/auxp.pt
timeout -k 10 600 python -u bench.py --no-cpu-baseline > gpurun_out/bench.log 2> gpurun_out/bench.err && echo bench-ok && tail -1 gpurun_out/bench.log | cut -c1-300 && python3 -c "import json;d=json.loads(open('gpurun_out/bench.log').read().strip().splitlines()[-1]);print('fp32',d['value'],d['roofline']['achieved'],d['roofline']['frac'],'fp16',d.get('low_precision',{}).get('value'))"
