# round 3: fp16 / bf16 modulated forward with the epilogue operands prefetched into the free halo
# buffer + the style row after the DMA issue — bitwise halo tests, then the modulated-forward timing
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_networks.py -x -q --timeout 120 --timeout-method thread -k "halo or modconv or styled or generator" > gpurun_out/halo_tests.log 2>&1; tail -2 gpurun_out/halo_tests.log; grep -E "^E  |FAILED" gpurun_out/halo_tests.log | head; tail -1 gpurun_out/halo_tests.log | grep -q " passed" && ! grep -q FAILED gpurun_out/halo_tests.log &&
timeout -k 10 200 python -u tools/probe/premod_ab.py --out gpurun_out/auxp.pt > gpurun_out/auxp.log 2>&1; grep -v amdgpu.ids gpurun_out/auxp.log; rm -f gpurun_out/auxp.pt
