# round 3: persistent fp16 / bf16 halo kernel — bitwise halo tests (default = persistent vs the
# rolled non-persistent runtime-epilogue loop), then the A/B timing of the 2-byte layers
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "halo or modconv or thin32 or wres32" > gpurun_out/pk_tests.log 2>&1; tail -2 gpurun_out/pk_tests.log; grep -E "^E  |FAILED" gpurun_out/pk_tests.log | head; tail -1 gpurun_out/pk_tests.log | grep -q " passed" && ! grep -q FAILED gpurun_out/pk_tests.log &&
timeout -k 10 300 python -u tools/conv_ab.py --batch 128 --dtype fp16 --only "mod 256|mod 128|mod 64|vgg|dgrad+sdot 256|dgrad+tap 64|dgrad 128" MIA_HALO_PERSIST=0,1 > gpurun_out/pk_ab.log 2>&1; grep -v amdgpu.ids gpurun_out/pk_ab.log
