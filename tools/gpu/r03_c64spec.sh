# round 3: specialised epilogues + unrolled taps on the 64-channel fp16 / bf16 halo tile
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "halo" > gpurun_out/c64_tests.log 2>&1; tail -2 gpurun_out/c64_tests.log; grep -E "^E  |FAILED" gpurun_out/c64_tests.log | head; tail -1 gpurun_out/c64_tests.log | grep -q " passed" && ! grep -q FAILED gpurun_out/c64_tests.log &&
timeout -k 10 200 python -u tools/conv_ab.py --batch 32 --dtype bf16 --only "512²" MIA_HALO_C64=0,1 > gpurun_out/c64_ab.log 2>&1 &&
timeout -k 10 200 python -u tools/conv_ab.py --batch 32 --dtype fp16 --only "512²" MIA_HALO_C64=0,1 >> gpurun_out/c64_ab.log 2>&1 &&
timeout -k 10 300 python -u tools/conv_ab.py --batch 128 --dtype fp16 --only "vgg 256² 64|dgrad+tap 256|dgrad 128" MIA_HALO_C64=0,1 >> gpurun_out/c64_ab.log 2>&1; grep -v amdgpu.ids gpurun_out/c64_ab.log
