# round 3: the LDS-halo 32-channel kernel (conv_wres32) — bitwise vs conv_thin32 + fp64 tests,
# then A/B timing of the 1024² 32→32 layers and of the 64-channel halo tile at 512²
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q --timeout 120 --timeout-method thread -k "wres32 or thin32" > gpurun_out/wres32_tests.log 2>&1; tail -3 gpurun_out/wres32_tests.log; tail -1 gpurun_out/wres32_tests.log &&
timeout -k 10 200 python -u tools/conv_ab.py --batch 32 --dtype bf16 --only "1024" MIA_CONV_WRES32=0,1 > gpurun_out/wres32_ab.log 2>&1 &&
timeout -k 10 200 python -u tools/conv_ab.py --batch 32 --dtype fp16 --only "1024" MIA_CONV_WRES32=0,1 >> gpurun_out/wres32_ab.log 2>&1; grep -v amdgpu.ids gpurun_out/wres32_ab.log
