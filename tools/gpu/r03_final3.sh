# round 3 closing run: thin-layer tests + A/B (MIA_THIN_F32 0/2/3), then the GPU suite, smoke and
# the default bench line at the final tree
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "thin_f32 or (thin_vgg and float32)" > gpurun_out/thinf32_tests.log 2>&1; tail -1 gpurun_out/thinf32_tests.log; tail -1 gpurun_out/thinf32_tests.log | grep -q " passed" && ! grep -q FAILED gpurun_out/thinf32_tests.log &&
timeout -k 10 300 python -u tools/conv_ab.py --batch 128 --dtype fp32 --iters 10 --only "thin" MIA_THIN_F32=0,2,3 > gpurun_out/thinf32_ab.log 2>&1 && grep -v amdgpu.ids gpurun_out/thinf32_ab.log &&
bash tools/gpu/r03_final1.sh
