# round 3: fp32 thin-layer launch modes (MIA_THIN_F32) — bitwise mode test + thin parity, then the
# A/B timing of the thin shapes (RGB-padded as in the attack, and all 8 channels real)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "thin_f32 or (thin_vgg and float32)" > gpurun_out/thinf32_tests.log 2>&1; tail -2 gpurun_out/thinf32_tests.log; tail -1 gpurun_out/thinf32_tests.log | grep -q " passed" && ! grep -q FAILED gpurun_out/thinf32_tests.log &&
timeout -k 10 300 python -u tools/conv_ab.py --batch 128 --dtype fp32 --iters 10 --only "thin" MIA_THIN_F32=0,2,3 > gpurun_out/thinf32_ab.log 2>&1; grep -v amdgpu.ids gpurun_out/thinf32_ab.log
