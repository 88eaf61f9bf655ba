# round 4: fp16 halo kernel block phases (timing build), the BMIX build's correctness on the
# halo tests, and the fp16 per-layer A/B product vs BMIX
set -o pipefail
mkdir -p gpurun_out
MIA_LIB_VARIANT=htime timeout -k 10 200 python -u tools/probe/halo_phases.py > gpurun_out/phases.log 2>&1; grep -v amdgpu.ids gpurun_out/phases.log
MIA_LIB_VARIANT=bmix timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "halo_lowp_unrolled or per_image_weights or modconv_fwd or halo_and_generic" -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/bmix_test.log 2>&1; tail -2 gpurun_out/bmix_test.log; tail -1 gpurun_out/bmix_test.log | grep -q " passed" && ! grep -q FAILED gpurun_out/bmix_test.log &&
timeout -k 10 400 python -u tools/layer_table.py --dtype fp16 --top 40 > gpurun_out/layers_a.log 2>&1 &&
MIA_LIB_VARIANT=bmix timeout -k 10 400 python -u tools/layer_table.py --dtype fp16 --top 40 > gpurun_out/layers_b.log 2>&1 && head -20 gpurun_out/layers_a.log && echo ---- && head -20 gpurun_out/layers_b.log
