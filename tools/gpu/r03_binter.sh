# round 3: A/B of the interleaved weight DMA (B-waves) in the fp16 / bf16 halo kernel
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "halo_lowp_unrolled_bitwise" > gpurun_out/binter_tests.log 2>&1; tail -1 gpurun_out/binter_tests.log
for v in default binter default binter; do
  if [ $v = default ]; then timeout -k 10 300 python -u tools/conv_ab.py --batch 128 --dtype fp16 --only "mod 256|mod 128|mod 64|vgg 128² 128|vgg 64²|vgg 32²|dgrad+sdot 256" > gpurun_out/bi_$v.log 2>&1 || exit 1;
  else MIA_LIB_VARIANT=$v timeout -k 10 300 python -u tools/conv_ab.py --batch 128 --dtype fp16 --only "mod 256|mod 128|mod 64|vgg 128² 128|vgg 64²|vgg 32²|dgrad+sdot 256" > gpurun_out/bi_$v.log 2>&1 || exit 1; fi
  echo "== $v"; grep -v amdgpu.ids gpurun_out/bi_$v.log
done
