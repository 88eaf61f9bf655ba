# round 6: the blur strip kernel with 32-bit index math, out-of-range taps read from a zero page
# (address select instead of zeroing the loaded values) and lrelu as max(v, 0.2v) (product;
# bit-identical) against the round-5 form (libmiattack_blurv1.so: -DMIA_BLUR_V2=0, with the same
# lrelu): blur tests on both, per-shape timings at fp16 / fp32 alternating.
set -o pipefail
mkdir -p gpurun_out
for v in "" blurv1; do MIA_LIB_VARIANT=$v timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "blur" > gpurun_out/r06_blurv2_tests_${v:-v2}.log 2>&1 || { tail -20 gpurun_out/r06_blurv2_tests_${v:-v2}.log; exit 1; }; echo "== tests ${v:-v2}: $(tail -1 gpurun_out/r06_blurv2_tests_${v:-v2}.log)"; done &&
for d in fp16 fp32 bf16; do for v in blurv1 "" blurv1 ""; do echo "== $d ${v:-v2}"; MIA_LIB_VARIANT=$v timeout -k 10 300 python -u tools/probe/blur_ab.py --dtype $d 2>&1 | grep -v amdgpu.ids || exit 1; done; done && echo ok
