# round 6: streaming / small kernels — blur strip blocks dealt XCD-contiguously (neighbouring strips
# meet in one L2), ToRGB forward with a reduce-scatter of its 12 sums and the skip taps prefetched,
# demod_bwd and the SE FCs with their loads batched — against the tree before them
# (libmiattack_head.so, built from the previous commit): the kernels' GPU tests on the product,
# bit-identity of the outputs across the two libraries, per-shape timings alternating.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_e4e.py -k "blur or torgb or demod or se_" > gpurun_out/r06_ew_tests.log 2>&1 || { tail -30 gpurun_out/r06_ew_tests.log; exit 1; }
echo "== tests: $(tail -1 gpurun_out/r06_ew_tests.log)"
for d in fp32 fp16; do for v in head "" head ""; do echo "== ew $d ${v:-new}"; MIA_LIB_VARIANT=$v timeout -k 10 300 python -u tools/probe/small_ab.py --dtype $d --save /tmp/ew_${d}_${v:-new}.pt 2>&1 | grep -v amdgpu.ids || exit 1; done; echo "== ew $d bit-identity"; timeout -k 10 120 python -u tools/probe/small_ab.py --compare /tmp/ew_${d}_head.pt /tmp/ew_${d}_new.pt; done &&
for d in fp32 fp16; do for v in head "" head ""; do echo "== blur $d ${v:-new}"; MIA_LIB_VARIANT=$v timeout -k 10 300 python -u tools/probe/blur_ab.py --dtype $d 2>&1 | grep -v amdgpu.ids || exit 1; done; done && echo ok
