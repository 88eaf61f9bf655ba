# round 6: blur strip kernel with 3 / 4 input rows in flight per thread (libmiattack_pf3/pf4.so,
# -DMIA_BLUR_PF=3/4) against 2 (product): blur tests on each, per-shape timings alternating
set -o pipefail
mkdir -p gpurun_out
for v in "" pf3 pf4; do MIA_LIB_VARIANT=$v timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "blur" > gpurun_out/r06_blurpf_tests_${v:-pf2}.log 2>&1 || { tail -20 gpurun_out/r06_blurpf_tests_${v:-pf2}.log; exit 1; }; echo "== tests ${v:-pf2}: $(tail -1 gpurun_out/r06_blurpf_tests_${v:-pf2}.log)"; done &&
for d in fp32 fp16; do for v in "" pf3 pf4 "" pf3 pf4; do echo "== $d ${v:-pf2}"; MIA_LIB_VARIANT=$v timeout -k 10 300 python -u tools/probe/blur_ab.py --dtype $d 2>&1 | grep -v amdgpu.ids || exit 1; done; done && echo ok
# ToRGB backward with 4 pixels' loads batched (product) against one at a time (libmiattack_tb1.so,
# -DMIA_TORGB_BWD_BATCH=1): torgb tests, timings, bit-identity
MIA_LIB_VARIANT=tb1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "torgb" > gpurun_out/r06_tb_tests_tb1.log 2>&1 &&
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "torgb" > gpurun_out/r06_tb_tests.log 2>&1 && echo "== torgb tests: $(tail -1 gpurun_out/r06_tb_tests.log)" &&
for d in fp32 fp16; do for v in tb1 "" tb1 ""; do echo "== small $d ${v:-tb4}"; MIA_LIB_VARIANT=$v timeout -k 10 300 python -u tools/probe/small_ab.py --dtype $d --save /tmp/sm_${d}_${v:-tb4}.pt 2>&1 | grep -v amdgpu.ids | grep torgb || exit 1; done; timeout -k 10 120 python -u tools/probe/small_ab.py --compare /tmp/sm_${d}_tb1.pt /tmp/sm_${d}_tb4.pt | grep torgb; done && echo ok2
