# round 6: blur strip kernel with 3 / 4 input rows in flight per thread (libmiattack_pf3/pf4.so,
# -DMIA_BLUR_PF=3/4) against 2 (product): blur tests on each, per-shape timings alternating
set -o pipefail
mkdir -p gpurun_out
for v in "" pf3 pf4; do MIA_LIB_VARIANT=$v timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "blur" > gpurun_out/r06_blurpf_tests_${v:-pf2}.log 2>&1 || { tail -20 gpurun_out/r06_blurpf_tests_${v:-pf2}.log; exit 1; }; echo "== tests ${v:-pf2}: $(tail -1 gpurun_out/r06_blurpf_tests_${v:-pf2}.log)"; done &&
for d in fp32 fp16; do for v in "" pf3 pf4 "" pf3 pf4; do echo "== $d ${v:-pf2}"; MIA_LIB_VARIANT=$v timeout -k 10 300 python -u tools/probe/blur_ab.py --dtype $d 2>&1 | grep -v amdgpu.ids || exit 1; done; done && echo ok
