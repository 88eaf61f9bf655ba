# round 6: blur strip height 2·KQ = 10 / 12 output rows (libmiattack_kq5/kq6.so, -DMIA_BLUR_KQ=5/6)
# against 8 (product), all at 4 input rows in flight: blur tests, per-shape timings alternating
set -o pipefail
mkdir -p gpurun_out
for v in kq5 kq6; do MIA_LIB_VARIANT=$v timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "blur" > gpurun_out/r06_blurkq_tests_$v.log 2>&1 || { tail -20 gpurun_out/r06_blurkq_tests_$v.log; exit 1; }; echo "== tests $v: $(tail -1 gpurun_out/r06_blurkq_tests_$v.log)"; done &&
for d in fp32 fp16; do for v in "" kq5 kq6 "" kq5 kq6; do echo "== $d ${v:-kq4}"; MIA_LIB_VARIANT=$v timeout -k 10 300 python -u tools/probe/blur_ab.py --dtype $d 2>&1 | grep -v amdgpu.ids || exit 1; done; done && echo ok
