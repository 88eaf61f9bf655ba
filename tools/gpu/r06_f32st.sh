# round 6: the fp32 up-conv edge launch (modulated input, ≈ 516 128×128 tiles) on 64×64 tiles
# (libmiattack_f32st.so, -DMIA_F32_PRO_SMALLTILE=1) against 128×128 (product): up-conv tests on
# the variant, per-call times alternating, bit-identity of T
set -o pipefail
mkdir -p gpurun_out
MIA_LIB_VARIANT=f32st timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "upconv" > gpurun_out/r06_f32st_tests.log 2>&1 || { tail -30 gpurun_out/r06_f32st_tests.log; exit 1; }
echo "== tests f32st: $(tail -1 gpurun_out/r06_f32st_tests.log)"
for v in "" f32st "" f32st; do echo "== ${v:-prod}"; MIA_LIB_VARIANT=$v timeout -k 10 300 python -u tools/probe/upconv_premod_ab.py --dtypes fp32 --out /tmp/st_${v:-prod}.pt 2>&1 | grep -v amdgpu.ids || exit 1; done &&
timeout -k 10 120 python -u tools/probe/upconv_premod_ab.py --compare /tmp/st_prod.pt /tmp/st_f32st.pt && echo ok
