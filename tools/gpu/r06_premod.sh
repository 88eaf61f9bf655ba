# Reproduce at commit bb82676 (before the MIA_UPCONV_PREMOD=0 path was removed; results in profiles/r06_upconv_premod_ab.txt).
# round 6: the 2-byte up-conv forward with its halo modulated once in LDS per channel block
# (conv_upconv.hip PREMOD, the product) against the round-5 per-fragment modulation
# (libmiattack_premod0.so: make variant VARIANT=premod0 VARIANT_FLAGS=-DMIA_UPCONV_PREMOD=0):
# outputs bit for bit and per-call times at the generator shapes, then fp16 / bf16 layer tables.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "upconv or modconv or blur" > gpurun_out/r06_premod_tests.log 2>&1 || { tail -20 gpurun_out/r06_premod_tests.log; exit 1; }
echo "== tests: $(tail -1 gpurun_out/r06_premod_tests.log)"
for v in premod0 "" premod0 ""; do echo "== ${v:-premod1}"; MIA_LIB_VARIANT=$v timeout -k 10 300 python -u tools/probe/upconv_premod_ab.py --out /tmp/up_${v:-premod1}.pt || exit 1; done &&
python -u tools/probe/upconv_premod_ab.py --compare /tmp/up_premod0.pt /tmp/up_premod1.pt &&
for d in fp16 bf16; do for v in "" premod0; do echo "== layers $d ${v:-premod1}"; env MIA_HEAD_STREAMS=1 MIA_LIB_VARIANT=$v timeout -k 10 400 python -u tools/layer_table.py --dtype $d --top 80 > gpurun_out/layers_${d}_premod_${v:-1}.log 2>&1 || exit 1; grep -E "^step|upconv_fwd|modulated" gpurun_out/layers_${d}_premod_${v:-1}.log; done; done && echo ok
