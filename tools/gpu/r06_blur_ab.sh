# round 6: the row-walking LDS blur (pointwise.hip blur4_walk_kernel, the product) against the
# round-5 strip kernel (libmiattack_blur0.so: make variant VARIANT=blur0
# VARIANT_FLAGS=-DMIA_BLUR_WALK=0): the blur test on both libraries, then per-shape timings at
# fp16 and fp32, alternating.
set -o pipefail
mkdir -p gpurun_out
for v in "" blur0; do MIA_LIB_VARIANT=$v timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "blur" > gpurun_out/r06_blur_test_${v:-walk}.log 2>&1 || { tail -20 gpurun_out/r06_blur_test_${v:-walk}.log; exit 1; }; echo "== tests ${v:-walk}: $(tail -1 gpurun_out/r06_blur_test_${v:-walk}.log)"; done &&
for d in fp16 fp32; do for v in "" blur0 ""; do echo "== $d ${v:-walk}"; MIA_LIB_VARIANT=$v timeout -k 10 300 python -u tools/probe/blur_ab.py --dtype $d || exit 1; done; done && echo ok
# timing probe: the 2-byte up-conv forward without its in-loop style modulation
# (libmiattack_nomod.so: -DMIA_PROBE_UPNOMOD, wrong numerics) — what a per-image modulated-weight
# up-conv could save at most
for d in fp16 bf16; do for v in "" nomod; do echo "== upconv $d ${v:-prod}"; env MIA_HEAD_STREAMS=1 MIA_LIB_VARIANT=$v timeout -k 10 400 python -u tools/layer_table.py --dtype $d --top 80 > gpurun_out/layers_${d}_nomod_${v:-prod}.log 2>&1 || exit 1; grep -E "^step|upconv_fwd|modulated" gpurun_out/layers_${d}_nomod_${v:-prod}.log; done; done && echo ok2
