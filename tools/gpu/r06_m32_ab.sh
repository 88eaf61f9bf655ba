# round 6 timing probe (verdict r05 item 2): the fp32 x6 halo main loop on 32×32×16 MFMAs with the
# same fragment reads and FLOPs (libmiattack_m32.so: make variant VARIANT=m32
# VARIANT_FLAGS=-DMIA_PROBE_MFMA32; wrong numerics, timing only) against the product library.
# fp32 layer tables, alternating.
set -o pipefail
mkdir -p gpurun_out
for v in "" m32 "" m32; do env MIA_HEAD_STREAMS=1 MIA_LIB_VARIANT=$v timeout -k 10 400 python -u tools/layer_table.py --dtype fp32 --top 60 > gpurun_out/layers_fp32_m32_${v:-def}.log 2>&1 || exit 1; echo "== ${v:-def}"; head -4 gpurun_out/layers_fp32_m32_${v:-def}.log; done && echo ok
