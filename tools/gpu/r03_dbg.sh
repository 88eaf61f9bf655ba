# round 3 (diagnostic build): which generic-tile variant each conv launch of one bench attack takes
set -o pipefail
mkdir -p gpurun_out
MIA_LIB_VARIANT=dbg timeout -k 10 400 python -u tools/layer_table.py --dtype fp32 --pgd-steps 1 --top 5 > gpurun_out/dbg_f32.log 2> gpurun_out/dbg_f32.err && echo f32-ok &&
MIA_LIB_VARIANT=dbg timeout -k 10 400 python -u tools/layer_table.py --dtype fp16 --pgd-steps 1 --top 5 > gpurun_out/dbg_f16.log 2> gpurun_out/dbg_f16.err && echo f16-ok &&
grep -h MIA_LAUNCH gpurun_out/dbg_f32.err | sort | uniq -c | sort -rn | head -40 > gpurun_out/dbg_f32_summary.txt && grep -h MIA_LAUNCH gpurun_out/dbg_f16.err | sort | uniq -c | sort -rn | head -40 > gpurun_out/dbg_f16_summary.txt && gzip -f gpurun_out/dbg_f32.err gpurun_out/dbg_f16.err
