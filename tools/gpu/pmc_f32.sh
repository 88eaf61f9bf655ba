# fp32 conv kernels: isolated timings (both arithmetics) + PMC passes of the split build
# (VALU vs MFMA issue, waits) on a few attack shapes; run from the repo root under gpurun
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
ONLY="${ONLY:-mod 256²|vgg 64² 256|dgrad+sdot 256²|e4e acc 32²|head s2 →16²|up 64²}"
timeout -k 10 300 python -u tools/conv_ab.py --dtype fp32 --batch 64 --iters 3 --only "$ONLY" > gpurun_out/ab_f32.log 2>&1 &&
MIA_F32_ARITH=native timeout -k 10 300 python -u tools/conv_ab.py --dtype fp32 --batch 64 --iters 3 --only "$ONLY" > gpurun_out/ab_f32native.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY --output-format csv -d gpurun_out/pmc_f32a -o run -- python3 tools/conv_ab.py --dtype fp32 --batch 64 --iters 1 --only "$ONLY" > gpurun_out/pmc_f32a.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_f32b -o run -- python3 tools/conv_ab.py --dtype fp32 --batch 64 --iters 1 --only "$ONLY" > gpurun_out/pmc_f32b.log 2>&1 &&
echo done && cat gpurun_out/ab_f32.log gpurun_out/ab_f32native.log
