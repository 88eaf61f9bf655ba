# PMC passes of the split-once fp32 halo kernel on a few attack shapes
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
ONLY="${ONLY:-mod 128²|vgg 64² 256}"
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY --output-format csv -d gpurun_out/pmc_x6a -o run -- python3 tools/conv_ab.py --dtype fp32 --batch 64 --iters 1 --only "$ONLY" > gpurun_out/pmc_x6a.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_x6b -o run -- python3 tools/conv_ab.py --dtype fp32 --batch 64 --iters 1 --only "$ONLY" > gpurun_out/pmc_x6b.log 2>&1 && echo done
