# which switch moves the e4e patch-step parity
set -o pipefail
mkdir -p gpurun_out
T="tests/test_gpu_patch.py::test_patch_attack_e4e_first_step_branch_forced"
for v in NONE=1 MIA_S2DG_X6=0 MIA_CONV_THIN=0 MIA_X6_EARLY=0 MIA_CONV_REGEPI=0 MIA_UPCONV_X6=0; do
  env $v timeout -k 10 300 python -u -m pytest "$T" -m gpu -x -q -s --timeout 200 --timeout-method thread > gpurun_out/patchab_$v.log 2>&1; echo "$v rc=$?"; grep -E "rel [0-9]" gpurun_out/patchab_$v.log | head -2
done
