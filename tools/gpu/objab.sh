# which change moved the e4e objective: the parity test under each A/B switch
set -o pipefail
mkdir -p gpurun_out
T="tests/test_gpu_parity.py::test_objective_and_gradient_match_reference_optimize_vgg"
for v in NONE=1 MIA_CONV_THIN=0 MIA_UPCONV_X6=0 MIA_CONV_REGEPI=0; do
  env $v timeout -k 10 300 python -u -m pytest "$T" -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/objab_$v.log 2>&1; echo "$v rc=$?"; grep -E "AssertionError: \(" gpurun_out/objab_$v.log | head -2
done
