# round 3: the new smoke (bench networks vs the mask-forced oracle + split arithmetic) and the
# tests against the reference-executed fixtures (patch attack, patch_white_box, partial fusion)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo smoke-ok && cat gpurun_out/smoke.log | grep -v amdgpu.ids &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_patch.py tests/test_gpu_parity.py "tests/test_gpu_networks.py::test_partial_fusion_matches_reference" -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r03_new.log 2>&1 && echo tests-ok; grep -E "PASS|FAIL|Error|rel |norm|passed|failed" gpurun_out/r03_new.log | tail -40
