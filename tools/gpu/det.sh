# deterministic SE sums: determinism probe, e4e / parity / patch suites
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/probe/e4e_det.py > gpurun_out/det_probe.log 2>&1; echo probe-rc=$?; grep -E "run|fwd" gpurun_out/det_probe.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_e4e.py tests/test_gpu_parity.py tests/test_gpu_patch.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/det_tests.log 2>&1; echo tests-rc=$?; tail -2 gpurun_out/det_tests.log
