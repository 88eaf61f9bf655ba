# round 4: the 2-byte thin input gradient (64 -> 8) on sliding-window row strips — tests, then the
# fp16 per-layer table A/B against the 2-row-item build (MIA_LIB_VARIANT=rs2) and its FETCH_SIZE
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_e4e.py -k "thin or e4e" -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/thin_test.log 2>&1; tail -2 gpurun_out/thin_test.log; grep -E "^E  |FAILED" gpurun_out/thin_test.log | head; tail -1 gpurun_out/thin_test.log | grep -q " passed" && ! grep -q FAILED gpurun_out/thin_test.log &&
MIA_LIB_VARIANT=rs2 timeout -k 10 400 python -u tools/layer_table.py --dtype fp16 --top 80 > gpurun_out/layers_a.log 2>&1 &&
timeout -k 10 400 python -u tools/layer_table.py --dtype fp16 --top 80 > gpurun_out/layers_b.log 2>&1 &&
grep -E "^step|64->8" gpurun_out/layers_a.log; echo ----; grep -E "^step|64->8" gpurun_out/layers_b.log &&
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/thin_fetch -o run -- python3 tools/layer_table.py --dtype fp16 --top 5 > gpurun_out/thin_fetch.log 2>&1 && echo fetch-ok
