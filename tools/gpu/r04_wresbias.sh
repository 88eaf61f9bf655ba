# round 4: the fp16 / bf16 64 -> 64 bias-only launches (e4e conv2) on the weights-resident kernel
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -k "register_epilogue_paths" -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/wres_test.log 2>&1; tail -2 gpurun_out/wres_test.log; grep -E "^E  |FAILED" gpurun_out/wres_test.log | head; tail -1 gpurun_out/wres_test.log | grep -q " passed" && ! grep -q FAILED gpurun_out/wres_test.log &&
timeout -k 10 400 python -u tools/layer_table.py --dtype fp16 --top 80 > gpurun_out/layers_b.log 2>&1 && grep -E "^step|64->64" gpurun_out/layers_b.log
