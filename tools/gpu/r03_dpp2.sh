# round 3: full GPU suite on the DPP-row-sum build (+ 64-channel bf16 halo forward), then the
# 1024² configs (tools/gpu/r03_configs.sh)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest.log 2>&1; tail -2 gpurun_out/gputest.log; grep -E "^E  |FAILED" gpurun_out/gputest.log | head -20; tail -1 gpurun_out/gputest.log | grep -q " passed" && ! grep -q FAILED gpurun_out/gputest.log &&
timeout -k 10 200 python -u tools/conv_ab.py --batch 32 --dtype bf16 --only "1024|512²" > gpurun_out/wres32_ab2.log 2>&1 && grep -v amdgpu.ids gpurun_out/wres32_ab2.log &&
bash tools/gpu/r03_configs.sh
