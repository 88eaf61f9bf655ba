# round 3: DPP row sums in the register epilogues + conv_wres32 — full GPU suite, 1024² layer A/B,
# then the default bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest.log 2>&1; tail -3 gpurun_out/gputest.log; grep -E "^E  |FAILED" gpurun_out/gputest.log | head -20; tail -1 gpurun_out/gputest.log | grep -q " passed" && ! grep -q FAILED gpurun_out/gputest.log &&
timeout -k 10 200 python -u tools/conv_ab.py --batch 32 --dtype bf16 --only "1024|512²" MIA_CONV_WRES32=0,1 > gpurun_out/wres32_ab.log 2>&1 &&
timeout -k 10 200 python -u tools/conv_ab.py --batch 32 --dtype fp16 --only "1024|512²" MIA_CONV_WRES32=0,1 >> gpurun_out/wres32_ab.log 2>&1; grep -v amdgpu.ids gpurun_out/wres32_ab.log &&
timeout -k 10 600 python -u bench.py --no-cpu-baseline > gpurun_out/bench.log 2> gpurun_out/bench.err && echo bench-ok && tail -1 gpurun_out/bench.log | cut -c1-400
