# round 3: chunked ordered reduction finish — determinism tests + the 1024² bf16 layer table +
# halo phase probe (timing variant) for the fp16 modulated forward
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest.log 2>&1; tail -2 gpurun_out/gputest.log; grep -E "^E  |FAILED" gpurun_out/gputest.log | head -20; tail -1 gpurun_out/gputest.log | grep -q " passed" && ! grep -q FAILED gpurun_out/gputest.log &&
timeout -k 10 300 python -u tools/layer_table.py --size 1024 --dtype bf16 --batch 32 --pgd-steps 4 --top 40 > gpurun_out/layers1024.log 2>&1 && echo layers-ok && head -12 gpurun_out/layers1024.log | grep -v amdgpu &&
MIA_LIB_VARIANT=htime timeout -k 10 200 python -u tools/probe/halo_phases.py > gpurun_out/halo_phases.log 2>&1; grep -v amdgpu.ids gpurun_out/halo_phases.log
