# round 3: the full GPU suite after the tuning-table refactor (variant switches via
# mia_set_tuning), then the fp16 / bf16 modulated-forward tile A/B (16×16 patches on 8 or 4 waves)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest.log 2>&1 && echo gpu-tests-ok && tail -1 gpurun_out/gputest.log &&
timeout -k 10 200 python -u tools/probe/premod_ab.py --out gpurun_out/t8.pt > gpurun_out/t8.log 2>&1 &&
MIA_LIB_VARIANT=t16w8 timeout -k 10 200 python -u tools/probe/premod_ab.py --out gpurun_out/t16w8.pt > gpurun_out/t16w8.log 2>&1 &&
MIA_LIB_VARIANT=t16w4 timeout -k 10 200 python -u tools/probe/premod_ab.py --out gpurun_out/t16w4.pt > gpurun_out/t16w4.log 2>&1 &&
python tools/probe/premod_ab.py --compare gpurun_out/t8.pt gpurun_out/t16w8.pt > gpurun_out/tcmp.log 2>&1 &&
python tools/probe/premod_ab.py --compare gpurun_out/t8.pt gpurun_out/t16w4.pt >> gpurun_out/tcmp.log 2>&1; cat gpurun_out/tcmp.log; rm -f gpurun_out/t8.pt gpurun_out/t16w8.pt gpurun_out/t16w4.pt
