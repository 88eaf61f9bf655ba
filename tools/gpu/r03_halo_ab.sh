# round 3: fp16 / bf16 halo kernel (unrolled taps + halo modulated once) — bitwise tests, then the
# modulated forward A/B vs the per-fragment modulation build (premod0)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "halo_lowp_unrolled_bitwise or modconv or halo_and_generic or upconv_halo" > gpurun_out/halo_tests.log 2>&1 && echo halo-tests-ok && tail -1 gpurun_out/halo_tests.log &&
MIA_LIB_VARIANT=premod0 timeout -k 10 200 python -u tools/probe/premod_ab.py --out gpurun_out/premod0.pt > gpurun_out/premod0.log 2>&1 &&
timeout -k 10 200 python -u tools/probe/premod_ab.py --out gpurun_out/premod1.pt > gpurun_out/premod1.log 2>&1 &&
python tools/probe/premod_ab.py --compare gpurun_out/premod0.pt gpurun_out/premod1.pt > gpurun_out/premod_cmp.log 2>&1; cat gpurun_out/premod_cmp.log; rm -f gpurun_out/premod0.pt gpurun_out/premod1.pt
