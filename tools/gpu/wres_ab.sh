# weights-resident 64-channel kernel: parity and A/B against the generic tile
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "register_epilogue or halo_and_generic" > gpurun_out/t_wres.log 2>&1 && echo tests-ok &&
timeout -k 10 300 python -u tools/conv_ab.py --only "64→64|e4e" MIA_CONV_WRES=0,1 > gpurun_out/ab_wres.log 2>&1 && echo ab1-ok &&
timeout -k 10 300 python -u tools/conv_ab.py --only "e4e" MIA_HALO_EPI=2,1 > gpurun_out/ab_epi.log 2>&1 && echo ab2-ok
