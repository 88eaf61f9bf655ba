# round 4: the 2-byte halo tile with one halo buffer + a 3-stage weight ring (MIA_HALO_S3) —
# bitwise tests, then the fp16 per-layer table A/B (MIA_HALO_S3=0 vs every Cin)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -k "halo_lowp_unrolled" -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/s3_test.log 2>&1; tail -3 gpurun_out/s3_test.log; grep -E "^E  |FAILED" gpurun_out/s3_test.log | head -20; tail -1 gpurun_out/s3_test.log | grep -q " passed" && ! grep -q FAILED gpurun_out/s3_test.log &&
DT=fp16 bash tools/gpu/layers_ab.sh MIA_HALO_S3=0,4096 && head -40 gpurun_out/layers_a.log && echo ---- && head -40 gpurun_out/layers_b.log
