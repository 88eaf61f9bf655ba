set -o pipefail
mkdir -p gpurun_out
for v in 512 512 512; do
  MIA_CONV_SMALLTILE=$v timeout -k 10 200 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_networks.py -k "cw_mode" > gpurun_out/t_cw_$v.log 2>&1; echo "smalltile=$v rc=$? $(tail -1 gpurun_out/t_cw_$v.log)"
done
