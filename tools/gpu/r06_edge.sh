# round 6: the up-conv forward's generic edge launch (last T row / column) on its in-range taps
# only (product) against the full 2- or 4-tap windows (libmiattack_edgefull.so:
# -DMIA_UPCONV_EDGE_TRIM=0): up-conv tests on the product, bit-identity of T at every generator
# shape, per-call times (halo kernel + edge launch) alternating.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_networks.py -k "upconv or up_conv or generator" > gpurun_out/r06_edge_tests.log 2>&1 || { tail -30 gpurun_out/r06_edge_tests.log; exit 1; }
echo "== tests: $(tail -1 gpurun_out/r06_edge_tests.log)"
for v in edgefull "" edgefull ""; do echo "== ${v:-trim}"; MIA_LIB_VARIANT=$v timeout -k 10 300 python -u tools/probe/upconv_premod_ab.py --dtypes fp32,fp16 --out /tmp/edge_${v:-trim}.pt 2>&1 | grep -v amdgpu.ids || exit 1; done &&
timeout -k 10 120 python -u tools/probe/upconv_premod_ab.py --compare /tmp/edge_edgefull.pt /tmp/edge_trim.pt && echo ok
