# backward-front epilogue change: parity of every kernel / network test, then the bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest.log 2>&1 && echo tests-ok &&
bash tools/gpu/layers_ab.sh MIA_EPI_PRERED=1,1
