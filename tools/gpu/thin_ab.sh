#!/bin/bash
# A/B of the thin-channel input-layer kernels (conv_thin.hip): the tree's library against variant
# builds (make variant VARIANT=... VARIANT_FLAGS=... in csrc/), on the conv_ab thin shapes.
set -e
mkdir -p gpurun_out
for d in fp16 fp32; do
  for v in "" ${THIN_VARIANTS:-thinnt}; do
    echo "== $d variant '${v:-default}'"
    MIA_LIB_VARIANT=$v timeout -k 10 180 python -u tools/conv_ab.py --dtype $d --iters 20 --only "thin|e4e in"
  done
done
