# round 3: fp32 thin-layer launch modes (MIA_THIN_F32) — bitwise mode test + thin parity, then the
# A/B timing of the two thin shapes
set -o pipefail
mkdir -p gpurun_out
true &&
timeout -k 10 300 python -u tools/conv_ab.py --batch 128 --dtype fp32 --iters 10 --only "thin rgb" MIA_THIN_F32=0,1,2 > gpurun_out/thinf32_ab.log 2>&1; grep -v amdgpu.ids gpurun_out/thinf32_ab.log
