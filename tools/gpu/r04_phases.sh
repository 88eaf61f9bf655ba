# round 4: block phases of the fp16 halo kernel on the StyledConv forward shapes (timing variant)
set -o pipefail
mkdir -p gpurun_out
test -f adversarial-attacks-on-gan-based-image-fusion_amd/libmiattack_htime.so &&
MIA_LIB_VARIANT=htime timeout -k 10 200 python -u tools/probe/halo_phases.py > gpurun_out/phases.log 2>&1; cat gpurun_out/phases.log | grep -v amdgpu.ids
