# round evidence, part 2: rocprofv3 trace + PMC passes of the default (fp32) bench, VGG cascade
set -o pipefail
mkdir -p gpurun_out
bash tools/profile_bench.sh > gpurun_out/profile.log 2>&1 && echo profile-ok &&
bash tools/profile_vgg.sh > gpurun_out/profile_vgg.log 2>&1 && echo vgg-ok
