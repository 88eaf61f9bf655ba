# round 3: A/B of the fp16 / bf16 halo prologue / epilogue changes (bit-identical outputs)
set -o pipefail
mkdir -p gpurun_out
for v in old2 stab0 default old2 default; do
  if [ $v = default ]; then timeout -k 10 200 python -u tools/probe/premod_ab.py --out gpurun_out/ab_$v.pt > gpurun_out/ab_$v.log 2>&1 || exit 1;
  else MIA_LIB_VARIANT=$v timeout -k 10 200 python -u tools/probe/premod_ab.py --out gpurun_out/ab_$v.pt > gpurun_out/ab_$v.log 2>&1 || exit 1; fi
  echo "== $v"; grep -v amdgpu.ids gpurun_out/ab_$v.log | head -3
done
python tools/probe/premod_ab.py --compare gpurun_out/ab_old2.pt gpurun_out/ab_default.pt; python tools/probe/premod_ab.py --compare gpurun_out/ab_stab0.pt gpurun_out/ab_default.pt; rm -f gpurun_out/ab_*.pt
