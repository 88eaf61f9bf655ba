# bench A/B: style-head side streams (MIA_HEAD_STREAMS) with and without the per-conv HIP events
set -o pipefail
mkdir -p gpurun_out
for n in 1 4; do
  for r in "" "--no-roofline"; do
    MIA_HEAD_STREAMS=$n timeout -k 10 300 python -u bench.py --no-cpu-baseline $r > gpurun_out/bench_s$n$r.log 2>&1 || exit 1
    echo "streams=$n $r: $(tail -1 gpurun_out/bench_s$n$r.log | cut -c100-190)"
  done
done
