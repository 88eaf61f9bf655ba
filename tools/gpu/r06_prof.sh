# round 6 evidence: rocprofv3 trace + FETCH_SIZE / WRITE_SIZE / MFMA-busy passes of the default
# bench at fp32 (the headline) and fp16 (the low-precision sub-record), tools/profile_bench.sh;
# summarised on the box (profiles/summarize_rocprof.py) so only the summaries, the kernel stats and
# the gzipped kernel traces come back
set -o pipefail
mkdir -p gpurun_out/sum
summ() {  # $1 = tag, $2 = title
  local T=$1 st fe wr mf tr
  st=$(find gpurun_out/prof_trace$T -name '*kernel_stats.csv' | head -1)
  tr=$(find gpurun_out/prof_trace$T -name '*kernel_trace.csv' | head -1)
  fe=$(find gpurun_out/prof_fetch$T -name '*counter_collection.csv' | head -1)
  wr=$(find gpurun_out/prof_write$T -name '*counter_collection.csv' | head -1)
  mf=$(find gpurun_out/prof_mfma$T -name '*counter_collection.csv' | head -1)
  grep '^{' gpurun_out/prof_trace$T.log | tail -1 > gpurun_out/sum/bench_line$T.json &&
  python3 profiles/summarize_rocprof.py "$st" --fetch "$fe" --write "$wr" --mfma "$mf" --steps 3 \
    --bench-line gpurun_out/sum/bench_line$T.json --title "$2" --out gpurun_out/sum/bench$T &&
  cp "$st" gpurun_out/sum/bench${T}_kernel_stats.csv && gzip -c "$tr" > gpurun_out/sum/bench${T}_kernel_trace.csv.gz &&
  rm -rf gpurun_out/prof_trace$T gpurun_out/prof_fetch$T gpurun_out/prof_write$T gpurun_out/prof_mfma$T
}
TAG=_f32 bash tools/profile_bench.sh > gpurun_out/profile_f32.log 2>&1 && echo f32-ok &&
summ _f32 "fp32 PGD-20 step, 128 x 256^2, e4e IR-SE50 (round 6)" && echo f32-sum-ok &&
TAG=_f16 EXTRA="--dtype fp16" bash tools/profile_bench.sh > gpurun_out/profile_f16.log 2>&1 && echo f16-ok &&
summ _f16 "fp16 PGD-20 step, 128 x 256^2, e4e IR-SE50 (round 6)" && echo f16-sum-ok
