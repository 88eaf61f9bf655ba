# round 4: per-layer rocprofv3 evidence of the fp32 (bf16x6 product build) VGG cascade:
# kernel trace + FETCH_SIZE / WRITE_SIZE / MFMA-busy passes, joined by tools/vgg_layers_summary.py
set -o pipefail
mkdir -p gpurun_out
SARGS="--batch 128 --dtype fp32" timeout -k 10 900 bash tools/profile_vgg.sh > gpurun_out/vgg_prof.log 2>&1; rc=$?
tail -5 gpurun_out/vgg_prof.log
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/vgg_trace/**/*kernel_trace.csv", recursive=True)
rows = list(csv.DictReader(open(f[0])))
print(len(rows), "dispatches")
for r in rows[-45:]:
    print(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), r["Kernel_Name"][:110])
PY
exit $rc
