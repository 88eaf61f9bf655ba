# round 3: rocprofv3 kernel trace + stats of the cfg3 bench (PGD-40, 1024², bf16, 32 images)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_cfg3 -o run -- python3 bench.py --size 1024 --pgd-steps 40 --dtype bf16 --batch 32 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/prof_cfg3.log 2>&1 && echo prof-ok && tail -1 gpurun_out/prof_cfg3.log | cut -c1-200
