# round 3: halo prologue/epilogue A/B (tools/gpu/r03_auxab.sh), then the cfg3 rocprofv3 trace
set -o pipefail
bash tools/gpu/r03_auxab.sh && bash tools/gpu/r03_cfg3prof.sh
