#!/bin/bash
# SQ counter pass (instruction mix and stall cycles per kernel), one bench step:
#   tools/pmc_sq.sh <tag> [bench args...]
set -euo pipefail
tag=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/sq_$tag
mkdir -p "$out"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU \
  --output-format csv -d "$out/a" -o run -- \
  python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu --no-profile "$@" > "$out/bench_a.json" 2> "$out/a.err"
timeout -k 10 300 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT \
  --output-format csv -d "$out/b" -o run -- \
  python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu --no-profile "$@" > "$out/bench_b.json" 2> "$out/b.err"
echo "sq $tag done"
