#!/bin/bash
# MFMA counter pass (int8 MFMA instructions, MOPs and MFMA-pipe busy cycles per kernel), one
# bench step: tools/pmc_mfma.sh <tag> [bench args...].  One --pmc pass (6 SQ + 1 GRBM counters,
# within the per-block limits), never combined with tracing.
set -euo pipefail
tag=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/mfma_$tag
mkdir -p "$out"
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_I8 SQ_INSTS_VALU_MFMA_MOPS_I8 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE \
  --output-format csv -d "$out/m" -o run -- \
  python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu --no-profile "$@" > "$out/bench_m.json" 2> "$out/m.err"
echo "mfma $tag done"
