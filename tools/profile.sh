#!/bin/bash
# rocprofv3 evidence for one bench configuration (run on the GPU box from the repo root):
#   tools/profile.sh <tag> [bench args...]
# 1) --kernel-trace --stats (per-kernel durations; compare with the bench line's live events)
# 2) --pmc FETCH_SIZE and 3) --pmc WRITE_SIZE in separate passes (TCC slots), one bench step
# each, never combined with sys/runtime tracing.
set -euo pipefail
tag=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/prof_$tag
mkdir -p "$out"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- \
  python3 "$R/bench.py" --steps ${PROF_STEPS:-5} --warmup ${PROF_WARMUP:-1} --no-cpu "$@" > "$out/bench_trace.json" 2> "$out/trace.err"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/fetch" -o run -- \
  python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu --no-profile "$@" > "$out/bench_fetch.json" 2> "$out/fetch.err"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/write" -o run -- \
  python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu --no-profile "$@" > "$out/bench_write.json" 2> "$out/write.err"
echo "profile $tag done"
