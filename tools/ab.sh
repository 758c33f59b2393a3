#!/bin/bash
# A/B timing of library variants inside ONE GPU call (boxes differ by a few % in clock):
#   tools/ab.sh <rounds> <tag>... -- [bench args]
# tag "default" = the in-tree libqrkem.so, else variants/libqrkem_<tag>.so.  Runs are
# interleaved (A B A B ...); one JSON summary line per run on stdout.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
rounds=$1; shift
tags=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do tags+=("$1"); shift; done
[ $# -gt 0 ] && shift
for r in $(seq 1 "$rounds"); do
  for t in "${tags[@]}"; do
    if [ "$t" = default ]; then lib=$R/quantum-resistant-p2p_amd/qrkem/libqrkem.so
    else lib=$R/quantum-resistant-p2p_amd/qrkem/variants/libqrkem_$t.so; fi
    out=$(QRKEM_LIBRARY=$lib timeout -k 10 200 python3 "$R/bench.py" --no-cpu "$@" 2>/dev/null)
    python3 -c "
import json,sys
d=json.loads(sys.argv[2]); k=d.get('kernels') or d.get('kernels_timed_region') or {}
print(json.dumps({'tag':sys.argv[1],'value':d['value'],'kernels':{n:round(v['avg_ms'],4) for n,v in k.items()}}))" "$t" "$out"
  done
done
