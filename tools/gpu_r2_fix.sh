# Full GPU suite on the default build (Keccak 2 rounds / iteration, fix-up on the side stream),
# then A/B of the fix-up overlap (default) against fix-up on the main stream (variants/fix0).
set -o pipefail
O=gpurun_out/fix
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/t.log 2>&1 &&
timeout -k 10 600 bash tools/ab.sh 3 default fix0 -- > $O/ab_mlkem768.jsonl 2> $O/ab.err
