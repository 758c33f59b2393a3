# Regression check: the committed default vs the build at 2618d46 (before the tile-width knob and the
# HQC LDS changes), ML-KEM-768 default bench, interleaved.
set -o pipefail
O=gpurun_out/regcheck
mkdir -p $O
timeout -k 10 600 bash tools/ab.sh 3 default old2618 > $O/ab_mlkem768.jsonl 2> $O/ab.err
