# HQC-128 A/B of the workgroup-spread decode dedupe, more rounds.
set -o pipefail
O=gpurun_out/dwg
mkdir -p $O
timeout -k 10 500 bash tools/ab.sh 4 default dwg0 -- --alg HQC-128 > $O/ab_hqc128_r4.jsonl 2> $O/ab128.err
