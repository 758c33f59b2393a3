# A/B: Keccak rounds per loop iteration (QRK_KECCAK_UNROLL 1 default, variants u2 / u6), interleaved.
set -o pipefail
O=gpurun_out/unroll
mkdir -p $O
timeout -k 10 500 bash tools/ab.sh 2 default u2 u6 -- > $O/ab_mlkem768.jsonl 2> $O/ab.err &&
timeout -k 10 300 bash tools/ab.sh 1 default u2 u6 -- --alg FrodoKEM-640-SHAKE > $O/ab_frodo640.jsonl 2>> $O/ab.err &&
timeout -k 10 300 bash tools/ab.sh 1 default u2 u6 -- --alg HQC-128 > $O/ab_hqc128.jsonl 2>> $O/ab.err
