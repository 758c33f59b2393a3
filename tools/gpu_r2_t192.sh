# HQC-192 workgroup width on the in-place enc_mul: 256 threads (default) vs 512 / 384 at 8 waves/SIMD.
set -o pipefail
O=gpurun_out/t192
mkdir -p $O
timeout -k 10 600 bash tools/ab.sh 3 default t512 t384 -- --alg HQC-192 > $O/ab_hqc192.jsonl 2> $O/ab.err
