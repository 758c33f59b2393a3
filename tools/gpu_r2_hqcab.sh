set -o pipefail
mkdir -p gpurun_out/hqcab
timeout -k 10 900 bash tools/ab.sh 2 default cf0g0 cf1g0 cf0g1 hqcold -- --alg HQC-128 > gpurun_out/hqcab/hqc128.jsonl &&
timeout -k 10 900 bash tools/ab.sh 1 default cf0g0 cf1g0 cf0g1 hqcold -- --alg HQC-256 > gpurun_out/hqcab/hqc256.jsonl
