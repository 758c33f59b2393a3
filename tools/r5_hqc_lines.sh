# round 5: HQC bench lines with the products priced against the LDS (bench.py SPARSE_OPS note)
set -o pipefail
cd /root/repo && source tools/gpu.sh
out r5/hqc/lines
for a in 128 192 256; do bench hqc$a --alg HQC-$a || exit 1; done
bench hqc128_tampered --alg HQC-128 --mode decaps-tampered || exit 1
echo lines_done
