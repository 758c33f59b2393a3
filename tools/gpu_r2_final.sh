# Round-2 bench lines for every BASELINE config and §8f mode (one line each, saved under
# gpurun_out/final_r2/); each step under its own time limit, stop at the first failure.
set -o pipefail
O=gpurun_out/final_r2
mkdir -p $O
run() { tag=$1; shift; timeout -k 10 400 python3 bench.py "$@" > $O/$tag.json 2> $O/$tag.err; }
run mlkem512 --alg ML-KEM-512 &&
run mlkem1024 --alg ML-KEM-1024 &&
run mlkem1024_tampered --alg ML-KEM-1024 --mode decaps-tampered &&
run frodo640 --alg FrodoKEM-640-SHAKE &&
run frodo976 --alg FrodoKEM-976-SHAKE &&
run frodo1344 --alg FrodoKEM-1344-SHAKE --steps 3 --warmup 1 &&
run frodo640aes --alg FrodoKEM-640-AES &&
run frodo976aes --alg FrodoKEM-976-AES &&
run frodo1344aes --alg FrodoKEM-1344-AES --steps 3 --warmup 1 &&
run hqc128 --alg HQC-128 &&
run hqc192 --alg HQC-192 &&
run hqc256 --alg HQC-256 &&
run hqc128_tampered --alg HQC-128 --mode decaps-tampered &&
run handshake_mlkem768 --mode handshake &&
run handshake_frodo976aes --alg FrodoKEM-976-AES --mode handshake --steps 3 --warmup 1 &&
run handshake_hqc128 --alg HQC-128 --mode handshake &&
run wire_mlkem768 --mode wire
