# Round 2 (second session) final build, part A: GPU suite, smoke, ML-KEM / HQC / handshake / wire
# bench lines into gpurun_out/final_r2b/.  Each step under its own limit, stop at the first failure.
set -o pipefail
O=gpurun_out/final_r2b
mkdir -p $O
run() { tag=$1; shift; timeout -k 10 400 python3 bench.py "$@" > $O/$tag.json 2> $O/$tag.err; }
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1 &&
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
run mlkem768 &&
run mlkem768_configs2_g1 --global-log2-batch 24 --steps 2 --warmup 1 &&
run mlkem512 --alg ML-KEM-512 &&
run mlkem1024 --alg ML-KEM-1024 &&
run mlkem1024_tampered --alg ML-KEM-1024 --mode decaps-tampered &&
run hqc128 --alg HQC-128 &&
run hqc192 --alg HQC-192 &&
run hqc256 --alg HQC-256 &&
run hqc128_tampered --alg HQC-128 --mode decaps-tampered &&
run handshake_mlkem768 --mode handshake &&
run handshake_hqc128 --alg HQC-128 --mode handshake &&
run wire_mlkem768 --mode wire
