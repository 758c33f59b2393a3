# Closing check after the in-place HQC enc_mul / decode LDS changes: GPU suite, smoke, default
# bench line, the HQC lines into gpurun_out/final_r2d/
set -o pipefail
O=gpurun_out/final_r2d
mkdir -p $O
run() { tag=$1; shift; timeout -k 10 400 python3 bench.py "$@" > $O/$tag.json 2> $O/$tag.err; }
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1 &&
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
run mlkem768_final &&
run hqc128 --alg HQC-128 &&
run hqc192 --alg HQC-192 &&
run hqc256 --alg HQC-256 &&
run hqc128_tampered --alg HQC-128 --mode decaps-tampered &&
run handshake_hqc128 --alg HQC-128 --mode handshake
