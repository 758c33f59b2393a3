# HQC-256 KeyGen product pinned at 6 waves/SIMD (variants/libqrkem_kg6.so) vs unpinned, handshake
# driver line (keypair + encaps + decaps); HQC GPU tests on the variant first.
set -o pipefail
O=gpurun_out/kg
mkdir -p $O
QRKEM_LIBRARY=$PWD/quantum-resistant-p2p_amd/qrkem/variants/libqrkem_kg6.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_hqc.py > $O/t.log 2>&1 &&
timeout -k 10 400 bash tools/ab.sh 2 default kg6 -- --alg HQC-256 --mode handshake > $O/ab_hqc256_hs.jsonl 2> $O/ab.err
