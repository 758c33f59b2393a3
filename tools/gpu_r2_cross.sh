set -o pipefail
mkdir -p gpurun_out/cross
timeout -k 10 300 python3 tools/small_crossover.py default > gpurun_out/cross/default.json 2> gpurun_out/cross/err &&
QRKEM_LIBRARY=quantum-resistant-p2p_amd/qrkem/variants/libqrkem_small64k.so timeout -k 10 300 python3 tools/small_crossover.py small64k > gpurun_out/cross/small64k.json 2>> gpurun_out/cross/err
