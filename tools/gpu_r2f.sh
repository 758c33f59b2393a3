set -o pipefail
for lib in quantum-resistant-p2p_amd/qrkem/libqrkem.so quantum-resistant-p2p_amd/qrkem/variants/libqrkem_kgaccvalu.so; do
  QRKEM_LIBRARY=$lib timeout -k 10 120 python3 tools/dbg/kg_diff.py FrodoKEM-640-SHAKE
done > gpurun_out/kgdiff2.txt 2>&1
