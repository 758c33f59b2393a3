set -o pipefail
mkdir -p gpurun_out/r2s
bash tools/coop_ab.sh || exit 1
for v in sstrace_v2 sstrace_v2chi; do
  QRKEM_LIBRARY=quantum-resistant-p2p_amd/qrkem/variants/libqrkem_$v.so timeout -k 10 200 python3 tools/single_shot_trace.py > gpurun_out/r2s/trace_$v.json 2> gpurun_out/r2s/ss_$v.err || exit 1
done
