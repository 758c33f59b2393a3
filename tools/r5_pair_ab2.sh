# round 5: lane-pair fronts, J on pairs or not -- interleaved A/B at 2^14 / 2^15, then profiled lines
set -o pipefail
cd /root/repo && source tools/gpu.sh
for lb in 14 15; do
  out r5/pair2/b$lb
  abx 3 pair=default noj=pairnoj off=pairoff -- --log2-batch $lb --steps 60 --warmup 10 --no-profile || exit 1
done
out r5/pair2/prof && for lb in 14 15; do for t in default pairnoj pairoff; do
  L=quantum-resistant-p2p_amd/qrkem/libqrkem.so; [ $t != default ] && L=quantum-resistant-p2p_amd/qrkem/variants/libqrkem_$t.so
  QRKEM_LIBRARY=$L bench ${t}_$lb --log2-batch $lb --steps 60 --warmup 10 --no-cpu || exit 1
done; done
