# round 5, HQC: k_hqc_enc_mul's two-operand product with the next support word
# prefetched (QRK_HQC_SUP_PREFETCH) -- HQC tests, same-box A/B against the round-2 loop (variant
# sup0), the phase trace of the new kernel, profiled bench lines
set -o pipefail
cd /root/repo && source tools/gpu.sh
out r5/hqc
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_hqc.py \
  > $O/tests_hqc.log 2>&1 || { tail -30 $O/tests_hqc.log; exit 1; }
tail -2 $O/tests_hqc.log
for a in 128 192 256; do
  out r5/hqc/ab$a && abx 3 pf=default sup0=sup0 -- --alg HQC-$a --steps 20 --warmup 3 --no-profile --no-cpu || exit 1
done
out r5/hqc && QRKEM_LIBRARY=quantum-resistant-p2p_amd/qrkem/variants/libqrkem_hqctrace.so timeout -k 10 300 \
  python3 -u tools/hqc_trace.py HQC-128 > $O/hqc128_phase_trace_pf.json || exit 1
for a in 128 256; do bench hqc${a}_pf --alg HQC-$a --steps 20 --warmup 3 --no-cpu || exit 1; done
echo hqc_done
